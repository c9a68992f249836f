// TSan / ASan self-test of the native GPU monitor (the in-process native code runs
// threads next to the interpreter, so it is sanitized): the real sampler and event-listener threads of monitor_core.hpp run
// against the stub amd-smi (amdsmi_stub.cpp) and a fake procfs tree while the main
// thread hammers every reader (snapshot, devices, history, peak_between, drain_events,
// inject_event) and the test hooks mutate the stub.  Built with -fsanitize=thread (and
// address,undefined) by `python -m nexus_supervisor_amd._build --sanitize thread`;
// tests/test_sanitizers.py fails on any sanitizer report.
//
//   monitor_selftest <proc_root> <sys_root> [seconds]
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>

#include "monitor_core.hpp"

extern "C" {
void nexus_stub_set_vram(int gpu, uint32_t used_mb);
void nexus_stub_set_proc(int gpu, uint32_t pid, uint64_t vram);
void nexus_stub_end_proc(int gpu, uint32_t pid);
void nexus_stub_set_links_down(int gpu, int down);
void nexus_stub_push_event(int gpu, int type, const char* message);
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s <proc_root> <sys_root> [seconds]\n", argv[0]);
    return 2;
  }
  double secs = argc > 3 ? atof(argv[3]) : 2.0;
  int rc = 0;
  for (const char* mode : {"drm", "kfd", "amdsmi"}) {
    nexus_gpu::MonitorOptions o;
    o.interval_ms = 2;
    o.proc_source = mode;
    o.proc_root = argv[1];
    o.sys_root = argv[2];
    o.health_every = 3;
    o.retain_s = 0.05;
    // heap-allocated: TSan forgets a freed block's mutexes, not a reused stack slot's
    auto mp = std::make_unique<nexus_gpu::GpuMonitor>(o);
    nexus_gpu::GpuMonitor& m = *mp;
    m.start();
    double t0 = nexus_gpu::now_s();
    uint64_t iters = 0, procs_seen = 0, events_seen = 0;
    while (nexus_gpu::now_s() - t0 < secs / 3) {
      int i = static_cast<int>(iters % 2);
      nexus_stub_set_vram(i, 1000 + static_cast<uint32_t>(iters % 5000));
      nexus_stub_set_proc(i, 4242, (iters % 7) << 30);
      if (iters % 11 == 0) nexus_stub_end_proc(i, 4242);
      if (iters % 17 == 0) nexus_stub_push_event(i, AMDSMI_EVT_NOTIF_VMFAULT, "stub fault");
      if (iters % 23 == 0) nexus_stub_set_links_down(i, static_cast<int>(iters % 3));
      if (iters % 29 == 0) m.inject_event(i, "QUEUE_EVICTION", "injected");
      for (auto& v : m.snapshot(true)) procs_seen += v.procs.size();
      events_seen += m.drain_events().size();
      (void)m.devices();
      (void)m.history(0, t0);
      (void)m.peak_between(1, t0, nexus_gpu::now_s());
      if (iters % 97 == 0) m.reset_peaks();
      ++iters;
    }
    uint64_t samples = m.samples();
    m.stop();
    printf("mode=%s iters=%llu samples=%llu procs_seen=%llu events=%llu\n", mode,
           static_cast<unsigned long long>(iters), static_cast<unsigned long long>(samples),
           static_cast<unsigned long long>(procs_seen), static_cast<unsigned long long>(events_seen));
    if (samples < 3 || events_seen == 0) rc = 1;
  }
  return rc;
}
