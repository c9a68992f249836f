// Stub amd-smi backend: the subset of the amd-smi C API that monitor_core.hpp calls,
// over an in-memory model of an MI355X node (N GPUs, 288 GB HBM3E each, all-to-all
// xGMI).  It lets the CPU test suite drive the real sampler / listener threads
// (`_amdsmi_monitor_stub`) and the TSan self-test (`monitor_selftest`) on hosts with
// no GPU.  Test hooks (`nexus_stub_*`) program VRAM, processes, links and events.
// Every entry point takes the stub's own mutex: the monitor calls it from its sampler,
// its event listener and the caller's thread at once.
#include <amd_smi/amdsmi.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

struct StubProc {
  uint32_t pid;
  uint64_t vram;
};

struct StubGpu {
  int bus;
  uint32_t vram_total_mb = 294896, vram_used_mb = 283;
  uint64_t ecc_uncorrectable = 0;
  int links_down = 0;
  std::vector<StubProc> procs;
  std::vector<uint32_t> vanished;  // printed once by the next process-list call
};

struct StubEvent {
  int gpu;
  int type;
  std::string message;
};

std::mutex g_mu;
std::vector<StubGpu> g_gpus;
std::deque<StubEvent> g_events;
bool g_init = false;
uint64_t g_calls = 0;

void ensure_gpus_locked() {
  if (!g_gpus.empty()) return;
  const char* n = getenv("NEXUS_STUB_GPUS");
  int count = n ? atoi(n) : 2;
  if (count < 1) count = 1;
  if (count > 8) count = 8;
  for (int i = 0; i < count; ++i) {
    StubGpu g;
    g.bus = 0x0a + i;
    g_gpus.push_back(g);
  }
}

int handle_index(amdsmi_processor_handle h) {
  intptr_t v = reinterpret_cast<intptr_t>(h);
  return static_cast<int>(v) - 1;
}

bool valid(amdsmi_processor_handle h) {
  int i = handle_index(h);
  return i >= 0 && i < static_cast<int>(g_gpus.size());
}

}  // namespace

extern "C" {

// ---- test hooks
void nexus_stub_set_vram(int gpu, uint32_t used_mb) {
  std::lock_guard<std::mutex> lk(g_mu);
  ensure_gpus_locked();
  if (gpu >= 0 && gpu < static_cast<int>(g_gpus.size())) g_gpus[gpu].vram_used_mb = used_mb;
}

void nexus_stub_set_proc(int gpu, uint32_t pid, uint64_t vram) {
  std::lock_guard<std::mutex> lk(g_mu);
  ensure_gpus_locked();
  if (gpu < 0 || gpu >= static_cast<int>(g_gpus.size())) return;
  for (auto& p : g_gpus[gpu].procs)
    if (p.pid == pid) {
      p.vram = vram;
      return;
    }
  g_gpus[gpu].procs.push_back(StubProc{pid, vram});
}

void nexus_stub_end_proc(int gpu, uint32_t pid) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (gpu < 0 || gpu >= static_cast<int>(g_gpus.size())) return;
  auto& ps = g_gpus[gpu].procs;
  for (size_t i = 0; i < ps.size(); ++i)
    if (ps[i].pid == pid) {
      ps.erase(ps.begin() + static_cast<long>(i));
      return;
    }
}

void nexus_stub_set_links_down(int gpu, int down) {
  std::lock_guard<std::mutex> lk(g_mu);
  ensure_gpus_locked();
  if (gpu >= 0 && gpu < static_cast<int>(g_gpus.size())) g_gpus[gpu].links_down = down;
}

void nexus_stub_add_vanished(int gpu, uint32_t pid) {
  std::lock_guard<std::mutex> lk(g_mu);
  ensure_gpus_locked();
  if (gpu >= 0 && gpu < static_cast<int>(g_gpus.size())) g_gpus[gpu].vanished.push_back(pid);
}

void nexus_stub_push_event(int gpu, int type, const char* message) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_events.push_back(StubEvent{gpu, type, message ? message : ""});
}

uint64_t nexus_stub_calls() {
  std::lock_guard<std::mutex> lk(g_mu);
  return g_calls;
}

// ---- amd-smi subset
amdsmi_status_t amdsmi_init(uint64_t) {
  std::lock_guard<std::mutex> lk(g_mu);
  ensure_gpus_locked();
  g_init = true;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_shut_down() {
  std::lock_guard<std::mutex> lk(g_mu);
  g_init = false;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_status_code_to_string(amdsmi_status_t, const char** s) {
  *s = "stub status";
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_socket_handles(uint32_t* count, amdsmi_socket_handle* handles) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_init) return AMDSMI_STATUS_NOT_INIT;
  if (handles && *count >= 1) handles[0] = reinterpret_cast<amdsmi_socket_handle>(static_cast<intptr_t>(1));
  *count = 1;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_processor_handles(amdsmi_socket_handle, uint32_t* count,
                                             amdsmi_processor_handle* handles) {
  std::lock_guard<std::mutex> lk(g_mu);
  uint32_t n = static_cast<uint32_t>(g_gpus.size());
  if (handles)
    for (uint32_t i = 0; i < n && i < *count; ++i)
      handles[i] = reinterpret_cast<amdsmi_processor_handle>(static_cast<intptr_t>(i + 1));
  *count = n;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_device_bdf(amdsmi_processor_handle h, amdsmi_bdf_t* bdf) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!valid(h)) return AMDSMI_STATUS_INVAL;
  memset(bdf, 0, sizeof *bdf);
  bdf->bus_number = static_cast<uint64_t>(g_gpus[handle_index(h)].bus) & 0xff;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_device_uuid(amdsmi_processor_handle h, unsigned int* len, char* uuid) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!valid(h)) return AMDSMI_STATUS_INVAL;
  snprintf(uuid, *len, "stub-%04d-1000-80cc-38ccaef3a999", handle_index(h));
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_enumeration_info(amdsmi_processor_handle h, amdsmi_enumeration_info_t* en) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!valid(h)) return AMDSMI_STATUS_INVAL;
  int i = handle_index(h);
  en->hip_id = static_cast<uint32_t>(i);
  snprintf(en->hip_uuid, sizeof en->hip_uuid, "GPU-stub%012d", i);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_asic_info(amdsmi_processor_handle h, amdsmi_asic_info_t* asic) {
  if (!valid(h)) return AMDSMI_STATUS_INVAL;
  snprintf(asic->market_name, sizeof asic->market_name, "AMD Instinct MI355X (stub)");
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_kfd_info(amdsmi_processor_handle h, amdsmi_kfd_info_t* info) {
  if (!valid(h)) return AMDSMI_STATUS_INVAL;
  info->kfd_id = 20000 + static_cast<uint64_t>(handle_index(h));
  info->node_id = static_cast<uint32_t>(handle_index(h)) + 1;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_xgmi_info(amdsmi_processor_handle h, amdsmi_xgmi_info_t* info) {
  if (!valid(h)) return AMDSMI_STATUS_INVAL;
  info->xgmi_hive_id = 0x5a7e0000ULL;
  info->xgmi_node_id = static_cast<uint64_t>(handle_index(h));
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_link_metrics(amdsmi_processor_handle h, amdsmi_link_metrics_t* lm) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!valid(h)) return AMDSMI_STATUS_INVAL;
  ++g_calls;
  int self = handle_index(h);
  uint32_t k = 0;
  // peers first (up to 7 on an 8-GPU node), the remaining ports unconnected
  for (int j = 0; j < static_cast<int>(g_gpus.size()) && k < 7; ++j) {
    if (j == self) continue;
    auto& l = lm->links[k++];
    memset(&l, 0, sizeof l);
    l.bdf.bus_number = static_cast<uint64_t>(g_gpus[j].bus) & 0xff;
    l.bit_rate = 38;
    l.max_bandwidth = 608;
    l.link_type = AMDSMI_LINK_TYPE_XGMI;
    l.read = g_calls * 10;
    l.write = g_calls * 12;
  }
  while (k < 7) {
    auto& l = lm->links[k++];
    memset(&l, 0xff, sizeof l.bdf);
    l.link_type = AMDSMI_LINK_TYPE_XGMI;
    l.bit_rate = 38;
    l.max_bandwidth = 608;
    l.read = l.write = 0;
  }
  lm->num_links = 7;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_vram_usage(amdsmi_processor_handle h, amdsmi_vram_usage_t* v) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!valid(h)) return AMDSMI_STATUS_INVAL;
  ++g_calls;
  v->vram_total = g_gpus[handle_index(h)].vram_total_mb;
  v->vram_used = g_gpus[handle_index(h)].vram_used_mb;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_total_ecc_count(amdsmi_processor_handle h, amdsmi_error_count_t* ec) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!valid(h)) return AMDSMI_STATUS_INVAL;
  ec->correctable_count = 0;
  ec->uncorrectable_count = g_gpus[handle_index(h)].ecc_uncorrectable;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_process_list(amdsmi_processor_handle h, uint32_t* max, amdsmi_proc_info_t* list) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!valid(h)) return AMDSMI_STATUS_INVAL;
  auto& ps = g_gpus[handle_index(h)].procs;
  // a process that exited while the real library listed it: its stderr line, once
  for (uint32_t pid : g_gpus[handle_index(h)].vanished)
    fprintf(stderr, "Unable to open queues directory for process %u: No such file or directory\n", pid);
  g_gpus[handle_index(h)].vanished.clear();
  uint32_t n = static_cast<uint32_t>(ps.size());
  if (n > *max) {
    *max = n;
    return AMDSMI_STATUS_OUT_OF_RESOURCES;
  }
  for (uint32_t i = 0; i < n; ++i) {
    memset(&list[i], 0, sizeof list[i]);
    snprintf(list[i].name, sizeof list[i].name, "N/A");
    list[i].pid = ps[i].pid;
    list[i].mem = ps[i].vram;
    list[i].memory_usage.vram_mem = ps[i].vram;
  }
  *max = n;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_xgmi_link_status(amdsmi_processor_handle h, amdsmi_xgmi_link_status_t* st) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!valid(h)) return AMDSMI_STATUS_INVAL;
  st->total_links = 8;
  int down = g_gpus[handle_index(h)].links_down;
  st->status[0] = AMDSMI_XGMI_LINK_DISABLE;
  for (int k = 1; k < 8; ++k) st->status[k] = (k <= down) ? AMDSMI_XGMI_LINK_DOWN : AMDSMI_XGMI_LINK_UP;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_gpu_xgmi_error_status(amdsmi_processor_handle h, amdsmi_xgmi_status_t* st) {
  if (!valid(h)) return AMDSMI_STATUS_INVAL;
  *st = AMDSMI_XGMI_STATUS_NO_ERRORS;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_init_gpu_event_notification(amdsmi_processor_handle h) {
  return valid(h) ? AMDSMI_STATUS_SUCCESS : AMDSMI_STATUS_INVAL;
}

amdsmi_status_t amdsmi_set_gpu_event_notification_mask(amdsmi_processor_handle h, uint64_t) {
  return valid(h) ? AMDSMI_STATUS_SUCCESS : AMDSMI_STATUS_INVAL;
}

amdsmi_status_t amdsmi_stop_gpu_event_notification(amdsmi_processor_handle h) {
  return valid(h) ? AMDSMI_STATUS_SUCCESS : AMDSMI_STATUS_INVAL;
}

amdsmi_status_t amdsmi_get_gpu_event_notification(int timeout_ms, uint32_t* num, amdsmi_evt_notification_data_t* data) {
  std::this_thread::sleep_for(std::chrono::milliseconds(timeout_ms < 20 ? timeout_ms : 20));
  std::lock_guard<std::mutex> lk(g_mu);
  uint32_t n = 0;
  while (!g_events.empty() && n < *num) {
    StubEvent e = g_events.front();
    g_events.pop_front();
    memset(&data[n], 0, sizeof data[n]);
    data[n].processor_handle = reinterpret_cast<amdsmi_processor_handle>(static_cast<intptr_t>(e.gpu + 1));
    data[n].event = static_cast<amdsmi_evt_notification_type_t>(e.type);
    snprintf(data[n].message, sizeof data[n].message, "%s", e.message.c_str());
    ++n;
  }
  *num = n;
  return n ? AMDSMI_STATUS_SUCCESS : AMDSMI_STATUS_NO_DATA;
}

}  // extern "C"
