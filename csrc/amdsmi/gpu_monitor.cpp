// Python binding of the native MI355X GPU monitor (monitor_core.hpp) and of the
// procfs / sysfs attribution scanners (procscan.hpp).  Snapshots are copied out of the
// core under its mutex and converted to Python objects afterwards, so neither native
// thread ever waits on the GIL.  Built twice: against libamd_smi (`_amdsmi_monitor`,
// the production module) and against the stub amd-smi (`_amdsmi_monitor_stub`, CPU
// tests of the sampler / attribution path).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "monitor_core.hpp"

#ifndef NEXUS_MONITOR_MODULE
#define NEXUS_MONITOR_MODULE _amdsmi_monitor
#endif

namespace py = pybind11;
using namespace nexus_gpu;

namespace {

py::dict proc_dict(const ProcRec& p) {
  py::dict d;
  d["pid"] = p.pid;
  d["name"] = p.name;
  d["source"] = p.source;
  d["vram_bytes"] = p.vram;
  d["peak_vram_bytes"] = p.peak_vram;
  d["gtt_bytes"] = p.gtt;
  d["cu_occupancy"] = p.cu_occupancy;
  d["alive"] = p.alive;
  d["first_seen"] = p.first_seen;
  d["last_seen"] = p.last_seen;
  if (!p.pod_uid.empty()) d["pod_uid"] = p.pod_uid;
  if (!p.cgroup.empty()) d["cgroup"] = p.cgroup;
  py::dict env;
  for (auto& kv : p.env) env[py::str(kv.first)] = kv.second;
  d["env"] = env;
  return d;
}

py::dict event_dict(const EventRec& e) {
  py::dict d;
  d["gpu"] = e.gpu;
  d["type"] = e.type;
  d["message"] = e.message;
  d["t"] = e.t;
  return d;
}

py::list links_list(const GpuRec& g) {
  py::list out;
  for (auto& l : g.links) {
    py::dict d;
    d["peer_bdf"] = l.peer_bdf;
    d["peer_index"] = l.peer_index;
    d["type"] = link_type_name(l.type);
    d["bit_rate_gbps"] = l.bit_rate;
    d["max_bandwidth_gbps"] = l.max_bandwidth;
    d["read_kb"] = l.read_kb;
    d["write_kb"] = l.write_kb;
    out.append(d);
  }
  return out;
}

void device_fields(py::dict& d, const GpuRec& g) {
  d["index"] = g.index;
  d["bdf"] = g.bdf;
  d["uuid"] = g.uuid;
  d["hip_uuid"] = g.hip_uuid;
  d["hip_id"] = g.hip_id;
  d["vram_total_mb"] = g.vram_total_mb;
  if (g.kfd_id) d["kfd_id"] = g.kfd_id;
  if (g.hive_id) d["xgmi_hive_id"] = g.hive_id;
  if (!g.links.empty()) d["links"] = links_list(g);
}

class PyMonitor {
 public:
  PyMonitor(int interval_ms, bool events, double retain_s, bool read_proc, std::string proc_source,
            std::string proc_root, std::string sys_root, int health_every)
      : m_(MonitorOptions{interval_ms, events, retain_s, read_proc, std::move(proc_source), std::move(proc_root),
                          std::move(sys_root), health_every}) {}

  void start() {
    py::gil_scoped_release nogil;
    m_.start();
  }
  void stop() {
    py::gil_scoped_release nogil;
    m_.stop();
  }

  py::list devices() {
    std::vector<GpuRec> gs;
    {
      py::gil_scoped_release nogil;
      gs = m_.devices();
    }
    py::list out;
    for (auto& g : gs) {
      py::dict d;
      device_fields(d, g);
      d["market_name"] = g.market_name;
      d["events"] = g.events_ok;
      out.append(d);
    }
    return out;
  }

  py::list snapshot(bool include_exited) {
    std::vector<GpuView> vs;
    {
      py::gil_scoped_release nogil;
      vs = m_.snapshot(include_exited);
    }
    py::list out;
    for (auto& v : vs) {
      const GpuRec& g = v.gpu;
      py::dict d;
      device_fields(d, g);
      d["vram_used_mb"] = g.vram_used_mb;
      d["vram_peak_mb"] = g.vram_peak_mb;
      d["ecc_correctable"] = g.ecc_correctable;
      d["ecc_uncorrectable"] = g.ecc_uncorrectable;
      if (g.xgmi_links_total >= 0) {
        d["xgmi_links_total"] = g.xgmi_links_total;
        d["xgmi_links_up"] = g.xgmi_links_up;
        d["xgmi_links_down"] = g.xgmi_links_down;
      }
      if (g.xgmi_error >= 0) d["xgmi_error"] = g.xgmi_error;
      if (g.foreign_procs) {
        d["foreign_procs"] = g.foreign_procs;
        d["foreign_vram_bytes"] = g.foreign_vram;
      }
      py::list procs;
      for (auto& p : v.procs) procs.append(proc_dict(p));
      d["procs"] = procs;
      py::list evs;
      for (auto& e : v.events) evs.append(event_dict(e));
      d["events"] = evs;
      out.append(d);
    }
    return out;
  }

  py::list drain_events() {
    std::vector<EventRec> es;
    {
      py::gil_scoped_release nogil;
      es = m_.drain_events();
    }
    py::list out;
    for (auto& e : es) out.append(event_dict(e));
    return out;
  }

  py::list history(int gpu_index, double since) {
    std::vector<std::pair<double, uint32_t>> h;
    {
      py::gil_scoped_release nogil;
      h = m_.history(gpu_index, since);
    }
    py::list l;
    for (auto& smp : h) l.append(py::make_tuple(smp.first, smp.second));
    return l;
  }

  GpuMonitor m_;
};

py::list uses_list(const std::vector<ProcGpuUse>& us) {
  py::list out;
  for (auto& u : us) {
    py::dict d;
    d["pid"] = u.pid;
    d["bdf"] = u.bdf;
    d["vram_bytes"] = u.vram_bytes;
    d["gtt_bytes"] = u.gtt_bytes;
    d["evicted_vram_bytes"] = u.evicted_vram_bytes;
    d["clients"] = u.clients;
    out.append(d);
  }
  return out;
}

class PyDrmScanner {
 public:
  PyDrmScanner(std::string root, int rescan_every) : s_(std::move(root), rescan_every) {}
  py::list scan() { return uses_list(s_.scan()); }
  uint64_t fd_scans() const { return s_.fd_scans(); }
  DrmScanner s_;
};

}  // namespace

#ifdef NEXUS_AMDSMI_STUB
extern "C" {
void nexus_stub_set_vram(int gpu, uint32_t used_mb);
void nexus_stub_set_proc(int gpu, uint32_t pid, uint64_t vram);
void nexus_stub_end_proc(int gpu, uint32_t pid);
void nexus_stub_set_links_down(int gpu, int down);
void nexus_stub_add_vanished(int gpu, uint32_t pid);
void nexus_stub_push_event(int gpu, int type, const char* message);
}
#endif

PYBIND11_MODULE(NEXUS_MONITOR_MODULE, m) {
  m.doc() = "Native amd-smi GPU monitor: VRAM peaks, per-process attribution, xGMI links, GPU event listener";
  m.def("pod_uid_from_cgroup", &pod_uid_from_cgroup, "Extract a K8s pod UID from a /proc/<pid>/cgroup text");
  m.def("host_pid_namespace", &host_pid_namespace, py::arg("proc_root") = "/proc",
        "True when proc_root belongs to the initial PID namespace (amd-smi / KFD PIDs are valid there)");
  m.def(
      "parse_drm_fdinfo",
      [](const std::string& text) {
        DrmFdInfo r = parse_drm_fdinfo(text);
        py::dict d;
        d["amdgpu"] = r.amdgpu;
        d["pdev"] = r.pdev;
        d["client_id"] = r.client_id;
        d["vram_bytes"] = r.vram_bytes;
        d["gtt_bytes"] = r.gtt_bytes;
        d["evicted_vram_bytes"] = r.evicted_vram_bytes;
        return d;
      },
      "Parse one amdgpu DRM fdinfo text");
  m.def("kfd_gpu_bdfs", &kfd_gpu_bdfs, py::arg("sys_root") = "/sys", "KFD topology gpu_id -> PCI BDF");
  m.def(
      "denials",
      []() {
        py::dict d;
        for (int k = 0; k < kDenySources; ++k) d[deny_source_name(k)] = deny_counters()[k].load();
        return d;
      },
      "Process / sysfs reads refused by the kernel (EACCES / EPERM) so far, by source");
  m.def(
      "reset_denials",
      []() {
        for (int k = 0; k < kDenySources; ++k) deny_counters()[k].store(0);
      },
      "Zero the refusal counters");
  m.def(
      "stderr_filter",
      [](bool on) { Fd2Filter::instance().set_enabled(on); },
      py::arg("enabled"),
      "Keep libamd_smi's per-process stderr noise out of fd 2 (on by default; stderr_filter.hpp)");
  m.def(
      "stderr_filter_stats",
      []() {
        py::dict d;
        d["noise_lines"] = Fd2Filter::instance().noise_lines();
        d["forwarded_bytes"] = Fd2Filter::instance().forwarded_bytes();
        return d;
      },
      "Noise lines dropped and other threads' stderr bytes forwarded so far");
  m.def(
      "kfd_proc_usage",
      [](const std::string& sys_root) { return uses_list(kfd_proc_usage(sys_root, kfd_gpu_bdfs(sys_root))); },
      py::arg("sys_root") = "/sys", "Per-process VRAM from KFD sysfs (init-namespace PIDs)");
  py::class_<PyDrmScanner>(m, "DrmScanner")
      .def(py::init<std::string, int>(), py::arg("proc_root") = "/proc", py::arg("rescan_every") = 8)
      .def("scan", &PyDrmScanner::scan)
      .def_property_readonly("fd_scans", &PyDrmScanner::fd_scans);
  py::class_<PyMonitor>(m, "GpuMonitor")
      .def(py::init<int, bool, double, bool, std::string, std::string, std::string, int>(), py::arg("interval_ms") = 250,
           py::arg("events") = true, py::arg("retain_s") = 600.0, py::arg("read_proc") = true,
           py::arg("proc_source") = "auto", py::arg("proc_root") = "/proc", py::arg("sys_root") = "/sys",
           py::arg("health_every") = 10)
      .def("start", &PyMonitor::start)
      .def("stop", &PyMonitor::stop)
      .def("devices", &PyMonitor::devices)
      .def("snapshot", &PyMonitor::snapshot, py::arg("include_exited") = true)
      .def("drain_events", &PyMonitor::drain_events)
      .def("inject_event", [](PyMonitor& s, int gpu, const std::string& type,
                              const std::string& msg) { s.m_.inject_event(gpu, type, msg); })
      .def("reset_peaks", [](PyMonitor& s) { s.m_.reset_peaks(); })
      .def("peak_between", [](PyMonitor& s, int gpu, double t0, double t1) { return s.m_.peak_between(gpu, t0, t1); })
      .def("history", &PyMonitor::history, py::arg("gpu_index"), py::arg("since") = 0.0)
      .def_property_readonly("samples", [](PyMonitor& s) { return s.m_.samples(); })
      .def_property_readonly("process_vanished", [](PyMonitor& s) { return s.m_.process_vanished(); })
      .def_property_readonly("last_sample", [](PyMonitor& s) { return s.m_.last_sample_seconds(); })
      .def_property_readonly("n_gpus", [](PyMonitor& s) { return s.m_.n_gpus(); })
      .def_property_readonly("proc_mode", [](PyMonitor& s) { return s.m_.proc_mode(); })
      .def_property_readonly("host_pid_ns", [](PyMonitor& s) { return s.m_.host_pid_ns(); });
#ifdef NEXUS_AMDSMI_STUB
  m.attr("STUB") = true;
  m.def("stub_set_vram", &nexus_stub_set_vram);
  m.def("stub_set_proc", &nexus_stub_set_proc);
  m.def("stub_end_proc", &nexus_stub_end_proc);
  m.def("stub_set_links_down", &nexus_stub_set_links_down);
  m.def("stub_add_vanished", &nexus_stub_add_vanished);
  m.def("stub_push_event", [](int gpu, const std::string& type, const std::string& msg) {
    int t = AMDSMI_EVT_NOTIF_VMFAULT;
    if (type == "GPU_PRE_RESET") t = AMDSMI_EVT_NOTIF_GPU_PRE_RESET;
    else if (type == "QUEUE_EVICTION") t = AMDSMI_EVT_NOTIF_QUEUE_EVICTION;
    else if (type == "PROCESS_END") t = AMDSMI_EVT_NOTIF_PROCESS_END;
    nexus_stub_push_event(gpu, t, msg.c_str());
  });
#else
  m.attr("STUB") = false;
#endif
}
