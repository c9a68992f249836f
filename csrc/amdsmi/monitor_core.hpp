// Native MI355X GPU monitor core for per-GPU failure attribution (north star in
// BASELINE.json).  The reference supervisor has no GPU awareness at all
// (/root/reference/services/supervisor.go:137-259 only reads K8s event reasons), so
// this module has no counterpart there.
//
// Two native threads run against the amd-smi C API (libamd_smi):
//   * a sampler (every `interval_ms`): per-GPU VRAM used/total, ECC totals, xGMI link
//     status + per-link traffic, and the processes on each GPU with their VRAM.  It
//     keeps per-GPU and per-PID VRAM *peaks* and, the first time a PID shows up on a GPU,
//     captures its /proc/<pid>/cgroup (→ pod UID) and rank/device env from
//     /proc/<pid>/environ while the process is still alive — after an HBM OOM kill it is
//     gone.  Exited processes are retained for `retain_s` seconds.
//   * an event listener blocked in amdsmi_get_gpu_event_notification: VM faults, queue
//     evictions, GPU pre/post reset, KFD process start/end.
//
// Process sources (procscan.hpp), chosen by PID namespace: with hostPID (the node
// agent) amd-smi's list, with KFD sysfs filling in VRAM amd-smi could not read; in a
// private PID namespace (a container without hostPID, as on the gpurun box) amd-smi's
// PIDs are *host* PIDs that mean other processes here, so they are only tallied as
// foreign usage and the processes come from DRM fdinfo of our own /proc instead.
//
// xGMI: at discovery each GPU's hive id and physical links (peer BDF, type, bit rate,
// max bandwidth) are read with amdsmi_get_link_metrics; the health poll refreshes the
// link status and the per-link read/write counters.  That is the real fabric the
// supervised job's RCCL ring ran on, recorded in the trace row.
//
// This header holds no Python types: the pybind module (gpu_monitor.cpp) converts the
// plain snapshots, and the TSan self-test (monitor_selftest.cpp) drives the same class
// against a stub amd-smi (amdsmi_stub.cpp).
#pragma once

#include <amd_smi/amdsmi.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "procscan.hpp"
#include "stderr_filter.hpp"

namespace nexus_gpu {

inline double now_s() {
  return std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
}

inline const char* event_name(int e) {
  switch (e) {
    case AMDSMI_EVT_NOTIF_VMFAULT: return "VMFAULT";
    case AMDSMI_EVT_NOTIF_THERMAL_THROTTLE: return "THERMAL_THROTTLE";
    case AMDSMI_EVT_NOTIF_GPU_PRE_RESET: return "GPU_PRE_RESET";
    case AMDSMI_EVT_NOTIF_GPU_POST_RESET: return "GPU_POST_RESET";
    case AMDSMI_EVT_NOTIF_MIGRATE_START: return "MIGRATE_START";
    case AMDSMI_EVT_NOTIF_MIGRATE_END: return "MIGRATE_END";
    case AMDSMI_EVT_NOTIF_PAGE_FAULT_START: return "PAGE_FAULT_START";
    case AMDSMI_EVT_NOTIF_PAGE_FAULT_END: return "PAGE_FAULT_END";
    case AMDSMI_EVT_NOTIF_QUEUE_EVICTION: return "QUEUE_EVICTION";
    case AMDSMI_EVT_NOTIF_QUEUE_RESTORE: return "QUEUE_RESTORE";
    case AMDSMI_EVT_NOTIF_UNMAP_FROM_GPU: return "UNMAP_FROM_GPU";
    case AMDSMI_EVT_NOTIF_PROCESS_START: return "PROCESS_START";
    case AMDSMI_EVT_NOTIF_PROCESS_END: return "PROCESS_END";
    default: return "NONE";
  }
}

inline const char* link_type_name(int t) {
  switch (t) {
    case AMDSMI_LINK_TYPE_INTERNAL: return "internal";
    case AMDSMI_LINK_TYPE_PCIE: return "pcie";
    case AMDSMI_LINK_TYPE_XGMI: return "xgmi";
    case AMDSMI_LINK_TYPE_NOT_APPLICABLE: return "n/a";
    default: return "unknown";
  }
}

// Rank / device variables worth keeping from a process environment.
inline bool keep_env_var(const std::string& k) {
  static const char* names[] = {"RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "NODE_RANK",
                                "MASTER_ADDR", "MASTER_PORT", "HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES",
                                "CUDA_VISIBLE_DEVICES", "GPU_DEVICE_ORDINAL", "JOB_COMPLETION_INDEX", "HOSTNAME"};
  for (const char* n : names)
    if (k == n) return true;
  // the collective families models/kube.py ENV_PREFIXES keeps from pod specs
  static const char* prefixes[] = {"NCCL_", "RCCL_", "TORCH_NCCL_", "HSA_", "MSCCL", "UCX_"};
  for (const char* p : prefixes)
    if (k.rfind(p, 0) == 0) return true;
  return false;
}

// Pod UID from a cgroup path: kubepods[-burstable|-besteffort]-pod<uid>.slice (systemd
// driver, '_' for '-') or /kubepods/<qos>/pod<uid>/ (cgroupfs driver).
inline std::string pod_uid_from_cgroup(const std::string& cg) {
  size_t p = 0;
  while ((p = cg.find("pod", p)) != std::string::npos) {
    size_t s = p + 3;
    size_t e = s;
    while (e < cg.size() && (isxdigit(static_cast<unsigned char>(cg[e])) || cg[e] == '-' || cg[e] == '_')) ++e;
    if (e - s >= 32) {
      std::string uid = cg.substr(s, e - s);
      for (auto& c : uid)
        if (c == '_') c = '-';
      return uid;
    }
    p = s;
  }
  return {};
}

inline std::string bdf_string(const amdsmi_bdf_t& bdf) {
  char b[64];
  snprintf(b, sizeof b, "%04llx:%02x:%02x.%x", static_cast<unsigned long long>(bdf.domain_number),
           static_cast<unsigned>(bdf.bus_number), static_cast<unsigned>(bdf.device_number),
           static_cast<unsigned>(bdf.function_number));
  return b;
}

inline std::string status_str(amdsmi_status_t st) {
  const char* s = nullptr;
  if (amdsmi_status_code_to_string(st, &s) == AMDSMI_STATUS_SUCCESS && s) return s;
  return "amdsmi status " + std::to_string(static_cast<int>(st));
}

struct ProcRec {
  uint32_t pid = 0;
  int gpu = -1;
  std::string name, source;
  uint64_t vram = 0, peak_vram = 0, gtt = 0;
  uint32_t cu_occupancy = 0;
  double first_seen = 0, last_seen = 0;
  bool alive = true;
  std::string cgroup, pod_uid;
  std::map<std::string, std::string> env;
};

struct LinkRec {
  std::string peer_bdf;
  int peer_index = -1;  // index of the peer among this monitor's GPUs; -1 = not visible here
  int type = AMDSMI_LINK_TYPE_UNKNOWN;
  uint32_t bit_rate = 0, max_bandwidth = 0;  // Gb/s
  uint64_t read_kb = 0, write_kb = 0;
};

struct GpuRec {
  amdsmi_processor_handle h = nullptr;
  int index = 0;
  std::string bdf, uuid, hip_uuid, market_name;
  int hip_id = -1;
  uint64_t kfd_id = 0, hive_id = 0, xgmi_node_id = 0;
  uint32_t vram_total_mb = 0, vram_used_mb = 0, vram_peak_mb = 0;
  uint64_t ecc_correctable = 0, ecc_uncorrectable = 0;
  bool events_ok = false;
  int xgmi_links_total = -1, xgmi_links_up = -1, xgmi_links_down = -1;
  int xgmi_error = -1;  // amdsmi_xgmi_status_t
  bool health_seen = false;
  std::vector<LinkRec> links;
  // processes on this GPU that belong to another PID namespace (host PIDs seen from a
  // container): counted, never attributed
  uint32_t foreign_procs = 0;
  uint64_t foreign_vram = 0;
};

struct EventRec {
  int gpu;
  std::string type, message;
  double t;
};

struct GpuView {
  GpuRec gpu;
  std::vector<ProcRec> procs;
  std::vector<EventRec> events;
};

struct MonitorOptions {
  int interval_ms = 250;
  bool events = true;
  double retain_s = 600.0;
  bool read_proc = true;
  std::string proc_source = "auto";  // auto | amdsmi | kfd | drm
  std::string proc_root = "/proc";
  std::string sys_root = "/sys";
  int health_every = 10;             // samples between link / ECC-health polls
};

class GpuMonitor {
 public:
  explicit GpuMonitor(MonitorOptions o) : o_(std::move(o)), drm_(o_.proc_root, 8) {
    if (o_.interval_ms < 1) o_.interval_ms = 1;
    if (o_.health_every < 1) o_.health_every = 1;
  }
  ~GpuMonitor() { stop(); }

  void start() {
    std::lock_guard<std::mutex> life(life_mu_);
    if (running_) return;
    amdsmi_status_t st = amdsmi_init(AMDSMI_INIT_AMD_GPUS);
    if (st != AMDSMI_STATUS_SUCCESS) throw std::runtime_error("amdsmi_init failed: " + status_str(st));
    inited_ = true;
    {
      std::lock_guard<std::mutex> lk(mu_);
      host_ns_ = host_pid_namespace(o_.proc_root);
      mode_ = o_.proc_source;
      if (mode_ == "auto") mode_ = host_ns_ ? "amdsmi" : "drm";
    }
    discover();
    bool listen = false;
    if (o_.events) {
      uint64_t mask = 0;
      for (int e : {AMDSMI_EVT_NOTIF_VMFAULT, AMDSMI_EVT_NOTIF_GPU_PRE_RESET, AMDSMI_EVT_NOTIF_GPU_POST_RESET,
                    AMDSMI_EVT_NOTIF_QUEUE_EVICTION, AMDSMI_EVT_NOTIF_QUEUE_RESTORE, AMDSMI_EVT_NOTIF_PROCESS_START,
                    AMDSMI_EVT_NOTIF_PROCESS_END, AMDSMI_EVT_NOTIF_THERMAL_THROTTLE})
        mask |= AMDSMI_EVENT_MASK_FROM_INDEX(e);
      // registered before either thread starts; the flags are published under mu_
      std::lock_guard<std::mutex> lk(mu_);
      for (auto& g : gpus_) {
        g.events_ok = amdsmi_init_gpu_event_notification(g.h) == AMDSMI_STATUS_SUCCESS &&
                      amdsmi_set_gpu_event_notification_mask(g.h, mask) == AMDSMI_STATUS_SUCCESS;
        listen = listen || g.events_ok;
      }
    }
    sample_once();
    running_ = true;
    sampler_ = std::thread([this] { sampler_loop(); });
    if (listen) listener_ = std::thread([this] { event_loop(); });
  }

  void stop() {
    std::lock_guard<std::mutex> life(life_mu_);
    if (!running_) {
      if (inited_) {
        amdsmi_shut_down();
        inited_ = false;
      }
      return;
    }
    {
      std::lock_guard<std::mutex> lk(wake_mu_);
      running_ = false;
    }
    wake_cv_.notify_all();
    if (sampler_.joinable()) sampler_.join();
    if (listener_.joinable()) listener_.join();
    Fd2Filter::instance().flush();  // a write still in flight at the last swap back
    std::vector<amdsmi_processor_handle> registered;
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (auto& g : gpus_)
        if (g.events_ok) registered.push_back(g.h);
    }
    for (auto h : registered) amdsmi_stop_gpu_event_notification(h);
    amdsmi_shut_down();
    inited_ = false;
  }

  std::vector<GpuRec> devices() {
    std::lock_guard<std::mutex> lk(mu_);
    return gpus_;
  }

  // Per-GPU snapshot (copies, taken under the lock); `include_exited` keeps processes
  // that ended within retain_s.
  std::vector<GpuView> snapshot(bool include_exited) {
    std::lock_guard<std::mutex> lk(mu_);
    std::vector<GpuView> out;
    out.reserve(gpus_.size());
    for (auto& g : gpus_) {
      GpuView v;
      v.gpu = g;
      for (auto& kv : procs_)
        if (kv.second.gpu == g.index && (kv.second.alive || include_exited)) v.procs.push_back(kv.second);
      for (auto& e : events_)
        if (e.gpu == g.index) v.events.push_back(e);
      out.push_back(std::move(v));
    }
    return out;
  }

  std::vector<EventRec> drain_events() {
    std::lock_guard<std::mutex> lk(mu_);
    std::vector<EventRec> out(pending_events_.begin(), pending_events_.end());
    pending_events_.clear();
    return out;
  }

  // Inject a synthetic event (tests / chaos): goes through the same bookkeeping.
  void inject_event(int gpu, const std::string& type, const std::string& message) {
    std::lock_guard<std::mutex> lk(mu_);
    record_event_locked(EventRec{gpu, type, message, now_s()});
  }

  void reset_peaks() {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& g : gpus_) g.vram_peak_mb = g.vram_used_mb;
    for (auto& kv : procs_) kv.second.peak_vram = kv.second.vram;
  }

  // Device-wide VRAM peak (MB) among samples taken in [t0, t1] — the window a pod's
  // processes were alive; a lifetime peak would blame every later failure on an old OOM.
  uint32_t peak_between(int gpu_index, double t0, double t1) {
    std::lock_guard<std::mutex> lk(mu_);
    uint32_t peak = 0;
    for (size_t i = 0; i < gpus_.size() && i < hist_.size(); ++i) {
      if (gpus_[i].index != gpu_index) continue;
      for (auto& s : hist_[i])
        if (s.first >= t0 && s.first <= t1 && s.second > peak) peak = s.second;
    }
    return peak;
  }

  // VRAM samples of one GPU taken after `since` (seconds, wall clock): [(t, vram_used_mb)].
  std::vector<std::pair<double, uint32_t>> history(int gpu_index, double since) {
    std::vector<std::pair<double, uint32_t>> out;
    std::lock_guard<std::mutex> lk(mu_);
    for (size_t i = 0; i < gpus_.size() && i < hist_.size(); ++i) {
      if (gpus_[i].index != gpu_index) continue;
      for (auto& smp : hist_[i])
        if (smp.first > since) out.push_back(smp);
    }
    return out;
  }

  uint64_t samples() const { return samples_.load(); }
  // processes amd-smi could not read because they exited while it listed them
  uint64_t process_vanished() const { return vanished_.load(); }
  double last_sample_seconds() const { return last_sample_s_.load(); }
  size_t n_gpus() {
    std::lock_guard<std::mutex> lk(mu_);
    return gpus_.size();
  }
  std::string proc_mode() {
    std::lock_guard<std::mutex> lk(mu_);
    return mode_;
  }
  bool host_pid_ns() {
    std::lock_guard<std::mutex> lk(mu_);
    return host_ns_;
  }

 private:
  void discover() {
    uint32_t nsock = 0;
    amdsmi_status_t st = amdsmi_get_socket_handles(&nsock, nullptr);
    if (st != AMDSMI_STATUS_SUCCESS) throw std::runtime_error("amdsmi_get_socket_handles: " + status_str(st));
    std::vector<amdsmi_socket_handle> socks(nsock);
    amdsmi_get_socket_handles(&nsock, socks.data());
    std::vector<amdsmi_processor_handle> handles;
    for (auto s : socks) {
      uint32_t n = 0;
      if (amdsmi_get_processor_handles(s, &n, nullptr) != AMDSMI_STATUS_SUCCESS) continue;
      std::vector<amdsmi_processor_handle> hs(n);
      amdsmi_get_processor_handles(s, &n, hs.data());
      handles.insert(handles.end(), hs.begin(), hs.begin() + n);
    }
    std::vector<GpuRec> gs;
    for (size_t i = 0; i < handles.size(); ++i) {
      GpuRec g;
      g.h = handles[i];
      g.index = static_cast<int>(i);
      amdsmi_bdf_t bdf;
      if (amdsmi_get_gpu_device_bdf(g.h, &bdf) == AMDSMI_STATUS_SUCCESS) g.bdf = bdf_string(bdf);
      char uuid[AMDSMI_GPU_UUID_SIZE] = {0};
      unsigned int ul = AMDSMI_GPU_UUID_SIZE;
      if (amdsmi_get_gpu_device_uuid(g.h, &ul, uuid) == AMDSMI_STATUS_SUCCESS) g.uuid = uuid;
      amdsmi_enumeration_info_t en;
      memset(&en, 0, sizeof en);
      if (amdsmi_get_gpu_enumeration_info(g.h, &en) == AMDSMI_STATUS_SUCCESS) {
        g.hip_id = static_cast<int>(en.hip_id);
        g.hip_uuid = en.hip_uuid;
        g.index = static_cast<int>(en.hip_id);  // hip enumeration order == HIP_VISIBLE_DEVICES numbering
      }
      amdsmi_asic_info_t asic;
      memset(&asic, 0, sizeof asic);
      if (amdsmi_get_gpu_asic_info(g.h, &asic) == AMDSMI_STATUS_SUCCESS) g.market_name = asic.market_name;
      amdsmi_kfd_info_t kfd;
      memset(&kfd, 0, sizeof kfd);
      if (amdsmi_get_gpu_kfd_info(g.h, &kfd) == AMDSMI_STATUS_SUCCESS && kfd.kfd_id != ~0ULL) g.kfd_id = kfd.kfd_id;
      amdsmi_xgmi_info_t xi;
      memset(&xi, 0, sizeof xi);
      if (amdsmi_get_xgmi_info(g.h, &xi) == AMDSMI_STATUS_SUCCESS) {
        g.hive_id = xi.xgmi_hive_id;
        g.xgmi_node_id = xi.xgmi_node_id;
      }
      read_links(g, true);
      gs.push_back(g);
    }
    for (auto& g : gs)
      for (auto& l : g.links)
        for (auto& p : gs)
          if (p.bdf == l.peer_bdf) l.peer_index = p.index;
    std::lock_guard<std::mutex> lk(mu_);
    gpus_ = std::move(gs);
    bdf_index_.clear();
    for (auto& g : gpus_) bdf_index_[lower(g.bdf)] = g.index;
  }

  // Physical links of one GPU.  `structure` re-reads peers / rates; otherwise only the
  // counters of the already-known links are refreshed (positionally, same API order).
  static void read_links(GpuRec& g, bool structure) {
    amdsmi_link_metrics_t lm;
    memset(&lm, 0, sizeof lm);
    if (amdsmi_get_link_metrics(g.h, &lm) != AMDSMI_STATUS_SUCCESS) return;
    uint32_t n = std::min<uint32_t>(lm.num_links, AMDSMI_MAX_NUM_XGMI_PHYSICAL_LINK);
    if (structure) {
      g.links.clear();
      for (uint32_t k = 0; k < n; ++k) {
        const auto& s = lm.links[k];
        LinkRec l;
        l.peer_bdf = lower(bdf_string(s.bdf));
        l.type = static_cast<int>(s.link_type);
        l.bit_rate = s.bit_rate;
        l.max_bandwidth = s.max_bandwidth;
        l.read_kb = s.read;
        l.write_kb = s.write;
        g.links.push_back(l);
      }
      return;
    }
    for (uint32_t k = 0; k < n && k < g.links.size(); ++k) {
      g.links[k].read_kb = lm.links[k].read;
      g.links[k].write_kb = lm.links[k].write;
      g.links[k].bit_rate = lm.links[k].bit_rate;
    }
  }

  void record_event_locked(const EventRec& e) {
    events_.push_back(e);
    while (events_.size() > 256) events_.pop_front();
    pending_events_.push_back(e);
    while (pending_events_.size() > 4096) pending_events_.pop_front();
  }

  void capture_proc(ProcRec& p) const {
    if (!o_.read_proc) return;
    std::string base = o_.proc_root + "/" + std::to_string(p.pid);
    p.cgroup = read_small(base + "/cgroup", 4096);
    while (!p.cgroup.empty() && (p.cgroup.back() == '\n')) p.cgroup.pop_back();
    p.pod_uid = pod_uid_from_cgroup(p.cgroup);
    if (p.name.empty() || p.name == "N/A") {
      p.name = read_small(base + "/comm", 64);
      while (!p.name.empty() && p.name.back() == '\n') p.name.pop_back();
    }
    std::string env = read_small(base + "/environ", 1 << 17, kDenyEnviron);
    size_t s = 0;
    while (s < env.size()) {
      size_t e = env.find('\0', s);
      if (e == std::string::npos) e = env.size();
      size_t eq = env.find('=', s);
      if (eq != std::string::npos && eq < e) {
        std::string k = env.substr(s, eq - s);
        if (keep_env_var(k)) p.env[k] = env.substr(eq + 1, e - eq - 1);
      }
      s = e + 1;
    }
  }

  struct Obs {
    int gpu;
    uint32_t pid;
    std::string name, source;
    uint64_t vram, gtt;
    uint32_t cu;
  };

  void sample_once() {
    std::vector<GpuRec> gs;
    std::unordered_map<std::string, int> bdf_index;
    std::string mode;
    bool host_ns;
    {
      std::lock_guard<std::mutex> lk(mu_);
      gs = gpus_;
      bdf_index = bdf_index_;
      mode = mode_;
      host_ns = host_ns_;
    }
    double t = now_s();
    std::vector<Obs> seen;
    std::vector<amdsmi_vram_usage_t> vram(gs.size());
    std::vector<amdsmi_error_count_t> ecc(gs.size());
    std::vector<bool> vram_ok(gs.size()), ecc_ok(gs.size());
    std::vector<uint32_t> foreign_n(gs.size(), 0);
    std::vector<uint64_t> foreign_v(gs.size(), 0);
    std::vector<amdsmi_proc_info_t> buf(64);
    const bool health = (samples_.load() % static_cast<uint64_t>(o_.health_every)) == 0;
    std::vector<amdsmi_xgmi_link_status_t> links(gs.size());
    std::vector<bool> links_ok(gs.size(), false);
    std::vector<int> xerr(gs.size(), -1);
    bool smi_listed = false;
    for (size_t i = 0; i < gs.size(); ++i) {
      if (health) {
        memset(&links[i], 0, sizeof links[i]);
        links_ok[i] = amdsmi_get_gpu_xgmi_link_status(gs[i].h, &links[i]) == AMDSMI_STATUS_SUCCESS;
        amdsmi_xgmi_status_t xs;
        if (amdsmi_gpu_xgmi_error_status(gs[i].h, &xs) == AMDSMI_STATUS_SUCCESS) xerr[i] = static_cast<int>(xs);
        read_links(gs[i], false);
      }
      memset(&vram[i], 0, sizeof vram[i]);
      vram_ok[i] = amdsmi_get_gpu_vram_usage(gs[i].h, &vram[i]) == AMDSMI_STATUS_SUCCESS;
      memset(&ecc[i], 0, sizeof ecc[i]);
      ecc_ok[i] = amdsmi_get_gpu_total_ecc_count(gs[i].h, &ecc[i]) == AMDSMI_STATUS_SUCCESS;
      if (mode == "kfd") continue;
      uint32_t n = static_cast<uint32_t>(buf.size());
      amdsmi_status_t st = AMDSMI_STATUS_SUCCESS;
      // libamd_smi prints a line to stderr per process that exits mid-listing: counted
      // (gpu_process_vanished), not printed (stderr_filter.hpp)
      auto& fd2 = Fd2Filter::instance();
      vanished_ += fd2.run([&] { st = amdsmi_get_gpu_process_list(gs[i].h, &n, buf.data()); });
      if (st == AMDSMI_STATUS_OUT_OF_RESOURCES || n > buf.size()) {
        buf.resize(std::min<uint32_t>(n, 4096) + 16);  // a count read while processes exit: bounded
        n = static_cast<uint32_t>(buf.size());
        vanished_ += fd2.run([&] { st = amdsmi_get_gpu_process_list(gs[i].h, &n, buf.data()); });
      }
      if (st != AMDSMI_STATUS_SUCCESS) continue;
      for (uint32_t k = 0; k < n && k < buf.size(); ++k) {
        const auto& pi = buf[k];
        uint64_t v = pi.memory_usage.vram_mem ? pi.memory_usage.vram_mem : pi.mem;
        if (!host_ns && mode != "amdsmi") {  // host PIDs seen from a private namespace
          ++foreign_n[i];
          foreign_v[i] += v;
          continue;
        }
        smi_listed = true;
        seen.push_back(Obs{gs[i].index, static_cast<uint32_t>(pi.pid), std::string(pi.name, strnlen(pi.name, sizeof pi.name)),
                           "amdsmi", v, pi.memory_usage.gtt_mem, pi.cu_occupancy});
      }
    }
    if (mode == "drm") {
      for (auto& u : drm_.scan()) {
        auto it = bdf_index.find(u.bdf);
        if (it != bdf_index.end())
          seen.push_back(Obs{it->second, u.pid, "", "drm-fdinfo", u.vram_bytes, u.gtt_bytes, 0});
      }
    } else if (host_ns || mode == "kfd") {
      // KFD sysfs: the only source in kfd mode; in amdsmi mode it fills in VRAM amd-smi
      // reported as 0 ("Unable to open queues directory") and processes it missed.
      if (kfd_bdfs_.empty() || health) kfd_bdfs_ = kfd_gpu_bdfs(o_.sys_root);
      std::map<std::pair<int, uint32_t>, size_t> at;
      for (size_t k = 0; k < seen.size(); ++k) at[{seen[k].gpu, seen[k].pid}] = k;
      for (auto& u : kfd_proc_usage(o_.sys_root, kfd_bdfs_)) {
        auto it = bdf_index.find(u.bdf);
        if (it == bdf_index.end()) continue;
        auto j = at.find({it->second, u.pid});
        if (j != at.end()) {
          if (!seen[j->second].vram) seen[j->second].vram = u.vram_bytes;
        } else if (mode == "kfd" || !smi_listed || u.vram_bytes) {
          seen.push_back(Obs{it->second, u.pid, "", "kfd", u.vram_bytes, 0, 0});
        }
      }
    }
    // /proc reads happen outside the lock, only for PIDs not seen before.
    std::vector<ProcRec> fresh;
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (auto& o : seen) {
        uint64_t key = (static_cast<uint64_t>(o.gpu) << 32) | o.pid;
        if (!procs_.count(key)) {
          ProcRec p;
          p.pid = o.pid;
          p.gpu = o.gpu;
          p.name = o.name;
          fresh.push_back(p);
        }
      }
    }
    for (auto& p : fresh) capture_proc(p);
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& p : fresh) {
      uint64_t key = (static_cast<uint64_t>(p.gpu) << 32) | p.pid;
      p.first_seen = t;
      procs_.emplace(key, std::move(p));
    }
    for (auto& kv : procs_) kv.second.alive = false;
    for (auto& o : seen) {
      uint64_t key = (static_cast<uint64_t>(o.gpu) << 32) | o.pid;
      ProcRec& p = procs_[key];
      p.alive = true;
      p.last_seen = t;
      if (!o.name.empty() && o.name != "N/A") p.name = o.name;
      p.source = o.source;
      p.vram = o.vram;
      p.gtt = o.gtt;
      if (o.vram > p.peak_vram) p.peak_vram = o.vram;
      p.cu_occupancy = o.cu;
    }
    for (auto it = procs_.begin(); it != procs_.end();) {
      if (!it->second.alive && t - it->second.last_seen > o_.retain_s)
        it = procs_.erase(it);
      else
        ++it;
    }
    if (hist_.size() != gpus_.size()) hist_.resize(gpus_.size());
    const size_t hist_cap = static_cast<size_t>(o_.retain_s * 1000.0 / o_.interval_ms) + 8;
    for (size_t i = 0; i < gs.size() && i < gpus_.size(); ++i) {
      GpuRec& g = gpus_[i];
      g.foreign_procs = foreign_n[i];
      g.foreign_vram = foreign_v[i];
      if (vram_ok[i]) {
        g.vram_total_mb = vram[i].vram_total;
        g.vram_used_mb = vram[i].vram_used;
        if (g.vram_used_mb > g.vram_peak_mb) g.vram_peak_mb = g.vram_used_mb;
        hist_[i].emplace_back(t, g.vram_used_mb);
        while (hist_[i].size() > hist_cap) hist_[i].pop_front();
      }
      if (ecc_ok[i]) {
        if (g.health_seen && ecc[i].uncorrectable_count > g.ecc_uncorrectable)
          record_event_locked(EventRec{g.index, "ECC_UNCORRECTABLE",
                                       std::to_string(ecc[i].uncorrectable_count - g.ecc_uncorrectable) +
                                           " new uncorrectable ECC error(s)", t});
        g.ecc_correctable = ecc[i].correctable_count;
        g.ecc_uncorrectable = ecc[i].uncorrectable_count;
      }
      if (health) {
        for (size_t k = 0; k < g.links.size() && k < gs[i].links.size(); ++k) {
          g.links[k].read_kb = gs[i].links[k].read_kb;
          g.links[k].write_kb = gs[i].links[k].write_kb;
          g.links[k].bit_rate = gs[i].links[k].bit_rate;
        }
        if (links_ok[i]) {
          uint32_t n = std::min<uint32_t>(links[i].total_links, AMDSMI_MAX_NUM_XGMI_LINKS);
          int up = 0, down = 0;
          for (uint32_t k = 0; k < n; ++k) {
            if (links[i].status[k] == AMDSMI_XGMI_LINK_UP) ++up;
            else if (links[i].status[k] == AMDSMI_XGMI_LINK_DOWN) ++down;
          }
          if (g.health_seen && g.xgmi_links_down >= 0 && down > g.xgmi_links_down)
            record_event_locked(EventRec{g.index, "XGMI_LINK_DOWN",
                                         std::to_string(down) + "/" + std::to_string(n) + " xGMI links down", t});
          g.xgmi_links_total = static_cast<int>(n);
          g.xgmi_links_up = up;
          g.xgmi_links_down = down;
        }
        if (xerr[i] >= 0) {
          if (g.health_seen && xerr[i] > 0 && g.xgmi_error == 0)
            record_event_locked(EventRec{g.index, "XGMI_ERROR", "xGMI error status " + std::to_string(xerr[i]), t});
          g.xgmi_error = xerr[i];
        }
        g.health_seen = true;
      }
    }
    samples_.fetch_add(1);
    last_sample_s_.store(t);
  }

  void sampler_loop() {
    std::unique_lock<std::mutex> lk(wake_mu_);
    while (running_) {
      lk.unlock();
      // a sampler thread must never take the process down: an exception escaping a
      // std::thread is std::terminate (abort) — count it and sample again next tick
      try {
        sample_once();
      } catch (...) {
        sample_errors_.fetch_add(1);
      }
      lk.lock();
      // system_clock deadline → pthread_cond_timedwait: a steady_clock wait_for compiles to
      // pthread_cond_clockwait, which GCC 11's TSan runtime does not intercept (it then
      // reports the re-lock as a double lock).  A wall-clock jump only stretches one sample.
      wake_cv_.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(o_.interval_ms),
                          [this] { return !running_; });
    }
  }

  void event_loop() {
    std::vector<amdsmi_evt_notification_data_t> buf(32);
    std::vector<std::pair<amdsmi_processor_handle, int>> handles;
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (auto& g : gpus_) handles.emplace_back(g.h, g.index);
    }
    while (running_) {
      uint32_t n = static_cast<uint32_t>(buf.size());
      amdsmi_status_t st = amdsmi_get_gpu_event_notification(200, &n, buf.data());
      if (st != AMDSMI_STATUS_SUCCESS || n == 0) continue;
      double t = now_s();
      try {
        std::lock_guard<std::mutex> lk(mu_);
        for (uint32_t i = 0; i < n && i < buf.size(); ++i) {
          int gpu = -1;
          for (auto& h : handles)
            if (h.first == buf[i].processor_handle) gpu = h.second;
          record_event_locked(EventRec{gpu, event_name(buf[i].event),
                                       std::string(buf[i].message, strnlen(buf[i].message, sizeof buf[i].message)), t});
        }
      } catch (...) {  // as in the sampler: never std::terminate from a monitor thread
        sample_errors_.fetch_add(1);
      }
    }
  }

  MonitorOptions o_;
  DrmScanner drm_;                          // sampler thread only
  std::map<uint32_t, std::string> kfd_bdfs_;  // sampler thread only
  bool inited_ = false;
  bool host_ns_ = false;
  std::string mode_;
  std::atomic<bool> running_{false};
  std::thread sampler_, listener_;
  std::mutex mu_, wake_mu_, life_mu_;
  std::condition_variable wake_cv_;
  std::vector<GpuRec> gpus_;
  std::unordered_map<std::string, int> bdf_index_;
  std::vector<std::deque<std::pair<double, uint32_t>>> hist_;  // per-GPU (t, vram_used_mb) samples
  std::unordered_map<uint64_t, ProcRec> procs_;
  std::deque<EventRec> events_, pending_events_;
  std::atomic<uint64_t> samples_{0};
  std::atomic<uint64_t> vanished_{0};
  std::atomic<uint64_t> sample_errors_{0};  // exceptions caught in the monitor threads
  std::atomic<double> last_sample_s_{0};
};

}  // namespace nexus_gpu
