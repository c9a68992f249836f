// Native MI355X GPU monitor for per-GPU failure attribution (north star in
// BASELINE.json).  The reference supervisor has no GPU awareness
// at all (/root/reference/services/supervisor.go:137-259 only reads K8s event
// reasons), so this module has no counterpart there.
//
// Two native threads run against the amd-smi C API (libamd_smi):
//   * a sampler (every `interval_ms`): per-GPU VRAM used/total, the KFD process
//     list with per-process VRAM, ECC totals.  It keeps per-GPU and per-PID VRAM
//     *peaks* and, the first time a PID shows up on a GPU, captures its
//     /proc/<pid>/cgroup (→ pod UID) and rank/device env from /proc/<pid>/environ
//     while the process is still alive — after an HBM OOM kill it is gone.
//     Exited processes are retained for `retain_s` seconds so a supervisor that
//     sees the K8s failure later can still read the peak.
//   * an event listener blocked in amdsmi_get_gpu_event_notification: VM faults,
//     queue evictions, GPU pre/post reset, KFD process start/end.
//
// Python reads snapshots under a mutex; neither thread ever takes the GIL.
#include <algorithm>
#include <amd_smi/amdsmi.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
}

const char* event_name(int e) {
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

std::string read_file(const std::string& path, size_t cap = 1 << 16) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return {};
  std::string s;
  s.resize(cap);
  f.read(&s[0], static_cast<std::streamsize>(cap));
  s.resize(static_cast<size_t>(f.gcount()));
  return s;
}

// Rank / device variables worth keeping from a process environment.
bool keep_env_var(const std::string& k) {
  static const char* names[] = {"RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "NODE_RANK",
                                "MASTER_ADDR", "MASTER_PORT", "HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES",
                                "CUDA_VISIBLE_DEVICES", "JOB_COMPLETION_INDEX", "HOSTNAME"};
  for (const char* n : names)
    if (k == n) return true;
  return false;
}

// Pod UID from a cgroup path: kubepods[-burstable|-besteffort]-pod<uid>.slice (systemd
// driver, '_' for '-') or /kubepods/<qos>/pod<uid>/ (cgroupfs driver).
std::string pod_uid_from_cgroup(const std::string& cg) {
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

struct ProcRec {
  uint32_t pid = 0;
  int gpu = -1;
  std::string name;
  uint64_t vram = 0;
  uint64_t peak_vram = 0;
  uint32_t cu_occupancy = 0;
  double first_seen = 0, last_seen = 0;
  bool alive = true;
  std::string cgroup, pod_uid;
  std::map<std::string, std::string> env;
};

struct GpuRec {
  amdsmi_processor_handle h = nullptr;
  int index = 0;
  std::string bdf, uuid, hip_uuid, market_name;
  int hip_id = -1;
  uint32_t vram_total_mb = 0, vram_used_mb = 0, vram_peak_mb = 0;
  uint64_t ecc_correctable = 0, ecc_uncorrectable = 0;
  bool events_ok = false;
  // xGMI fabric health (RCCL's transport between the node's GPUs); -1 = not reported
  int xgmi_links_total = -1, xgmi_links_up = -1, xgmi_links_down = -1;
  int xgmi_error = -1;  // amdsmi_xgmi_status_t
  bool health_seen = false;
};

struct EventRec {
  int gpu;
  std::string type, message;
  double t;
};

std::string status_str(amdsmi_status_t st) {
  const char* s = nullptr;
  if (amdsmi_status_code_to_string(st, &s) == AMDSMI_STATUS_SUCCESS && s) return s;
  return "amdsmi status " + std::to_string(static_cast<int>(st));
}

class GpuMonitor {
 public:
  GpuMonitor(int interval_ms, bool events, double retain_s, bool read_proc)
      : interval_ms_(interval_ms < 1 ? 1 : interval_ms), want_events_(events), retain_s_(retain_s), read_proc_(read_proc) {}

  ~GpuMonitor() { stop(); }

  void start() {
    if (running_) return;
    amdsmi_status_t st = amdsmi_init(AMDSMI_INIT_AMD_GPUS);
    if (st != AMDSMI_STATUS_SUCCESS) throw std::runtime_error("amdsmi_init failed: " + status_str(st));
    inited_ = true;
    discover();
    sample_once();
    running_ = true;
    sampler_ = std::thread([this] { sampler_loop(); });
    if (want_events_) {
      uint64_t mask = 0;
      for (int e : {AMDSMI_EVT_NOTIF_VMFAULT, AMDSMI_EVT_NOTIF_GPU_PRE_RESET, AMDSMI_EVT_NOTIF_GPU_POST_RESET,
                    AMDSMI_EVT_NOTIF_QUEUE_EVICTION, AMDSMI_EVT_NOTIF_QUEUE_RESTORE, AMDSMI_EVT_NOTIF_PROCESS_START,
                    AMDSMI_EVT_NOTIF_PROCESS_END, AMDSMI_EVT_NOTIF_THERMAL_THROTTLE})
        mask |= AMDSMI_EVENT_MASK_FROM_INDEX(e);
      int ok = 0;
      for (auto& g : gpus_) {
        if (amdsmi_init_gpu_event_notification(g.h) == AMDSMI_STATUS_SUCCESS &&
            amdsmi_set_gpu_event_notification_mask(g.h, mask) == AMDSMI_STATUS_SUCCESS) {
          g.events_ok = true;
          ++ok;
        }
      }
      if (ok) listener_ = std::thread([this] { event_loop(); });
    }
  }

  void stop() {
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
    for (auto& g : gpus_)
      if (g.events_ok) amdsmi_stop_gpu_event_notification(g.h);
    amdsmi_shut_down();
    inited_ = false;
  }

  py::list devices() {
    std::lock_guard<std::mutex> lk(mu_);
    py::list out;
    for (auto& g : gpus_) {
      py::dict d;
      d["index"] = g.index;
      d["bdf"] = g.bdf;
      d["uuid"] = g.uuid;
      d["hip_uuid"] = g.hip_uuid;
      d["hip_id"] = g.hip_id;
      d["market_name"] = g.market_name;
      d["vram_total_mb"] = g.vram_total_mb;
      d["events"] = g.events_ok;
      out.append(d);
    }
    return out;
  }

  // Per-GPU snapshot; `include_exited` keeps processes that ended within retain_s.
  py::list snapshot(bool include_exited) {
    std::lock_guard<std::mutex> lk(mu_);
    py::list out;
    for (auto& g : gpus_) {
      py::dict d;
      d["index"] = g.index;
      d["uuid"] = g.uuid;
      d["hip_uuid"] = g.hip_uuid;
      d["bdf"] = g.bdf;
      d["vram_total_mb"] = g.vram_total_mb;
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
      py::list procs;
      for (auto& kv : procs_) {
        const ProcRec& p = kv.second;
        if (p.gpu != g.index || (!p.alive && !include_exited)) continue;
        procs.append(proc_dict(p));
      }
      d["procs"] = procs;
      py::list evs;
      for (auto& e : events_)
        if (e.gpu == g.index) evs.append(event_dict(e));
      d["events"] = evs;
      out.append(d);
    }
    return out;
  }

  py::list drain_events() {
    std::lock_guard<std::mutex> lk(mu_);
    py::list out;
    for (auto& e : pending_events_) out.append(event_dict(e));
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
  // Lets one process own the amd-smi session and forward history to others (shard workers).
  py::list history(int gpu_index, double since) {
    std::vector<std::pair<double, uint32_t>> out;
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (size_t i = 0; i < gpus_.size() && i < hist_.size(); ++i) {
        if (gpus_[i].index != gpu_index) continue;
        for (auto& smp : hist_[i])
          if (smp.first > since) out.push_back(smp);
      }
    }
    py::list l;
    for (auto& smp : out) l.append(py::make_tuple(smp.first, smp.second));
    return l;
  }

  uint64_t samples() const { return samples_.load(); }
  double last_sample_seconds() const { return last_sample_s_.load(); }
  size_t n_gpus() const { return gpus_.size(); }

 private:
  py::dict proc_dict(const ProcRec& p) {
    py::dict d;
    d["pid"] = p.pid;
    d["name"] = p.name;
    d["vram_bytes"] = p.vram;
    d["peak_vram_bytes"] = p.peak_vram;
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

  static py::dict event_dict(const EventRec& e) {
    py::dict d;
    d["gpu"] = e.gpu;
    d["type"] = e.type;
    d["message"] = e.message;
    d["t"] = e.t;
    return d;
  }

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
    std::lock_guard<std::mutex> lk(mu_);
    gpus_.clear();
    for (size_t i = 0; i < handles.size(); ++i) {
      GpuRec g;
      g.h = handles[i];
      g.index = static_cast<int>(i);
      amdsmi_bdf_t bdf;
      if (amdsmi_get_gpu_device_bdf(g.h, &bdf) == AMDSMI_STATUS_SUCCESS) {
        char b[64];
        snprintf(b, sizeof b, "%04llx:%02x:%02x.%x", static_cast<unsigned long long>(bdf.domain_number),
                 static_cast<unsigned>(bdf.bus_number), static_cast<unsigned>(bdf.device_number),
                 static_cast<unsigned>(bdf.function_number));
        g.bdf = b;
      }
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
      gpus_.push_back(g);
    }
  }

  void record_event_locked(const EventRec& e) {
    events_.push_back(e);
    while (events_.size() > 256) events_.pop_front();
    pending_events_.push_back(e);
    while (pending_events_.size() > 4096) pending_events_.pop_front();
  }

  void capture_proc(ProcRec& p) {
    if (!read_proc_) return;
    std::string base = "/proc/" + std::to_string(p.pid);
    p.cgroup = read_file(base + "/cgroup", 4096);
    while (!p.cgroup.empty() && (p.cgroup.back() == '\n')) p.cgroup.pop_back();
    p.pod_uid = pod_uid_from_cgroup(p.cgroup);
    std::string env = read_file(base + "/environ", 1 << 17);
    size_t s = 0;
    while (s < env.size()) {
      size_t e = env.find('\0', s);
      if (e == std::string::npos) e = env.size();
      std::string kv = env.substr(s, e - s);
      size_t eq = kv.find('=');
      if (eq != std::string::npos) {
        std::string k = kv.substr(0, eq);
        if (keep_env_var(k) || k.rfind("NCCL_", 0) == 0 || k.rfind("RCCL_", 0) == 0) p.env[k] = kv.substr(eq + 1);
      }
      s = e + 1;
    }
  }

  void sample_once() {
    std::vector<GpuRec> gs;
    {
      std::lock_guard<std::mutex> lk(mu_);
      gs = gpus_;
    }
    double t = now_s();
    struct Obs {
      int gpu;
      amdsmi_proc_info_t info;
    };
    std::vector<Obs> seen;
    std::vector<amdsmi_vram_usage_t> vram(gs.size());
    std::vector<amdsmi_error_count_t> ecc(gs.size());
    std::vector<bool> vram_ok(gs.size()), ecc_ok(gs.size());
    std::vector<amdsmi_proc_info_t> buf(64);
    // link / fabric health changes slowly: poll it every 10th sample
    const bool health = (samples_.load() % 10) == 0;
    std::vector<amdsmi_xgmi_link_status_t> links(gs.size());
    std::vector<bool> links_ok(gs.size(), false);
    std::vector<int> xerr(gs.size(), -1);
    for (size_t i = 0; i < gs.size(); ++i) {
      if (health) {
        memset(&links[i], 0, sizeof links[i]);
        links_ok[i] = amdsmi_get_gpu_xgmi_link_status(gs[i].h, &links[i]) == AMDSMI_STATUS_SUCCESS;
        amdsmi_xgmi_status_t xs;
        if (amdsmi_gpu_xgmi_error_status(gs[i].h, &xs) == AMDSMI_STATUS_SUCCESS) xerr[i] = static_cast<int>(xs);
      }
      memset(&vram[i], 0, sizeof vram[i]);
      vram_ok[i] = amdsmi_get_gpu_vram_usage(gs[i].h, &vram[i]) == AMDSMI_STATUS_SUCCESS;
      memset(&ecc[i], 0, sizeof ecc[i]);
      ecc_ok[i] = amdsmi_get_gpu_total_ecc_count(gs[i].h, &ecc[i]) == AMDSMI_STATUS_SUCCESS;
      uint32_t n = static_cast<uint32_t>(buf.size());
      amdsmi_status_t st = amdsmi_get_gpu_process_list(gs[i].h, &n, buf.data());
      if (st == AMDSMI_STATUS_OUT_OF_RESOURCES || n > buf.size()) {
        buf.resize(n + 16);
        n = static_cast<uint32_t>(buf.size());
        st = amdsmi_get_gpu_process_list(gs[i].h, &n, buf.data());
      }
      if (st == AMDSMI_STATUS_SUCCESS)
        for (uint32_t k = 0; k < n && k < buf.size(); ++k) seen.push_back(Obs{gs[i].index, buf[k]});
    }
    // /proc reads happen outside the lock, only for PIDs not seen before.
    std::vector<ProcRec> fresh;
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (auto& o : seen) {
        uint64_t key = (static_cast<uint64_t>(o.gpu) << 32) | o.info.pid;
        if (!procs_.count(key)) {
          ProcRec p;
          p.pid = o.info.pid;
          p.gpu = o.gpu;
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
      uint64_t key = (static_cast<uint64_t>(o.gpu) << 32) | o.info.pid;
      ProcRec& p = procs_[key];
      p.alive = true;
      p.last_seen = t;
      p.name = o.info.name;
      uint64_t v = o.info.memory_usage.vram_mem ? o.info.memory_usage.vram_mem : o.info.mem;
      p.vram = v;
      if (v > p.peak_vram) p.peak_vram = v;
      p.cu_occupancy = o.info.cu_occupancy;
    }
    for (auto it = procs_.begin(); it != procs_.end();) {
      if (!it->second.alive && t - it->second.last_seen > retain_s_)
        it = procs_.erase(it);
      else
        ++it;
    }
    if (hist_.size() != gpus_.size()) hist_.resize(gpus_.size());
    const size_t hist_cap = static_cast<size_t>(retain_s_ * 1000.0 / interval_ms_) + 8;
    for (size_t i = 0; i < gs.size() && i < gpus_.size(); ++i) {
      GpuRec& g = gpus_[i];
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
      sample_once();
      lk.lock();
      wake_cv_.wait_for(lk, std::chrono::milliseconds(interval_ms_), [this] { return !running_; });
    }
  }

  void event_loop() {
    std::vector<amdsmi_evt_notification_data_t> buf(32);
    while (running_) {
      uint32_t n = static_cast<uint32_t>(buf.size());
      amdsmi_status_t st = amdsmi_get_gpu_event_notification(200, &n, buf.data());
      if (st != AMDSMI_STATUS_SUCCESS || n == 0) continue;
      double t = now_s();
      std::lock_guard<std::mutex> lk(mu_);
      for (uint32_t i = 0; i < n && i < buf.size(); ++i) {
        int gpu = -1;
        for (auto& g : gpus_)
          if (g.h == buf[i].processor_handle) gpu = g.index;
        record_event_locked(EventRec{gpu, event_name(buf[i].event), buf[i].message, t});
      }
    }
  }

  int interval_ms_;
  bool want_events_;
  double retain_s_;
  bool read_proc_;
  bool inited_ = false;
  std::atomic<bool> running_{false};
  std::thread sampler_, listener_;
  std::mutex mu_, wake_mu_;
  std::condition_variable wake_cv_;
  std::vector<GpuRec> gpus_;
  std::vector<std::deque<std::pair<double, uint32_t>>> hist_;  // per-GPU (t, vram_used_mb) samples
  std::unordered_map<uint64_t, ProcRec> procs_;
  std::deque<EventRec> events_, pending_events_;
  std::atomic<uint64_t> samples_{0};
  std::atomic<double> last_sample_s_{0};
};

}  // namespace

PYBIND11_MODULE(_amdsmi_monitor, m) {
  m.doc() = "Native amd-smi GPU monitor: VRAM peaks, per-process attribution, GPU event listener";
  m.def("pod_uid_from_cgroup", &pod_uid_from_cgroup, "Extract a K8s pod UID from a /proc/<pid>/cgroup text");
  py::class_<GpuMonitor>(m, "GpuMonitor")
      .def(py::init<int, bool, double, bool>(), py::arg("interval_ms") = 250, py::arg("events") = true,
           py::arg("retain_s") = 600.0, py::arg("read_proc") = true)
      .def("start", &GpuMonitor::start, py::call_guard<py::gil_scoped_release>())
      .def("stop", &GpuMonitor::stop, py::call_guard<py::gil_scoped_release>())
      .def("devices", &GpuMonitor::devices)
      .def("snapshot", &GpuMonitor::snapshot, py::arg("include_exited") = true)
      .def("drain_events", &GpuMonitor::drain_events)
      .def("inject_event", &GpuMonitor::inject_event)
      .def("reset_peaks", &GpuMonitor::reset_peaks)
      .def("peak_between", &GpuMonitor::peak_between)
      .def("history", &GpuMonitor::history, py::arg("gpu_index"), py::arg("since") = 0.0)
      .def_property_readonly("samples", &GpuMonitor::samples)
      .def_property_readonly("last_sample", &GpuMonitor::last_sample_seconds)
      .def_property_readonly("n_gpus", &GpuMonitor::n_gpus);
}
