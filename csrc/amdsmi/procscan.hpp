// Per-process GPU attribution sources that do not depend on amd-smi's process list
// (on an MI355X box amd-smi reported host-namespace PIDs with zero VRAM, so PID→GPU
// never matched from its process list alone).  Three sources, all plain file reads:
//
//   * DRM fdinfo (`/proc/<pid>/fdinfo/<fd>` of an amdgpu render node): `drm-pdev`
//     (PCI BDF of the GPU) and `drm-memory-vram` / `drm-total-vram` (KiB) per DRM
//     client.  PIDs are those of the reader's own PID namespace, so this is the
//     source that works inside a container without hostPID.
//   * KFD sysfs (`/sys/class/kfd/kfd/proc/<pid>/vram_<gpu_id>`, bytes): what amd-smi
//     reads itself.  sysfs is not PID-namespaced: the directory names are
//     init-namespace PIDs, so it is only usable when the reader shares that namespace.
//   * KFD topology (`/sys/class/kfd/kfd/topology/nodes/<n>/{gpu_id,properties}`):
//     gpu_id → PCI BDF (`domain` + `location_id` = bus<<8 | dev<<3 | fn).
//
// Everything here is pure string / file handling with an injectable root directory,
// so the CPU test suite drives it against a fake procfs / sysfs tree.  No amd-smi,
// no Python.  No counterpart in the reference (it has no GPU awareness).
#pragma once

#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <set>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace nexus_gpu {

// Inode of the initial PID namespace (PROC_PID_INIT_INO in the kernel).
constexpr unsigned long long kInitPidNsIno = 0xEFFFFFFCULL;

// Reads refused by the kernel (EACCES / EPERM), per source.  An agent without the
// privileges it needs — a non-root UID gets no effective capabilities even in a privileged
// container — cannot open another user's /proc/<pid>/fd, fdinfo or environ (ptrace-read
// check) and attribution silently degrades; these counters make that loud (the node
// agent exports them as agent_proc_scan_denied{source} and logs the first one).
enum DenySource { kDenyFdDir = 0, kDenyFdInfo, kDenyEnviron, kDenyProcMeta, kDenySysfs, kDenySources };
inline const char* deny_source_name(int k) {
  static const char* const names[kDenySources] = {"fd", "fdinfo", "environ", "proc", "sysfs"};
  return (k >= 0 && k < kDenySources) ? names[k] : "other";
}
inline std::atomic<uint64_t>* deny_counters() {
  static std::atomic<uint64_t> counters[kDenySources];
  return counters;
}
inline void note_errno(int err, int source) {
  if ((err == EACCES || err == EPERM) && source >= 0 && source < kDenySources)
    deny_counters()[source].fetch_add(1, std::memory_order_relaxed);
}

// Up to `cap` bytes of a (proc / sys) file; empty when it cannot be read.  A refusal is
// counted under `source`.
inline std::string read_small(const std::string& path, size_t cap = 1 << 16, int source = kDenyProcMeta) {
  int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) {
    note_errno(errno, source);
    return {};
  }
  std::string s;
  s.resize(cap);
  size_t n = 0;
  while (n < cap) {
    ssize_t r = ::read(fd, &s[n], cap - n);
    if (r < 0) {
      if (errno == EINTR) continue;
      note_errno(errno, source);
      break;
    }
    if (r == 0) break;
    n += static_cast<size_t>(r);
  }
  ::close(fd);
  s.resize(n);
  return s;
}

inline bool is_digits(const char* s) {
  if (!s || !*s) return false;
  for (; *s; ++s)
    if (*s < '0' || *s > '9') return false;
  return true;
}

// True when `proc_root` belongs to the initial PID namespace (hostPID agents):
// then amd-smi / KFD PIDs are valid /proc PIDs for us.
inline bool host_pid_namespace(const std::string& proc_root) {
  struct stat st;
  if (stat((proc_root + "/self/ns/pid").c_str(), &st) != 0) return false;
  return static_cast<unsigned long long>(st.st_ino) == kInitPidNsIno;
}

inline std::vector<uint32_t> list_pids(const std::string& proc_root) {
  std::vector<uint32_t> out;
  DIR* d = opendir(proc_root.c_str());
  if (!d) {
    note_errno(errno, kDenyProcMeta);
    return out;
  }
  while (dirent* e = readdir(d))
    if (is_digits(e->d_name)) out.push_back(static_cast<uint32_t>(strtoul(e->d_name, nullptr, 10)));
  closedir(d);
  return out;
}

// Field 22 of /proc/<pid>/stat (clock ticks since boot): distinguishes a reused PID.
inline uint64_t proc_start_ticks(const std::string& proc_root, uint32_t pid) {
  std::string s = read_small(proc_root + "/" + std::to_string(pid) + "/stat", 2048);
  size_t rp = s.rfind(')');
  if (rp == std::string::npos) return 0;
  int field = 2;  // the ')' closes field 2 (comm)
  size_t i = rp + 1;
  while (i < s.size() && field < 22) {
    while (i < s.size() && s[i] == ' ') ++i;
    ++field;
    if (field == 22) return strtoull(s.c_str() + i, nullptr, 10);
    while (i < s.size() && s[i] != ' ') ++i;
  }
  return 0;
}

// fds of `pid` that point at a DRM render node (`/dev/dri/renderD*`).
inline std::vector<int> drm_render_fds(const std::string& proc_root, uint32_t pid) {
  std::vector<int> out;
  std::string dir = proc_root + "/" + std::to_string(pid) + "/fd";
  DIR* d = opendir(dir.c_str());
  if (!d) {
    note_errno(errno, kDenyFdDir);
    return out;
  }
  char buf[256];
  while (dirent* e = readdir(d)) {
    if (!is_digits(e->d_name)) continue;
    ssize_t n = readlink((dir + "/" + e->d_name).c_str(), buf, sizeof buf - 1);
    if (n <= 0) continue;
    buf[n] = 0;
    if (strncmp(buf, "/dev/dri/renderD", 16) == 0) out.push_back(atoi(e->d_name));
  }
  closedir(d);
  return out;
}

struct DrmFdInfo {
  bool amdgpu = false;
  std::string pdev;          // PCI BDF, lower-case
  uint64_t client_id = 0;    // drm-client-id (dup'ed fds share one)
  uint64_t vram_bytes = 0;   // drm-memory-vram, else drm-total-vram / drm-resident-vram
  uint64_t gtt_bytes = 0;
  uint64_t evicted_vram_bytes = 0;
};

// Value in bytes of a "<key>:\t<n> [KiB|MiB]" fdinfo line; false if absent.
inline bool fdinfo_value(const std::string& text, const char* key, uint64_t& out) {
  size_t klen = strlen(key);
  size_t p = 0;
  while ((p = text.find(key, p)) != std::string::npos) {
    bool line_start = (p == 0 || text[p - 1] == '\n');
    if (line_start && p + klen < text.size() && text[p + klen] == ':') {
      const char* s = text.c_str() + p + klen + 1;
      while (*s == ' ' || *s == '\t') ++s;
      char* end = nullptr;
      unsigned long long v = strtoull(s, &end, 10);
      if (end == s) return false;
      while (*end == ' ' || *end == '\t') ++end;
      uint64_t mul = 1;
      if (strncmp(end, "KiB", 3) == 0) mul = 1024;
      else if (strncmp(end, "MiB", 3) == 0) mul = 1024ULL * 1024;
      else if (strncmp(end, "GiB", 3) == 0) mul = 1024ULL * 1024 * 1024;
      out = static_cast<uint64_t>(v) * mul;
      return true;
    }
    p += klen;
  }
  return false;
}

inline std::string fdinfo_string(const std::string& text, const char* key) {
  size_t klen = strlen(key);
  size_t p = 0;
  while ((p = text.find(key, p)) != std::string::npos) {
    if ((p == 0 || text[p - 1] == '\n') && p + klen < text.size() && text[p + klen] == ':') {
      size_t s = p + klen + 1;
      while (s < text.size() && (text[s] == ' ' || text[s] == '\t')) ++s;
      size_t e = text.find('\n', s);
      if (e == std::string::npos) e = text.size();
      while (e > s && (text[e - 1] == ' ' || text[e - 1] == '\t' || text[e - 1] == '\r')) --e;
      return text.substr(s, e - s);
    }
    p += klen;
  }
  return {};
}

inline std::string lower(std::string s) {
  for (auto& c : s) c = static_cast<char>(tolower(static_cast<unsigned char>(c)));
  return s;
}

inline DrmFdInfo parse_drm_fdinfo(const std::string& text) {
  DrmFdInfo r;
  r.amdgpu = fdinfo_string(text, "drm-driver") == "amdgpu";
  r.pdev = lower(fdinfo_string(text, "drm-pdev"));
  fdinfo_value(text, "drm-client-id", r.client_id);
  if (!fdinfo_value(text, "drm-memory-vram", r.vram_bytes) && !fdinfo_value(text, "drm-total-vram", r.vram_bytes))
    fdinfo_value(text, "drm-resident-vram", r.vram_bytes);
  if (!fdinfo_value(text, "drm-memory-gtt", r.gtt_bytes)) fdinfo_value(text, "drm-total-gtt", r.gtt_bytes);
  fdinfo_value(text, "amd-evicted-vram", r.evicted_vram_bytes);
  return r;
}

// One process's use of one GPU (by PCI BDF).
struct ProcGpuUse {
  uint32_t pid = 0;
  std::string bdf;
  uint64_t vram_bytes = 0;
  uint64_t gtt_bytes = 0;
  uint64_t evicted_vram_bytes = 0;
  int clients = 0;
};

// DRM-fdinfo scanner with per-PID state: a PID's fd table is re-listed only when the
// PID is new (or reused: start time changed) and then every `rescan_every` scans, while
// the fdinfo of known render fds is re-read every scan (VRAM moves fast, fd tables don't).
class DrmScanner {
 public:
  explicit DrmScanner(std::string proc_root = "/proc", int rescan_every = 8)
      : root_(std::move(proc_root)), rescan_every_(rescan_every < 1 ? 1 : rescan_every) {}

  // `candidates` empty = every PID under the root.
  std::vector<ProcGpuUse> scan(const std::vector<uint32_t>* candidates = nullptr) {
    ++scans_;
    std::vector<uint32_t> pids = candidates ? *candidates : list_pids(root_);
    std::set<uint32_t> live(pids.begin(), pids.end());
    for (auto it = state_.begin(); it != state_.end();)
      it = live.count(it->first) ? std::next(it) : state_.erase(it);
    std::vector<ProcGpuUse> out;
    for (uint32_t pid : pids) {
      PidState& st = state_[pid];
      bool due = st.scanned_at == 0 || (scans_ - st.scanned_at) >= static_cast<uint64_t>(rescan_every_);
      if (due) {
        uint64_t start = proc_start_ticks(root_, pid);
        if (st.scanned_at != 0 && start != st.start) st.fds.clear();
        st.start = start;
        st.fds = drm_render_fds(root_, pid);
        st.scanned_at = scans_;
        ++fd_scans_;
      }
      if (st.fds.empty()) continue;
      std::map<std::string, ProcGpuUse> by_bdf;
      std::set<std::pair<std::string, uint64_t>> seen_clients;
      std::vector<int> keep;
      for (int fd : st.fds) {
        std::string txt =
            read_small(root_ + "/" + std::to_string(pid) + "/fdinfo/" + std::to_string(fd), 8192, kDenyFdInfo);
        if (txt.empty()) continue;  // fd closed since the last listing
        keep.push_back(fd);
        DrmFdInfo fi = parse_drm_fdinfo(txt);
        if (!fi.amdgpu || fi.pdev.empty()) continue;
        if (fi.client_id && !seen_clients.insert({fi.pdev, fi.client_id}).second) continue;
        ProcGpuUse& u = by_bdf[fi.pdev];
        u.pid = pid;
        u.bdf = fi.pdev;
        u.vram_bytes += fi.vram_bytes;
        u.gtt_bytes += fi.gtt_bytes;
        u.evicted_vram_bytes += fi.evicted_vram_bytes;
        ++u.clients;
      }
      st.fds.swap(keep);
      for (auto& kv : by_bdf) out.push_back(kv.second);
    }
    return out;
  }

  uint64_t scans() const { return scans_; }
  uint64_t fd_scans() const { return fd_scans_; }

 private:
  struct PidState {
    uint64_t start = 0;
    uint64_t scanned_at = 0;
    std::vector<int> fds;
  };
  std::string root_;
  int rescan_every_;
  uint64_t scans_ = 0, fd_scans_ = 0;
  std::unordered_map<uint32_t, PidState> state_;
};

// KFD topology: gpu_id → PCI BDF (GPU nodes only; CPU nodes have gpu_id 0).
inline std::map<uint32_t, std::string> kfd_gpu_bdfs(const std::string& sys_root) {
  std::map<uint32_t, std::string> out;
  std::string base = sys_root + "/class/kfd/kfd/topology/nodes";
  DIR* d = opendir(base.c_str());
  if (!d) return out;
  while (dirent* e = readdir(d)) {
    if (!is_digits(e->d_name)) continue;
    std::string node = base + "/" + e->d_name;
    uint32_t gpu_id =
        static_cast<uint32_t>(strtoul(read_small(node + "/gpu_id", 64, kDenySysfs).c_str(), nullptr, 10));
    if (!gpu_id) continue;
    std::string props = read_small(node + "/properties", 1 << 14, kDenySysfs);
    uint64_t loc = 0, dom = 0;
    bool have_loc = false;
    size_t p = 0;
    while (p < props.size()) {
      size_t e2 = props.find('\n', p);
      if (e2 == std::string::npos) e2 = props.size();
      std::string line = props.substr(p, e2 - p);
      size_t sp = line.find(' ');
      if (sp != std::string::npos) {
        std::string k = line.substr(0, sp);
        uint64_t v = strtoull(line.c_str() + sp + 1, nullptr, 10);
        if (k == "location_id") {
          loc = v;
          have_loc = true;
        } else if (k == "domain") {
          dom = v;
        }
      }
      p = e2 + 1;
    }
    if (!have_loc) continue;
    char b[32];
    snprintf(b, sizeof b, "%04llx:%02llx:%02llx.%llx", static_cast<unsigned long long>(dom),
             static_cast<unsigned long long>((loc >> 8) & 0xff), static_cast<unsigned long long>((loc >> 3) & 0x1f),
             static_cast<unsigned long long>(loc & 0x7));
    out[gpu_id] = b;
  }
  closedir(d);
  return out;
}

// KFD per-process VRAM (`proc/<pid>/vram_<gpu_id>`, bytes), resolved to BDFs.  PIDs are
// init-namespace PIDs.
inline std::vector<ProcGpuUse> kfd_proc_usage(const std::string& sys_root, const std::map<uint32_t, std::string>& bdfs) {
  std::vector<ProcGpuUse> out;
  std::string base = sys_root + "/class/kfd/kfd/proc";
  DIR* d = opendir(base.c_str());
  if (!d) return out;
  std::vector<std::string> pids;
  while (dirent* e = readdir(d))
    if (is_digits(e->d_name)) pids.push_back(e->d_name);
  closedir(d);
  for (auto& ps : pids) {
    std::string dir = base + "/" + ps;
    DIR* pd = opendir(dir.c_str());
    if (!pd) continue;
    while (dirent* e = readdir(pd)) {
      if (strncmp(e->d_name, "vram_", 5) != 0 || !is_digits(e->d_name + 5)) continue;
      uint32_t gid = static_cast<uint32_t>(strtoul(e->d_name + 5, nullptr, 10));
      auto it = bdfs.find(gid);
      if (it == bdfs.end()) continue;
      ProcGpuUse u;
      u.pid = static_cast<uint32_t>(strtoul(ps.c_str(), nullptr, 10));
      u.bdf = it->second;
      u.vram_bytes = strtoull(read_small(dir + "/" + e->d_name, 64, kDenySysfs).c_str(), nullptr, 10);
      u.clients = 1;
      out.push_back(u);
    }
    closedir(pd);
  }
  return out;
}

}  // namespace nexus_gpu
