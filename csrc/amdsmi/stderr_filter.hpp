// Keeps libamd_smi's per-process noise out of the process's stderr.
//
// amdsmi_get_gpu_process_list() walks KFD's /sys/class/kfd/kfd/proc/<pid> entries and, for
// every process whose `queues` directory is gone by the time it looks (the process exited
// between the directory listing and the read — routine on a busy node, every sample),
// prints "Unable to open queues directory for process <pid>: No such file or directory"
// straight to fd 2.  A node agent sampling twice a second filled its logs with it, and
// every bench run's stderr tail was nothing else.
//
// Fd2Filter::run(fn) points fd 2 at an anonymous in-memory file (memfd, O_APPEND) for
// the duration of `fn` (one amd-smi call, well under a millisecond), then puts the real
// stderr back and forwards every captured line that is not amd-smi noise — anything
// another thread wrote to stderr in that window — to it, in order (a write racing the
// swap back by microseconds can come out a few lines late, never lost).  Nothing can block
// (a memfd never fills like a pipe), nothing is lost unless the process dies inside the
// window (a write still in flight at the swap back is forwarded by the next drain, or by
// flush() when the monitor stops), and the noise lines are counted (the vanished
// processes) instead of printed.
// The swap is process-wide, so all monitors in the process share one mutex.
#pragma once

#include <fcntl.h>
#include <linux/falloc.h>
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>

namespace nexus_gpu {

class Fd2Filter {
 public:
  // lines starting with one of these are libamd_smi's, counted and dropped
  static bool is_noise(const char* s, size_t n) {
    static const char* kNoise[] = {"Unable to open queues directory for process"};
    for (const char* p : kNoise) {
      size_t m = strlen(p);
      if (n >= m && memcmp(s, p, m) == 0) return true;
    }
    return false;
  }

  static Fd2Filter& instance() {
    static Fd2Filter f;
    return f;
  }

  // Runs fn() with fd 2 captured; returns the number of noise lines it (or anything else
  // in the window) printed.  Falls back to a plain call when fd 2 cannot be swapped.
  template <class F>
  uint32_t run(F&& fn) {
    std::lock_guard<std::mutex> lk(mu_);
    if (!enabled_.load(std::memory_order_relaxed)) {
      fn();
      return 0;
    }
    if (memfd_ < 0) {
      memfd_ = memfd_create("nexus-amdsmi-stderr", MFD_CLOEXEC);
      if (memfd_ >= 0) fcntl(memfd_, F_SETFL, O_APPEND);
    }
    int saved = memfd_ >= 0 ? dup(2) : -1;
    if (saved < 0) {
      fn();
      return 0;
    }
    fflush(stderr);
    if (dup2(memfd_, 2) < 0) {
      close(saved);
      fn();
      return 0;
    }
    fn();
    fflush(stderr);
    dup2(saved, 2);
    close(saved);
    return drain();
  }

  // Forward what late writers appended after the last window (call when sampling stops).
  uint32_t flush() {
    std::lock_guard<std::mutex> lk(mu_);
    return memfd_ >= 0 ? drain(true) : 0;
  }

  void set_enabled(bool on) { enabled_.store(on); }
  uint64_t noise_lines() const { return noise_.load(); }
  uint64_t forwarded_bytes() const { return forwarded_.load(); }

 private:
  Fd2Filter() = default;

  // Reads what was appended since the last drain.  The file is never truncated: a write
  // another thread started while fd 2 still pointed here can complete after the swap back,
  // and it must land where the next drain reads it (a truncate could drop it).  The pages
  // already read are released with a hole punch, so memory stays flat.
  uint32_t drain(bool all = false) {
    off_t end = lseek(memfd_, 0, SEEK_END);
    if (end <= off_) return 0;
    std::string buf(static_cast<size_t>(end - off_), '\0');
    ssize_t got = pread(memfd_, &buf[0], buf.size(), off_);
    if (got <= 0) return 0;
    buf.resize(static_cast<size_t>(got));
    // only whole lines (a line written in pieces is read whole by the next drain), except
    // on the final flush
    size_t whole = buf.rfind('\n');
    if (!all) {
      if (whole == std::string::npos) return 0;
      buf.resize(whole + 1);
    }
    off_ += static_cast<off_t>(buf.size());
    const off_t page = 4096;
    if (off_ / page > punched_ / page) {
      off_t upto = (off_ / page) * page;
      if (fallocate(memfd_, FALLOC_FL_PUNCH_HOLE | FALLOC_FL_KEEP_SIZE, punched_, upto - punched_) == 0) punched_ = upto;
    }
    uint32_t noise = 0;
    std::string keep;
    size_t s = 0;
    while (s < buf.size()) {
      size_t e = buf.find('\n', s);
      size_t len = (e == std::string::npos ? buf.size() : e + 1) - s;
      if (is_noise(buf.data() + s, len)) {
        ++noise;
      } else {
        keep.append(buf, s, len);
      }
      s += len;
    }
    size_t off = 0;
    while (off < keep.size()) {  // the real stderr again: another thread's lines, in order
      ssize_t w = write(2, keep.data() + off, keep.size() - off);
      if (w <= 0) break;
      off += static_cast<size_t>(w);
    }
    forwarded_ += keep.size();
    noise_ += noise;
    return noise;
  }

  std::mutex mu_;
  int memfd_ = -1;
  off_t off_ = 0;       // bytes of the file already drained
  off_t punched_ = 0;   // bytes released with a hole punch
  std::atomic<bool> enabled_{true};
  std::atomic<uint64_t> noise_{0};
  std::atomic<uint64_t> forwarded_{0};
};

}  // namespace nexus_gpu
