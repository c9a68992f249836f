// nexus-kubesim — a native kube-apiserver simulator for benchmarks and tests.
//
// The reference runs client-go informers against a real API server (LIST+WATCH of
// Events, Pods and Jobs in one namespace, Job DELETE with Background propagation:
// /root/reference/services/supervisor.go:70-75,262-270).  The benchmark needs an API
// server that is never the bottleneck while 10k live runs churn at thousands of
// failures per second and every supervisor shard-worker process holds its own three
// watch streams.  The Python fake (nexus_supervisor_amd/testing/fake_apiserver.py)
// keeps the fault-injection surface for tests; this server implements the same REST
// + watch wire protocol on one epoll thread:
//
//   GET    …/{plural}                 LIST (labelSelector / fieldSelector, limit+continue
//                                      over a consistent snapshot)
//   GET    …/{plural}?watch=1         WATCH from resourceVersion: history replay, 410 Gone
//                                      below the compaction point, BOOKMARKs, timeoutSeconds;
//                                      chunked JSON lines, one chunk per burst per stream
//   GET    …/{plural}/{name}          GET
//   POST   …/{plural}                 create (generateName, uid, creationTimestamp, RV)
//   PUT    …/{plural}/{name}          replace (409 on a stale resourceVersion)
//   PATCH  …/{plural}/{name}          JSON merge patch
//   DELETE …/{plural}/{name}          delete; Background/Foreground propagation deletes the
//                                      Job's pods (batch.kubernetes.io/job-name) like the GC
//                                      (--async-gc: Background's pods after the answer, on a
//                                      GC thread, as kube-controller-manager's GC does)
//   POST   /sim/apply[?expire=1]      bulk NDJSON {"type": ADDED|MODIFIED|DELETED, "object": …}
//                                      (the benchmark's cluster generator); answers the
//                                      CLOCK_MONOTONIC commit time of the batch; expire=1
//                                      then compacts past undelivered lines (watchers get 410)
//   POST   /sim/expire[?kind=Pod]     compact history (resuming watches get 410) + cut streams
//   POST   /sim/close-watches         cut every watch stream
//   GET    /sim/stats                 counters
//   GET    …/pods/{name}/log          the container log a bench LOG line stored for the pod
//                                      (container / tailLines / limitBytes; 400 when none)
//   (/sim/apply also takes {"type":"LOG","object":{"namespace","pod","container","text"}}:
//    a failed container's log, never sent to watchers, dropped with its pod)
//
// Pricing the API server (a real apiserver is not free): --api-latency-us answers every object
// request (GET / DELETE / POST / PUT / PATCH; not LIST / WATCH) that long after it was
// applied, in order per connection (an etcd write + admission); --write-qps caps mutating
// requests with a token bucket and answers the excess 429 + Retry-After, as API Priority and
// Fairness does; --throttle-deletes N answers the first N Job DELETEs 429 + Retry-After
// (--retry-after S) for the client's flow-control path.
//
// Paths: /api/v1/namespaces/{ns}/{plural}[/{name}], /apis/{group}/{version}/namespaces/…,
// and the cluster-wide /api/v1/{plural}.  Optional bearer token (--token).
//
// nexus-kubesim [--host 127.0.0.1] [--port 0] [--ready-file F] [--history N]
//               [--bookmark-ms 1000] [--token T] [--api-latency-us US] [--write-qps Q]
//               [--write-burst B] [--throttle-deletes N] [--retry-after S]
#include <arpa/inet.h>
#include <dirent.h>
#include <dlfcn.h>
#include <execinfo.h>
#include <fcntl.h>
#include <malloc.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <pthread.h>
#include <signal.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/time.h>
#include <sys/uio.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <charconv>
#include <functional>
#include <cerrno>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <random>
#include <set>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "json.hpp"

using kjson::Value;

namespace {

// ------------------------------------------------------------ CPU sampler (diagnostics)
// NEXUS_KUBESIM_PROF=<file>: SIGPROF every 1 ms of process CPU time records the stack;
// at exit every sample is written as "module+offset" frames (leaf first), one line per
// sample, for tools/native_prof.py to symbolise (the last 128k samples: older ones are
// overwritten).  Off unless the variable is set.
namespace prof {
constexpr int kMaxSamples = 1 << 17;
constexpr int kDepth = 12;
void* g_frames[kMaxSamples][kDepth];
unsigned char g_depth[kMaxSamples];
unsigned char g_helper[kMaxSamples];  // sampled on an apply / fan-out thread, not the loop
std::atomic<int> g_n{0};
pthread_t g_loop;
std::string g_path;

void on_sigprof(int) {
  // a ring: a long run keeps its last kMaxSamples samples (the timed steps, not the setup)
  int i = g_n.fetch_add(1, std::memory_order_relaxed) & (kMaxSamples - 1);
  g_helper[i] = pthread_equal(pthread_self(), g_loop) ? 0 : 1;
  g_depth[i] = static_cast<unsigned char>(backtrace(g_frames[i], kDepth));
}

void start() {
  const char* p = getenv("NEXUS_KUBESIM_PROF");
  if (!p || !*p) return;
  g_path = p;
  g_loop = pthread_self();
  void* warm[2];
  backtrace(warm, 2);  // first call loads the unwinder: not inside the handler
  struct sigaction sa {};
  sa.sa_handler = on_sigprof;
  sa.sa_flags = SA_RESTART;
  sigaction(SIGPROF, &sa, nullptr);
  itimerval it{};
  it.it_interval.tv_usec = 1000;
  it.it_value.tv_usec = 1000;
  setitimer(ITIMER_PROF, &it, nullptr);
}

void dump() {
  if (g_path.empty()) return;
  itimerval off{};
  setitimer(ITIMER_PROF, &off, nullptr);
  FILE* f = fopen(g_path.c_str(), "w");
  if (!f) return;
  int n = std::min(g_n.load(), kMaxSamples);
  for (int i = 0; i < n; ++i) {
    // frames 0-1 are the handler and the signal trampoline
    for (int d = 2; d < g_depth[i]; ++d) {
      Dl_info info{};
      uintptr_t a = reinterpret_cast<uintptr_t>(g_frames[i][d]);
      if (dladdr(g_frames[i][d], &info) && info.dli_fname)
        fprintf(f, "%s%s+0x%lx", d > 2 ? " " : "", info.dli_fname,
                static_cast<unsigned long>(a - reinterpret_cast<uintptr_t>(info.dli_fbase) - (d > 2 ? 1 : 0)));
      else
        fprintf(f, "%s?+0x%lx", d > 2 ? " " : "", static_cast<unsigned long>(a));
    }
    // the sampled thread as the outermost frame
    fprintf(f, " %s+0x0\n", g_helper[i] ? "[helper-thread]" : "[event-loop]");
  }
  fclose(f);
}
}  // namespace prof

// ============================================================ options / clock
struct Options {
  std::string host = "127.0.0.1";
  int port = 0;
  std::string ready_file;
  size_t history = 400000;
  int64_t bookmark_ms = 1000;
  std::string token;
  // watch fan-out threads: the dirty watch streams of one loop iteration are written by
  // this many threads (the apiserver's watch cache serves many watchers in parallel; a
  // sharded supervisor deployment has every replica watching the whole namespace)
  int flush_threads = 1;
  int apply_threads = 1;  // threads scanning a /sim/apply chunk's lines before the in-order commit
  int64_t api_latency_us = 0;   // answer object requests this long after applying them
  double write_qps = 0;         // mutating requests per second (token bucket); 0 = no cap
  int write_burst = 0;          // bucket size (0 = max(1, write_qps))
  int64_t throttle_deletes = 0; // answer this many first Job DELETEs 429
  int retry_after_s = 1;        // Retry-After of every 429
  size_t prefault_mb = 0;       // heap pages touched at startup (kept: trim threshold 1 GiB)
  // a kubelet's /var/log/pods: every bench LOG line (with the pod's uid) is also written as
  // <root>/<ns>_<pod>_<uid>/<container>/<restart>.log in the CRI format, for a node agent
  // process reading the node's logs (the deployed default-pod path); empty = off
  std::string log_root;
  // Background propagation as the kube-controller-manager's garbage collector does it: the
  // Job DELETE is answered at once and the Job's pods are deleted afterwards, on a GC thread
  // of the simulator's (the loop then answers DELETEs without the pod cascade); off = the
  // pods go inside the DELETE, before its answer
  bool async_gc = false;
} g_opt;

int64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<int64_t>(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}
int64_t mono_ms() { return mono_ns() / 1000000; }

std::string now_rfc3339() {
  static time_t cached_t = 0;
  static std::string cached;
  time_t t = time(nullptr);
  if (t != cached_t) {
    char buf[32];
    tm g;
    gmtime_r(&t, &g);
    strftime(buf, sizeof buf, "%Y-%m-%dT%H:%M:%SZ", &g);
    cached = buf;
    cached_t = t;
  }
  return cached;
}

std::mt19937_64 g_rng(0x6b756265u ^ static_cast<uint64_t>(mono_ns()));

std::string random_suffix(int n) {
  static const char* al = "bcdfghjklmnpqrstvwxz2456789";
  std::string s;
  for (int i = 0; i < n; ++i) s += al[g_rng() % 27];
  return s;
}

std::string uuid4() {
  uint64_t a = g_rng(), b = g_rng();
  a = (a & 0xFFFFFFFFFFFF0FFFULL) | 0x0000000000004000ULL;
  b = (b & 0x3FFFFFFFFFFFFFFFULL) | 0x8000000000000000ULL;
  char buf[40];
  snprintf(buf, sizeof buf, "%08x-%04x-%04x-%04x-%012llx", static_cast<unsigned>(a >> 32),
           static_cast<unsigned>((a >> 16) & 0xFFFF), static_cast<unsigned>(a & 0xFFFF), static_cast<unsigned>(b >> 48),
           static_cast<unsigned long long>(b & 0xFFFFFFFFFFFFULL));
  return buf;
}

// ============================================================ kinds
struct KindInfo {
  const char* kind;
  const char* api_version;
  const char* plural;
};
const KindInfo KINDS[] = {{"Event", "v1", "events"},
                          {"Pod", "v1", "pods"},
                          {"Job", "batch/v1", "jobs"},
                          {"Lease", "coordination.k8s.io/v1", "leases"},
                          {"Node", "v1", "nodes"}};
constexpr int NKINDS = sizeof(KINDS) / sizeof(KINDS[0]);
constexpr int K_EVENT = 0, K_POD = 1, K_JOB = 2;

int kind_by_plural(std::string_view p) {
  for (int i = 0; i < NKINDS; ++i)
    if (p == KINDS[i].plural) return i;
  return -1;
}
int kind_by_name(std::string_view k) {
  for (int i = 0; i < NKINDS; ++i)
    if (k == KINDS[i].kind) return i;
  return -1;
}

// ============================================================ selectors
// Selectable attributes of an object: its labels plus a fixed set of field paths
// (prefixed "\x01f:" so they never collide with a label key).
// Packed into one buffer ([u32 len][key][u32 len][value]...): one allocation per object
// version instead of two strings per attribute (allocation was a quarter of the
// simulator's time under the benchmark's churn).
class Attrs {
 public:
  void add(std::string_view k, std::string_view v) {
    put(k);
    put(v);
  }
  void reserve(size_t bytes) { buf_.reserve(bytes); }
  bool find(std::string_view k, std::string_view& v) const {
    size_t i = 0;
    while (i < buf_.size()) {
      std::string_view key = get(i);
      std::string_view val = get(i);
      if (key == k) {
        v = val;
        return true;
      }
    }
    return false;
  }

 private:
  void put(std::string_view x) {
    uint32_t n = static_cast<uint32_t>(x.size());
    buf_.append(reinterpret_cast<const char*>(&n), sizeof n);
    buf_.append(x.data(), x.size());
  }
  std::string_view get(size_t& i) const {
    uint32_t n;
    std::memcpy(&n, buf_.data() + i, sizeof n);
    i += sizeof n;
    std::string_view x(buf_.data() + i, n);
    i += n;
    return x;
  }
  std::string buf_;
};
const char* const FIELD_PATHS[][3] = {{"metadata", "name", nullptr},        {"metadata", "namespace", nullptr},
                                      {"spec", "nodeName", nullptr},        {"status", "phase", nullptr},
                                      {"involvedObject", "kind", nullptr}, {"involvedObject", "name", nullptr},
                                      {"reason", nullptr, nullptr},         {"type", nullptr, nullptr}};

std::shared_ptr<const Attrs> attrs_of(const Value& obj) {
  auto a = std::make_shared<Attrs>();
  const Value* md = obj.get("metadata");
  const Value* labels = md ? md->get("labels") : nullptr;
  if (labels && labels->t == Value::OBJ)
    for (auto& kv : labels->o)
      if (kv.second.t == Value::STR) a->add(kv.first, kv.second.s);
  for (auto& fp : FIELD_PATHS) {
    const Value* cur = &obj;
    std::string key = "\x01" "f:";
    for (int i = 0; i < 3 && fp[i]; ++i) {
      cur = cur->get(fp[i]);
      if (!cur) break;
      if (i) key += '.';
      key += fp[i];
    }
    if (cur && cur->t == Value::STR) a->add(key, cur->s);
  }
  return a;
}

struct Req {
  std::string key;
  char op;  // '=', '!', 'e' (exists), 'n' (not exists), 'i' (in set), 'o' (notin set)
  std::string val;
  std::vector<std::string> vals;  // 'i' / 'o'
};
using Selector = std::vector<Req>;

std::string_view trim_view(std::string_view s) {
  size_t b = 0, e = s.size();
  while (b < e && isspace(static_cast<unsigned char>(s[b]))) ++b;
  while (e > b && isspace(static_cast<unsigned char>(s[e - 1]))) --e;
  return s.substr(b, e - b);
}

// ASCII case-insensitive equality; `lower` must already be lower case
bool iequals(std::string_view s, std::string_view lower) {
  if (s.size() != lower.size()) return false;
  for (size_t i = 0; i < s.size(); ++i)
    if (static_cast<char>(tolower(static_cast<unsigned char>(s[i]))) != lower[i]) return false;
  return true;
}

std::string trim(std::string_view s) {
  size_t b = 0, e = s.size();
  while (b < e && isspace(static_cast<unsigned char>(s[b]))) ++b;
  while (e > b && isspace(static_cast<unsigned char>(s[e - 1]))) --e;
  return std::string(s.substr(b, e - b));
}

// set-based requirement "key in (a,b)" / "key notin (a,b)": true and filled when `part` is one
bool parse_set_req(const std::string& part, Req& r) {
  size_t lp = part.find('(');
  if (lp == std::string::npos || part.back() != ')') return false;
  std::string head = trim(std::string_view(part).substr(0, lp));
  size_t sp = head.find_last_of(" \t");
  if (sp == std::string::npos) return false;
  std::string op = trim(std::string_view(head).substr(sp + 1));
  if (op != "in" && op != "notin") return false;
  r.key = trim(std::string_view(head).substr(0, sp));
  r.op = op == "in" ? 'i' : 'o';
  std::string_view body(part.data() + lp + 1, part.size() - lp - 2);
  size_t b = 0;
  while (b <= body.size()) {
    size_t c = body.find(',', b);
    if (c == std::string_view::npos) c = body.size();
    std::string v = trim(body.substr(b, c - b));
    if (!v.empty()) r.vals.push_back(std::move(v));
    b = c + 1;
  }
  return true;
}

void parse_selector(std::string_view sel, bool fields, Selector& out) {
  size_t pos = 0;
  while (pos <= sel.size()) {
    size_t comma = sel.find(',', pos);
    size_t paren = sel.find('(', pos);
    if (paren != std::string_view::npos && paren < comma) {  // a set: its commas are inside ( )
      size_t close = sel.find(')', paren);
      comma = close == std::string_view::npos ? sel.size() : sel.find(',', close);
    }
    if (comma == std::string_view::npos) comma = sel.size();
    std::string part = trim(sel.substr(pos, comma - pos));
    pos = comma + 1;
    if (part.empty()) {
      if (comma >= sel.size()) break;
      continue;
    }
    Req r;
    size_t i;
    if (parse_set_req(part, r)) {
      // "key in (...)" / "key notin (...)"
    } else if ((i = part.find("!=")) != std::string::npos) {
      r = {trim(part.substr(0, i)), '!', trim(part.substr(i + 2)), {}};
    } else if ((i = part.find("==")) != std::string::npos) {
      r = {trim(part.substr(0, i)), '=', trim(part.substr(i + 2)), {}};
    } else if ((i = part.find('=')) != std::string::npos) {
      r = {trim(part.substr(0, i)), '=', trim(part.substr(i + 1)), {}};
    } else if (part[0] == '!') {
      r = {trim(part.substr(1)), 'n', "", {}};
    } else {
      r = {part, 'e', "", {}};
    }
    if (fields) r.key = "\x01" "f:" + r.key;
    out.push_back(std::move(r));
    if (comma >= sel.size()) break;
  }
}

bool matches(const Attrs& a, const Selector& sel) {
  for (auto& r : sel) {
    std::string_view v;
    bool has = a.find(r.key, v);
    switch (r.op) {
      case '=': if (!has || v != r.val) return false; break;
      case '!': if (has && v == r.val) return false; break;
      case 'e': if (!has) return false; break;
      case 'n': if (has) return false; break;
      case 'i': if (!has || std::find(r.vals.begin(), r.vals.end(), v) == r.vals.end()) return false; break;
      case 'o': if (has && std::find(r.vals.begin(), r.vals.end(), v) != r.vals.end()) return false; break;
    }
  }
  return true;
}

// ============================================================ store
struct Obj {
  std::shared_ptr<const std::string> json;
  std::shared_ptr<const Attrs> attrs;
  std::string ns, name, job;  // job: batch.kubernetes.io/job-name label (pods)
  std::string uid, created;   // kept so an update that omits them can be completed by splicing
  int64_t rv = 0;
  size_t rv_off = std::string::npos;  // offset of the resourceVersion digits in *json
  size_t rv_len = 0;
};

// locate metadata.resourceVersion's digits in a serialised object (the value is unique: it is
// the object's own RV, so the first `"resourceVersion":"<rv>"` is it)
void locate_rv(Obj& o) {
  std::string needle = "\"resourceVersion\":\"" + std::to_string(o.rv) + "\"";
  size_t at = o.json->find(needle);
  if (at != std::string::npos) {
    o.rv_off = at + 19;
    o.rv_len = needle.size() - 20;
  } else {
    o.rv_off = std::string::npos;
  }
}

// One watch line, `{"type":"<T>","object":` + object text + `}\n`, kept as the static type
// prefix plus the object's own immutable (shared) text: recording a change copies nothing,
// and a watch chunk goes out as three iovecs per line over the store's buffers.
// A DELETED line carries the deletion's resourceVersion in `rv`, replacing the digits at
// json[rv_off, rv_off + rv_len) when sent (the removed object's text is not copied).
struct Line {
  const std::string* prefix;
  std::shared_ptr<const std::string> json;
  uint32_t rv_off = 0, rv_len = 0;
  uint8_t rvn = 0;
  char rv[23];
  size_t size() const { return prefix->size() + json->size() - rv_len + rvn + 2; }
};

const std::string* line_prefix(const char* etype) {
  static const std::string added = "{\"type\":\"ADDED\",\"object\":";
  static const std::string modified = "{\"type\":\"MODIFIED\",\"object\":";
  static const std::string deleted = "{\"type\":\"DELETED\",\"object\":";
  if (etype[0] == 'A') return &added;
  if (etype[0] == 'M') return &modified;
  return &deleted;
}

char g_line_end[] = "}\n";

void append_line(std::string& out, const Line& l) {
  out += *l.prefix;
  if (l.rvn) {
    out.append(*l.json, 0, l.rv_off);
    out.append(l.rv, l.rvn);
    out.append(*l.json, l.rv_off + l.rv_len, std::string::npos);
  } else {
    out += *l.json;
  }
  out.append(g_line_end, 2);
}

struct Hist {
  int64_t rv;
  std::string ns;
  Line line;
  std::shared_ptr<const Attrs> attrs;
};

// Watch-cache history: a ring over one growing power-of-two buffer.  A std::deque allocated
// and freed a block every few commits (and re-centred its block map as the front was popped)
// — ~7 % of the simulator's time at saturation (tools/kubesim_bench.py, -fno-inline profile).
template <typename T>
class Ring {
 public:
  size_t size() const { return n_; }
  bool empty() const { return n_ == 0; }
  T& operator[](size_t i) { return buf_[(head_ + i) & mask_]; }
  const T& operator[](size_t i) const { return buf_[(head_ + i) & mask_]; }
  T& front() { return buf_[head_]; }
  T& back() { return (*this)[n_ - 1]; }
  void push_back(T&& v) {
    if (n_ == buf_.size()) grow();
    buf_[(head_ + n_) & mask_] = std::move(v);
    ++n_;
  }
  void pop_front() {
    buf_[head_] = T();  // drop the line text / attrs references now, as the deque did
    head_ = (head_ + 1) & mask_;
    --n_;
  }
  void clear() {
    for (size_t i = 0; i < n_; ++i) (*this)[i] = T();
    head_ = n_ = 0;
  }

 private:
  void grow() {
    std::vector<T> nb(buf_.empty() ? 1024 : buf_.size() * 2);
    for (size_t i = 0; i < n_; ++i) nb[i] = std::move((*this)[i]);
    buf_.swap(nb);
    head_ = 0;
    mask_ = buf_.size() - 1;
  }
  std::vector<T> buf_;
  size_t head_ = 0, n_ = 0, mask_ = 0;
};

struct Conn;

struct Watch {
  int fd;
  int kind;
  std::string ns;
  Selector sel;
  bool bookmarks;
  int64_t deadline_ms;
  int64_t last_ms;
  std::string pending;  // control lines (ERROR / BOOKMARK) for the next chunk
  // event lines committed this loop iteration: shared with the history, sent as one
  // chunk straight from these buffers (sendmsg iovecs; no per-watch copy)
  std::vector<Line> lines;
  size_t lines_bytes = 0;
  bool idle() const { return pending.empty() && lines.empty(); }
  void clear() {
    pending.clear();
    lines.clear();
    lines_bytes = 0;
  }
};

struct KindStore {
  std::unordered_map<std::string, Obj> objs;  // ns \x01 name → object (LIST sorts)
  Ring<Hist> history;
  int64_t compacted = 0;
  std::vector<Watch*> watchers;
};

KindStore g_store[NKINDS];
std::unordered_map<std::string, std::set<std::string>> g_pods_by_job;  // ns \x01 job → pod names
// A LOG line's text as the container runtime would have written it (--log-root): one CRI
// record per line, "<RFC3339Nano> stderr F <text>", into the instance's file.  The
// directory of a deleted pod is removed with it (the kubelet's log GC).
bool plain_component(std::string_view s) {
  return !s.empty() && s != "." && s != ".." && s.find('/') == std::string_view::npos;
}

std::string pod_log_dir(std::string_view ns, std::string_view pod, std::string_view uid) {
  std::string d = g_opt.log_root;
  d += '/';
  d.append(ns);
  d += '_';
  d.append(pod);
  d += '_';
  d.append(uid);
  return d;
}

void write_cri_log(std::string_view ns, std::string_view pod, std::string_view uid, std::string_view container,
                   long restart, std::string_view text) {
  if (!plain_component(ns) || !plain_component(pod) || !plain_component(uid) || !plain_component(container)) return;
  std::string dir = pod_log_dir(ns, pod, uid);
  mkdir(dir.c_str(), 0755);
  dir += '/';
  dir.append(container);
  mkdir(dir.c_str(), 0755);
  std::string path = dir + "/" + std::to_string(restart) + ".log";
  std::string out;
  size_t s = 0;
  while (s < text.size()) {
    size_t e = text.find('\n', s);
    if (e == std::string_view::npos) e = text.size();
    out += "2026-01-01T00:00:00.000000000Z stderr F ";
    out.append(text.substr(s, e - s));
    out += '\n';
    s = e + 1;
  }
  int fd = open(path.c_str(), O_WRONLY | O_CREAT | O_APPEND | O_CLOEXEC, 0644);
  if (fd < 0) return;
  size_t off = 0;
  while (off < out.size()) {
    ssize_t w = write(fd, out.data() + off, out.size() - off);
    if (w <= 0) break;
    off += static_cast<size_t>(w);
  }
  close(fd);
}

// ns \x01 pod → pod uid of the log directories written (--log-root), for their removal
std::unordered_map<std::string, std::string> g_log_dirs;

void remove_pod_logs(std::string_view ns, std::string_view pod) {
  auto it = g_log_dirs.find(std::string(ns) + '\x01' + std::string(pod));
  if (it == g_log_dirs.end()) return;
  std::string dir = pod_log_dir(ns, pod, it->second);
  g_log_dirs.erase(it);
  // <dir>/<container>/<n>.log: two levels
  if (DIR* d = opendir(dir.c_str())) {
    while (dirent* c = readdir(d)) {
      if (!strcmp(c->d_name, ".") || !strcmp(c->d_name, "..")) continue;
      std::string sub = dir + "/" + c->d_name;
      if (DIR* f = opendir(sub.c_str())) {
        while (dirent* x = readdir(f))
          if (strcmp(x->d_name, ".") && strcmp(x->d_name, "..")) unlink((sub + "/" + x->d_name).c_str());
        closedir(f);
      }
      rmdir(sub.c_str());
    }
    closedir(d);
  }
  rmdir(dir.c_str());
}

// ns \x01 pod → container → log text (bench LOG lines; pods/log answers from it)
std::unordered_map<std::string, std::unordered_map<std::string, std::string>> g_pod_logs;
// the store's resourceVersion counter: per-kind commit threads take from it concurrently
// (each kind's history stays increasing; rvs are unique, not contiguous per kind)
std::atomic<int64_t> g_rv{1000};
// The store (objects, histories, watchers' pending lines, the pod index and logs, the
// connection table and the dirty set) is the event loop's, except while the apply thread
// commits a bulk apply: both take g_store_mu for every touch.  The loop holds it while it
// handles requests and timers, never across epoll_wait, recv or a watch's sendmsg.
std::mutex g_store_mu;
// --async-gc: pods of Jobs deleted with Background propagation, (namespace, name), waiting for
// the GC thread; guarded by g_store_mu
std::deque<std::pair<std::string, std::string>> g_gc;
std::condition_variable g_gc_cv;
// --async-gc: removed objects (their strings, attrs and text references), destroyed on the GC
// thread outside the lock — the loop answers a Job DELETE without freeing the Job
std::vector<Obj> g_graves;
// remove() runs on the loop, the GC thread and a bulk apply's per-kind commit threads (those
// two at once, under the one store lock the apply thread holds): the graves have a lock of
// their own
std::mutex g_graves_mu;

struct Stats {
  uint64_t requests = 0, watch_requests = 0, applied = 0, throttled = 0, delayed = 0;
  std::atomic<uint64_t> deleted{0};  // also counted by per-kind commit threads
  uint64_t loops = 0;
  std::atomic<uint64_t> sends{0}, send_bytes{0}, eagain{0};  // also counted by fan-out threads
  // wall time spent per phase of the event loop (ns): where a saturated simulator goes
  int64_t apply_ns = 0, request_ns = 0, flush_ns = 0, recv_ns = 0, busy_ns = 0;
  int64_t prepare_ns = 0;  // the parallel part of apply_ns (wall time)
  int64_t store_ns = 0;    // time g_store_mu was held (loop + apply thread): the serial part
  std::atomic<int64_t> apply_thread_ns{0};  // the apply port's busy time (reading, applying), all connections
  std::atomic<int64_t> gc_ns{0};  // the GC thread's busy time (--async-gc: pod deletions + frees)
  uint64_t gc_pods = 0;
  uint64_t commit_parallel = 0;  // bulk-apply chunks committed per kind on threads
} g_stats;

// busy time per apply connection: each connection is served by one thread, so each is a
// serial part of its own; with several generators (node mode: one per slot) the sum over
// connections is not any one thread's load
std::mutex g_apply_conn_mu;
std::map<int, int64_t> g_apply_conn_ns;
std::atomic<int> g_apply_conn_seq{0};

// g_store_mu held for the scope; the hold time counts into g_stats.store_ns
struct StoreLock {
  std::unique_lock<std::mutex> lk;
  int64_t t0;
  StoreLock() : lk(g_store_mu), t0(mono_ns()) {}
  ~StoreLock() { g_stats.store_ns += mono_ns() - t0; }
};

struct Snapshot {
  int64_t rv;
  std::vector<std::shared_ptr<const std::string>> items;
};
std::map<std::string, Snapshot> g_snapshots;
std::deque<std::string> g_snapshot_order;

std::string okey(std::string_view ns, std::string_view name) {
  std::string k(ns);
  k += '\x01';
  k += name;
  return k;
}

// The same key in a reused buffer (lookups only: no allocation once it has grown), one per
// thread (the per-kind commit threads of a bulk apply look objects up too).
const std::string& okey_scratch(std::string_view ns, std::string_view name) {
  thread_local std::string k;
  k.assign(ns.data(), ns.size());
  k += '\x01';
  k.append(name.data(), name.size());
  return k;
}

void watch_push(Watch* w, const Line& line);

// `new_rv` > 0: a deletion at that resourceVersion of `o` (text still at o.rv), spliced on send
void record(int kind, const char* etype, const Obj& o, int64_t new_rv = 0) {
  Line lp{line_prefix(etype), o.json, 0, 0, 0, {}};
  int64_t rv = o.rv;
  if (new_rv > 0) {
    rv = new_rv;
    lp.rv_off = static_cast<uint32_t>(o.rv_off);
    lp.rv_len = static_cast<uint32_t>(o.rv_len);
    lp.rvn = static_cast<uint8_t>(snprintf(lp.rv, sizeof lp.rv, "%lld", static_cast<long long>(new_rv)));
  }
  KindStore& ks = g_store[kind];
  ks.history.push_back(Hist{rv, o.ns, lp, o.attrs});
  while (ks.history.size() > g_opt.history) {
    ks.compacted = ks.history.front().rv;
    ks.history.pop_front();
  }
  for (Watch* w : ks.watchers)
    if ((w->ns.empty() || w->ns == o.ns) && matches(*o.attrs, w->sel)) watch_push(w, lp);
}

// Fills metadata defaults, assigns the next resourceVersion, serialises and indexes.
// `src` is the text `doc` was parsed from: when nothing but the resourceVersion changes
// (the usual case for fully-formed objects) the new text is spliced instead of re-dumped.
Obj finish(int kind, Value& doc, const Obj* prev, std::string_view src = {}) {
  // Text edits against `src` (offset, bytes removed, text inserted) when the object only
  // needs server-owned metadata filled in; anything else falls back to a DOM re-dump.
  struct Edit {
    size_t off, del;
    std::string ins;
    bool rv;
  };
  std::vector<Edit> edits;
  bool dirty = src.empty();
  if (!doc.get("kind")) {
    doc.at("kind") = Value::str(KINDS[kind].kind);
    dirty = true;
  }
  if (!doc.get("apiVersion")) {
    doc.at("apiVersion") = Value::str(KINDS[kind].api_version);
    dirty = true;
  }
  const Value* md0 = doc.get("metadata");
  if (!md0 || md0->t != Value::OBJ || md0->o.empty()) dirty = true;
  Value& md = doc.at("metadata");
  const size_t md_open = md.src_off + 1;  // just after the metadata object's '{'
  if (md.path({"name"}).empty()) {
    dirty = true;
    std::string gen(md.path({"generateName"}));
    md.at("name") = Value::str(gen + random_suffix(5));
  }
  Obj o;
  const Value* uid = md.get("uid");
  if (!uid || uid->t != Value::STR || uid->s.empty()) {
    std::string u = prev ? prev->uid : std::string();
    if (prev && !prev->created.empty() && !md.get("creationTimestamp")) {
      md.at("creationTimestamp") = Value::str(prev->created);
      edits.push_back({md_open, 0, "\"creationTimestamp\":\"" + prev->created + "\",", false});
    }
    if (u.empty()) u = uuid4();
    md.at("uid") = Value::str(u);
    edits.push_back({md_open, 0, "\"uid\":\"" + u + "\",", false});
  }
  if (!md.get("creationTimestamp")) {
    std::string ts = now_rfc3339();
    md.at("creationTimestamp") = Value::str(ts);
    edits.push_back({md_open, 0, "\"creationTimestamp\":\"" + ts + "\",", false});
  }
  o.rv = ++g_rv;
  std::string rvs = std::to_string(o.rv);
  const Value* old_rv = md.get("resourceVersion");
  if (!old_rv) {
    edits.push_back({md_open, 0, "\"resourceVersion\":\"" + rvs + "\",", true});
  } else if (old_rv->t != Value::STR || old_rv->escaped) {
    dirty = true;
  } else {
    edits.push_back({old_rv->src_off, old_rv->src_len, rvs, true});
  }
  md.at("resourceVersion") = Value::str(rvs);
  o.ns = std::string(md.path({"namespace"}));
  o.name = std::string(md.path({"name"}));
  o.uid = std::string(md.path({"uid"}));
  o.created = std::string(md.path({"creationTimestamp"}));
  if (kind == K_POD) {
    const Value* labels = md.get("labels");
    const Value* j = labels ? labels->get("batch.kubernetes.io/job-name") : nullptr;
    if (j && j->t == Value::STR) o.job = j->s;
  }
  o.attrs = attrs_of(doc);
  if (dirty) {
    o.json = std::make_shared<const std::string>(kjson::dump(doc));
    locate_rv(o);
    return o;
  }
  // src holds the text doc was parsed from (offsets are relative to src)
  std::stable_sort(edits.begin(), edits.end(), [](const Edit& a, const Edit& b) { return a.off < b.off; });
  size_t b = doc.src_off, e = static_cast<size_t>(doc.src_off) + doc.src_len, at = b;
  auto j = std::make_shared<std::string>();
  j->reserve(e - b + 128);
  for (auto& ed : edits) {
    j->append(src.data() + at, ed.off - at);
    if (ed.rv) {
      size_t q = ed.ins.find(rvs);  // digits position inside the inserted text
      o.rv_off = j->size() + (ed.del ? 0 : q);
      o.rv_len = rvs.size();
    }
    j->append(ed.ins);
    at = ed.off + ed.del;
  }
  j->append(src.data() + at, e - at);
  o.json = std::move(j);
  return o;
}

void index_pod(const Obj& o, bool add);
bool remove(int kind, std::string_view ns, std::string_view name, std::string_view propagation);

// ------------------------------------------------------------ raw fast path (bulk apply)
// The benchmark generator sends fully-formed objects by the thousand.  Building a DOM for
// each only to read a dozen fields costs more than everything else the simulator does, so
// /sim/apply scans the raw text once instead: the fields the store needs (kind, name,
// namespace, labels, the selectable field paths) and the byte positions the server edits
// (metadata's '{', resourceVersion).  Anything unusual (escapes in a needed field,
// generateName, a missing kind/metadata) falls back to the DOM path.
struct Raw {
  bool ok = true;
  std::string_view kind, name, ns, uid, created, job;
  std::string_view node, phase, ikind, iname, reason, type;
  bool has_kind = false, has_api = false, has_md = false, has_rv = false, has_gen = false;
  size_t md_open = 0, md_keys = 0, rv_off = 0, rv_len = 0;
  // labels inline (no heap: a bulk apply's lines are scanned on pool threads and dropped
  // on the loop); an object with more goes the DOM path
  static constexpr size_t kMaxLabels = 24;
  std::pair<std::string_view, std::string_view> label_buf[kMaxLabels];
  size_t nlabels = 0;
  const std::pair<std::string_view, std::string_view>* labels_begin() const { return label_buf; }
  const std::pair<std::string_view, std::string_view>* labels_end() const { return label_buf + nlabels; }
};

class RawScan {
 public:
  RawScan(const char* s, size_t n) : s_(s), n_(n) {}

  // {"type": "...", "object": {...}} → type + the object's [begin, end) and fields
  bool envelope(std::string_view& type, size_t& ob, size_t& oe, Raw& r) {
    try {
      ws();
      if (!eat('{')) return false;
      bool have_obj = false;
      while (true) {
        ws();
        if (peek() == '}') break;
        bool esc;
        std::string_view k = str(esc);
        ws();
        if (!eat(':')) return false;
        ws();
        if (k == "type" && peek() == '"') {
          type = str(esc);
          if (esc) return false;
        } else if (k == "object" && peek() == '{') {
          ob = i_;
          object(r);
          oe = i_;
          have_obj = true;
        } else {
          skip();
        }
        ws();
        if (peek() == ',') ++i_;
      }
      return have_obj && r.ok;
    } catch (const kjson::ParseError&) {
      return false;
    }
  }

 private:
  const char* s_;
  size_t n_;
  size_t i_ = 0;

  void ws() {
    while (i_ < n_ && (s_[i_] == ' ' || s_[i_] == '\t' || s_[i_] == '\r' || s_[i_] == '\n')) ++i_;
  }
  char peek() {
    if (i_ >= n_) throw kjson::ParseError("unexpected end");
    return s_[i_];
  }
  bool eat(char c) {
    if (peek() != c) return false;
    ++i_;
    return true;
  }
  // memchr to the closing quote (a quote preceded by an odd run of backslashes is escaped):
  // most of a line's bytes are inside strings, and skip() goes through here too
  std::string_view str(bool& esc) {
    if (!eat('"')) throw kjson::ParseError("expected string");
    size_t st = i_;
    while (i_ < n_) {
      const char* q = static_cast<const char*>(memchr(s_ + i_, '"', n_ - i_));
      if (!q) break;
      size_t j = static_cast<size_t>(q - s_);
      size_t bs = 0;
      while (j > st + bs && s_[j - 1 - bs] == '\\') ++bs;
      i_ = j + 1;
      if (bs % 2 == 0) {
        esc = memchr(s_ + st, '\\', j - st) != nullptr;
        return std::string_view(s_ + st, j - st);
      }
    }
    throw kjson::ParseError("unterminated string");
  }
  void skip() {
    ws();
    char c = peek();
    if (c == '"') {
      bool e;
      str(e);
      return;
    }
    if (c == '{' || c == '[') {
      int depth = 0;
      while (i_ < n_) {
        char d = s_[i_];
        if (d == '"') {
          bool e;
          str(e);
          continue;
        }
        if (d == '{' || d == '[') ++depth;
        else if ((d == '}' || d == ']') && --depth == 0) {
          ++i_;
          return;
        }
        ++i_;
      }
      throw kjson::ParseError("unterminated container");
    }
    while (i_ < n_ && s_[i_] != ',' && s_[i_] != '}' && s_[i_] != ']') ++i_;
  }
  // string value of a field the store reads: escapes → DOM fallback; non-strings are absent
  void field(std::string_view& out, Raw& r) {
    ws();
    if (peek() != '"') {
      skip();
      return;
    }
    bool esc;
    out = str(esc);
    if (esc) r.ok = false;
  }
  // iterate an object's members: fn(key) handles the value at i_ (must consume it)
  template <class F>
  void members(F&& fn) {
    ws();
    if (!eat('{')) {
      skip();
      return;
    }
    while (true) {
      ws();
      if (peek() == '}') {
        ++i_;
        return;
      }
      bool esc;
      std::string_view k = str(esc);
      ws();
      if (!eat(':')) throw kjson::ParseError("expected ':'");
      ws();
      if (esc) skip();
      else fn(k);
      ws();
      if (peek() == ',') ++i_;
    }
  }
  void object(Raw& r) {
    members([&](std::string_view k) {
      if (k == "kind") {
        r.has_kind = true;
        field(r.kind, r);
      } else if (k == "apiVersion") {
        r.has_api = true;
        skip();
      } else if (k == "metadata" && peek() == '{') {
        r.has_md = true;
        r.md_open = i_ + 1;
        members([&](std::string_view m) {
          ++r.md_keys;
          if (m == "name") field(r.name, r);
          else if (m == "namespace") field(r.ns, r);
          else if (m == "uid") field(r.uid, r);
          else if (m == "creationTimestamp") field(r.created, r);
          else if (m == "generateName") {
            r.has_gen = true;
            skip();
          } else if (m == "resourceVersion" && peek() == '"') {
            bool esc;
            size_t st = i_ + 1;
            str(esc);
            r.has_rv = true;
            r.rv_off = st;
            r.rv_len = i_ - 1 - st;
            if (esc) r.ok = false;
          } else if (m == "labels" && peek() == '{') {
            members([&](std::string_view lk) {
              std::string_view lv;
              field(lv, r);
              if (lv.data()) {
                if (r.nlabels < Raw::kMaxLabels) r.label_buf[r.nlabels++] = {lk, lv};
                else r.ok = false;
                if (lk == "batch.kubernetes.io/job-name") r.job = lv;
              }
            });
          } else {
            skip();
          }
        });
      } else if (k == "spec" && peek() == '{') {
        members([&](std::string_view f) { f == "nodeName" ? field(r.node, r) : skip(); });
      } else if (k == "status" && peek() == '{') {
        members([&](std::string_view f) { f == "phase" ? field(r.phase, r) : skip(); });
      } else if (k == "involvedObject" && peek() == '{') {
        members([&](std::string_view f) {
          if (f == "kind") field(r.ikind, r);
          else if (f == "name") field(r.iname, r);
          else skip();
        });
      } else if (k == "reason") {
        field(r.reason, r);
      } else if (k == "type") {
        field(r.type, r);
      } else {
        skip();
      }
    });
  }
};

std::shared_ptr<const Attrs> attrs_raw(const Raw& r) {
  auto a = std::make_shared<Attrs>();
  size_t bytes = 8 * 40;
  for (auto* kv = r.labels_begin(); kv != r.labels_end(); ++kv) bytes += kv->first.size() + kv->second.size() + 8;
  a->reserve(bytes + r.name.size() + r.ns.size() + r.node.size() + r.iname.size());
  for (auto* kv = r.labels_begin(); kv != r.labels_end(); ++kv) a->add(kv->first, kv->second);
  const std::pair<const char*, std::string_view> fields[] = {
      {"\x01" "f:metadata.name", r.name},  {"\x01" "f:metadata.namespace", r.ns},
      {"\x01" "f:spec.nodeName", r.node},   {"\x01" "f:status.phase", r.phase},
      {"\x01" "f:involvedObject.kind", r.ikind}, {"\x01" "f:involvedObject.name", r.iname},
      {"\x01" "f:reason", r.reason},       {"\x01" "f:type", r.type}};
  for (auto& f : fields)
    if (f.second.data()) a->add(f.first, f.second);
  return a;
}

// Store text for a raw-scanned object: server metadata spliced in (src = the line, the
// object spans [ob, oe)).  Same edits as finish() without the DOM.
Obj finish_raw(const Raw& r, std::string_view src, size_t ob, size_t oe, const Obj* prev, int64_t rv = 0) {
  Obj o;
  o.ns = std::string(r.ns);
  o.name = std::string(r.name);
  o.job = std::string(r.job);
  o.rv = rv > 0 ? rv : ++g_rv;
  std::string rvs = std::to_string(o.rv);
  std::string ins;  // inserted right after metadata's '{'
  if (r.uid.empty()) {
    o.uid = prev && !prev->uid.empty() ? prev->uid : uuid4();
    ins += "\"uid\":\"" + o.uid + "\",";
  } else {
    o.uid = std::string(r.uid);
  }
  if (!r.created.data()) {
    o.created = prev && !prev->created.empty() ? prev->created : now_rfc3339();
    ins += "\"creationTimestamp\":\"" + o.created + "\",";
  } else {
    o.created = std::string(r.created);
  }
  size_t rv_in_ins = std::string::npos;
  if (!r.has_rv) {
    rv_in_ins = ins.size() + 19;
    ins += "\"resourceVersion\":\"" + rvs + "\",";
  }
  auto j = std::make_shared<std::string>();
  j->reserve(oe - ob + ins.size() + 8);
  j->append(src.data() + ob, r.md_open - ob);
  size_t ins_at = j->size();
  j->append(ins);
  if (r.has_rv) {
    j->append(src.data() + r.md_open, r.rv_off - r.md_open);
    o.rv_off = j->size();
    j->append(rvs);
    j->append(src.data() + r.rv_off + r.rv_len, oe - r.rv_off - r.rv_len);
  } else {
    o.rv_off = ins_at + rv_in_ins;
    j->append(src.data() + r.md_open, oe - r.md_open);
  }
  o.rv_len = rvs.size();
  o.json = std::move(j);
  o.attrs = attrs_raw(r);
  return o;
}

// ------------------------------------------------------------ parallel prepare (bulk apply)
// Most of a bulk apply reads nothing of the store: scanning a line and building its store
// text and selectable attributes.  /sim/apply therefore prepares a chunk's lines on
// `--apply-threads` threads (the event loop thread included) and then commits them in
// order on the event loop — store lookup, resourceVersion, history, pod index — so the
// store stays single-threaded.  The resourceVersion is not known while preparing: the text
// gets a placeholder of the width the next one has, filled in at commit (a line whose
// resourceVersion turned out wider — a power of ten crossed mid-chunk — is rebuilt there).
struct Prep {
  std::string_view line, type;
  int kind = -1;
  // 0: not raw (DOM path), 1: DELETED, 2: text prepared, 3: raw but needs the stored
  // object (uid / creationTimestamp / resourceVersion to complete): built at commit,
  // 4: a bench LOG line (pods/log text; DOM path), 5: complete, built at commit (Pods and
  // Jobs: the loop thread that commits them also frees them — Job DELETEs, pod GC — so
  // their memory comes from that thread's heap cache, not a pool thread's)
  int mode = 0;
  Raw r;
  size_t ob = 0, oe = 0;
  Obj o;
  std::shared_ptr<std::string> text;
};

size_t digits(int64_t v) {
  size_t n = 1;
  while (v >= 10) {
    v /= 10;
    ++n;
  }
  return n;
}

void prepare(Prep& p, size_t width, bool build_all) {
  RawScan sc(p.line.data(), p.line.size());
  Raw& r = p.r;
  if (!sc.envelope(p.type, p.ob, p.oe, r)) return;
  if (p.type == "LOG") {
    p.mode = 4;
    return;
  }
  if (!r.has_kind || !r.has_api || !r.has_md || r.md_keys == 0 || r.name.empty() || r.has_gen) return;
  p.kind = kind_by_name(r.kind);
  if (p.kind < 0) return;
  if (p.type == "DELETED") {
    p.mode = 1;
    return;
  }
  if (r.uid.empty() || !r.created.data() || !r.has_rv) {
    p.mode = 3;
    return;
  }
  if (p.kind != K_EVENT && !build_all) {
    p.mode = 5;
    return;
  }
  Obj& o = p.o;
  o.ns = std::string(r.ns);
  o.name = std::string(r.name);
  o.job = std::string(r.job);
  o.uid = std::string(r.uid);
  o.created = std::string(r.created);
  auto j = std::make_shared<std::string>();
  j->reserve(p.oe - p.ob + width);
  j->append(p.line.data() + p.ob, r.rv_off - p.ob);
  o.rv_off = j->size();
  o.rv_len = width;
  j->append(width, '0');
  j->append(p.line.data() + r.rv_off + r.rv_len, p.oe - r.rv_off - r.rv_len);
  p.text = std::move(j);
  o.attrs = attrs_raw(r);
  p.mode = 2;
}

// false → the caller takes the DOM path
bool commit(Prep& p) {
  if (p.mode == 0 || p.mode == 4) return false;
  if (p.mode == 1) {
    remove(p.kind, p.r.ns, p.r.name, "Background");
    return true;
  }
  KindStore& ks = g_store[p.kind];
  auto it = ks.objs.find(okey_scratch(p.r.ns, p.r.name));
  const Obj* prev = it == ks.objs.end() ? nullptr : &it->second;
  Obj o;
  int64_t rv = ++g_rv;
  if (p.mode == 2 && digits(rv) == p.o.rv_len) {
    o = std::move(p.o);
    o.rv = rv;
    std::to_chars(&(*p.text)[o.rv_off], &(*p.text)[o.rv_off] + o.rv_len, o.rv);
    o.json = std::move(p.text);
  } else {
    o = finish_raw(p.r, p.line, p.ob, p.oe, prev, rv);
  }
  if (p.kind == K_POD && !(prev && prev->job == o.job)) {
    if (prev) index_pod(*prev, false);
    index_pod(o, true);
  }
  record(p.kind, prev ? "MODIFIED" : "ADDED", o);
  if (prev) it->second = std::move(o);
  else ks.objs.emplace(okey(p.r.ns, p.r.name), std::move(o));
  return true;
}

// fn(i) for i in [0, n) on `threads` threads (the caller's included), blocks of 16
class ParallelFor {
 public:
  void start(int threads) {
    for (int i = 1; i < threads; ++i) workers_.emplace_back([this] { loop(); });
  }
  void stop() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
    workers_.clear();
  }
  // blocks of `block` indexes; fewer than `min_n` run inline on the caller
  void run(size_t n, const std::function<void(size_t)>& fn, size_t block = 16, size_t min_n = 64) {
    if (workers_.empty() || n < min_n) {
      for (size_t i = 0; i < n; ++i) fn(i);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &fn;
      n_ = n;
      block_ = block;
      next_.store(0);
      pending_ = workers_.size();
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [this] { return pending_ == 0; });
    fn_ = nullptr;
  }

  // fn(0) on the caller, fn(1..n-1) on the pool threads only (the caller waits for them)
  void run_pinned(size_t n, const std::function<void(size_t)>& fn) {
    if (workers_.empty() || n < 2) {
      for (size_t i = 0; i < n; ++i) fn(i);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &fn;
      n_ = n;
      block_ = 1;
      next_.store(1);
      pending_ = workers_.size();
      ++gen_;
    }
    cv_.notify_all();
    fn(0);
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [this] { return pending_ == 0; });
    fn_ = nullptr;
  }

 private:
  void work() {
    size_t b;
    while ((b = next_.fetch_add(block_)) < n_)
      for (size_t i = b; i < std::min(n_, b + block_); ++i) (*fn_)(i);
  }
  void loop() {
    uint64_t seen = 0;
    while (true) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      work();
      std::lock_guard<std::mutex> lk(mu_);
      if (--pending_ == 0) done_.notify_one();
    }
  }
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  const std::function<void(size_t)>* fn_ = nullptr;
  size_t n_ = 0, block_ = 16;
  std::atomic<size_t> next_{0};
  size_t pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
} g_apply_pool;

void index_pod(const Obj& o, bool add) {
  if (o.job.empty()) return;
  const std::string& k = okey_scratch(o.ns, o.job);
  if (add) {
    auto it = g_pods_by_job.find(k);
    if (it == g_pods_by_job.end()) it = g_pods_by_job.emplace(okey(o.ns, o.job), std::set<std::string>()).first;
    it->second.insert(o.name);
  } else {
    auto it = g_pods_by_job.find(k);
    if (it != g_pods_by_job.end()) {
      it->second.erase(o.name);
      if (it->second.empty()) g_pods_by_job.erase(it);
    }
  }
}

// returns false when the object exists already
bool create(int kind, Value& doc, std::string* out_json, std::string_view src = {}) {
  Value& md = doc.at("metadata");
  if (md.path({"name"}).empty() && md.path({"generateName"}).empty()) throw kjson::ParseError("metadata.name required");
  if (!md.path({"name"}).empty()) {
    if (g_store[kind].objs.count(okey(md.path({"namespace"}), md.path({"name"})))) return false;
  }
  Obj o = finish(kind, doc, nullptr, src);
  while (g_store[kind].objs.count(okey(o.ns, o.name))) {  // generateName collision
    md.at("name") = Value::str(std::string(md.path({"generateName"})) + random_suffix(5));
    o = finish(kind, doc, nullptr);
  }
  if (kind == K_POD) index_pod(o, true);
  record(kind, "ADDED", o);
  if (out_json) *out_json = *o.json;
  g_store[kind].objs[okey(o.ns, o.name)] = std::move(o);
  return true;
}

// 0 ok, 1 not found, 2 conflict
int update(int kind, Value& doc, bool check_rv, std::string* out_json, std::string_view src = {}) {
  Value& md = doc.at("metadata");
  std::string k = okey(md.path({"namespace"}), md.path({"name"}));
  auto it = g_store[kind].objs.find(k);
  if (it == g_store[kind].objs.end()) return 1;
  std::string want(md.path({"resourceVersion"}));
  if (check_rv && !want.empty() && want != std::to_string(it->second.rv)) return 2;
  Obj o = finish(kind, doc, &it->second, src);
  if (kind == K_POD && it->second.job != o.job) {
    index_pod(it->second, false);
    index_pod(o, true);
  }
  record(kind, "MODIFIED", o);
  if (out_json) *out_json = *o.json;
  it->second = std::move(o);
  return 0;
}

bool remove(int kind, std::string_view ns, std::string_view name, std::string_view propagation) {
  auto it = g_store[kind].objs.find(okey_scratch(ns, name));
  if (it == g_store[kind].objs.end()) return false;
  Obj o = std::move(it->second);
  g_store[kind].objs.erase(it);
  if (kind == K_POD) {
    index_pod(o, false);
    if (!g_pod_logs.empty()) g_pod_logs.erase(okey_scratch(o.ns, o.name));
    if (!g_log_dirs.empty()) remove_pod_logs(o.ns, o.name);
  }
  if (o.rv_off != std::string::npos) {
    record(kind, "DELETED", o, ++g_rv);  // new resourceVersion spliced in on send
  } else {
    Value doc = kjson::parse(*o.json);
    o.rv = ++g_rv;
    doc.at("metadata").at("resourceVersion") = Value::str(std::to_string(o.rv));
    o.json = std::make_shared<const std::string>(kjson::dump(doc));
    record(kind, "DELETED", o);
  }
  ++g_stats.deleted;
  if (kind == K_JOB && (propagation == "Background" || propagation == "Foreground")) {
    auto pit = g_pods_by_job.find(okey_scratch(o.ns, o.name));
    if (pit != g_pods_by_job.end()) {
      // take the job's pod set out of the index (the pods' own unindexing then finds
      // nothing to do) instead of copying every name
      auto node = g_pods_by_job.extract(pit);
      if (g_opt.async_gc && propagation == "Background") {
        for (auto& p : node.mapped()) g_gc.emplace_back(o.ns, p);
        g_gc_cv.notify_one();
      } else {
        for (auto& p : node.mapped()) remove(K_POD, o.ns, p, propagation);
      }
    }
  }
  if (g_opt.async_gc) {
    std::lock_guard<std::mutex> glk(g_graves_mu);
    g_graves.push_back(std::move(o));
    if (g_graves.size() >= 1024) g_gc_cv.notify_one();
  }
  return true;
}

// ============================================================ connections
struct Conn {
  int fd;
  std::string in;
  std::string out;
  // --api-latency-us: answers held until their due time (CLOCK_MONOTONIC ns), FIFO so a
  // pipelined connection's answers keep their order
  std::deque<std::pair<int64_t, std::string>> delayed;
  Watch* watch = nullptr;
  bool close_after = false;
  uint32_t mask = EPOLLIN | EPOLLRDHUP;  // registered epoll interest (skip redundant epoll_ctl)
};

int g_ep = -1;
std::unordered_map<int, std::unique_ptr<Conn>> g_conns;
std::set<Conn*> g_dirty;  // connections with queued output
std::set<Conn*> g_delayed;  // connections holding answers for --api-latency-us
bool g_delay_this = false;  // the request being handled is answered after the latency

void set_nonblock(int fd) { fcntl(fd, F_SETFL, fcntl(fd, F_GETFL, 0) | O_NONBLOCK); }

void interest(Conn& c) {
  uint32_t want = EPOLLIN | EPOLLRDHUP | (c.out.empty() ? 0u : static_cast<uint32_t>(EPOLLOUT));
  if (want == c.mask) return;  // one syscall per response saved on the hot path
  epoll_event ev{};
  ev.events = want;
  ev.data.fd = c.fd;
  epoll_ctl(g_ep, EPOLL_CTL_MOD, c.fd, &ev);
  c.mask = want;
}

void end_watch(Conn& c, bool terminate_chunked) {
  Watch* w = c.watch;
  if (!w) return;
  auto& ws = g_store[w->kind].watchers;
  for (size_t i = 0; i < ws.size(); ++i)
    if (ws[i] == w) {
      ws.erase(ws.begin() + static_cast<long>(i));
      break;
    }
  if (terminate_chunked) {
    if (!w->idle()) {
      char hdr[24];
      snprintf(hdr, sizeof hdr, "%zx\r\n", w->pending.size() + w->lines_bytes);
      c.out += hdr;
      c.out += w->pending;
      for (auto& l : w->lines) append_line(c.out, l);
      c.out += "\r\n";
    }
    c.out += "0\r\n\r\n";
    g_dirty.insert(&c);
  }
  delete w;
  c.watch = nullptr;
}

void close_conn(int fd) {
  auto it = g_conns.find(fd);
  if (it == g_conns.end()) return;
  Conn* c = it->second.get();
  end_watch(*c, false);
  g_dirty.erase(c);
  g_delayed.erase(c);
  epoll_ctl(g_ep, EPOLL_CTL_DEL, fd, nullptr);
  close(fd);
  g_conns.erase(it);
}

std::mutex g_dirty_mu;  // a bulk apply's per-kind commit threads mark watch connections dirty

void watch_push(Watch* w, const Line& line) {
  if (w->idle()) {
    auto it = g_conns.find(w->fd);
    if (it != g_conns.end()) {
      std::lock_guard<std::mutex> lk(g_dirty_mu);
      g_dirty.insert(it->second.get());
    }
  }
  w->lines_bytes += line.size();
  w->lines.push_back(line);
}

// Sends a watch's committed lines as one chunk.  With nothing queued ahead of it the
// chunk goes out as iovecs over the shared line buffers; whatever the socket does not
// take is copied into c.out.  false = connection error.
bool flush_watch(Conn& c) {
  Watch* w = c.watch;
  // the committed lines are taken under the store lock (the apply thread may be appending)
  // and sent without it; the taken Lines keep their texts alive
  thread_local std::vector<Line> lines;
  thread_local std::string pending;
  size_t lines_bytes;
  {
    StoreLock lk;
    if (w->idle()) return true;
    lines.swap(w->lines);
    pending.swap(w->pending);
    lines_bytes = w->lines_bytes;
    w->clear();
    w->last_ms = mono_ms();
  }
  struct Done {
    ~Done() {
      lines.clear();
      pending.clear();
    }
  } done;
  char hdr[24];
  int hl = snprintf(hdr, sizeof hdr, "%zx\r\n", pending.size() + lines_bytes);
  if (!c.out.empty()) {  // keep the byte order: append behind what is queued
    c.out.append(hdr, static_cast<size_t>(hl));
    c.out += pending;
    for (auto& l : lines) append_line(c.out, l);
    c.out += "\r\n";
    return true;
  }
  static char crlf[] = "\r\n";
  thread_local std::vector<iovec> iov;  // reused across flushes (one per fan-out thread)
  iov.clear();
  iov.reserve(5 * lines.size() + 3);
  iov.push_back({hdr, static_cast<size_t>(hl)});
  if (!pending.empty()) iov.push_back({pending.data(), pending.size()});
  for (auto& l : lines) {  // pointers into the taken lines stay valid until they are cleared
    iov.push_back({const_cast<char*>(l.prefix->data()), l.prefix->size()});
    char* j = const_cast<char*>(l.json->data());
    if (l.rvn) {
      iov.push_back({j, l.rv_off});
      iov.push_back({const_cast<char*>(l.rv), l.rvn});
      iov.push_back({j + l.rv_off + l.rv_len, l.json->size() - l.rv_off - l.rv_len});
    } else {
      iov.push_back({j, l.json->size()});
    }
    iov.push_back({g_line_end, 2});
  }
  iov.push_back({crlf, 2});
  size_t i = 0;
  bool ok = true;
  while (i < iov.size()) {
    msghdr m{};
    m.msg_iov = &iov[i];
    m.msg_iovlen = std::min<size_t>(iov.size() - i, 1024);  // IOV_MAX
    ssize_t n = sendmsg(c.fd, &m, MSG_NOSIGNAL);
    g_stats.sends.fetch_add(1, std::memory_order_relaxed);
    if (n > 0) {
      g_stats.send_bytes.fetch_add(static_cast<uint64_t>(n), std::memory_order_relaxed);
      size_t k = static_cast<size_t>(n);
      while (k > 0) {
        if (k >= iov[i].iov_len) {
          k -= iov[i].iov_len;
          ++i;
        } else {
          iov[i].iov_base = static_cast<char*>(iov[i].iov_base) + k;
          iov[i].iov_len -= k;
          k = 0;
        }
      }
      continue;
    }
    if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
      g_stats.eagain.fetch_add(1, std::memory_order_relaxed);
      break;
    }
    if (n < 0 && errno == EINTR) continue;
    ok = false;
    break;
  }
  for (; ok && i < iov.size(); ++i) c.out.append(static_cast<const char*>(iov[i].iov_base), iov[i].iov_len);
  return ok;
}

// write out a connection's queued bytes (and its watch's committed lines)
bool flush(Conn& c) {
  if (c.watch && !flush_watch(c)) return false;
  size_t off = 0;
  while (off < c.out.size()) {
    ssize_t n = send(c.fd, c.out.data() + off, c.out.size() - off, MSG_NOSIGNAL);
    g_stats.sends.fetch_add(1, std::memory_order_relaxed);
    if (n > 0) {
      off += static_cast<size_t>(n);
      g_stats.send_bytes.fetch_add(static_cast<uint64_t>(n), std::memory_order_relaxed);
      continue;
    }
    if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
      g_stats.eagain.fetch_add(1, std::memory_order_relaxed);
      break;
    }
    if (n < 0 && errno == EINTR) continue;
    return false;
  }
  c.out.erase(0, off);
  if (c.out.empty() && c.close_after) return false;
  interest(c);
  return true;
}

// Fan-out pool: flushes of distinct connections are independent (each touches only its
// connection, its watch and the immutable shared line texts), so one loop iteration's
// dirty connections are split across `flush_threads` threads; the event loop thread
// takes part and waits for the rest before it touches any connection again.
class FlushPool {
 public:
  void start(int threads) {
    for (int i = 1; i < threads; ++i) workers_.emplace_back([this] { loop(); });
  }
  void stop() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
    workers_.clear();
  }
  // ok[i] = flush(*dirty[i])
  void run(const std::vector<Conn*>& dirty, std::vector<uint8_t>& ok) {
    if (workers_.empty() || dirty.size() < 2) {
      for (size_t i = 0; i < dirty.size(); ++i) ok[i] = flush(*dirty[i]);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = &dirty;
      ok_ = &ok;
      next_.store(0);
      pending_ = workers_.size();
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [this] { return pending_ == 0; });
    job_ = nullptr;
  }

 private:
  void work() {
    const auto& d = *job_;
    size_t i;
    while ((i = next_.fetch_add(1)) < d.size()) (*ok_)[i] = flush(*d[i]) ? 1 : 0;
  }
  void loop() {
    uint64_t seen = 0;
    while (true) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      work();
      std::lock_guard<std::mutex> lk(mu_);
      if (--pending_ == 0) done_.notify_one();
    }
  }
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  const std::vector<Conn*>* job_ = nullptr;
  std::vector<uint8_t>* ok_ = nullptr;
  std::atomic<size_t> next_{0};
  size_t pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
} g_flush_pool;

// ============================================================ HTTP
std::string status_text(int code) {
  switch (code) {
    case 200: return "OK";
    case 201: return "Created";
    case 400: return "Bad Request";
    case 401: return "Unauthorized";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 409: return "Conflict";
    case 410: return "Gone";
    case 411: return "Length Required";
    case 429: return "Too Many Requests";
    case 500: return "Internal Server Error";
  }
  return "Unknown";
}

void respond(Conn& c, int code, const std::string& body, const char* extra = "") {
  char hdr[200];
  snprintf(hdr, sizeof hdr, "HTTP/1.1 %d %s\r\nContent-Type: application/json\r\nContent-Length: %zu\r\n%s%s\r\n", code,
           status_text(code).c_str(), body.size(), extra, c.close_after ? "Connection: close\r\n" : "");
  if (g_delay_this || !c.delayed.empty()) {
    // priced answer (or one queued behind a priced answer on this connection)
    int64_t due = mono_ns() + (g_delay_this ? g_opt.api_latency_us * 1000 : 0);
    if (!c.delayed.empty()) due = std::max(due, c.delayed.back().first);
    std::string msg(hdr);
    msg += body;
    c.delayed.emplace_back(due, std::move(msg));
    g_delayed.insert(&c);
    ++g_stats.delayed;
    return;
  }
  c.out += hdr;
  c.out += body;
  g_dirty.insert(&c);
}

// move due answers to the output buffers; returns ms until the next one is due (-1: none)
int release_delayed() {
  if (g_delayed.empty()) return -1;
  int64_t now = mono_ns(), next = INT64_MAX;
  for (auto it = g_delayed.begin(); it != g_delayed.end();) {
    Conn* c = *it;
    while (!c->delayed.empty() && c->delayed.front().first <= now) {
      c->out += c->delayed.front().second;
      c->delayed.pop_front();
      g_dirty.insert(c);
    }
    if (c->delayed.empty()) {
      it = g_delayed.erase(it);
    } else {
      next = std::min(next, c->delayed.front().first);
      ++it;
    }
  }
  if (next == INT64_MAX) return -1;
  return static_cast<int>(std::max<int64_t>(0, (next - now + 999999) / 1000000));
}

// --write-qps: token bucket over mutating requests
double g_wtokens = -1;
int64_t g_wlast = 0;
bool write_admitted() {
  if (g_opt.write_qps <= 0) return true;
  double burst = g_opt.write_burst > 0 ? g_opt.write_burst : std::max(1.0, g_opt.write_qps);
  int64_t now = mono_ns();
  if (g_wtokens < 0) g_wtokens = burst;
  else g_wtokens = std::min(burst, g_wtokens + (now - g_wlast) * 1e-9 * g_opt.write_qps);
  g_wlast = now;
  if (g_wtokens < 1.0) return false;
  g_wtokens -= 1.0;
  return true;
}

std::string status_body(int code, const std::string& reason, const std::string& message);

void too_many(Conn& c) {
  ++g_stats.throttled;
  char extra[48];
  snprintf(extra, sizeof extra, "Retry-After: %d\r\n", g_opt.retry_after_s);
  bool d = g_delay_this;
  g_delay_this = false;  // a rejection is cheap: answered at once (still in order)
  respond(c, 429, status_body(429, "TooManyRequests", "too many requests, please try again later"), extra);
  g_delay_this = d;
}

std::string status_body(int code, const std::string& reason, const std::string& message) {
  std::string s = "{\"kind\":\"Status\",\"apiVersion\":\"v1\",\"status\":\"Failure\",\"message\":";
  kjson::escape(s, message);
  s += ",\"reason\":";
  kjson::escape(s, reason);
  s += ",\"code\":" + std::to_string(code) + "}";
  return s;
}

std::string pct_decode(std::string_view s) {
  auto hv = [](char ch) -> int {
    if (ch >= '0' && ch <= '9') return ch - '0';
    if (ch >= 'a' && ch <= 'f') return ch - 'a' + 10;
    if (ch >= 'A' && ch <= 'F') return ch - 'A' + 10;
    return -1;
  };
  std::string out;
  out.reserve(s.size());
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '+') {
      out += ' ';
    } else if (s[i] == '%' && i + 2 < s.size() && hv(s[i + 1]) >= 0 && hv(s[i + 2]) >= 0) {
      out += static_cast<char>(hv(s[i + 1]) * 16 + hv(s[i + 2]));
      i += 2;
    } else {
      out += s[i];
    }
  }
  return out;
}

struct Request {
  std::string method, path;
  std::map<std::string, std::string> query;
  std::string auth;
  std::string_view body;  // points into the connection's input buffer (valid while handled)
  bool close = false;
};

std::string q(const Request& r, const char* k, const char* dflt = "") {
  auto it = r.query.find(k);
  return it == r.query.end() ? std::string(dflt) : it->second;
}

// splits /api/v1/namespaces/{ns}/{plural}[/{name}] (and /apis/{g}/{v}/..., cluster-wide)
bool route(const std::string& path, int& kind, std::string& ns, std::string& name) {
  std::vector<std::string_view> seg;
  std::string_view p(path);
  size_t i = 0;
  while (i < p.size()) {
    while (i < p.size() && p[i] == '/') ++i;
    size_t j = p.find('/', i);
    if (j == std::string_view::npos) j = p.size();
    if (j > i) seg.push_back(p.substr(i, j - i));
    i = j;
  }
  size_t k;
  if (seg.size() >= 2 && seg[0] == "api") k = 2;
  else if (seg.size() >= 3 && seg[0] == "apis") k = 3;
  else return false;
  ns.clear();
  name.clear();
  if (seg.size() > k + 1 && seg[k] == "namespaces" && kind_by_plural(seg[k]) < 0) {
    ns = std::string(seg[k + 1]);
    k += 2;
  }
  if (seg.size() <= k) return false;
  kind = kind_by_plural(seg[k]);
  if (kind < 0) return false;
  if (seg.size() == k + 2) name = std::string(seg[k + 1]);
  else if (seg.size() > k + 2) return false;
  return true;
}

void h_list(Conn& c, const Request& r, int kind, const std::string& ns) {
  std::string cont = q(r, "continue");
  long limit = atol(q(r, "limit", "0").c_str());
  const Snapshot* snap = nullptr;
  Snapshot fresh;
  std::string sid;
  size_t start = 0;
  if (!cont.empty()) {
    size_t colon = cont.find(':');
    sid = cont.substr(0, colon);
    auto it = g_snapshots.find(sid);
    if (it == g_snapshots.end() || colon == std::string::npos) {
      respond(c, 410, status_body(410, "Expired", "the provided continue parameter is too old"));
      return;
    }
    snap = &it->second;
    start = static_cast<size_t>(atol(cont.c_str() + colon + 1));
  } else {
    Selector sel;
    parse_selector(q(r, "labelSelector"), false, sel);
    parse_selector(q(r, "fieldSelector"), true, sel);
    fresh.rv = g_rv;
    for (auto& kv : g_store[kind].objs)
      if ((ns.empty() || kv.second.ns == ns) && matches(*kv.second.attrs, sel)) fresh.items.push_back(kv.second.json);
    snap = &fresh;
  }
  size_t end = snap->items.size();
  std::string next;
  if (limit > 0 && start + static_cast<size_t>(limit) < snap->items.size()) {
    end = start + static_cast<size_t>(limit);
    if (cont.empty()) {
      sid = uuid4().substr(0, 12);
      g_snapshots[sid] = std::move(fresh);
      snap = &g_snapshots[sid];
      g_snapshot_order.push_back(sid);
      while (g_snapshot_order.size() > 64) {
        g_snapshots.erase(g_snapshot_order.front());
        g_snapshot_order.pop_front();
      }
    }
    next = sid + ":" + std::to_string(end);
  }
  std::string body = "{\"kind\":\"";
  body += KINDS[kind].kind;
  body += "List\",\"apiVersion\":\"";
  body += KINDS[kind].api_version;
  body += "\",\"metadata\":{\"resourceVersion\":\"" + std::to_string(snap->rv) + "\"";
  if (!next.empty()) body += ",\"continue\":\"" + next + "\"";
  body += "},\"items\":[";
  for (size_t i = start; i < end && i < snap->items.size(); ++i) {
    if (i > start) body += ',';
    body += *snap->items[i];
  }
  body += "]}";
  respond(c, 200, body);
}

void h_watch(Conn& c, const Request& r, int kind, const std::string& ns) {
  ++g_stats.watch_requests;
  auto* w = new Watch{c.fd, kind, ns, {}, q(r, "allowWatchBookmarks") == "true" || q(r, "allowWatchBookmarks") == "1", 0, 0, {}, {}, 0};
  parse_selector(q(r, "labelSelector"), false, w->sel);
  parse_selector(q(r, "fieldSelector"), true, w->sel);
  long timeout = atol(q(r, "timeoutSeconds", "0").c_str());
  w->deadline_ms = mono_ms() + (timeout > 0 ? timeout : 1800) * 1000;
  w->last_ms = mono_ms();
  c.out += "HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nTransfer-Encoding: chunked\r\n\r\n";
  c.watch = w;
  KindStore& ks = g_store[kind];
  std::string rv_s = q(r, "resourceVersion");
  if (!rv_s.empty() && rv_s != "0") {
    int64_t rv = atoll(rv_s.c_str());
    if (rv < ks.compacted) {
      std::string msg = "too old resource version: " + rv_s + " (" + std::to_string(ks.compacted) + ")";
      w->pending = "{\"type\":\"ERROR\",\"object\":" + status_body(410, "Expired", msg) + "}\n";
      ks.watchers.push_back(w);
      end_watch(c, true);
      return;
    }
    // history is in RV order: binary-search the first entry after rv
    size_t lo = 0, hi = ks.history.size();
    while (lo < hi) {
      size_t mid = (lo + hi) / 2;
      if (ks.history[mid].rv <= rv) lo = mid + 1;
      else hi = mid;
    }
    for (size_t i = lo; i < ks.history.size(); ++i) {
      const Hist& h = ks.history[i];
      if ((ns.empty() || h.ns == ns) && matches(*h.attrs, w->sel)) {
        w->lines_bytes += h.line.size();
        w->lines.push_back(h.line);
      }
    }
  }
  ks.watchers.push_back(w);
  g_dirty.insert(&c);
}

void expire_kind(int kind) {
  KindStore& ks = g_store[kind];
  if (!ks.history.empty()) ks.compacted = ks.history.back().rv;
  ks.history.clear();
}

void close_watches(int only_kind) {
  std::vector<Conn*> cs;
  for (auto& kv : g_conns)
    if (kv.second->watch && (only_kind < 0 || kv.second->watch->kind == only_kind)) cs.push_back(kv.second.get());
  for (Conn* c : cs) end_watch(*c, true);
}

std::mutex g_pool_mu;  // one bulk apply at a time uses the apply pool (loop port or apply port)

// Applies an NDJSON body of watch events; returns the /sim/apply answer.  `locked`: the
// caller (the event loop) holds g_store_mu.  Otherwise (the apply port) the lines are
// prepared without it — every object's text built on the pool — and committed under it.
std::string apply_body(std::string_view b, bool expire, bool locked) {
  std::lock_guard<std::mutex> pool_lk(g_pool_mu);
  int64_t t0 = mono_ns();
  size_t pos = 0, n = 0;
  std::vector<Prep> preps;
  preps.reserve(b.size() / 512 + 16);  // a guess (objects are ~0.6-1.5 KB): no pass over the body
  while (pos < b.size()) {
    size_t nl = b.find('\n', pos);
    if (nl == std::string::npos) nl = b.size();
    std::string_view line(b.data() + pos, nl - pos);
    pos = nl + 1;
    if (line.find_first_not_of(" \t\r") == std::string_view::npos) continue;
    preps.emplace_back().line = line;
  }
  size_t width = digits(g_rv + 1);
  g_apply_pool.run(preps.size(), [&](size_t i) { prepare(preps[i], width, !locked); });
  int64_t t_prep = mono_ns() - t0;
  std::unique_ptr<StoreLock> lk;
  if (!locked) lk = std::make_unique<StoreLock>();
  // Kinds are independent stores with their own histories and watchers: when every line is
  // a prepared object, an Event deletion or a LOG line, each kind's lines are committed in
  // order on a thread of their own (the Events, half of a benchmark's lines, beside the Pods
  // and Jobs).  Anything that crosses kinds or needs the serial helpers — a Job or Pod
  // deletion (GC cascade, pod index, pod logs), a line for the DOM path, an object to
  // complete from the stored one — keeps the whole chunk on one thread, in order.
  bool by_kind = g_opt.apply_threads > 1;
  std::vector<std::vector<Prep*>> kinds(NKINDS);
  for (Prep& p : preps) {
    if (!by_kind) break;
    if (p.mode == 2 || p.mode == 5 || (p.mode == 1 && p.kind != K_JOB && p.kind != K_POD)) kinds[p.kind].push_back(&p);
    else if (p.mode != 4) by_kind = false;
  }
  if (by_kind) {
    // the Events (most lines, and all the expiry deletions) on a pool thread; Pods and Jobs on
    // the calling thread (on the loop port: the loop, which also deletes them — Job DELETE
    // requests, GC — so their memory is freed by the thread whose heap cache it came from)
    std::vector<std::vector<int>> groups(1);
    for (int k = 0; k < NKINDS; ++k) {
      if (kinds[k].empty()) continue;
      if (k == K_EVENT) groups.push_back({k});
      else groups[0].push_back(k);
    }
    g_apply_pool.run_pinned(groups.size(), [&](size_t i) {
      for (int k : groups[i])
        for (Prep* p : kinds[k]) commit(*p);
    });
    g_stats.commit_parallel += 1;
  }
  for (Prep& p : preps) {
    std::string_view line = p.line;
    if (by_kind ? p.mode != 4 : commit(p)) {
      ++n;
      continue;
    }
    Value ev = kjson::parse(line);
    std::string type(ev.path({"type"}));
    Value* obj = ev.get("object");
    std::string_view osrc = line;  // obj's source offsets are relative to the line
    if (!obj || obj->t != Value::OBJ) throw kjson::ParseError("event without object");
    if (type == "LOG") {
      g_pod_logs[okey(obj->path({"namespace"}), obj->path({"pod"}))][std::string(obj->path({"container"}))] =
          std::string(obj->path({"text"}));
      if (!g_opt.log_root.empty() && !obj->path({"uid"}).empty()) {
        std::string_view ns = obj->path({"namespace"}), pod = obj->path({"pod"}), uid = obj->path({"uid"});
        write_cri_log(ns, pod, uid, obj->path({"container"}), 0, obj->path({"text"}));
        g_log_dirs[std::string(ns) + '\x01' + std::string(pod)] = std::string(uid);
      }
      ++n;
      continue;
    }
    int kind = kind_by_name(obj->path({"kind"}));
    if (kind < 0) throw kjson::ParseError("unknown kind");
    if (type == "DELETED") {
      remove(kind, std::string(obj->path({"metadata", "namespace"})), std::string(obj->path({"metadata", "name"})),
             "Background");
    } else if (type == "MODIFIED") {
      if (update(kind, *obj, false, nullptr, osrc) == 1) create(kind, *obj, nullptr, osrc);
    } else {
      if (!create(kind, *obj, nullptr, osrc)) update(kind, *obj, false, nullptr, osrc);
    }
    ++n;
  }
  g_stats.applied += n;
  g_stats.prepare_ns += t_prep;
  if (expire) {
    // compaction that overtakes the watchers: undelivered lines are lost, resuming
    // streams get 410 Gone and must re-list (exercises the informer's relist diff)
    for (auto& kv : g_conns)
      if (kv.second->watch) kv.second->watch->clear();
    for (int k = 0; k < NKINDS; ++k) expire_kind(k);
    close_watches(-1);
  }
  g_stats.apply_ns += mono_ns() - t0;
  char buf[160];
  snprintf(buf, sizeof buf, "{\"applied\":%zu,\"rv\":%lld,\"t_push\":%.9f}", n, static_cast<long long>(g_rv),
           static_cast<double>(t0) / 1e9);
  return buf;
}

void h_apply(Conn& c, const Request& r) { respond(c, 200, apply_body(r.body, q(r, "expire") == "1", true)); }

// GET /api/v1/namespaces/{ns}/pods/{name}/log?container=&tailLines=&limitBytes= (kubelet-proxied
// in a real cluster; priced like any object request with --api-latency-us)
// false: not a pods/{name}/log path (the caller routes it as an object path)
bool h_pod_log(Conn& c, const Request& r) {
  std::string_view p(r.path);
  const std::string_view pre = "/api/v1/namespaces/";
  if (p.substr(0, pre.size()) != pre) return false;
  p.remove_prefix(pre.size());
  size_t a = p.find('/');
  if (a == std::string_view::npos || p.substr(a, 6) != "/pods/") return false;
  std::string ns(p.substr(0, a));
  std::string_view rest = p.substr(a + 6);
  if (rest.size() <= 4 || rest.find('/') != rest.size() - 4) return false;  // exactly "<name>/log"
  std::string name(rest.substr(0, rest.size() - 4));
  struct DelayScope {
    DelayScope() { g_delay_this = g_opt.api_latency_us > 0; }
    ~DelayScope() { g_delay_this = false; }
  } delay_scope;
  if (!g_store[K_POD].objs.count(okey(ns, name))) {
    respond(c, 404, status_body(404, "NotFound", "pods \"" + name + "\" not found"));
    return true;
  }
  std::string container = q(r, "container");
  auto pit = g_pod_logs.find(okey(ns, name));
  const std::string* text = nullptr;
  if (pit != g_pod_logs.end()) {
    auto cit = container.empty() ? pit->second.begin() : pit->second.find(container);
    if (cit != pit->second.end()) text = &cit->second;
  }
  if (!text) {
    respond(c, 400, status_body(400, "BadRequest", "container \"" + container + "\" has no log"));
    return true;
  }
  std::string_view body(*text);
  long tail = atol(q(r, "tailLines", "0").c_str());
  if (tail > 0) {
    size_t cut = body.size();
    long lines = 0;
    size_t end = body.size();
    if (end && body[end - 1] == '\n') --end;
    for (size_t i = end; i > 0; --i)
      if (body[i - 1] == '\n' && ++lines == tail) {
        cut = i;
        break;
      }
    if (lines >= tail) body = body.substr(cut);
  }
  long limit = atol(q(r, "limitBytes", "0").c_str());
  if (limit > 0 && static_cast<size_t>(limit) < body.size()) body = body.substr(0, static_cast<size_t>(limit));
  respond(c, 200, std::string(body));
  return true;
}

void handle(Conn& c, Request& r) {
  ++g_stats.requests;
  c.close_after = r.close;
  if (r.path.rfind("/sim/", 0) == 0) {
    if (r.path == "/sim/apply" && r.method == "POST") return h_apply(c, r);
    if (r.path == "/sim/stats") {
      std::string s = "{\"requests\":" + std::to_string(g_stats.requests) +
                      ",\"watch_requests\":" + std::to_string(g_stats.watch_requests) + ",\"rv\":" + std::to_string(g_rv) +
                      ",\"deleted\":" + std::to_string(g_stats.deleted) + ",\"applied\":" + std::to_string(g_stats.applied) +
                      ",\"throttled\":" + std::to_string(g_stats.throttled) + ",\"delayed\":" + std::to_string(g_stats.delayed) +
                      ",\"loops\":" + std::to_string(g_stats.loops) + ",\"sends\":" + std::to_string(g_stats.sends) +
                      ",\"send_bytes\":" + std::to_string(g_stats.send_bytes) + ",\"eagain\":" + std::to_string(g_stats.eagain) +
                      ",\"apply_ns\":" + std::to_string(g_stats.apply_ns) + ",\"prepare_ns\":" + std::to_string(g_stats.prepare_ns) + ",\"commit_parallel\":" + std::to_string(g_stats.commit_parallel) + ",\"request_ns\":" + std::to_string(g_stats.request_ns) +
                      ",\"flush_ns\":" + std::to_string(g_stats.flush_ns) + ",\"recv_ns\":" + std::to_string(g_stats.recv_ns) +
                      ",\"busy_ns\":" + std::to_string(g_stats.busy_ns) +
                      ",\"store_ns\":" + std::to_string(g_stats.store_ns) +
                      ",\"apply_thread_ns\":" + std::to_string(g_stats.apply_thread_ns.load()) +
                      ",\"gc_ns\":" + std::to_string(g_stats.gc_ns.load()) + ",\"gc_pods\":" + std::to_string(g_stats.gc_pods) +
                      ",\"gc_pending\":" + std::to_string(g_gc.size()) +
                      ",\"apply_conn_ns\":{";
      {
        std::lock_guard<std::mutex> lk(g_apply_conn_mu);
        bool first = true;
        for (const auto& [id, ns] : g_apply_conn_ns) {
          if (!first) s += ',';
          first = false;
          s += "\"" + std::to_string(id) + "\":" + std::to_string(ns);
        }
      }
      s += "},\"objects\":{";
      for (int k = 0; k < NKINDS; ++k) {
        if (k) s += ',';
        s += "\"" + std::string(KINDS[k].kind) + "\":" + std::to_string(g_store[k].objs.size());
      }
      s += "}}";
      return respond(c, 200, s);
    }
    if (r.path == "/sim/expire" || r.path == "/sim/close-watches") {
      std::string k = q(r, "kind");
      int kind = k.empty() ? -1 : kind_by_name(k);
      if (r.path == "/sim/expire")
        for (int i = 0; i < NKINDS; ++i)
          if (kind < 0 || kind == i) expire_kind(i);
      close_watches(kind);
      return respond(c, 200, "{}");
    }
    return respond(c, 404, status_body(404, "NotFound", "no such simulator endpoint"));
  }
  if (!g_opt.token.empty() && r.auth != "Bearer " + g_opt.token)
    return respond(c, 401, status_body(401, "Unauthorized", "Unauthorized"));
  if (r.method == "GET" && r.path.size() > 4 && r.path.compare(r.path.size() - 4, 4, "/log") == 0 && h_pod_log(c, r))
    return;
  int kind;
  std::string ns, name;
  if (!route(r.path, kind, ns, name)) return respond(c, 404, status_body(404, "NotFound", "the server could not find the requested resource"));
  const char* kn = KINDS[kind].kind;
  std::string lower(kn);
  for (auto& ch : lower) ch = static_cast<char>(tolower(static_cast<unsigned char>(ch)));
  if (r.method == "GET" && name.empty()) {
    std::string wq = q(r, "watch");
    if (wq == "1" || wq == "true") return h_watch(c, r, kind, ns);
    return h_list(c, r, kind, ns);
  }
  if (r.method != "GET") {
    if (r.method == "DELETE" && kind == K_JOB && g_opt.throttle_deletes > 0) {
      --g_opt.throttle_deletes;
      return too_many(c);
    }
    if (!write_admitted()) return too_many(c);
  }
  struct DelayScope {
    DelayScope() { g_delay_this = g_opt.api_latency_us > 0; }
    ~DelayScope() { g_delay_this = false; }
  } delay_scope;
  if (r.method == "GET") {
    auto it = g_store[kind].objs.find(okey(ns, name));
    if (it == g_store[kind].objs.end()) return respond(c, 404, status_body(404, "NotFound", lower + "s \"" + name + "\" not found"));
    return respond(c, 200, *it->second.json);
  }
  if (r.method == "DELETE" && !name.empty()) {
    std::string prop = "Background";
    if (!r.body.empty()) {
      // DeleteOptions: only propagationPolicy matters here; a plain scan for its string
      // value (an enum, never escaped) instead of a DOM parse per DELETE
      size_t k = r.body.find("\"propagationPolicy\"");
      size_t c = k == std::string_view::npos ? k : r.body.find(':', k + 19);
      size_t q1 = c == std::string_view::npos ? c : r.body.find('"', c + 1);
      size_t q2 = q1 == std::string_view::npos ? q1 : r.body.find('"', q1 + 1);
      if (q2 != std::string_view::npos && q2 > q1 + 1) prop = std::string(r.body.substr(q1 + 1, q2 - q1 - 1));
      else if (k == std::string_view::npos) kjson::parse(r.body);  // still reject malformed bodies
    }
    std::string qp = q(r, "propagationPolicy");
    if (!qp.empty()) prop = qp;
    if (!remove(kind, ns, name, prop))
      return respond(c, 404, status_body(404, "NotFound", lower + "s" + (kind == K_JOB ? ".batch" : "") + " \"" + name + "\" not found"));
    std::string s = "{\"kind\":\"Status\",\"apiVersion\":\"v1\",\"status\":\"Success\",\"details\":{\"name\":";
    kjson::escape(s, name);
    s += ",\"kind\":\"" + lower + "s\"}}";
    return respond(c, 200, s);
  }
  if (r.method == "POST" && name.empty()) {
    Value doc = kjson::parse(r.body);
    doc.at("kind") = Value::str(kn);
    doc.at("metadata").at("namespace") = Value::str(ns);
    std::string out;
    if (!create(kind, doc, &out))
      return respond(c, 409, status_body(409, "AlreadyExists", lower + "s \"" + std::string(doc.path({"metadata", "name"})) + "\" already exists"));
    return respond(c, 201, out);
  }
  if (r.method == "PUT" && !name.empty()) {
    Value doc = kjson::parse(r.body);
    doc.at("kind") = Value::str(kn);
    Value& md = doc.at("metadata");
    md.at("namespace") = Value::str(ns);
    md.at("name") = Value::str(name);
    std::string out;
    int rc = update(kind, doc, true, &out);
    if (rc == 1) return respond(c, 404, status_body(404, "NotFound", "not found"));
    if (rc == 2) return respond(c, 409, status_body(409, "Conflict", "the object has been modified; please apply your changes to the latest version"));
    return respond(c, 200, out);
  }
  if (r.method == "PATCH" && !name.empty()) {
    auto it = g_store[kind].objs.find(okey(ns, name));
    if (it == g_store[kind].objs.end()) return respond(c, 404, status_body(404, "NotFound", "not found"));
    Value cur = kjson::parse(*it->second.json);
    kjson::merge_patch(cur, kjson::parse(r.body));
    cur.at("metadata").erase("resourceVersion");
    std::string out;
    update(kind, cur, false, &out);
    return respond(c, 200, out);
  }
  respond(c, 405, status_body(405, "MethodNotAllowed", "method not allowed"));
}

// parses as many complete requests as the buffer holds; false = protocol error (close)
bool on_input(Conn& c) {
  // requests are consumed by advancing `at`; the buffer is compacted once at the end
  // (erasing each request from the front made a pipelined burst O(n^2) in bytes moved)
  size_t at = 0;
  struct Compact {
    std::string& in;
    size_t& at;
    ~Compact() {
      if (at) in.erase(0, at);
    }
  } compact{c.in, at};
  while (!c.watch) {
    size_t he = c.in.find("\r\n\r\n", at);
    if (he == std::string::npos) return c.in.size() - at < (1u << 20);
    Request r;
    std::string_view head(c.in.data() + at, he - at);
    size_t le = head.find("\r\n");
    std::string_view rl = head.substr(0, le);
    size_t s1 = rl.find(' '), s2 = rl.rfind(' ');
    if (s1 == std::string_view::npos || s2 <= s1) return false;
    r.method = std::string(rl.substr(0, s1));
    std::string_view target = rl.substr(s1 + 1, s2 - s1 - 1);
    std::string_view version = rl.substr(s2 + 1);
    size_t qm = target.find('?');
    r.path = pct_decode(target.substr(0, qm));
    if (qm != std::string_view::npos) {
      std::string_view qs = target.substr(qm + 1);
      size_t p = 0;
      while (p <= qs.size()) {
        size_t amp = qs.find('&', p);
        if (amp == std::string_view::npos) amp = qs.size();
        std::string_view kv = qs.substr(p, amp - p);
        size_t eq = kv.find('=');
        if (!kv.empty()) r.query[pct_decode(kv.substr(0, eq))] = eq == std::string_view::npos ? "" : pct_decode(kv.substr(eq + 1));
        p = amp + 1;
      }
    }
    size_t clen = 0;
    bool chunked = false;
    r.close = version == "HTTP/1.0";
    size_t pos = le == std::string_view::npos ? head.size() : le + 2;
    while (pos < head.size()) {
      size_t e = head.find("\r\n", pos);
      if (e == std::string_view::npos) e = head.size();
      std::string_view line = head.substr(pos, e - pos);
      pos = e + 2;
      size_t colon = line.find(':');
      if (colon == std::string_view::npos) continue;
      // header names / connection tokens compared case-insensitively in place (no copies)
      std::string_view name = line.substr(0, colon);
      std::string_view val = trim_view(line.substr(colon + 1));
      if (iequals(name, "content-length")) clen = static_cast<size_t>(strtoull(std::string(val).c_str(), nullptr, 10));
      else if (iequals(name, "authorization")) r.auth = std::string(val);
      else if (iequals(name, "transfer-encoding") && val.find("chunked") != std::string_view::npos) chunked = true;
      else if (iequals(name, "connection")) {
        if (iequals(val, "close")) r.close = true;
        else if (iequals(val, "keep-alive")) r.close = false;
      }
    }
    if (chunked) {
      c.close_after = true;
      respond(c, 411, status_body(411, "LengthRequired", "chunked request bodies are not supported"));
      at = c.in.size();
      return true;
    }
    if (c.in.size() < he + 4 + clen) {  // body incomplete: grow once, not by doubling per recv
      if (c.in.capacity() < he + 4 + clen) c.in.reserve(he + 4 + clen);
      return true;
    }
    r.body = std::string_view(c.in.data() + he + 4, clen);  // no copy: c.in is compacted after the loop
    at = he + 4 + clen;
    int64_t th = mono_ns();
    try {
      handle(c, r);
    } catch (const std::exception& e) {
      respond(c, 400, status_body(400, "BadRequest", e.what()));
    }
    g_stats.request_ns += mono_ns() - th;  // includes bulk applies (apply_ns is their share)
    if (c.close_after) return true;
  }
  return true;
}

std::atomic<int> g_stop{0};  // read by the apply threads too (lock-free: signal-safe)
void on_signal(int) { g_stop.store(1); }

// ------------------------------------------------------------ apply port
// The benchmark's traffic generator posts its bulk applies to a port of their own, served
// by their own threads: reading a multi-megabyte body and preparing its lines happen beside
// the event loop, which keeps serving the supervisor's requests and watches; only the commit
// takes the store lock.  The loop port still accepts /sim/apply (on the loop).
int g_wake_fd = -1;  // eventfd: an apply committed watch lines the loop must send

// --async-gc: deletes the queued pods of Background-deleted Jobs, up to 256 per hold of the
// store lock (the loop and the apply port get it between batches), then wakes the loop to
// send the DELETED lines
void gc_thread() {
  std::unique_lock<std::mutex> lk(g_store_mu);
  std::vector<Obj> dead;
  while (!g_stop) {
    size_t graves;
    {
      std::lock_guard<std::mutex> glk(g_graves_mu);
      graves = g_graves.size();
    }
    if (g_gc.empty() && graves < 1024) {
      g_gc_cv.wait_for(lk, std::chrono::milliseconds(100));
      std::lock_guard<std::mutex> glk(g_graves_mu);
      if (g_gc.empty() && g_graves.empty()) continue;
    }
    int64_t t0 = mono_ns();
    bool removed = !g_gc.empty();
    for (int n = 0; n < 256 && !g_gc.empty(); ++n) {
      std::pair<std::string, std::string> p = std::move(g_gc.front());
      g_gc.pop_front();
      if (remove(K_POD, p.first, p.second, "Background")) ++g_stats.gc_pods;
    }
    {
      std::lock_guard<std::mutex> glk(g_graves_mu);
      dead.swap(g_graves);
    }
    int64_t t1 = mono_ns();
    g_stats.store_ns += t1 - t0;
    lk.unlock();
    if (removed) {
      uint64_t one = 1;
      if (write(g_wake_fd, &one, sizeof one) < 0) { /* the loop wakes within 100 ms anyway */ }
    }
    dead.clear();  // the frees, outside the store lock
    g_stats.gc_ns += mono_ns() - t0;
    lk.lock();
  }
}

void apply_conn(int fd) {
  const int conn_id = ++g_apply_conn_seq;
  std::string in;
  std::vector<char> buf(1 << 16);
  while (!g_stop) {
    size_t he;
    while ((he = in.find("\r\n\r\n")) == std::string::npos) {
      ssize_t r = recv(fd, buf.data(), buf.size(), 0);
      if (r <= 0) {
        close(fd);
        return;
      }
      in.append(buf.data(), static_cast<size_t>(r));
    }
    int64_t t0 = mono_ns();
    std::string_view head(in.data(), he);
    size_t le = head.find("\r\n");
    std::string_view rl = head.substr(0, le);
    size_t s1 = rl.find(' '), s2 = rl.rfind(' ');
    // copies: reading the rest of the body may reallocate `in`
    std::string method(rl.substr(0, s1));
    std::string target(s1 == std::string_view::npos || s2 <= s1 ? std::string_view() : rl.substr(s1 + 1, s2 - s1 - 1));
    size_t clen = 0;
    size_t pos = le == std::string_view::npos ? head.size() : le + 2;
    while (pos < head.size()) {
      size_t e = head.find("\r\n", pos);
      if (e == std::string_view::npos) e = head.size();
      std::string_view line = head.substr(pos, e - pos);
      pos = e + 2;
      size_t colon = line.find(':');
      if (colon != std::string_view::npos && iequals(line.substr(0, colon), "content-length"))
        clen = static_cast<size_t>(strtoull(std::string(trim_view(line.substr(colon + 1))).c_str(), nullptr, 10));
    }
    if (in.capacity() < he + 4 + clen) in.reserve(he + 4 + clen);
    while (in.size() < he + 4 + clen) {
      ssize_t r = recv(fd, buf.data(), buf.size(), 0);
      if (r <= 0) {
        close(fd);
        return;
      }
      in.append(buf.data(), static_cast<size_t>(r));
    }
    std::string_view body(in.data() + he + 4, clen);
    int code = 200;
    std::string out;
    if (method == "POST" && target.substr(0, target.find('?')) == "/sim/apply" &&
        target.find("expire=1") == std::string::npos) {
      try {
        out = apply_body(body, false, false);
      } catch (const std::exception& e) {
        code = 400;
        out = status_body(400, "BadRequest", e.what());
      }
      uint64_t one = 1;
      if (write(g_wake_fd, &one, sizeof one) < 0) { /* the loop wakes within 100 ms anyway */ }
    } else {
      code = 404;
      out = status_body(404, "NotFound", "the apply port serves POST /sim/apply (without expire) only");
    }
    std::string resp = "HTTP/1.1 " + std::to_string(code) + " " + status_text(code) +
                       "\r\nContent-Type: application/json\r\nContent-Length: " + std::to_string(out.size()) + "\r\n\r\n" + out;
    size_t off = 0;
    while (off < resp.size()) {
      ssize_t w = send(fd, resp.data() + off, resp.size() - off, MSG_NOSIGNAL);
      if (w <= 0) {
        close(fd);
        return;
      }
      off += static_cast<size_t>(w);
    }
    in.erase(0, he + 4 + clen);
    int64_t dt = mono_ns() - t0;
    g_stats.apply_thread_ns += dt;
    {
      std::lock_guard<std::mutex> lk(g_apply_conn_mu);
      g_apply_conn_ns[conn_id] += dt;
    }
  }
  close(fd);
}

void apply_server(int afd) {
  int one = 1;
  while (!g_stop) {
    int cfd = accept(afd, nullptr, nullptr);
    if (cfd < 0) {
      if (errno == EINTR) continue;
      return;
    }
    setsockopt(cfd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    std::thread(apply_conn, cfd).detach();
  }
}

void usage() {
  fprintf(stderr,
          "nexus-kubesim [--host H] [--port P] [--ready-file F] [--history N] [--bookmark-ms MS] [--token T]\n"
          "              [--flush-threads N] [--apply-threads N] [--async-gc] [--api-latency-us US] [--write-qps Q] [--write-burst B]\n"
          "              [--throttle-deletes N] [--retry-after S] [--log-root DIR]\n");
}

}  // namespace

int main(int argc, char** argv) {
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) {
        usage();
        exit(2);
      }
      return argv[++i];
    };
    if (a == "--host") g_opt.host = next();
    else if (a == "--port") g_opt.port = atoi(next().c_str());
    else if (a == "--ready-file") g_opt.ready_file = next();
    else if (a == "--history") g_opt.history = static_cast<size_t>(atol(next().c_str()));
    else if (a == "--prefault-mb") g_opt.prefault_mb = static_cast<size_t>(atol(next().c_str()));
    else if (a == "--bookmark-ms") g_opt.bookmark_ms = atol(next().c_str());
    else if (a == "--token") g_opt.token = next();
    else if (a == "--flush-threads") g_opt.flush_threads = std::max(1, atoi(next().c_str()));
    else if (a == "--apply-threads") g_opt.apply_threads = std::max(1, std::min(16, atoi(next().c_str())));
    else if (a == "--async-gc") g_opt.async_gc = true;
    else if (a == "--api-latency-us") g_opt.api_latency_us = std::max(0L, atol(next().c_str()));
    else if (a == "--write-qps") g_opt.write_qps = atof(next().c_str());
    else if (a == "--write-burst") g_opt.write_burst = atoi(next().c_str());
    else if (a == "--throttle-deletes") g_opt.throttle_deletes = atol(next().c_str());
    else if (a == "--retry-after") g_opt.retry_after_s = std::max(0, atoi(next().c_str()));
    else if (a == "--log-root") g_opt.log_root = next();
    else {
      usage();
      return 2;
    }
  }
  signal(SIGPIPE, SIG_IGN);
  // Keep freed memory in the heap: bulk applies allocate and free megabytes per step, and
  // glibc's default trimming hands it back to the kernel only to fault it in again
  // (brk + page faults were a quarter of the simulator's CPU time).
  mallopt(M_TRIM_THRESHOLD, 1 << 30);
  mallopt(M_TOP_PAD, 64 << 20);
  mallopt(M_MMAP_THRESHOLD, 1 << 30);
  // No fastbins: every object line / JSON text is a >1 KiB "large" request, and glibc
  // consolidates all fastbin chunks before serving one — with the many small key / name
  // strings freed in between, that consolidation was most of malloc's time.  Small
  // chunks still go through the per-thread tcache.
  mallopt(M_MXFAST, 0);
  if (g_opt.prefault_mb > 0) {
    // Grow and touch the heap once: the watch history and the live objects fill hundreds of
    // MB in the first steps of a benchmark, and every brk extension and first-touch page
    // fault of that growth landed on the event loop (a quarter of its time in a 20-step run).
    // Freed at once, the pages stay in the heap (M_TRIM_THRESHOLD above) for the run.
    size_t n = g_opt.prefault_mb << 20;
    if (char* p = static_cast<char*>(malloc(n))) {
      for (size_t i = 0; i < n; i += 4096) p[i] = 1;
      free(p);
    }
  }
  // Sparse buckets sized for a benchmark's namespace (10k runs, their pods and tens of
  // thousands of live Events): short chains, and no rehash of the whole table mid-run
  for (auto& ks : g_store) {
    ks.objs.max_load_factor(0.5f);
    ks.objs.reserve(1 << 16);
  }
  g_pods_by_job.max_load_factor(0.5f);
  g_pods_by_job.reserve(1 << 15);
  prof::start();
  signal(SIGTERM, on_signal);
  signal(SIGINT, on_signal);

  int lfd = socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons(static_cast<uint16_t>(g_opt.port));
  if (inet_pton(AF_INET, g_opt.host.c_str(), &addr.sin_addr) != 1) {
    fprintf(stderr, "bad --host %s\n", g_opt.host.c_str());
    return 2;
  }
  if (bind(lfd, reinterpret_cast<sockaddr*>(&addr), sizeof addr) < 0 || listen(lfd, 1024) < 0) {
    perror("bind/listen");
    return 1;
  }
  socklen_t alen = sizeof addr;
  getsockname(lfd, reinterpret_cast<sockaddr*>(&addr), &alen);
  int port = ntohs(addr.sin_port);
  set_nonblock(lfd);
  g_ep = epoll_create1(0);
  epoll_event lev{};
  lev.events = EPOLLIN;
  lev.data.fd = lfd;
  epoll_ctl(g_ep, EPOLL_CTL_ADD, lfd, &lev);

  // the apply port (bulk applies on their own threads) and the loop's wake-up eventfd
  int afd = socket(AF_INET, SOCK_STREAM, 0);
  setsockopt(afd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in aaddr = addr;
  aaddr.sin_port = 0;
  if (bind(afd, reinterpret_cast<sockaddr*>(&aaddr), sizeof aaddr) < 0 || listen(afd, 64) < 0) {
    perror("bind/listen (apply port)");
    return 1;
  }
  socklen_t aalen = sizeof aaddr;
  getsockname(afd, reinterpret_cast<sockaddr*>(&aaddr), &aalen);
  int aport = ntohs(aaddr.sin_port);
  g_wake_fd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  epoll_event wev{};
  wev.events = EPOLLIN;
  wev.data.fd = g_wake_fd;
  epoll_ctl(g_ep, EPOLL_CTL_ADD, g_wake_fd, &wev);

  char info[256];
  snprintf(info, sizeof info, "{\"port\":%d,\"pid\":%d,\"url\":\"http://%s:%d\",\"apply_url\":\"http://%s:%d\"}\n", port,
           getpid(), g_opt.host.c_str(), port, g_opt.host.c_str(), aport);
  if (!g_opt.ready_file.empty()) {
    std::string tmp = g_opt.ready_file + ".tmp";
    FILE* f = fopen(tmp.c_str(), "w");
    if (!f) {
      perror("ready-file");
      return 1;
    }
    fputs(info, f);
    fclose(f);
    rename(tmp.c_str(), g_opt.ready_file.c_str());
  }
  fputs(info, stdout);
  fflush(stdout);

  g_flush_pool.start(g_opt.flush_threads);
  g_apply_pool.start(g_opt.apply_threads);
  std::thread(apply_server, afd).detach();
  std::thread gc;
  if (g_opt.async_gc) gc = std::thread(gc_thread);
  std::vector<epoll_event> evs(512);
  int64_t last_tick = mono_ms();
  char buf[1 << 16];
  while (!g_stop) {
    int wait_ms = 100;
    {
      StoreLock lk;
      if (!g_delayed.empty()) {
        int d = release_delayed();
        if (d >= 0) wait_ms = std::min(wait_ms, d);
      }
      if (!g_dirty.empty()) wait_ms = 0;
    }
    int n = epoll_wait(g_ep, evs.data(), static_cast<int>(evs.size()), wait_ms);
    int64_t t_loop = mono_ns();
    ++g_stats.loops;
    if (n < 0 && errno != EINTR) {
      perror("epoll_wait");
      break;
    }
    for (int i = 0; i < n; ++i) {
      int fd = evs[i].data.fd;
      if (fd == g_wake_fd) {
        uint64_t v;
        if (read(g_wake_fd, &v, sizeof v) < 0) { /* drained */ }
        continue;
      }
      if (fd == lfd) {
        while (true) {
          int cfd = accept(lfd, nullptr, nullptr);
          if (cfd < 0) break;
          set_nonblock(cfd);
          setsockopt(cfd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
          auto c = std::make_unique<Conn>();
          c->fd = cfd;
          epoll_event ev{};
          ev.events = EPOLLIN | EPOLLRDHUP;
          ev.data.fd = cfd;
          epoll_ctl(g_ep, EPOLL_CTL_ADD, cfd, &ev);
          StoreLock lk;
          g_conns[cfd] = std::move(c);
        }
        continue;
      }
      Conn* cp;
      {
        StoreLock lk;
        auto it = g_conns.find(fd);
        if (it == g_conns.end()) continue;
        cp = it->second.get();
      }
      Conn& c = *cp;  // only the loop erases connections
      bool dead = false;
      if (evs[i].events & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR)) {
        int64_t tr = mono_ns();
        while (true) {
          ssize_t r = recv(fd, buf, sizeof buf, 0);
          if (r > 0) {
            c.in.append(buf, static_cast<size_t>(r));
            // a short read drained the socket: skip the EAGAIN probe (level-triggered
            // epoll reports anything that arrives later)
            if (static_cast<size_t>(r) < sizeof buf) break;
            continue;
          }
          if (r == 0) dead = true;
          else if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) dead = true;
          break;
        }
        g_stats.recv_ns += mono_ns() - tr;
        if (!dead) {
          StoreLock lk;
          if (!on_input(c)) dead = true;
        }
      }
      StoreLock lk;
      if (dead) {
        close_conn(fd);
        continue;
      }
      if (evs[i].events & EPOLLOUT) g_dirty.insert(&c);
    }
    StoreLock tick_lk;
    if (!g_delayed.empty()) release_delayed();
    int64_t now = mono_ms();
    if (now - last_tick >= 50) {
      last_tick = now;
      std::vector<Conn*> ended;
      for (auto& kv : g_conns) {
        Watch* w = kv.second->watch;
        if (!w) continue;
        if (now >= w->deadline_ms) {
          ended.push_back(kv.second.get());
        } else if (w->bookmarks && w->idle() && now - w->last_ms >= g_opt.bookmark_ms) {
          w->pending = std::string("{\"type\":\"BOOKMARK\",\"object\":{\"kind\":\"") + KINDS[w->kind].kind +
                       "\",\"apiVersion\":\"" + KINDS[w->kind].api_version + "\",\"metadata\":{\"resourceVersion\":\"" +
                       std::to_string(g_rv) + "\"}}}\n";
          g_dirty.insert(kv.second.get());
        }
      }
      for (Conn* c : ended) end_watch(*c, true);
    }
    std::vector<Conn*> dirty(g_dirty.begin(), g_dirty.end());
    g_dirty.clear();
    tick_lk.lk.unlock();
    g_stats.store_ns += mono_ns() - tick_lk.t0;
    tick_lk.t0 = mono_ns();  // (the destructor adds the re-locked span below)
    if (!dirty.empty()) {
      int64_t tf = mono_ns();
      std::vector<uint8_t> ok(dirty.size(), 1);
      g_flush_pool.run(dirty, ok);
      tick_lk.lk.lock();
      tick_lk.t0 = mono_ns();
      for (size_t i = 0; i < dirty.size(); ++i)
        if (!ok[i]) close_conn(dirty[i]->fd);
      g_stats.flush_ns += mono_ns() - tf;
    } else {
      tick_lk.lk.lock();
      tick_lk.t0 = mono_ns();
    }
    g_stats.busy_ns += mono_ns() - t_loop;
  }
  g_flush_pool.stop();
  g_apply_pool.stop();
  if (gc.joinable()) {
    g_gc_cv.notify_all();
    gc.join();
  }
  for (auto& kv : g_conns) close(kv.first);
  close(lfd);
  prof::dump();
  return 0;
}
