// _kube_native — projected JSON decoding of Kubernetes watch streams and LIST bodies.
//
// The reference relies on client-go reflectors that decode every Event/Pod/Job change
// into full Go structs (/root/reference/services/supervisor.go:73-75; SURVEY §3B: "the
// hot part is decoding every Event/Pod/Job change in the namespace").  Real pods carry
// kilobytes the supervisor never reads (managedFields, volumes, affinity, probes...).
// This decoder walks the JSON once and materialises Python objects only for the paths
// in a projection schema (the analog of an informer TransformFunc, applied *during*
// parsing): everything else is skipped by a byte scanner without allocating.
//
// Projection schema (compiled once from Python):
//   True                          keep the whole value
//   {"key": sub, ...}             object: keep only these keys (projected)
//   ["list", sub]                 array: project every element with `sub`
//   ["prefix", "p1", "p2", ...]   object: keep entries whose key starts with a prefix
//   ["map", sub]                  object: keep all keys, project every value with `sub`
//   {"$deleted": sub, ...}        (watch envelope) project "object" with `sub` instead when
//                                 "type" is "DELETED" and precedes it: a deletion needs only
//                                 the object's identity, the informer already holds the rest
// A non-object value where an object projection was expected is kept whole (so
// Status objects in ERROR events survive any kind's schema).
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <time.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <deque>
#include <memory>
#include <memory_resource>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

// CPython static type objects are declared with only their header and filled in at
// module init; the remaining slots are zero by static initialisation.
#pragma GCC diagnostic ignored "-Wmissing-field-initializers"

namespace {

struct Proj {
  enum Kind { KEEP, OBJECT, LIST, PREFIX, MAP, KV } kind = KEEP;
  std::vector<std::pair<std::string, std::unique_ptr<Proj>>> fields;  // OBJECT (small: linear scan)
  std::unique_ptr<Proj> elem;                                         // LIST / MAP
  std::unique_ptr<Proj> on_deleted;                                   // OBJECT: "object" of a DELETED envelope
  std::vector<std::string> prefixes;                                  // PREFIX, KV
  // KV: a list of {key_field: k, value_field: v} objects becomes one {k: v} dict, keeping
  // only keys in `keep` or starting with one of `prefixes` (both empty: every key); the
  // first definition of a key wins and entries without a string value are dropped
  std::string key_field, value_field;
  std::vector<std::string> keep;

  bool kv_wanted(std::string_view k) const {
    if (keep.empty() && prefixes.empty()) return true;
    for (auto& w : keep)
      if (w == k) return true;
    for (auto& pre : prefixes)
      if (k.substr(0, pre.size()) == pre) return true;
    return false;
  }

  const Proj* field(std::string_view k) const {
    for (auto& f : fields)
      if (f.first == k) return f.second.get();
    return nullptr;
  }
};

std::unique_ptr<Proj> compile(PyObject* spec) {
  auto p = std::make_unique<Proj>();
  if (spec == Py_True) return p;
  if (PyDict_Check(spec)) {
    p->kind = Proj::OBJECT;
    PyObject *k, *v;
    Py_ssize_t pos = 0;
    while (PyDict_Next(spec, &pos, &k, &v)) {
      Py_ssize_t n;
      const char* s = PyUnicode_AsUTF8AndSize(k, &n);
      if (!s) return nullptr;
      auto sub = compile(v);
      if (!sub) return nullptr;
      if (std::string_view(s, static_cast<size_t>(n)) == "$deleted") {
        p->on_deleted = std::move(sub);
        continue;
      }
      p->fields.emplace_back(std::string(s, static_cast<size_t>(n)), std::move(sub));
    }
    return p;
  }
  if ((PyList_Check(spec) || PyTuple_Check(spec)) && PySequence_Size(spec) >= 1) {
    PyObject* head = PySequence_GetItem(spec, 0);
    const char* h = head && PyUnicode_Check(head) ? PyUnicode_AsUTF8(head) : nullptr;
    Py_XDECREF(head);
    if (h && (!strcmp(h, "list") || !strcmp(h, "map")) && PySequence_Size(spec) == 2) {
      p->kind = !strcmp(h, "list") ? Proj::LIST : Proj::MAP;
      PyObject* sub = PySequence_GetItem(spec, 1);
      p->elem = compile(sub);
      Py_XDECREF(sub);
      return p->elem ? std::move(p) : nullptr;
    }
    if (h && !strcmp(h, "kv") && PySequence_Size(spec) == 5) {
      p->kind = Proj::KV;
      auto text = [&](Py_ssize_t i, std::string& out) {
        PyObject* o = PySequence_GetItem(spec, i);
        const char* c = o && PyUnicode_Check(o) ? PyUnicode_AsUTF8(o) : nullptr;
        if (c) out = c;
        Py_XDECREF(o);
        return c != nullptr;
      };
      auto texts = [&](Py_ssize_t i, std::vector<std::string>& out) {
        PyObject* o = PySequence_GetItem(spec, i);
        bool ok = o && (PyList_Check(o) || PyTuple_Check(o));
        for (Py_ssize_t k = 0; ok && k < PySequence_Size(o); ++k) {
          PyObject* e = PySequence_GetItem(o, k);
          const char* c = e && PyUnicode_Check(e) ? PyUnicode_AsUTF8(e) : nullptr;
          if (c) out.emplace_back(c);
          else ok = false;
          Py_XDECREF(e);
        }
        Py_XDECREF(o);
        return ok;
      };
      if (text(1, p->key_field) && text(2, p->value_field) && texts(3, p->keep) && texts(4, p->prefixes)) return p;
      PyErr_Clear();
      PyErr_SetString(PyExc_ValueError, "kv projection: [\"kv\", key_field, value_field, [keep...], [prefix...]]");
      return nullptr;
    }
    if (h && !strcmp(h, "prefix")) {
      p->kind = Proj::PREFIX;
      for (Py_ssize_t i = 1; i < PySequence_Size(spec); ++i) {
        PyObject* s = PySequence_GetItem(spec, i);
        const char* c = s && PyUnicode_Check(s) ? PyUnicode_AsUTF8(s) : nullptr;
        if (c) p->prefixes.emplace_back(c);
        Py_XDECREF(s);
      }
      return p;
    }
  }
  PyErr_SetString(PyExc_ValueError, "bad projection spec");
  return nullptr;
}

// str from UTF-8 bytes.  Kubernetes objects are almost entirely ASCII: build those directly
// (one allocation + memcpy) instead of going through the generic decoder with an error
// handler looked up by name on every call.
PyObject* make_str(const char* p, size_t n) {
  const unsigned char* u = reinterpret_cast<const unsigned char*>(p);
  unsigned char any = 0;
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    memcpy(&w, u + i, 8);
    if (w & 0x8080808080808080ULL) {
      any = 0x80;
      break;
    }
  }
  for (; !any && i < n; ++i) any |= u[i];
  if (!(any & 0x80)) {
    PyObject* o = PyUnicode_New(static_cast<Py_ssize_t>(n), 127);
    if (o) memcpy(PyUnicode_DATA(o), p, n);
    return o;
  }
  return PyUnicode_DecodeUTF8(p, static_cast<Py_ssize_t>(n), "replace");
}

// Interned Python strings (object keys and short repeated values), looked up by bytes
// without allocating (open addressing).  ONE cache per process, shared by every decoder:
// the three informers' decoders see the same keys, and a shard worker touches the cache
// between long stretches of other work, so it must stay small enough to be cache-resident —
// a slot is (hash, object) and the key bytes are compared against the str's own buffer
// (8192 slots of hash + std::string + object per decoder were ~1.2 MB per worker).
class KeyCache {
 public:
  KeyCache() : slots_(kCap) {}
  // New reference to the Python str for `k`.
  PyObject* get(std::string_view k) {
    uint64_t h = 1469598103934665603ULL;
    for (unsigned char c : k) h = (h ^ c) * 1099511628211ULL;
    size_t i = h & (kCap - 1);
    for (size_t probe = 0; probe < kProbe; ++probe, i = (i + 1) & (kCap - 1)) {
      Slot& sl = slots_[i];
      if (!sl.obj) {
        PyObject* o = make_str(k.data(), k.size());
        if (!o) return nullptr;
        if (used_ < kCap * 3 / 4) {
          sl.hash = h;
          sl.obj = o;
          Py_INCREF(o);
          ++used_;
        }
        return o;
      }
      if (sl.hash == h && same(sl.obj, k)) {
        Py_INCREF(sl.obj);
        return sl.obj;
      }
    }
    return make_str(k.data(), k.size());
  }

 private:
  static bool same(PyObject* o, std::string_view k) {
    if (PyUnicode_IS_COMPACT_ASCII(o))
      return static_cast<size_t>(PyUnicode_GET_LENGTH(o)) == k.size() && memcmp(PyUnicode_DATA(o), k.data(), k.size()) == 0;
    Py_ssize_t n;
    const char* u = PyUnicode_AsUTF8AndSize(o, &n);
    if (!u) {
      PyErr_Clear();
      return false;
    }
    return static_cast<size_t>(n) == k.size() && memcmp(u, k.data(), k.size()) == 0;
  }
  static constexpr size_t kCap = 4096;  // 64 KB of slots
  static constexpr size_t kProbe = 8;
  struct Slot {
    uint64_t hash = 0;
    PyObject* obj = nullptr;
  };
  std::vector<Slot> slots_;
  size_t used_ = 0;
};

KeyCache* shared_keys() {
  static KeyCache* k = new KeyCache();  // process lifetime (interned strs stay alive)
  return k;
}

// Short values worth interning: they repeat across objects ("Pending", "True", label
// values, env values).  Digit runs (resourceVersions, counts) and RFC 3339 timestamps are
// unique per object: interning them would fill the shared cache with one-off entries.
inline bool internable(const char* p, size_t n) {
  if (n > 24) return false;
  bool digits = n > 0;
  for (size_t i = 0; i < n && digits; ++i) digits = p[i] >= '0' && p[i] <= '9';
  if (digits && n > 2) return false;
  if (n >= 20 && p[4] == '-' && p[10] == 'T') return false;
  return true;
}

struct ParseError {
  const char* msg;
  size_t at;
};

class Parser {
 public:
  Parser(const char* s, size_t n, KeyCache* keys) : s_(s), n_(n), keys_(keys) {}

  size_t pos() const { return i_; }
  void set_pos(size_t p) { i_ = p; }

  void ws() {
    while (i_ < n_ && (s_[i_] == ' ' || s_[i_] == '\t' || s_[i_] == '\r' || s_[i_] == '\n')) ++i_;
  }

  // Parse one value with projection `p` (nullptr = keep whole).  New reference.
  PyObject* value(const Proj* p) {
    ws();
    if (i_ >= n_) throw ParseError{"unexpected end", i_};
    char c = s_[i_];
    if (c == '{') {
      if (p && p->kind == Proj::OBJECT) return object_proj(p);
      if (p && p->kind == Proj::PREFIX) return object_prefix(p);
      if (p && p->kind == Proj::MAP) return object_map(p->elem.get());
      return object_full();
    }
    if (c == '[') {
      if (p && p->kind == Proj::LIST) return array(p->elem.get());
      if (p && p->kind == Proj::KV) return kv_array(p);
      return array(nullptr);
    }
    if (c == '"') return string_obj();
    if (c == 't') return lit("true", Py_True);
    if (c == 'f') return lit("false", Py_False);
    if (c == 'n') return lit("null", Py_None);
    return number();
  }

  void skip() {
    ws();
    if (i_ >= n_) throw ParseError{"unexpected end", i_};
    char c = s_[i_];
    if (c == '"') {
      skip_string();
      return;
    }
    if (c == '{' || c == '[') {
      int depth = 0;
      while (i_ < n_) {
        char d = s_[i_];
        if (d == '"') {
          skip_string();
          continue;
        }
        if (d == '{' || d == '[') ++depth;
        else if (d == '}' || d == ']') {
          if (--depth == 0) {
            ++i_;
            return;
          }
        }
        ++i_;
      }
      throw ParseError{"unterminated container", i_};
    }
    while (i_ < n_ && s_[i_] != ',' && s_[i_] != '}' && s_[i_] != ']' && s_[i_] != ' ' && s_[i_] != '\n') ++i_;
  }

 private:
  PyObject* lit(const char* w, PyObject* o) {
    size_t k = strlen(w);
    if (i_ + k > n_ || memcmp(s_ + i_, w, k) != 0) throw ParseError{"bad literal", i_};
    i_ += k;
    Py_INCREF(o);
    return o;
  }

  PyObject* number() {
    size_t st = i_;
    bool flt = false;
    if (i_ < n_ && (s_[i_] == '-' || s_[i_] == '+')) ++i_;
    while (i_ < n_) {
      char c = s_[i_];
      if (c >= '0' && c <= '9') ++i_;
      else if (c == '.' || c == 'e' || c == 'E' || c == '+' || c == '-') {
        flt = true;
        ++i_;
      } else
        break;
    }
    if (i_ == st) throw ParseError{"bad value", i_};
    size_t len = i_ - st;
    if (!flt && len < 18) {  // fits in int64: no temporary string
      const char* q = s_ + st;
      bool neg = *q == '-';
      if (*q == '-' || *q == '+') ++q;
      long long v = 0;
      for (; q < s_ + i_; ++q) v = v * 10 + (*q - '0');
      return PyLong_FromLongLong(neg ? -v : v);
    }
    std::string tok(s_ + st, len);
    if (!flt) return PyLong_FromString(tok.c_str(), nullptr, 10);
    return PyFloat_FromDouble(std::stod(tok));
  }

  void skip_string() {
    ++i_;  // opening quote
    while (i_ < n_) {
      const char* q = static_cast<const char*>(memchr(s_ + i_, '"', n_ - i_));
      if (!q) break;
      size_t j = static_cast<size_t>(q - s_);
      size_t bs = 0;
      while (j > i_ + bs && s_[j - 1 - bs] == '\\') ++bs;
      i_ = j + 1;
      if (bs % 2 == 0) return;
    }
    throw ParseError{"unterminated string", i_};
  }

  // Raw string span [a, b) and whether it contains escapes.
  void string_span(size_t& a, size_t& b, bool& esc) {
    ++i_;
    a = i_;
    esc = false;
    while (i_ < n_) {
      char c = s_[i_];
      if (c == '"') {
        b = i_;
        ++i_;
        return;
      }
      if (c == '\\') {
        esc = true;
        i_ += 2;
        continue;
      }
      ++i_;
    }
    throw ParseError{"unterminated string", i_};
  }

  static void put_utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) out.push_back(static_cast<char>(cp));
    else if (cp < 0x800) {
      out.push_back(static_cast<char>(0xC0 | (cp >> 6)));
      out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      out.push_back(static_cast<char>(0xE0 | (cp >> 12)));
      out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else {
      out.push_back(static_cast<char>(0xF0 | (cp >> 18)));
      out.push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3F)));
      out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    }
  }

  uint32_t hex4(size_t at) {
    if (at + 4 > n_) throw ParseError{"bad \\u escape", at};
    uint32_t v = 0;
    for (size_t k = 0; k < 4; ++k) {
      char c = s_[at + k];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= static_cast<uint32_t>(c - '0');
      else if (c >= 'a' && c <= 'f') v |= static_cast<uint32_t>(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') v |= static_cast<uint32_t>(c - 'A' + 10);
      else throw ParseError{"bad \\u escape", at};
    }
    return v;
  }

  std::string unescape(size_t a, size_t b) {
    std::string out;
    out.reserve(b - a);
    for (size_t k = a; k < b; ++k) {
      char c = s_[k];
      if (c != '\\') {
        out.push_back(c);
        continue;
      }
      char e = s_[++k];
      switch (e) {
        case '"': out.push_back('"'); break;
        case '\\': out.push_back('\\'); break;
        case '/': out.push_back('/'); break;
        case 'b': out.push_back('\b'); break;
        case 'f': out.push_back('\f'); break;
        case 'n': out.push_back('\n'); break;
        case 'r': out.push_back('\r'); break;
        case 't': out.push_back('\t'); break;
        case 'u': {
          uint32_t cp = hex4(k + 1);
          k += 4;
          if (cp >= 0xD800 && cp <= 0xDBFF && k + 6 < b + 1 && s_[k + 1] == '\\' && s_[k + 2] == 'u') {
            uint32_t lo = hex4(k + 3);
            if (lo >= 0xDC00 && lo <= 0xDFFF) {
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
              k += 6;
            }
          }
          put_utf8(out, cp);
          break;
        }
        default: throw ParseError{"bad escape", k};
      }
    }
    return out;
  }

  PyObject* string_obj() {
    size_t a, b;
    bool esc;
    string_span(a, b, esc);
    if (!esc) {
      // short values repeat across objects ("Pending", "True", "Always", label values):
      // interned like keys, so they cost a lookup instead of an allocation
      if (internable(s_ + a, b - a)) return keys_->get(std::string_view(s_ + a, b - a));
      return make_str(s_ + a, b - a);
    }
    std::string u = unescape(a, b);
    return make_str(u.data(), u.size());
  }

  // Key text as a view into the buffer (or into scratch_ when it had escapes).
  std::string_view key_text() {
    ws();
    if (i_ >= n_ || s_[i_] != '"') throw ParseError{"expected key", i_};
    size_t a, b;
    bool esc;
    string_span(a, b, esc);
    std::string_view k;
    if (esc) {
      scratch_ = unescape(a, b);
      k = scratch_;
    } else {
      k = std::string_view(s_ + a, b - a);
    }
    ws();
    if (i_ >= n_ || s_[i_] != ':') throw ParseError{"expected ':'", i_};
    ++i_;
    return k;
  }

  PyObject* key_obj(std::string_view k) { return keys_->get(k); }

  template <typename F>
  PyObject* object_loop(F&& on_member) {
    ++i_;  // '{'
    PyObject* d = PyDict_New();
    if (!d) return nullptr;
    try {
      ws();
      if (i_ < n_ && s_[i_] == '}') {
        ++i_;
        return d;
      }
      while (true) {
        std::string_view k = key_text();
        std::string owned;
        if (k.data() == scratch_.data()) {  // nested keys reuse scratch_: keep our own copy
          owned.assign(k.data(), k.size());
          k = owned;
        }
        if (!on_member(d, k)) {
          Py_DECREF(d);
          return nullptr;
        }
        ws();
        if (i_ >= n_) throw ParseError{"unterminated object", i_};
        if (s_[i_] == ',') {
          ++i_;
          continue;
        }
        if (s_[i_] == '}') {
          ++i_;
          return d;
        }
        throw ParseError{"expected ',' or '}'", i_};
      }
    } catch (...) {
      Py_DECREF(d);
      throw;
    }
  }

  bool set_item(PyObject* d, std::string_view k, PyObject* v) {
    if (!v) return false;
    PyObject* ko = key_obj(k);
    if (!ko) {
      Py_DECREF(v);
      return false;
    }
    int rc = PyDict_SetItem(d, ko, v);
    Py_DECREF(ko);
    Py_DECREF(v);
    return rc == 0;
  }

  PyObject* object_full() {
    return object_loop([&](PyObject* d, std::string_view k) { return set_item(d, k, value(nullptr)); });
  }

  PyObject* object_proj(const Proj* p) {
    bool deleted = false;
    return object_loop([&](PyObject* d, std::string_view k) {
      const Proj* sub = p->field(k);
      if (!sub) {
        skip();
        return true;
      }
      if (p->on_deleted) {
        if (k == "type") {
          ws();
          deleted = n_ - i_ >= 9 && std::memcmp(s_ + i_, "\"DELETED\"", 9) == 0;
        } else if (deleted && k == "object") {
          sub = p->on_deleted.get();
        }
      }
      return set_item(d, k, value(sub->kind == Proj::KEEP ? nullptr : sub));
    });
  }

  PyObject* object_prefix(const Proj* p) {
    return object_loop([&](PyObject* d, std::string_view k) {
      for (auto& pre : p->prefixes)
        if (k.substr(0, pre.size()) == pre) return set_item(d, k, value(nullptr));
      skip();
      return true;
    });
  }

  PyObject* object_map(const Proj* elem) {
    return object_loop([&](PyObject* d, std::string_view k) {
      return set_item(d, k, value(elem && elem->kind != Proj::KEEP ? elem : nullptr));
    });
  }

  // Text of a string member value into `out` (unescaped); false when not a string.
  bool string_value(std::string& out) {
    ws();
    if (i_ >= n_ || s_[i_] != '"') {
      skip();
      return false;
    }
    size_t a, b;
    bool esc;
    string_span(a, b, esc);
    if (esc) out = unescape(a, b);
    else out.assign(s_ + a, b - a);
    return true;
  }

  PyObject* kv_array(const Proj* p) {
    ++i_;  // '['
    PyObject* d = PyDict_New();
    if (!d) return nullptr;
    try {
      std::string k, v, tmp;
      while (true) {
        ws();
        if (i_ >= n_) throw ParseError{"unterminated array", i_};
        if (s_[i_] == ']') {
          ++i_;
          return d;
        }
        if (s_[i_] != '{') {
          skip();
        } else {
          ++i_;
          bool has_k = false, has_v = false;
          ws();
          if (i_ < n_ && s_[i_] == '}') ++i_;
          else {
            while (true) {
              std::string_view name = key_text();
              if (name == p->key_field) has_k = string_value(k);
              else if (name == p->value_field) has_v = string_value(v);
              else skip();
              ws();
              if (i_ >= n_) throw ParseError{"unterminated object", i_};
              if (s_[i_] == ',') {
                ++i_;
                continue;
              }
              if (s_[i_] == '}') {
                ++i_;
                break;
              }
              throw ParseError{"expected ',' or '}'", i_};
            }
          }
          if (has_k && has_v && p->kv_wanted(k)) {
            PyObject* ko = keys_->get(k);
            if (!ko) {
              Py_DECREF(d);
              return nullptr;
            }
            int have = PyDict_Contains(d, ko);
            if (have == 0) {  // first definition wins (container env semantics)
              PyObject* vo = internable(v.data(), v.size()) ? keys_->get(v) : make_str(v.data(), v.size());
              int rc = vo ? PyDict_SetItem(d, ko, vo) : -1;
              Py_XDECREF(vo);
              if (rc != 0) have = -1;
            }
            Py_DECREF(ko);
            if (have < 0) {
              Py_DECREF(d);
              return nullptr;
            }
          }
        }
        ws();
        if (i_ < n_ && s_[i_] == ',') ++i_;
      }
    } catch (...) {
      Py_DECREF(d);
      throw;
    }
  }

  PyObject* array(const Proj* elem) {
    ++i_;  // '['
    PyObject* l = PyList_New(0);
    if (!l) return nullptr;
    try {
      ws();
      if (i_ < n_ && s_[i_] == ']') {
        ++i_;
        return l;
      }
      while (true) {
        PyObject* v = value(elem && elem->kind != Proj::KEEP ? elem : nullptr);
        if (!v || PyList_Append(l, v) != 0) {
          Py_XDECREF(v);
          Py_DECREF(l);
          return nullptr;
        }
        Py_DECREF(v);
        ws();
        if (i_ >= n_) throw ParseError{"unterminated array", i_};
        if (s_[i_] == ',') {
          ++i_;
          continue;
        }
        if (s_[i_] == ']') {
          ++i_;
          return l;
        }
        throw ParseError{"expected ',' or ']'", i_};
      }
    } catch (...) {
      Py_DECREF(l);
      throw;
    }
  }

  const char* s_;
  size_t n_;
  size_t i_ = 0;
  KeyCache* keys_;
  std::string scratch_;
};


// ------------------------------------------------------------------ shard routing
// A supervisor replica split into shard-worker processes (parallel/workers.py) has
// every worker read every watch stream, but each owns only the runs whose Job name
// hashes to it.  The router decides ownership from the raw line *before* the line
// is materialised: a scan that skips everything except the few key paths
// (object.metadata.name, the job-name label, involvedObject.kind/name) costs a
// fraction of building the projected dict, so a non-owned object costs the worker
// almost nothing.  Placement is zlib.crc32(job_name, seed) % count (same as the
// Python WorkerShard); pods map name → owner so Pod Events can be routed too.

uint32_t crc32_update(uint32_t start, const char* p, size_t n) {
  static uint32_t table[256];
  static bool init = false;
  if (!init) {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      table[i] = c;
    }
    init = true;
  }
  uint32_t c = start ^ 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) c = table[(c ^ static_cast<uint8_t>(p[i])) & 0xFF] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

double mono_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<double>(ts.tv_sec) + static_cast<double>(ts.tv_nsec) * 1e-9;
}

// Allocation-free path lookup in one JSON document.  Finds the string at a key path
// (each step an object key); returns false when absent, not a string, or escaped.
class Scan {
 public:
  Scan(const char* s, size_t n) : s_(s), n_(n) {}

  bool find(const char* const* path, size_t depth, std::string_view& out) {
    i_ = 0;
    try {
      return walk(path, depth, out);
    } catch (const ParseError&) {
      return false;
    }
  }

  // Everything routing needs from one watch line (or bare LIST item) in ONE pass:
  // type, metadata.name / resourceVersion / labels[job_label], involvedObject.kind / name.
  // Stops after the object's metadata (and involvedObject when wanted) — both come before
  // the large spec / status — so a line costs one short prefix walk instead of the four
  // from-the-start path lookups it used to (the hub's splitter: ~20 % less per line).
  struct Info {
    std::string_view type, name, rv, job, ikind, iname, reason;
    bool has_type = false, has_name = false, has_rv = false, has_job = false, has_ikind = false, has_iname = false;
    bool has_reason = false;
  };

  bool envelope(bool wrapped, std::string_view job_label, bool want_involved, Info& in) {
    i_ = 0;
    try {
      if (!wrapped) return object_fields(job_label, want_involved, in);
      ws();
      if (i_ >= n_ || s_[i_] != '{') return false;
      ++i_;
      while (true) {
        ws();
        if (i_ >= n_ || s_[i_] == '}') return true;
        if (s_[i_] != '"') return false;
        bool esc;
        std::string_view k = str(esc);
        ws();
        if (i_ >= n_ || s_[i_] != ':') return false;
        ++i_;
        ws();
        if (!esc && k == "type" && i_ < n_ && s_[i_] == '"') {
          in.type = str(esc);
          in.has_type = !esc;
        } else if (!esc && k == "object" && i_ < n_ && s_[i_] == '{') {
          // the scan stops inside the object: a type after it is left to the caller
          // (the API server always writes "type" first)
          return object_fields(job_label, want_involved, in);
        } else {
          skip_value();
        }
        ws();
        if (i_ < n_ && s_[i_] == ',') ++i_;
      }
    } catch (const ParseError&) {
      return false;
    }
  }

  // LIST body: metadata.resourceVersion and the byte range of every element of "items"
  bool list_items(std::string_view& rv, std::vector<std::pair<size_t, size_t>>& items) {
    static const char* const P_RV[] = {"metadata", "resourceVersion"};
    find(P_RV, 2, rv);
    i_ = 0;
    try {
      ws();
      if (i_ >= n_ || s_[i_] != '{') return false;
      ++i_;
      while (true) {
        ws();
        if (i_ >= n_ || s_[i_] != '"') return false;
        bool esc;
        std::string_view k = str(esc);
        ws();
        if (i_ >= n_ || s_[i_] != ':') return false;
        ++i_;
        ws();
        if (k == "items" && i_ < n_ && s_[i_] == '[') {
          ++i_;
          while (true) {
            ws();
            if (i_ >= n_) return false;
            if (s_[i_] == ']') return true;
            size_t b = i_;
            skip_value();
            items.emplace_back(b, i_);
            ws();
            if (i_ < n_ && s_[i_] == ',') ++i_;
          }
        }
        skip_value();
        ws();
        if (i_ < n_ && s_[i_] == ',') ++i_;
        else return false;
      }
    } catch (const ParseError&) {
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
  // raw string token at i_ (on the opening quote); escaped = contains a backslash
  std::string_view str(bool& escaped) {
    size_t st = ++i_;
    escaped = false;
    while (i_ < n_) {
      char c = s_[i_];
      if (c == '\\') {
        escaped = true;
        i_ += 2;
        continue;
      }
      if (c == '"') {
        std::string_view v(s_ + st, i_ - st);
        ++i_;
        return v;
      }
      ++i_;
    }
    throw ParseError{"unterminated string", i_};
  }
  void skip_value() {
    ws();
    if (i_ >= n_) throw ParseError{"unexpected end", i_};
    char c = s_[i_];
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
      throw ParseError{"unterminated container", i_};
    }
    while (i_ < n_ && s_[i_] != ',' && s_[i_] != '}' && s_[i_] != ']') ++i_;
  }
  // string members of a flat object at i_ (on its '{'): each key in `keys` (with its slot in
  // `vals` / `got`); other members are skipped
  template <size_t N>
  void members(const std::string_view (&keys)[N], std::string_view (&vals)[N], bool (&got)[N]) {
    ++i_;
    while (true) {
      ws();
      if (i_ >= n_) throw ParseError{"unexpected end", i_};
      if (s_[i_] == '}') {
        ++i_;
        return;
      }
      if (s_[i_] != '"') throw ParseError{"expected key", i_};
      bool esc;
      std::string_view k = str(esc);
      bool kesc = esc;
      ws();
      if (i_ >= n_ || s_[i_] != ':') throw ParseError{"expected ':'", i_};
      ++i_;
      ws();
      size_t hit = N;
      if (!kesc && i_ < n_ && s_[i_] == '"')
        for (size_t j = 0; j < N; ++j)
          if (!got[j] && k == keys[j]) {
            hit = j;
            break;
          }
      if (hit < N) {
        std::string_view v = str(esc);
        if (!esc) {
          vals[hit] = v;
          got[hit] = true;
        }
      } else {
        skip_value();
      }
      ws();
      if (i_ < n_ && s_[i_] == ',') ++i_;
    }
  }

  // the object at i_: metadata (name, resourceVersion, labels[job_label]) and, when wanted,
  // an Event's involvedObject (kind, name) and reason; returns once those are read, leaving
  // i_ inside the object
  bool object_fields(std::string_view job_label, bool want_involved, Info& in) {
    ws();
    if (i_ >= n_ || s_[i_] != '{') return false;
    ++i_;
    bool meta_done = false, inv_done = !want_involved, reason_done = !want_involved;
    while (true) {
      ws();
      if (i_ >= n_ || s_[i_] == '}') return true;
      if (s_[i_] != '"') return false;
      bool esc;
      std::string_view k = str(esc);
      ws();
      if (i_ >= n_ || s_[i_] != ':') return false;
      ++i_;
      ws();
      if (!esc && k == "metadata" && i_ < n_ && s_[i_] == '{') {
        ++i_;
        while (true) {
          ws();
          if (i_ >= n_) return false;
          if (s_[i_] == '}') {
            ++i_;
            break;
          }
          if (s_[i_] != '"') return false;
          std::string_view mk = str(esc);
          bool kesc = esc;
          ws();
          if (i_ >= n_ || s_[i_] != ':') return false;
          ++i_;
          ws();
          if (!kesc && i_ < n_ && s_[i_] == '"' && (mk == "name" || mk == "resourceVersion")) {
            std::string_view v = str(esc);
            if (!esc) {
              if (mk == "name") {
                in.name = v;
                in.has_name = true;
              } else {
                in.rv = v;
                in.has_rv = true;
              }
            }
          } else if (!kesc && mk == "labels" && i_ < n_ && s_[i_] == '{' && !job_label.empty()) {
            const std::string_view keys[1] = {job_label};
            std::string_view vals[1];
            bool got[1] = {false};
            members(keys, vals, got);
            if (got[0]) {
              in.job = vals[0];
              in.has_job = true;
            }
          } else {
            skip_value();
          }
          ws();
          if (i_ < n_ && s_[i_] == ',') ++i_;
        }
        meta_done = true;
      } else if (!esc && k == "involvedObject" && want_involved && i_ < n_ && s_[i_] == '{') {
        static const std::string_view keys[2] = {"kind", "name"};
        std::string_view vals[2];
        bool got[2] = {false, false};
        members(keys, vals, got);
        if (got[0]) {
          in.ikind = vals[0];
          in.has_ikind = true;
        }
        if (got[1]) {
          in.iname = vals[1];
          in.has_iname = true;
        }
        inv_done = true;
      } else if (!esc && k == "reason" && want_involved && i_ < n_ && s_[i_] == '"') {
        std::string_view v = str(esc);
        if (!esc) {
          in.reason = v;
          in.has_reason = true;
        }
        reason_done = true;
      } else {
        skip_value();
      }
      if (meta_done && inv_done && reason_done) return true;
      ws();
      if (i_ < n_ && s_[i_] == ',') ++i_;
    }
  }

  bool walk(const char* const* path, size_t depth, std::string_view& out) {
    ws();
    if (i_ >= n_ || s_[i_] != '{') return false;
    ++i_;
    while (true) {
      ws();
      if (i_ >= n_) return false;
      if (s_[i_] == '}') return false;
      if (s_[i_] != '"') return false;
      bool esc;
      std::string_view k = str(esc);
      ws();
      if (i_ >= n_ || s_[i_] != ':') return false;
      ++i_;
      if (!esc && k == path[0]) {
        if (depth == 1) {
          ws();
          if (i_ >= n_ || s_[i_] != '"') return false;
          out = str(esc);
          return !esc;
        }
        return walk(path + 1, depth - 1, out);
      }
      skip_value();
      ws();
      if (i_ < n_ && s_[i_] == ',') ++i_;
    }
  }
};

// A pod's placement: its worker inside the replica and the replica-shard hash of its
// run (kept raw so a later change of the owned shard set re-evaluates it).
struct PodOwner {
  int worker;
  uint32_t rhash;
  bool labeled;
};

// Deleted pods are remembered (for Pod Events still in flight) in two generations, each
// a hash map living in a bump arena: a generation is dropped by handing its arena's blocks
// back to a shared pool — never by erasing its entries one by one.  Erasing them (a budget
// per pod line, before) touched every cold entry once more: a saturated phase deletes ~20k
// pods a second, and 30 s later the hub's pump spent ~1 ms per chunk for seconds erasing
// them (the open-loop probe's recurring tail window, profiles/r6/README.md).  Blocks are
// kept for the next generation (up to POOL_KEEP bytes), so a rotation makes no syscall.
constexpr size_t ARENA_BLOCK = 1 << 20;
constexpr size_t POOL_KEEP = size_t(96) << 20;

struct BlockPool {
  std::vector<char*> blocks;                    // free ARENA_BLOCK blocks
  std::vector<std::pair<char*, size_t>> large;  // free oversized blocks (hash bucket arrays)
  size_t kept = 0;
  char* take(size_t n, size_t& got) {
    if (n <= ARENA_BLOCK) {
      got = ARENA_BLOCK;
      if (!blocks.empty()) {
        char* b = blocks.back();
        blocks.pop_back();
        kept -= ARENA_BLOCK;
        return b;
      }
      return static_cast<char*>(::operator new(ARENA_BLOCK));
    }
    for (size_t i = 0; i < large.size(); ++i)
      if (large[i].second >= n) {
        auto b = large[i];
        large[i] = large.back();
        large.pop_back();
        kept -= b.second;
        got = b.second;
        return b.first;
      }
    got = n;
    return static_cast<char*>(::operator new(n));
  }
  void give(char* b, size_t n) {
    if (kept + n > POOL_KEEP) {
      ::operator delete(b);
      return;
    }
    kept += n;
    if (n == ARENA_BLOCK) blocks.push_back(b);
    else large.emplace_back(b, n);
  }
  ~BlockPool() {
    for (char* b : blocks) ::operator delete(b);
    for (auto& b : large) ::operator delete(b.first);
  }
};

class GenArena : public std::pmr::memory_resource {
 public:
  explicit GenArena(BlockPool* pool) : pool_(pool) {}
  ~GenArena() override { reset(); }
  // hand every block back to the pool: the objects in them are simply forgotten (their
  // types own nothing outside this arena)
  void reset() {
    for (auto& b : used_) pool_->give(b.first, b.second);
    used_.clear();
    cur_ = end_ = nullptr;
  }

 private:
  static char* align_up(char* p, size_t align) {
    return reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(p) + align - 1) & ~(uintptr_t(align) - 1));
  }
  void* do_allocate(size_t n, size_t align) override {
    size_t got = 0;
    if (n + align > ARENA_BLOCK / 4) {  // a big object (a bucket array) gets a block of its own
      char* b = pool_->take(n + align, got);
      used_.emplace_back(b, got);
      return align_up(b, align);
    }
    char* p = cur_ ? align_up(cur_, align) : nullptr;
    if (p == nullptr || p + n > end_) {
      char* b = pool_->take(ARENA_BLOCK, got);
      used_.emplace_back(b, got);
      cur_ = b;
      end_ = b + got;
      p = align_up(cur_, align);
    }
    cur_ = p + n;
    return p;
  }
  void do_deallocate(void*, size_t, size_t) override {}  // freed wholesale by reset()
  bool do_is_equal(const std::pmr::memory_resource& o) const noexcept override { return this == &o; }

  BlockPool* pool_;
  std::vector<std::pair<char*, size_t>> used_;
  char* cur_ = nullptr;
  char* end_ = nullptr;
};

struct GoneGen {
  using Map = std::pmr::unordered_map<std::string_view, PodOwner>;
  GenArena arena;
  Map* map = nullptr;  // constructed in the arena, never destructed: dropped with it
  explicit GoneGen(BlockPool* pool) : arena(pool) { fresh(); }
  void fresh() {
    arena.reset();
    map = new (arena.allocate(sizeof(Map), alignof(Map))) Map(&arena);
  }
  const PodOwner* find(std::string_view k) const;
  void put(std::string_view k, const PodOwner& po);
  size_t size() const { return map->size(); }
};

struct Owners {
  std::unordered_map<std::string, PodOwner> pod;  // pods not deleted (yet)
  BlockPool pool;                                 // outlives the generations below
  std::unique_ptr<GoneGen> gone_cur = std::make_unique<GoneGen>(&pool);
  std::unique_ptr<GoneGen> gone_prev = std::make_unique<GoneGen>(&pool);
  double rotate_at = 0.0;
  std::string tmp;  // lookup key buffer
};

const PodOwner* GoneGen::find(std::string_view k) const {
  auto it = map->find(k);
  return it == map->end() ? nullptr : &it->second;
}

void GoneGen::put(std::string_view k, const PodOwner& po) {
  auto it = map->find(k);
  if (it != map->end()) {
    it->second = po;
    return;
  }
  char* c = static_cast<char*>(arena.allocate(k.size() ? k.size() : 1, 1));
  std::memcpy(c, k.data(), k.size());
  map->emplace(std::string_view(c, k.size()), po);
}


typedef struct {
  PyObject_HEAD
  int index;
  int count;
  uint32_t seed;
  double forget_after;
  std::string* job_label;
  Owners* owners;
  unsigned long long passed;
  unsigned long long dropped;
  // replica sharding (parallel/sharding.py): runs whose crc32(job name, rseed) % rcount
  // is not in `owned` belong to another replica and are dropped before decode
  int rcount;
  uint32_t rseed;
  std::vector<uint8_t>* owned;
  unsigned long long foreign;
  // Event reasons the supervisor's rules read (empty = all): an Event with another reason
  // (Scheduled, Pulling, Pulled, Created, Killing, SuccessfulCreate, ...) decides nothing,
  // so it is dropped here — no worker decodes, caches or dispatches it
  std::vector<std::string>* reasons;
  unsigned long long unread;
} Router;

enum Role { ROLE_NONE = 0, ROLE_JOB, ROLE_POD, ROLE_EVENT };

int owner_of(const Router* r, std::string_view key) {
  return static_cast<int>(crc32_update(r->seed, key.data(), key.size()) % static_cast<uint32_t>(r->count));
}

// murmur3 finaliser over the CRC: CRC32 is affine in its seed, so without it the replica
// shard would be correlated with the worker placement (parallel/sharding.py shard_of)
uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

uint32_t replica_hash(const Router* r, std::string_view key) {
  return fmix32(crc32_update(r->rseed, key.data(), key.size()));
}

bool replica_owns_hash(const Router* r, uint32_t h) {
  if (r->rcount <= 1) return true;
  return (*r->owned)[h % static_cast<uint32_t>(r->rcount)] != 0;
}

// A deleted pod leaves the live map (its entry was just touched: a cheap erase) for the
// current generation; generations rotate every forget_after seconds, so a deleted pod is
// remembered for forget_after to twice that.
void note_deleted(Router* r, const std::string& name, const PodOwner& po) {
  Owners& ow = *r->owners;
  double now = mono_s();
  if (now >= ow.rotate_at) {
    ow.gone_prev->fresh();
    std::swap(ow.gone_prev, ow.gone_cur);
    ow.rotate_at = now + r->forget_after;
  }
  ow.pod.erase(name);
  ow.gone_cur->put(name, po);
}

const PodOwner* find_pod(const Owners& ow, const std::string& name) {
  auto it = ow.pod.find(name);
  if (it != ow.pod.end()) return &it->second;
  if (const PodOwner* g = ow.gone_cur->find(name)) return g;
  return ow.gone_prev->find(name);
}

// Owner worker of one object: a watch line ({"type", "object"} envelope) or a bare LIST
// item.  -1 = every worker must see it (bookmarks, errors, unparsable lines, Events about a
// Pod not seen yet).  Pod lines also record the pod's owner for Pod-Event routing.
constexpr int OWNER_ALL = -1;
constexpr int OWNER_NONE = -2;  // another replica's run: nobody here sees it
constexpr int OWNER_SKIP = -3;  // an Event whose reason no rule reads: nobody decodes it

bool reason_read(const Router* r, std::string_view reason) {
  for (const auto& x : *r->reasons)
    if (x == reason) return true;
  return false;
}

int pod_owner_now(const Router* r, const PodOwner& po) {
  if (po.labeled && !replica_owns_hash(r, po.rhash)) return OWNER_NONE;
  return po.worker;
}

int route_info(Router* r, int role, const Scan::Info& in, bool envelope) {
  if (role == ROLE_JOB) {
    if (!in.has_name) return OWNER_ALL;  // BOOKMARK / ERROR / unparsable
    if (!replica_owns_hash(r, replica_hash(r, in.name))) return OWNER_NONE;
    return owner_of(r, in.name);
  }
  if (role == ROLE_POD) {
    if (!in.has_name) return OWNER_ALL;
    PodOwner po{0, 0, false};
    if (in.has_job) po = PodOwner{owner_of(r, in.job), replica_hash(r, in.job), true};
    Owners& ow = *r->owners;
    ow.tmp.assign(in.name.data(), in.name.size());  // reused buffer: no allocation for a known pod
    if (envelope && in.has_type && in.type == "DELETED") {
      note_deleted(r, ow.tmp, po);
    } else {
      auto it = ow.pod.find(ow.tmp);
      if (it == ow.pod.end()) ow.pod.emplace(ow.tmp, po);
      else it->second = po;
    }
    return pod_owner_now(r, po);
  }
  if (role == ROLE_EVENT) {
    if (!r->reasons->empty() && in.has_reason && !reason_read(r, in.reason)) return OWNER_SKIP;
    if (!in.has_ikind || !in.has_iname) return OWNER_ALL;
    if (in.ikind == "Job") {
      if (!replica_owns_hash(r, replica_hash(r, in.iname))) return OWNER_NONE;
      return owner_of(r, in.iname);
    }
    if (in.ikind == "Pod") {
      Owners& ow = *r->owners;
      ow.tmp.assign(in.iname.data(), in.iname.size());
      const PodOwner* po = find_pod(ow, ow.tmp);
      // unknown pod: everyone parks it until the pod shows up
      return po == nullptr ? OWNER_ALL : pod_owner_now(r, *po);
    }
    return 0;
  }
  return OWNER_ALL;
}

int route_owner(Router* r, int role, const char* s, size_t n, bool envelope) {
  Scan sc(s, n);
  Scan::Info in;
  sc.envelope(envelope, role == ROLE_POD ? std::string_view(*r->job_label) : std::string_view(), role == ROLE_EVENT, in);
  return route_info(r, role, in, envelope);
}

// true = this worker owns (or must see) the watch line
bool route_line(Router* r, int role, const char* s, size_t n) {
  int owner = route_owner(r, role, s, n, true);
  if (owner == OWNER_NONE) ++r->foreign;
  else if (owner == OWNER_SKIP) ++r->unread;
  return owner == OWNER_ALL || owner == r->index;
}

void Router_dealloc(Router* self) {
  delete self->job_label;
  delete self->owners;
  delete self->owned;
  delete self->reasons;
  Py_TYPE(self)->tp_free(reinterpret_cast<PyObject*>(self));
}

PyObject* Router_new(PyTypeObject* type, PyObject*, PyObject*) {
  Router* self = reinterpret_cast<Router*>(type->tp_alloc(type, 0));
  if (self) {
    self->index = 0;
    self->count = 1;
    self->seed = 0;
    self->forget_after = 120.0;
    self->job_label = new std::string("batch.kubernetes.io/job-name");
    self->owners = new Owners();
    self->passed = self->dropped = 0;
    self->rcount = 1;
    self->rseed = 0;
    self->owned = new std::vector<uint8_t>(1, 1);
    self->foreign = 0;
    self->reasons = new std::vector<std::string>();
    self->unread = 0;
  }
  return reinterpret_cast<PyObject*>(self);
}

int Router_init(Router* self, PyObject* args, PyObject* kw) {
  static const char* kwlist[] = {"index", "count", "seed", "job_label", "forget_after", nullptr};
  unsigned long seed = 0;
  const char* label = nullptr;
  double forget = 120.0;
  if (!PyArg_ParseTupleAndKeywords(args, kw, "iik|sd", const_cast<char**>(kwlist), &self->index, &self->count, &seed,
                                   &label, &forget))
    return -1;
  if (self->count < 1 || self->index < 0 || self->index >= self->count) {
    PyErr_SetString(PyExc_ValueError, "index must be in [0, count)");
    return -1;
  }
  self->seed = static_cast<uint32_t>(seed);
  self->forget_after = forget;
  if (label) *self->job_label = label;
  return 0;
}

PyObject* Router_owner_of(Router* self, PyObject* arg) {
  Py_ssize_t n;
  const char* s = PyUnicode_AsUTF8AndSize(arg, &n);
  if (!s) return nullptr;
  return PyLong_FromLong(owner_of(self, std::string_view(s, static_cast<size_t>(n))));
}

PyObject* Router_pod_owner(Router* self, PyObject* arg) {
  Py_ssize_t n;
  const char* s = PyUnicode_AsUTF8AndSize(arg, &n);
  if (!s) return nullptr;
  const PodOwner* po = find_pod(*self->owners, std::string(s, static_cast<size_t>(n)));
  if (po == nullptr) Py_RETURN_NONE;
  return PyLong_FromLong(pod_owner_now(self, *po));
}

// note_pod(name, owner[, deleted[, job]]) — job: the pod's run (job name) for replica sharding
PyObject* Router_note_pod(Router* self, PyObject* args) {
  const char* name;
  int owner;
  int deleted = 0;
  const char* job = nullptr;
  Py_ssize_t job_n = 0;
  if (!PyArg_ParseTuple(args, "si|pz#", &name, &owner, &deleted, &job, &job_n)) return nullptr;
  PodOwner po{owner, 0, false};
  if (job) po = PodOwner{owner, replica_hash(self, std::string_view(job, static_cast<size_t>(job_n))), true};
  if (deleted) note_deleted(self, name, po);
  else self->owners->pod[name] = po;
  Py_RETURN_NONE;
}

// set_replica(count, seed, owned) — replica shards: drop runs of shards not in `owned`
PyObject* Router_set_replica(Router* self, PyObject* args) {
  int count;
  unsigned long seed;
  PyObject* owned;
  if (!PyArg_ParseTuple(args, "ikO", &count, &seed, &owned)) return nullptr;
  if (count < 1) {
    PyErr_SetString(PyExc_ValueError, "count must be >= 1");
    return nullptr;
  }
  std::vector<uint8_t> bits(static_cast<size_t>(count), 0);
  PyObject* it = PyObject_GetIter(owned);
  if (!it) return nullptr;
  PyObject* item;
  while ((item = PyIter_Next(it)) != nullptr) {
    long k = PyLong_AsLong(item);
    Py_DECREF(item);
    if (k == -1 && PyErr_Occurred()) break;
    if (k < 0 || k >= count) {
      PyErr_SetString(PyExc_ValueError, "owned shard out of range [0, count)");
      break;
    }
    bits[static_cast<size_t>(k)] = 1;
  }
  Py_DECREF(it);
  if (PyErr_Occurred()) return nullptr;
  self->rcount = count;
  self->rseed = static_cast<uint32_t>(seed);
  *self->owned = std::move(bits);
  Py_RETURN_NONE;
}

// set_event_reasons(reasons or None) — Event lines with another reason are dropped
PyObject* Router_set_event_reasons(Router* self, PyObject* arg) {
  std::vector<std::string> v;
  if (arg != Py_None) {
    PyObject* it = PyObject_GetIter(arg);
    if (!it) return nullptr;
    PyObject* item;
    while ((item = PyIter_Next(it)) != nullptr) {
      Py_ssize_t n;
      const char* c = PyUnicode_AsUTF8AndSize(item, &n);
      if (c) v.emplace_back(c, static_cast<size_t>(n));
      Py_DECREF(item);
      if (!c) break;
    }
    Py_DECREF(it);
    if (PyErr_Occurred()) return nullptr;
  }
  *self->reasons = std::move(v);
  Py_RETURN_NONE;
}

PyObject* Router_stats(Router* self, void*) {
  const Owners& ow = *self->owners;
  return Py_BuildValue("{s:K,s:K,s:K,s:K,s:n,s:n,s:n}", "passed", self->passed, "dropped", self->dropped, "foreign",
                       self->foreign, "unread", self->unread, "pods", static_cast<Py_ssize_t>(ow.pod.size()),
                       "gone", static_cast<Py_ssize_t>(ow.gone_cur->size() + ow.gone_prev->size()), "pool_bytes",
                       static_cast<Py_ssize_t>(ow.pool.kept));
}

PyMethodDef Router_methods[] = {
    {"owner_of", reinterpret_cast<PyCFunction>(Router_owner_of), METH_O, "Owner worker of a job name"},
    {"pod_owner", reinterpret_cast<PyCFunction>(Router_pod_owner), METH_O,
     "Owner worker of a pod seen so far (None = unknown, -2 = another replica's run)"},
    {"note_pod", reinterpret_cast<PyCFunction>(Router_note_pod), METH_VARARGS,
     "Record a pod's owner (name, owner[, deleted[, job name]])"},
    {"set_replica", reinterpret_cast<PyCFunction>(Router_set_replica), METH_VARARGS,
     "Replica sharding: (shard count, seed, owned shard indexes)"},
    {"set_event_reasons", reinterpret_cast<PyCFunction>(Router_set_event_reasons), METH_O,
     "Event reasons any rule reads (None = all): Events with another reason are dropped"},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef Router_getset[] = {{"stats", reinterpret_cast<getter>(Router_stats), nullptr, nullptr, nullptr},
                               {nullptr, nullptr, nullptr, nullptr, nullptr}};

PyTypeObject RouterType = {PyVarObject_HEAD_INIT(nullptr, 0)};

int role_from(const char* role) {
  if (!role) return -1;
  return !strcmp(role, "job") ? ROLE_JOB : !strcmp(role, "pod") ? ROLE_POD : !strcmp(role, "event") ? ROLE_EVENT : -1;
}

// ------------------------------------------------------------------ watch hub splitter
// One watch stream per replica, demultiplexed to the shard workers (parallel/watchhub.py):
// feed(chunk) routes every complete line to its owner's output (bookmarks are consumed
// here, errors handed back), split_list(body) does the same for a LIST body's items.
typedef struct {
  PyObject_HEAD
  Router* router;
  int role;
  std::string* buf;
  unsigned long long lines;
} Splitter;

void Splitter_dealloc(Splitter* self) {
  Py_XDECREF(reinterpret_cast<PyObject*>(self->router));
  delete self->buf;
  Py_TYPE(self)->tp_free(reinterpret_cast<PyObject*>(self));
}

PyObject* Splitter_new(PyTypeObject* type, PyObject*, PyObject*) {
  Splitter* self = reinterpret_cast<Splitter*>(type->tp_alloc(type, 0));
  if (self) {
    self->router = nullptr;
    self->role = ROLE_NONE;
    self->buf = new std::string();
    self->lines = 0;
  }
  return reinterpret_cast<PyObject*>(self);
}

int Splitter_init(Splitter* self, PyObject* args, PyObject*) {
  PyObject* r;
  const char* role;
  if (!PyArg_ParseTuple(args, "Os", &r, &role)) return -1;
  if (!PyObject_TypeCheck(r, &RouterType)) {
    PyErr_SetString(PyExc_TypeError, "router must be a ShardRouter");
    return -1;
  }
  int rl = role_from(role);
  if (rl < 0) {
    PyErr_SetString(PyExc_ValueError, "role must be job, pod or event");
    return -1;
  }
  Py_INCREF(r);
  Py_XDECREF(reinterpret_cast<PyObject*>(self->router));
  self->router = reinterpret_cast<Router*>(r);
  self->role = rl;
  return 0;
}

PyObject* bytes_list(const std::vector<std::string>& outs) {
  PyObject* l = PyList_New(static_cast<Py_ssize_t>(outs.size()));
  if (!l) return nullptr;
  for (size_t w = 0; w < outs.size(); ++w) {
    PyObject* b = PyBytes_FromStringAndSize(outs[w].data(), static_cast<Py_ssize_t>(outs[w].size()));
    if (!b) {
      Py_DECREF(l);
      return nullptr;
    }
    PyList_SET_ITEM(l, static_cast<Py_ssize_t>(w), b);
  }
  return l;
}

// feed(chunk) -> (per-worker NDJSON bytes, last resourceVersion or None, [error lines])
PyObject* Splitter_feed(Splitter* self, PyObject* arg) {
  Py_buffer view;
  if (PyObject_GetBuffer(arg, &view, PyBUF_SIMPLE) != 0) return nullptr;
  std::string& buf = *self->buf;
  buf.append(static_cast<const char*>(view.buf), static_cast<size_t>(view.len));
  PyBuffer_Release(&view);
  Router* r = self->router;
  std::vector<std::string> outs(static_cast<size_t>(r->count));
  std::string last_rv;
  PyObject* errors = PyList_New(0);
  if (!errors) return nullptr;
  size_t start = 0;
  while (true) {
    const void* nl = memchr(buf.data() + start, '\n', buf.size() - start);
    if (!nl) break;
    size_t end = static_cast<size_t>(static_cast<const char*>(nl) - buf.data());
    const char* line = buf.data() + start;
    size_t n = end - start;
    start = end + 1;
    if (n == 0 || (n == 1 && line[0] == '\r')) continue;
    ++self->lines;
    Scan sc(line, n);
    Scan::Info in;
    sc.envelope(true, self->role == ROLE_POD ? std::string_view(*r->job_label) : std::string_view(),
                self->role == ROLE_EVENT, in);
    std::string_view type = in.has_type ? in.type : std::string_view();
    if (!in.has_type) {  // an envelope whose object came before its type: look the type up
      static const char* const P_TYPE1[] = {"type"};
      sc.find(P_TYPE1, 1, type);
    }
    if (in.has_rv) last_rv.assign(in.rv.data(), in.rv.size());
    if (type == "BOOKMARK") continue;
    if (type == "ERROR") {
      PyObject* b = PyBytes_FromStringAndSize(line, static_cast<Py_ssize_t>(n));
      if (!b || PyList_Append(errors, b) != 0) {
        Py_XDECREF(b);
        Py_DECREF(errors);
        return nullptr;
      }
      Py_DECREF(b);
      continue;
    }
    int owner = route_info(r, self->role, in, true);
    if (owner == OWNER_NONE || owner == OWNER_SKIP) {
      ++(owner == OWNER_NONE ? r->foreign : r->unread);
      continue;
    }
    if (owner == OWNER_ALL) {
      for (auto& o : outs) {
        o.append(line, n);
        o += '\n';
      }
      ++r->passed;
    } else {
      outs[static_cast<size_t>(owner)].append(line, n);
      outs[static_cast<size_t>(owner)] += '\n';
      r->dropped += static_cast<unsigned long long>(r->count - 1);
    }
  }
  buf.erase(0, start);
  PyObject* l = bytes_list(outs);
  if (!l) {
    Py_DECREF(errors);
    return nullptr;
  }
  PyObject* rvo = last_rv.empty() ? (Py_INCREF(Py_None), Py_None)
                                  : PyUnicode_FromStringAndSize(last_rv.data(), static_cast<Py_ssize_t>(last_rv.size()));
  return Py_BuildValue("(NNN)", l, rvo, errors);
}

// split_list(body) -> (resourceVersion, per-worker JSON arrays of the LIST's items)
PyObject* Splitter_split_list(Splitter* self, PyObject* arg) {
  Py_buffer view;
  if (PyObject_GetBuffer(arg, &view, PyBUF_SIMPLE) != 0) return nullptr;
  const char* s = static_cast<const char*>(view.buf);
  Scan sc(s, static_cast<size_t>(view.len));
  std::string_view rv;
  std::vector<std::pair<size_t, size_t>> items;
  if (!sc.list_items(rv, items)) {
    PyBuffer_Release(&view);
    PyErr_SetString(PyExc_ValueError, "not a LIST body with an items array");
    return nullptr;
  }
  Router* r = self->router;
  std::vector<std::string> outs(static_cast<size_t>(r->count), std::string("["));
  for (auto& it : items) {
    int owner = route_owner(r, self->role, s + it.first, it.second - it.first, false);
    if (owner == OWNER_NONE || owner == OWNER_SKIP) {
      ++(owner == OWNER_NONE ? r->foreign : r->unread);
      continue;
    }
    for (int w = 0; w < r->count; ++w) {
      if (owner != OWNER_ALL && owner != w) continue;
      std::string& o = outs[static_cast<size_t>(w)];
      if (o.size() > 1) o += ',';
      o.append(s + it.first, it.second - it.first);
    }
  }
  for (auto& o : outs) o += ']';
  std::string rvs(rv);
  PyBuffer_Release(&view);
  PyObject* l = bytes_list(outs);
  if (!l) return nullptr;
  return Py_BuildValue("(s#N)", rvs.data(), static_cast<Py_ssize_t>(rvs.size()), l);
}

PyObject* Splitter_reset(Splitter* self, PyObject*) {
  self->buf->clear();
  Py_RETURN_NONE;
}

PyMethodDef Splitter_methods[] = {
    {"feed", reinterpret_cast<PyCFunction>(Splitter_feed), METH_O,
     "Route complete watch lines: (per-worker bytes, last resourceVersion, error lines)"},
    {"split_list", reinterpret_cast<PyCFunction>(Splitter_split_list), METH_O,
     "Split a LIST body: (resourceVersion, per-worker JSON item arrays)"},
    {"reset", reinterpret_cast<PyCFunction>(Splitter_reset), METH_NOARGS, "Drop a partial line"},
    {nullptr, nullptr, 0, nullptr}};

PyTypeObject SplitterType = {PyVarObject_HEAD_INIT(nullptr, 0)};

// ------------------------------------------------------------------ Python type
typedef struct {
  PyObject_HEAD
  Proj* proj;        // projection of the whole document (watch envelope or list body)
  std::string* buf;  // pending partial line (watch streams)
  KeyCache* keys;
  unsigned long long docs;
  unsigned long long bytes;
  Router* router;    // optional shard filter (owned reference)
  int role;
} Decoder;

void Decoder_dealloc(Decoder* self) {
  delete self->proj;
  delete self->buf;
  Py_XDECREF(reinterpret_cast<PyObject*>(self->router));
  Py_TYPE(self)->tp_free(reinterpret_cast<PyObject*>(self));
}

int Decoder_init(Decoder* self, PyObject* args, PyObject* kw) {
  PyObject* spec = Py_True;
  static const char* kwlist[] = {"projection", nullptr};
  if (!PyArg_ParseTupleAndKeywords(args, kw, "|O", const_cast<char**>(kwlist), &spec)) return -1;
  auto p = compile(spec);
  if (!p) return -1;
  delete self->proj;
  self->proj = p.release();
  if (!self->buf) self->buf = new std::string();
  self->keys = shared_keys();
  return 0;
}

PyObject* Decoder_new(PyTypeObject* type, PyObject*, PyObject*) {
  Decoder* self = reinterpret_cast<Decoder*>(type->tp_alloc(type, 0));
  if (self) {
    self->proj = nullptr;
    self->buf = nullptr;
    self->keys = nullptr;
    self->docs = self->bytes = 0;
    self->router = nullptr;
    self->role = ROLE_NONE;
  }
  return reinterpret_cast<PyObject*>(self);
}

PyObject* decode_one(Decoder* self, const char* s, size_t n) {
  Parser ps(s, n, self->keys);
  try {
    PyObject* v = ps.value(self->proj->kind == Proj::KEEP ? nullptr : self->proj);
    if (!v) return nullptr;
    ps.ws();
    if (ps.pos() != n) {
      Py_DECREF(v);
      PyErr_Format(PyExc_ValueError, "trailing data at offset %zu", ps.pos());
      return nullptr;
    }
    ++self->docs;
    self->bytes += n;
    return v;
  } catch (const ParseError& e) {
    PyErr_Format(PyExc_ValueError, "JSON parse error: %s at offset %zu", e.msg, e.at);
    return nullptr;
  } catch (const std::exception& e) {
    PyErr_Format(PyExc_ValueError, "JSON parse error: %s", e.what());
    return nullptr;
  }
}

// decode(bytes) -> projected object (one JSON document, e.g. a LIST body)
PyObject* Decoder_decode(Decoder* self, PyObject* arg) {
  Py_buffer view;
  if (PyObject_GetBuffer(arg, &view, PyBUF_SIMPLE) != 0) return nullptr;
  PyObject* r = decode_one(self, static_cast<const char*>(view.buf), static_cast<size_t>(view.len));
  PyBuffer_Release(&view);
  return r;
}

// Watch envelope -> (type, object) with object["kind"] defaulted to `kind` (the informer's
// batched path; what watchhub.HubListWatch.watch_batches did per line in Python).  A missing
// or empty object becomes a fresh {} like `ev.get("object") or {}`.
PyObject* envelope_pair(PyObject* ev, PyObject* kind) {
  static PyObject* k_type = PyUnicode_InternFromString("type");
  static PyObject* k_object = PyUnicode_InternFromString("object");
  static PyObject* k_kind = PyUnicode_InternFromString("kind");
  static PyObject* empty = PyUnicode_InternFromString("");
  if (!PyDict_Check(ev)) {
    PyErr_SetString(PyExc_ValueError, "watch line is not a JSON object");
    return nullptr;
  }
  PyObject* t = PyDict_GetItemWithError(ev, k_type);
  if (!t && PyErr_Occurred()) return nullptr;
  PyObject* o = PyDict_GetItemWithError(ev, k_object);
  if (!o && PyErr_Occurred()) return nullptr;
  PyObject* obj;
  if (o && PyObject_IsTrue(o) == 1) {
    Py_INCREF(o);
    obj = o;
  } else {
    obj = PyDict_New();
    if (!obj) return nullptr;
  }
  if (PyDict_Check(obj)) {
    PyObject* k = PyDict_GetItemWithError(obj, k_kind);
    if (!k && PyErr_Occurred()) {
      Py_DECREF(obj);
      return nullptr;
    }
    if ((!k || k == Py_None) && PyDict_SetItem(obj, k_kind, kind) != 0) {
      Py_DECREF(obj);
      return nullptr;
    }
  }
  PyObject* pair = PyTuple_Pack(2, t ? t : empty, obj);
  Py_DECREF(obj);
  return pair;
}

PyObject* feed_impl(Decoder* self, PyObject* arg, PyObject* kind);

// feed(bytes) -> [projected documents] for every complete '\n'-terminated line
PyObject* Decoder_feed(Decoder* self, PyObject* arg) { return feed_impl(self, arg, nullptr); }

// feed_events(bytes, kind) -> [(type, object)] for every complete line (object kind defaulted)
PyObject* Decoder_feed_events(Decoder* self, PyObject* args) {
  PyObject* data;
  PyObject* kind;
  if (!PyArg_ParseTuple(args, "OU", &data, &kind)) return nullptr;
  return feed_impl(self, data, kind);
}

PyObject* feed_impl(Decoder* self, PyObject* arg, PyObject* kind) {
  Py_buffer view;
  if (PyObject_GetBuffer(arg, &view, PyBUF_SIMPLE) != 0) return nullptr;
  std::string& buf = *self->buf;
  buf.append(static_cast<const char*>(view.buf), static_cast<size_t>(view.len));
  PyBuffer_Release(&view);
  PyObject* out = PyList_New(0);
  if (!out) return nullptr;
  size_t start = 0;
  while (true) {
    const void* nl = memchr(buf.data() + start, '\n', buf.size() - start);
    if (!nl) break;
    size_t end = static_cast<size_t>(static_cast<const char*>(nl) - buf.data());
    size_t a = start, b = end;
    while (a < b && (buf[a] == ' ' || buf[a] == '\r')) ++a;
    while (b > a && (buf[b - 1] == ' ' || buf[b - 1] == '\r')) --b;
    if (b > a && self->router && !route_line(self->router, self->role, buf.data() + a, b - a)) {
      ++self->router->dropped;
      start = end + 1;
      continue;
    }
    if (b > a) {
      if (self->router) ++self->router->passed;
      PyObject* v = decode_one(self, buf.data() + a, b - a);
      if (v && kind) {
        PyObject* pair = envelope_pair(v, kind);
        Py_DECREF(v);
        v = pair;
      }
      if (!v || PyList_Append(out, v) != 0) {
        Py_XDECREF(v);
        Py_DECREF(out);
        buf.erase(0, end + 1);
        return nullptr;
      }
      Py_DECREF(v);
    }
    start = end + 1;
  }
  buf.erase(0, start);
  return out;
}

// set_router(router, role) — role: "job" | "pod" | "event" | None (clears)
PyObject* Decoder_set_router(Decoder* self, PyObject* args) {
  PyObject* r;
  const char* role = nullptr;
  if (!PyArg_ParseTuple(args, "O|z", &r, &role)) return nullptr;
  Py_XDECREF(reinterpret_cast<PyObject*>(self->router));
  self->router = nullptr;
  self->role = ROLE_NONE;
  if (r == Py_None) Py_RETURN_NONE;
  if (!PyObject_TypeCheck(r, &RouterType)) {
    PyErr_SetString(PyExc_TypeError, "router must be a ShardRouter");
    return nullptr;
  }
  int rl = role == nullptr ? ROLE_NONE : role_from(role);
  if (rl < 0) {
    PyErr_SetString(PyExc_ValueError, "role must be job, pod or event");
    return nullptr;
  }
  Py_INCREF(r);
  self->router = reinterpret_cast<Router*>(r);
  self->role = rl;
  Py_RETURN_NONE;
}

PyObject* Decoder_reset(Decoder* self, PyObject*) {
  self->buf->clear();
  Py_RETURN_NONE;
}

PyObject* Decoder_stats(Decoder* self, void*) {
  return Py_BuildValue("{s:K,s:K,s:n}", "docs", self->docs, "bytes", self->bytes, "buffered",
                       static_cast<Py_ssize_t>(self->buf->size()));
}

PyMethodDef Decoder_methods[] = {
    {"decode", reinterpret_cast<PyCFunction>(Decoder_decode), METH_O, "Decode one JSON document with projection"},
    {"feed", reinterpret_cast<PyCFunction>(Decoder_feed), METH_O, "Feed stream bytes; decode complete lines"},
    {"feed_events", reinterpret_cast<PyCFunction>(Decoder_feed_events), METH_VARARGS,
     "Feed watch stream bytes; [(type, object)] per complete line, object kind defaulted"},
    {"reset", reinterpret_cast<PyCFunction>(Decoder_reset), METH_NOARGS, "Drop a partial line"},
    {"set_router", reinterpret_cast<PyCFunction>(Decoder_set_router), METH_VARARGS,
     "Drop watch lines another shard worker owns (router, role)"},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef Decoder_getset[] = {{"stats", reinterpret_cast<getter>(Decoder_stats), nullptr, nullptr, nullptr},
                                {nullptr, nullptr, nullptr, nullptr, nullptr}};

PyTypeObject DecoderType = {PyVarObject_HEAD_INIT(nullptr, 0)};

}  // namespace

extern "C" PyObject* nexus_json_dumps(PyObject*, PyObject* args, PyObject* kw);  // json_encode.cpp
extern "C" int nexus_register_histogram(PyObject* m);                            // histogram.cpp
extern "C" PyObject* nexus_apply_lines(PyObject*, PyObject* args);               // informer_apply.cpp
extern "C" int nexus_register_shared_bucket(PyObject* m);                        // shared_bucket.cpp

namespace {

PyMethodDef module_methods[] = {
    {"dumps", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(nexus_json_dumps)),
     METH_VARARGS | METH_KEYWORDS, "dumps(obj, sort_keys=False, default=None, newline=False) -> bytes (compact UTF-8 JSON)"},
    {"apply_lines", nexus_apply_lines, METH_VARARGS,
     "apply_lines(batch, start, end, items, labels, indices, adds, updates, deletes, on_error, kind) -> "
     "(error_object, seen, resource_version): one watch batch into an informer cache + handlers"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef moddef = {PyModuleDef_HEAD_INIT, "_kube_native",
                      "Projected JSON decoding of Kubernetes watch streams and LIST bodies; fast JSON encoding", -1,
                      module_methods, nullptr, nullptr, nullptr, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__kube_native(void) {
  DecoderType.tp_name = "_kube_native.ProjectedDecoder";
  DecoderType.tp_basicsize = sizeof(Decoder);
  DecoderType.tp_flags = Py_TPFLAGS_DEFAULT;
  DecoderType.tp_new = Decoder_new;
  DecoderType.tp_init = reinterpret_cast<initproc>(Decoder_init);
  DecoderType.tp_dealloc = reinterpret_cast<destructor>(Decoder_dealloc);
  DecoderType.tp_methods = Decoder_methods;
  DecoderType.tp_getset = Decoder_getset;
  DecoderType.tp_doc = "ProjectedDecoder(projection=True)";
  if (PyType_Ready(&DecoderType) < 0) return nullptr;
  RouterType.tp_name = "_kube_native.ShardRouter";
  RouterType.tp_basicsize = sizeof(Router);
  RouterType.tp_flags = Py_TPFLAGS_DEFAULT;
  RouterType.tp_new = Router_new;
  RouterType.tp_init = reinterpret_cast<initproc>(Router_init);
  RouterType.tp_dealloc = reinterpret_cast<destructor>(Router_dealloc);
  RouterType.tp_methods = Router_methods;
  RouterType.tp_getset = Router_getset;
  RouterType.tp_doc = "ShardRouter(index, count, seed, job_label='batch.kubernetes.io/job-name', forget_after=120.0)";
  if (PyType_Ready(&RouterType) < 0) return nullptr;
  SplitterType.tp_name = "_kube_native.WatchSplitter";
  SplitterType.tp_basicsize = sizeof(Splitter);
  SplitterType.tp_flags = Py_TPFLAGS_DEFAULT;
  SplitterType.tp_new = Splitter_new;
  SplitterType.tp_init = reinterpret_cast<initproc>(Splitter_init);
  SplitterType.tp_dealloc = reinterpret_cast<destructor>(Splitter_dealloc);
  SplitterType.tp_methods = Splitter_methods;
  SplitterType.tp_doc = "WatchSplitter(router, role) — demultiplex one watch stream / LIST body to shard workers";
  if (PyType_Ready(&SplitterType) < 0) return nullptr;
  PyObject* m = PyModule_Create(&moddef);
  if (!m) return nullptr;
  Py_INCREF(&DecoderType);
  PyModule_AddObject(m, "ProjectedDecoder", reinterpret_cast<PyObject*>(&DecoderType));
  Py_INCREF(&RouterType);
  PyModule_AddObject(m, "ShardRouter", reinterpret_cast<PyObject*>(&RouterType));
  Py_INCREF(&SplitterType);
  PyModule_AddObject(m, "WatchSplitter", reinterpret_cast<PyObject*>(&SplitterType));
  if (nexus_register_histogram(m) < 0 || nexus_register_shared_bucket(m) < 0) {
    Py_DECREF(m);
    return nullptr;
  }
  return m;
}
