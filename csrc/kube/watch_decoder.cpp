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
// A non-object value where an object projection was expected is kept whole (so
// Status objects in ERROR events survive any kind's schema).
#include <Python.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

namespace {

struct Proj {
  enum Kind { KEEP, OBJECT, LIST, PREFIX, MAP } kind = KEEP;
  std::vector<std::pair<std::string, std::unique_ptr<Proj>>> fields;  // OBJECT (small: linear scan)
  std::unique_ptr<Proj> elem;                                         // LIST / MAP
  std::vector<std::string> prefixes;                                  // PREFIX

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

// Interned Python key strings, looked up by bytes without allocating (open addressing).
class KeyCache {
 public:
  KeyCache() : slots_(kCap) {}
  ~KeyCache() {
    for (auto& sl : slots_) Py_XDECREF(sl.obj);
  }
  // New reference to the Python str for `k`.
  PyObject* get(std::string_view k) {
    uint64_t h = 1469598103934665603ULL;
    for (unsigned char c : k) h = (h ^ c) * 1099511628211ULL;
    size_t i = h & (kCap - 1);
    for (size_t probe = 0; probe < 16; ++probe, i = (i + 1) & (kCap - 1)) {
      Slot& sl = slots_[i];
      if (!sl.obj) {
        PyObject* o = PyUnicode_DecodeUTF8(k.data(), static_cast<Py_ssize_t>(k.size()), "replace");
        if (!o) return nullptr;
        if (used_ < kCap / 2) {
          sl.hash = h;
          sl.key.assign(k.data(), k.size());
          sl.obj = o;
          Py_INCREF(o);
          ++used_;
        }
        return o;
      }
      if (sl.hash == h && sl.key.size() == k.size() && memcmp(sl.key.data(), k.data(), k.size()) == 0) {
        Py_INCREF(sl.obj);
        return sl.obj;
      }
    }
    return PyUnicode_DecodeUTF8(k.data(), static_cast<Py_ssize_t>(k.size()), "replace");
  }

 private:
  static constexpr size_t kCap = 8192;
  struct Slot {
    uint64_t hash = 0;
    std::string key;
    PyObject* obj = nullptr;
  };
  std::vector<Slot> slots_;
  size_t used_ = 0;
};

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
    std::string tok(s_ + st, i_ - st);
    if (!flt) {
      if (tok.size() < 18) return PyLong_FromLongLong(std::stoll(tok));
      return PyLong_FromString(tok.c_str(), nullptr, 10);
    }
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
    if (!esc) return PyUnicode_DecodeUTF8(s_ + a, static_cast<Py_ssize_t>(b - a), "replace");
    std::string u = unescape(a, b);
    return PyUnicode_DecodeUTF8(u.data(), static_cast<Py_ssize_t>(u.size()), "replace");
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
    return object_loop([&](PyObject* d, std::string_view k) {
      const Proj* sub = p->field(k);
      if (!sub) {
        skip();
        return true;
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

// ------------------------------------------------------------------ Python type
typedef struct {
  PyObject_HEAD
  Proj* proj;        // projection of the whole document (watch envelope or list body)
  std::string* buf;  // pending partial line (watch streams)
  KeyCache* keys;
  unsigned long long docs;
  unsigned long long bytes;
} Decoder;

void Decoder_dealloc(Decoder* self) {
  delete self->proj;
  delete self->buf;
  delete self->keys;
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
  if (!self->keys) self->keys = new KeyCache();
  return 0;
}

PyObject* Decoder_new(PyTypeObject* type, PyObject*, PyObject*) {
  Decoder* self = reinterpret_cast<Decoder*>(type->tp_alloc(type, 0));
  if (self) {
    self->proj = nullptr;
    self->buf = nullptr;
    self->keys = nullptr;
    self->docs = self->bytes = 0;
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

// feed(bytes) -> [projected documents] for every complete '\n'-terminated line
PyObject* Decoder_feed(Decoder* self, PyObject* arg) {
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
    if (b > a) {
      PyObject* v = decode_one(self, buf.data() + a, b - a);
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
    {"reset", reinterpret_cast<PyCFunction>(Decoder_reset), METH_NOARGS, "Drop a partial line"},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef Decoder_getset[] = {{"stats", reinterpret_cast<getter>(Decoder_stats), nullptr, nullptr, nullptr},
                                {nullptr, nullptr, nullptr, nullptr, nullptr}};

PyTypeObject DecoderType = {PyVarObject_HEAD_INIT(nullptr, 0)};

}  // namespace

extern "C" PyObject* nexus_json_dumps(PyObject*, PyObject* args, PyObject* kw);  // json_encode.cpp

namespace {

PyMethodDef module_methods[] = {
    {"dumps", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(nexus_json_dumps)),
     METH_VARARGS | METH_KEYWORDS, "dumps(obj, sort_keys=False, default=None, newline=False) -> bytes (compact UTF-8 JSON)"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef moddef = {PyModuleDef_HEAD_INIT, "_kube_native",
                      "Projected JSON decoding of Kubernetes watch streams and LIST bodies; fast JSON encoding", -1,
                      module_methods};

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
  PyObject* m = PyModule_Create(&moddef);
  if (!m) return nullptr;
  Py_INCREF(&DecoderType);
  PyModule_AddObject(m, "ProjectedDecoder", reinterpret_cast<PyObject*>(&DecoderType));
  return m;
}
