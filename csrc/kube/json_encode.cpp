// Fast JSON encoding of plain Python containers (dict / list / tuple / str / int /
// float / bool / None) for the watch-event producer side (fake apiserver in the wire
// benchmark) and other hot serialisers.
//
// Compared with CPython's C encoder this skips the per-container circular-reference
// markers dict (a depth limit guards runaway recursion instead), reuses UTF-8 caches of
// compact strings without copying, and writes straight into one growing buffer.
// Output is UTF-8 (ensure_ascii=False semantics) with compact separators.  A value of a
// bytes *subclass* is pre-encoded JSON and is copied verbatim (classify.RawJSON: a
// sub-document shared by many outputs is encoded once); plain bytes go to default=.
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

namespace {

constexpr int kMaxDepth = 256;

struct Enc {
  std::string out;
  bool sort_keys = false;
  PyObject* dflt = nullptr;  // borrowed: called for unsupported objects

  bool str(PyObject* s) {
    Py_ssize_t n = 0;
    const char* p = PyUnicode_AsUTF8AndSize(s, &n);
    if (!p) return false;
    out.push_back('"');
    const char* run = p;
    const char* end = p + n;
    // most strings need no escaping: test 8 bytes at a time for a byte < 0x20, '"' or '\\'
    // (SWAR zero-byte tests) and copy a clean run in one append
    const char* c = p;
    for (; c + 8 <= end; c += 8) {
      uint64_t w;
      memcpy(&w, c, 8);
      const uint64_t ones = 0x0101010101010101ULL, high = 0x8080808080808080ULL;
      uint64_t lt20 = (w - ones * 0x20) & ~w & high;
      uint64_t xq = w ^ (ones * '"'), xb = w ^ (ones * '\\');
      uint64_t q = (xq - ones) & ~xq & high, b = (xb - ones) & ~xb & high;
      if (lt20 | q | b) break;
    }
    for (; c < end; ++c) {
      unsigned char ch = static_cast<unsigned char>(*c);
      if (ch >= 0x20 && ch != '"' && ch != '\\') continue;
      out.append(run, c - run);
      switch (ch) {
        case '"': out.append("\\\""); break;
        case '\\': out.append("\\\\"); break;
        case '\n': out.append("\\n"); break;
        case '\r': out.append("\\r"); break;
        case '\t': out.append("\\t"); break;
        case '\b': out.append("\\b"); break;
        case '\f': out.append("\\f"); break;
        default: {
          char buf[8];
          snprintf(buf, sizeof buf, "\\u%04x", ch);
          out.append(buf);
        }
      }
      run = c + 1;
    }
    out.append(run, end - run);
    out.push_back('"');
    return true;
  }

  bool number_float(PyObject* o) {
    double d = PyFloat_AS_DOUBLE(o);
    if (d != d) {
      out.append("NaN");
      return true;
    }
    if (d == HUGE_VAL) {
      out.append("Infinity");
      return true;
    }
    if (d == -HUGE_VAL) {
      out.append("-Infinity");
      return true;
    }
    double a = std::fabs(d);
    if (a == 0.0 || (a >= 1e-4 && a < 1e16)) {
      // Python's repr: the shortest round-trip digits, fixed notation in this range (and a
      // ".0" on integral values) — std::to_chars(fixed) gives exactly those digits without
      // the malloc + format machinery of PyOS_double_to_string
      char buf[64];
      auto res = std::to_chars(buf, buf + sizeof buf, d, std::chars_format::fixed);
      if (res.ec == std::errc()) {
        size_t k = static_cast<size_t>(res.ptr - buf);
        out.append(buf, k);
        if (!memchr(buf, '.', k)) out.append(".0");
        return true;
      }
    }
    char* s = PyOS_double_to_string(d, 'r', 0, Py_DTSF_ADD_DOT_0, nullptr);
    if (!s) return false;
    out.append(s);
    PyMem_Free(s);
    return true;
  }

  bool number_int(PyObject* o) {
    int overflow = 0;
    long long v = PyLong_AsLongLongAndOverflow(o, &overflow);
    if (overflow == 0) {
      if (v == -1 && PyErr_Occurred()) return false;
      char buf[24];
      auto res = std::to_chars(buf, buf + sizeof buf, v);  // no locale / format parsing (snprintf)
      out.append(buf, static_cast<size_t>(res.ptr - buf));
      return true;
    }
    PyObject* s = PyObject_Str(o);
    if (!s) return false;
    Py_ssize_t n = 0;
    const char* p = PyUnicode_AsUTF8AndSize(s, &n);
    if (p) out.append(p, n);
    Py_DECREF(s);
    return p != nullptr;
  }

  // dict keys: str as-is; int/float/bool/None stringified like the json module
  bool key(PyObject* k) {
    if (PyUnicode_Check(k)) return str(k);
    out.push_back('"');
    bool ok = true;
    if (k == Py_True) out.append("true");
    else if (k == Py_False) out.append("false");
    else if (k == Py_None) out.append("null");
    else if (PyLong_Check(k)) ok = number_int(k);
    else if (PyFloat_Check(k)) ok = number_float(k);
    else {
      PyErr_Format(PyExc_TypeError, "keys must be str, int, float, bool or None, not %s", Py_TYPE(k)->tp_name);
      ok = false;
    }
    out.push_back('"');
    return ok;
  }

  bool dict(PyObject* d, int depth) {
    out.push_back('{');
    bool first = true;
    if (!sort_keys) {
      Py_ssize_t pos = 0;
      PyObject *k, *v;
      while (PyDict_Next(d, &pos, &k, &v)) {
        if (!first) out.push_back(',');
        first = false;
        if (!key(k)) return false;
        out.push_back(':');
        if (!value(v, depth + 1)) return false;
      }
    } else {
      // order by the key's code points (== its UTF-8 bytes), not by the escaped form
      struct Item {
        std::string sort, rendered;
        PyObject* v;
      };
      std::vector<Item> items;
      items.reserve(PyDict_GET_SIZE(d));
      Py_ssize_t pos = 0;
      PyObject *k, *v;
      while (PyDict_Next(d, &pos, &k, &v)) {
        std::string rendered;
        rendered.swap(out);
        bool ok = key(k);
        rendered.swap(out);
        if (!ok) return false;
        std::string sort;
        if (PyUnicode_Check(k)) {
          Py_ssize_t n = 0;
          const char* p = PyUnicode_AsUTF8AndSize(k, &n);
          if (!p) return false;
          sort.assign(p, n);
        } else {
          sort = rendered.substr(1, rendered.size() - 2);
        }
        items.push_back(Item{std::move(sort), std::move(rendered), v});
      }
      std::sort(items.begin(), items.end(), [](const Item& a, const Item& b) { return a.sort < b.sort; });
      for (auto& it : items) {
        if (!first) out.push_back(',');
        first = false;
        out.append(it.rendered);
        out.push_back(':');
        if (!value(it.v, depth + 1)) return false;
      }
    }
    out.push_back('}');
    return true;
  }

  bool seq(PyObject* s, int depth) {
    PyObject* fast = PySequence_Fast(s, "expected a sequence");
    if (!fast) return false;
    Py_ssize_t n = PySequence_Fast_GET_SIZE(fast);
    PyObject** items = PySequence_Fast_ITEMS(fast);
    out.push_back('[');
    bool ok = true;
    for (Py_ssize_t i = 0; i < n && ok; ++i) {
      if (i) out.push_back(',');
      ok = value(items[i], depth + 1);
    }
    out.push_back(']');
    Py_DECREF(fast);
    return ok;
  }

  bool value(PyObject* o, int depth) {
    if (depth > kMaxDepth) {
      PyErr_SetString(PyExc_ValueError, "JSON nesting too deep (circular reference?)");
      return false;
    }
    if (PyUnicode_Check(o)) return str(o);
    if (PyDict_Check(o)) return dict(o, depth);
    if (o == Py_None) {
      out.append("null");
      return true;
    }
    if (o == Py_True) {
      out.append("true");
      return true;
    }
    if (o == Py_False) {
      out.append("false");
      return true;
    }
    if (PyLong_Check(o)) return number_int(o);
    if (PyList_Check(o) || PyTuple_Check(o)) return seq(o, depth);
    if (PyFloat_Check(o)) return number_float(o);
    if (PyBytes_Check(o) && Py_TYPE(o) != &PyBytes_Type) {  // bytes subclass = pre-encoded JSON (RawJSON)
      out.append(PyBytes_AS_STRING(o), static_cast<size_t>(PyBytes_GET_SIZE(o)));
      return true;
    }
    if (dflt) {
      PyObject* r = PyObject_CallOneArg(dflt, o);
      if (!r) return false;
      bool ok = value(r, depth + 1);
      Py_DECREF(r);
      return ok;
    }
    PyErr_Format(PyExc_TypeError, "Object of type %s is not JSON serializable", Py_TYPE(o)->tp_name);
    return false;
  }
};

}  // namespace

// dumps(obj, sort_keys=False, default=None, newline=False) -> bytes
extern "C" PyObject* nexus_json_dumps(PyObject*, PyObject* args, PyObject* kw) {
  static const char* kwlist[] = {"obj", "sort_keys", "default", "newline", nullptr};
  PyObject* obj = nullptr;
  int sort_keys = 0, newline = 0;
  PyObject* dflt = Py_None;
  if (!PyArg_ParseTupleAndKeywords(args, kw, "O|pOp:dumps", const_cast<char**>(kwlist), &obj, &sort_keys, &dflt,
                                   &newline))
    return nullptr;
  Enc e;
  e.sort_keys = sort_keys != 0;
  e.dflt = dflt == Py_None ? nullptr : dflt;
  e.out.reserve(2048);
  if (!e.value(obj, 0)) return nullptr;
  if (newline) e.out.push_back('\n');
  return PyBytes_FromStringAndSize(e.out.data(), static_cast<Py_ssize_t>(e.out.size()));
}
