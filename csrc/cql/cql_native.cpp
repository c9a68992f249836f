// _cql_native — Python binding of the CQL v4 codec (cql_proto.hpp).
//
// The supervisor's checkpoint I/O (nexus-core CqlStore: one SELECT + ≤1 write per
// decision, /root/reference/services/supervisor.go:264-364) runs through this
// module: request frames are serialised and response frames split + decoded in
// C++; the asyncio client (nexus_supervisor_amd/store/cql.py) only moves bytes
// and matches stream ids.  Murmur3 tokens for token-aware routing of the
// composite partition key ((algorithm, id)) are computed here too.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cmath>
#include <unordered_map>

#include "cql_proto.hpp"

namespace py = pybind11;
using namespace nxcql;

namespace {

// ms -> Python timestamp object (None: keep int ms).  Heap-held and never destroyed: a
// static py::object would be DECREF'd by the C++ runtime after interpreter finalisation.
py::object& g_ts_factory = *new py::object();

// ---------------------------------------------------------------- types <-> Python
Type type_from_py(const py::handle& h) {
  Type t;
  if (py::isinstance<py::int_>(h)) {
    t.id = h.cast<uint16_t>();
    return t;
  }
  py::tuple tup = py::reinterpret_borrow<py::tuple>(h);
  if (tup.size() == 0) throw std::invalid_argument("empty type tuple");
  if (py::isinstance<py::str>(tup[0])) {  // ("custom", name)
    t.id = T_CUSTOM;
    t.custom = tup[1].cast<std::string>();
    return t;
  }
  t.id = tup[0].cast<uint16_t>();
  for (size_t i = 1; i < tup.size(); ++i) t.sub.push_back(type_from_py(tup[i]));
  return t;
}

py::object type_to_py(const Type& t) {
  if (t.id == T_CUSTOM) return py::make_tuple("custom", t.custom);
  if (t.sub.empty()) return py::int_(t.id);
  py::tuple out(t.sub.size() + 1);
  out[0] = py::int_(t.id);
  for (size_t i = 0; i < t.sub.size(); ++i) out[i + 1] = type_to_py(t.sub[i]);
  return out;
}

std::vector<Type> types_from_py(const py::handle& h) {
  std::vector<Type> v;
  if (h.is_none()) return v;
  for (auto item : h) v.push_back(type_from_py(item));
  return v;
}

// ---------------------------------------------------------------- value serialisation
int64_t to_ms(const py::handle& v) {
  if (py::isinstance<py::int_>(v)) return v.cast<int64_t>();
  if (py::hasattr(v, "timestamp")) {
    double s = v.attr("timestamp")().cast<double>();
    return static_cast<int64_t>(std::llround(s * 1000.0));
  }
  if (py::isinstance<py::float_>(v)) return static_cast<int64_t>(std::llround(v.cast<double>() * 1000.0));
  throw std::invalid_argument("timestamp value must be int ms, float seconds or datetime");
}

int hexval(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

std::string uuid_bytes(const py::handle& v) {
  if (py::isinstance<py::bytes>(v)) return v.cast<std::string>();
  if (py::hasattr(v, "bytes")) return v.attr("bytes").cast<std::string>();
  std::string s = py::str(v).cast<std::string>();
  std::string out;
  int hi = -1;
  for (char c : s) {
    if (c == '-') continue;
    int x = hexval(c);
    if (x < 0) throw std::invalid_argument("bad uuid string");
    if (hi < 0) hi = x;
    else {
      out.push_back(static_cast<char>((hi << 4) | x));
      hi = -1;
    }
  }
  if (out.size() != 16) throw std::invalid_argument("uuid must have 16 bytes");
  return out;
}

Type infer_type(const py::handle& v) {
  Type t;
  if (py::isinstance<py::bool_>(v)) t.id = T_BOOLEAN;
  else if (py::isinstance<py::int_>(v)) t.id = T_BIGINT;
  else if (py::isinstance<py::float_>(v)) t.id = T_DOUBLE;
  else if (py::isinstance<py::bytes>(v)) t.id = T_BLOB;
  else if (py::hasattr(v, "timestamp")) t.id = T_TIMESTAMP;
  else t.id = T_VARCHAR;
  return t;
}

void write_value(Writer& w, const py::handle& v, const Type& t);

std::string serialize(const py::handle& v, const Type& t) {
  Writer w;
  switch (t.id) {
    case T_VARCHAR:
    case T_ASCII:
      if (py::isinstance<py::bytes>(v)) return v.cast<std::string>();
      return py::str(v).cast<std::string>();
    case T_BLOB:
      if (py::isinstance<py::str>(v)) return v.cast<std::string>();
      return py::bytes(py::reinterpret_borrow<py::object>(v)).cast<std::string>();
    case T_TIMESTAMP: w.i64(to_ms(v)); return w.buf;
    case T_BIGINT:
    case T_COUNTER:
    case T_TIME: w.i64(v.cast<int64_t>()); return w.buf;
    case T_INT: w.i32(v.cast<int32_t>()); return w.buf;
    case T_SMALLINT: w.u16(static_cast<uint16_t>(v.cast<int16_t>())); return w.buf;
    case T_TINYINT: w.u8(static_cast<uint8_t>(v.cast<int8_t>())); return w.buf;
    case T_DATE: w.i32(static_cast<int32_t>(static_cast<uint32_t>(v.cast<int64_t>() + (int64_t(1) << 31)))); return w.buf;
    case T_BOOLEAN: w.u8(v.cast<bool>() ? 1 : 0); return w.buf;
    case T_DOUBLE: {
      double d = v.cast<double>();
      int64_t bits;
      memcpy(&bits, &d, 8);
      w.i64(bits);
      return w.buf;
    }
    case T_FLOAT: {
      float f = v.cast<float>();
      int32_t bits;
      memcpy(&bits, &f, 4);
      w.i32(bits);
      return w.buf;
    }
    case T_UUID:
    case T_TIMEUUID: return uuid_bytes(v);
    case T_LIST:
    case T_SET: {
      py::list items = py::list(py::reinterpret_borrow<py::object>(v));
      w.i32(static_cast<int32_t>(items.size()));
      for (auto it : items) write_value(w, it, t.sub.at(0));
      return w.buf;
    }
    case T_MAP: {
      py::dict d = py::reinterpret_borrow<py::dict>(v);
      w.i32(static_cast<int32_t>(d.size()));
      for (auto kv : d) {
        write_value(w, kv.first, t.sub.at(0));
        write_value(w, kv.second, t.sub.at(1));
      }
      return w.buf;
    }
    default: throw std::invalid_argument("cannot serialise CQL type id " + std::to_string(t.id));
  }
}

void write_value(Writer& w, const py::handle& v, const Type& t) {
  if (v.is_none()) {
    w.null_bytes();
    return;
  }
  std::string s = serialize(v, t);
  w.bytes(s);
}

// ---------------------------------------------------------------- value deserialisation
std::string fmt_uuid(const uint8_t* p) {
  static const char* hx = "0123456789abcdef";
  std::string s;
  s.reserve(36);
  for (int i = 0; i < 16; ++i) {
    if (i == 4 || i == 6 || i == 8 || i == 10) s.push_back('-');
    s.push_back(hx[p[i] >> 4]);
    s.push_back(hx[p[i] & 15]);
  }
  return s;
}

py::object decode_value(const uint8_t* p, int32_t n, const Type& t);

py::object decode_nullable(Reader& r, const Type& t) {
  const uint8_t* d;
  int32_t n;
  if (!r.bytes(d, n)) return py::none();
  return decode_value(d, n, t);
}

py::object decode_value(const uint8_t* p, int32_t n, const Type& t) {
  Reader r(p, static_cast<size_t>(n));
  switch (t.id) {
    case T_VARCHAR:
    case T_ASCII: {
      PyObject* o = PyUnicode_DecodeUTF8(reinterpret_cast<const char*>(p), n, "replace");
      if (!o) throw py::error_already_set();
      return py::reinterpret_steal<py::object>(o);
    }
    case T_BLOB:
    case T_CUSTOM:
    case T_DECIMAL:
    case T_VARINT: return py::bytes(reinterpret_cast<const char*>(p), static_cast<size_t>(n));
    case T_TIMESTAMP: {
      if (n != 8) throw ProtocolError("bad timestamp length");
      int64_t ms = r.i64();
      if (g_ts_factory && !g_ts_factory.is_none()) return g_ts_factory(ms);
      return py::int_(ms);
    }
    case T_BIGINT:
    case T_COUNTER:
    case T_TIME: return py::int_(r.i64());
    case T_INT: return py::int_(r.i32());
    case T_SMALLINT: return py::int_(static_cast<int16_t>(r.u16()));
    case T_TINYINT: return py::int_(static_cast<int8_t>(r.u8()));
    case T_DATE: return py::int_(static_cast<int64_t>(static_cast<uint32_t>(r.i32())) - (int64_t(1) << 31));
    case T_BOOLEAN: return py::bool_(n > 0 && p[0] != 0);
    case T_DOUBLE: {
      int64_t bits = r.i64();
      double d;
      memcpy(&d, &bits, 8);
      return py::float_(d);
    }
    case T_FLOAT: {
      int32_t bits = r.i32();
      float f;
      memcpy(&f, &bits, 4);
      return py::float_(f);
    }
    case T_UUID:
    case T_TIMEUUID:
      if (n != 16) throw ProtocolError("bad uuid length");
      return py::str(fmt_uuid(p));
    case T_INET: {
      char buf[64];
      if (n == 4) snprintf(buf, sizeof buf, "%u.%u.%u.%u", p[0], p[1], p[2], p[3]);
      else {
        std::string s;
        for (int i = 0; i < n; i += 2) {
          char b[8];
          snprintf(b, sizeof b, "%s%x", i ? ":" : "", (p[i] << 8) | p[i + 1]);
          s += b;
        }
        return py::str(s);
      }
      return py::str(buf);
    }
    case T_LIST:
    case T_SET: {
      int32_t k = r.i32();
      py::list out;
      for (int32_t i = 0; i < k; ++i) out.append(decode_nullable(r, t.sub.at(0)));
      return std::move(out);
    }
    case T_MAP: {
      int32_t k = r.i32();
      py::dict out;
      for (int32_t i = 0; i < k; ++i) {
        py::object key = decode_nullable(r, t.sub.at(0));
        out[key] = decode_nullable(r, t.sub.at(1));
      }
      return std::move(out);
    }
    case T_TUPLE: {
      py::tuple out(t.sub.size());
      for (size_t i = 0; i < t.sub.size(); ++i) out[i] = decode_nullable(r, t.sub[i]);
      return std::move(out);
    }
    default: return py::bytes(reinterpret_cast<const char*>(p), static_cast<size_t>(n));
  }
}

// ---------------------------------------------------------------- request encoders
void write_params(Writer& w, const py::handle& values, const std::vector<Type>& types, uint16_t consistency,
                  bool skip_metadata, int32_t page_size, const py::handle& paging_state, const py::handle& serial,
                  const py::handle& timestamp) {
  w.u16(consistency);
  uint8_t flags = 0;
  bool has_values = !values.is_none() && py::len(values) > 0;
  if (has_values) flags |= QF_VALUES;
  if (skip_metadata) flags |= QF_SKIP_METADATA;
  if (page_size > 0) flags |= QF_PAGE_SIZE;
  if (!paging_state.is_none()) flags |= QF_PAGING_STATE;
  if (!serial.is_none()) flags |= QF_SERIAL_CONSISTENCY;
  if (!timestamp.is_none()) flags |= QF_DEFAULT_TIMESTAMP;
  w.u8(flags);
  if (has_values) {
    py::sequence seq = py::reinterpret_borrow<py::sequence>(values);
    size_t n = seq.size();
    if (!types.empty() && types.size() != n)
      throw std::invalid_argument("expected " + std::to_string(types.size()) + " bind values, got " + std::to_string(n));
    w.u16(static_cast<uint16_t>(n));
    for (size_t i = 0; i < n; ++i) {
      py::object v = seq[i];
      write_value(w, v, types.empty() ? infer_type(v) : types[i]);
    }
  }
  if (page_size > 0) w.i32(page_size);
  if (!paging_state.is_none()) w.bytes(paging_state.cast<std::string>());
  if (!serial.is_none()) w.u16(serial.cast<uint16_t>());
  if (!timestamp.is_none()) w.i64(timestamp.cast<int64_t>());
}

py::bytes to_frame(int16_t stream, uint8_t op, const std::string& body) {
  std::string f = frame(VERSION_REQ, stream, op, body);
  return py::bytes(f);
}

py::bytes encode_startup(int16_t stream, const std::map<std::string, std::string>& opts) {
  Writer w;
  std::vector<std::pair<std::string, std::string>> m(opts.begin(), opts.end());
  w.string_map(m);
  return to_frame(stream, OP_STARTUP, w.buf);
}

py::bytes encode_options(int16_t stream) { return to_frame(stream, OP_OPTIONS, std::string()); }

py::bytes encode_auth_response(int16_t stream, const std::string& token) {
  Writer w;
  w.bytes(token);
  return to_frame(stream, OP_AUTH_RESPONSE, w.buf);
}

py::bytes encode_register(int16_t stream, const std::vector<std::string>& events) {
  Writer w;
  w.string_list(events);
  return to_frame(stream, OP_REGISTER, w.buf);
}

py::bytes encode_prepare(int16_t stream, const std::string& query) {
  Writer w;
  w.long_string(query);
  return to_frame(stream, OP_PREPARE, w.buf);
}

py::bytes encode_query(int16_t stream, const std::string& query, const py::object& values, const py::object& types,
                       uint16_t consistency, int32_t page_size, const py::object& paging_state, const py::object& serial,
                       const py::object& timestamp) {
  Writer w;
  w.buf.reserve(query.size() + 64);
  w.long_string(query);
  write_params(w, values, types_from_py(types), consistency, false, page_size, paging_state, serial, timestamp);
  return to_frame(stream, OP_QUERY, w.buf);
}

py::bytes encode_execute(int16_t stream, const std::string& qid, const py::object& values, const py::object& types,
                         uint16_t consistency, bool skip_metadata, int32_t page_size, const py::object& paging_state,
                         const py::object& serial, const py::object& timestamp) {
  Writer w;
  w.buf.reserve(256);
  w.short_bytes(qid);
  write_params(w, values, types_from_py(types), consistency, skip_metadata, page_size, paging_state, serial, timestamp);
  return to_frame(stream, OP_EXECUTE, w.buf);
}

// ---------------------------------------------------------------- EXECUTE fast path
// encode_execute_fast(stream, query_id: bytes, values: list|tuple, codes: bytes, consistency,
//                     skip_metadata, serial) -> bytes | NotImplemented
// The two statements of every decision (status read, owned-columns write) bind only scalar
// columns.  ``codes`` holds one CQL type id per bind marker (precomputed at prepare time);
// strings are written from CPython's cached UTF-8 buffer and the frame is built in one
// buffer (pybind's 10-argument dispatch, per-call type vector and three copies of the
// ~2 KB trace were ~2/3 of encode_execute's cost).  Anything outside the scalar set, or a
// value of an unexpected Python type, answers NotImplemented: the caller uses encode_execute.
namespace {

struct Buf {
  std::string s;
  void u8(uint8_t v) { s.push_back(static_cast<char>(v)); }
  void u16(uint16_t v) {
    char b[2] = {static_cast<char>(v >> 8), static_cast<char>(v)};
    s.append(b, 2);
  }
  void i32(int32_t v) {
    uint32_t u = static_cast<uint32_t>(v);
    char b[4] = {static_cast<char>(u >> 24), static_cast<char>(u >> 16), static_cast<char>(u >> 8), static_cast<char>(u)};
    s.append(b, 4);
  }
  void i64(int64_t v) {
    uint64_t u = static_cast<uint64_t>(v);
    char b[8];
    for (int i = 7; i >= 0; --i) {
      b[i] = static_cast<char>(u);
      u >>= 8;
    }
    s.append(b, 8);
  }
};

// 1 = written, 0 = not handled (caller falls back), -1 = Python error set
int fast_value(Buf& w, PyObject* v, uint8_t code) {
  if (v == Py_None) {
    w.i32(-1);
    return 1;
  }
  switch (code) {
    case T_VARCHAR:
    case T_ASCII: {
      Py_ssize_t n;
      const char* p;
      if (PyUnicode_Check(v)) {
        p = PyUnicode_AsUTF8AndSize(v, &n);
        if (!p) return -1;
      } else if (PyBytes_Check(v)) {
        p = PyBytes_AS_STRING(v);
        n = PyBytes_GET_SIZE(v);
      } else {
        return 0;
      }
      w.i32(static_cast<int32_t>(n));
      w.s.append(p, static_cast<size_t>(n));
      return 1;
    }
    case T_BLOB:
      if (!PyBytes_Check(v)) return 0;
      w.i32(static_cast<int32_t>(PyBytes_GET_SIZE(v)));
      w.s.append(PyBytes_AS_STRING(v), static_cast<size_t>(PyBytes_GET_SIZE(v)));
      return 1;
    case T_BIGINT:
    case T_COUNTER:
    case T_TIME:
    case T_INT:
    case T_TIMESTAMP: {
      int64_t x;
      if (PyLong_Check(v) && !PyBool_Check(v)) {
        x = PyLong_AsLongLong(v);
        if (x == -1 && PyErr_Occurred()) return -1;
      } else if (code == T_TIMESTAMP && PyFloat_Check(v)) {
        x = static_cast<int64_t>(std::llround(PyFloat_AS_DOUBLE(v) * 1000.0));
      } else if (code == T_TIMESTAMP) {
        PyObject* r = PyObject_CallMethod(v, "timestamp", nullptr);  // datetime
        if (!r) {
          PyErr_Clear();
          return 0;
        }
        double s = PyFloat_AsDouble(r);
        Py_DECREF(r);
        if (s == -1.0 && PyErr_Occurred()) return -1;
        x = static_cast<int64_t>(std::llround(s * 1000.0));
      } else {
        return 0;
      }
      if (code == T_INT) {
        if (x < INT32_MIN || x > INT32_MAX) return 0;
        w.i32(4);
        w.i32(static_cast<int32_t>(x));
      } else {
        w.i32(8);
        w.i64(x);
      }
      return 1;
    }
    case T_BOOLEAN: {
      if (!PyBool_Check(v)) return 0;
      w.i32(1);
      w.u8(v == Py_True ? 1 : 0);
      return 1;
    }
    case T_DOUBLE: {
      if (!PyFloat_Check(v) && !PyLong_Check(v)) return 0;
      double d = PyFloat_AsDouble(v);
      if (d == -1.0 && PyErr_Occurred()) return -1;
      int64_t bits;
      memcpy(&bits, &d, 8);
      w.i32(8);
      w.i64(bits);
      return 1;
    }
    default: return 0;
  }
}

PyObject* encode_execute_fast(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 7) {
    PyErr_SetString(PyExc_TypeError, "encode_execute_fast(stream, query_id, values, codes, consistency, skip, serial)");
    return nullptr;
  }
  long stream = PyLong_AsLong(args[0]);
  if (stream == -1 && PyErr_Occurred()) return nullptr;
  PyObject* qid = args[1];
  PyObject* values = args[2];
  PyObject* codes = args[3];
  long consistency = PyLong_AsLong(args[4]);
  if (consistency == -1 && PyErr_Occurred()) return nullptr;
  int skip = PyObject_IsTrue(args[5]);
  if (skip < 0) return nullptr;
  PyObject* serial = args[6];
  if (!PyBytes_Check(qid) || !PyBytes_Check(codes) || !(PyList_Check(values) || PyTuple_Check(values))) Py_RETURN_NOTIMPLEMENTED;
  Py_ssize_t n = PySequence_Fast_GET_SIZE(values);
  if (n != PyBytes_GET_SIZE(codes) || n > 0xFFFF) Py_RETURN_NOTIMPLEMENTED;
  long serial_cl = 0;
  if (serial != Py_None) {
    serial_cl = PyLong_AsLong(serial);
    if (serial_cl == -1 && PyErr_Occurred()) return nullptr;
  }
  PyObject** items = PySequence_Fast_ITEMS(values);
  const uint8_t* cd = reinterpret_cast<const uint8_t*>(PyBytes_AS_STRING(codes));
  Buf w;
  size_t guess = HEADER_LEN + 2 + static_cast<size_t>(PyBytes_GET_SIZE(qid)) + 8 + 16 * static_cast<size_t>(n);
  for (Py_ssize_t i = 0; i < n; ++i)
    if (PyUnicode_Check(items[i])) guess += static_cast<size_t>(PyUnicode_GET_LENGTH(items[i]));
  w.s.reserve(guess + 64);
  w.s.append(HEADER_LEN, '\0');  // patched below
  w.u16(static_cast<uint16_t>(PyBytes_GET_SIZE(qid)));
  w.s.append(PyBytes_AS_STRING(qid), static_cast<size_t>(PyBytes_GET_SIZE(qid)));
  w.u16(static_cast<uint16_t>(consistency));
  uint8_t flags = 0;
  if (n > 0) flags |= QF_VALUES;
  if (skip) flags |= QF_SKIP_METADATA;
  if (serial != Py_None) flags |= QF_SERIAL_CONSISTENCY;
  w.u8(flags);
  if (n > 0) {
    w.u16(static_cast<uint16_t>(n));
    for (Py_ssize_t i = 0; i < n; ++i) {
      int rc = fast_value(w, items[i], cd[i]);
      if (rc < 0) return nullptr;
      if (rc == 0) Py_RETURN_NOTIMPLEMENTED;
    }
  }
  if (serial != Py_None) w.u16(static_cast<uint16_t>(serial_cl));
  std::string head;
  write_header(head, VERSION_REQ, 0, static_cast<int16_t>(stream), OP_EXECUTE,
               static_cast<uint32_t>(w.s.size() - HEADER_LEN));
  memcpy(&w.s[0], head.data(), HEADER_LEN);
  return PyBytes_FromStringAndSize(w.s.data(), static_cast<Py_ssize_t>(w.s.size()));
}

PyMethodDef g_fast_defs[] = {
    {"encode_execute_fast", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(encode_execute_fast)),
     METH_FASTCALL, "EXECUTE frame for scalar bind values (NotImplemented: use encode_execute)"},
    {nullptr, nullptr, 0, nullptr}};

}  // namespace

// statements: iterable of (kind, query_or_id, values, types) with kind 0 = query string, 1 = prepared id.
py::bytes encode_batch(int16_t stream, uint8_t batch_type, const py::object& statements, uint16_t consistency,
                       const py::object& serial, const py::object& timestamp) {
  Writer w;
  w.u8(batch_type);
  py::list st = py::list(statements);
  w.u16(static_cast<uint16_t>(st.size()));
  for (auto item : st) {
    py::tuple t = py::reinterpret_borrow<py::tuple>(item);
    int kind = t[0].cast<int>();
    w.u8(static_cast<uint8_t>(kind));
    if (kind == 0) w.long_string(t[1].cast<std::string>());
    else w.short_bytes(t[1].cast<std::string>());
    py::object values = t[2];
    std::vector<Type> types = types_from_py(t[3]);
    size_t n = values.is_none() ? 0 : py::len(values);
    w.u16(static_cast<uint16_t>(n));
    if (n) {
      py::sequence seq = py::reinterpret_borrow<py::sequence>(values);
      for (size_t i = 0; i < n; ++i) {
        py::object v = seq[i];
        write_value(w, v, types.empty() ? infer_type(v) : types.at(i));
      }
    }
  }
  w.u16(consistency);
  uint8_t flags = 0;
  if (!serial.is_none()) flags |= QF_SERIAL_CONSISTENCY;
  if (!timestamp.is_none()) flags |= QF_DEFAULT_TIMESTAMP;
  w.u8(flags);
  if (!serial.is_none()) w.u16(serial.cast<uint16_t>());
  if (!timestamp.is_none()) w.i64(timestamp.cast<int64_t>());
  return to_frame(stream, OP_BATCH, w.buf);
}

// ---------------------------------------------------------------- response decoding
std::vector<ColSpec> read_colspecs(Reader& r, int32_t flags, int32_t count) {
  std::vector<ColSpec> cols;
  std::string gks, gtable;
  if (flags & MF_GLOBAL_TABLES_SPEC) {
    gks = r.string();
    gtable = r.string();
  }
  for (int32_t i = 0; i < count; ++i) {
    ColSpec c;
    if (flags & MF_GLOBAL_TABLES_SPEC) {
      c.keyspace = gks;
      c.table = gtable;
    } else {
      c.keyspace = r.string();
      c.table = r.string();
    }
    c.name = r.string();
    c.type = r.type();
    cols.push_back(std::move(c));
  }
  return cols;
}

py::object decode_rows(Reader& r, const std::vector<Type>* hint) {
  int32_t flags = r.i32();
  int32_t ncols = r.i32();
  py::object paging = py::none();
  if (flags & MF_HAS_MORE_PAGES) {
    const uint8_t* d;
    int32_t n;
    if (r.bytes(d, n)) paging = py::bytes(reinterpret_cast<const char*>(d), static_cast<size_t>(n));
  }
  std::vector<Type> types;
  py::tuple names;
  if (flags & MF_NO_METADATA) {
    if (!hint) throw ProtocolError("rows without metadata and no type hint");
    types = *hint;
    names = py::tuple(0);
  } else {
    auto cols = read_colspecs(r, flags, ncols);
    names = py::tuple(cols.size());
    for (size_t i = 0; i < cols.size(); ++i) {
      names[i] = py::str(cols[i].name);
      types.push_back(cols[i].type);
    }
  }
  if (static_cast<int32_t>(types.size()) != ncols) throw ProtocolError("column count mismatch");
  int32_t nrows = r.i32();
  py::list rows;
  for (int32_t i = 0; i < nrows; ++i) {
    py::tuple row(ncols);
    for (int32_t c = 0; c < ncols; ++c) row[c] = decode_nullable(r, types[c]);
    rows.append(row);
  }
  py::list tl;
  for (auto& t : types) tl.append(type_to_py(t));
  return py::make_tuple("rows", names, rows, paging, tl);
}

py::object decode_result(Reader& r, const std::vector<Type>* hint) {
  int32_t kind = r.i32();
  switch (kind) {
    case RK_VOID: return py::make_tuple("void");
    case RK_ROWS: return decode_rows(r, hint);
    case RK_SET_KEYSPACE: return py::make_tuple("set_keyspace", r.string());
    case RK_PREPARED: {
      std::string id = r.short_bytes();
      int32_t flags = r.i32();
      int32_t ncols = r.i32();
      int32_t npk = r.i32();
      py::list pk;
      for (int32_t i = 0; i < npk; ++i) pk.append(r.u16());
      auto bind = read_colspecs(r, flags, ncols);
      py::list bl;
      for (auto& c : bind) bl.append(py::make_tuple(c.keyspace, c.table, c.name, type_to_py(c.type)));
      int32_t rflags = r.i32();
      int32_t rcols = r.i32();
      py::object rl = py::none();
      if (!(rflags & MF_NO_METADATA)) {
        if (rflags & MF_HAS_MORE_PAGES) {
          const uint8_t* d;
          int32_t n;
          r.bytes(d, n);
        }
        auto res = read_colspecs(r, rflags, rcols);
        py::list l;
        for (auto& c : res) l.append(py::make_tuple(c.name, type_to_py(c.type)));
        rl = l;
      }
      return py::make_tuple("prepared", py::bytes(id), bl, pk, rl);
    }
    case RK_SCHEMA_CHANGE: {
      std::string change = r.string();
      std::string target = r.string();
      std::string ks = r.string();
      std::string name = target == "KEYSPACE" ? std::string() : r.string();
      return py::make_tuple("schema_change", change, target, ks, name);
    }
    default: throw ProtocolError("unknown result kind " + std::to_string(kind));
  }
}

py::object decode_error(Reader& r) {
  int32_t code = r.i32();
  std::string msg = r.string();
  py::dict extra;
  try {
    switch (code) {
      case ERR_UNAVAILABLE:
        extra["consistency"] = r.u16();
        extra["required"] = r.i32();
        extra["alive"] = r.i32();
        break;
      case ERR_WRITE_TIMEOUT:
        extra["consistency"] = r.u16();
        extra["received"] = r.i32();
        extra["block_for"] = r.i32();
        extra["write_type"] = r.string();
        break;
      case ERR_READ_TIMEOUT:
        extra["consistency"] = r.u16();
        extra["received"] = r.i32();
        extra["block_for"] = r.i32();
        extra["data_present"] = r.u8() != 0;
        break;
      case ERR_ALREADY_EXISTS:
        extra["keyspace"] = r.string();
        extra["table"] = r.string();
        break;
      case ERR_UNPREPARED: extra["id"] = py::bytes(r.short_bytes()); break;
      default: break;
    }
  } catch (const ProtocolError&) {
    // extra fields are advisory
  }
  return py::make_tuple("error", code, msg, extra);
}

py::object decode_body(uint8_t opcode, uint8_t flags, const uint8_t* body, size_t len, const std::vector<Type>* hint) {
  Reader r(body, len);
  if (flags & 0x02) r.raw(16);  // tracing id
  if (flags & 0x08) r.string_list();  // warnings
  if (flags & 0x04) {  // custom payload: [bytes map]
    uint16_t k = r.u16();
    for (uint16_t i = 0; i < k; ++i) {
      r.string();
      const uint8_t* d;
      int32_t n;
      r.bytes(d, n);
    }
  }
  switch (opcode) {
    case OP_READY: return py::make_tuple("ready");
    case OP_AUTHENTICATE: return py::make_tuple("authenticate", r.string());
    case OP_AUTH_SUCCESS:
    case OP_AUTH_CHALLENGE: {
      const uint8_t* d;
      int32_t n;
      py::object tok = py::none();
      if (r.remaining() >= 4 && r.bytes(d, n)) tok = py::bytes(reinterpret_cast<const char*>(d), static_cast<size_t>(n));
      return py::make_tuple(opcode == OP_AUTH_SUCCESS ? "auth_success" : "auth_challenge", tok);
    }
    case OP_SUPPORTED: {
      auto mm = r.string_multimap();
      py::dict d;
      for (auto& kv : mm) d[py::str(kv.first)] = kv.second;
      return py::make_tuple("supported", d);
    }
    case OP_ERROR: return decode_error(r);
    case OP_RESULT: return decode_result(r, hint);
    case OP_EVENT: {
      std::string type = r.string();
      if (type == "TOPOLOGY_CHANGE" || type == "STATUS_CHANGE") {
        std::string change = r.string();
        uint8_t alen = r.u8();
        std::string addr = r.raw(alen);
        int32_t port = r.i32();
        std::string a;
        if (alen == 4) {
          char b[32];
          snprintf(b, sizeof b, "%u.%u.%u.%u", uint8_t(addr[0]), uint8_t(addr[1]), uint8_t(addr[2]), uint8_t(addr[3]));
          a = b;
        }
        return py::make_tuple("event", type, change, a, port);
      }
      return py::make_tuple("event", type);
    }
    default: return py::make_tuple("unknown", opcode);
  }
}

// Incremental response reader: feed() bytes, get [(stream, opcode, decoded), ...].
class FrameReader {
 public:
  py::list feed(const py::bytes& data) {
    char* buf;
    Py_ssize_t n;
    PyBytes_AsStringAndSize(data.ptr(), &buf, &n);
    split_.feed(buf, static_cast<size_t>(n));
    py::list out;
    FrameHeader h;
    const uint8_t* body;
    while (split_.next(h, body)) {
      const std::vector<Type>* hint = nullptr;
      auto it = hints_.find(h.stream);
      if (it != hints_.end()) hint = &it->second;
      py::object dec = decode_body(h.opcode, h.flags, body, h.length, hint);
      if (it != hints_.end()) hints_.erase(it);
      out.append(py::make_tuple(h.stream, h.opcode, dec));
      ++frames_;
    }
    return out;
  }
  // Column types for a skip-metadata EXECUTE response on `stream`.
  void expect(int16_t stream, const py::object& types) { hints_[stream] = types_from_py(types); }
  void forget(int16_t stream) { hints_.erase(stream); }
  uint64_t frames() const { return frames_; }
  size_t buffered() const { return split_.pending.size() - split_.start; }

 private:
  FrameSplitter split_;
  std::unordered_map<int16_t, std::vector<Type>> hints_;
  uint64_t frames_ = 0;
};

int64_t token_of(const py::bytes& key) {
  char* buf;
  Py_ssize_t n;
  PyBytes_AsStringAndSize(key.ptr(), &buf, &n);
  return murmur3_token(reinterpret_cast<const uint8_t*>(buf), static_cast<size_t>(n));
}

int64_t h1_of(const py::bytes& key) {
  char* buf;
  Py_ssize_t n;
  PyBytes_AsStringAndSize(key.ptr(), &buf, &n);
  return murmur3_h1(reinterpret_cast<const uint8_t*>(buf), static_cast<size_t>(n));
}

std::string component_bytes(const py::handle& h) {
  if (py::isinstance<py::bytes>(h)) return h.cast<std::string>();
  return py::str(h).cast<std::string>();
}

py::bytes routing_key(const py::iterable& parts) {
  std::vector<std::string> v;
  for (auto p : parts) v.push_back(component_bytes(p));
  return py::bytes(composite_routing_key(v));
}

int64_t token_for(const py::iterable& parts) {
  std::vector<std::string> v;
  for (auto p : parts) v.push_back(component_bytes(p));
  std::string k = composite_routing_key(v);
  return murmur3_token(reinterpret_cast<const uint8_t*>(k.data()), k.size());
}

py::object decode_value_py(const py::bytes& data, const py::object& type) {
  char* buf;
  Py_ssize_t n;
  PyBytes_AsStringAndSize(data.ptr(), &buf, &n);
  return decode_value(reinterpret_cast<const uint8_t*>(buf), static_cast<int32_t>(n), type_from_py(type));
}

py::bytes serialize_py(const py::object& v, const py::object& type) { return py::bytes(serialize(v, type_from_py(type))); }

}  // namespace

PYBIND11_MODULE(_cql_native, m) {
  m.doc() = "CQL native protocol v4 codec + Cassandra Murmur3 tokens (native core of the checkpoint store client)";
  m.attr("HEADER_LEN") = HEADER_LEN;
  m.def("set_timestamp_factory", [](py::object f) { g_ts_factory = std::move(f); });
  {
    PyObject* f = PyCFunction_NewEx(&g_fast_defs[0], nullptr, m.attr("__name__").ptr());
    if (!f) throw py::error_already_set();
    m.add_object("encode_execute_fast", py::reinterpret_steal<py::object>(f));
  }
  m.def("murmur3_token", &token_of, "Murmur3Partitioner token of a routing key");
  m.def("murmur3_h1", &h1_of, "Raw MurmurHash3_x64_128 h1 (Cassandra variant, no normalisation)");
  m.def("routing_key", &routing_key, "Composite routing key of partition-key components");
  m.def("token_for", &token_for, "Token of a (possibly composite) partition key");
  m.def("serialize", &serialize_py, py::arg("value"), py::arg("type"));
  m.def("deserialize", &decode_value_py, py::arg("data"), py::arg("type"));
  m.def("encode_startup", &encode_startup);
  m.def("encode_options", &encode_options);
  m.def("encode_auth_response", &encode_auth_response);
  m.def("encode_register", &encode_register);
  m.def("encode_prepare", &encode_prepare);
  m.def("encode_query", &encode_query, py::arg("stream"), py::arg("query"), py::arg("values") = py::none(),
        py::arg("types") = py::none(), py::arg("consistency") = static_cast<uint16_t>(CL_LOCAL_QUORUM),
        py::arg("page_size") = -1, py::arg("paging_state") = py::none(), py::arg("serial") = py::none(),
        py::arg("timestamp") = py::none());
  m.def("encode_execute", &encode_execute, py::arg("stream"), py::arg("query_id"), py::arg("values") = py::none(),
        py::arg("types") = py::none(), py::arg("consistency") = static_cast<uint16_t>(CL_LOCAL_QUORUM),
        py::arg("skip_metadata") = false, py::arg("page_size") = -1, py::arg("paging_state") = py::none(),
        py::arg("serial") = py::none(), py::arg("timestamp") = py::none());
  m.def("encode_batch", &encode_batch, py::arg("stream"), py::arg("batch_type"), py::arg("statements"),
        py::arg("consistency") = static_cast<uint16_t>(CL_LOCAL_QUORUM), py::arg("serial") = py::none(),
        py::arg("timestamp") = py::none());
  m.def("decode_body", [](uint8_t opcode, uint8_t flags, const py::bytes& body, const py::object& hint) {
    char* buf;
    Py_ssize_t n;
    PyBytes_AsStringAndSize(body.ptr(), &buf, &n);
    std::vector<Type> h = types_from_py(hint);
    return decode_body(opcode, flags, reinterpret_cast<const uint8_t*>(buf), static_cast<size_t>(n), hint.is_none() ? nullptr : &h);
  }, py::arg("opcode"), py::arg("flags"), py::arg("body"), py::arg("hint") = py::none());
  py::class_<FrameReader>(m, "FrameReader")
      .def(py::init<>())
      .def("feed", &FrameReader::feed)
      .def("expect", &FrameReader::expect)
      .def("forget", &FrameReader::forget)
      .def_property_readonly("frames", &FrameReader::frames)
      .def_property_readonly("buffered", &FrameReader::buffered);
  py::register_exception<ProtocolError>(m, "ProtocolError", PyExc_ValueError);
}
