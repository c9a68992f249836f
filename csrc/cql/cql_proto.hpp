// CQL native protocol v4: framing, primitive notation, type options, value
// (de)serialisation and Cassandra's Murmur3 partitioner token.
//
// The reference talks CQL through gocql/gocqlx inside nexus-core's CqlStore
// (ReadCheckpoint / UpsertCheckpoint at /root/reference/services/supervisor.go:264,301;
// driver pinned at /root/reference/go.mod:66,93).  No CQL driver is available
// offline here, so the protocol is implemented natively: this header is shared by
// the Python extension (_cql_native, the supervisor's client codec) and the
// native in-memory CQL server used by tests and benchmarks (nexus-cqlsrv).
#pragma once

#include <cstdint>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace nxcql {

enum Opcode : uint8_t {
  OP_ERROR = 0x00,
  OP_STARTUP = 0x01,
  OP_READY = 0x02,
  OP_AUTHENTICATE = 0x03,
  OP_OPTIONS = 0x05,
  OP_SUPPORTED = 0x06,
  OP_QUERY = 0x07,
  OP_RESULT = 0x08,
  OP_PREPARE = 0x09,
  OP_EXECUTE = 0x0A,
  OP_REGISTER = 0x0B,
  OP_EVENT = 0x0C,
  OP_BATCH = 0x0D,
  OP_AUTH_CHALLENGE = 0x0E,
  OP_AUTH_RESPONSE = 0x0F,
  OP_AUTH_SUCCESS = 0x10,
};

enum ResultKind : int32_t { RK_VOID = 1, RK_ROWS = 2, RK_SET_KEYSPACE = 3, RK_PREPARED = 4, RK_SCHEMA_CHANGE = 5 };

enum ErrorCode : int32_t {
  ERR_SERVER = 0x0000,
  ERR_PROTOCOL = 0x000A,
  ERR_BAD_CREDENTIALS = 0x0100,
  ERR_UNAVAILABLE = 0x1000,
  ERR_OVERLOADED = 0x1001,
  ERR_IS_BOOTSTRAPPING = 0x1002,
  ERR_TRUNCATE = 0x1003,
  ERR_WRITE_TIMEOUT = 0x1100,
  ERR_READ_TIMEOUT = 0x1200,
  ERR_READ_FAILURE = 0x1300,
  ERR_FUNCTION_FAILURE = 0x1400,
  ERR_WRITE_FAILURE = 0x1500,
  ERR_SYNTAX = 0x2000,
  ERR_UNAUTHORIZED = 0x2100,
  ERR_INVALID = 0x2200,
  ERR_CONFIG = 0x2300,
  ERR_ALREADY_EXISTS = 0x2400,
  ERR_UNPREPARED = 0x2500,
};

// Query-parameter flags (v4).
enum QFlag : uint8_t {
  QF_VALUES = 0x01,
  QF_SKIP_METADATA = 0x02,
  QF_PAGE_SIZE = 0x04,
  QF_PAGING_STATE = 0x08,
  QF_SERIAL_CONSISTENCY = 0x10,
  QF_DEFAULT_TIMESTAMP = 0x20,
  QF_NAMES = 0x40,
};

// Rows-metadata flags.
enum MFlag : int32_t { MF_GLOBAL_TABLES_SPEC = 0x0001, MF_HAS_MORE_PAGES = 0x0002, MF_NO_METADATA = 0x0004 };

enum TypeId : uint16_t {
  T_CUSTOM = 0x0000,
  T_ASCII = 0x0001,
  T_BIGINT = 0x0002,
  T_BLOB = 0x0003,
  T_BOOLEAN = 0x0004,
  T_COUNTER = 0x0005,
  T_DECIMAL = 0x0006,
  T_DOUBLE = 0x0007,
  T_FLOAT = 0x0008,
  T_INT = 0x0009,
  T_TIMESTAMP = 0x000B,
  T_UUID = 0x000C,
  T_VARCHAR = 0x000D,
  T_VARINT = 0x000E,
  T_TIMEUUID = 0x000F,
  T_INET = 0x0010,
  T_DATE = 0x0011,
  T_TIME = 0x0012,
  T_SMALLINT = 0x0013,
  T_TINYINT = 0x0014,
  T_LIST = 0x0020,
  T_MAP = 0x0021,
  T_SET = 0x0022,
  T_TUPLE = 0x0031,
};

enum Consistency : uint16_t {
  CL_ANY = 0,
  CL_ONE = 1,
  CL_TWO = 2,
  CL_THREE = 3,
  CL_QUORUM = 4,
  CL_ALL = 5,
  CL_LOCAL_QUORUM = 6,
  CL_EACH_QUORUM = 7,
  CL_SERIAL = 8,
  CL_LOCAL_SERIAL = 9,
  CL_LOCAL_ONE = 10,
};

constexpr size_t HEADER_LEN = 9;
constexpr uint8_t VERSION_REQ = 0x04;
constexpr uint8_t VERSION_RESP = 0x84;
constexpr uint32_t MAX_FRAME = 256u << 20;

struct ProtocolError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// A column type option ([option] notation); collections nest.
struct Type {
  uint16_t id = T_VARCHAR;
  std::string custom;
  std::vector<Type> sub;
};

struct ColSpec {
  std::string keyspace, table, name;
  Type type;
};

// ------------------------------------------------------------------ writer
struct Writer {
  std::string buf;

  void u8(uint8_t v) { buf.push_back(static_cast<char>(v)); }
  void u16(uint16_t v) {
    char b[2] = {static_cast<char>(v >> 8), static_cast<char>(v)};
    buf.append(b, 2);
  }
  void i32(int32_t v) {
    uint32_t u = static_cast<uint32_t>(v);
    char b[4] = {static_cast<char>(u >> 24), static_cast<char>(u >> 16), static_cast<char>(u >> 8), static_cast<char>(u)};
    buf.append(b, 4);
  }
  void i64(int64_t v) {
    uint64_t u = static_cast<uint64_t>(v);
    char b[8];
    for (int i = 7; i >= 0; --i) {
      b[i] = static_cast<char>(u);
      u >>= 8;
    }
    buf.append(b, 8);
  }
  void string(const std::string& s) {
    if (s.size() > 0xFFFF) throw ProtocolError("[string] too long");
    u16(static_cast<uint16_t>(s.size()));
    buf.append(s);
  }
  void long_string(const std::string& s) {
    i32(static_cast<int32_t>(s.size()));
    buf.append(s);
  }
  void bytes(const char* p, size_t n) {
    i32(static_cast<int32_t>(n));
    buf.append(p, n);
  }
  void bytes(const std::string& s) { bytes(s.data(), s.size()); }
  void null_bytes() { i32(-1); }
  void short_bytes(const std::string& s) {
    u16(static_cast<uint16_t>(s.size()));
    buf.append(s);
  }
  void string_map(const std::vector<std::pair<std::string, std::string>>& m) {
    u16(static_cast<uint16_t>(m.size()));
    for (auto& kv : m) {
      string(kv.first);
      string(kv.second);
    }
  }
  void string_list(const std::vector<std::string>& l) {
    u16(static_cast<uint16_t>(l.size()));
    for (auto& s : l) string(s);
  }
  void type(const Type& t) {
    u16(t.id);
    if (t.id == T_CUSTOM) string(t.custom);
    else if (t.id == T_LIST || t.id == T_SET) type(t.sub.at(0));
    else if (t.id == T_MAP) {
      type(t.sub.at(0));
      type(t.sub.at(1));
    } else if (t.id == T_TUPLE) {
      u16(static_cast<uint16_t>(t.sub.size()));
      for (auto& s : t.sub) type(s);
    }
  }
};

// ------------------------------------------------------------------ reader
struct Reader {
  const uint8_t* p;
  size_t n;
  size_t off = 0;

  Reader(const void* data, size_t len) : p(static_cast<const uint8_t*>(data)), n(len) {}

  void need(size_t k) const {
    if (off + k > n) throw ProtocolError("truncated frame body");
  }
  size_t remaining() const { return n - off; }
  uint8_t u8() {
    need(1);
    return p[off++];
  }
  uint16_t u16() {
    need(2);
    uint16_t v = static_cast<uint16_t>((p[off] << 8) | p[off + 1]);
    off += 2;
    return v;
  }
  int32_t i32() {
    need(4);
    uint32_t v = (uint32_t(p[off]) << 24) | (uint32_t(p[off + 1]) << 16) | (uint32_t(p[off + 2]) << 8) | uint32_t(p[off + 3]);
    off += 4;
    return static_cast<int32_t>(v);
  }
  int64_t i64() {
    need(8);
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v = (v << 8) | p[off + i];
    off += 8;
    return static_cast<int64_t>(v);
  }
  std::string raw(size_t k) {
    need(k);
    std::string s(reinterpret_cast<const char*>(p + off), k);
    off += k;
    return s;
  }
  std::string string() { return raw(u16()); }
  std::string long_string() {
    int32_t k = i32();
    if (k < 0) throw ProtocolError("negative [long string] length");
    return raw(static_cast<size_t>(k));
  }
  // [bytes]: returns false for null (negative length).
  bool bytes(const uint8_t*& data, int32_t& len) {
    len = i32();
    if (len < 0) {
      data = nullptr;
      return false;
    }
    need(static_cast<size_t>(len));
    data = p + off;
    off += static_cast<size_t>(len);
    return true;
  }
  std::string short_bytes() { return raw(u16()); }
  std::vector<std::pair<std::string, std::string>> string_map() {
    std::vector<std::pair<std::string, std::string>> m;
    uint16_t k = u16();
    for (uint16_t i = 0; i < k; ++i) {
      std::string a = string();
      std::string b = string();
      m.emplace_back(std::move(a), std::move(b));
    }
    return m;
  }
  std::vector<std::string> string_list() {
    std::vector<std::string> l;
    uint16_t k = u16();
    for (uint16_t i = 0; i < k; ++i) l.push_back(string());
    return l;
  }
  std::map<std::string, std::vector<std::string>> string_multimap() {
    std::map<std::string, std::vector<std::string>> m;
    uint16_t k = u16();
    for (uint16_t i = 0; i < k; ++i) {
      std::string key = string();
      m[key] = string_list();
    }
    return m;
  }
  Type type() {
    Type t;
    t.id = u16();
    if (t.id == T_CUSTOM) t.custom = string();
    else if (t.id == T_LIST || t.id == T_SET) t.sub.push_back(type());
    else if (t.id == T_MAP) {
      t.sub.push_back(type());
      t.sub.push_back(type());
    } else if (t.id == 0x0030) {
      throw ProtocolError("UDT columns are not supported");
    } else if (t.id == T_TUPLE) {
      uint16_t k = u16();
      for (uint16_t i = 0; i < k; ++i) t.sub.push_back(type());
    }
    return t;
  }
};

// ------------------------------------------------------------------ frames
struct FrameHeader {
  uint8_t version = 0, flags = 0, opcode = 0;
  int16_t stream = 0;
  uint32_t length = 0;
};

inline FrameHeader parse_header(const uint8_t* h) {
  FrameHeader f;
  f.version = h[0];
  f.flags = h[1];
  f.stream = static_cast<int16_t>((h[2] << 8) | h[3]);
  f.opcode = h[4];
  f.length = (uint32_t(h[5]) << 24) | (uint32_t(h[6]) << 16) | (uint32_t(h[7]) << 8) | uint32_t(h[8]);
  return f;
}

inline void write_header(std::string& out, uint8_t version, uint8_t flags, int16_t stream, uint8_t opcode, uint32_t len) {
  char h[HEADER_LEN] = {static_cast<char>(version),
                        static_cast<char>(flags),
                        static_cast<char>(static_cast<uint16_t>(stream) >> 8),
                        static_cast<char>(stream),
                        static_cast<char>(opcode),
                        static_cast<char>(len >> 24),
                        static_cast<char>(len >> 16),
                        static_cast<char>(len >> 8),
                        static_cast<char>(len)};
  out.append(h, HEADER_LEN);
}

inline std::string frame(uint8_t version, int16_t stream, uint8_t opcode, const std::string& body, uint8_t flags = 0) {
  std::string out;
  out.reserve(HEADER_LEN + body.size());
  write_header(out, version, flags, stream, opcode, static_cast<uint32_t>(body.size()));
  out.append(body);
  return out;
}

// Incremental frame splitter for a byte stream.
struct FrameSplitter {
  std::string pending;
  size_t start = 0;

  void feed(const char* data, size_t n) {
    if (start > 0 && start == pending.size()) {
      pending.clear();
      start = 0;
    }
    pending.append(data, n);
  }
  // Returns true and fills hdr/body pointers when a whole frame is available.
  bool next(FrameHeader& hdr, const uint8_t*& body) {
    size_t avail = pending.size() - start;
    if (avail < HEADER_LEN) {
      compact();
      return false;
    }
    const uint8_t* h = reinterpret_cast<const uint8_t*>(pending.data() + start);
    hdr = parse_header(h);
    if (hdr.length > MAX_FRAME) throw ProtocolError("frame too large");
    if (avail < HEADER_LEN + hdr.length) {
      compact();
      return false;
    }
    body = h + HEADER_LEN;
    start += HEADER_LEN + hdr.length;
    return true;
  }
  void compact() {
    if (start > (1 << 16) || (start > 0 && start * 2 > pending.size())) {
      pending.erase(0, start);
      start = 0;
    }
  }
};

// ------------------------------------------------------------------ murmur3 (Cassandra variant)
inline uint64_t rotl64(uint64_t v, int r) { return (v << r) | (v >> (64 - r)); }
inline uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

// MurmurHash3_x64_128 with seed 0, returning h1 — as Cassandra's Murmur3Partitioner,
// including its quirk of sign-extending the tail bytes (Java `byte` is signed).
inline int64_t murmur3_h1(const uint8_t* key, size_t len) {
  const uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
  uint64_t h1 = 0, h2 = 0;
  const size_t nblocks = len / 16;
  auto block = [&](size_t off) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; --i) v = (v << 8) | key[off + i];
    return v;
  };
  for (size_t i = 0; i < nblocks; ++i) {
    uint64_t k1 = block(i * 16), k2 = block(i * 16 + 8);
    k1 *= c1;
    k1 = rotl64(k1, 31);
    k1 *= c2;
    h1 ^= k1;
    h1 = rotl64(h1, 27);
    h1 += h2;
    h1 = h1 * 5 + 0x52dce729;
    k2 *= c2;
    k2 = rotl64(k2, 33);
    k2 *= c1;
    h2 ^= k2;
    h2 = rotl64(h2, 31);
    h2 += h1;
    h2 = h2 * 5 + 0x38495ab5;
  }
  const uint8_t* tail = key + nblocks * 16;
  auto sb = [&](size_t i) { return static_cast<uint64_t>(static_cast<int64_t>(static_cast<int8_t>(tail[i]))); };
  uint64_t k1 = 0, k2 = 0;
  switch (len & 15) {
    case 15: k2 ^= sb(14) << 48; [[fallthrough]];
    case 14: k2 ^= sb(13) << 40; [[fallthrough]];
    case 13: k2 ^= sb(12) << 32; [[fallthrough]];
    case 12: k2 ^= sb(11) << 24; [[fallthrough]];
    case 11: k2 ^= sb(10) << 16; [[fallthrough]];
    case 10: k2 ^= sb(9) << 8; [[fallthrough]];
    case 9:
      k2 ^= sb(8);
      k2 *= c2;
      k2 = rotl64(k2, 33);
      k2 *= c1;
      h2 ^= k2;
      [[fallthrough]];
    case 8: k1 ^= sb(7) << 56; [[fallthrough]];
    case 7: k1 ^= sb(6) << 48; [[fallthrough]];
    case 6: k1 ^= sb(5) << 40; [[fallthrough]];
    case 5: k1 ^= sb(4) << 32; [[fallthrough]];
    case 4: k1 ^= sb(3) << 24; [[fallthrough]];
    case 3: k1 ^= sb(2) << 16; [[fallthrough]];
    case 2: k1 ^= sb(1) << 8; [[fallthrough]];
    case 1:
      k1 ^= sb(0);
      k1 *= c1;
      k1 = rotl64(k1, 31);
      k1 *= c2;
      h1 ^= k1;
      break;
    default: break;
  }
  h1 ^= static_cast<uint64_t>(len);
  h2 ^= static_cast<uint64_t>(len);
  h1 += h2;
  h2 += h1;
  h1 = fmix64(h1);
  h2 = fmix64(h2);
  h1 += h2;
  return static_cast<int64_t>(h1);
}

// Murmur3Partitioner token: INT64_MIN is reserved (minimum token) and maps to INT64_MAX.
inline int64_t murmur3_token(const uint8_t* key, size_t len) {
  int64_t h = murmur3_h1(key, len);
  return h == INT64_MIN ? INT64_MAX : h;
}

// Routing key of a composite partition key: each component as [short len][bytes][0x00].
inline std::string composite_routing_key(const std::vector<std::string>& parts) {
  if (parts.size() == 1) return parts[0];
  std::string out;
  for (auto& p : parts) {
    out.push_back(static_cast<char>((p.size() >> 8) & 0xFF));
    out.push_back(static_cast<char>(p.size() & 0xFF));
    out.append(p);
    out.push_back('\0');
  }
  return out;
}

// ------------------------------------------------------------------ misc helpers
inline const char* consistency_name(uint16_t c) {
  static const char* names[] = {"ANY",         "ONE",    "TWO",          "THREE",        "QUORUM",   "ALL",
                                "LOCAL_QUORUM", "EACH_QUORUM", "SERIAL", "LOCAL_SERIAL", "LOCAL_ONE"};
  return c <= 10 ? names[c] : "UNKNOWN";
}

}  // namespace nxcql
