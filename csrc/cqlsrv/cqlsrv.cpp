// nexus-cqlsrv — a small in-memory CQL (native protocol v4) server standing in for
// Scylla in tests and benchmarks.
//
// The reference's integration test needs a real Scylla from docker-compose
// (/root/reference/docker-compose.yaml:4-29, seeded by test-resources/prepare-scylla.sh
// and checkpoints.cql); neither docker nor Scylla exists offline, so this server
// implements the CQL subset a checkpoint store uses, over real TCP framing:
//
//   OPTIONS/STARTUP/AUTH (PasswordAuthenticator)/REGISTER, QUERY, PREPARE, EXECUTE, BATCH
//   USE · CREATE KEYSPACE/TABLE/INDEX · DROP · TRUNCATE
//   INSERT [IF NOT EXISTS] · UPDATE … SET … WHERE pk [IF EXISTS | IF col = x | col IN (…)]
//   SELECT cols|*|COUNT(*) FROM t [WHERE pk | indexed col = x] [LIMIT n]   DELETE
//   system.local / system.peers (token ring for token-aware clients), system.cqlsrv_stats
//
// Lightweight-transaction cost (--lwt-latency-us): a conditional write is a Paxos round —
// prepare/promise, read, propose/accept, commit: ~4 replica round trips where a plain write
// takes 1 — so its answer is held --lwt-latency-us longer than a plain one's (default 3 ×
// --latency-us), and conditional writes to ONE partition are serialised (each Paxos round
// on a partition starts when the previous one committed), as on Scylla / Cassandra.
// Fault injection for chaos tests: --latency-us, --error-rate (Overloaded errors),
// SIGUSR1 drops every client connection; --data FILE keeps a write-ahead log so a
// killed + restarted server ("Scylla node restart") keeps its rows.
//
// Scylla shard emulation (--shards N): N shard threads, each with its own epoll loop
// and connections, and the Scylla protocol extensions a shard-aware driver uses —
// SUPPORTED carries SCYLLA_SHARD / SCYLLA_NR_SHARDS / SCYLLA_SHARDING_ALGORITHM
// (biased-token-round-robin) / SCYLLA_SHARDING_IGNORE_MSB / SCYLLA_SHARD_AWARE_PORT,
// and a connection to the shard-aware port lands on shard (client source port % N).
// Every EXECUTE with a partition key counts whether it arrived on the shard owning
// its token (system.cqlsrv_stats shard_hits / shard_misses: a miss is the cross-shard
// hop real Scylla pays).  The data itself sits behind one lock; the shards parallelise
// framing, parsing, encoding and socket I/O.  Without --shards: one shard, no
// extensions.  Responses delayed by --latency-us go through a per-shard timer heap.
#include <arpa/inet.h>
#include <csignal>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <mutex>
#include <thread>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include <functional>
#include <memory>
#include <optional>
#include <queue>
#include <random>
#include <set>
#include <unordered_map>

#include "cql_proto.hpp"

using namespace nxcql;

namespace {

// ============================================================ options
struct Options {
  std::string host = "127.0.0.1";
  int port = 9042;
  std::string user, password;
  int64_t latency_us = 0;
  int64_t lwt_latency_us = -1;  // extra latency of a conditional write; -1 = 3 × latency_us
  double error_rate = 0.0;
  uint64_t seed = 1;
  std::string data_file;
  std::string ready_file;
  std::string dc = "datacenter1", rack = "rack1";
  std::vector<std::string> tokens;  // this node's tokens
  std::vector<std::string> peers;   // host:port:token[;token]
  bool verbose = false;
  int shards = 0;        // Scylla shard emulation: 0 = off (one shard, no extensions)
  int shard_port = 0;    // shard-aware port (0 = ephemeral) when --shards is given
  int advertise_shard_port = -1;  // test hook: advertise this port (e.g. a closed one) instead
  int ignore_msb = 12;   // SCYLLA_SHARDING_IGNORE_MSB
};

Options g_opt;
// set from the signal handler, read by every shard thread: lock-free atomics (async-signal-safe)
std::atomic<int> g_stop{0};
std::atomic<int> g_drop{0};
static_assert(std::atomic<int>::is_always_lock_free, "signal flags must be lock-free");

int64_t now_us() {
  return std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

std::string lower(std::string s) {
  for (auto& c : s) c = static_cast<char>(tolower(static_cast<unsigned char>(c)));
  return s;
}

// ============================================================ lexer
enum TokKind { TK_IDENT, TK_STRING, TK_NUMBER, TK_QMARK, TK_PUNCT, TK_END };
struct Tok {
  TokKind kind;
  std::string text;  // identifiers lower-cased unless quoted
};

struct CqlError : std::runtime_error {
  int32_t code;
  CqlError(int32_t c, const std::string& m) : std::runtime_error(m), code(c) {}
};

std::vector<Tok> lex(const std::string& q) {
  std::vector<Tok> out;
  size_t i = 0, n = q.size();
  while (i < n) {
    char c = q[i];
    if (isspace(static_cast<unsigned char>(c))) {
      ++i;
      continue;
    }
    if (c == '-' && i + 1 < n && q[i + 1] == '-') {
      while (i < n && q[i] != '\n') ++i;
      continue;
    }
    if (c == '\'') {
      std::string s;
      ++i;
      while (i < n) {
        if (q[i] == '\'') {
          if (i + 1 < n && q[i + 1] == '\'') {
            s.push_back('\'');
            i += 2;
            continue;
          }
          break;
        }
        s.push_back(q[i++]);
      }
      if (i >= n) throw CqlError(ERR_SYNTAX, "unterminated string literal");
      ++i;
      out.push_back({TK_STRING, s});
      continue;
    }
    if (c == '"') {
      std::string s;
      ++i;
      while (i < n && q[i] != '"') s.push_back(q[i++]);
      ++i;
      out.push_back({TK_IDENT, s});
      continue;
    }
    if (isalpha(static_cast<unsigned char>(c)) || c == '_') {
      size_t s = i;
      while (i < n && (isalnum(static_cast<unsigned char>(q[i])) || q[i] == '_')) ++i;
      // uuid literal: 8-4-4-4-12 hex starting with a letter
      if (i < n && q[i] == '-' && i - s == 8) {
        size_t j = i;
        while (j < n && (isxdigit(static_cast<unsigned char>(q[j])) || q[j] == '-')) ++j;
        if (j - s == 36) {
          out.push_back({TK_NUMBER, q.substr(s, 36)});
          i = j;
          continue;
        }
      }
      out.push_back({TK_IDENT, lower(q.substr(s, i - s))});
      continue;
    }
    if (isdigit(static_cast<unsigned char>(c)) || ((c == '-' || c == '+') && i + 1 < n && isdigit(static_cast<unsigned char>(q[i + 1])))) {
      size_t s = i++;
      while (i < n && (isalnum(static_cast<unsigned char>(q[i])) || q[i] == '.' || q[i] == '-')) {
        if (q[i] == '-' && !(i - s == 8 || i - s == 13 || i - s == 18 || i - s == 23)) break;
        ++i;
      }
      out.push_back({TK_NUMBER, q.substr(s, i - s)});
      continue;
    }
    if (c == '?') {
      out.push_back({TK_QMARK, "?"});
      ++i;
      continue;
    }
    if ((c == '!' || c == '<' || c == '>') && i + 1 < n && q[i + 1] == '=') {
      out.push_back({TK_PUNCT, q.substr(i, 2)});
      i += 2;
      continue;
    }
    out.push_back({TK_PUNCT, std::string(1, c)});
    ++i;
  }
  out.push_back({TK_END, ""});
  return out;
}

// ============================================================ AST
// A term is a literal, a bind marker (index into the values list) or NULL.
struct Term {
  enum Kind { LIT_STR, LIT_NUM, LIT_BOOL, NUL, BIND } kind = NUL;
  std::string text;
  int bind = -1;
};

struct Cond {
  std::string col;
  std::string op;  // "=", "in", "!="
  std::vector<Term> terms;
};

enum StmtKind { S_USE, S_CREATE_KS, S_CREATE_TABLE, S_CREATE_INDEX, S_DROP, S_TRUNCATE, S_INSERT, S_UPDATE, S_SELECT, S_DELETE };

struct ColDef {
  std::string name;
  Type type;
};

struct Stmt {
  StmtKind kind;
  std::string ks, table;            // target
  bool if_not_exists = false, if_exists = false;
  std::vector<std::string> cols;    // INSERT columns / SELECT columns (empty = *)
  bool count = false;
  std::vector<Term> values;         // INSERT values
  std::vector<std::pair<std::string, Term>> sets;  // UPDATE
  std::vector<Cond> where, ifs;
  int64_t limit = -1;
  // CREATE TABLE
  std::vector<ColDef> defs;
  std::vector<std::string> pk, ck;
  std::string index_col;
  int nbind = 0;
  std::string text;
};

Type parse_type_name(const std::string& tn) {
  Type t;
  static const std::map<std::string, uint16_t> m = {
      {"text", T_VARCHAR}, {"varchar", T_VARCHAR}, {"ascii", T_ASCII},    {"bigint", T_BIGINT},  {"blob", T_BLOB},
      {"boolean", T_BOOLEAN}, {"counter", T_COUNTER}, {"double", T_DOUBLE}, {"float", T_FLOAT}, {"int", T_INT},
      {"timestamp", T_TIMESTAMP}, {"uuid", T_UUID}, {"timeuuid", T_TIMEUUID}, {"inet", T_INET}, {"date", T_DATE},
      {"time", T_TIME}, {"smallint", T_SMALLINT}, {"tinyint", T_TINYINT}, {"varint", T_VARINT}, {"decimal", T_DECIMAL}};
  auto it = m.find(tn);
  if (it == m.end()) throw CqlError(ERR_INVALID, "unsupported type " + tn);
  t.id = it->second;
  return t;
}

class Parser {
 public:
  explicit Parser(const std::string& q) : toks_(lex(q)) { st_.text = q; }

  Stmt parse() {
    std::string kw = ident();
    if (kw == "use") {
      st_.kind = S_USE;
      st_.ks = ident();
    } else if (kw == "create") {
      parse_create();
    } else if (kw == "drop") {
      st_.kind = S_DROP;
      std::string what = ident();
      if (accept_kw("if")) {
        expect_kw("exists");
        st_.if_exists = true;
      }
      if (what == "keyspace") st_.ks = ident();
      else qualified_name();
      st_.cols.push_back(what);
    } else if (kw == "truncate") {
      st_.kind = S_TRUNCATE;
      accept_kw("table");
      qualified_name();
    } else if (kw == "insert") {
      parse_insert();
    } else if (kw == "update") {
      parse_update();
    } else if (kw == "select") {
      parse_select();
    } else if (kw == "delete") {
      st_.kind = S_DELETE;
      expect_kw("from");
      qualified_name();
      expect_kw("where");
      st_.where = conds();
      if (accept_kw("if")) {
        if (accept_kw("exists")) st_.if_exists = true;
        else st_.ifs = conds();
      }
    } else {
      throw CqlError(ERR_SYNTAX, "unsupported statement: " + kw);
    }
    accept_punct(";");
    if (peek().kind != TK_END) throw CqlError(ERR_SYNTAX, "unexpected trailing input near '" + peek().text + "'");
    return st_;
  }

 private:
  const Tok& peek() const { return toks_[pos_]; }
  const Tok& next() { return toks_[pos_ < toks_.size() - 1 ? pos_++ : pos_]; }
  std::string ident() {
    const Tok& t = next();
    if (t.kind != TK_IDENT) throw CqlError(ERR_SYNTAX, "expected identifier near '" + t.text + "'");
    return t.text;
  }
  bool accept_kw(const char* k) {
    if (peek().kind == TK_IDENT && peek().text == k) {
      ++pos_;
      return true;
    }
    return false;
  }
  void expect_kw(const char* k) {
    if (!accept_kw(k)) throw CqlError(ERR_SYNTAX, std::string("expected ") + k + " near '" + peek().text + "'");
  }
  bool accept_punct(const char* p) {
    if (peek().kind == TK_PUNCT && peek().text == p) {
      ++pos_;
      return true;
    }
    return false;
  }
  void expect_punct(const char* p) {
    if (!accept_punct(p)) throw CqlError(ERR_SYNTAX, std::string("expected '") + p + "' near '" + peek().text + "'");
  }
  void qualified_name() {
    std::string a = ident();
    if (accept_punct(".")) {
      st_.ks = a;
      st_.table = ident();
    } else {
      st_.table = a;
    }
  }
  Term term() {
    const Tok& t = next();
    Term out;
    switch (t.kind) {
      case TK_STRING: out.kind = Term::LIT_STR; out.text = t.text; break;
      case TK_NUMBER: out.kind = Term::LIT_NUM; out.text = t.text; break;
      case TK_QMARK: out.kind = Term::BIND; out.bind = st_.nbind++; break;
      case TK_IDENT:
        if (t.text == "null") out.kind = Term::NUL;
        else if (t.text == "true" || t.text == "false") {
          out.kind = Term::LIT_BOOL;
          out.text = t.text;
        } else
          throw CqlError(ERR_SYNTAX, "unexpected identifier in term: " + t.text);
        break;
      default: throw CqlError(ERR_SYNTAX, "expected a term near '" + t.text + "'");
    }
    return out;
  }
  std::vector<Cond> conds() {
    std::vector<Cond> cs;
    do {
      Cond c;
      c.col = ident();
      if (accept_punct("=")) {
        c.op = "=";
        c.terms.push_back(term());
      } else if (accept_punct("!=")) {
        c.op = "!=";
        c.terms.push_back(term());
      } else if (accept_kw("in")) {
        c.op = "in";
        expect_punct("(");
        if (!accept_punct(")")) {
          do c.terms.push_back(term());
          while (accept_punct(","));
          expect_punct(")");
        }
      } else {
        throw CqlError(ERR_SYNTAX, "unsupported operator near '" + peek().text + "'");
      }
      cs.push_back(std::move(c));
    } while (accept_kw("and"));
    return cs;
  }
  void skip_using() {
    if (accept_kw("using")) {
      do {
        ident();
        term();
      } while (accept_kw("and"));
    }
  }
  void skip_balanced_rest() {
    while (peek().kind != TK_END && !(peek().kind == TK_PUNCT && peek().text == ";")) ++pos_;
  }
  void parse_create() {
    std::string what = ident();
    if (what == "keyspace") {
      st_.kind = S_CREATE_KS;
      if (accept_kw("if")) {
        expect_kw("not");
        expect_kw("exists");
        st_.if_not_exists = true;
      }
      st_.ks = ident();
      skip_balanced_rest();
      return;
    }
    if (what == "index" || what == "custom") {
      if (what == "custom") expect_kw("index");
      st_.kind = S_CREATE_INDEX;
      if (accept_kw("if")) {
        expect_kw("not");
        expect_kw("exists");
        st_.if_not_exists = true;
      }
      if (!accept_kw("on")) {
        ident();  // index name
        expect_kw("on");
      }
      qualified_name();
      expect_punct("(");
      st_.index_col = ident();
      expect_punct(")");
      skip_balanced_rest();
      return;
    }
    if (what != "table" && what != "columnfamily") throw CqlError(ERR_SYNTAX, "unsupported CREATE " + what);
    st_.kind = S_CREATE_TABLE;
    if (accept_kw("if")) {
      expect_kw("not");
      expect_kw("exists");
      st_.if_not_exists = true;
    }
    qualified_name();
    expect_punct("(");
    do {
      if (accept_kw("primary")) {
        expect_kw("key");
        expect_punct("(");
        if (accept_punct("(")) {
          do st_.pk.push_back(ident());
          while (accept_punct(","));
          expect_punct(")");
        } else {
          st_.pk.push_back(ident());
        }
        while (accept_punct(",")) st_.ck.push_back(ident());
        expect_punct(")");
        continue;
      }
      ColDef d;
      d.name = ident();
      d.type = col_type();
      if (accept_kw("primary")) {
        expect_kw("key");
        st_.pk.push_back(d.name);
      }
      st_.defs.push_back(d);
    } while (accept_punct(","));
    expect_punct(")");
    skip_balanced_rest();
    if (st_.pk.empty()) throw CqlError(ERR_INVALID, "table has no primary key");
  }
  Type col_type() {
    std::string tn = ident();
    if (tn == "list" || tn == "set" || tn == "map" || tn == "frozen") {
      expect_punct("<");
      Type t;
      if (tn == "frozen") {
        t = col_type();
        expect_punct(">");
        return t;
      }
      t.id = tn == "list" ? T_LIST : tn == "set" ? T_SET : T_MAP;
      t.sub.push_back(col_type());
      if (tn == "map") {
        expect_punct(",");
        t.sub.push_back(col_type());
      }
      expect_punct(">");
      return t;
    }
    return parse_type_name(tn);
  }
  void parse_insert() {
    st_.kind = S_INSERT;
    expect_kw("into");
    qualified_name();
    expect_punct("(");
    do st_.cols.push_back(ident());
    while (accept_punct(","));
    expect_punct(")");
    expect_kw("values");
    expect_punct("(");
    do st_.values.push_back(term());
    while (accept_punct(","));
    expect_punct(")");
    if (accept_kw("if")) {
      expect_kw("not");
      expect_kw("exists");
      st_.if_not_exists = true;
    }
    skip_using();
    if (st_.cols.size() != st_.values.size()) throw CqlError(ERR_INVALID, "column/value count mismatch");
  }
  void parse_update() {
    st_.kind = S_UPDATE;
    qualified_name();
    skip_using();
    expect_kw("set");
    do {
      std::string c = ident();
      expect_punct("=");
      st_.sets.emplace_back(c, term());
    } while (accept_punct(","));
    expect_kw("where");
    st_.where = conds();
    if (accept_kw("if")) {
      if (accept_kw("exists")) st_.if_exists = true;
      else st_.ifs = conds();
    }
  }
  void parse_select() {
    st_.kind = S_SELECT;
    if (accept_punct("*")) {
    } else if (peek().kind == TK_IDENT && peek().text == "count" && toks_[pos_ + 1].text == "(") {
      pos_ += 2;
      if (!accept_punct("*")) ident();
      expect_punct(")");
      st_.count = true;
    } else {
      do st_.cols.push_back(ident());
      while (accept_punct(","));
    }
    expect_kw("from");
    qualified_name();
    if (accept_kw("where")) st_.where = conds();
    if (accept_kw("limit")) st_.limit = std::stoll(next().text);
    if (accept_kw("allow")) expect_kw("filtering");
  }

  std::vector<Tok> toks_;
  size_t pos_ = 0;
  Stmt st_;
};

// ============================================================ values
using Val = std::optional<std::string>;  // serialized CQL value, nullopt = null

int64_t parse_timestamp_literal(const std::string& s) {
  bool digits = !s.empty();
  for (char c : s)
    if (!isdigit(static_cast<unsigned char>(c)) && c != '-') digits = false;
  if (digits && s.find('-', 1) == std::string::npos) return std::stoll(s);
  int Y = 0, M = 0, D = 0, h = 0, m = 0;
  double sec = 0;
  int n = sscanf(s.c_str(), "%d-%d-%d%*c%d:%d:%lf", &Y, &M, &D, &h, &m, &sec);
  if (n < 3) throw CqlError(ERR_INVALID, "bad timestamp literal '" + s + "'");
  struct tm tmv = {};
  tmv.tm_year = Y - 1900;
  tmv.tm_mon = M - 1;
  tmv.tm_mday = D;
  tmv.tm_hour = h;
  tmv.tm_min = m;
  tmv.tm_sec = static_cast<int>(sec);
  int64_t ms = static_cast<int64_t>(timegm(&tmv)) * 1000 + static_cast<int64_t>(std::llround((sec - static_cast<int>(sec)) * 1000.0));
  // trailing zone offset +hhmm / -hhmm (Z or none = UTC)
  size_t tpos = s.find_last_of("+-");
  if (tpos != std::string::npos && tpos > 10 && s.size() - tpos >= 5) {
    int off = std::stoi(s.substr(tpos + 1, 2)) * 60 + std::stoi(s.substr(s.size() - 2, 2));
    ms -= (s[tpos] == '+' ? 1 : -1) * static_cast<int64_t>(off) * 60000;
  }
  return ms;
}

std::string literal_to_value(const Term& t, const Type& ty) {
  Writer w;
  const std::string& s = t.text;
  switch (ty.id) {
    case T_VARCHAR:
    case T_ASCII:
      return s;
    case T_BLOB: {
      std::string out;
      size_t i = (s.rfind("0x", 0) == 0) ? 2 : 0;
      for (; i + 1 < s.size(); i += 2) out.push_back(static_cast<char>(std::stoi(s.substr(i, 2), nullptr, 16)));
      return out;
    }
    case T_TIMESTAMP: w.i64(parse_timestamp_literal(s)); return w.buf;
    case T_BIGINT:
    case T_COUNTER:
    case T_TIME: w.i64(std::stoll(s)); return w.buf;
    case T_INT: w.i32(static_cast<int32_t>(std::stol(s))); return w.buf;
    case T_SMALLINT: w.u16(static_cast<uint16_t>(std::stoi(s))); return w.buf;
    case T_TINYINT: w.u8(static_cast<uint8_t>(std::stoi(s))); return w.buf;
    case T_BOOLEAN: w.u8(lower(s) == "true" ? 1 : 0); return w.buf;
    case T_DOUBLE: {
      double d = std::stod(s);
      int64_t b;
      memcpy(&b, &d, 8);
      w.i64(b);
      return w.buf;
    }
    case T_FLOAT: {
      float f = std::stof(s);
      int32_t b;
      memcpy(&b, &f, 4);
      w.i32(b);
      return w.buf;
    }
    case T_UUID:
    case T_TIMEUUID: {
      std::string out;
      int hi = -1;
      for (char c : s) {
        if (c == '-') continue;
        int x = isdigit(static_cast<unsigned char>(c)) ? c - '0' : (tolower(c) - 'a' + 10);
        if (hi < 0) hi = x;
        else {
          out.push_back(static_cast<char>((hi << 4) | x));
          hi = -1;
        }
      }
      if (out.size() != 16) throw CqlError(ERR_INVALID, "bad uuid literal");
      return out;
    }
    case T_INET: {
      in_addr a;
      if (inet_pton(AF_INET, s.c_str(), &a) == 1) return std::string(reinterpret_cast<char*>(&a), 4);
      throw CqlError(ERR_INVALID, "bad inet literal");
    }
    default: throw CqlError(ERR_INVALID, "literal not supported for this column type");
  }
}

// ============================================================ schema + data
struct Table {
  std::string ks, name;
  std::vector<ColDef> cols;
  std::unordered_map<std::string, int> idx;
  std::vector<int> pk, ck;
  std::set<int> indexed;
  std::unordered_map<std::string, std::vector<Val>> rows;
  std::vector<std::string> order;  // insertion order of keys for stable scans (may contain deleted keys)
};

struct Prepared {
  Stmt stmt;
  std::vector<ColSpec> bind;    // one per bind marker
  std::vector<uint16_t> pk_idx;  // bind positions of partition-key columns (pk order)
  std::vector<ColSpec> result;   // SELECT result columns (empty for mutations)
};

struct Stats {
  std::atomic<uint64_t> requests{0}, queries{0}, executes{0}, prepares{0}, batches{0}, reads{0}, writes{0}, lwt{0},
      errors{0}, injected_errors{0}, connections{0}, dropped{0}, shard_hits{0}, shard_misses{0}, lwt_waits{0};
};

class Db {
 public:
  std::map<std::string, std::unique_ptr<Table>> tables;  // "ks.table"
  std::set<std::string> keyspaces;
  std::unordered_map<std::string, Prepared> prepared;
  Stats stats;
  FILE* wal = nullptr;
  bool replaying = false;

  Table* find(const std::string& ks, const std::string& t) {
    auto it = tables.find(ks + "." + t);
    return it == tables.end() ? nullptr : it->second.get();
  }

  Table& need(const std::string& ks, const std::string& t) {
    Table* tb = find(ks, t);
    if (!tb) throw CqlError(ERR_INVALID, "unconfigured table " + t);
    return *tb;
  }

  // ---------- WAL ("S" schema text | "R" full row image | "D" delete | "T" truncate)
  void wal_write(char kind, const std::string& a, const std::string& b = std::string()) {
    if (!wal || replaying) return;
    Writer w;
    w.u8(static_cast<uint8_t>(kind));
    w.long_string(a);
    w.long_string(b);
    fwrite(w.buf.data(), 1, w.buf.size(), wal);
    fflush(wal);
  }
  static std::string encode_row(const std::vector<Val>& row) {
    Writer w;
    w.i32(static_cast<int32_t>(row.size()));
    for (auto& v : row) {
      if (v) w.bytes(*v);
      else w.null_bytes();
    }
    return w.buf;
  }
  void wal_row(const Table& t, const std::vector<Val>& row) { wal_write('R', t.ks + "." + t.name, encode_row(row)); }

  void replay(const std::string& path) {
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) return;
    std::string data;
    char buf[1 << 16];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) data.append(buf, n);
    fclose(f);
    replaying = true;
    Reader r(data.data(), data.size());
    size_t good = 0;
    try {
      while (r.remaining() > 0) {
        char kind = static_cast<char>(r.u8());
        std::string a = r.long_string();
        std::string b = r.long_string();
        if (kind == 'S') {
          Parser p(a);
          Stmt st = p.parse();
          std::string cur;
          run_schema(st, cur);
        } else if (kind == 'R' || kind == 'D' || kind == 'T') {
          auto it = tables.find(a);
          if (it == tables.end()) continue;
          Table& t = *it->second;
          if (kind == 'T') {
            t.rows.clear();
            t.order.clear();
          } else if (kind == 'D') {
            t.rows.erase(b);
          } else {
            Reader rr(b.data(), b.size());
            int32_t k = rr.i32();
            std::vector<Val> row(static_cast<size_t>(k));
            for (int32_t i = 0; i < k; ++i) {
              const uint8_t* d;
              int32_t len;
              if (rr.bytes(d, len)) row[i] = std::string(reinterpret_cast<const char*>(d), static_cast<size_t>(len));
            }
            row.resize(t.cols.size());
            std::string key = key_of(t, row);
            if (!t.rows.count(key)) t.order.push_back(key);
            t.rows[key] = std::move(row);
          }
        }
        good = r.off;
      }
    } catch (const std::exception&) {
      // torn tail record from a crash: truncate it away
    }
    replaying = false;
    if (good < data.size()) {
      if (truncate(path.c_str(), static_cast<off_t>(good)) != 0) perror("truncate wal");
    }
  }

  static std::string key_of(const Table& t, const std::vector<Val>& row) {
    std::string k;
    for (int i : t.pk) {
      const Val& v = row[static_cast<size_t>(i)];
      if (!v) throw CqlError(ERR_INVALID, "missing partition key column " + t.cols[static_cast<size_t>(i)].name);
      Writer w;
      w.bytes(*v);
      k += w.buf;
    }
    for (int i : t.ck) {
      const Val& v = row[static_cast<size_t>(i)];
      if (!v) throw CqlError(ERR_INVALID, "missing clustering column " + t.cols[static_cast<size_t>(i)].name);
      Writer w;
      w.bytes(*v);
      k += w.buf;
    }
    return k;
  }

  // ---------- schema
  std::string run_schema(const Stmt& st, std::string& cur_ks) {
    std::string ks = st.ks.empty() ? cur_ks : st.ks;
    switch (st.kind) {
      case S_CREATE_KS:
        if (keyspaces.count(st.ks)) {
          if (st.if_not_exists) return "";
          throw CqlError(ERR_ALREADY_EXISTS, "keyspace " + st.ks + " already exists");
        }
        keyspaces.insert(st.ks);
        wal_write('S', st.text);
        return "KEYSPACE";
      case S_CREATE_TABLE: {
        if (ks.empty()) throw CqlError(ERR_INVALID, "no keyspace specified");
        if (!keyspaces.count(ks)) throw CqlError(ERR_INVALID, "keyspace " + ks + " does not exist");
        if (find(ks, st.table)) {
          if (st.if_not_exists) return "";
          throw CqlError(ERR_ALREADY_EXISTS, "table " + st.table + " already exists");
        }
        auto t = std::make_unique<Table>();
        t->ks = ks;
        t->name = st.table;
        t->cols = st.defs;
        for (size_t i = 0; i < t->cols.size(); ++i) t->idx[t->cols[i].name] = static_cast<int>(i);
        for (auto& c : st.pk) {
          auto it = t->idx.find(c);
          if (it == t->idx.end()) throw CqlError(ERR_INVALID, "unknown primary key column " + c);
          t->pk.push_back(it->second);
        }
        for (auto& c : st.ck) {
          auto it = t->idx.find(c);
          if (it == t->idx.end()) throw CqlError(ERR_INVALID, "unknown clustering column " + c);
          t->ck.push_back(it->second);
        }
        tables[ks + "." + st.table] = std::move(t);
        if (!replaying) {
          Stmt copy = st;
          wal_write('S', with_keyspace(st.text, ks));
        }
        return "TABLE";
      }
      case S_CREATE_INDEX: {
        Table& t = need(ks, st.table);
        auto it = t.idx.find(st.index_col);
        if (it == t.idx.end()) throw CqlError(ERR_INVALID, "unknown column " + st.index_col);
        t.indexed.insert(it->second);
        wal_write('S', with_keyspace(st.text, ks));
        return "TABLE";
      }
      case S_DROP: {
        const std::string& what = st.cols.at(0);
        if (what == "keyspace") {
          if (!keyspaces.erase(st.ks) && !st.if_exists) throw CqlError(ERR_INVALID, "keyspace does not exist");
          for (auto it = tables.begin(); it != tables.end();)
            it = it->second->ks == st.ks ? tables.erase(it) : std::next(it);
        } else if (what == "table") {
          if (!tables.erase(ks + "." + st.table) && !st.if_exists) throw CqlError(ERR_INVALID, "table does not exist");
        }
        wal_write('S', with_keyspace(st.text, ks));
        prepared.clear();
        return "DROPPED";
      }
      default: return "";
    }
  }

  // CREATE TABLE/INDEX text run under USE: make the keyspace explicit for WAL replay.
  static std::string with_keyspace(const std::string& text, const std::string& ks) {
    (void)ks;
    return text;
  }
};

Db g_db;

// ============================================================ statement execution
struct Bound {
  const std::vector<Val>* values = nullptr;
};

Val term_value(const Term& t, const Type& ty, const std::vector<Val>& vals) {
  switch (t.kind) {
    case Term::NUL: return std::nullopt;
    case Term::BIND:
      if (t.bind < 0 || static_cast<size_t>(t.bind) >= vals.size()) throw CqlError(ERR_INVALID, "missing bind value");
      return vals[static_cast<size_t>(t.bind)];
    default: return literal_to_value(t, ty);
  }
}

int col_of(const Table& t, const std::string& c) {
  auto it = t.idx.find(c);
  if (it == t.idx.end()) throw CqlError(ERR_INVALID, "undefined column name " + c);
  return it->second;
}

bool cond_holds(const Table& t, const std::vector<Val>* row, const Cond& c, const std::vector<Val>& vals) {
  int ci = col_of(t, c.col);
  const Type& ty = t.cols[static_cast<size_t>(ci)].type;
  Val cur = row ? (*row)[static_cast<size_t>(ci)] : std::nullopt;
  if (c.op == "=") return cur == term_value(c.terms.at(0), ty, vals);
  if (c.op == "!=") return cur != term_value(c.terms.at(0), ty, vals);
  for (auto& term : c.terms)
    if (cur == term_value(term, ty, vals)) return true;
  return false;
}

// Partition-key lookups for WHERE clauses that pin the full primary key (IN allowed on one column).
std::vector<std::string> keys_from_where(const Table& t, const std::vector<Cond>& where, const std::vector<Val>& vals,
                                         bool* full_key) {
  std::vector<int> keycols = t.pk;
  keycols.insert(keycols.end(), t.ck.begin(), t.ck.end());
  std::vector<std::vector<Val>> choices(keycols.size());
  size_t matched = 0;
  for (size_t k = 0; k < keycols.size(); ++k) {
    for (auto& c : where) {
      if (col_of(t, c.col) != keycols[k]) continue;
      const Type& ty = t.cols[static_cast<size_t>(keycols[k])].type;
      if (c.op == "=") choices[k].push_back(term_value(c.terms.at(0), ty, vals));
      else if (c.op == "in")
        for (auto& term : c.terms) choices[k].push_back(term_value(term, ty, vals));
    }
    if (!choices[k].empty()) ++matched;
  }
  *full_key = matched == keycols.size();
  std::vector<std::string> keys;
  if (!*full_key) return keys;
  std::vector<size_t> pos(keycols.size(), 0);
  while (true) {
    std::string k;
    for (size_t i = 0; i < keycols.size(); ++i) {
      const Val& v = choices[i][pos[i]];
      if (!v) throw CqlError(ERR_INVALID, "null primary key value");
      Writer w;
      w.bytes(*v);
      k += w.buf;
    }
    keys.push_back(k);
    size_t i = 0;
    while (i < keycols.size() && ++pos[i] == choices[i].size()) pos[i++] = 0;
    if (i == keycols.size()) break;
  }
  return keys;
}

struct ResultSet {
  std::vector<ColSpec> cols;
  std::vector<std::vector<Val>> rows;
};

std::vector<ColSpec> specs_of(const Table& t, const std::vector<int>& which) {
  std::vector<ColSpec> out;
  for (int i : which) out.push_back(ColSpec{t.ks, t.name, t.cols[static_cast<size_t>(i)].name, t.cols[static_cast<size_t>(i)].type});
  return out;
}

std::vector<int> select_cols(const Table& t, const Stmt& st) {
  std::vector<int> which;
  if (st.cols.empty())
    for (size_t i = 0; i < t.cols.size(); ++i) which.push_back(static_cast<int>(i));
  else
    for (auto& c : st.cols) which.push_back(col_of(t, c));
  return which;
}

// set by execute() when the statement was a conditional write (its partition); read and
// cleared by the request handler to price the Paxos round (see --lwt-latency-us)
thread_local std::string t_lwt_partition;

ColSpec applied_spec(const Table& t) {
  Type b;
  b.id = T_BOOLEAN;
  return ColSpec{t.ks, t.name, "[applied]", b};
}

Val bool_val(bool b) { return std::string(1, b ? '\x01' : '\x00'); }

ResultSet lwt_result(const Table& t, bool applied, const std::vector<Val>* existing) {
  ResultSet rs;
  rs.cols.push_back(applied_spec(t));
  std::vector<Val> row{bool_val(applied)};
  if (!applied && existing) {
    for (size_t i = 0; i < t.cols.size(); ++i) rs.cols.push_back(specs_of(t, {static_cast<int>(i)})[0]);
    row.insert(row.end(), existing->begin(), existing->end());
  }
  rs.rows.push_back(std::move(row));
  return rs;
}

ResultSet system_local_rows(const Stmt& st);
ResultSet system_peers_rows(const Stmt& st);
ResultSet stats_rows();

// Execute; returns true with `rs` filled when the statement produces rows.
bool execute(const Stmt& st, const std::vector<Val>& vals, std::string& cur_ks, ResultSet& rs, std::string& set_ks,
             std::string& schema_change) {
  std::string ks = st.ks.empty() ? cur_ks : st.ks;
  switch (st.kind) {
    case S_USE:
      if (!g_db.keyspaces.count(st.ks) && st.ks != "system") throw CqlError(ERR_INVALID, "keyspace " + st.ks + " does not exist");
      cur_ks = st.ks;
      set_ks = st.ks;
      return false;
    case S_CREATE_KS:
    case S_CREATE_TABLE:
    case S_CREATE_INDEX:
    case S_DROP:
      schema_change = g_db.run_schema(st, cur_ks);
      return false;
    case S_TRUNCATE: {
      Table& t = g_db.need(ks, st.table);
      t.rows.clear();
      t.order.clear();
      g_db.wal_write('T', t.ks + "." + t.name);
      return false;
    }
    case S_INSERT: {
      Table& t = g_db.need(ks, st.table);
      std::vector<Val> row(t.cols.size());
      std::vector<bool> given(t.cols.size(), false);
      for (size_t i = 0; i < st.cols.size(); ++i) {
        int ci = col_of(t, st.cols[i]);
        row[static_cast<size_t>(ci)] = term_value(st.values[i], t.cols[static_cast<size_t>(ci)].type, vals);
        given[static_cast<size_t>(ci)] = true;
      }
      std::string key = Db::key_of(t, row);
      auto it = t.rows.find(key);
      ++g_db.stats.writes;
      if (st.if_not_exists) {
        ++g_db.stats.lwt;
        t_lwt_partition = t.ks + "." + t.name + "/" + key;
        if (it != t.rows.end()) {
          rs = lwt_result(t, false, &it->second);
          return true;
        }
      }
      if (it == t.rows.end()) {
        t.order.push_back(key);
        it = t.rows.emplace(key, std::vector<Val>(t.cols.size())).first;
      }
      for (size_t i = 0; i < row.size(); ++i)
        if (given[i]) it->second[i] = row[i];
      g_db.wal_row(t, it->second);
      if (st.if_not_exists) {
        rs = lwt_result(t, true, nullptr);
        return true;
      }
      return false;
    }
    case S_UPDATE:
    case S_DELETE: {
      Table& t = g_db.need(ks, st.table);
      bool full = false;
      auto keys = keys_from_where(t, st.where, vals, &full);
      if (!full) throw CqlError(ERR_INVALID, "some partition key parts are missing");
      bool lwt = st.if_exists || !st.ifs.empty();
      if (lwt && keys.size() != 1) throw CqlError(ERR_INVALID, "IN on the primary key is not supported with conditions");
      ++g_db.stats.writes;
      for (auto& key : keys) {
        auto it = t.rows.find(key);
        if (lwt) {
          ++g_db.stats.lwt;
          t_lwt_partition = t.ks + "." + t.name + "/" + key;
          const std::vector<Val>* existing = it == t.rows.end() ? nullptr : &it->second;
          bool ok = st.if_exists ? existing != nullptr : existing != nullptr;
          for (auto& c : st.ifs) ok = ok && cond_holds(t, existing, c, vals);
          if (!ok) {
            rs = lwt_result(t, false, existing);
            return true;
          }
        }
        if (st.kind == S_DELETE) {
          if (it != t.rows.end()) {
            t.rows.erase(it);
            g_db.wal_write('D', t.ks + "." + t.name, key);
          }
          continue;
        }
        if (it == t.rows.end()) {
          // UPDATE is an upsert: materialise the primary key from the WHERE clause
          std::vector<Val> row(t.cols.size());
          for (auto& c : st.where) {
            int ci = col_of(t, c.col);
            row[static_cast<size_t>(ci)] = term_value(c.terms.at(0), t.cols[static_cast<size_t>(ci)].type, vals);
          }
          t.order.push_back(key);
          it = t.rows.emplace(key, std::move(row)).first;
        }
        for (auto& s : st.sets) {
          int ci = col_of(t, s.first);
          for (int p : t.pk)
            if (p == ci) throw CqlError(ERR_INVALID, "PRIMARY KEY part " + s.first + " found in SET part");
          it->second[static_cast<size_t>(ci)] = term_value(s.second, t.cols[static_cast<size_t>(ci)].type, vals);
        }
        g_db.wal_row(t, it->second);
      }
      if (lwt) {
        rs = lwt_result(t, true, nullptr);
        return true;
      }
      return false;
    }
    case S_SELECT: {
      if (ks == "system" && (st.table == "local")) {
        rs = system_local_rows(st);
        return true;
      }
      if (ks == "system" && (st.table == "peers" || st.table == "peers_v2")) {
        rs = system_peers_rows(st);
        return true;
      }
      if (ks == "system" && st.table == "cqlsrv_stats") {
        rs = stats_rows();
        return true;
      }
      if (ks.rfind("system", 0) == 0 && !g_db.find(ks, st.table)) {
        rs.cols.clear();
        rs.rows.clear();
        Type tx;
        tx.id = T_VARCHAR;
        rs.cols.push_back(ColSpec{ks, st.table, "keyspace_name", tx});
        return true;
      }
      Table& t = g_db.need(ks, st.table);
      ++g_db.stats.reads;
      std::vector<int> which = select_cols(t, st);
      std::vector<const std::vector<Val>*> hits;
      bool full = false;
      auto keys = keys_from_where(t, st.where, vals, &full);
      if (full) {
        for (auto& k : keys) {
          auto it = t.rows.find(k);
          if (it != t.rows.end()) hits.push_back(&it->second);
        }
      } else {
        // scan (secondary-index or ALLOW FILTERING semantics; stable insertion order)
        for (auto& k : t.order) {
          auto it = t.rows.find(k);
          if (it == t.rows.end()) continue;
          bool ok = true;
          for (auto& c : st.where) ok = ok && cond_holds(t, &it->second, c, vals);
          if (ok) hits.push_back(&it->second);
        }
      }
      if (full)
        for (auto it = hits.begin(); it != hits.end();) {
          bool ok = true;
          for (auto& c : st.where) ok = ok && cond_holds(t, *it, c, vals);
          it = ok ? std::next(it) : hits.erase(it);
        }
      if (st.count) {
        Type bi;
        bi.id = T_BIGINT;
        rs.cols = {ColSpec{t.ks, t.name, "count", bi}};
        Writer w;
        w.i64(static_cast<int64_t>(hits.size()));
        rs.rows = {{w.buf}};
        return true;
      }
      rs.cols = specs_of(t, which);
      for (auto* r : hits) {
        if (st.limit >= 0 && static_cast<int64_t>(rs.rows.size()) >= st.limit) break;
        std::vector<Val> out;
        out.reserve(which.size());
        for (int i : which) out.push_back((*r)[static_cast<size_t>(i)]);
        rs.rows.push_back(std::move(out));
      }
      return true;
    }
  }
  return false;
}

// ---------------------------------------------------------------- system tables
Val text_val(const std::string& s) { return s; }
Val inet_val(const std::string& ip) {
  in_addr a;
  if (inet_pton(AF_INET, ip.c_str(), &a) != 1) return std::nullopt;
  return std::string(reinterpret_cast<char*>(&a), 4);
}
Val int_val(int32_t v) {
  Writer w;
  w.i32(v);
  return w.buf;
}
Val set_text_val(const std::vector<std::string>& items) {
  Writer w;
  w.i32(static_cast<int32_t>(items.size()));
  for (auto& s : items) w.bytes(s);
  return w.buf;
}
Val uuid_val(uint64_t seed) {
  std::string s(16, '\0');
  for (int i = 0; i < 16; ++i) s[static_cast<size_t>(i)] = static_cast<char>((seed >> ((i % 8) * 8)) ^ (i * 37));
  s[6] = static_cast<char>((s[6] & 0x0F) | 0x40);
  s[8] = static_cast<char>((s[8] & 0x3F) | 0x80);
  return s;
}

Type ty(uint16_t id) {
  Type t;
  t.id = id;
  return t;
}
Type set_of_text() {
  Type t;
  t.id = T_SET;
  t.sub.push_back(ty(T_VARCHAR));
  return t;
}

ResultSet project(const std::vector<ColSpec>& all, const std::vector<std::vector<Val>>& rows, const Stmt& st) {
  ResultSet rs;
  std::vector<size_t> which;
  if (st.cols.empty())
    for (size_t i = 0; i < all.size(); ++i) which.push_back(i);
  else
    for (auto& c : st.cols) {
      size_t i = 0;
      while (i < all.size() && all[i].name != c) ++i;
      if (i == all.size()) throw CqlError(ERR_INVALID, "undefined column name " + c);
      which.push_back(i);
    }
  for (size_t i : which) rs.cols.push_back(all[i]);
  for (auto& r : rows) {
    std::vector<Val> out;
    for (size_t i : which) out.push_back(r[i]);
    rs.rows.push_back(std::move(out));
  }
  return rs;
}

std::vector<std::string> my_tokens() {
  if (!g_opt.tokens.empty()) return g_opt.tokens;
  return {"-9223372036854775807"};  // single node owns the whole ring
}

ResultSet system_local_rows(const Stmt& st) {
  std::vector<ColSpec> all = {
      {"system", "local", "key", ty(T_VARCHAR)},          {"system", "local", "data_center", ty(T_VARCHAR)},
      {"system", "local", "rack", ty(T_VARCHAR)},         {"system", "local", "release_version", ty(T_VARCHAR)},
      {"system", "local", "cluster_name", ty(T_VARCHAR)}, {"system", "local", "partitioner", ty(T_VARCHAR)},
      {"system", "local", "rpc_address", ty(T_INET)},     {"system", "local", "broadcast_address", ty(T_INET)},
      {"system", "local", "host_id", ty(T_UUID)},         {"system", "local", "tokens", set_of_text()},
      {"system", "local", "native_port", ty(T_INT)}};
  std::vector<std::vector<Val>> rows = {{text_val("local"), text_val(g_opt.dc), text_val(g_opt.rack), text_val("3.0.8"),
                                         text_val("nexus-cqlsrv"), text_val("org.apache.cassandra.dht.Murmur3Partitioner"),
                                         inet_val(g_opt.host), inet_val(g_opt.host), uuid_val(static_cast<uint64_t>(g_opt.port)),
                                         set_text_val(my_tokens()), int_val(g_opt.port)}};
  return project(all, rows, st);
}

ResultSet system_peers_rows(const Stmt& st) {
  std::vector<ColSpec> all = {{"system", "peers", "peer", ty(T_INET)},          {"system", "peers", "data_center", ty(T_VARCHAR)},
                              {"system", "peers", "rack", ty(T_VARCHAR)},        {"system", "peers", "rpc_address", ty(T_INET)},
                              {"system", "peers", "host_id", ty(T_UUID)},        {"system", "peers", "tokens", set_of_text()},
                              {"system", "peers", "release_version", ty(T_VARCHAR)}, {"system", "peers", "native_port", ty(T_INT)}};
  std::vector<std::vector<Val>> rows;
  for (auto& p : g_opt.peers) {
    // host:port:tok1;tok2
    size_t a = p.find(':'), b = p.find(':', a + 1);
    if (a == std::string::npos || b == std::string::npos) continue;
    std::string host = p.substr(0, a);
    int port = std::stoi(p.substr(a + 1, b - a - 1));
    std::vector<std::string> toks;
    std::string rest = p.substr(b + 1);
    size_t s = 0;
    while (s <= rest.size()) {
      size_t e = rest.find(';', s);
      if (e == std::string::npos) e = rest.size();
      if (e > s) toks.push_back(rest.substr(s, e - s));
      s = e + 1;
    }
    rows.push_back({inet_val(host), text_val(g_opt.dc), text_val(g_opt.rack), inet_val(host), uuid_val(static_cast<uint64_t>(port)),
                    set_text_val(toks), text_val("3.0.8"), int_val(port)});
  }
  return project(all, rows, st);
}

ResultSet stats_rows() {
  ResultSet rs;
  const Stats& s = g_db.stats;
  std::vector<std::pair<const char*, uint64_t>> kv = {
      {"requests", s.requests},       {"queries", s.queries},       {"executes", s.executes},
      {"prepares", s.prepares},       {"batches", s.batches},       {"reads", s.reads},
      {"writes", s.writes},           {"lwt", s.lwt},               {"errors", s.errors},
      {"injected_errors", s.injected_errors}, {"connections", s.connections}, {"dropped", s.dropped},
      {"shard_hits", s.shard_hits},   {"shard_misses", s.shard_misses}, {"lwt_waits", s.lwt_waits}};
  for (auto& p : kv) rs.cols.push_back(ColSpec{"system", "cqlsrv_stats", p.first, ty(T_BIGINT)});
  std::vector<Val> row;
  for (auto& p : kv) {
    Writer w;
    w.i64(static_cast<int64_t>(p.second));
    row.push_back(w.buf);
  }
  rs.rows.push_back(std::move(row));
  return rs;
}

// ============================================================ response builders
std::string rows_body(const ResultSet& rs, bool skip_meta) {
  Writer w;
  w.i32(RK_ROWS);
  bool global = !rs.cols.empty();
  for (auto& c : rs.cols) global = global && c.keyspace == rs.cols[0].keyspace && c.table == rs.cols[0].table;
  int32_t flags = skip_meta ? MF_NO_METADATA : (global ? MF_GLOBAL_TABLES_SPEC : 0);
  w.i32(flags);
  w.i32(static_cast<int32_t>(rs.cols.size()));
  if (!skip_meta) {
    if (global) {
      w.string(rs.cols[0].keyspace);
      w.string(rs.cols[0].table);
    }
    for (auto& c : rs.cols) {
      if (!global) {
        w.string(c.keyspace);
        w.string(c.table);
      }
      w.string(c.name);
      w.type(c.type);
    }
  }
  w.i32(static_cast<int32_t>(rs.rows.size()));
  for (auto& r : rs.rows)
    for (auto& v : r) {
      if (v) w.bytes(*v);
      else w.null_bytes();
    }
  return w.buf;
}

std::string void_body() {
  Writer w;
  w.i32(RK_VOID);
  return w.buf;
}

std::string error_body(int32_t code, const std::string& msg, const std::string& extra = std::string()) {
  Writer w;
  w.i32(code);
  w.string(msg.size() > 60000 ? msg.substr(0, 60000) : msg);
  w.buf += extra;
  return w.buf;
}

std::string schema_change_body(const std::string& target, const std::string& ks, const std::string& name) {
  Writer w;
  w.i32(RK_SCHEMA_CHANGE);
  w.string("CREATED");
  w.string(target);
  w.string(ks);
  if (target != "KEYSPACE") w.string(name);
  return w.buf;
}

std::string prepare_id(const std::string& ks, const std::string& q) {
  std::string key = ks + "\x1f" + q;
  int64_t a = murmur3_h1(reinterpret_cast<const uint8_t*>(key.data()), key.size());
  std::string salted = "nx" + key;
  int64_t b = murmur3_h1(reinterpret_cast<const uint8_t*>(salted.data()), salted.size());
  Writer w;
  w.i64(a);
  w.i64(b);
  return w.buf;
}

// ============================================================ connections
struct Conn {
  int fd;
  FrameSplitter in;
  std::string out;
  size_t out_off = 0;
  bool ready = false;        // STARTUP done
  bool authed = false;
  std::string ks;
  bool want_write = false;
};

struct Delayed {
  int64_t due;
  int fd;
  uint64_t gen;
  std::string bytes;
  bool operator>(const Delayed& o) const { return due > o.due; }
};

// One shard: an epoll loop over its own connections (Scylla's shard-per-core model).
struct Shard {
  int id = 0;
  int epfd = -1;
  int wake = -1;  // eventfd: new connections handed over by the acceptor
  std::mutex inbox_mu;
  std::vector<int> inbox;
  std::unordered_map<int, std::unique_ptr<Conn>> conns;
  std::unordered_map<int, uint64_t> gen;  // fd generation (reuse guard for delayed writes)
  std::priority_queue<Delayed, std::vector<Delayed>, std::greater<Delayed>> delayed;
  std::mt19937_64 rng;
  uint64_t drop_seen = 0;
};

std::mutex g_db_mu;  // tables, prepared statements, WAL, the Paxos clocks
// per partition: when the last Paxos round on it commits (µs, now_us clock); a new round on
// the partition starts no earlier (guarded by g_db_mu)
std::unordered_map<std::string, int64_t> g_paxos_busy;

int64_t lwt_extra_us() { return g_opt.lwt_latency_us >= 0 ? g_opt.lwt_latency_us : 3 * g_opt.latency_us; }
std::atomic<uint64_t> g_drop_gen{0};
std::vector<std::unique_ptr<Shard>> g_shards;
int g_shard_port = 0;

void set_nonblock(int fd) { fcntl(fd, F_SETFL, fcntl(fd, F_GETFL, 0) | O_NONBLOCK); }

void close_conn(Shard& s, int fd) {
  epoll_ctl(s.epfd, EPOLL_CTL_DEL, fd, nullptr);
  close(fd);
  s.conns.erase(fd);
  s.gen[fd]++;
}

void update_interest(Shard& s, Conn& c) {
  bool want = c.out.size() > c.out_off;
  if (want == c.want_write) return;
  c.want_write = want;
  epoll_event ev{};
  ev.events = EPOLLIN | (want ? static_cast<uint32_t>(EPOLLOUT) : 0u);
  ev.data.fd = c.fd;
  epoll_ctl(s.epfd, EPOLL_CTL_MOD, c.fd, &ev);
}

bool flush(Shard& s, Conn& c) {
  while (c.out_off < c.out.size()) {
    ssize_t n = ::send(c.fd, c.out.data() + c.out_off, c.out.size() - c.out_off, MSG_NOSIGNAL);
    if (n > 0) {
      c.out_off += static_cast<size_t>(n);
      continue;
    }
    if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
    return false;
  }
  if (c.out_off == c.out.size()) {
    c.out.clear();
    c.out_off = 0;
  } else if (c.out_off > (1 << 20)) {
    c.out.erase(0, c.out_off);
    c.out_off = 0;
  }
  update_interest(s, c);
  return true;
}

void respond(Shard& s, Conn& c, int16_t stream, uint8_t op, const std::string& body) {
  std::string f = frame(VERSION_RESP, stream, op, body);
  if (g_opt.latency_us > 0) {
    s.delayed.push(Delayed{now_us() + g_opt.latency_us, c.fd, s.gen[c.fd], std::move(f)});
    return;
  }
  c.out += f;
}

// [g_db_mu held] the answer of a statement: a conditional write's waits for its Paxos round
// (queued behind the partition's previous round, then --lwt-latency-us on top of the plain
// write latency); anything else goes out after --latency-us as before
void respond_stmt(Shard& s, Conn& c, int16_t stream, uint8_t op, const std::string& body) {
  if (t_lwt_partition.empty()) return respond(s, c, stream, op, body);
  std::string part;
  part.swap(t_lwt_partition);
  int64_t extra = lwt_extra_us();
  if (extra <= 0 && g_opt.latency_us <= 0) return respond(s, c, stream, op, body);
  int64_t now = now_us();
  int64_t& busy = g_paxos_busy[part];
  int64_t start = now;
  if (busy > now) {
    start = busy;
    ++g_db.stats.lwt_waits;  // queued behind another round on the partition
  }
  int64_t done = start + g_opt.latency_us + extra;
  busy = done;
  if (g_paxos_busy.size() > 200000) {  // forget partitions whose last round is long over
    for (auto it = g_paxos_busy.begin(); it != g_paxos_busy.end();) {
      if (it->second < now) it = g_paxos_busy.erase(it);
      else ++it;
    }
  }
  s.delayed.push(Delayed{done, c.fd, s.gen[c.fd], frame(VERSION_RESP, stream, op, body)});
}

// Scylla "biased-token-round-robin": shard of a Murmur3 token.
int shard_of_token(int64_t token) {
  int n = std::max(1, g_opt.shards);
  uint64_t z = static_cast<uint64_t>(token) + (1ULL << 63);
  z <<= g_opt.ignore_msb;
  return static_cast<int>((static_cast<unsigned __int128>(z) * static_cast<uint64_t>(n)) >> 64);
}

// Parse [query parameters]; fills values; returns flags.
uint8_t read_params(Reader& r, std::vector<Val>& vals, uint16_t& consistency) {
  consistency = r.u16();
  uint8_t flags = r.u8();
  if (flags & QF_VALUES) {
    uint16_t n = r.u16();
    for (uint16_t i = 0; i < n; ++i) {
      if (flags & QF_NAMES) r.string();
      const uint8_t* d;
      int32_t len;
      if (r.bytes(d, len)) vals.emplace_back(std::string(reinterpret_cast<const char*>(d), static_cast<size_t>(len)));
      else vals.emplace_back(std::nullopt);
    }
  }
  if (flags & QF_PAGE_SIZE) r.i32();
  if (flags & QF_PAGING_STATE) {
    const uint8_t* d;
    int32_t len;
    r.bytes(d, len);
  }
  if (flags & QF_SERIAL_CONSISTENCY) r.u16();
  if (flags & QF_DEFAULT_TIMESTAMP) r.i64();
  return flags;
}

Prepared prepare(const std::string& q, const std::string& cur_ks) {
  Parser p(q);
  Prepared pr;
  pr.stmt = p.parse();
  const Stmt& st = pr.stmt;
  std::string ks = st.ks.empty() ? cur_ks : st.ks;
  Table* t = (st.kind == S_INSERT || st.kind == S_UPDATE || st.kind == S_SELECT || st.kind == S_DELETE) ? g_db.find(ks, st.table) : nullptr;
  pr.bind.resize(static_cast<size_t>(st.nbind));
  auto bind_col = [&](const Term& term, const std::string& col) {
    if (term.kind != Term::BIND) return;
    ColSpec cs{ks, st.table, col, ty(T_VARCHAR)};
    if (t) cs.type = t->cols[static_cast<size_t>(col_of(*t, col))].type;
    pr.bind[static_cast<size_t>(term.bind)] = cs;
  };
  if (st.kind == S_INSERT)
    for (size_t i = 0; i < st.cols.size(); ++i) bind_col(st.values[i], st.cols[i]);
  for (auto& s : st.sets) bind_col(s.second, s.first);
  for (auto& c : st.where)
    for (auto& term : c.terms) bind_col(term, c.col);
  for (auto& c : st.ifs)
    for (auto& term : c.terms) bind_col(term, c.col);
  if (t) {
    for (int pkc : t->pk) {
      const std::string& name = t->cols[static_cast<size_t>(pkc)].name;
      for (size_t i = 0; i < pr.bind.size(); ++i)
        if (pr.bind[i].name == name) {
          pr.pk_idx.push_back(static_cast<uint16_t>(i));
          break;
        }
    }
    if (pr.pk_idx.size() != t->pk.size()) pr.pk_idx.clear();
    if (st.kind == S_SELECT && !st.count) pr.result = specs_of(*t, select_cols(*t, st));
    // a conditional (LWT) write prepares with result metadata [applied] alone, as Cassandra
    // does: the not-applied answer carries more columns, so a client that executes it with
    // skip_metadata would decode that row with the wrong shape
    bool conditional = (st.kind == S_UPDATE || st.kind == S_DELETE || st.kind == S_INSERT) &&
                       (st.if_exists || !st.ifs.empty() || (st.kind == S_INSERT && st.if_not_exists));
    if (conditional) pr.result = {applied_spec(*t)};
  } else if (st.kind == S_SELECT || st.kind == S_INSERT || st.kind == S_UPDATE || st.kind == S_DELETE) {
    if (!(ks == "system" || ks.rfind("system", 0) == 0)) throw CqlError(ERR_INVALID, "unconfigured table " + st.table);
  }
  return pr;
}

std::string prepared_body(const std::string& id, const Prepared& pr) {
  Writer w;
  w.i32(RK_PREPARED);
  w.short_bytes(id);
  w.i32(MF_GLOBAL_TABLES_SPEC);
  w.i32(static_cast<int32_t>(pr.bind.size()));
  w.i32(static_cast<int32_t>(pr.pk_idx.size()));
  for (auto i : pr.pk_idx) w.u16(i);
  w.string(pr.stmt.ks);
  w.string(pr.stmt.table);
  for (auto& c : pr.bind) {
    w.string(c.name);
    w.type(c.type);
  }
  if (pr.result.empty()) {
    w.i32(MF_NO_METADATA);
    w.i32(0);
  } else {
    w.i32(MF_GLOBAL_TABLES_SPEC);
    w.i32(static_cast<int32_t>(pr.result.size()));
    w.string(pr.result[0].keyspace);
    w.string(pr.result[0].table);
    for (auto& c : pr.result) {
      w.string(c.name);
      w.type(c.type);
    }
  }
  return w.buf;
}

// Runs one statement and produces (opcode, body).
std::pair<uint8_t, std::string> run_stmt(Conn& c, const Stmt& st, const std::vector<Val>& vals, bool skip_meta) {
  ResultSet rs;
  std::string set_ks, change;
  bool rows = execute(st, vals, c.ks, rs, set_ks, change);
  if (rows) return {OP_RESULT, rows_body(rs, skip_meta)};
  if (!set_ks.empty()) {
    Writer w;
    w.i32(RK_SET_KEYSPACE);
    w.string(set_ks);
    return {OP_RESULT, w.buf};
  }
  if (!change.empty() && change != "DROPPED") {
    std::string ks = st.ks.empty() ? c.ks : st.ks;
    return {OP_RESULT, schema_change_body(change, ks, change == "KEYSPACE" ? "" : st.table)};
  }
  return {OP_RESULT, void_body()};
}

void handle_frame(Shard& sh, Conn& c, const FrameHeader& h, const uint8_t* body) {
  Reader r(body, h.length);
  ++g_db.stats.requests;
  try {
    if ((h.version & 0x7F) != 4) {
      respond(sh, c, h.stream, OP_ERROR, error_body(ERR_PROTOCOL, "Invalid or unsupported protocol version; only v4 is supported"));
      return;
    }
    switch (h.opcode) {
      case OP_OPTIONS: {
        Writer w;
        bool scylla = g_opt.shards > 0;
        w.u16(scylla ? 8 : 2);
        w.string("CQL_VERSION");
        w.string_list({"3.3.1"});
        w.string("COMPRESSION");
        w.string_list({});
        if (scylla) {
          w.string("SCYLLA_SHARD");
          w.string_list({std::to_string(sh.id)});
          w.string("SCYLLA_NR_SHARDS");
          w.string_list({std::to_string(g_opt.shards)});
          w.string("SCYLLA_PARTITIONER");
          w.string_list({"org.apache.cassandra.dht.Murmur3Partitioner"});
          w.string("SCYLLA_SHARDING_ALGORITHM");
          w.string_list({"biased-token-round-robin"});
          w.string("SCYLLA_SHARDING_IGNORE_MSB");
          w.string_list({std::to_string(g_opt.ignore_msb)});
          w.string("SCYLLA_SHARD_AWARE_PORT");
          w.string_list({std::to_string(g_opt.advertise_shard_port >= 0 ? g_opt.advertise_shard_port : g_shard_port)});
        }
        respond(sh, c, h.stream, OP_SUPPORTED, w.buf);
        return;
      }
      case OP_STARTUP: {
        r.string_map();
        c.ready = true;
        if (!g_opt.user.empty()) {
          Writer w;
          w.string("org.apache.cassandra.auth.PasswordAuthenticator");
          respond(sh, c, h.stream, OP_AUTHENTICATE, w.buf);
        } else {
          c.authed = true;
          respond(sh, c, h.stream, OP_READY, std::string());
        }
        return;
      }
      case OP_AUTH_RESPONSE: {
        const uint8_t* d;
        int32_t n;
        std::string tok;
        if (r.bytes(d, n)) tok.assign(reinterpret_cast<const char*>(d), static_cast<size_t>(n));
        // SASL PLAIN: \0user\0password
        size_t a = tok.find('\0'), b = tok.find('\0', a + 1);
        std::string u = a == std::string::npos || b == std::string::npos ? "" : tok.substr(a + 1, b - a - 1);
        std::string p = b == std::string::npos ? "" : tok.substr(b + 1);
        if (u == g_opt.user && p == g_opt.password) {
          c.authed = true;
          Writer w;
          w.null_bytes();
          respond(sh, c, h.stream, OP_AUTH_SUCCESS, w.buf);
        } else {
          respond(sh, c, h.stream, OP_ERROR, error_body(ERR_BAD_CREDENTIALS, "Provided username " + u + " and/or password are incorrect"));
        }
        return;
      }
      case OP_REGISTER:
        r.string_list();
        respond(sh, c, h.stream, OP_READY, std::string());
        return;
      default: break;
    }
    if (!c.ready) throw CqlError(ERR_PROTOCOL, "STARTUP required first");
    if (!c.authed) throw CqlError(ERR_UNAUTHORIZED, "authentication required");
    if (g_opt.error_rate > 0 && (h.opcode == OP_QUERY || h.opcode == OP_EXECUTE || h.opcode == OP_BATCH)) {
      std::uniform_real_distribution<double> u(0, 1);
      if (u(sh.rng) < g_opt.error_rate) {
        ++g_db.stats.injected_errors;
        throw CqlError(ERR_OVERLOADED, "Injected overload (--error-rate)");
      }
    }
    std::lock_guard<std::mutex> lk(g_db_mu);  // the data is shared by every shard
    switch (h.opcode) {
      case OP_QUERY: {
        ++g_db.stats.queries;
        std::string q = r.long_string();
        std::vector<Val> vals;
        uint16_t cl;
        uint8_t flags = read_params(r, vals, cl);
        Parser p(q);
        Stmt st = p.parse();
        t_lwt_partition.clear();
        auto res = run_stmt(c, st, vals, (flags & QF_SKIP_METADATA) != 0);
        respond_stmt(sh, c, h.stream, res.first, res.second);
        return;
      }
      case OP_PREPARE: {
        ++g_db.stats.prepares;
        std::string q = r.long_string();
        std::string id = prepare_id(c.ks, q);
        auto it = g_db.prepared.find(id);
        if (it == g_db.prepared.end()) it = g_db.prepared.emplace(id, prepare(q, c.ks)).first;
        respond(sh, c, h.stream, OP_RESULT, prepared_body(id, it->second));
        return;
      }
      case OP_EXECUTE: {
        ++g_db.stats.executes;
        std::string id = r.short_bytes();
        auto it = g_db.prepared.find(id);
        if (it == g_db.prepared.end()) {
          Writer w;
          w.short_bytes(id);
          respond(sh, c, h.stream, OP_ERROR, error_body(ERR_UNPREPARED, "Prepared query with ID not found", w.buf));
          return;
        }
        std::vector<Val> vals;
        uint16_t cl;
        uint8_t flags = read_params(r, vals, cl);
        if (g_opt.shards > 0 && !it->second.pk_idx.empty()) {
          // did the driver send this to the shard owning the partition? (a miss is a cross-shard hop)
          std::vector<std::string> parts;
          bool full = true;
          for (auto i : it->second.pk_idx) {
            if (i >= vals.size() || !vals[i]) {
              full = false;
              break;
            }
            parts.push_back(*vals[i]);
          }
          if (full) {
            std::string key = composite_routing_key(parts);
            int64_t tok = murmur3_token(reinterpret_cast<const uint8_t*>(key.data()), key.size());
            if (shard_of_token(tok) == sh.id) ++g_db.stats.shard_hits;
            else ++g_db.stats.shard_misses;
          }
        }
        if (vals.size() != it->second.bind.size())
          throw CqlError(ERR_INVALID, "There were " + std::to_string(it->second.bind.size()) + " markers(?) in CQL but " +
                                           std::to_string(vals.size()) + " bound variables");
        std::string saved = c.ks;
        if (!it->second.stmt.ks.empty()) c.ks = it->second.stmt.ks;
        t_lwt_partition.clear();
        auto res = run_stmt(c, it->second.stmt, vals, (flags & QF_SKIP_METADATA) != 0);
        c.ks = saved;
        respond_stmt(sh, c, h.stream, res.first, res.second);
        return;
      }
      case OP_BATCH: {
        ++g_db.stats.batches;
        r.u8();  // type
        uint16_t n = r.u16();
        std::vector<std::pair<Stmt, std::vector<Val>>> items;
        for (uint16_t i = 0; i < n; ++i) {
          uint8_t kind = r.u8();
          Stmt st;
          if (kind == 0) {
            Parser p(r.long_string());
            st = p.parse();
          } else {
            std::string id = r.short_bytes();
            auto it = g_db.prepared.find(id);
            if (it == g_db.prepared.end()) {
              Writer w;
              w.short_bytes(id);
              respond(sh, c, h.stream, OP_ERROR, error_body(ERR_UNPREPARED, "Prepared query with ID not found", w.buf));
              return;
            }
            st = it->second.stmt;
          }
          uint16_t k = r.u16();
          std::vector<Val> vals;
          for (uint16_t j = 0; j < k; ++j) {
            const uint8_t* d;
            int32_t len;
            if (r.bytes(d, len)) vals.emplace_back(std::string(reinterpret_cast<const char*>(d), static_cast<size_t>(len)));
            else vals.emplace_back(std::nullopt);
          }
          items.emplace_back(std::move(st), std::move(vals));
        }
        for (auto& it : items) {
          if (it.first.kind != S_INSERT && it.first.kind != S_UPDATE && it.first.kind != S_DELETE)
            throw CqlError(ERR_INVALID, "only INSERT, UPDATE and DELETE are allowed in a BATCH");
        }
        ResultSet last;
        for (auto& it : items) {
          ResultSet rs;
          std::string sk, ch;
          if (execute(it.first, it.second, c.ks, rs, sk, ch)) last = rs;
        }
        if (!last.cols.empty()) respond(sh, c, h.stream, OP_RESULT, rows_body(last, false));
        else respond(sh, c, h.stream, OP_RESULT, void_body());
        return;
      }
      default: throw CqlError(ERR_PROTOCOL, "unsupported opcode " + std::to_string(h.opcode));
    }
  } catch (const CqlError& e) {
    ++g_db.stats.errors;
    respond(sh, c, h.stream, OP_ERROR, error_body(e.code, e.what()));
  } catch (const ProtocolError& e) {
    ++g_db.stats.errors;
    respond(sh, c, h.stream, OP_ERROR, error_body(ERR_PROTOCOL, e.what()));
  } catch (const std::exception& e) {
    ++g_db.stats.errors;
    respond(sh, c, h.stream, OP_ERROR, error_body(ERR_SERVER, e.what()));
  }
}

bool on_readable(Shard& sh, Conn& c) {
  char buf[1 << 16];
  while (true) {
    ssize_t n = ::recv(c.fd, buf, sizeof buf, 0);
    if (n > 0) {
      c.in.feed(buf, static_cast<size_t>(n));
      FrameHeader h;
      const uint8_t* body;
      try {
        while (c.in.next(h, body)) handle_frame(sh, c, h, body);
      } catch (const ProtocolError&) {
        return false;
      }
      if (static_cast<size_t>(n) < sizeof buf) break;
      continue;
    }
    if (n == 0) return false;
    if (errno == EAGAIN || errno == EWOULDBLOCK) break;
    return false;
  }
  return flush(sh, c);
}

void shard_loop(Shard& s) {
  std::vector<epoll_event> evs(256);
  static bool have_pwait2 = true;
  while (!g_stop) {
    // wait until the next delayed answer is due, with microsecond precision (epoll_pwait2):
    // millisecond epoll timeouts rounded every emulated round trip up to the next ms, which
    // made a 500 µs server twice as slow per request as configured
    int64_t dt_us = 200000;
    if (!s.delayed.empty()) dt_us = std::min<int64_t>(dt_us, std::max<int64_t>(0, s.delayed.top().due - now_us()));
    int n;
    if (have_pwait2) {
      timespec ts{static_cast<time_t>(dt_us / 1000000), static_cast<long>((dt_us % 1000000) * 1000)};
      n = epoll_pwait2(s.epfd, evs.data(), static_cast<int>(evs.size()), &ts, nullptr);
      if (n < 0 && errno == ENOSYS) {
        have_pwait2 = false;
        continue;
      }
    } else {
      n = epoll_wait(s.epfd, evs.data(), static_cast<int>(evs.size()), static_cast<int>((dt_us + 999) / 1000));
    }
    uint64_t dg = g_drop_gen.load();
    if (dg != s.drop_seen) {
      s.drop_seen = dg;
      std::vector<int> fds;
      for (auto& kv : s.conns) fds.push_back(kv.first);
      for (int fd : fds) close_conn(s, fd);
      g_db.stats.dropped += fds.size();
    }
    for (int i = 0; i < n; ++i) {
      int fd = evs[static_cast<size_t>(i)].data.fd;
      if (fd == s.wake) {
        uint64_t v;
        if (read(s.wake, &v, sizeof v) < 0 && errno != EAGAIN) perror("eventfd read");
        std::vector<int> fresh;
        {
          std::lock_guard<std::mutex> lk(s.inbox_mu);
          fresh.swap(s.inbox);
        }
        for (int cfd : fresh) {
          auto c = std::make_unique<Conn>();
          c->fd = cfd;
          epoll_event ev{};
          ev.events = EPOLLIN;
          ev.data.fd = cfd;
          epoll_ctl(s.epfd, EPOLL_CTL_ADD, cfd, &ev);
          s.conns[cfd] = std::move(c);
        }
        continue;
      }
      auto it = s.conns.find(fd);
      if (it == s.conns.end()) continue;
      Conn& c = *it->second;
      bool ok = true;
      if (evs[static_cast<size_t>(i)].events & (EPOLLERR | EPOLLHUP)) ok = false;
      if (ok && (evs[static_cast<size_t>(i)].events & EPOLLIN)) ok = on_readable(s, c);
      if (ok && (evs[static_cast<size_t>(i)].events & EPOLLOUT)) ok = flush(s, c);
      if (!ok) close_conn(s, fd);
    }
    if (!s.delayed.empty()) {
      int64_t t = now_us();
      std::set<int> touched;
      while (!s.delayed.empty() && s.delayed.top().due <= t) {
        const Delayed& d = s.delayed.top();
        auto it = s.conns.find(d.fd);
        if (it != s.conns.end() && s.gen[d.fd] == d.gen) {
          it->second->out += d.bytes;
          touched.insert(d.fd);
        }
        s.delayed.pop();
      }
      for (int fd : touched) {
        auto it = s.conns.find(fd);
        if (it != s.conns.end() && !flush(s, *it->second)) close_conn(s, fd);
      }
    }
  }
}

void hand_over(Shard& s, int cfd) {
  {
    std::lock_guard<std::mutex> lk(s.inbox_mu);
    s.inbox.push_back(cfd);
  }
  uint64_t one = 1;
  if (write(s.wake, &one, sizeof one) < 0) perror("eventfd write");
}

int listen_on(int port, int& bound) {
  int fd = socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons(static_cast<uint16_t>(port));
  if (inet_pton(AF_INET, g_opt.host.c_str(), &addr.sin_addr) != 1) {
    fprintf(stderr, "bad --host\n");
    exit(2);
  }
  if (bind(fd, reinterpret_cast<sockaddr*>(&addr), sizeof addr) != 0 || listen(fd, 1024) != 0) {
    perror("bind/listen");
    exit(1);
  }
  socklen_t alen = sizeof addr;
  getsockname(fd, reinterpret_cast<sockaddr*>(&addr), &alen);
  bound = ntohs(addr.sin_port);
  set_nonblock(fd);
  return fd;
}

void on_signal(int sig) {
  if (sig == SIGUSR1) g_drop = 1;
  else g_stop = 1;
}

void usage() {
  fprintf(stderr,
          "nexus-cqlsrv [--host H] [--port P (0 = ephemeral)] [--user U --password P] [--latency-us N]\n"
          "             [--lwt-latency-us N (extra for a conditional write; default 3 x latency-us)]\n"
          "             [--error-rate F] [--seed N] [--data WAL] [--ready-file PATH] [--dc DC] [--rack R]\n"
          "             [--tokens t1,t2] [--peer host:port:tok1;tok2]... [--exec FILE.cql] [-v]\n"
          "             [--shards N [--shard-aware-port P] [--ignore-msb B] [--advertise-shard-aware-port P]]\n");
}

void exec_file(const std::string& path) {
  FILE* f = fopen(path.c_str(), "r");
  if (!f) {
    perror(path.c_str());
    exit(2);
  }
  std::string text;
  char buf[4096];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) text.append(buf, n);
  fclose(f);
  // split on ';' outside quotes
  std::string cur;
  bool q = false;
  Conn dummy{};
  dummy.ready = dummy.authed = true;
  for (char ch : text) {
    if (ch == '\'') q = !q;
    if (ch == ';' && !q) {
      bool blank = true;
      for (char x : cur) blank = blank && isspace(static_cast<unsigned char>(x));
      if (!blank) {
        Parser p(cur);
        Stmt st = p.parse();
        std::vector<Val> none;
        ResultSet rs;
        std::string sk, chg;
        execute(st, none, dummy.ks, rs, sk, chg);
      }
      cur.clear();
      continue;
    }
    cur.push_back(ch);
  }
}

}  // namespace

int main(int argc, char** argv) {
  std::vector<std::string> exec_files;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&]() -> std::string {
      if (i + 1 >= argc) {
        usage();
        exit(2);
      }
      return argv[++i];
    };
    if (a == "--host") g_opt.host = val();
    else if (a == "--port") g_opt.port = std::stoi(val());
    else if (a == "--user") g_opt.user = val();
    else if (a == "--password") g_opt.password = val();
    else if (a == "--latency-us") g_opt.latency_us = std::stoll(val());
    else if (a == "--lwt-latency-us") g_opt.lwt_latency_us = std::stoll(val());
    else if (a == "--error-rate") g_opt.error_rate = std::stod(val());
    else if (a == "--seed") g_opt.seed = std::stoull(val());
    else if (a == "--data") g_opt.data_file = val();
    else if (a == "--ready-file") g_opt.ready_file = val();
    else if (a == "--dc") g_opt.dc = val();
    else if (a == "--rack") g_opt.rack = val();
    else if (a == "--exec") exec_files.push_back(val());
    else if (a == "--tokens") {
      std::string s = val();
      size_t p = 0;
      while (p <= s.size()) {
        size_t e = s.find(',', p);
        if (e == std::string::npos) e = s.size();
        if (e > p) g_opt.tokens.push_back(s.substr(p, e - p));
        p = e + 1;
      }
    } else if (a == "--peer") g_opt.peers.push_back(val());
    else if (a == "--shards") g_opt.shards = std::stoi(val());
    else if (a == "--shard-aware-port") g_opt.shard_port = std::stoi(val());
    else if (a == "--advertise-shard-aware-port") g_opt.advertise_shard_port = std::stoi(val());
    else if (a == "--ignore-msb") g_opt.ignore_msb = std::stoi(val());
    else if (a == "-v") g_opt.verbose = true;
    else {
      usage();
      return 2;
    }
  }
  signal(SIGPIPE, SIG_IGN);
  struct sigaction sa {};
  sa.sa_handler = on_signal;
  sigaction(SIGTERM, &sa, nullptr);
  sigaction(SIGINT, &sa, nullptr);
  sigaction(SIGUSR1, &sa, nullptr);

  g_db.keyspaces.insert("system");
  if (!g_opt.data_file.empty()) {
    g_db.replay(g_opt.data_file);
    g_db.wal = fopen(g_opt.data_file.c_str(), "ab");
    if (!g_db.wal) {
      perror("open wal");
      return 1;
    }
  }
  for (auto& f : exec_files) {
    try {
      exec_file(f);
    } catch (const std::exception& e) {
      fprintf(stderr, "--exec %s: %s\n", f.c_str(), e.what());
      return 1;
    }
  }

  int lfd = listen_on(g_opt.port, g_opt.port);
  int sfd = -1;
  if (g_opt.shards > 0 && g_opt.shard_port >= 0) sfd = listen_on(g_opt.shard_port, g_shard_port);  // -1: none
  int nshards = std::max(1, g_opt.shards);
  for (int k = 0; k < nshards; ++k) {
    auto sh = std::make_unique<Shard>();
    sh->id = k;
    sh->epfd = epoll_create1(0);
    sh->wake = eventfd(0, EFD_NONBLOCK);
    sh->rng.seed(g_opt.seed + static_cast<uint64_t>(k));
    epoll_event wev{};
    wev.events = EPOLLIN;
    wev.data.fd = sh->wake;
    epoll_ctl(sh->epfd, EPOLL_CTL_ADD, sh->wake, &wev);
    g_shards.push_back(std::move(sh));
  }
  int epfd = epoll_create1(0);
  for (int fd : {lfd, sfd}) {
    if (fd < 0) continue;
    epoll_event lev{};
    lev.events = EPOLLIN;
    lev.data.fd = fd;
    epoll_ctl(epfd, EPOLL_CTL_ADD, fd, &lev);
  }
  if (!g_opt.ready_file.empty()) {
    std::string tmp = g_opt.ready_file + ".tmp";
    FILE* f = fopen(tmp.c_str(), "w");
    if (f) {
      fprintf(f, "%d\n%d\n", g_opt.port, g_shard_port);
      fclose(f);
      rename(tmp.c_str(), g_opt.ready_file.c_str());
    }
  }
  fprintf(stderr, "nexus-cqlsrv listening on %s:%d (shards %d, shard-aware port %d)\n", g_opt.host.c_str(), g_opt.port,
          g_opt.shards, g_shard_port);
  fflush(stderr);
  std::vector<std::thread> threads;
  for (auto& sh : g_shards) threads.emplace_back(shard_loop, std::ref(*sh));

  // acceptor: the regular port spreads connections round-robin over the shards (Scylla
  // picks the least loaded one); the shard-aware port maps source port % shards
  int one = 1;
  size_t rr = 0;
  std::vector<epoll_event> evs(8);
  while (!g_stop) {
    int n = epoll_wait(epfd, evs.data(), static_cast<int>(evs.size()), 200);
    if (g_drop) {
      g_drop = 0;
      ++g_drop_gen;
    }
    for (int i = 0; i < n; ++i) {
      int fd = evs[static_cast<size_t>(i)].data.fd;
      while (true) {
        sockaddr_in peer{};
        socklen_t plen = sizeof peer;
        int cfd = accept(fd, reinterpret_cast<sockaddr*>(&peer), &plen);
        if (cfd < 0) break;
        set_nonblock(cfd);
        setsockopt(cfd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
        ++g_db.stats.connections;
        size_t k = fd == sfd ? static_cast<size_t>(ntohs(peer.sin_port)) % g_shards.size() : rr++ % g_shards.size();
        hand_over(*g_shards[k], cfd);
      }
    }
  }
  for (auto& t : threads) t.join();
  if (g_db.wal) fclose(g_db.wal);
  fprintf(stderr, "nexus-cqlsrv: requests=%llu reads=%llu writes=%llu errors=%llu\n",
          static_cast<unsigned long long>(g_db.stats.requests), static_cast<unsigned long long>(g_db.stats.reads),
          static_cast<unsigned long long>(g_db.stats.writes), static_cast<unsigned long long>(g_db.stats.errors));
  return 0;
}
