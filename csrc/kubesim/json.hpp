// Minimal JSON DOM for nexus-kubesim: parse, edit, serialise.
//
// Numbers keep their source text (the simulator never does arithmetic on object
// fields), strings are stored decoded (UTF-8), objects keep insertion order so a
// re-serialised object matches what the client sent field for field.
#pragma once

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace kjson {

struct ParseError : std::runtime_error {
  explicit ParseError(const char* m) : std::runtime_error(m) {}
};

struct Value {
  enum Type : uint8_t { NUL, BOOL, NUM, STR, ARR, OBJ } t = NUL;
  bool b = false;
  bool escaped = false;  // STR: the source text contained escapes
  uint32_t src_off = 0;  // offset/length in the parsed text: STR the raw contents between the
  uint32_t src_len = 0;  // quotes, others the whole token (lets callers splice instead of re-dump)
  std::string s;  // STR (decoded) or NUM (raw text)
  std::vector<Value> a;
  std::vector<std::pair<std::string, Value>> o;

  static Value str(std::string v) {
    Value x;
    x.t = STR;
    x.s = std::move(v);
    return x;
  }
  static Value object() {
    Value x;
    x.t = OBJ;
    return x;
  }

  const Value* get(std::string_view k) const {
    if (t != OBJ) return nullptr;
    for (auto& kv : o)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  Value* get(std::string_view k) {
    if (t != OBJ) return nullptr;
    for (auto& kv : o)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  // object member, created (as null) when absent; turns a non-object into an object
  Value& at(std::string_view k) {
    if (t != OBJ) {
      *this = object();
    }
    for (auto& kv : o)
      if (kv.first == k) return kv.second;
    o.emplace_back(std::string(k), Value());
    return o.back().second;
  }
  void erase(std::string_view k) {
    for (size_t i = 0; i < o.size(); ++i)
      if (o[i].first == k) {
        o.erase(o.begin() + static_cast<long>(i));
        return;
      }
  }
  std::string_view sv() const { return t == STR ? std::string_view(s) : std::string_view(); }
  // dotted-path string lookup ("metadata.name")
  std::string_view path(std::initializer_list<const char*> keys) const {
    const Value* cur = this;
    for (const char* k : keys) {
      cur = cur->get(k);
      if (!cur) return {};
    }
    return cur->sv();
  }
};

class Parser {
 public:
  Parser(const char* s, size_t n) : s_(s), n_(n) {}
  Value parse() {
    Value v;
    ws();
    value(v, 0);
    ws();
    if (i_ != n_) throw ParseError("trailing data");
    return v;
  }

 private:
  const char* s_;
  size_t n_;
  size_t i_ = 0;

  void ws() {
    while (i_ < n_ && (s_[i_] == ' ' || s_[i_] == '\t' || s_[i_] == '\n' || s_[i_] == '\r')) ++i_;
  }
  char peek() {
    if (i_ >= n_) throw ParseError("unexpected end");
    return s_[i_];
  }
  void expect(char c) {
    if (peek() != c) throw ParseError("unexpected character");
    ++i_;
  }
  void literal(const char* w) {
    size_t k = strlen(w);
    if (i_ + k > n_ || memcmp(s_ + i_, w, k) != 0) throw ParseError("bad literal");
    i_ += k;
  }
  static void utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) {
      out += static_cast<char>(cp);
    } else if (cp < 0x800) {
      out += static_cast<char>(0xC0 | (cp >> 6));
      out += static_cast<char>(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      out += static_cast<char>(0xE0 | (cp >> 12));
      out += static_cast<char>(0x80 | ((cp >> 6) & 0x3F));
      out += static_cast<char>(0x80 | (cp & 0x3F));
    } else {
      out += static_cast<char>(0xF0 | (cp >> 18));
      out += static_cast<char>(0x80 | ((cp >> 12) & 0x3F));
      out += static_cast<char>(0x80 | ((cp >> 6) & 0x3F));
      out += static_cast<char>(0x80 | (cp & 0x3F));
    }
  }
  uint32_t hex4() {
    if (i_ + 4 > n_) throw ParseError("bad \\u escape");
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) {
      char c = s_[i_++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= static_cast<uint32_t>(c - '0');
      else if (c >= 'a' && c <= 'f') v |= static_cast<uint32_t>(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') v |= static_cast<uint32_t>(c - 'A' + 10);
      else throw ParseError("bad \\u escape");
    }
    return v;
  }
  bool string(std::string& out) {
    expect('"');
    size_t run = i_;
    bool esc = false;
    while (true) {
      if (i_ >= n_) throw ParseError("unterminated string");
      char c = s_[i_];
      if (c == '"') {
        out.append(s_ + run, i_ - run);
        ++i_;
        return esc;
      }
      if (static_cast<unsigned char>(c) < 0x20) throw ParseError("control character in string");
      if (c != '\\') {
        ++i_;
        continue;
      }
      out.append(s_ + run, i_ - run);
      esc = true;
      ++i_;
      if (i_ >= n_) throw ParseError("bad escape");
      char e = s_[i_++];
      switch (e) {
        case '"': out += '"'; break;
        case '\\': out += '\\'; break;
        case '/': out += '/'; break;
        case 'b': out += '\b'; break;
        case 'f': out += '\f'; break;
        case 'n': out += '\n'; break;
        case 'r': out += '\r'; break;
        case 't': out += '\t'; break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp <= 0xDBFF && i_ + 6 <= n_ && s_[i_] == '\\' && s_[i_ + 1] == 'u') {
            i_ += 2;
            uint32_t lo = hex4();
            if (lo >= 0xDC00 && lo <= 0xDFFF) cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            else { utf8(out, cp); cp = lo; }
          }
          utf8(out, cp);
          break;
        }
        default: throw ParseError("bad escape");
      }
      run = i_;
    }
  }
  void value(Value& v, int depth) {
    size_t st = i_;
    value_inner(v, depth);
    if (v.t != Value::STR) {  // containers / scalars: the whole token
      v.src_off = static_cast<uint32_t>(st);
      v.src_len = static_cast<uint32_t>(i_ - st);
    }
  }
  void value_inner(Value& v, int depth) {
    if (depth > 128) throw ParseError("nesting too deep");
    char c = peek();
    if (c == '{') {
      v.t = Value::OBJ;
      ++i_;
      ws();
      if (peek() == '}') { ++i_; return; }
      while (true) {
        ws();
        std::string k;
        string(k);
        ws();
        expect(':');
        ws();
        v.o.emplace_back(std::move(k), Value());
        value(v.o.back().second, depth + 1);
        ws();
        char d = peek();
        ++i_;
        if (d == '}') return;
        if (d != ',') throw ParseError("expected ',' or '}'");
      }
    } else if (c == '[') {
      v.t = Value::ARR;
      ++i_;
      ws();
      if (peek() == ']') { ++i_; return; }
      while (true) {
        ws();
        v.a.emplace_back();
        value(v.a.back(), depth + 1);
        ws();
        char d = peek();
        ++i_;
        if (d == ']') return;
        if (d != ',') throw ParseError("expected ',' or ']'");
      }
    } else if (c == '"') {
      v.t = Value::STR;
      size_t st = i_ + 1;
      v.escaped = string(v.s);
      v.src_off = static_cast<uint32_t>(st);
      v.src_len = static_cast<uint32_t>(i_ - 1 - st);
    } else if (c == 't') {
      literal("true");
      v.t = Value::BOOL;
      v.b = true;
    } else if (c == 'f') {
      literal("false");
      v.t = Value::BOOL;
    } else if (c == 'n') {
      literal("null");
    } else {
      size_t st = i_;
      while (i_ < n_ && (isdigit(static_cast<unsigned char>(s_[i_])) || s_[i_] == '-' || s_[i_] == '+' || s_[i_] == '.' ||
                         s_[i_] == 'e' || s_[i_] == 'E'))
        ++i_;
      if (i_ == st) throw ParseError("bad value");
      v.t = Value::NUM;
      v.s.assign(s_ + st, i_ - st);
    }
  }
};

inline Value parse(std::string_view s) { return Parser(s.data(), s.size()).parse(); }

inline void escape(std::string& out, std::string_view s) {
  static const char* hex = "0123456789abcdef";
  out += '"';
  size_t run = 0;
  for (size_t i = 0; i < s.size(); ++i) {
    unsigned char c = static_cast<unsigned char>(s[i]);
    if (c >= 0x20 && c != '"' && c != '\\') continue;
    out.append(s.data() + run, i - run);
    run = i + 1;
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      default:
        out += "\\u00";
        out += hex[c >> 4];
        out += hex[c & 15];
    }
  }
  out.append(s.data() + run, s.size() - run);
  out += '"';
}

inline void dump(const Value& v, std::string& out) {
  switch (v.t) {
    case Value::NUL: out += "null"; break;
    case Value::BOOL: out += v.b ? "true" : "false"; break;
    case Value::NUM: out += v.s; break;
    case Value::STR: escape(out, v.s); break;
    case Value::ARR:
      out += '[';
      for (size_t i = 0; i < v.a.size(); ++i) {
        if (i) out += ',';
        dump(v.a[i], out);
      }
      out += ']';
      break;
    case Value::OBJ:
      out += '{';
      for (size_t i = 0; i < v.o.size(); ++i) {
        if (i) out += ',';
        escape(out, v.o[i].first);
        out += ':';
        dump(v.o[i].second, out);
      }
      out += '}';
      break;
  }
}

inline std::string dump(const Value& v) {
  std::string out;
  out.reserve(512);
  dump(v, out);
  return out;
}

// RFC 7386 JSON merge patch
inline void merge_patch(Value& dst, const Value& patch) {
  if (patch.t != Value::OBJ) {
    dst = patch;
    return;
  }
  if (dst.t != Value::OBJ) dst = Value::object();
  for (auto& kv : patch.o) {
    if (kv.second.t == Value::NUL) {
      dst.erase(kv.first);
    } else {
      merge_patch(dst.at(kv.first), kv.second);
    }
  }
}

}  // namespace kjson
