// Minimal order-preserving JSON DOM for the host-side native tools (OCI runtime spec editing).
//
// OCI config.json files are produced by containerd and consumed by runc; amd-container-runtime
// must edit a few fields and hand everything else through untouched, so this DOM keeps object key
// order and keeps numbers as their original text (no float round-trip of e.g. uid/gid/major/minor
// or 64-bit memory limits).  Host-only C++17, no third-party dependency in the runtime path.
#pragma once

#include <cstdint>
#include <cstdio>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace amdk8s {
namespace json {

struct Value;
using Object = std::vector<std::pair<std::string, Value>>;
using Array = std::vector<Value>;

struct Value {
  enum Type { Null, Bool, Number, String, Arr, Obj } type = Null;
  bool b = false;
  std::string s;  // String payload, or Number's literal text
  std::shared_ptr<Array> a;
  std::shared_ptr<Object> o;

  static Value null() { return Value(); }
  static Value boolean(bool v) { Value x; x.type = Bool; x.b = v; return x; }
  static Value number(long long v) { Value x; x.type = Number; x.s = std::to_string(v); return x; }
  static Value number_text(std::string t) { Value x; x.type = Number; x.s = std::move(t); return x; }
  static Value string(std::string v) { Value x; x.type = String; x.s = std::move(v); return x; }
  static Value array() { Value x; x.type = Arr; x.a = std::make_shared<Array>(); return x; }
  static Value object() { Value x; x.type = Obj; x.o = std::make_shared<Object>(); return x; }

  bool is_obj() const { return type == Obj; }
  bool is_arr() const { return type == Arr; }
  bool is_str() const { return type == String; }

  // object access (nullptr when absent / not an object)
  Value* get(const std::string& k) {
    if (type != Obj) return nullptr;
    for (auto& kv : *o)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  const Value* get(const std::string& k) const { return const_cast<Value*>(this)->get(k); }
  // get-or-create a child of the given type (replaces a wrongly-typed child)
  Value& ensure(const std::string& k, Type t) {
    if (type != Obj) *this = object();
    if (Value* v = get(k)) {
      if (v->type != t) *v = (t == Obj ? object() : t == Arr ? array() : Value());
      return *v;
    }
    o->emplace_back(k, t == Obj ? object() : t == Arr ? array() : Value());
    return o->back().second;
  }
  void set(const std::string& k, Value v) {
    if (type != Obj) *this = object();
    if (Value* cur = get(k)) *cur = std::move(v);
    else o->emplace_back(k, std::move(v));
  }
  long long as_int(long long def = 0) const {
    if (type != Number) return def;
    try { return std::stoll(s); } catch (...) { return def; }
  }
};

class ParseError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

class Parser {
 public:
  explicit Parser(const std::string& t) : t_(t) {}
  Value parse() {
    Value v = value();
    ws();
    if (i_ != t_.size()) fail("trailing characters");
    return v;
  }

 private:
  const std::string& t_;
  size_t i_ = 0;

  [[noreturn]] void fail(const char* what) {
    throw ParseError(std::string("JSON: ") + what + " at offset " + std::to_string(i_));
  }
  void ws() {
    while (i_ < t_.size() && (t_[i_] == ' ' || t_[i_] == '\n' || t_[i_] == '\r' || t_[i_] == '\t')) ++i_;
  }
  bool lit(const char* w) {
    size_t n = std::char_traits<char>::length(w);
    if (t_.compare(i_, n, w) == 0) { i_ += n; return true; }
    return false;
  }
  Value value() {
    ws();
    if (i_ >= t_.size()) fail("unexpected end");
    char c = t_[i_];
    if (c == '{') return obj();
    if (c == '[') return arr();
    if (c == '"') return Value::string(str());
    if (lit("true")) return Value::boolean(true);
    if (lit("false")) return Value::boolean(false);
    if (lit("null")) return Value::null();
    if (c == '-' || (c >= '0' && c <= '9')) return num();
    fail("unexpected character");
  }
  Value num() {
    size_t st = i_;
    if (t_[i_] == '-') ++i_;
    while (i_ < t_.size() && ((t_[i_] >= '0' && t_[i_] <= '9') || t_[i_] == '.' || t_[i_] == 'e' ||
                              t_[i_] == 'E' || t_[i_] == '+' || t_[i_] == '-'))
      ++i_;
    if (i_ == st || (i_ == st + 1 && t_[st] == '-')) fail("bad number");
    return Value::number_text(t_.substr(st, i_ - st));
  }
  static void put_utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) out += (char)cp;
    else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) {
      out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    } else {
      out += (char)(0xF0 | (cp >> 18)); out += (char)(0x80 | ((cp >> 12) & 0x3F));
      out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F));
    }
  }
  uint32_t hex4() {
    if (i_ + 4 > t_.size()) fail("short \\u escape");
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) {
      char c = t_[i_++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad \\u escape");
    }
    return v;
  }
  std::string str() {
    ++i_;  // opening quote
    std::string out;
    while (true) {
      if (i_ >= t_.size()) fail("unterminated string");
      char c = t_[i_++];
      if (c == '"') break;
      if ((unsigned char)c < 0x20) fail("control character in string");
      if (c != '\\') { out += c; continue; }
      if (i_ >= t_.size()) fail("bad escape");
      char e = t_[i_++];
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
          if (cp >= 0xD800 && cp <= 0xDBFF && i_ + 6 <= t_.size() && t_[i_] == '\\' && t_[i_ + 1] == 'u') {
            i_ += 2;
            uint32_t lo = hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          put_utf8(out, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
    return out;
  }
  Value arr() {
    ++i_;
    Value v = Value::array();
    ws();
    if (i_ < t_.size() && t_[i_] == ']') { ++i_; return v; }
    while (true) {
      v.a->push_back(value());
      ws();
      if (i_ >= t_.size()) fail("unterminated array");
      if (t_[i_] == ',') { ++i_; continue; }
      if (t_[i_] == ']') { ++i_; return v; }
      fail("expected , or ]");
    }
  }
  Value obj() {
    ++i_;
    Value v = Value::object();
    ws();
    if (i_ < t_.size() && t_[i_] == '}') { ++i_; return v; }
    while (true) {
      ws();
      if (i_ >= t_.size() || t_[i_] != '"') fail("expected key");
      std::string k = str();
      ws();
      if (i_ >= t_.size() || t_[i_] != ':') fail("expected :");
      ++i_;
      v.o->emplace_back(std::move(k), value());
      ws();
      if (i_ >= t_.size()) fail("unterminated object");
      if (t_[i_] == ',') { ++i_; continue; }
      if (t_[i_] == '}') { ++i_; return v; }
      fail("expected , or }");
    }
  }
};

inline Value parse(const std::string& text) { return Parser(text).parse(); }

inline void escape_into(std::string& out, const std::string& s) {
  out += '"';
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      default:
        if (c < 0x20) {
          char b[8];
          std::snprintf(b, sizeof b, "\\u%04x", c);
          out += b;
        } else {
          out += (char)c;
        }
    }
  }
  out += '"';
}

inline void dump_into(std::string& out, const Value& v) {
  switch (v.type) {
    case Value::Null: out += "null"; break;
    case Value::Bool: out += v.b ? "true" : "false"; break;
    case Value::Number: out += v.s; break;
    case Value::String: escape_into(out, v.s); break;
    case Value::Arr: {
      out += '[';
      bool first = true;
      for (const auto& x : *v.a) {
        if (!first) out += ',';
        first = false;
        dump_into(out, x);
      }
      out += ']';
      break;
    }
    case Value::Obj: {
      out += '{';
      bool first = true;
      for (const auto& kv : *v.o) {
        if (!first) out += ',';
        first = false;
        escape_into(out, kv.first);
        out += ':';
        dump_into(out, kv.second);
      }
      out += '}';
      break;
    }
  }
}

inline std::string dump(const Value& v) {
  std::string out;
  dump_into(out, v);
  return out;
}

}  // namespace json
}  // namespace amdk8s
