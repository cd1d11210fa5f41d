// Minimal JSON value / parser / serializer for the native node tools (OCI
// config.json, hooks.d specs, CDI specs, topology output).  Object key order is
// preserved (vector of pairs) so rewritten config.json files diff cleanly.
#pragma once
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace kgcjson {

struct Value;
using Object = std::vector<std::pair<std::string, Value>>;
using Array = std::vector<Value>;

struct Value {
  enum Kind { Null, Bool, Number, String, Arr, Obj } kind = Null;
  bool b = false;
  double num = 0;
  bool is_int = false;
  int64_t i = 0;
  std::string s;
  std::shared_ptr<Array> a;
  std::shared_ptr<Object> o;

  Value() = default;
  static Value null() { return Value(); }
  static Value boolean(bool v) { Value x; x.kind = Bool; x.b = v; return x; }
  static Value integer(int64_t v) { Value x; x.kind = Number; x.is_int = true; x.i = v; x.num = (double)v; return x; }
  static Value number(double v) { Value x; x.kind = Number; x.num = v; return x; }
  static Value str(const std::string& v) { Value x; x.kind = String; x.s = v; return x; }
  static Value array() { Value x; x.kind = Arr; x.a = std::make_shared<Array>(); return x; }
  static Value object() { Value x; x.kind = Obj; x.o = std::make_shared<Object>(); return x; }

  bool is_obj() const { return kind == Obj; }
  bool is_arr() const { return kind == Arr; }
  bool is_str() const { return kind == String; }

  Value* get(const std::string& k) {
    if (kind != Obj) return nullptr;
    for (auto& kv : *o) if (kv.first == k) return &kv.second;
    return nullptr;
  }
  const Value* get(const std::string& k) const {
    if (kind != Obj) return nullptr;
    for (auto& kv : *o) if (kv.first == k) return &kv.second;
    return nullptr;
  }
  // get-or-create child (object member), converting a null into an object
  Value& at(const std::string& k) {
    if (kind == Null) { kind = Obj; o = std::make_shared<Object>(); }
    if (kind != Obj) throw std::runtime_error("json: not an object at key " + k);
    for (auto& kv : *o) if (kv.first == k) return kv.second;
    o->emplace_back(k, Value());
    return o->back().second;
  }
  void set(const std::string& k, Value v) { at(k) = std::move(v); }
  void push(Value v) {
    if (kind == Null) { kind = Arr; a = std::make_shared<Array>(); }
    a->push_back(std::move(v));
  }
  std::string as_str(const std::string& dflt = "") const { return kind == String ? s : dflt; }
  int64_t as_int(int64_t dflt = 0) const { return kind == Number ? (is_int ? i : (int64_t)num) : dflt; }
};

class Parser {
 public:
  explicit Parser(const std::string& t) : t_(t) {}
  Value parse() {
    Value v = value();
    ws();
    if (p_ != t_.size()) fail("trailing characters");
    return v;
  }

 private:
  const std::string& t_;
  size_t p_ = 0;
  [[noreturn]] void fail(const std::string& m) {
    throw std::runtime_error("json parse error at " + std::to_string(p_) + ": " + m);
  }
  void ws() { while (p_ < t_.size() && (t_[p_] == ' ' || t_[p_] == '\n' || t_[p_] == '\t' || t_[p_] == '\r')) ++p_; }
  bool eat(char c) { ws(); if (p_ < t_.size() && t_[p_] == c) { ++p_; return true; } return false; }
  void expect(char c) { if (!eat(c)) fail(std::string("expected '") + c + "'"); }
  Value value() {
    ws();
    if (p_ >= t_.size()) fail("unexpected end");
    char c = t_[p_];
    if (c == '{') return object();
    if (c == '[') return array();
    if (c == '"') return Value::str(string());
    if (t_.compare(p_, 4, "true") == 0) { p_ += 4; return Value::boolean(true); }
    if (t_.compare(p_, 5, "false") == 0) { p_ += 5; return Value::boolean(false); }
    if (t_.compare(p_, 4, "null") == 0) { p_ += 4; return Value::null(); }
    return number();
  }
  Value object() {
    expect('{');
    Value v = Value::object();
    if (eat('}')) return v;
    do {
      ws();
      std::string k = string();
      expect(':');
      v.o->emplace_back(k, value());
    } while (eat(','));
    expect('}');
    return v;
  }
  Value array() {
    expect('[');
    Value v = Value::array();
    if (eat(']')) return v;
    do { v.a->push_back(value()); } while (eat(','));
    expect(']');
    return v;
  }
  static void utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) out += (char)cp;
    else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) { out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F)); }
    else { out += (char)(0xF0 | (cp >> 18)); out += (char)(0x80 | ((cp >> 12) & 0x3F)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F)); }
  }
  std::string string() {
    if (p_ >= t_.size() || t_[p_] != '"') fail("expected string");
    ++p_;
    std::string out;
    while (true) {
      if (p_ >= t_.size()) fail("unterminated string");
      char c = t_[p_++];
      if (c == '"') break;
      if (c != '\\') { out += c; continue; }
      if (p_ >= t_.size()) fail("bad escape");
      char e = t_[p_++];
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
          if (p_ + 4 > t_.size()) fail("bad \\u");
          uint32_t cp = std::stoul(t_.substr(p_, 4), nullptr, 16);
          p_ += 4;
          if (cp >= 0xD800 && cp < 0xDC00 && p_ + 6 <= t_.size() && t_[p_] == '\\' && t_[p_ + 1] == 'u') {
            uint32_t lo = std::stoul(t_.substr(p_ + 2, 4), nullptr, 16);
            p_ += 6;
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          utf8(out, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
    return out;
  }
  Value number() {
    size_t st = p_;
    bool isf = false;
    if (t_[p_] == '-') ++p_;
    while (p_ < t_.size() && (isdigit((unsigned char)t_[p_]) || t_[p_] == '.' || t_[p_] == 'e' ||
                              t_[p_] == 'E' || t_[p_] == '+' || t_[p_] == '-')) {
      if (t_[p_] == '.' || t_[p_] == 'e' || t_[p_] == 'E') isf = true;
      ++p_;
    }
    std::string n = t_.substr(st, p_ - st);
    if (n.empty() || n == "-") fail("bad number");
    if (!isf) return Value::integer(std::stoll(n));
    return Value::number(std::stod(n));
  }
};

inline Value parse(const std::string& t) { return Parser(t).parse(); }

inline void dump_str(std::ostringstream& os, const std::string& s) {
  os << '"';
  for (unsigned char c : s) {
    switch (c) {
      case '"': os << "\\\""; break;
      case '\\': os << "\\\\"; break;
      case '\n': os << "\\n"; break;
      case '\r': os << "\\r"; break;
      case '\t': os << "\\t"; break;
      default:
        if (c < 0x20) { char b[8]; snprintf(b, sizeof b, "\\u%04x", c); os << b; }
        else os << c;
    }
  }
  os << '"';
}

inline void dump(std::ostringstream& os, const Value& v, int indent, int depth) {
  auto nl = [&](int d) { if (indent) { os << '\n'; for (int i = 0; i < d * indent; ++i) os << ' '; } };
  switch (v.kind) {
    case Value::Null: os << "null"; break;
    case Value::Bool: os << (v.b ? "true" : "false"); break;
    case Value::Number:
      if (v.is_int) os << v.i;
      else { char b[64]; snprintf(b, sizeof b, "%.17g", v.num); os << b; }
      break;
    case Value::String: dump_str(os, v.s); break;
    case Value::Arr: {
      os << '[';
      for (size_t k = 0; k < v.a->size(); ++k) {
        if (k) os << ',';
        nl(depth + 1);
        dump(os, (*v.a)[k], indent, depth + 1);
      }
      if (!v.a->empty()) nl(depth);
      os << ']';
      break;
    }
    case Value::Obj: {
      os << '{';
      for (size_t k = 0; k < v.o->size(); ++k) {
        if (k) os << ',';
        nl(depth + 1);
        dump_str(os, (*v.o)[k].first);
        os << (indent ? ": " : ":");
        dump(os, (*v.o)[k].second, indent, depth + 1);
      }
      if (!v.o->empty()) nl(depth);
      os << '}';
      break;
    }
  }
}

inline std::string dump(const Value& v, int indent = 0) {
  std::ostringstream os;
  dump(os, v, indent, 0);
  return os.str();
}

}  // namespace kgcjson
