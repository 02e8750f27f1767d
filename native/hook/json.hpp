// Minimal JSON value / parser / writer for the OCI hook (no third-party deps).
// Objects keep insertion order so rewritten config.json files stay diffable.
#pragma once

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace mj {

class Value {
 public:
  enum Type { Null, Bool, Number, String, Array, Object };

  Value() : t_(Null) {}
  Value(bool b) : t_(Bool), b_(b) {}
  Value(double d) : t_(Number), d_(d) {}
  Value(int i) : t_(Number), d_(i) {}
  Value(long i) : t_(Number), d_((double)i) {}
  Value(long long i) : t_(Number), d_((double)i) {}
  Value(unsigned i) : t_(Number), d_(i) {}
  Value(unsigned long i) : t_(Number), d_((double)i) {}
  Value(unsigned long long i) : t_(Number), d_((double)i) {}
  Value(const char* s) : t_(String), s_(s) {}
  Value(std::string s) : t_(String), s_(std::move(s)) {}

  static Value array() {
    Value v;
    v.t_ = Array;
    return v;
  }
  static Value object() {
    Value v;
    v.t_ = Object;
    return v;
  }

  Type type() const { return t_; }
  bool is_null() const { return t_ == Null; }
  bool is_object() const { return t_ == Object; }
  bool is_array() const { return t_ == Array; }
  bool is_string() const { return t_ == String; }
  bool is_number() const { return t_ == Number; }
  bool is_bool() const { return t_ == Bool; }

  const std::string& str() const { return s_; }
  double num() const { return d_; }
  bool boolean() const { return b_; }

  // array
  std::vector<Value>& arr() { return a_; }
  const std::vector<Value>& arr() const { return a_; }
  void push(Value v) {
    if (t_ == Null) t_ = Array;
    a_.push_back(std::move(v));
  }

  // object
  std::vector<std::pair<std::string, Value>>& items() { return o_; }
  const std::vector<std::pair<std::string, Value>>& items() const { return o_; }
  bool has(const std::string& k) const {
    for (auto& kv : o_)
      if (kv.first == k) return true;
    return false;
  }
  const Value* find(const std::string& k) const {
    for (auto& kv : o_)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  Value* find(const std::string& k) {
    for (auto& kv : o_)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  Value& operator[](const std::string& k) {
    if (t_ == Null) t_ = Object;
    for (auto& kv : o_)
      if (kv.first == k) return kv.second;
    o_.emplace_back(k, Value());
    return o_.back().second;
  }

  std::string dump(int indent = 2) const {
    std::string out;
    write(out, indent, 0);
    return out;
  }

 private:
  static void esc(std::string& out, const std::string& s) {
    out += '"';
    for (unsigned char c : s) {
      switch (c) {
        case '"': out += "\\\""; break;
        case '\\': out += "\\\\"; break;
        case '\n': out += "\\n"; break;
        case '\r': out += "\\r"; break;
        case '\t': out += "\\t"; break;
        default:
          if (c < 0x20) {
            char b[8];
            snprintf(b, sizeof(b), "\\u%04x", c);
            out += b;
          } else {
            out += (char)c;
          }
      }
    }
    out += '"';
  }
  void nl(std::string& out, int indent, int depth) const {
    if (indent <= 0) return;
    out += '\n';
    out.append((size_t)(indent * depth), ' ');
  }
  void write(std::string& out, int indent, int depth) const {
    switch (t_) {
      case Null: out += "null"; break;
      case Bool: out += b_ ? "true" : "false"; break;
      case Number: {
        char b[64];
        if (std::isfinite(d_) && d_ == std::floor(d_) && std::fabs(d_) < 9.007199254740992e15)
          snprintf(b, sizeof(b), "%lld", (long long)d_);
        else
          snprintf(b, sizeof(b), "%.17g", d_);
        out += b;
        break;
      }
      case String: esc(out, s_); break;
      case Array:
        if (a_.empty()) {
          out += "[]";
          break;
        }
        out += '[';
        for (size_t i = 0; i < a_.size(); ++i) {
          if (i) out += ',';
          nl(out, indent, depth + 1);
          a_[i].write(out, indent, depth + 1);
        }
        nl(out, indent, depth);
        out += ']';
        break;
      case Object:
        if (o_.empty()) {
          out += "{}";
          break;
        }
        out += '{';
        for (size_t i = 0; i < o_.size(); ++i) {
          if (i) out += ',';
          nl(out, indent, depth + 1);
          esc(out, o_[i].first);
          out += indent > 0 ? ": " : ":";
          o_[i].second.write(out, indent, depth + 1);
        }
        nl(out, indent, depth);
        out += '}';
        break;
    }
  }

  Type t_;
  bool b_ = false;
  double d_ = 0;
  std::string s_;
  std::vector<Value> a_;
  std::vector<std::pair<std::string, Value>> o_;
};

class Parser {
 public:
  explicit Parser(const std::string& s) : s_(s) {}
  Value parse() {
    Value v = value(0);
    ws();
    if (i_ != s_.size()) fail("trailing characters");
    return v;
  }

 private:
  [[noreturn]] void fail(const char* m) { throw std::runtime_error(std::string("json: ") + m + " at offset " + std::to_string(i_)); }
  void ws() {
    while (i_ < s_.size() && (s_[i_] == ' ' || s_[i_] == '\n' || s_[i_] == '\t' || s_[i_] == '\r')) ++i_;
  }
  bool lit(const char* w) {
    size_t n = strlen_(w);
    if (s_.compare(i_, n, w) == 0) {
      i_ += n;
      return true;
    }
    return false;
  }
  static size_t strlen_(const char* w) {
    size_t n = 0;
    while (w[n]) ++n;
    return n;
  }
  Value value(int depth) {
    if (depth > 256) fail("nesting too deep");
    ws();
    if (i_ >= s_.size()) fail("unexpected end");
    char c = s_[i_];
    if (c == '{') return object(depth);
    if (c == '[') return array(depth);
    if (c == '"') return Value(string());
    if (lit("true")) return Value(true);
    if (lit("false")) return Value(false);
    if (lit("null")) return Value();
    return number();
  }
  Value object(int depth) {
    Value v = Value::object();
    ++i_;
    ws();
    if (i_ < s_.size() && s_[i_] == '}') {
      ++i_;
      return v;
    }
    for (;;) {
      ws();
      if (i_ >= s_.size() || s_[i_] != '"') fail("expected key");
      std::string k = string();
      ws();
      if (i_ >= s_.size() || s_[i_] != ':') fail("expected ':'");
      ++i_;
      v[k] = value(depth + 1);
      ws();
      if (i_ < s_.size() && s_[i_] == ',') {
        ++i_;
        continue;
      }
      if (i_ < s_.size() && s_[i_] == '}') {
        ++i_;
        return v;
      }
      fail("expected ',' or '}'");
    }
  }
  Value array(int depth) {
    Value v = Value::array();
    ++i_;
    ws();
    if (i_ < s_.size() && s_[i_] == ']') {
      ++i_;
      return v;
    }
    for (;;) {
      v.push(value(depth + 1));
      ws();
      if (i_ < s_.size() && s_[i_] == ',') {
        ++i_;
        continue;
      }
      if (i_ < s_.size() && s_[i_] == ']') {
        ++i_;
        return v;
      }
      fail("expected ',' or ']'");
    }
  }
  static void utf8(std::string& out, unsigned cp) {
    if (cp < 0x80) {
      out += (char)cp;
    } else if (cp < 0x800) {
      out += (char)(0xC0 | (cp >> 6));
      out += (char)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      out += (char)(0xE0 | (cp >> 12));
      out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    } else {
      out += (char)(0xF0 | (cp >> 18));
      out += (char)(0x80 | ((cp >> 12) & 0x3F));
      out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    }
  }
  unsigned hex4() {
    if (i_ + 4 > s_.size()) fail("bad \\u escape");
    unsigned v = 0;
    for (int k = 0; k < 4; ++k) {
      char c = s_[i_++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= (unsigned)(c - '0');
      else if (c >= 'a' && c <= 'f') v |= (unsigned)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') v |= (unsigned)(c - 'A' + 10);
      else fail("bad hex digit");
    }
    return v;
  }
  std::string string() {
    std::string out;
    ++i_;
    while (i_ < s_.size()) {
      char c = s_[i_++];
      if (c == '"') return out;
      if ((unsigned char)c < 0x20) fail("control character in string");
      if (c != '\\') {
        out += c;
        continue;
      }
      if (i_ >= s_.size()) break;
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
          unsigned cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00 && i_ + 6 <= s_.size() && s_[i_] == '\\' && s_[i_ + 1] == 'u') {
            i_ += 2;
            unsigned lo = hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          utf8(out, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
    fail("unterminated string");
  }
  Value number() {
    size_t st = i_;
    if (i_ < s_.size() && (s_[i_] == '-' || s_[i_] == '+')) ++i_;
    while (i_ < s_.size() && ((s_[i_] >= '0' && s_[i_] <= '9') || s_[i_] == '.' || s_[i_] == 'e' || s_[i_] == 'E' ||
                              s_[i_] == '-' || s_[i_] == '+'))
      ++i_;
    if (st == i_) fail("unexpected character");
    std::string tok = s_.substr(st, i_ - st);
    char* end = nullptr;
    double d = strtod(tok.c_str(), &end);
    if (!end || *end) fail("bad number");
    return Value(d);
  }

  const std::string& s_;
  size_t i_ = 0;
};

inline Value parse(const std::string& s) { return Parser(s).parse(); }

}  // namespace mj
