// Minimal JSON reader for the oracle (TEST INFRASTRUCTURE ONLY).
// The oracle deliberately does not share code with the product engine.
#pragma once
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace ojson {

struct Value {
  enum Kind { NUL, BOOL, NUM, STR, ARR, OBJ } kind = NUL;
  bool b = false;
  double num = 0;
  long long inum = 0;
  bool is_int = false;
  std::string str;
  std::vector<Value> arr;
  std::map<std::string, Value> obj;

  bool has(const std::string& k) const { return kind == OBJ && obj.count(k) && obj.at(k).kind != NUL; }
  const Value& operator[](const std::string& k) const {
    static Value nul;
    auto it = obj.find(k);
    return it == obj.end() ? nul : it->second;
  }
  const Value& operator[](size_t i) const { return arr.at(i); }
  long long as_int() const { return is_int ? inum : (long long)num; }
  double as_num() const { return is_int ? (double)inum : num; }
  bool truthy() const { return kind == BOOL ? b : (kind == NUM ? as_num() != 0 : false); }
};

class Parser {
 public:
  explicit Parser(const std::string& s) : s_(s) {}
  Value parse() {
    Value v = value();
    ws();
    if (i_ != s_.size()) throw std::runtime_error("json: trailing data");
    return v;
  }

 private:
  const std::string& s_;
  size_t i_ = 0;
  void ws() { while (i_ < s_.size() && isspace((unsigned char)s_[i_])) i_++; }
  Value value() {
    ws();
    if (i_ >= s_.size()) throw std::runtime_error("json: eof");
    char c = s_[i_];
    Value v;
    if (c == '{') {
      v.kind = Value::OBJ;
      i_++;
      ws();
      if (s_[i_] == '}') { i_++; return v; }
      for (;;) {
        ws();
        std::string k = string_();
        ws();
        if (s_[i_++] != ':') throw std::runtime_error("json: expected :");
        v.obj[k] = value();
        ws();
        if (s_[i_] == ',') { i_++; continue; }
        if (s_[i_] == '}') { i_++; break; }
        throw std::runtime_error("json: expected , or }");
      }
      return v;
    }
    if (c == '[') {
      v.kind = Value::ARR;
      i_++;
      ws();
      if (s_[i_] == ']') { i_++; return v; }
      for (;;) {
        v.arr.push_back(value());
        ws();
        if (s_[i_] == ',') { i_++; continue; }
        if (s_[i_] == ']') { i_++; break; }
        throw std::runtime_error("json: expected , or ]");
      }
      return v;
    }
    if (c == '"') { v.kind = Value::STR; v.str = string_(); return v; }
    if (s_.compare(i_, 4, "true") == 0) { i_ += 4; v.kind = Value::BOOL; v.b = true; return v; }
    if (s_.compare(i_, 5, "false") == 0) { i_ += 5; v.kind = Value::BOOL; return v; }
    if (s_.compare(i_, 4, "null") == 0) { i_ += 4; return v; }
    size_t st = i_;
    bool isint = true;
    if (s_[i_] == '-') i_++;
    while (i_ < s_.size() && (isdigit((unsigned char)s_[i_]) || s_[i_] == '.' || s_[i_] == 'e' ||
                              s_[i_] == 'E' || s_[i_] == '+' || s_[i_] == '-')) {
      if (!isdigit((unsigned char)s_[i_])) isint = false;
      i_++;
    }
    std::string t = s_.substr(st, i_ - st);
    v.kind = Value::NUM;
    v.is_int = isint;
    if (isint) v.inum = strtoll(t.c_str(), nullptr, 10);
    v.num = strtod(t.c_str(), nullptr);
    return v;
  }
  std::string string_() {
    if (s_[i_] != '"') throw std::runtime_error("json: expected string");
    i_++;
    std::string out;
    while (s_[i_] != '"') {
      if (s_[i_] == '\\') {
        i_++;
        char e = s_[i_++];
        if (e == 'n') out += '\n';
        else if (e == 't') out += '\t';
        else if (e == 'u') { out += '?'; i_ += 4; }
        else out += e;
      } else {
        out += s_[i_++];
      }
    }
    i_++;
    return out;
  }
};

inline Value parse(const std::string& s) { return Parser(s).parse(); }

}  // namespace ojson
