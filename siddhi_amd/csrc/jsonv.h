// Small JSON DOM used to read NFA programs at engine creation (host only).
#pragma once
#include <cctype>
#include <cstring>
#include <cstdlib>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

namespace shp {

struct JV {
  enum T { NIL, BOOLEAN, NUMBER, STRING, ARRAY, OBJECT } t = NIL;
  bool bv = false;
  double dv = 0;
  long long iv = 0;
  bool integral = false;
  std::string sv;
  std::vector<JV> av;
  std::vector<std::pair<std::string, JV>> ov;

  const JV& get(const char* k) const {
    static const JV nil;
    for (auto& p : ov)
      if (p.first == k) return p.second;
    return nil;
  }
  bool present(const char* k) const { return get(k).t != NIL; }
  long long i() const { return integral ? iv : (long long)dv; }
  double d() const { return integral ? (double)iv : dv; }
  bool b() const { return t == BOOLEAN ? bv : (t == NUMBER && d() != 0); }
  size_t size() const { return av.size(); }
  const JV& operator[](size_t k) const { return av.at(k); }
};

class JReader {
 public:
  explicit JReader(const char* s) : p_(s) {}
  JV read() {
    JV v = val();
    skip();
    if (*p_) throw std::runtime_error("program json: trailing characters");
    return v;
  }

 private:
  const char* p_;
  void skip() {
    while (*p_ && isspace((unsigned char)*p_)) ++p_;
  }
  void expect(char c) {
    skip();
    if (*p_ != c) throw std::runtime_error(std::string("program json: expected ") + c);
    ++p_;
  }
  std::string str() {
    expect('"');
    std::string o;
    while (*p_ && *p_ != '"') {
      if (*p_ == '\\') {
        ++p_;
        switch (*p_) {
          case 'n': o += '\n'; break;
          case 't': o += '\t'; break;
          case 'u': o += '?'; p_ += 4; break;
          default: o += *p_;
        }
        ++p_;
      } else {
        o += *p_++;
      }
    }
    if (*p_ != '"') throw std::runtime_error("program json: unterminated string");
    ++p_;
    return o;
  }
  JV val() {
    skip();
    JV v;
    if (*p_ == '{') {
      ++p_;
      v.t = JV::OBJECT;
      skip();
      if (*p_ == '}') { ++p_; return v; }
      while (true) {
        std::string k = str();
        expect(':');
        v.ov.emplace_back(k, val());
        skip();
        if (*p_ == ',') { ++p_; continue; }
        expect('}');
        return v;
      }
    }
    if (*p_ == '[') {
      ++p_;
      v.t = JV::ARRAY;
      skip();
      if (*p_ == ']') { ++p_; return v; }
      while (true) {
        v.av.push_back(val());
        skip();
        if (*p_ == ',') { ++p_; continue; }
        expect(']');
        return v;
      }
    }
    if (*p_ == '"') { v.t = JV::STRING; v.sv = str(); return v; }
    if (!strncmp(p_, "true", 4)) { p_ += 4; v.t = JV::BOOLEAN; v.bv = true; return v; }
    if (!strncmp(p_, "false", 5)) { p_ += 5; v.t = JV::BOOLEAN; return v; }
    if (!strncmp(p_, "null", 4)) { p_ += 4; return v; }
    char* end = nullptr;
    const char* st = p_;
    bool integral = true;
    for (const char* q = p_; *q && (isdigit((unsigned char)*q) || strchr("+-.eE", *q)); ++q)
      if (!isdigit((unsigned char)*q) && !(q == st && *q == '-')) integral = false;
    v.t = JV::NUMBER;
    v.integral = integral;
    if (integral) {
      v.iv = strtoll(p_, &end, 10);
      v.dv = (double)v.iv;
    } else {
      v.dv = strtod(p_, &end);
    }
    if (end == p_) throw std::runtime_error("program json: bad value");
    p_ = end;
    return v;
  }
};

}  // namespace shp
