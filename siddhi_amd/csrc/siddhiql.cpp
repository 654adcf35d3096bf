// siddhi-hip: SiddhiQL -> NFA program JSON inside the library (host code only).
//
// The Java host keeps SiddhiQL and its AST (north_star); what it hands the engine is the query
// text.  This file lowers that text to the program JSON shp_engine_create reads, following the
// reference's build-time wiring:
//   * the grammar subset of the state path: SiddhiQL.g4:200-345 (pattern / sequence sources),
//     built into trees the way SiddhiQLBaseVisitorImpl.java:760-1120 builds them (`a -> b -> c`
//     is left-associative Next; `A and not B` is Logical(absent B, AND, A), State.java:52-69);
//   * state ids in MetaStateEvent order = the recursive parse order of
//     StateInputStreamParser.parse (core/util/parser/StateInputStreamParser.java:148-408), a
//     logical element parsing its second operand first (:339-352);
//   * variable chain indexes per ExpressionParser.parseVariable (ExpressionParser.java:1253-1416):
//     filters default to CURRENT, selectors to 0, `[last-k]` becomes CURRENT-k except on the
//     filter's own state; an index-less selector reference to a count state is multi-valued;
//   * arithmetic result types per ExpressionParser.java:1425-1446.
// It is the C++ form of siddhi_amd/query/siddhiql.py + compiler.py and emits the same bytes
// (json.dumps(sort_keys=True) layout, Python float repr): tests/test_siddhiql_native.py checks
// that on every transcribed reference fixture.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/siddhi_hip.h"

namespace shpql {

struct ParseError : std::runtime_error {  // SiddhiParserException
  using std::runtime_error::runtime_error;
};
struct CreationError : std::runtime_error {  // SiddhiAppCreationException
  using std::runtime_error::runtime_error;
};

// ------------------------------------------------------------------ tokens (siddhiql.py _TOKEN_RE)
enum TK { T_STRL, T_NUM, T_ID, T_OP, T_EOF };
struct Tok {
  TK kind;
  std::string text;
  size_t pos;
};

static bool is_ws(unsigned char c) { return c == ' ' || (c >= 9 && c <= 13) || (c >= 0x1c && c <= 0x1f); }
static bool is_dig(char c) { return c >= '0' && c <= '9'; }
static bool is_idstart(char c) { return (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || c == '_'; }
static bool is_idchar(char c) { return is_idstart(c) || is_dig(c); }

static std::vector<Tok> tokenize(const std::string& s) {
  std::vector<Tok> out;
  size_t p = 0, n = s.size();
  while (p < n) {
    const char c = s[p];
    // ws: \s+ | --[^\n]* | /\*.*?\*/
    if (is_ws((unsigned char)c)) {
      while (p < n && is_ws((unsigned char)s[p])) p++;
      continue;
    }
    if (c == '-' && p + 1 < n && s[p + 1] == '-') {
      while (p < n && s[p] != '\n') p++;
      continue;
    }
    if (c == '/' && p + 1 < n && s[p + 1] == '*') {
      const size_t e = s.find("*/", p + 2);
      if (e != std::string::npos) {
        p = e + 2;
        continue;
      }
      // no closing */: the alternation falls through to the op '/'
    }
    // str: '[^']*' | "[^"]*"
    if (c == '\'' || c == '"') {
      const size_t e = s.find(c, p + 1);
      if (e != std::string::npos) {
        out.push_back({T_STRL, s.substr(p, e + 1 - p), p});
        p = e + 1;
        continue;
      }
    }
    // num: (\d+\.\d*|\.\d+|\d+)([eE][-+]?\d+)?[lLfFdD]?
    {
      size_t q = p;
      bool ok = false;
      if (is_dig(s[q])) {
        while (q < n && is_dig(s[q])) q++;
        ok = true;
        if (q < n && s[q] == '.') {
          q++;
          while (q < n && is_dig(s[q])) q++;
        }
      } else if (c == '.' && p + 1 < n && is_dig(s[p + 1])) {
        q = p + 1;
        while (q < n && is_dig(s[q])) q++;
        ok = true;
      }
      if (ok) {
        if (q < n && (s[q] == 'e' || s[q] == 'E')) {
          size_t r = q + 1;
          if (r < n && (s[r] == '-' || s[r] == '+')) r++;
          if (r < n && is_dig(s[r])) {
            while (r < n && is_dig(s[r])) r++;
            q = r;
          }
        }
        if (q < n && strchr("lLfFdD", s[q]) && s[q]) q++;
        out.push_back({T_NUM, s.substr(p, q - p), p});
        p = q;
        continue;
      }
    }
    if (is_idstart(c)) {
      size_t q = p + 1;
      while (q < n && is_idchar(s[q])) q++;
      out.push_back({T_ID, s.substr(p, q - p), p});
      p = q;
      continue;
    }
    static const char* two[] = {"->", "==", "!=", ">=", "<="};
    bool got = false;
    for (const char* t : two)
      if (p + 1 < n && s[p] == t[0] && s[p + 1] == t[1]) {
        out.push_back({T_OP, std::string(t), p});
        p += 2;
        got = true;
        break;
      }
    if (got) continue;
    if (c && strchr("-+*/%<>=(),;[]:.@#!?", c)) {
      out.push_back({T_OP, std::string(1, c), p});
      p++;
      continue;
    }
    throw ParseError("unexpected character at " + std::to_string(p));
  }
  out.push_back({T_EOF, "", p});
  return out;
}

static std::string lower(std::string s) {
  for (auto& c : s) c = (char)tolower((unsigned char)c);
  return s;
}

// ------------------------------------------------------------------ AST (siddhiql.py)
// A constant's value: Python int, float, str, bool or None
struct Val {
  enum K { NONE, INT, FLT, STR, BOOL } k = NONE;
  int64_t i = 0;
  double d = 0;
  std::string s;
  bool b = false;
};

struct Expr;
using EP = std::shared_ptr<Expr>;
struct Expr {
  std::string op;
  std::vector<EP> args;
  Val value;          // const value; cmp name (STR); function name (STR)
  std::string vtype;  // const type
  bool has_ref = false, has_attr = false, has_index = false;
  std::string stream_ref, attr;
  int64_t index = 0;
};

struct BasicSource {
  bool has_ref = false;
  std::string ref, stream;
  std::vector<EP> filters;
};

struct StateNode;
using SP = std::shared_ptr<StateNode>;
struct StateNode {
  std::string kind;  // stream | absent | next | every | count | logical
  std::shared_ptr<BasicSource> src;
  bool has_waiting = false;
  int64_t waiting = 0;
  SP a, b;
  int64_t mn = -1, mx = -1;
  std::string logical;
};

struct SelectItem {
  EP expr;
  std::string name;
};

struct StreamDef {
  std::string name;
  std::vector<std::pair<std::string, std::string>> attrs;
};

struct Query {
  std::string name, seq_type;
  SP root;
  bool has_within = false;
  int64_t within = 0;
  std::vector<SelectItem> select;
  bool select_all = false;
  std::string out_stream;
  bool partitioned = false;
  std::vector<std::pair<std::string, std::string>> partition;  // stream -> key attr (dict order)
  std::string output_events = "current";
};

struct App {
  std::vector<StreamDef> streams;  // dict order: first definition's position, last definition's attrs
  std::vector<Query> queries;
  bool playback = false;
  const StreamDef* stream(const std::string& n) const {
    for (auto& s : streams)
      if (s.name == n) return &s;
    return nullptr;
  }
};

static const std::map<std::string, int64_t>& time_units() {
  static const std::map<std::string, int64_t> m = {
      {"millisecond", 1},     {"milliseconds", 1},     {"millisec", 1},     {"millis", 1},      {"ms", 1},
      {"sec", 1000},          {"second", 1000},        {"seconds", 1000},   {"secs", 1000},     {"min", 60000},
      {"minute", 60000},      {"minutes", 60000},      {"mins", 60000},     {"hour", 3600000},  {"hours", 3600000},
      {"day", 86400000},      {"days", 86400000},      {"week", 604800000}, {"weeks", 604800000},
      {"month", 2630000000},  {"months", 2630000000},  {"year", 31556900000}, {"years", 31556900000}};
  return m;
}

static int64_t py_int(const std::string& t) {  // int(text): decimal digits
  if (t.empty()) throw ParseError("expected a number");
  errno = 0;
  char* e = nullptr;
  const long long v = strtoll(t.c_str(), &e, 10);
  if (errno || !e || *e) throw ParseError("integer literal out of range or malformed: " + t);
  return v;
}

// ------------------------------------------------------------------ parser (siddhiql.py Parser)
class Parser {
 public:
  explicit Parser(const std::string& text) : toks_(tokenize(text)) {}

  App parse_app() {
    App app;
    bool has_info = false;
    std::string info;
    while (peek().kind != T_EOF) {
      if (at("@")) {
        std::string name;
        std::vector<std::pair<std::string, std::string>> props;
        annotation(name, props);
        const std::string l = lower(name);
        if (l == "app:playback") {
          app.playback = true;
        } else if (l == "info") {
          has_info = false;
          for (auto& p : props)
            if (p.first == "name") {
              has_info = true;
              info = p.second;
            }
        }
        continue;
      }
      if (at(";")) {
        eat();
        continue;
      }
      if (at("define")) {
        StreamDef sd = define_stream();
        bool found = false;
        for (auto& s : app.streams)
          if (s.name == sd.name) {
            s = sd;  // dict assignment: the name keeps its position, the attributes are replaced
            found = true;
          }
        if (!found) app.streams.push_back(sd);
        continue;
      }
      if (at("partition")) {
        partition(app);
        has_info = false;
        continue;
      }
      if (at("from")) {
        const std::string nm = has_info && !info.empty() ? info : "query" + std::to_string(app.queries.size() + 1);
        app.queries.push_back(query(nm, nullptr));
        has_info = false;
        continue;
      }
      throw ParseError("unsupported construct at " + std::to_string(peek().pos) + ": '" + peek().text + "'");
    }
    return app;
  }

 private:
  std::vector<Tok> toks_;
  size_t i_ = 0;

  const Tok& peek(size_t k = 0) const { return toks_[std::min(i_ + k, toks_.size() - 1)]; }
  bool at(const char* text, size_t k = 0) const {
    const Tok& t = peek(k);
    if (t.kind == T_ID) return lower(t.text) == text;
    return t.text == text;
  }
  const Tok& eat(const char* text = nullptr) {
    const Tok& t = peek();
    if (text && !at(text)) throw ParseError(std::string("expected '") + text + "' at " + std::to_string(t.pos));
    i_++;
    return t;
  }
  bool accept(const char* text) {
    if (at(text)) {
      i_++;
      return true;
    }
    return false;
  }
  std::string ident() {
    const Tok& t = peek();
    if (t.kind != T_ID) throw ParseError("expected identifier at " + std::to_string(t.pos));
    i_++;
    return t.text;
  }
  static std::string strip_quotes(const std::string& s) {  // str.strip("'\"")
    size_t a = 0, b = s.size();
    while (a < b && (s[a] == '\'' || s[a] == '"')) a++;
    while (b > a && (s[b - 1] == '\'' || s[b - 1] == '"')) b--;
    return s.substr(a, b - a);
  }

  void annotation(std::string& name, std::vector<std::pair<std::string, std::string>>& props) {
    eat("@");
    name = ident();
    while (at(":") || at(".")) {
      eat();
      name += ":" + ident();
    }
    auto setp = [&](const std::string& k, const std::string& v, bool setdefault) {
      for (auto& p : props)
        if (p.first == k) {
          if (!setdefault) p.second = v;
          return;
        }
      props.push_back({k, v});
    };
    if (accept("(")) {
      while (!at(")")) {
        if (peek().kind == T_STRL) {
          const std::string t = eat().text;
          setp("_", t.substr(1, t.size() - 2), true);
        } else {
          std::string key = ident();
          while (at(".")) {
            eat();
            key += "." + ident();
          }
          eat("=");
          setp(key, strip_quotes(eat().text), false);
        }
        accept(",");
      }
      eat(")");
    }
  }

  StreamDef define_stream() {
    eat("define");
    eat("stream");
    StreamDef sd;
    sd.name = ident();
    eat("(");
    for (;;) {
      const std::string an = ident();
      const std::string at_ = lower(ident());
      static const char* types[] = {"int", "long", "float", "double", "bool", "string", "object"};
      bool ok = false;
      for (const char* t : types) ok = ok || at_ == t;
      if (!ok) throw ParseError("unknown type " + at_);
      sd.attrs.push_back({an, at_});
      if (!accept(",")) break;
    }
    eat(")");
    return sd;
  }

  void partition(App& app) {
    eat("partition");
    eat("with");
    eat("(");
    std::vector<std::pair<std::string, std::string>> keys;
    for (;;) {
      const std::string attr = ident();
      eat("of");
      const std::string stream = ident();
      bool found = false;
      for (auto& k : keys)
        if (k.first == stream) {
          k.second = attr;
          found = true;
        }
      if (!found) keys.push_back({stream, attr});
      if (!accept(",")) break;
    }
    eat(")");
    eat("begin");
    const size_t nq = app.queries.size();
    size_t nout = 0;
    bool has_info = false;
    std::string info;
    while (!at("end")) {
      if (at("@")) {
        std::string name;
        std::vector<std::pair<std::string, std::string>> props;
        annotation(name, props);
        if (lower(name) == "info") {
          has_info = false;
          for (auto& p : props)
            if (p.first == "name") {
              has_info = true;
              info = p.second;
            }
        }
        continue;
      }
      if (accept(";")) continue;
      const std::string nm = has_info && !info.empty() ? info : "query" + std::to_string(nq + nout + 1);
      app.queries.push_back(query(nm, &keys));
      nout++;
      has_info = false;
    }
    eat("end");
  }

  Query query(const std::string& name, const std::vector<std::pair<std::string, std::string>>* part) {
    eat("from");
    Query q;
    q.name = name;
    q.root = state_input(q.seq_type);
    if (accept("within")) {
      q.has_within = true;
      q.within = time_value();
    }
    eat("select");
    if (accept("*")) {
      q.select_all = true;
    } else {
      for (;;) {
        EP e = expr();
        std::string nm;
        if (accept("as")) nm = ident();
        else nm = e->op == "var" ? e->attr : "_c" + std::to_string(q.select.size());
        q.select.push_back({e, nm});
        if (!accept(",")) break;
      }
    }
    if (at("group") || at("having") || at("output"))
      throw ParseError("group by / having / output rate limiting are outside the state path");
    if (accept("insert")) {
      if (accept("all")) {
        eat("events");
        q.output_events = "all";
      } else if (accept("expired")) {
        eat("events");
        q.output_events = "expired";
      } else if (accept("current")) {
        eat("events");
      }
      eat("into");
      q.out_stream = ident();
    } else if (accept("return")) {
      q.out_stream = "__return__";
    } else {
      throw ParseError("expected insert into");
    }
    accept(";");
    if (part) {
      q.partitioned = true;
      q.partition = *part;
    }
    return q;
  }

  int64_t time_value() {
    double total = 0;  // Python: total += int(float(num) * unit) (int accumulator)
    int64_t itotal = 0;
    bool got = false;
    while (peek().kind == T_NUM) {
      std::string num = eat().text;
      const std::string unit = lower(ident());
      auto it = time_units().find(unit);
      if (it == time_units().end()) throw ParseError("unknown time unit " + unit);
      while (!num.empty() && strchr("lLfFdD", num.back())) num.pop_back();
      const double v = strtod(num.c_str(), nullptr) * (double)it->second;
      itotal += (int64_t)std::trunc(v);
      got = true;
    }
    (void)total;
    if (!got) throw ParseError("expected time value");
    return itotal;
  }

  // pattern vs sequence by a top-level ',' or '->' before select / within
  SP state_input(std::string& seq_type) {
    int depth = 0;
    size_t j = i_;
    bool comma = false, arrow = false;
    for (;;) {
      const Tok& t = toks_[j];
      if (t.kind == T_EOF) break;
      if (t.text == "(" || t.text == "[") depth++;
      else if (t.text == ")" || t.text == "]") depth--;
      else if (depth == 0 && t.kind == T_ID && (lower(t.text) == "select" || lower(t.text) == "within")) break;
      else if (t.text == "->") arrow = true;
      else if (t.text == "," && depth == 0) comma = true;
      j++;
    }
    if (comma && arrow) throw ParseError("cannot mix '->' and ',' in one query");
    if (comma) {
      seq_type = "sequence";
      return sequence_chain();
    }
    seq_type = "pattern";
    return pattern_chain();
  }

  static SP node(const char* kind) {
    auto n = std::make_shared<StateNode>();
    n->kind = kind;
    return n;
  }

  SP pattern_chain() {
    SP nd = pattern_item();
    while (accept("->")) {
      SP x = node("next");
      x->a = nd;
      x->b = pattern_item();
      nd = x;
    }
    return nd;
  }

  SP pattern_item() {
    if (at("every")) {
      eat();
      SP x = node("every");
      if (at("(")) {
        eat("(");
        x->a = pattern_chain();
        eat(")");
        return x;
      }
      x->a = pattern_source(false);
      return x;
    }
    if (at("(")) {
      eat("(");
      SP inner = pattern_chain();
      eat(")");
      return inner;
    }
    return pattern_source(false);
  }

  SP sequence_chain() {
    SP first = sequence_item(true);
    std::vector<SP> rest;
    while (accept(",")) rest.push_back(sequence_item(false));
    if (rest.empty()) return first;
    SP chain = rest[0];
    for (size_t k = 1; k < rest.size(); k++) {
      SP x = node("next");
      x->a = chain;
      x->b = rest[k];
      chain = x;
    }
    SP x = node("next");
    x->a = first;
    x->b = chain;
    return x;
  }

  SP sequence_item(bool top) {
    if (at("every")) {
      if (!top) throw ParseError("'every' only allowed at the start of a sequence");
      eat();
      SP x = node("every");
      if (at("(")) {
        eat("(");
        x->a = sequence_chain();
        eat(")");
        return x;
      }
      x->a = pattern_source(true);
      return x;
    }
    if (at("(")) {
      eat("(");
      SP inner = sequence_chain();
      eat(")");
      return inner;
    }
    return pattern_source(true);
  }

  SP pattern_source(bool allow_count_seq) {
    if (at("(")) {
      eat("(");
      SP n = pattern_source(allow_count_seq);
      eat(")");
      return n;
    }
    SP left = stateful_or_absent();
    if (at("and") || at("or")) {
      const std::string op = lower(eat().text);
      SP right = stateful_or_absent();
      return make_logical(op, left, right);
    }
    if (left->kind == "absent") {
      if (!left->has_waiting) throw ParseError("'not' without 'for' is only valid inside 'and'");
      return left;
    }
    if (at("<")) {
      eat("<");
      int64_t mn, mx;
      collect(mn, mx);
      eat(">");
      SP x = node("count");
      x->a = left;
      x->mn = mn;
      x->mx = mx;
      return x;
    }
    if (allow_count_seq) {
      int64_t mn = 0, mx = 0;
      bool c = false;
      if (accept("*")) {
        mn = 0, mx = -1, c = true;
      } else if (accept("+")) {
        mn = 1, mx = -1, c = true;
      } else if (accept("?")) {
        mn = 0, mx = 1, c = true;
      }
      if (c) {
        SP x = node("count");
        x->a = left;
        x->mn = mn;
        x->mx = mx;
        return x;
      }
    }
    return left;
  }

  void collect(int64_t& mn, int64_t& mx) {
    if (at(":")) {
      eat();
      mn = -1;
      mx = py_int(eat().text);
      return;
    }
    const int64_t a = py_int(eat().text);
    if (accept(":")) {
      if (peek().kind == T_NUM) {
        mn = a;
        mx = py_int(eat().text);
        return;
      }
      mn = a;
      mx = -1;
      return;
    }
    mn = mx = a;
  }

  SP make_logical(const std::string& op, SP left, SP right) {
    const bool la = left->kind == "absent", ra = right->kind == "absent";
    SP x = node("logical");
    x->logical = op;
    if (op == "and") {
      if (!la && ra) {  // A and not B [for t]
        x->a = right;
        x->b = left;
      } else {
        x->a = left;
        x->b = right;
      }
      return x;
    }
    for (const SP& n : {left, right})
      if (n->kind == "absent" && !n->has_waiting) throw ParseError("'not' in 'or' requires 'for'");
    if (!la && ra) {  // A or not B for t -> logicalOr(absent B, A)
      x->a = right;
      x->b = left;
    } else {
      x->a = left;
      x->b = right;
    }
    return x;
  }

  SP stateful_or_absent() {
    if (accept("not")) {
      SP x = node("absent");
      x->src = basic_source(false, "");
      if (accept("for")) {
        x->has_waiting = true;
        x->waiting = time_value();
      }
      return x;
    }
    bool has_ref = false;
    std::string ref;
    if (peek().kind == T_ID && at("=", 1)) {
      ref = ident();
      eat("=");
      has_ref = true;
    }
    SP x = node("stream");
    x->src = basic_source(has_ref, ref);
    return x;
  }

  std::shared_ptr<BasicSource> basic_source(bool has_ref, const std::string& ref) {
    auto b = std::make_shared<BasicSource>();
    b->has_ref = has_ref;
    b->ref = ref;
    accept("#");
    b->stream = ident();
    while (at("[")) {
      eat("[");
      b->filters.push_back(expr());
      eat("]");
    }
    if (at("#")) throw ParseError("stream functions/windows inside states are outside the state path");
    return b;
  }

  static EP mk(const std::string& op, std::vector<EP> args = {}) {
    auto e = std::make_shared<Expr>();
    e->op = op;
    e->args = std::move(args);
    return e;
  }

  EP expr() {
    EP e = and_expr();
    while (accept("or")) e = mk("or", {e, and_expr()});
    return e;
  }
  EP and_expr() {
    EP e = not_expr();
    while (accept("and")) e = mk("and", {e, not_expr()});
    return e;
  }
  EP not_expr() {
    if (accept("not")) return mk("not", {not_expr()});
    return cmp_expr();
  }
  EP cmp_expr() {
    EP e = add_expr();
    static const std::pair<const char*, const char*> ops[] = {{">", "gt"}, {"<", "lt"}, {">=", "ge"},
                                                               {"<=", "le"}, {"==", "eq"}, {"!=", "ne"}};
    const Tok& t = peek();
    if (t.kind == T_OP)
      for (auto& o : ops)
        if (t.text == o.first) {
          eat();
          EP c = mk("cmp", {e, add_expr()});
          c->value.k = Val::STR;
          c->value.s = o.second;
          return c;
        }
    if (at("is")) {
      eat();
      eat("null");
      return mk("isnull", {e});
    }
    return e;
  }
  EP add_expr() {
    EP e = mul_expr();
    while (at("+") || at("-")) {
      const std::string op = eat().text == "+" ? "add" : "sub";
      e = mk(op, {e, mul_expr()});
    }
    return e;
  }
  EP mul_expr() {
    EP e = unary();
    while (at("*") || at("/") || at("%")) {
      const std::string t = eat().text;
      e = mk(t == "*" ? "mul" : (t == "/" ? "div" : "mod"), {e, unary()});
    }
    return e;
  }
  EP unary() {
    if (at("-") && peek(1).kind == T_NUM) {
      eat();
      return number(true);
    }
    if (accept("(")) {
      EP e = expr();
      eat(")");
      return e;
    }
    const Tok t = peek();
    if (t.kind == T_NUM) return number(false);
    if (t.kind == T_STRL) {
      eat();
      EP e = mk("const");
      e->value.k = Val::STR;
      e->value.s = t.text.substr(1, t.text.size() - 2);
      e->vtype = "string";
      return e;
    }
    if (at("true") || at("false")) {
      eat();
      EP e = mk("const");
      e->value.k = Val::BOOL;
      e->value.b = lower(t.text) == "true";
      e->vtype = "bool";
      return e;
    }
    if (at("null")) {
      eat();
      EP e = mk("const");
      e->vtype = "null";
      return e;
    }
    if (t.kind == T_ID) {
      const std::string name = ident();
      if (at("(") && !at("[")) {  // function call
        eat("(");
        EP f = mk("func");
        if (!at(")")) {
          for (;;) {
            f->args.push_back(expr());
            if (!accept(",")) break;
          }
        }
        eat(")");
        f->value.k = Val::STR;
        f->value.s = lower(name);
        return f;
      }
      bool has_index = false;
      int64_t index = 0;
      if (at("[")) {
        eat("[");
        index = attribute_index();
        has_index = true;
        eat("]");
      }
      if (accept(".")) {
        EP e = mk("var");
        e->has_ref = true;
        e->stream_ref = name;
        e->has_attr = true;
        e->attr = ident();
        e->has_index = has_index;
        e->index = index;
        return e;
      }
      if (has_index) {
        EP e = mk("stateref");
        e->has_ref = true;
        e->stream_ref = name;
        e->has_index = true;
        e->index = index;
        return e;
      }
      EP e = mk("var");
      e->has_attr = true;
      e->attr = name;
      return e;
    }
    throw ParseError("unexpected token '" + t.text + "' at " + std::to_string(t.pos));
  }
  int64_t attribute_index() {
    if (accept("last")) {
      int64_t idx = -2;  // SiddhiConstants.LAST (visitAttribute_index, visitor:2340-2346)
      if (accept("-")) idx -= py_int(eat().text);
      return idx;
    }
    return py_int(eat().text);
  }
  EP number(bool negate) {
    const std::string txt = eat().text;
    const char sfx = (char)tolower((unsigned char)txt.back());
    EP e = mk("const");
    if (sfx == 'l') {
      e->value.k = Val::INT;
      e->value.i = py_int(txt.substr(0, txt.size() - 1));
      e->vtype = "long";
    } else if (sfx == 'f' || sfx == 'd') {
      e->value.k = Val::FLT;
      e->value.d = strtod(txt.substr(0, txt.size() - 1).c_str(), nullptr);
      e->vtype = sfx == 'f' ? "float" : "double";
    } else if (txt.find('.') != std::string::npos || txt.find('e') != std::string::npos ||
               txt.find('E') != std::string::npos) {
      e->value.k = Val::FLT;
      e->value.d = strtod(txt.c_str(), nullptr);
      e->vtype = "double";
    } else {
      e->value.k = Val::INT;
      e->value.i = py_int(txt);
      e->vtype = "int";
      if (e->value.i > 2147483647ll) throw ParseError("int literal out of range: " + txt);
    }
    if (negate) {
      if (e->value.k == Val::INT) e->value.i = -e->value.i;
      else e->value.d = -e->value.d;
    }
    return e;
  }
};

// ------------------------------------------------------------------ JSON values (json.dumps(sort_keys=True))
struct J;
using JP = std::shared_ptr<J>;
struct J {
  enum K { NUL, BOOL, INT, FLT, STR, ARR, OBJ } k = NUL;
  bool b = false;
  int64_t i = 0;
  double d = 0;
  std::string s;
  std::vector<J> a;
  std::map<std::string, J> o;  // bytewise order = code point order of the (UTF-8) keys
  static J null() { return J(); }
  static J boolean(bool v) {
    J j;
    j.k = BOOL;
    j.b = v;
    return j;
  }
  static J integer(int64_t v) {
    J j;
    j.k = INT;
    j.i = v;
    return j;
  }
  static J flt(double v) {
    J j;
    j.k = FLT;
    j.d = v;
    return j;
  }
  static J str(const std::string& v) {
    J j;
    j.k = STR;
    j.s = v;
    return j;
  }
  static J arr() {
    J j;
    j.k = ARR;
    return j;
  }
  static J obj() {
    J j;
    j.k = OBJ;
    return j;
  }
  J& operator[](const std::string& key) {
    k = OBJ;
    return o[key];
  }
  void push(const J& v) {
    k = ARR;
    a.push_back(v);
  }
};

// Python repr(float): the shortest digits that round-trip; exponent form when the decimal
// exponent is < -4 or >= 16 (format_float_short, 'r' mode with Py_DTSF_ADD_DOT_0)
static std::string py_float(double x) {
  if (std::isnan(x)) return "NaN";
  if (std::isinf(x)) return x > 0 ? "Infinity" : "-Infinity";
  if (x == 0) return std::signbit(x) ? "-0.0" : "0.0";
  char buf[64];
  int prec = 1;
  for (; prec <= 17; prec++) {
    snprintf(buf, sizeof buf, "%.*e", prec - 1, x);
    if (strtod(buf, nullptr) == x) break;
  }
  // buf: [-]d[.ddd]e[+-]XX
  std::string t = buf;
  bool neg = false;
  if (t[0] == '-') {
    neg = true;
    t = t.substr(1);
  }
  const size_t ep = t.find('e');
  std::string mant = t.substr(0, ep);
  const int exp10 = atoi(t.c_str() + ep + 1);
  std::string digits;
  for (char c : mant)
    if (c != '.') digits += c;
  while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
  const int decpt = exp10 + 1;  // digits d1 d2 ... with the point after decpt of them
  std::string out;
  if (decpt <= -4 || decpt > 16) {
    out = digits.substr(0, 1);
    if (digits.size() > 1) out += "." + digits.substr(1);
    char eb[16];
    snprintf(eb, sizeof eb, "e%c%02d", exp10 < 0 ? '-' : '+', exp10 < 0 ? -exp10 : exp10);
    out += eb;
  } else if (decpt <= 0) {
    out = "0." + std::string((size_t)(-decpt), '0') + digits;
  } else if ((size_t)decpt >= digits.size()) {
    out = digits + std::string((size_t)decpt - digits.size(), '0') + ".0";
  } else {
    out = digits.substr(0, (size_t)decpt) + "." + digits.substr((size_t)decpt);
  }
  return neg ? "-" + out : out;
}

// json.dumps string escaping with ensure_ascii=True (UTF-8 in, \uXXXX with surrogate pairs out)
static void py_str(std::string& o, const std::string& s) {
  o += '"';
  for (size_t i = 0; i < s.size();) {
    const unsigned char c = (unsigned char)s[i];
    uint32_t cp = c;
    size_t len = 1;
    if (c >= 0x80) {
      if ((c & 0xE0) == 0xC0 && i + 1 < s.size()) {
        cp = ((c & 0x1Fu) << 6) | ((unsigned char)s[i + 1] & 0x3Fu);
        len = 2;
      } else if ((c & 0xF0) == 0xE0 && i + 2 < s.size()) {
        cp = ((c & 0x0Fu) << 12) | (((unsigned char)s[i + 1] & 0x3Fu) << 6) | ((unsigned char)s[i + 2] & 0x3Fu);
        len = 3;
      } else if ((c & 0xF8) == 0xF0 && i + 3 < s.size()) {
        cp = ((c & 0x07u) << 18) | (((unsigned char)s[i + 1] & 0x3Fu) << 12) |
             (((unsigned char)s[i + 2] & 0x3Fu) << 6) | ((unsigned char)s[i + 3] & 0x3Fu);
        len = 4;
      } else {
        cp = 0xFFFD;
      }
    }
    i += len;
    char b[16];
    switch (cp) {
      case '"': o += "\\\""; continue;
      case '\\': o += "\\\\"; continue;
      case '\n': o += "\\n"; continue;
      case '\r': o += "\\r"; continue;
      case '\t': o += "\\t"; continue;
      case '\b': o += "\\b"; continue;
      case '\f': o += "\\f"; continue;
      default: break;
    }
    if (cp < 0x20 || cp >= 0x7F) {
      if (cp >= 0x10000) {
        const uint32_t v = cp - 0x10000;
        snprintf(b, sizeof b, "\\u%04x\\u%04x", 0xD800 + (v >> 10), 0xDC00 + (v & 0x3FF));
      } else {
        snprintf(b, sizeof b, "\\u%04x", cp);
      }
      o += b;
    } else {
      o += (char)cp;
    }
  }
  o += '"';
}

static void dump(std::string& o, const J& j) {
  switch (j.k) {
    case J::NUL: o += "null"; break;
    case J::BOOL: o += j.b ? "true" : "false"; break;
    case J::INT: o += std::to_string(j.i); break;
    case J::FLT: o += py_float(j.d); break;
    case J::STR: py_str(o, j.s); break;
    case J::ARR: {
      o += '[';
      for (size_t k = 0; k < j.a.size(); k++) {
        if (k) o += ", ";
        dump(o, j.a[k]);
      }
      o += ']';
      break;
    }
    case J::OBJ: {
      o += '{';
      bool first = true;
      for (auto& kv : j.o) {
        if (!first) o += ", ";
        first = false;
        py_str(o, kv.first);
        o += ": ";
        dump(o, kv.second);
      }
      o += '}';
      break;
    }
  }
}

}  // namespace shpql

// ------------------------------------------------------------------ string dictionary (C-ABI)
struct shp_dict {
  std::mutex mu;
  std::unordered_map<std::string, int32_t> ids;
  std::vector<std::string> strings;
  int32_t max_ids = 0;  // 0: unbounded
  int32_t intern(const std::string& s) {
    std::lock_guard<std::mutex> g(mu);
    auto it = ids.find(s);
    if (it != ids.end()) return it->second;
    if (max_ids > 0 && (int32_t)strings.size() >= max_ids) return SHP_ERR_KEYS;
    const int32_t id = (int32_t)strings.size();
    ids.emplace(s, id);
    strings.push_back(s);
    return id;
  }
};

namespace shpql {

using StrTy = std::string;
static const std::map<std::string, int>& num_rank() {
  static const std::map<std::string, int> m = {{"int", 0}, {"long", 1}, {"float", 2}, {"double", 3}};
  return m;
}
static bool is_num(const std::string& t) { return num_rank().count(t) != 0; }
constexpr int64_t CURRENT = -1, LAST = -2;

struct Leaf {
  int id;
  bool has_ref;
  std::string ref, stream;
  bool absent;
  int64_t waiting;
  bool multi_value;
  std::vector<EP> filters;
  J filter;  // null when no filter
};

// compiler.py QueryCompiler
class QueryCompiler {
 public:
  QueryCompiler(const App& app, const Query& q, shp_dict* dict) : app_(app), q_(q), dict_(dict) {
    for (size_t i = 0; i < app.streams.size(); i++) sidx_[app.streams[i].name] = (int)i;
  }

  J compile() {
    J tree = build(q_.root, false);
    for (auto& lf : leaves_) {
      if (lf.filters.empty()) continue;
      J ex;
      bool have = false;
      for (auto& f : lf.filters) {
        std::string ty;
        J fe = cexpr(f, &lf, ty);
        if (ty != "bool") throw CreationError("filter expression must be of type BOOL");
        if (!have) {
          ex = fe;
          have = true;
        } else {
          J a = J::obj();
          a["op"] = J::str("and");
          a["a"] = ex;
          a["b"] = fe;
          ex = a;
        }
      }
      lf.filter = ex;
    }
    std::vector<J> sel = compile_select();
    J states = J::arr();
    for (auto& lf : leaves_) {
      J s = J::obj();
      s["id"] = J::integer(lf.id);
      s["ref"] = lf.has_ref ? J::str(lf.ref) : J::null();
      s["stream"] = J::integer(sidx_.at(lf.stream));
      s["absent"] = J::boolean(lf.absent);
      s["waiting"] = J::integer(lf.waiting);
      s["filter"] = lf.filter;
      states.push(s);
    }
    if (q_.partitioned)
      for (auto& lf : leaves_) {
        bool keyed = false;
        for (auto& p : q_.partition) keyed = keyed || p.first == lf.stream;
        if (!keyed) throw CreationError("stream " + lf.stream + " used in a partition without a partition key");
      }
    J prog = J::obj();
    prog["version"] = J::integer(1);
    prog["name"] = J::str(q_.name);
    prog["type"] = J::str(q_.seq_type);
    prog["within"] = J::integer(q_.has_within ? q_.within : -1);
    prog["playback"] = J::boolean(app_.playback);
    prog["partitioned"] = J::boolean(q_.partitioned);
    J streams = J::arr();
    for (auto& sd : app_.streams) {
      J s = J::obj();
      s["name"] = J::str(sd.name);
      J at = J::arr();
      for (auto& a : sd.attrs) {
        J p = J::arr();
        p.push(J::str(a.first));
        p.push(J::str(a.second));
        at.push(p);
      }
      s["attrs"] = at;
      streams.push(s);
    }
    prog["streams"] = streams;
    J cols = J::arr();
    for (auto& c : columns_) {
      J x = J::obj();
      x["stream"] = J::integer(c.s);
      x["attr"] = J::integer(c.a);
      x["type"] = J::str(c.t);
      cols.push(x);
    }
    prog["columns"] = cols;
    prog["states"] = states;
    prog["tree"] = tree;
    J agg;
    if (device_aggregate(sel, agg)) prog["aggregate"] = agg;
    return prog;
  }

 private:
  struct Col {
    int s, a;
    std::string t;
  };
  const App& app_;
  const Query& q_;
  shp_dict* dict_;
  std::map<std::string, int> sidx_;
  std::vector<Leaf> leaves_;
  std::vector<Col> columns_;

  const StreamDef& sdef(const std::string& n) const {
    const StreamDef* s = app_.stream(n);
    if (!s) throw CreationError("Stream " + n + " is not defined");
    return *s;
  }
  bool attr_type(const std::string& stream, const std::string& attr, std::string& t) const {
    for (auto& a : sdef(stream).attrs)
      if (a.first == attr) {
        t = a.second;
        return true;
      }
    return false;
  }
  int attr_idx(const std::string& stream, const std::string& attr) const {
    const auto& at = sdef(stream).attrs;
    for (size_t i = 0; i < at.size(); i++)
      if (at[i].first == attr) return (int)i;
    throw CreationError(attr + " not defined in " + stream);
  }
  Leaf* find_state(const std::string& ref) {
    for (auto& lf : leaves_)
      if (lf.has_ref && lf.ref == ref) return &lf;
    for (auto& lf : leaves_)
      if (!lf.has_ref && lf.stream == ref) return &lf;
    return nullptr;
  }
  int column(const std::string& stream, const std::string& attr) {
    const int s = sidx_.at(stream), a = attr_idx(stream, attr);
    for (size_t i = 0; i < columns_.size(); i++)
      if (columns_[i].s == s && columns_[i].a == a) return (int)i;
    std::string t;
    attr_type(stream, attr, t);
    columns_.push_back({s, a, t});
    return (int)columns_.size() - 1;
  }

  Leaf& leaf(const StateNode& n, bool absent, bool multi) {
    const BasicSource& src = *n.src;
    if (!app_.stream(src.stream)) throw CreationError("Stream " + src.stream + " is not defined");
    Leaf lf;
    lf.id = (int)leaves_.size();
    lf.has_ref = src.has_ref;
    lf.ref = src.ref;
    lf.stream = src.stream;
    lf.absent = absent;
    lf.waiting = n.has_waiting ? n.waiting : -1;
    lf.multi_value = multi;
    lf.filters = src.filters;
    leaves_.push_back(lf);
    return leaves_.back();
  }

  J build(const SP& n, bool multi) {
    const std::string& k = n->kind;
    J t = J::obj();
    if (k == "stream" || k == "absent") {
      t["t"] = J::str(k);
      t["state"] = J::integer(leaf(*n, k == "absent", multi).id);
      return t;
    }
    if (k == "next") {
      J a = build(n->a, multi);
      J b = build(n->b, multi);
      t["t"] = J::str("next");
      t["a"] = a;
      t["b"] = b;
      return t;
    }
    if (k == "every") {
      t["t"] = J::str("every");
      t["x"] = build(n->a, multi);
      return t;
    }
    if (k == "count") {
      if (n->a->kind != "stream") throw CreationError("count state must wrap a stream state");
      const int id = leaf(*n->a, false, true).id;
      t["t"] = J::str("count");
      t["state"] = J::integer(id);
      t["min"] = J::integer(n->mn == -1 ? 0 : n->mn);
      t["max"] = J::integer(n->mx == -1 ? -1 : n->mx);
      return t;
    }
    if (k == "logical") {  // element2 parsed before element1 (StateInputStreamParser.java:339-352)
      J s2 = build(n->b, multi);
      J s1 = build(n->a, multi);
      t["t"] = J::str("logical");
      t["op"] = J::str(n->logical);
      t["s1"] = s1;
      t["s2"] = s2;
      return t;
    }
    throw CreationError("unsupported state element " + k);
  }

  // ExpressionParser.parseVariable: (leaf, chain index, type, multi-valued)
  Leaf* resolve_var(const Expr& e, const Leaf* current, int64_t default_index, int64_t& index, std::string& t,
                    bool& multi) {
    multi = false;
    if (!e.has_ref) {
      Leaf* lf = nullptr;
      if (current) {
        if (!attr_type(current->stream, e.attr, t))
          throw CreationError(e.attr + " not defined in Input Stream: " + current->stream);
        lf = &leaves_[current->id];
      } else {
        std::vector<Leaf*> found;
        for (auto& x : leaves_) {
          std::string tt;
          if (attr_type(x.stream, e.attr, tt)) found.push_back(&x);
        }
        if (found.empty()) throw CreationError("attribute " + e.attr + " not found");
        if (found.size() > 1) throw CreationError("attribute " + e.attr + " is ambiguous across input streams");
        lf = found[0];
        attr_type(lf->stream, e.attr, t);
      }
      index = !e.has_index ? default_index : (e.index <= LAST ? e.index + 1 : e.index);
      return lf;
    }
    Leaf* lf = find_state(e.stream_ref);
    if (!lf) throw CreationError("Stream with reference : " + e.stream_ref + " not found");
    t.clear();
    if (e.has_attr && !attr_type(lf->stream, e.attr, t)) throw CreationError(e.attr + " not defined in " + lf->stream);
    if (!e.has_index) {
      index = default_index;
    } else if (e.index <= LAST) {
      index = e.index + 1;
      if (current && current->has_ref && lf->has_ref && e.stream_ref == current->ref) index = e.index;
    } else {
      index = e.index;
    }
    multi = !current && !e.has_index && lf->multi_value && lf->has_ref;
    return lf;
  }

  J cexpr(const EP& ep, const Leaf* current, std::string& ty) {
    const Expr& e = *ep;
    const std::string& op = e.op;
    J r = J::obj();
    if (op == "const") {
      r["op"] = J::str("const");
      if (e.vtype == "string") {
        const int32_t id = dict_->intern(e.value.s);
        if (id < 0) throw CreationError("string dictionary full");
        r["type"] = J::str("string");
        r["v"] = J::integer(id);
        ty = "string";
      } else if (e.vtype == "null") {
        r["type"] = J::str("null");
        r["v"] = J::integer(0);
        ty = "null";
      } else if (e.vtype == "bool") {
        r["type"] = J::str("bool");
        r["v"] = J::integer(e.value.b ? 1 : 0);
        ty = "bool";
      } else {
        r["type"] = J::str(e.vtype);
        r["v"] = e.value.k == Val::INT ? J::integer(e.value.i) : J::flt(e.value.d);
        ty = e.vtype;
      }
      return r;
    }
    if (op == "var") {
      std::string tt;
      if (!e.has_ref && find_state(e.attr) && !attr_type(current->stream, e.attr, tt))
        throw CreationError("state reference used as a value");
      int64_t index;
      std::string t;
      bool multi;
      Leaf* lf = resolve_var(e, current, CURRENT, index, t, multi);
      const int col = column(lf->stream, e.attr);
      r["op"] = J::str("var");
      r["state"] = J::integer(lf->id);
      r["col"] = J::integer(col);
      r["index"] = J::integer(index);
      r["type"] = J::str(t);
      ty = t;
      return r;
    }
    if (op == "stateref") throw CreationError("state reference used as a value");
    if (op == "and" || op == "or") {
      std::string ta, tb;
      J a = cexpr(e.args[0], current, ta);
      J b = cexpr(e.args[1], current, tb);
      if (ta != "bool" || tb != "bool") throw CreationError(op + " operands must be BOOL");
      r["op"] = J::str(op);
      r["a"] = a;
      r["b"] = b;
      ty = "bool";
      return r;
    }
    if (op == "not") {
      std::string ta;
      J a = cexpr(e.args[0], current, ta);
      if (ta != "bool") throw CreationError("not operand must be BOOL");
      r["op"] = J::str("not");
      r["a"] = a;
      ty = "bool";
      return r;
    }
    if (op == "isnull") {
      const Expr& in = *e.args[0];
      std::string tt;
      if (in.op == "stateref" ||
          (in.op == "var" && !in.has_ref && find_state(in.attr) && !attr_type(current->stream, in.attr, tt))) {
        const std::string ref = in.op == "stateref" ? in.stream_ref : in.attr;
        Leaf* lf = find_state(ref);
        if (!lf) throw CreationError("Stream with reference : " + ref + " not found");
        const int64_t idx = !in.has_index ? CURRENT : (in.index <= LAST ? in.index + 1 : in.index);
        r["op"] = J::str("isnullstate");
        r["state"] = J::integer(lf->id);
        r["index"] = J::integer(idx);
        ty = "bool";
        return r;
      }
      std::string ta;
      J a = cexpr(e.args[0], current, ta);
      r["op"] = J::str("isnull");
      r["a"] = a;
      ty = "bool";
      return r;
    }
    if (op == "cmp") {
      std::string ta, tb;
      J a = cexpr(e.args[0], current, ta);
      J b = cexpr(e.args[1], current, tb);
      const std::string& cmp = e.value.s;
      if (is_num(ta) && is_num(tb)) {
      } else if (ta == tb && (ta == "string" || ta == "bool") && (cmp == "eq" || cmp == "ne")) {
      } else if (ta == "null" || tb == "null") {
      } else {
        throw CreationError("cannot compare " + ta + " with " + tb + " using " + cmp);
      }
      r["op"] = J::str("cmp");
      r["cmp"] = J::str(cmp);
      r["a"] = a;
      r["b"] = b;
      ty = "bool";
      return r;
    }
    if (op == "add" || op == "sub" || op == "mul" || op == "div" || op == "mod") {
      std::string ta, tb;
      J a = cexpr(e.args[0], current, ta);
      J b = cexpr(e.args[1], current, tb);
      if (!is_num(ta) || !is_num(tb)) throw CreationError("arithmetic on " + ta + "/" + tb);
      const std::string rt = num_rank().at(ta) >= num_rank().at(tb) ? ta : tb;
      r["op"] = J::str(op);
      r["type"] = J::str(rt);
      r["a"] = a;
      r["b"] = b;
      ty = rt;
      return r;
    }
    if (op == "func") return cfunc(e, current, ty);
    throw CreationError("unsupported expression " + op + " in a state filter");
  }

  // scalar functions in filters (core/executor/function/*), with the reference's validation
  J cfunc(const Expr& e, const Leaf* current, std::string& ty) {
    const std::string& name = e.value.s;
    std::vector<J> args;
    std::vector<std::string> types;
    for (auto& a : e.args) {
      std::string t;
      args.push_back(cexpr(a, current, t));
      types.push_back(t);
    }
    J r = J::obj();
    if (name == "ifthenelse") {  // IfThenElseFunctionExecutor.java
      if (args.size() != 3)
        throw CreationError("Invalid no of arguments passed to ifThenElse() function, required only 3, but found " +
                            std::to_string(args.size()));
      if (types[0] != "bool") throw CreationError("Input type of if in ifThenElse function should be of type BOOL");
      if (types[1] != types[2])
        throw CreationError("Input type of then in ifThenElse function and else in ifThenElse function should be of "
                            "equivalent type");
      r["op"] = J::str("ifthenelse");
      r["type"] = J::str(types[1]);
      J a = J::arr();
      for (auto& x : args) a.push(x);
      r["args"] = a;
      ty = types[1];
      return r;
    }
    if (name == "coalesce") {  // CoalesceFunctionExecutor.java
      if (args.empty()) throw CreationError("Coalesce must have at least one parameter");
      for (auto& t : types)
        if (t != types[0]) throw CreationError("Coalesce cannot have parameters with different type");
      r["op"] = J::str("coalesce");
      r["type"] = J::str(types[0]);
      J a = J::arr();
      for (auto& x : args) a.push(x);
      r["args"] = a;
      ty = types[0];
      return r;
    }
    static const std::map<std::string, std::string> inst = {
        {"instanceofboolean", "bool"}, {"instanceofdouble", "double"}, {"instanceoffloat", "float"},
        {"instanceofinteger", "int"},  {"instanceoflong", "long"},     {"instanceofstring", "string"}};
    auto it = inst.find(name);
    if (it != inst.end()) {  // InstanceOf*FunctionExecutor.java
      if (args.size() != 1) throw CreationError("Invalid no of arguments passed to " + name);
      r["op"] = J::str("instanceof");
      r["tag"] = J::str(it->second);
      r["a"] = args[0];
      ty = "bool";
      return r;
    }
    throw CreationError("function " + name + " is not supported in a state filter");
  }

  // the selector (compile_select / _csel): validated here, emitted only through "aggregate"
  std::vector<J> compile_select() {
    if (q_.select_all) throw CreationError("select * is not supported on the state path");
    std::vector<J> out;
    for (auto& it : q_.select) out.push_back(csel(it.expr));
    return out;
  }
  J csel(const EP& ep) {
    const Expr& e = *ep;
    J r = J::obj();
    if (e.op == "const") {
      r["op"] = J::str("const");
      return r;
    }
    if (e.op == "var") {
      int64_t index;
      std::string t;
      bool multi;
      Leaf* lf = resolve_var(e, nullptr, 0, index, t, multi);
      r["op"] = J::str("var");
      r["state"] = J::integer(lf->id);
      r["attr"] = J::integer(attr_idx(lf->stream, e.attr));
      r["multi"] = J::boolean(multi);
      return r;
    }
    if (e.op == "func") {
      r["op"] = J::str("func");
      r["name"] = J::str(e.value.s);
      J a = J::arr();
      for (auto& x : e.args) a.push(csel(x));
      r["args"] = a;
      return r;
    }
    static const char* ops[] = {"add", "sub", "mul", "div", "mod", "cmp", "and", "or", "not", "isnull"};
    for (const char* o : ops)
      if (e.op == o) {
        r["op"] = J::str(e.op);
        for (auto& x : e.args) csel(x);
        return r;
      }
    throw CreationError("unsupported select expression " + e.op);
  }

  // compiler.py _device_aggregate: exactly one avg/sum/count/min/max over one state's filter column
  bool device_aggregate(const std::vector<J>& sel, J& out) {
    const J* f = nullptr;
    int nf = 0;
    for (auto& it : sel)
      if (it.o.at("op").s == "func") {
        nf++;
        f = &it;
      }
    if (nf != 1) return false;
    const std::string& name = f->o.at("name").s;
    if (name != "avg" && name != "sum" && name != "count" && name != "min" && name != "max") return false;
    const J& args = f->o.at("args");
    out = J::obj();
    if (name == "count") {
      if (!args.a.empty()) return false;
      out["fn"] = J::str("count");
      return true;
    }
    if (args.a.size() != 1 || args.a[0].o.at("op").s != "var" || args.a[0].o.at("multi").b) return false;
    const J& a = args.a[0];
    const int state = (int)a.o.at("state").i, attr = (int)a.o.at("attr").i;
    const int s = sidx_.at(leaves_[state].stream);
    for (size_t ci = 0; ci < columns_.size(); ci++)
      if (columns_[ci].s == s && columns_[ci].a == attr) {
        out["fn"] = J::str(name);
        out["state"] = J::integer(state);
        out["column"] = J::integer((int64_t)ci);
        return true;
      }
    return false;
  }
};

static thread_local std::string g_err;

static int64_t copy_out(const std::string& s, char* out, size_t cap) {
  if (out && cap) {
    const size_t n = std::min(cap - 1, s.size());
    memcpy(out, s.data(), n);
    out[n] = 0;
  }
  return (int64_t)s.size();
}

// the program JSON of the app's query `name` (NULL: the first query); dict interns string constants
std::string compile_query(const char* app_text, const char* name, shp_dict* dict) {
  App app = Parser(app_text).parse_app();
  if (app.queries.empty()) throw CreationError("the app has no query");
  const Query* q = nullptr;
  for (auto& x : app.queries)
    if (!name || x.name == name) {
      q = &x;
      break;
    }
  if (!q) throw CreationError(std::string("no query named ") + name);
  J prog = QueryCompiler(app, *q, dict).compile();
  std::string o;
  dump(o, prog);
  return o;
}

}  // namespace shpql

extern "C" {

shp_dict* shp_dict_create(int32_t max_ids) {
  auto* d = new shp_dict();
  d->max_ids = max_ids > 0 ? max_ids : 0;
  return d;
}

int32_t shp_dict_intern(shp_dict* d, const char* utf8, int64_t len) {
  if (!d || !utf8 || len < 0) return SHP_ERR_ARG;
  return d->intern(std::string(utf8, (size_t)len));
}

int32_t shp_dict_size(shp_dict* d) {
  if (!d) return SHP_ERR_ARG;
  std::lock_guard<std::mutex> g(d->mu);
  return (int32_t)d->strings.size();
}

int64_t shp_dict_string(shp_dict* d, int32_t id, char* out, size_t cap) {
  if (!d) return SHP_ERR_ARG;
  std::string s;
  {
    std::lock_guard<std::mutex> g(d->mu);
    if (id < 0 || id >= (int32_t)d->strings.size()) return SHP_ERR_ARG;
    s = d->strings[(size_t)id];
  }
  return shpql::copy_out(s, out, cap);
}

void shp_dict_destroy(shp_dict* d) { delete d; }

int64_t shp_compile_siddhiql(const char* app_text, const char* query_name, shp_dict* dict, char* out, size_t cap) {
  if (!app_text || !dict) {
    shpql::g_err = "null argument";
    return SHP_ERR_ARG;
  }
  try {
    return shpql::copy_out(shpql::compile_query(app_text, query_name, dict), out, cap);
  } catch (shpql::ParseError& e) {
    shpql::g_err = std::string("SiddhiParserException: ") + e.what();
    return SHP_ERR_ARG;
  } catch (shpql::CreationError& e) {
    shpql::g_err = std::string("SiddhiAppCreationException: ") + e.what();
    return SHP_ERR_UNSUPPORTED;
  } catch (std::exception& e) {
    shpql::g_err = e.what();
    return SHP_ERR_ARG;
  }
}

int64_t shp_siddhiql_queries(const char* app_text, char* out, size_t cap) {
  if (!app_text) {
    shpql::g_err = "null argument";
    return SHP_ERR_ARG;
  }
  try {
    using namespace shpql;
    App app = Parser(app_text).parse_app();
    J a = J::arr();
    for (auto& q : app.queries) {
      J x = J::obj();
      x["name"] = J::str(q.name);
      x["type"] = J::str(q.seq_type);
      x["out"] = J::str(q.out_stream);
      x["output_events"] = J::str(q.output_events);
      x["playback"] = J::boolean(app.playback);
      if (q.partitioned) {
        J p = J::obj();
        for (auto& kv : q.partition) p[kv.first] = J::str(kv.second);
        x["partition"] = p;
      } else {
        x["partition"] = J::null();
      }
      a.push(x);
    }
    std::string o;
    dump(o, a);
    return copy_out(o, out, cap);
  } catch (std::exception& e) {
    shpql::g_err = std::string("SiddhiParserException: ") + e.what();
    return SHP_ERR_ARG;
  }
}

const char* shp_compile_last_error(void) { return shpql::g_err.c_str(); }

}  // extern "C"
