// siddhi-hip: host-side NFA program compiler (program JSON -> DevProg).
//
// Reproduces the build-time wiring of StateInputStreamParser.parse
// (core/util/parser/StateInputStreamParser.java:148-408): processor creation per
// state element, next/every/partner links, within + start-state ids (:129-141),
// the first processor's thisLastProcessor (:142-143), the selector attachment of
// InnerStateRuntime.setQuerySelector and the receiver registration order of
// InnerStateRuntime.setup (state/runtime/*.java).  Condition trees are lowered to
// the predicate bytecode of prog.h (Java typing is already resolved in the JSON).
#pragma once
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "jsonv.h"
#include "prog.h"

namespace shp {

struct CompileError : std::runtime_error {
  int code;
  CompileError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

class ProgramCompiler {
 public:
  DevProg P{};
  FastShape fast{};
  CseqShape cseq{};
  LabsShape labs{};
  // select-side aggregate over the matches (SHP_LAYOUT_AGG): 0 none, 1 avg, 2 sum, 3 count, 4 min, 5 max;
  // over the value of state agg_state in predicate column agg_col (count: no argument)
  int agg_fn = 0, agg_state = -1, agg_col = -1;

  void compile(const char* json) {
    JV root = JReader(json).read();
    if (root.present("aggregate")) {
      const JV& a = root.get("aggregate");
      const std::string& fn = a.get("fn").sv;
      agg_fn = fn == "avg" ? 1 : fn == "sum" ? 2 : fn == "count" ? 3 : fn == "min" ? 4 : fn == "max" ? 5 : 0;
      if (!agg_fn) throw CompileError(-2, "aggregate: avg, sum, count, min or max");
      agg_state = a.present("state") ? (int)a.get("state").i() : -1;
      agg_col = a.present("column") ? (int)a.get("column").i() : -1;
      P.aggFn = (int8_t)agg_fn;
      P.aggState = (int8_t)agg_state;
      P.aggCol = (int8_t)agg_col;
    }
    P.type = root.get("type").sv == "sequence" ? SEQUENCE : PATTERN;
    P.within = root.get("within").i();
    P.playback = root.get("playback").b();
    P.partitioned = root.get("partitioned").b();
    const JV& states = root.get("states");
    P.nstates = (int)states.size();
    if (P.nstates < 1 || P.nstates > MAXS) throw CompileError(-2, "states: 1..8 supported");
    P.nstream = (int)root.get("streams").size();
    if (P.nstream > MAXSTREAM) throw CompileError(-2, "too many streams");
    const JV& cols = root.get("columns");
    P.ncol = (int)cols.size();
    if (P.ncol > MAXCOL) throw CompileError(-2, "too many predicate columns");
    for (int c = 0; c < P.ncol; c++) {
      int s = (int)cols[c].get("stream").i();
      P.colStream[c] = (int8_t)s;
      P.colTag[c] = tagOf(cols[c].get("type").sv);
      if (P.streamNcol[s] >= NV) throw CompileError(-2, "too many predicate columns on one stream");
      P.colPos[c] = P.streamNcol[s];
      P.streamCols[s][P.streamNcol[s]++] = (int8_t)c;
    }
    states_ = &states;
    for (int i = 0; i < P.nstates; i++) {
      filterPc_.push_back(-1);
      if (states[i].present("filter")) {
        if (depth(states[i].get("filter")) > MAXSTACK) throw CompileError(-2, "filter expression too deep");
        filterPc_[i] = (int)code_.size();
        emit(states[i].get("filter"));
        code_.push_back(Instr{OP_END, 0, 0, 0, 0, 0});
      }
    }
    if ((int)code_.size() > MAXCODE) throw CompileError(-2, "predicate program too long");
    verifyCode();
    P.ncode = (int)code_.size();
    for (size_t i = 0; i < code_.size(); i++) P.code[i] = code_[i];
    std::vector<int> all;
    Rt r = parse(root.get("tree"), -1, -1, true, all);
    for (int p : all) P.expireOrder[P.nexpire++] = (int8_t)p;
    if (P.within != -1) {
      for (int p : all)
        if (P.pre[p].isStart) P.startIds[P.nstart++] = P.pre[p].stateId;
    }
    P.pre[r.first].thisLast = (int16_t)r.last;
    setQuerySelector(r.node);
    setup(r.node);
    initOrder(r.node);
    resetOrder(r.node);
    updateOrder(r.node);
    for (int s = 0; s < P.nstream; s++) {
      P.recvMulti[s] = P.recvCount[s] > 1;
      if (P.recvCount[s] == 0) continue;
      if (P.recvMulti[s]) {
        int last = P.recvPre[s][P.recvCount[s] - 1];
        P.recvSelector[s] = P.post[P.pre[last].thisPost].hasNext;
      } else {
        int p = P.recvPre[s][0];
        P.recvSelector[s] = P.post[P.pre[p].thisLast].hasNext;
      }
    }
    detectFast(root);
    detectCseq(root);
    detectLabs(root);
  }

 private:
  const JV* states_ = nullptr;
  std::vector<Instr> code_;
  std::vector<int> filterPc_;

  struct TNode {
    enum T { STREAM, NEXT, EVERY, LOGICAL, COUNT } t;
    int first = -1, last = -1, leaf = -1;
    TNode *a = nullptr, *b = nullptr;
  };
  std::vector<std::unique_ptr<TNode>> nodes_;
  struct Rt {
    int first, last;
    TNode* node;
  };

  static int8_t tagOf(const std::string& t) {
    if (t == "int") return T_INT;
    if (t == "long") return T_LONG;
    if (t == "float") return T_FLOAT;
    if (t == "double") return T_DOUBLE;
    if (t == "bool") return T_BOOL;
    if (t == "string") return T_STR;
    return T_NULL;
  }

  void emit(const JV& e) {
    const std::string& op = e.get("op").sv;
    Instr in{};
    if (op == "const") {
      in.op = OP_CONST;
      in.a = (uint8_t)tagOf(e.get("type").sv);
      const JV& v = e.get("v");
      switch (in.a) {
        case T_FLOAT: { float f = (float)v.d(); uint32_t u; memcpy(&u, &f, 4); in.imm = u; break; }
        case T_DOUBLE: { double d = v.d(); memcpy(&in.imm, &d, 8); break; }
        case T_BOOL: in.imm = v.t == JV::BOOLEAN ? v.bv : v.i() != 0; break;
        default: in.imm = v.i(); break;
      }
      code_.push_back(in);
    } else if (op == "var") {
      in.op = OP_VAR;
      in.a = (uint8_t)e.get("state").i();
      in.b = (uint8_t)(int8_t)e.get("index").i();
      in.c = (uint8_t)e.get("col").i();
      code_.push_back(in);
    } else if (op == "isnullstate") {
      in.op = OP_ISNULLSTATE;
      in.a = (uint8_t)e.get("state").i();
      in.b = (uint8_t)(int8_t)e.get("index").i();
      code_.push_back(in);
    } else if (op == "and" || op == "or") {
      emit(e.get("a"));
      size_t j = code_.size();
      in.op = op == "and" ? OP_AND : OP_OR;
      code_.push_back(in);
      emit(e.get("b"));
      Instr end{};
      end.op = op == "and" ? OP_ANDEND : OP_OREND;
      code_.push_back(end);
      code_[j].d = (int32_t)code_.size();
    } else if (op == "not" || op == "isnull") {
      emit(e.get("a"));
      in.op = op == "not" ? OP_NOT : OP_ISNULL;
      code_.push_back(in);
    } else if (op == "cmp") {
      emit(e.get("a"));
      emit(e.get("b"));
      static const char* names[] = {"gt", "ge", "lt", "le", "eq", "ne"};
      in.op = OP_CMP;
      for (int i = 0; i < 6; i++)
        if (e.get("cmp").sv == names[i]) in.a = (uint8_t)i;
      in.b = promote(tagExpr(e.get("a")), tagExpr(e.get("b")));
      code_.push_back(in);
    } else if (op == "add" || op == "sub" || op == "mul" || op == "div" || op == "mod") {
      emit(e.get("a"));
      emit(e.get("b"));
      in.op = OP_ARITH;
      in.a = op == "add" ? 0 : op == "sub" ? 1 : op == "mul" ? 2 : op == "div" ? 3 : 4;
      in.b = (uint8_t)tagOf(e.get("type").sv);
      code_.push_back(in);
    } else if (op == "ifthenelse" || op == "coalesce") {
      const JV& a = e.get("args");
      for (size_t i = 0; i < a.size(); i++) emit(a[i]);
      in.op = op == "ifthenelse" ? OP_IFTE : OP_COALESCE;
      in.a = (uint8_t)a.size();
      if (op == "ifthenelse" && a.size() != 3) throw CompileError(-2, "ifThenElse takes 3 arguments");
      if (a.size() < 1 || a.size() > 8) throw CompileError(-2, "coalesce takes 1..8 arguments");
      code_.push_back(in);
    } else if (op == "instanceof") {
      emit(e.get("a"));
      in.op = OP_INSTOF;
      in.a = (uint8_t)tagOf(e.get("tag").sv);
      code_.push_back(in);
    } else {
      throw CompileError(-2, "unsupported predicate op " + op);
    }
  }

  // The device VM (run_filter) does no per-instruction bounds checks: every program is proven
  // safe here instead.  Abstract interpretation of the stack depth over every path of the
  // bytecode: each filter starts at depth 0, every pop has its operands, no push passes
  // MAXSTACK, jumps go forward and in range (so every run ends at its OP_END), and paths that
  // merge agree on the depth.
  void verifyCode() {
    const int n = (int)code_.size();
    std::vector<int> d(n + 1, -1);
    auto reach = [&](int pc, int depth) {
      if (pc < 0 || pc >= n) throw CompileError(-2, "predicate bytecode: jump out of range");
      if (depth < 0 || depth > MAXSTACK) throw CompileError(-2, "predicate bytecode: stack bound");
      if (d[pc] != -1 && d[pc] != depth) throw CompileError(-2, "predicate bytecode: inconsistent stack");
      d[pc] = depth;
    };
    for (int pc0 : filterPc_)
      if (pc0 >= 0) reach(pc0, 0);
    for (int pc = 0; pc < n; pc++) {  // forward-only jumps: one pass in pc order sees every path
      if (d[pc] < 0) continue;
      const Instr& in = code_[pc];
      const int s = d[pc];
      auto need = [&](int k) {
        if (s < k) throw CompileError(-2, "predicate bytecode: stack underflow");
      };
      switch (in.op) {
        case OP_END: need(1); break;
        case OP_CONST: case OP_VAR: case OP_ISNULLSTATE: reach(pc + 1, s + 1); break;
        case OP_AND: case OP_OR:
          need(1);
          if (in.d <= pc) throw CompileError(-2, "predicate bytecode: backward jump");
          reach(in.d, s);          // short circuit: the result replaces the operand
          reach(pc + 1, s - 1);
          break;
        case OP_ANDEND: case OP_OREND: case OP_NOT: case OP_ISNULL: case OP_INSTOF:
          need(1); reach(pc + 1, s); break;
        case OP_CMP: case OP_ARITH: need(2); reach(pc + 1, s - 1); break;
        case OP_IFTE: need(3); reach(pc + 1, s - 2); break;
        case OP_COALESCE:
          if (in.a < 1) throw CompileError(-2, "predicate bytecode: coalesce arity");
          need(in.a); reach(pc + 1, s - in.a + 1); break;
        default: throw CompileError(-2, "predicate bytecode: unknown op");
      }
    }
  }

  // evaluation-stack depth of an expression (the VM's stack holds MAXSTACK values)
  int depth(const JV& e) {
    const std::string& op = e.get("op").sv;
    if (op == "const" || op == "var" || op == "isnullstate") return 1;
    if (op == "and" || op == "or") return std::max(depth(e.get("a")), depth(e.get("b")));
    if (op == "not" || op == "isnull" || op == "instanceof") return depth(e.get("a"));
    if (op == "ifthenelse" || op == "coalesce") {
      const JV& a = e.get("args");
      int d = 0;
      for (size_t i = 0; i < a.size(); i++) d = std::max(d, (int)i + depth(a[i]));
      return d;
    }
    return std::max(depth(e.get("a")), 1 + depth(e.get("b")));  // cmp, arithmetic
  }

  int8_t tagExpr(const JV& e) {
    const std::string& op = e.get("op").sv;
    if (op == "const" || op == "var" || op == "add" || op == "sub" || op == "mul" || op == "div" || op == "mod" ||
        op == "ifthenelse" || op == "coalesce")
      return tagOf(e.get("type").sv);
    return T_BOOL;
  }
  static uint8_t promote(int8_t a, int8_t b) {
    if (a == T_STR || b == T_STR) return T_STR;
    if (a == T_BOOL || b == T_BOOL) return T_BOOL;
    if (a == T_NULL || b == T_NULL) return T_NULL;
    if (a == T_DOUBLE || b == T_DOUBLE) return T_DOUBLE;
    if (a == T_FLOAT || b == T_FLOAT) return T_FLOAT;
    if (a == T_LONG || b == T_LONG) return T_LONG;
    return T_INT;
  }

  int npost_ = 0;
  int newPre(int8_t kind) {
    if (P.npre >= MAXP) throw CompileError(-2, "too many processors");
    int id = P.npre++;
    DPre& p = P.pre[id];
    p.kind = kind;
    p.withinEvery = p.thisPost = p.thisLast = p.partner = p.countPost = -1;
    p.sched = -1;
    p.waiting = -1;
    return id;
  }
  int newPost(int8_t kind) {
    if (npost_ >= MAXP) throw CompileError(-2, "too many processors");
    int id = npost_++;
    DPost& q = P.post[id];
    q.kind = kind;
    q.nextState = q.nextEvery = q.thisPre = q.callbackPre = q.partnerPre = q.partnerPost = -1;
    return id;
  }
  int newSched(int pre) {
    if (P.nsched >= MAXQ) throw CompileError(-2, "too many absent states");
    P.schedPre[P.nsched] = (int8_t)pre;
    P.startup[P.nstartup++] = (int8_t)pre;
    return P.nsched++;
  }
  void setNextState(int q, int p) {
    DPost& Q = P.post[q];
    Q.nextState = (int16_t)p;
    if (Q.kind == K_LOGICAL || Q.kind == K_ABSENT_LOGICAL) {
      P.post[Q.partnerPost].nextState = (int16_t)p;
    } else if (Q.kind == K_COUNT) {
      DPre& tp = P.pre[Q.thisPre];
      if (tp.isStart && P.type == SEQUENCE && Q.minCount == 0) P.post[P.pre[p].thisPost].callbackPre = Q.thisPre;
    }
  }
  void setNextEvery(int q, int p) {
    DPost& Q = P.post[q];
    Q.nextEvery = (int16_t)p;
    if (Q.kind == K_LOGICAL || Q.kind == K_ABSENT_LOGICAL) P.post[Q.partnerPost].nextEvery = (int16_t)p;
  }

  TNode* mk(TNode::T t) {
    nodes_.push_back(std::make_unique<TNode>());
    nodes_.back()->t = t;
    return nodes_.back().get();
  }

  Rt parse(const JV& t, int pre, int post, bool isStart, std::vector<int>& list) {
    const std::string& k = t.get("t").sv;
    if (k == "stream" || k == "absent") {
      int sid = (int)t.get("state").i();
      const JV& sj = (*states_)[sid];
      bool absent = k == "absent";
      if (pre < 0) {
        if (absent) {
          pre = newPre(K_ABSENT_STREAM);
          P.pre[pre].waiting = sj.get("waiting").i();
          P.pre[pre].sched = (int8_t)newSched(pre);
        } else {
          pre = newPre(K_STREAM);
        }
      }
      DPre& p = P.pre[pre];
      p.stateId = (int8_t)sid;
      p.stream = (int8_t)sj.get("stream").i();
      p.isStart = isStart;
      p.filterPc = (int16_t)filterPc_[sid];
      if (post < 0) post = newPost(absent ? K_ABSENT_STREAM : K_STREAM);
      P.post[post].stateId = (int8_t)sid;
      P.post[post].thisPre = (int16_t)pre;
      p.thisPost = (int16_t)post;
      p.thisLast = (int16_t)post;
      list.push_back(pre);
      TNode* n = mk(TNode::STREAM);
      n->first = pre;
      n->last = post;
      n->leaf = pre;
      return {pre, post, n};
    }
    if (k == "next") {
      Rt a = parse(t.get("a"), pre, post, isStart, list);
      Rt b = parse(t.get("b"), pre, post, false, list);
      setNextState(a.last, b.first);
      TNode* n = mk(TNode::NEXT);
      n->a = a.node;
      n->b = b.node;
      n->first = a.first;
      n->last = b.last;
      return {a.first, b.last, n};
    }
    if (k == "every") {
      std::vector<int> inner;
      Rt a = parse(t.get("x"), pre, post, isStart, inner);
      setNextEvery(a.last, a.first);
      for (int p : inner) P.pre[p].withinEvery = (int16_t)a.first;
      list.insert(list.end(), inner.begin(), inner.end());
      TNode* n = mk(TNode::EVERY);
      n->a = a.node;
      n->first = a.first;
      n->last = a.last;
      return {a.first, a.last, n};
    }
    if (k == "logical") {
      int8_t lt = t.get("op").sv == "or" ? L_OR : L_AND;
      const JV& e1 = t.get("s1");
      const JV& e2 = t.get("s2");
      int p1, p2, q1, q2;
      auto make = [&](const JV& e, int& lp, int& lq) {
        bool abs = e.get("t").sv == "absent";
        lp = newPre(abs ? K_ABSENT_LOGICAL : K_LOGICAL);
        if (abs) {
          P.pre[lp].waiting = (*states_)[(int)e.get("state").i()].get("waiting").i();
          P.pre[lp].sched = (int8_t)newSched(lp);
        }
        P.pre[lp].logical = lt;
        lq = newPost(abs ? K_ABSENT_LOGICAL : K_LOGICAL);
        P.post[lq].logical = lt;
      };
      make(e1, p1, q1);
      make(e2, p2, q2);
      P.post[q1].partnerPre = (int16_t)p2;
      P.post[q2].partnerPre = (int16_t)p1;
      P.post[q1].partnerPost = (int16_t)q2;
      P.post[q2].partnerPost = (int16_t)q1;
      P.pre[p1].partner = (int16_t)p2;
      P.pre[p2].partner = (int16_t)p1;
      Rt r2 = parse(e2, p2, q2, isStart, list);
      Rt r1 = parse(e1, p1, q1, isStart, list);
      TNode* n = mk(TNode::LOGICAL);
      n->a = r1.node;
      n->b = r2.node;
      n->first = r1.first;
      n->last = r2.last;
      return {r1.first, r2.last, n};
    }
    if (k == "count") {
      int cp = newPre(K_COUNT), cq = newPost(K_COUNT);
      int mn = (int)t.get("min").i(), mx = (int)t.get("max").i();
      P.pre[cp].minCount = P.post[cq].minCount = mn;
      P.pre[cp].maxCount = P.post[cq].maxCount = mx < 0 ? 0x7fffffff : mx;
      P.pre[cp].countPost = (int16_t)cq;
      JV leaf;
      leaf.t = JV::OBJECT;
      JV ts;
      ts.t = JV::STRING;
      ts.sv = "stream";
      leaf.ov.emplace_back("t", ts);
      leaf.ov.emplace_back("state", t.get("state"));
      Rt r = parse(leaf, cp, cq, isStart, list);
      r.node->t = TNode::COUNT;
      return r;
    }
    throw CompileError(-2, "unsupported state element " + k);
  }

  void setQuerySelector(TNode* n) {
    switch (n->t) {
      case TNode::STREAM:
      case TNode::COUNT: P.post[n->last].hasNext = 1; break;
      case TNode::NEXT: setQuerySelector(n->b); break;
      case TNode::EVERY: setQuerySelector(n->a); break;
      case TNode::LOGICAL: setQuerySelector(n->b); setQuerySelector(n->a); break;
    }
  }
  void setup(TNode* n) {
    switch (n->t) {
      case TNode::STREAM:
      case TNode::COUNT: {
        int s = P.pre[n->leaf].stream;
        P.recvPre[s][P.recvCount[s]++] = (int8_t)n->leaf;
        break;
      }
      case TNode::NEXT: setup(n->a); setup(n->b); break;
      case TNode::EVERY: setup(n->a); break;
      case TNode::LOGICAL: setup(n->b); setup(n->a); break;
    }
  }
  void initOrder(TNode* n) {
    switch (n->t) {
      case TNode::STREAM:
      case TNode::COUNT: P.initOrder[P.ninit++] = (int8_t)n->leaf; break;
      case TNode::NEXT: initOrder(n->a); initOrder(n->b); break;
      case TNode::EVERY: initOrder(n->a); break;
      case TNode::LOGICAL: initOrder(n->b); initOrder(n->a); break;
    }
  }
  void resetOrder(TNode* n) {
    switch (n->t) {
      case TNode::NEXT: resetOrder(n->b); resetOrder(n->a); break;
      case TNode::LOGICAL: resetOrder(n->b); break;
      default: P.resetOrder[P.nreset++] = (int8_t)n->first; break;
    }
  }
  void updateOrder(TNode* n) {
    switch (n->t) {
      case TNode::NEXT: updateOrder(n->a); updateOrder(n->b); break;
      case TNode::LOGICAL: updateOrder(n->b); break;
      default: P.updateOrder[P.nupdate++] = (int8_t)n->first; break;
    }
  }

  bool fastOperand(const JV& e, FOperand& o) {
    const std::string& op = e.get("op").sv;
    o = FOperand{};
    if (op == "const") {
      o.kind = 0;
      o.tag = tagOf(e.get("type").sv);
      const JV& v = e.get("v");
      switch (o.tag) {
        case T_FLOAT: { float f = (float)v.d(); uint32_t u; memcpy(&u, &f, 4); o.imm = u; break; }
        case T_DOUBLE: { double d = v.d(); memcpy(&o.imm, &d, 8); break; }
        case T_BOOL: o.imm = v.t == JV::BOOLEAN ? v.bv : v.i() != 0; break;
        case T_NULL: return false;
        default: o.imm = v.i(); break;
      }
      return true;
    }
    if (op == "var") {
      int idx = (int)e.get("index").i();
      int stt = (int)e.get("state").i();
      if (!(idx == 0 || idx == -1) || stt < 0 || stt > 1) return false;
      o.kind = 1;
      o.state = (int8_t)stt;
      int col = (int)e.get("col").i();
      o.pos = P.colPos[col];
      o.tag = P.colTag[col];
      return true;
    }
    return false;
  }
  bool fastTerm(const JV& e, FTerm& t) {
    if (e.get("op").sv != "cmp") return false;
    static const char* names[] = {"gt", "ge", "lt", "le", "eq", "ne"};
    t = FTerm{};
    for (int i = 0; i < 6; i++)
      if (e.get("cmp").sv == names[i]) t.cmp = (int8_t)i;
    if (!fastOperand(e.get("a"), t.a) || !fastOperand(e.get("b"), t.b)) return false;
    t.ptype = (int8_t)promote(t.a.tag, t.b.tag);
    return t.ptype != T_NULL;
  }
  bool fastPred(const JV& f, FPred& p) {
    p = FPred{};
    if (f.t == JV::NIL) return true;
    const std::string& op = f.get("op").sv;
    if (op == "cmp") {
      p.n = 1;
      return fastTerm(f, p.t[0]);
    }
    if (op == "and" || op == "or") {
      p.n = 2;
      p.combine = op == "or";
      return fastTerm(f.get("a"), p.t[0]) && fastTerm(f.get("b"), p.t[1]);
    }
    return false;
  }

  // every e1=S[f1] -> e2=S[f2] within W  (SURVEY.md Appendix A.7 closed form)
  void detectFast(const JV& root) {
    fast.ok = 0;
    const JV& t = root.get("tree");
    if (P.type != PATTERN || P.nstates != 2 || P.within < 0 || P.nsched != 0) return;
    if (t.get("t").sv != "next") return;
    const JV& a = t.get("a");
    const JV& b = t.get("b");
    if (a.get("t").sv != "every" || a.get("x").get("t").sv != "stream" || b.get("t").sv != "stream") return;
    if (a.get("x").get("state").i() != 0 || b.get("state").i() != 1) return;
    if (P.pre[0].stream != P.pre[1].stream) return;
    if (P.ncol > 2) return;
    const JV& st = root.get("states");
    if (!fastPred(st[0].get("filter"), fast.f1) || !fastPred(st[1].get("filter"), fast.f2)) return;
    fast.ok = 1;
    fast.stream = P.pre[0].stream;
    fast.within = P.within;
  }

  // every var operand of state `st` in the filter has index `idx` (e1[last] in e2's filter)
  static bool varIndex(const JV& e, int st, int idx) {
    if (e.t != JV::OBJECT) return true;
    if (e.get("op").sv == "var") return e.get("state").i() != st || e.get("index").i() == idx;
    for (const char* k : {"a", "b"})
      if (!varIndex(e.get(k), st, idx)) return false;
    return true;
  }

  // ---- logical-absent shape (labs.h)
  bool laOperand(const JV& e, LaOperand& o, int s1, int s2, int s3) {
    const std::string& op = e.get("op").sv;
    o = LaOperand{};
    if (op == "const") {
      FOperand f;
      if (!fastOperand(e, f)) return false;
      o.kind = 0;
      o.tag = f.tag;
      o.imm = f.imm;
      return true;
    }
    if (op != "var") return false;
    const int idx = (int)e.get("index").i(), st = (int)e.get("state").i();
    if (!(idx == 0 || idx == -1) || !(st == s1 || st == s2 || st == s3)) return false;
    o.kind = 1;
    o.state = (int8_t)st;
    o.col = (int32_t)e.get("col").i();
    o.tag = P.colTag[o.col];
    return true;
  }
  bool laPred(const JV& f, LaPredS& p, int s1, int s2, int s3) {
    p = LaPredS{};
    if (f.t == JV::NIL) return true;
    auto term = [&](const JV& e, LaTermS& t) {
      if (e.get("op").sv != "cmp") return false;
      static const char* names[] = {"gt", "ge", "lt", "le", "eq", "ne"};
      t = LaTermS{};
      t.cmp = -1;
      for (int i = 0; i < 6; i++)
        if (e.get("cmp").sv == names[i]) t.cmp = (int8_t)i;
      if (t.cmp < 0 || !laOperand(e.get("a"), t.a, s1, s2, s3) || !laOperand(e.get("b"), t.b, s1, s2, s3)) return false;
      t.ptype = (int8_t)promote(t.a.tag, t.b.tag);
      return t.ptype != T_NULL && t.ptype != T_BOOL;
    };
    const std::string& op = f.get("op").sv;
    if (op == "cmp") {
      p.n = 1;
      return term(f, p.t[0]);
    }
    if (op == "and" || op == "or") {
      p.n = 2;
      p.combine = op == "or";
      return term(f.get("a"), p.t[0]) && term(f.get("b"), p.t[1]);
    }
    return false;
  }

  // every (x=X[fx] and y=Y[fy]) -> not Z[fz] for T [within W], playback, three distinct streams
  void detectLabs(const JV& root) {
    labs = LabsShape{};
    const JV& t = root.get("tree");
    if (P.type != PATTERN || P.nstates != 3 || !P.playback || P.nsched != 1) return;
    if (t.get("t").sv != "next") return;
    const JV& a = t.get("a");
    const JV& b = t.get("b");
    if (a.get("t").sv != "every" || b.get("t").sv != "absent") return;
    const JV& l = a.get("x");
    if (l.get("t").sv != "logical" || l.get("op").sv != "and") return;
    if (l.get("s1").get("t").sv != "stream" || l.get("s2").get("t").sv != "stream") return;
    const int sx = (int)l.get("s1").get("state").i(), sy = (int)l.get("s2").get("state").i();
    const int sz = (int)b.get("state").i();
    if (sx == sy || sx == sz || sy == sz || sx < 0 || sy < 0 || sz < 0 || sx > 2 || sy > 2 || sz > 2) return;
    const JV& st = root.get("states");
    const int stx = (int)st[sx].get("stream").i(), sty = (int)st[sy].get("stream").i(), stz = (int)st[sz].get("stream").i();
    if (stx == sty || stx == stz || sty == stz) return;
    if (st[sz].get("waiting").i() <= 0) return;
    for (int s : {stx, sty, stz})
      if (P.streamNcol[s] > 1) return;
    for (int c = 0; c < P.ncol; c++)
      if (!(P.colTag[c] == T_INT || P.colTag[c] == T_FLOAT || P.colTag[c] == T_STR)) return;
    // x's and y's filters read their own event only; z's reads the Z event, x and y
    if (!laPred(st[sx].get("filter"), labs.fx, sx, sx, sx) || !laPred(st[sy].get("filter"), labs.fy, sy, sy, sy) ||
        !laPred(st[sz].get("filter"), labs.fz, sx, sy, sz))
      return;
    labs.sx = sx;
    labs.sy = sy;
    labs.sz = sz;
    labs.stx = stx;
    labs.sty = sty;
    labs.stz = stz;
    labs.colx = P.streamNcol[stx] ? P.streamCols[stx][0] : -1;
    labs.coly = P.streamNcol[sty] ? P.streamCols[sty][0] : -1;
    labs.colz = P.streamNcol[stz] ? P.streamCols[stz][0] : -1;
    labs.wait = st[sz].get("waiting").i();
    labs.within = P.within;
    labs.ok = 1;
  }

  // every e1=S[f1]<1:M>, e2=S[f2] (sequence, no within): a per-key automaton over the count of
  // e1's chain (cseq.h).  f1 reads e1's own value, f2 e2's and e1[last]'s.
  void detectCseq(const JV& root) {
    cseq.ok = 0;
    const JV& t = root.get("tree");
    if (P.type != SEQUENCE || P.nstates != 2 || P.within >= 0 || P.nsched != 0 || P.playback || P.nstream != 1)
      return;
    if (t.get("t").sv != "next") return;
    const JV& a = t.get("a");
    const JV& b = t.get("b");
    if (b.get("t").sv != "stream" || b.get("state").i() != 1) return;
    const bool every = a.get("t").sv == "every";  // (without it the start is armed once: cseq.h cs_tables)
    const JV& c = every ? a.get("x") : a;
    if (c.get("t").sv != "count" || c.get("state").i() != 0) return;
    const int64_t mn = c.get("min").i(), mx = c.get("max").i();
    if (mx < 1 || mx > CSEQ_MAXM || mn < 1 || mn > mx) return;
    if (P.pre[0].stream != P.pre[1].stream || P.ncol > 1) return;
    const JV& st = root.get("states");
    const JV& f1 = st[0].get("filter");
    const JV& f2 = st[1].get("filter");
    // f1 reads only the arriving event (e1's own value), f2 e1[last] and e2
    if (!varIndex(f1, 1, 0x7fff) || !varIndex(f1, 0, -1) || !varIndex(f2, 0, -1)) return;
    if (!fastPred(f1, cseq.f1) || !fastPred(f2, cseq.f2)) return;
    cseq.M = (int32_t)mx;
    cseq.every = every ? 1 : 0;
    cseq.minc = (int32_t)mn;
    cseq.ok = 1;
  }
};

}  // namespace shp
