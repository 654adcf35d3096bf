// ============================================================================
// siddhi-hip ORACLE — TEST INFRASTRUCTURE ONLY.
//
// A CPU restatement, at the level of the reference's processor objects, of
// Siddhi's pattern/sequence path (io.siddhi.core.query.input.stream.state).
// It is the parity checker for libsiddhi_hip.so and the "port" CPU baseline.
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
// it; the product path never does.
//
// Parity pin: the reference (Java 8 / Maven) cannot be built or run in this
// image (no JDK, no jars). The restatement is pinned by the
// reference's own known-answer tests, transcribed as data into tests/golden/
// (tests/golden/extract_golden.py), which this oracle must reproduce exactly.
//
// Every method below names the Java method it restates (paths relative to
// modules/siddhi-core/src/main/java/io/siddhi/core/query/input/stream/state/
// unless noted). Object identity and aliasing are modelled with
// reference-counted StateEvent / StreamEvent objects exactly like the Java
// heap: StateEventCloner copies slot *pointers* (shallow), count chains are
// linked StreamEvents shared between StateEvents.
// ============================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <list>
#include <map>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "mini_json.h"

namespace oracle {

using std::shared_ptr;
using std::vector;

// ---------------------------------------------------------------- values
enum VT : uint8_t { T_NULL, T_INT, T_LONG, T_FLOAT, T_DOUBLE, T_BOOL, T_STR };

struct Val {
  VT t = T_NULL;
  int32_t i = 0;
  int64_t l = 0;
  float f = 0;
  double d = 0;
  bool b = false;
};

static VT type_of(const std::string& s) {
  if (s == "int") return T_INT;
  if (s == "long") return T_LONG;
  if (s == "float") return T_FLOAT;
  if (s == "double") return T_DOUBLE;
  if (s == "bool") return T_BOOL;
  if (s == "string") return T_STR;
  return T_NULL;
}

// ------------------------------------------------------------ event model
// StreamEvent (core/event/stream/StreamEvent.java): data is immutable on the
// state path, so a clone references the source event's row by `seq`.
struct StreamEv {
  int64_t seq;  // -1 = StreamEventFactory.newInstance() (all-null, ts -1)
  int64_t ts;
  shared_ptr<StreamEv> next;
};
using SEv = shared_ptr<StreamEv>;

enum EvType { CURRENT = 0, EXPIRED = 1 };

// StateEvent (core/event/state/StateEvent.java:42-258)
struct StateEv {
  vector<SEv> slots;
  int64_t ts = -1;
  int type = CURRENT;
  int64_t id = 0;
};
using StEv = shared_ptr<StateEv>;

// StateEvent.getStreamEvent(int[]) :138-189
static SEv get_stream_event(const StateEv& se, int state, int index) {
  SEv ev = se.slots[state];
  if (!ev) return nullptr;
  if (index >= 0) {
    for (int i = 1; i <= index; i++) {
      ev = ev->next;
      if (!ev) return nullptr;
    }
  } else if (index == -1) {  // CURRENT
    while (ev->next) ev = ev->next;
  } else if (index == -2) {  // LAST
    if (!ev->next) return nullptr;
    while (ev->next->next) ev = ev->next;
  } else {
    vector<SEv> lst;
    while (ev) { lst.push_back(ev); ev = ev->next; }
    long idx = (long)lst.size() + index;
    if (idx < 0) return nullptr;
    ev = lst[idx];
  }
  return ev;
}

// StateEvent.addEvent :212-222
static void add_event(StateEv& se, int pos, SEv ev) {
  SEv a = se.slots[pos];
  if (!a) { se.slots[pos] = ev; return; }
  while (a->next) a = a->next;
  a->next = ev;
}

// StateEvent.removeLastEvent :224-236
static void remove_last_event(StateEv& se, int pos) {
  SEv a = se.slots[pos];
  if (a) {
    while (a->next) {
      if (!a->next->next) { a->next = nullptr; return; }
      a = a->next;
    }
    se.slots[pos] = nullptr;
  }
}

// -------------------------------------------------------------- program
struct Expr {
  std::string op;
  VT type = T_NULL;
  Val cval;
  int state = -1, col = -1, index = -1;
  int cmp = 0;  // 0 gt 1 ge 2 lt 3 le 4 eq 5 ne
  vector<std::unique_ptr<Expr>> args;
};

enum Kind { K_STREAM, K_COUNT, K_LOGICAL, K_ABSENT_STREAM, K_ABSENT_LOGICAL };
enum SeqType { PATTERN, SEQUENCE };
enum LogicalType { L_AND, L_OR };

struct Engine;
struct Pre;

struct Post {
  int id = 0;
  Kind kind = K_STREAM;
  int stateId = 0;
  Pre* nextStatePre = nullptr;
  Pre* nextEveryPre = nullptr;
  Pre* thisPre = nullptr;
  bool hasNext = false;       // nextProcessor != null (the QuerySelector)
  Pre* callbackPre = nullptr;  // CountPreStateProcessor
  bool isEventReturned = false;  // NOTE: a plain field, shared by all keys (as in Java)
  int minCount = 0, maxCount = 0;
  int logicalType = L_AND;
  Pre* partnerPre = nullptr;
  Post* partnerPost = nullptr;
};

struct PreState {
  std::list<StEv> pending, newAndEvery;
  bool stateChanged = false, initialized = false, started = false;
  bool successCondition = false, startStateReset = false;
  int64_t lastScheduledTime = 0, lastArrivalTime = 0;
  bool active = true;
};

struct KeyCtx;

struct Pre {
  int id = 0;
  Kind kind = K_STREAM;
  int stateId = 0;
  int stream = 0;
  bool isStartState = false;
  SeqType stateType = PATTERN;
  int64_t withinTime = -1;
  vector<int> startStateIds;
  Pre* withinEveryPre = nullptr;
  Post* thisPost = nullptr;
  Post* thisLast = nullptr;
  const Expr* filter = nullptr;
  int minCount = 0, maxCount = 0;
  Post* countPost = nullptr;
  int logicalType = L_AND;
  Pre* partner = nullptr;
  int64_t waitingTime = -1;
  int scheduler = -1;
  bool isAbsent() const { return kind == K_ABSENT_STREAM || kind == K_ABSENT_LOGICAL; }
  bool isLogical() const { return kind == K_LOGICAL || kind == K_ABSENT_LOGICAL; }
};

struct SchedState {
  std::list<int64_t> queue;  // LinkedBlockingQueue: FIFO, not sorted (core/util/Scheduler.java:332)
};

struct KeyCtx {
  int32_t key;
  vector<PreState> pre;
  vector<SchedState> sched;
};

// inner state runtime tree (state/runtime/*.java)
struct Node {
  enum T { STREAM, NEXT, EVERY, LOGICAL, COUNT } t;
  Pre* first = nullptr;
  Post* last = nullptr;
  std::unique_ptr<Node> a, b;  // NEXT: a=current b=next; EVERY: a=inner; LOGICAL: a=r1, b=r2
  Pre* leafPre = nullptr;      // STREAM/COUNT
};

struct Receiver {
  bool multi = false;
  vector<Pre*> forStream;  // stateProcessorsForStream, registration (setup) order
};

struct Match {
  int32_t key;
  int64_t ts;
  int8_t type;
  int64_t pos;
  vector<vector<int64_t>> slots;
};

struct Column {
  VT type;
  int stream;
  vector<int32_t> i32;
  vector<int64_t> i64;
  vector<float> f32;
  vector<double> f64;
  vector<uint8_t> nul;
};

struct Engine {
  SeqType type = PATTERN;
  int64_t within = -1;
  bool playback = true;
  bool partitioned = false;
  int nstates = 0;
  vector<std::unique_ptr<Expr>> filters;
  vector<std::unique_ptr<Pre>> pres;    // created order
  vector<std::unique_ptr<Post>> posts;
  vector<Pre*> preStateProcessors;      // parse order == stateId order
  vector<Pre*> startup;                 // startupPreStateProcessors (absent)
  vector<Pre*> schedulers;              // scheduler index -> owning absent processor
  std::unique_ptr<Node> root;
  vector<Receiver> receivers;           // per stream id
  vector<int> streamStateCount;
  vector<Column> cols;

  // run-time
  int64_t clock = 0;
  int64_t nevents = 0;
  vector<int64_t> ev_ts;
  vector<int64_t> ev_clk;   // value handed to setCurrentTimestamp (the caller's clock column, else ts)
  vector<int64_t> ev_gseq;  // the caller's sequence numbers (seq column, else the running count)
  std::unordered_map<int32_t, size_t> keyIndex;
  vector<std::unique_ptr<KeyCtx>> keys;
  KeyCtx* cur = nullptr;
  vector<Match> out;
  int64_t emit_pos = 0;
  int64_t timer_ties = 0;
  int64_t dropped_returns = 0;
  int64_t next_id = 0;

  PreState& S(Pre* p) { return cur->pre[p->id]; }

  // ------------------------------------------------------------ factories
  StEv newStateEvent() {
    auto se = std::make_shared<StateEv>();
    se->slots.assign(nstates, nullptr);
    se->id = next_id++;
    return se;
  }
  // StateEventCloner.copyStateEvent (core/event/state/StateEventCloner.java:48-61): shallow slots
  StEv copyStateEvent(const StEv& s) {
    auto n = std::make_shared<StateEv>();
    n->slots = s->slots;
    n->type = s->type;
    n->ts = s->ts;
    n->id = s->id;
    return n;
  }
  // StreamEventCloner.copyStreamEvent: new object, next = null
  SEv cloneStreamEvent(int64_t seq) {
    auto e = std::make_shared<StreamEv>();
    e->seq = seq;
    e->ts = seq >= 0 ? ev_ts[seq] : -1;
    return e;
  }
  SEv emptyStreamEvent() {
    auto e = std::make_shared<StreamEv>();
    e->seq = -1;
    e->ts = -1;
    return e;
  }

  // --------------------------------------------------- expression executor
  Val attr(int64_t seq, int col) {
    Val v;
    if (seq < 0) return v;
    const Column& c = cols[col];
    if (!c.nul.empty() && c.nul[seq]) return v;
    v.t = c.type;
    switch (c.type) {
      case T_INT: v.i = c.i32[seq]; break;
      case T_STR: v.i = c.i32[seq]; break;
      case T_BOOL: v.b = c.i32[seq] != 0; break;
      case T_LONG: v.l = c.i64[seq]; break;
      case T_FLOAT: v.f = c.f32[seq]; break;
      case T_DOUBLE: v.d = c.f64[seq]; break;
      default: break;
    }
    return v;
  }

  static double asD(const Val& v) {
    switch (v.t) {
      case T_INT: return (double)v.i;
      case T_LONG: return (double)v.l;
      case T_FLOAT: return (double)v.f;
      default: return v.d;
    }
  }
  static float asF(const Val& v) {
    switch (v.t) {
      case T_INT: return (float)v.i;
      case T_LONG: return (float)v.l;
      case T_FLOAT: return v.f;
      default: return (float)v.d;
    }
  }
  static int64_t asL(const Val& v) { return v.t == T_INT ? (int64_t)v.i : v.l; }

  template <class T>
  static bool cmpT(int c, T a, T b) {
    switch (c) {
      case 0: return a > b;
      case 1: return a >= b;
      case 2: return a < b;
      case 3: return a <= b;
      case 4: return a == b;
      default: return a != b;
    }
  }

  Val eval(const Expr* e, const StateEv& se) {
    Val r;
    const std::string& op = e->op;
    if (op == "const") return e->cval;
    if (op == "var") {
      SEv ev = get_stream_event(se, e->state, e->index);
      if (!ev) return r;
      return attr(ev->seq, e->col);
    }
    if (op == "and") {  // AndConditionExpressionExecutor.java:65-74
      Val a = eval(e->args[0].get(), se);
      r.t = T_BOOL;
      if (a.t == T_BOOL && a.b) {
        Val b = eval(e->args[1].get(), se);
        r.b = b.t == T_BOOL && b.b;
      }
      return r;
    }
    if (op == "or") {  // OrConditionExpressionExecutor.java:65-76
      Val a = eval(e->args[0].get(), se);
      r.t = T_BOOL;
      if (a.t == T_BOOL && a.b) { r.b = true; return r; }
      Val b = eval(e->args[1].get(), se);
      r.b = b.t == T_BOOL && b.b;
      return r;
    }
    if (op == "not") {  // NotConditionExpressionExecutor.java:43-50 (null -> TRUE)
      Val a = eval(e->args[0].get(), se);
      r.t = T_BOOL;
      r.b = !(a.t == T_BOOL && a.b);
      return r;
    }
    if (op == "isnull") {
      Val a = eval(e->args[0].get(), se);
      r.t = T_BOOL;
      r.b = a.t == T_NULL;
      return r;
    }
    // scalar functions: FunctionExecutor.execute (core/executor/function/FunctionExecutor.java:85-99)
    // evaluates every argument, then the function body
    if (op == "ifthenelse") {  // IfThenElseFunctionExecutor.execute: Boolean.TRUE.equals(data[0])
      Val c = eval(e->args[0].get(), se);
      Val a = eval(e->args[1].get(), se);
      Val b = eval(e->args[2].get(), se);
      return (c.t == T_BOOL && c.b) ? a : b;
    }
    if (op == "coalesce") {  // CoalesceFunctionExecutor.execute: the first non-null argument
      Val out;
      bool found = false;
      for (auto& x : e->args) {
        Val v = eval(x.get(), se);
        if (!found && v.t != T_NULL) {
          out = v;
          found = true;
        }
      }
      return out;
    }
    if (op == "instanceof") {  // InstanceOf*FunctionExecutor.execute: data instanceof <Type>
      Val a = eval(e->args[0].get(), se);
      r.t = T_BOOL;
      r.b = a.t == e->type && a.t != T_NULL;
      return r;
    }
    if (op == "isnullstate") {  // IsNullStreamConditionExpressionExecutor.java:36-52
      r.t = T_BOOL;
      r.b = get_stream_event(se, e->state, e->index) == nullptr;
      return r;
    }
    if (op == "cmp") {  // CompareConditionExpressionExecutor.java:38-44 + typed leaves
      Val a = eval(e->args[0].get(), se);
      Val b = eval(e->args[1].get(), se);
      r.t = T_BOOL;
      if (a.t == T_NULL || b.t == T_NULL) { r.b = false; return r; }
      if (a.t == T_STR || b.t == T_STR || a.t == T_BOOL || b.t == T_BOOL) {
        bool eq = (a.t == T_BOOL) ? (a.b == b.b) : (a.i == b.i);
        r.b = e->cmp == 4 ? eq : !eq;
        return r;
      }
      if (a.t == T_DOUBLE || b.t == T_DOUBLE) r.b = cmpT<double>(e->cmp, asD(a), asD(b));
      else if (a.t == T_FLOAT || b.t == T_FLOAT) r.b = cmpT<float>(e->cmp, asF(a), asF(b));
      else if (a.t == T_LONG || b.t == T_LONG) r.b = cmpT<int64_t>(e->cmp, asL(a), asL(b));
      else r.b = cmpT<int32_t>(e->cmp, a.i, b.i);
      return r;
    }
    // arithmetic (core/executor/math/*): result type e->type, Java semantics
    Val a = eval(e->args[0].get(), se);
    Val b = eval(e->args[1].get(), se);
    if (a.t == T_NULL || b.t == T_NULL) return r;
    r.t = e->type;
    char o = op[0];  // add sub mul div mod
    if (e->type == T_DOUBLE) {
      double x = asD(a), y = asD(b);
      if ((op == "div" || op == "mod") && y == 0.0) return Val();
      r.d = op == "add" ? x + y : op == "sub" ? x - y : op == "mul" ? x * y : op == "div" ? x / y : std::fmod(x, y);
    } else if (e->type == T_FLOAT) {
      float x = asF(a), y = asF(b);
      if ((op == "div" || op == "mod") && y == 0.0f) return Val();
      r.f = op == "add" ? x + y : op == "sub" ? x - y : op == "mul" ? x * y : op == "div" ? x / y : std::fmod(x, y);
    } else if (e->type == T_LONG) {
      int64_t x = asL(a), y = asL(b);
      if ((op == "div" || op == "mod") && y == 0) return Val();
      uint64_t ux = (uint64_t)x, uy = (uint64_t)y;
      if (op == "add") r.l = (int64_t)(ux + uy);
      else if (op == "sub") r.l = (int64_t)(ux - uy);
      else if (op == "mul") r.l = (int64_t)(ux * uy);
      else if (op == "div") r.l = (x == INT64_MIN && y == -1) ? x : x / y;
      else r.l = (y == -1) ? 0 : x % y;
    } else {
      int32_t x = a.t == T_INT ? a.i : (int32_t)asL(a), y = b.t == T_INT ? b.i : (int32_t)asL(b);
      if ((op == "div" || op == "mod") && y == 0) return Val();
      uint32_t ux = (uint32_t)x, uy = (uint32_t)y;
      if (op == "add") r.i = (int32_t)(ux + uy);
      else if (op == "sub") r.i = (int32_t)(ux - uy);
      else if (op == "mul") r.i = (int32_t)(ux * uy);
      else if (op == "div") r.i = (x == INT32_MIN && y == -1) ? x : x / y;
      else r.i = (y == -1) ? 0 : x % y;
    }
    (void)o;
    return r;
  }

  // ----------------------------------------------------------- scheduler
  void notifyAt(int sched, int64_t t) { cur->sched[sched].queue.push_back(t); }  // Scheduler.notifyAt :113-127

  // --------------------------------------------------------------- emit
  void emit(const StEv& se) {
    Match m;
    m.key = cur->key;
    m.ts = se->ts;
    m.type = (int8_t)se->type;
    m.pos = emit_pos;
    m.slots.resize(nstates);
    for (int s = 0; s < nstates; s++) {
      for (SEv e = se->slots[s]; e; e = e->next) m.slots[s].push_back(e->seq);
    }
    out.push_back(std::move(m));
  }

  // =====================================================================
  // PreStateProcessor family
  // =====================================================================

  // StreamPreStateProcessor.init :178-194
  void init(Pre* p) {
    PreState& st = S(p);
    if (p->isStartState &&
        (!st.initialized || p->thisPost->nextEveryPre != nullptr ||
         (p->stateType == SEQUENCE && p->thisPost->nextStatePre && p->thisPost->nextStatePre->isAbsent()))) {
      StEv se = newStateEvent();
      addState(p, se);
      st.initialized = true;
    }
  }

  void addState(Pre* p, const StEv& se) {
    PreState& st = S(p);
    switch (p->kind) {
      case K_STREAM:  // StreamPreStateProcessor.addState :214-227
        if (p->stateType == SEQUENCE) {
          if (st.newAndEvery.empty()) st.newAndEvery.push_back(se);
        } else {
          st.newAndEvery.push_back(se);
        }
        break;
      case K_COUNT:  // CountPreStateProcessor.addState :114-138
        if (p->stateType == SEQUENCE) {
          if (st.newAndEvery.empty()) st.newAndEvery.push_back(se);
        } else {
          st.newAndEvery.push_back(se);
        }
        if (p->minCount == 0 && se->slots[p->stateId] == nullptr) processMinCountReached(p->countPost, se);
        break;
      case K_LOGICAL:
        logicalAddState(p, se);
        break;
      case K_ABSENT_STREAM:  // AbsentStreamPreStateProcessor.addState :80-103
        if (!st.active) return;
        if (p->stateType == SEQUENCE) {
          st.newAndEvery.clear();
          st.newAndEvery.push_back(se);
        } else {
          st.newAndEvery.push_back(se);
        }
        if (!p->isStartState) {
          st.lastScheduledTime = se->ts + p->waitingTime;
          notifyAt(p->scheduler, st.lastScheduledTime);
        }
        break;
      case K_ABSENT_LOGICAL:  // AbsentLogicalPreStateProcessor.addState :77-97
        if (!st.active) return;
        logicalAddState(p, se);
        if (!p->isStartState) {
          if (p->waitingTime != -1) {
            notifyAt(p->scheduler, se->ts + p->waitingTime);
            if (p->partner->kind == K_ABSENT_LOGICAL)
              notifyAt(p->partner->scheduler, se->ts + p->partner->waitingTime);
          }
        }
        break;
    }
  }

  // LogicalPreStateProcessor.addState :43-62
  void logicalAddState(Pre* p, const StEv& se) {
    PreState& st = S(p);
    if (p->isStartState || p->stateType == SEQUENCE) {
      if (st.newAndEvery.empty()) st.newAndEvery.push_back(se);
      if (p->partner && S(p->partner).newAndEvery.empty()) S(p->partner).newAndEvery.push_back(se);
    } else {
      st.newAndEvery.push_back(se);
      if (p->partner) S(p->partner).newAndEvery.push_back(se);
    }
  }

  void addEveryState(Pre* p, const StEv& se) {
    PreState& st = S(p);
    switch (p->kind) {
      case K_STREAM:
      case K_COUNT: {  // StreamPreStateProcessor.addEveryState :230-247, CountPre :141-158
        StEv c = copyStateEvent(se);
        c->type = CURRENT;
        for (int i = p->stateId; i < nstates; i++) c->slots[i] = nullptr;
        st.newAndEvery.push_back(c);
        break;
      }
      case K_LOGICAL: {  // LogicalPreStateProcessor.addEveryState :65-84
        StEv c = copyStateEvent(se);
        c->type = CURRENT;
        c->slots[p->stateId] = nullptr;
        for (int i = p->stateId; i < nstates; i++) c->slots[i] = nullptr;
        st.newAndEvery.push_back(c);
        if (p->partner) {
          c->slots[p->partner->stateId] = nullptr;
          S(p->partner).newAndEvery.push_back(c);
        }
        break;
      }
      case K_ABSENT_STREAM: {  // AbsentStreamPreStateProcessor.addEveryState :106-123
        StEv c = copyStateEvent(se);
        c->type = CURRENT;
        for (int i = p->stateId; i < nstates; i++) c->slots[i] = nullptr;
        st.newAndEvery.push_back(c);
        st.lastScheduledTime = se->ts + p->waitingTime;
        notifyAt(p->scheduler, st.lastScheduledTime);
        break;
      }
      case K_ABSENT_LOGICAL: {  // AbsentLogicalPreStateProcessor.addEveryState :100-118
        StEv c = copyStateEvent(se);
        c->type = CURRENT;
        if (c->slots[p->stateId]) c->ts = c->slots[p->stateId]->ts;
        c->slots[p->stateId] = nullptr;
        c->slots[p->partner->stateId] = nullptr;
        st.newAndEvery.push_back(c);
        S(p->partner).newAndEvery.push_back(c);
        break;
      }
    }
  }

  static bool pendingEmpty(Engine* E, Pre* q) { return q == nullptr || E->S(q).pending.empty(); }

  void resetState(Pre* p) {
    PreState& st = S(p);
    switch (p->kind) {
      case K_STREAM:
      case K_COUNT:  // StreamPreStateProcessor.resetState :288-305
        st.pending.clear();
        if (p->isStartState && st.newAndEvery.empty()) {
          if (p->stateType == SEQUENCE && p->thisPost->nextEveryPre == nullptr &&
              !pendingEmpty(this, p->thisPost->nextStatePre))
            return;
          init(p);
        }
        break;
      case K_LOGICAL:
      case K_ABSENT_LOGICAL: {  // LogicalPreStateProcessor.resetState :87-110
        PreState& ps = S(p->partner);
        if (p->logicalType == L_OR || st.pending.size() == ps.pending.size()) {
          st.pending.clear();
          ps.pending.clear();
          if (p->isStartState && st.newAndEvery.empty()) {
            if (p->stateType == SEQUENCE && p->thisPost->nextEveryPre == nullptr &&
                !pendingEmpty(this, p->thisPost->nextStatePre))
              return;
            init(p);
          }
        }
        break;
      }
      case K_ABSENT_STREAM:  // AbsentStreamPreStateProcessor.resetState :126-148
        st.pending.clear();
        if (p->isStartState) {
          if (p->stateType == SEQUENCE && p->thisPost->nextEveryPre == nullptr &&
              !pendingEmpty(this, p->thisPost->nextStatePre))
            return;
          init(p);
        }
        break;
    }
  }

  // eventTimeComparator (StreamPreStateProcessor.java:66-80): ts -1 sorts last, stable
  static void sortMove(PreState& st) {
    vector<StEv> v(st.newAndEvery.begin(), st.newAndEvery.end());
    std::stable_sort(v.begin(), v.end(), [](const StEv& a, const StEv& b) {
      if (a->ts == -1) return false;
      if (b->ts == -1) return true;
      return a->ts < b->ts;
    });
    for (auto& x : v) st.pending.push_back(x);
    st.newAndEvery.clear();
  }

  void updateState(Pre* p) {
    PreState& st = S(p);
    switch (p->kind) {
      case K_STREAM:
      case K_ABSENT_STREAM:  // StreamPreStateProcessor.updateState :308-323
        sortMove(st);
        break;
      case K_COUNT:  // CountPreStateProcessor.updateState :182-193
        if (st.startStateReset) {
          st.startStateReset = false;
          init(p);
        }
        sortMove(S(p));
        break;
      case K_LOGICAL:
      case K_ABSENT_LOGICAL:  // LogicalPreStateProcessor.updateState :113-125
        sortMove(st);
        sortMove(S(p->partner));
        break;
    }
  }

  // StreamPreStateProcessor.isExpired :118-129
  bool isExpired(Pre* p, const StEv& se, int64_t now) {
    if (p->withinTime != -1) {
      for (int sid : p->startStateIds) {
        SEv ev = se->slots[sid];
        if (ev && std::llabs(ev->ts - now) > p->withinTime) return true;
      }
    }
    return false;
  }

  // StreamPreStateProcessor.expireEvents :326-361
  void expireEvents(Pre* p, int64_t ts) {
    PreState& st = S(p);
    StEv expired;
    for (auto it = st.pending.begin(); it != st.pending.end();) {
      StEv se = *it;
      if (isExpired(p, se, ts)) {
        it = st.pending.erase(it);
        if (se->type != EXPIRED) {
          se->type = EXPIRED;
          expired = se;
        }
      } else {
        break;
      }
    }
    for (auto it = st.newAndEvery.begin(); it != st.newAndEvery.end();) {
      StEv se = *it;
      if (isExpired(p, se, ts)) {
        it = st.newAndEvery.erase(it);
        if (se->type != EXPIRED) {
          se->type = EXPIRED;
          expired = se;
        }
      } else {
        ++it;
      }
    }
    if (expired && p->withinEveryPre) {
      addEveryState(p->withinEveryPre, expired);
      updateState(p->withinEveryPre);
    }
  }

  // StreamPreStateProcessor.process(StateEvent) :131-142 + FilterProcessor.process
  void process(Pre* p, const StEv& se) {
    S(p).stateChanged = false;
    if (p->filter) {
      Val v = eval(p->filter, *se);
      if (!(v.t == T_BOOL && v.b)) return;
    }
    postProcess(p->thisPost, se);
  }

  vector<StEv> processAndReturn(Pre* p, int64_t seq) {
    vector<StEv> ret;
    PreState& st = S(p);
    switch (p->kind) {
      case K_STREAM:
        return streamProcessAndReturn(p, seq, true);
      case K_ABSENT_STREAM: {  // AbsentStreamPreStateProcessor.processAndReturn :257-274
        if (!st.active) return ret;
        streamProcessAndReturn(p, seq, false);
        return ret;  // always an empty chunk
      }
      case K_COUNT: {  // CountPreStateProcessor.processAndReturn :53-95
        for (auto it = st.pending.begin(); it != st.pending.end();) {
          StEv se = *it;
          if ((nstates > p->stateId + 1 && se->slots[p->stateId + 1]) ||
              (nstates > p->stateId + 2 && se->slots[p->stateId + 2])) {
            it = st.pending.erase(it);
            continue;
          }
          add_event(*se, p->stateId, cloneStreamEvent(seq));
          st.successCondition = false;
          process(p, se);
          if (p->thisLast->isEventReturned) {
            p->thisLast->isEventReturned = false;
            ret.push_back(se);
          }
          bool removed = false;
          if (st.stateChanged) {
            it = st.pending.erase(it);
            removed = true;
          }
          if (!st.successCondition) {
            remove_last_event(*se, p->stateId);
            if (p->stateType == SEQUENCE && !removed) {
              it = st.pending.erase(it);
              removed = true;
            }
          }
          if (!removed) ++it;
        }
        return ret;
      }
      case K_LOGICAL: {  // LogicalPreStateProcessor.processAndReturn :128-167
        for (auto it = st.pending.begin(); it != st.pending.end();) {
          StEv se = *it;
          if (p->logicalType == L_OR && se->slots[p->partner->stateId]) {
            it = st.pending.erase(it);
            continue;
          }
          se->slots[p->stateId] = cloneStreamEvent(seq);
          process(p, se);
          if (p->thisLast->isEventReturned) {
            p->thisLast->isEventReturned = false;
            ret.push_back(se);
          }
          if (st.stateChanged) {
            it = st.pending.erase(it);
          } else {
            se->slots[p->stateId] = nullptr;
            if (p->stateType == SEQUENCE) it = st.pending.erase(it);
            else ++it;
          }
        }
        return ret;
      }
      case K_ABSENT_LOGICAL: {  // AbsentLogicalPreStateProcessor.processAndReturn :262-319
        if (!st.active) return ret;
        for (auto it = st.pending.begin(); it != st.pending.end();) {
          StEv se = *it;
          if (p->logicalType == L_OR && se->slots[p->partner->stateId]) {
            it = st.pending.erase(it);
            continue;
          }
          SEv curEv = se->slots[p->stateId];
          se->slots[p->stateId] = cloneStreamEvent(seq);
          process(p, se);
          if (p->waitingTime != -1 ||
              (p->stateType == SEQUENCE && p->logicalType == L_AND && p->thisPost->nextEveryPre != nullptr))
            se->slots[p->stateId] = curEv;
          bool removed = false;
          if (p->thisLast->isEventReturned) {
            p->thisLast->isEventReturned = false;
            it = st.pending.erase(it);
            removed = true;
            if (p->stateType == SEQUENCE) {
              auto& pl = S(p->partner).pending;
              for (auto jt = pl.begin(); jt != pl.end(); ++jt)
                if (jt->get() == se.get()) { pl.erase(jt); break; }
            }
          }
          if (!st.stateChanged) {
            se->slots[p->stateId] = curEv;
            if (p->stateType == SEQUENCE && !removed) {
              it = st.pending.erase(it);
              removed = true;
            }
          }
          if (!removed) ++it;
        }
        return ret;
      }
    }
    return ret;
  }

  // StreamPreStateProcessor.processAndReturn :364-403 (removeOnNoStateChange: Stream=SEQUENCE, Absent=false)
  vector<StEv> streamProcessAndReturn(Pre* p, int64_t seq, bool removeOnNoChange) {
    vector<StEv> ret;
    PreState& st = S(p);
    for (auto it = st.pending.begin(); it != st.pending.end();) {
      StEv se = *it;
      se->slots[p->stateId] = cloneStreamEvent(seq);
      process(p, se);
      if (p->thisLast->isEventReturned) {
        p->thisLast->isEventReturned = false;
        ret.push_back(se);
      }
      if (st.stateChanged) {
        it = st.pending.erase(it);
      } else {
        se->slots[p->stateId] = nullptr;
        if (p->stateType == SEQUENCE) {
          bool rm = removeOnNoChange;
          if (p->thisPost->callbackPre) countStartStateReset(p->thisPost->callbackPre);
          if (rm) { it = st.pending.erase(it); continue; }
        }
        ++it;
      }
    }
    return ret;
  }

  // CountPreStateProcessor.startStateReset :168-179 (the self-recursion branch is not followed)
  void countStartStateReset(Pre* p) { S(p).startStateReset = true; }

  // AbsentStreamPostStateProcessor / AbsentLogical: updateLastArrivalTime
  void updateLastArrivalTime(Pre* p, int64_t ts) {
    PreState& st = S(p);
    if (p->kind == K_ABSENT_STREAM) {  // AbsentStreamPreStateProcessor :68-78
      st.lastScheduledTime = ts + p->waitingTime;
      notifyAt(p->scheduler, st.lastScheduledTime);
    } else {  // AbsentLogicalPreStateProcessor :66-75
      st.lastArrivalTime = ts;
    }
  }

  // =====================================================================
  // PostStateProcessor family
  // =====================================================================
  void postProcess(Post* q, const StEv& se) {
    switch (q->kind) {
      case K_STREAM:
        streamPost(q, se);
        break;
      case K_COUNT: {  // CountPostStateProcessor.process :39-65
        SEv ev = se->slots[q->stateId];
        int n = 1;
        while (ev->next) { n++; ev = ev->next; }
        S(q->thisPre).successCondition = true;
        se->ts = ev->ts;
        if (n >= q->minCount) {
          if (q->thisPre->stateType == SEQUENCE) {
            if (q->nextStatePre) addState(q->nextStatePre, se);
            if (n != q->maxCount) addState(q->thisPre, se);
          } else if (n == q->minCount) {
            processMinCountReached(q, se);
          }
          if (n == q->maxCount) S(q->thisPre).stateChanged = true;
        }
        break;
      }
      case K_LOGICAL: {  // LogicalPostStateProcessor.process :59-87
        if (q->logicalType == L_AND) {
          bool proc = false;
          if (q->partnerPre->kind == K_ABSENT_LOGICAL) proc = partnerCanProceed(q->partnerPre, se);
          else if (se->slots[q->partnerPre->stateId]) proc = true;
          if (proc) streamPost(q, se);
          else S(q->thisPre).stateChanged = true;
        } else {
          streamPost(q, se);
          if (q->partnerPost->hasNext && q->thisPre->thisLast == q->partnerPost)
            q->partnerPost->isEventReturned = true;
        }
        break;
      }
      case K_ABSENT_STREAM: {  // AbsentStreamPostStateProcessor.process :36-56
        S(q->thisPre).stateChanged = true;
        SEv ev = se->slots[q->stateId];
        se->ts = ev->ts;
        q->isEventReturned = true;
        if (q->thisPre->isStartState && q->nextEveryPre && q->nextEveryPre == q->thisPre)
          addEveryState(q->nextEveryPre, se);
        updateLastArrivalTime(q->thisPre, ev->ts);
        break;
      }
      case K_ABSENT_LOGICAL: {  // AbsentLogicalPostStateProcessor.process :37-49
        S(q->thisPre).stateChanged = true;
        SEv ev = se->slots[q->stateId];
        q->isEventReturned = true;
        updateLastArrivalTime(q->thisPre, ev->ts);
        break;
      }
    }
  }

  // StreamPostStateProcessor.process :64-83
  void streamPost(Post* q, const StEv& se) {
    S(q->thisPre).stateChanged = true;
    SEv ev = se->slots[q->stateId];
    se->ts = ev->ts;
    if (q->hasNext) q->isEventReturned = true;
    if (q->nextStatePre) addState(q->nextStatePre, se);
    if (q->nextEveryPre) addEveryState(q->nextEveryPre, se);
    if (q->callbackPre) countStartStateReset(q->callbackPre);
  }

  // CountPostStateProcessor.processMinCountReached :67-79
  void processMinCountReached(Post* q, const StEv& se) {
    if (q->hasNext) {
      S(q->thisPre).stateChanged = true;
      q->isEventReturned = true;
    }
    if (q->nextStatePre) addState(q->nextStatePre, se);
    if (q->nextEveryPre) addEveryState(q->nextEveryPre, se);
  }

  // AbsentLogicalPreStateProcessor.partnerCanProceed :353-388
  bool partnerCanProceed(Pre* p, const StEv& se) {
    PreState& st = S(p);
    if (p->stateType == SEQUENCE && p->thisPost->nextEveryPre == nullptr && st.lastArrivalTime > 0) return false;
    if (p->waitingTime == -1) {
      if (p->thisPost->nextEveryPre == nullptr) return se->slots[p->stateId] == nullptr;
      if (st.lastArrivalTime > 0) {
        st.lastArrivalTime = 0;
        init(p);
        return false;
      }
      return true;
    }
    return se->slots[p->stateId] != nullptr;
  }

  // =====================================================================
  // timers
  // =====================================================================
  // AbsentStreamPreStateProcessor.process(ComplexEventChunk) :151-227
  void absentStreamTimer(Pre* p, int64_t currentTime) {
    PreState& st = S(p);
    if (!st.active) return;
    vector<StEv> ret;
    bool initialize = p->isStartState && st.newAndEvery.empty() && st.pending.empty();
    if (initialize && p->stateType == SEQUENCE && p->thisPost->nextEveryPre == nullptr && st.lastScheduledTime > 0)
      initialize = false;
    if (initialize) {
      addState(p, newStateEvent());
    } else if (p->stateType == SEQUENCE && !st.newAndEvery.empty()) {
      resetState(p);
    }
    updateState(p);
    for (auto it = st.pending.begin(); it != st.pending.end();) {
      StEv ev = *it;
      if (isExpired(p, ev, currentTime)) {
        it = st.pending.erase(it);
        if (p->withinEveryPre && p->thisPost->nextEveryPre != p) {
          if (p->thisPost->nextEveryPre) addEveryState(p->thisPost->nextEveryPre, ev);
        }
        continue;
      }
      if ((ev->ts == -1 && currentTime >= st.lastScheduledTime) ||
          (ev->ts != -1 && currentTime >= ev->ts + p->waitingTime)) {
        it = st.pending.erase(it);
        ev->ts = currentTime;
        ret.push_back(ev);
        continue;
      }
      ++it;
    }
    if (p->withinEveryPre) updateState(p->withinEveryPre);
    bool notProcessed = ret.empty();
    for (auto& ev : ret) absentStreamSend(p, ev);
    int64_t actual = clock;
    if (actual > p->waitingTime + currentTime) st.lastScheduledTime = actual + p->waitingTime;
    if (notProcessed && st.lastScheduledTime < currentTime) {
      st.lastScheduledTime = currentTime + p->waitingTime;
      notifyAt(p->scheduler, st.lastScheduledTime);
    }
  }

  // AbsentStreamPreStateProcessor.sendEvent :238-254
  void absentStreamSend(Pre* p, const StEv& se) {
    Post* q = p->thisPost;
    if (q->hasNext) emit(se);
    if (q->nextStatePre) addState(q->nextStatePre, se);
    if (q->nextEveryPre) addEveryState(q->nextEveryPre, se);
    else if (p->isStartState) S(p).active = false;
    if (q->callbackPre) countStartStateReset(q->callbackPre);
  }

  // AbsentLogicalPreStateProcessor.process(ComplexEventChunk) :121-209
  void absentLogicalTimer(Pre* p, int64_t currentTime) {
    PreState& st = S(p);
    if (!st.active) return;
    bool notProcessed = true;
    vector<StEv> ret;
    if (currentTime >= st.lastArrivalTime + p->waitingTime) {
      if (p->isStartState && p->stateType == SEQUENCE && st.newAndEvery.empty() && st.pending.empty()) {
        addState(p, newStateEvent());
      } else if (p->stateType == SEQUENCE && !st.newAndEvery.empty()) {
        resetState(p);
      }
      updateState(p);
      StEv expired;
      for (auto it = st.pending.begin(); it != st.pending.end();) {
        StEv se = *it;
        if (isExpired(p, se, currentTime)) {
          expired = se;
          it = st.pending.erase(it);
          continue;
        }
        SEv mine = se->slots[p->stateId];
        bool passed = mine == nullptr ? currentTime >= se->ts + p->waitingTime
                                      : currentTime >= mine->ts + p->waitingTime;
        if (passed) {
          it = st.pending.erase(it);
          bool partnerFilled = se->slots[p->partner->stateId] != nullptr;
          if (p->logicalType == L_OR && !partnerFilled) {
            add_event(*se, p->stateId, emptyStreamEvent());
            ret.push_back(se);
          } else if (p->logicalType == L_AND && partnerFilled) {
            ret.push_back(se);
          } else if (p->logicalType == L_AND && !partnerFilled) {
            add_event(*se, p->stateId, emptyStreamEvent());
          }
          continue;
        }
        ++it;
      }
      if (expired && p->withinEveryPre) {
        addEveryState(p->withinEveryPre, expired);
        updateState(p->withinEveryPre);
      }
      notProcessed = ret.empty();
      for (auto& se : ret) {
        se->ts = currentTime;
        absentLogicalSend(p, se);
      }
      st.lastArrivalTime = 0;
    }
    if (p->thisPost->nextEveryPre != nullptr || (notProcessed && p->isStartState)) {
      int64_t nextBreak = st.lastArrivalTime == 0 ? clock + p->waitingTime : st.lastArrivalTime + p->waitingTime;
      notifyAt(p->scheduler, nextBreak);
    }
  }

  // AbsentLogicalPreStateProcessor.sendEvent :230-250
  void absentLogicalSend(Pre* p, const StEv& se) {
    Post* q = p->thisPost;
    if (q->hasNext) emit(se);
    if (q->nextStatePre) addState(q->nextStatePre, se);
    if (q->nextEveryPre) {
      addEveryState(q->nextEveryPre, se);
    } else if (p->isStartState) {
      S(p).active = false;
      if (p->logicalType == L_OR && p->partner->kind == K_ABSENT_LOGICAL) S(p->partner).active = false;
    }
    if (q->callbackPre) countStartStateReset(q->callbackPre);
  }

  // partitionCreated (AbsentStream :291-308, AbsentLogical :332-351)
  void partitionCreated(Pre* p) {
    PreState& st = S(p);
    if (!st.started) {
      st.started = true;
      if (p->isStartState && p->waitingTime != -1 && st.active) {
        if (p->kind == K_ABSENT_STREAM) {
          st.lastScheduledTime = clock + p->waitingTime;
          notifyAt(p->scheduler, st.lastScheduledTime);
        } else {
          notifyAt(p->scheduler, clock + p->waitingTime);
        }
      }
    }
  }

  // Scheduler.sendTimerEvents :171-209 for one (scheduler, key)
  void sendTimerEvents(int s, KeyCtx* k) {
    cur = k;
    auto& q = k->sched[s].queue;
    while (!q.empty() && q.front() - clock <= 0) {
      int64_t t = q.front();
      q.pop_front();
      Pre* p = schedulers[s];
      if (p->kind == K_ABSENT_STREAM) absentStreamTimer(p, t);
      else absentLogicalTimer(p, t);
    }
  }

  // Scheduler TimeChangeListener.onTimeChange :71-103 — one listener per scheduler,
  // registration order; TreeMultimap<Long, SchedulerState> with compareTo()==0
  // keeps ONE state per distinct due time (cross-key ties are deferred).
  void onTimeChange() {
    for (size_t s = 0; s < schedulers.size(); s++) {
      std::map<int64_t, KeyCtx*> sorted;
      for (auto& kp : keys) {
        auto& q = kp->sched[s].queue;
        if (!q.empty() && q.front() <= clock) {
          if (sorted.count(q.front())) timer_ties++;
          else sorted[q.front()] = kp.get();
        }
      }
      for (auto& e : sorted) sendTimerEvents((int)s, e.second);
    }
  }

  // non-playback: the live Scheduler's EventCaller fires each due head at its own time
  void liveTimersUpTo(int64_t now) {
    for (;;) {
      int64_t best = INT64_MAX;
      int bs = -1;
      KeyCtx* bk = nullptr;
      for (size_t s = 0; s < schedulers.size(); s++)
        for (auto& kp : keys) {
          auto& q = kp->sched[s].queue;
          if (!q.empty() && q.front() <= now && q.front() < best) {
            best = q.front();
            bs = (int)s;
            bk = kp.get();
          }
        }
      if (bs < 0) return;
      if (best > clock) clock = best;
      sendTimerEvents(bs, bk);
    }
  }

  // ------------------------------------------------------- runtime tree ops
  void treeInit(Node* n) {
    switch (n->t) {
      case Node::STREAM:
      case Node::COUNT: init(n->leafPre); break;
      case Node::NEXT: treeInit(n->a.get()); treeInit(n->b.get()); break;
      case Node::EVERY: treeInit(n->a.get()); break;
      case Node::LOGICAL: treeInit(n->b.get()); treeInit(n->a.get()); break;
    }
  }
  void treeReset(Node* n) {
    switch (n->t) {
      case Node::NEXT: treeReset(n->b.get()); treeReset(n->a.get()); break;
      case Node::LOGICAL: treeReset(n->b.get()); break;
      default: resetState(n->first); break;  // Stream/Count/Every: firstProcessor.resetState()
    }
  }
  void treeUpdate(Node* n) {
    switch (n->t) {
      case Node::NEXT: treeUpdate(n->a.get()); treeUpdate(n->b.get()); break;
      case Node::LOGICAL: treeUpdate(n->b.get()); break;
      default: updateState(n->first); break;
    }
  }

  KeyCtx* keyCtx(int32_t key, bool* created) {
    auto it = keyIndex.find(key);
    *created = false;
    if (it != keyIndex.end()) return keys[it->second].get();
    auto k = std::make_unique<KeyCtx>();
    k->key = key;
    k->pre.resize(pres.size());
    k->sched.resize(schedulers.size());
    keyIndex[key] = keys.size();
    keys.push_back(std::move(k));
    *created = true;
    return keys.back().get();
  }

  // StateStreamRuntime.initPartition :90-97
  void initPartition(KeyCtx* k) {
    cur = k;
    treeInit(root.get());
    for (Pre* p : startup) partitionCreated(p);
  }

  void emitReturned(const vector<StEv>& ret, bool selectorAttached) {
    for (auto& se : ret) {
      if (selectorAttached) emit(se);
      else dropped_returns++;
    }
  }

  // one InputHandler.send(ts, data) on stream `stream` for partition key `key`
  void sendEvent(int64_t seq) {
    int64_t ts = ev_clk[seq];  // the clock this send sets (= the event's ts unless given)
    emit_pos = seq;
    if (playback) {
      if (ts >= clock) {  // TimestampGeneratorImpl.setCurrentTimestamp :105-121
        clock = ts;
        onTimeChange();
      }
    } else {
      liveTimersUpTo(ts);
      if (ts > clock) clock = ts;
    }
    int stream = ev_stream[seq];
    // a clock-only event (stream -1: a send on a stream this query does not read) sets the
    // playback clock above and reaches no receiver, so no partition is created for it
    if (stream < 0 || stream >= (int)receivers.size()) return;
    KeyCtx* k;
    if (partitioned) {
      bool created;
      k = keyCtx(ev_key[seq], &created);
      if (created) initPartition(k);
    } else {
      k = keys[0].get();
    }
    cur = k;
    Receiver& r = receivers[stream];
    if (r.forStream.empty()) return;
    // stabilizeStates (state/receiver/*.java)
    for (Pre* p : preStateProcessors) expireEvents(p, ts);
    if (type == SEQUENCE) {
      treeReset(root.get());
      treeUpdate(root.get());
    } else if (r.multi) {
      for (Pre* p : r.forStream) updateState(p);
    } else {
      updateState(r.forStream[0]);
    }
    if (r.multi) {
      // PatternMultiProcessStreamReceiver / SequenceMulti: eventSequence reversed;
      // StateMultiProcessStreamReceiver forwards to the selector of the LAST registered processor
      bool sel = r.forStream.back()->thisPost->hasNext;
      for (int i = (int)r.forStream.size() - 1; i >= 0; i--) {
        vector<StEv> ret = processAndReturn(r.forStream[i], seq);
        emitReturned(ret, sel);
      }
    } else {
      Pre* p = r.forStream[0];
      vector<StEv> ret = processAndReturn(p, seq);
      emitReturned(ret, p->thisLast->hasNext);
    }
  }

  vector<int32_t> ev_key;
  vector<int32_t> ev_stream;

  // ------------------------------------------------------------- building
  std::unique_ptr<Expr> buildExpr(const ojson::Value& v) {
    auto e = std::make_unique<Expr>();
    e->op = v["op"].str;
    if (e->op == "const") {
      VT t = type_of(v["type"].str);
      e->cval.t = t;
      const ojson::Value& cv = v["v"];
      switch (t) {
        case T_INT: e->cval.i = (int32_t)cv.as_int(); break;
        case T_STR: e->cval.i = (int32_t)cv.as_int(); break;
        case T_LONG: e->cval.l = cv.as_int(); break;
        case T_FLOAT: e->cval.f = (float)cv.as_num(); break;
        case T_DOUBLE: e->cval.d = cv.as_num(); break;
        case T_BOOL: e->cval.b = cv.as_int() != 0; break;
        default: e->cval.t = T_NULL; break;
      }
    } else if (e->op == "var") {
      e->state = (int)v["state"].as_int();
      e->col = (int)v["col"].as_int();
      e->index = (int)v["index"].as_int();
      e->type = type_of(v["type"].str);
    } else if (e->op == "isnullstate") {
      e->state = (int)v["state"].as_int();
      e->index = (int)v["index"].as_int();
    } else if (e->op == "cmp") {
      static const char* names[] = {"gt", "ge", "lt", "le", "eq", "ne"};
      for (int i = 0; i < 6; i++)
        if (v["cmp"].str == names[i]) e->cmp = i;
      e->args.push_back(buildExpr(v["a"]));
      e->args.push_back(buildExpr(v["b"]));
    } else if (e->op == "not" || e->op == "isnull") {
      e->args.push_back(buildExpr(v["a"]));
    } else if (e->op == "ifthenelse" || e->op == "coalesce") {
      e->type = type_of(v["type"].str);
      const ojson::Value& a = v["args"];
      for (size_t i = 0; i < a.arr.size(); i++) e->args.push_back(buildExpr(a.arr[i]));
    } else if (e->op == "instanceof") {
      e->type = type_of(v["tag"].str);
      e->args.push_back(buildExpr(v["a"]));
    } else {
      e->type = type_of(v["type"].str);
      e->args.push_back(buildExpr(v["a"]));
      e->args.push_back(buildExpr(v["b"]));
    }
    return e;
  }

  Pre* newPre(Kind k) {
    pres.push_back(std::make_unique<Pre>());
    Pre* p = pres.back().get();
    p->id = (int)pres.size() - 1;
    p->kind = k;
    p->stateType = type;
    return p;
  }
  Post* newPost(Kind k) {
    posts.push_back(std::make_unique<Post>());
    Post* q = posts.back().get();
    q->id = (int)posts.size() - 1;
    q->kind = k;
    return q;
  }
  int newScheduler(Pre* p) {
    schedulers.push_back(p);
    return (int)schedulers.size() - 1;
  }

  const ojson::Value* statesJson = nullptr;

  // LogicalPostStateProcessor.setNextStatePreProcessor / CountPost.setNextStatePreProcessor
  void setNextStatePre(Post* q, Pre* p) {
    q->nextStatePre = p;
    if (q->kind == K_LOGICAL || q->kind == K_ABSENT_LOGICAL) {
      q->partnerPost->nextStatePre = p;
    } else if (q->kind == K_COUNT) {
      if (q->thisPre->isStartState && q->thisPre->stateType == SEQUENCE && q->minCount == 0)
        p->thisPost->callbackPre = q->thisPre;
    }
  }
  void setNextEveryPre(Post* q, Pre* p) {
    q->nextEveryPre = p;
    if (q->kind == K_LOGICAL || q->kind == K_ABSENT_LOGICAL) q->partnerPost->nextEveryPre = p;
  }

  // StateInputStreamParser.parse :148-408
  std::unique_ptr<Node> parse(const ojson::Value& t, Pre* pre, Post* post, bool isStart, vector<Pre*>& list) {
    auto n = std::make_unique<Node>();
    const std::string& kind = t["t"].str;
    if (kind == "stream" || kind == "absent") {
      int sid = (int)t["state"].as_int();
      const ojson::Value& sj = (*statesJson)[sid];
      bool absent = kind == "absent";
      if (!pre) {
        if (absent) {
          pre = newPre(K_ABSENT_STREAM);
          pre->waitingTime = sj["waiting"].as_int();
          startup.push_back(pre);
          pre->scheduler = newScheduler(pre);
        } else {
          pre = newPre(K_STREAM);
        }
      }
      pre->stateId = sid;
      pre->stream = (int)sj["stream"].as_int();
      pre->isStartState = isStart;
      if (sj.has("filter")) pre->filter = filters[sid].get();
      if (!post) post = newPost(absent ? K_ABSENT_STREAM : K_STREAM);
      post->stateId = sid;
      post->thisPre = pre;
      pre->thisPost = post;
      pre->thisLast = post;
      list.push_back(pre);
      n->t = Node::STREAM;
      n->first = pre;
      n->last = post;
      n->leafPre = pre;
      return n;
    }
    if (kind == "next") {
      n->t = Node::NEXT;
      n->a = parse(t["a"], pre, post, isStart, list);
      n->b = parse(t["b"], pre, post, false, list);
      setNextStatePre(n->a->last, n->b->first);
      n->first = n->a->first;
      n->last = n->b->last;
      return n;
    }
    if (kind == "every") {
      n->t = Node::EVERY;
      vector<Pre*> inner;
      n->a = parse(t["x"], pre, post, isStart, inner);
      n->first = n->a->first;
      n->last = n->a->last;
      setNextEveryPre(n->last, n->first);
      for (Pre* p : inner) p->withinEveryPre = n->first;
      list.insert(list.end(), inner.begin(), inner.end());
      return n;
    }
    if (kind == "logical") {
      int lt = t["op"].str == "or" ? L_OR : L_AND;
      const ojson::Value& e1 = t["s1"];
      const ojson::Value& e2 = t["s2"];
      auto mk = [&](const ojson::Value& e, Pre*& lp, Post*& lq) {
        bool abs = e["t"].str == "absent";
        if (abs) {
          lp = newPre(K_ABSENT_LOGICAL);
          lp->waitingTime = (*statesJson)[(int)e["state"].as_int()]["waiting"].as_int();
          startup.push_back(lp);
          lp->scheduler = newScheduler(lp);
        } else {
          lp = newPre(K_LOGICAL);
        }
        lp->logicalType = lt;
        lq = newPost(abs ? K_ABSENT_LOGICAL : K_LOGICAL);
        lq->logicalType = lt;
      };
      Pre *p1, *p2;
      Post *q1, *q2;
      mk(e1, p1, q1);
      mk(e2, p2, q2);
      q1->partnerPre = p2;
      q2->partnerPre = p1;
      q1->partnerPost = q2;
      q2->partnerPost = q1;
      p1->partner = p2;
      p2->partner = p1;
      n->t = Node::LOGICAL;
      n->b = parse(e2, p2, q2, isStart, list);
      n->a = parse(e1, p1, q1, isStart, list);
      n->first = n->a->first;
      n->last = n->b->last;
      return n;
    }
    if (kind == "count") {
      Pre* cp = newPre(K_COUNT);
      Post* cq = newPost(K_COUNT);
      cp->minCount = (int)t["min"].as_int();
      int mx = (int)t["max"].as_int();
      cp->maxCount = mx < 0 ? INT32_MAX : mx;
      cq->minCount = cp->minCount;
      cq->maxCount = cp->maxCount;
      cp->countPost = cq;
      ojson::Value leaf;
      leaf.kind = ojson::Value::OBJ;
      leaf.obj["t"].kind = ojson::Value::STR;
      leaf.obj["t"].str = "stream";
      leaf.obj["state"] = t["state"];
      auto inner = parse(leaf, cp, cq, isStart, list);
      inner->t = Node::COUNT;
      return inner;
    }
    throw std::runtime_error("unknown state element " + kind);
  }

  // InnerStateRuntime.setQuerySelector
  void setQuerySelector(Node* n) {
    switch (n->t) {
      case Node::STREAM:
      case Node::COUNT: n->last->hasNext = true; break;
      case Node::NEXT: setQuerySelector(n->b.get()); break;
      case Node::EVERY: setQuerySelector(n->a.get()); break;
      case Node::LOGICAL: setQuerySelector(n->b.get()); setQuerySelector(n->a.get()); break;
    }
  }
  // InnerStateRuntime.setup: register each state's first processor with its receiver
  void setup(Node* n) {
    switch (n->t) {
      case Node::STREAM:
      case Node::COUNT: receivers[n->leafPre->stream].forStream.push_back(n->leafPre); break;
      case Node::NEXT: setup(n->a.get()); setup(n->b.get()); break;
      case Node::EVERY: setup(n->a.get()); break;
      case Node::LOGICAL: setup(n->b.get()); setup(n->a.get()); break;
    }
  }

  void build(const std::string& json, int64_t start_clock) {
    ojson::Value prog = ojson::parse(json);
    type = prog["type"].str == "sequence" ? SEQUENCE : PATTERN;
    within = prog["within"].as_int();
    playback = prog["playback"].truthy();
    partitioned = prog["partitioned"].truthy();
    const ojson::Value& states = prog["states"];
    statesJson = &states;
    nstates = (int)states.arr.size();
    filters.resize(nstates);
    for (int i = 0; i < nstates; i++)
      if (states[i].has("filter")) filters[i] = buildExpr(states[i]["filter"]);
    size_t nstreams = prog["streams"].arr.size();
    receivers.resize(nstreams);
    streamStateCount.assign(nstreams, 0);
    for (int i = 0; i < nstates; i++) streamStateCount[states[i]["stream"].as_int()]++;
    for (auto& c : prog["columns"].arr) {
      Column col;
      col.type = type_of(c["type"].str);
      col.stream = (int)c["stream"].as_int();
      cols.push_back(std::move(col));
    }
    root = parse(prog["tree"], nullptr, nullptr, true, preStateProcessors);
    if (within != -1) {
      vector<int> ids;
      for (Pre* p : preStateProcessors)
        if (p->isStartState) ids.push_back(p->stateId);
      for (Pre* p : preStateProcessors) {
        p->startStateIds = ids;
        p->withinTime = within;
      }
    }
    root->first->thisLast = root->last;
    setQuerySelector(root.get());
    setup(root.get());
    for (size_t s = 0; s < nstreams; s++) receivers[s].multi = streamStateCount[s] > 1;
    clock = start_clock;
    if (!partitioned) {
      bool created;
      KeyCtx* k = keyCtx(0, &created);
      initPartition(k);  // QueryRuntimeImpl.start -> initPartition at app start
    }
  }

  void push(int64_t n, const int64_t* ts, const int32_t* key, const int32_t* stream,
            const void* const* colp, const uint8_t* const* nulls, const int64_t* clk = nullptr,
            const int64_t* gseq = nullptr) {
    int64_t base = nevents;
    ev_ts.insert(ev_ts.end(), ts, ts + n);
    ev_clk.insert(ev_clk.end(), clk ? clk : ts, (clk ? clk : ts) + n);
    for (int64_t i = 0; i < n; i++) ev_gseq.push_back(gseq ? gseq[i] : base + i);
    ev_key.insert(ev_key.end(), key, key + n);
    ev_stream.insert(ev_stream.end(), stream, stream + n);
    for (size_t c = 0; c < cols.size(); c++) {
      Column& col = cols[c];
      switch (col.type) {
        case T_LONG: {
          const int64_t* p = (const int64_t*)colp[c];
          col.i64.insert(col.i64.end(), p, p + n);
          break;
        }
        case T_FLOAT: {
          const float* p = (const float*)colp[c];
          col.f32.insert(col.f32.end(), p, p + n);
          break;
        }
        case T_DOUBLE: {
          const double* p = (const double*)colp[c];
          col.f64.insert(col.f64.end(), p, p + n);
          break;
        }
        case T_BOOL: {
          const uint8_t* p = (const uint8_t*)colp[c];
          for (int64_t i = 0; i < n; i++) col.i32.push_back(p[i]);
          break;
        }
        default: {
          const int32_t* p = (const int32_t*)colp[c];
          col.i32.insert(col.i32.end(), p, p + n);
          break;
        }
      }
      if (nulls && nulls[c]) {
        if (col.nul.empty()) col.nul.assign(base, 0);
        col.nul.insert(col.nul.end(), nulls[c], nulls[c] + n);
      } else if (!col.nul.empty()) {
        col.nul.insert(col.nul.end(), n, 0);
      }
    }
    nevents += n;
    for (int64_t i = 0; i < n; i++) sendEvent(base + i);
  }

  void advance(int64_t now) {
    emit_pos = nevents;
    if (playback) {
      if (now >= clock) {
        clock = now;
        onTimeChange();
      }
    } else {
      liveTimersUpTo(now);
      if (now > clock) clock = now;
    }
  }
};

}  // namespace oracle

// ============================================================================
// C API (ctypes), test infrastructure only
// ============================================================================
using oracle::Engine;

struct OracleHandle {
  Engine e;
  std::string err;
};

extern "C" {

void* oracle_create(const char* program_json, int64_t start_clock, char* err, int errlen) {
  auto* h = new OracleHandle();
  try {
    h->e.build(program_json, start_clock);
  } catch (std::exception& ex) {
    if (err && errlen > 0) {
      strncpy(err, ex.what(), errlen - 1);
      err[errlen - 1] = 0;
    }
    delete h;
    return nullptr;
  }
  return h;
}

int oracle_push(void* hp, int64_t n, const int64_t* ts, const int32_t* key, const int32_t* stream,
                const void* const* cols, const uint8_t* const* nulls) {
  auto* h = (OracleHandle*)hp;
  h->e.push(n, ts, key, stream, cols, nulls);
  return 0;
}

// the same with the optional columns of shp_batch: clock (setCurrentTimestamp value per event)
// and seq (sequence numbers the match records use); either may be NULL
int oracle_push2(void* hp, int64_t n, const int64_t* ts, const int32_t* key, const int32_t* stream,
                 const void* const* cols, const uint8_t* const* nulls, const int64_t* clock, const int64_t* seq) {
  auto* h = (OracleHandle*)hp;
  h->e.push(n, ts, key, stream, cols, nulls, clock, seq);
  return 0;
}

int oracle_advance(void* hp, int64_t now) {
  ((OracleHandle*)hp)->e.advance(now);
  return 0;
}

int oracle_num_states(void* hp) { return ((OracleHandle*)hp)->e.nstates; }
int64_t oracle_num_matches(void* hp) { return (int64_t)((OracleHandle*)hp)->e.out.size(); }
int64_t oracle_num_refs(void* hp) {
  int64_t r = 0;
  for (auto& m : ((OracleHandle*)hp)->e.out)
    for (auto& s : m.slots) r += (int64_t)s.size();
  return r;
}
int64_t oracle_timer_ties(void* hp) { return ((OracleHandle*)hp)->e.timer_ties; }
int64_t oracle_dropped_returns(void* hp) { return ((OracleHandle*)hp)->e.dropped_returns; }

// Fetch and clear accumulated matches. slot_len: m*S, refs: concatenated event seqs.
int oracle_fetch(void* hp, int32_t* key, int64_t* ts, int8_t* type, int64_t* pos, int32_t* slot_len,
                 int64_t* refs) {
  Engine& e = ((OracleHandle*)hp)->e;
  int64_t r = 0;
  const int64_t ne = (int64_t)e.ev_gseq.size();
  // internal event numbers -> the caller's sequence numbers (an emission after the last event,
  // e.g. from an advance, sits one past the last event's number)
  auto g = [&](int64_t x) -> int64_t {
    if (x < 0) return x;
    if (x < ne) return e.ev_gseq[x];
    return ne > 0 ? e.ev_gseq[ne - 1] + (x - ne + 1) : x;
  };
  for (size_t i = 0; i < e.out.size(); i++) {
    auto& m = e.out[i];
    key[i] = m.key;
    ts[i] = m.ts;
    type[i] = m.type;
    pos[i] = g(m.pos);
    for (int s = 0; s < e.nstates; s++) {
      slot_len[i * e.nstates + s] = (int32_t)m.slots[s].size();
      for (int64_t x : m.slots[s]) refs[r++] = g(x);
    }
  }
  e.out.clear();
  return 0;
}

// The oldest event (caller's sequence number) any open partial still holds: every StateEvent on a
// pending or new-and-every list of every key and processor, each slot's chain followed to its end
// (StreamPreStateProcessor.java:364-403 keeps a partial's StreamEvents alive for as long as it sits
// on a list).  The next sequence number when nothing is open.  The checker of
// shp_engine_oldest_live_seq (tests/test_retention.py).
int64_t oracle_oldest_live_seq(void* hp) {
  Engine& e = ((OracleHandle*)hp)->e;
  const int64_t ne = (int64_t)e.ev_gseq.size();
  int64_t lo = INT64_MAX;
  for (auto& k : e.keys)
    for (auto& ps : k->pre)
      for (const auto* lst : {&ps.pending, &ps.newAndEvery})
        for (auto& se : *lst)
          for (auto& slot : se->slots)
            for (auto ev = slot; ev; ev = ev->next)
              if (ev->seq >= 0 && ev->seq < ne) lo = std::min(lo, e.ev_gseq[ev->seq]);
  if (lo != INT64_MAX) return lo;
  return ne > 0 ? e.ev_gseq[ne - 1] + 1 : 0;
}

// The earliest head of any key's Scheduler queue (Scheduler.java:113-127: a FIFO; the live
// EventCaller is scheduled at the head's due time, :129-155): 1 and *out, or 0 when none is pending.
// The checker of shp_engine_next_due.
int oracle_next_due(void* hp, int64_t* out) {
  Engine& e = ((OracleHandle*)hp)->e;
  int64_t best = INT64_MAX;
  for (auto& k : e.keys)
    for (size_t s = 0; s < e.schedulers.size(); s++)
      if (!k->sched[s].queue.empty()) best = std::min(best, k->sched[s].queue.front());
  if (best == INT64_MAX) return 0;
  *out = best;
  return 1;
}

// Debugging aid (tests only): key `key`'s timer queue of scheduler 0 into out[0..cap), then the
// absent processor's lastScheduledTime; returns the queue length (or -1: no such key)
int64_t oracle_debug_queue(void* hp, int32_t key, int64_t* out, int64_t cap) {
  Engine& e = ((OracleHandle*)hp)->e;
  auto it = e.keyIndex.find(key);
  if (it == e.keyIndex.end() || e.schedulers.empty()) return -1;
  oracle::KeyCtx* k = e.keys[it->second].get();
  int64_t n = 0;
  for (int64_t t : k->sched[0].queue) {
    if (n < cap) out[n] = t;
    n++;
  }
  if (n < cap) out[n] = k->pre[e.schedulers[0]->id].lastScheduledTime;
  return n;
}

void oracle_destroy(void* hp) { delete (OracleHandle*)hp; }
}
