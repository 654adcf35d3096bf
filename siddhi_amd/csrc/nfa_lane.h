// siddhi-hip: the general per-partition-key NFA lane.
//
// One lane owns one partition key. Its partial matches (StateEvents), captured
// events (StreamEvent nodes, chained for count states), per-processor pending /
// new-and-every lists, flags and absent-state timer FIFOs live in HBM in a
// lane-interleaved SoA layout (element i of lane l at field[i * L + l], so a
// wave touching the same element is coalesced).  The lane replays, event by
// event, the processor semantics of io.siddhi.core.query.input.stream.state
// (every routine names the Java method it follows), with fixed-capacity pools
// and index-based lists instead of heap objects; aliasing (shared count chains,
// logical partners sharing one StateEvent) is kept by sharing indices.
// Overflow of any pool sets the lane's error word.  The pools come in capacity tiers
// (LaneCaps<T>): the engine runs every push on a copy of the committed arena, and a push that
// overflows tier T is re-run from the committed state at tier T + 1 (the arena migrated to the
// larger layout), as the reference's lists are unbounded (StreamPreStateProcessor.java:437-438).
#pragma once
#include <math.h>
#include <stdint.h>

#include "prog.h"

namespace shp {

// per-key capacities of tier T (x1, x4, x16, x64, x128: pool, list and queue indices are int16, so
// x128 -- 16384 nodes, 4096 partials per list, 8192 queued timers per key -- is the last tier)
SHP_HD constexpr int lane_scale(int t) { return t == 0 ? 1 : (t == 1 ? 4 : (t == 2 ? 16 : (t == 3 ? 64 : 128))); }
template <int T>
struct LaneCaps {
  static constexpr int SCALE = lane_scale(T);
  static constexpr int NSE = 64 * SCALE;   // StateEvent pool per key
  static constexpr int NN = 128 * SCALE;   // StreamEvent node pool per key
  static constexpr int LCAP = 32 * SCALE;  // capacity of each pending / new-and-every list
  static constexpr int QCAP = 64 * SCALE;  // timer FIFO capacity per scheduler per key
  // the lane collects garbage before an event when fewer are free: one event may allocate a
  // StateEvent / node per partial on the lists it walks, so the reserves scale with the lists
  static constexpr int GC_SE_RESERVE = 24 * SCALE;
  static constexpr int GC_ND_RESERVE = 48 * SCALE;
};
constexpr int LANE_TIERS = 5;

enum LaneErr : int32_t { E_SE = 1, E_ND = 2, E_LIST = 4, E_Q = 8, E_OUT = 16, E_REF = 32, E_AGGNULL = 64 };
enum PFlag : uint8_t { F_CHANGED = 1, F_INIT = 2, F_STARTED = 4, F_SUCCESS = 8, F_SSRESET = 16, F_INACTIVE = 32 };

struct LaneLayout {
  int64_t L;  // lanes (keys) in the arena
  int32_t tier, nse, nn, lcap, qcap, pad_;  // the capacity tier (LaneCaps) the layout is built for
  int64_t o_se_ts, o_se_slot, o_se_type, o_nd_seq, o_nd_ts, o_nd_val, o_nd_next, o_nd_null;
  int64_t o_se_used, o_nd_used, o_lst_len, o_lst, o_pflags, o_lsched, o_larr, o_ret, o_q, o_qhead, o_qlen;
  int64_t o_kinit, o_err, o_agg, bytes;
  // the field table (offset, elements per lane, element bytes), for copying one lane's state
  // between two layouts (k_nfa_lanes_lds)
  int32_t nf;
  int64_t f_off[24];
  int32_t f_elems[24], f_sz[24];

  void build(int64_t lanes, int t = 0) {
    L = lanes;
    tier = t;
    nse = 64 * lane_scale(t);  // LaneCaps<t>
    nn = 128 * lane_scale(t);
    lcap = 32 * lane_scale(t);
    qcap = 64 * lane_scale(t);
    const int NSE = nse, NN = nn, LCAP = lcap, QCAP = qcap;
    int64_t o = 0;
    nf = 0;
    auto f = [&](int64_t& off, int64_t elems, int64_t sz) {
      off = o;
      f_off[nf] = o;
      f_elems[nf] = (int32_t)elems;
      f_sz[nf++] = (int32_t)sz;
      o += ((elems * L * sz + 255) / 256) * 256;
    };
    f(o_se_ts, NSE, 8);
    f(o_se_slot, NSE * MAXS, 2);
    f(o_se_type, NSE, 1);
    f(o_nd_seq, NN, 8);
    f(o_nd_ts, NN, 8);
    f(o_nd_val, NN * NV, 8);
    f(o_nd_next, NN, 2);
    f(o_nd_null, NN, 1);
    f(o_se_used, NSE / 64, 8);
    f(o_nd_used, NN / 64, 8);
    f(o_lst_len, 2 * MAXP, 2);
    f(o_lst, 2 * MAXP * LCAP, 2);
    f(o_pflags, MAXP, 1);
    f(o_lsched, MAXP, 8);
    f(o_larr, MAXP, 8);
    f(o_ret, 1, 4);
    f(o_q, MAXQ * QCAP, 8);
    f(o_qhead, MAXQ, 2);
    f(o_qlen, MAXQ, 2);
    f(o_kinit, 1, 1);
    f(o_err, 1, 4);
    f(o_agg, 2, 8);  // the key's selector aggregate (SHP_LAYOUT_AGG): value / sum, count
    bytes = o;
  }
};

// One batch, as seen by the lanes.  Events are in arrival (seq) order; the
// lane walks its key's events through perm[kbeg[k] .. kend[k]).
struct BatchView {
  int64_t n;
  int64_t seq0;          // global sequence number of event 0
  int64_t clock0;        // event-time clock before event 0
  int64_t init_clock;    // clock at start() for a non-partitioned query (QueryRuntimeImpl.start)
  int32_t partitioned;
  int32_t pad;
  const int64_t* ts;
  const int32_t* stream;
  const int64_t* rmax;   // clock after event g (running max of tclk, seeded with clock0)
  const void* cols[MAXCOL];
  const uint8_t* nulls[MAXCOL];
  // optional columns (shp_batch.seq / .clock): the events' sequence numbers (NULL: seq0 + g) and
  // the value each event hands TimestampGenerator.setCurrentTimestamp (= ts when the caller gives
  // no clock column; a key-sharded rank gets the global playback clock here)
  const int64_t* seq;
  const int64_t* tclk;
};

// sequence number of batch event g
SHP_HD inline int64_t bseq(const BatchView& B, int64_t g) { return B.seq ? B.seq[g] : B.seq0 + g; }

// Match sink: records are appended with atomics, per-lane order preserved.
struct MatchOut {
  int64_t cap, refcap;
  unsigned long long* count;   // [0]=matches, [1]=refs
  int32_t* key;
  int64_t* ts;
  int8_t* type;
  int64_t* pos;
  int64_t* ref_off;
  int16_t* slot_len;           // cap * MAXS
  int64_t* refs;
  double* agg;                 // SHP_LAYOUT_AGG (sweep): aggregate value per match
};

struct Val {
  int8_t tag;
  int64_t bits;
};

SHP_HD inline float bits_f(int64_t b) {
  union { uint32_t u; float f; } c;
  c.u = (uint32_t)b;
  return c.f;
}
SHP_HD inline int64_t f_bits(float f) {
  union { uint32_t u; float f; } c;
  c.f = f;
  return (int64_t)c.u;
}
SHP_HD inline double bits_d(int64_t b) {
  union { int64_t i; double d; } c;
  c.i = b;
  return c.d;
}
SHP_HD inline int64_t d_bits(double d) {
  union { int64_t i; double d; } c;
  c.d = d;
  return c.i;
}

// Java binary numeric promotion of one operand to `to` (JLS 5.6.2)
SHP_HD inline double asD(const Val& v) {
  switch (v.tag) {
    case T_INT: return (double)(int32_t)v.bits;
    case T_LONG: return (double)v.bits;
    case T_FLOAT: return (double)bits_f(v.bits);
    default: return bits_d(v.bits);
  }
}
SHP_HD inline float asF(const Val& v) {
  switch (v.tag) {
    case T_INT: return (float)(int32_t)v.bits;
    case T_LONG: return (float)v.bits;
    case T_FLOAT: return bits_f(v.bits);
    default: return (float)bits_d(v.bits);
  }
}
SHP_HD inline int64_t asL(const Val& v) { return v.tag == T_INT ? (int64_t)(int32_t)v.bits : v.bits; }

template <class T>
SHP_HD inline bool cmp_op(int c, T a, T b) {
  switch (c) {
    case 0: return a > b;
    case 1: return a >= b;
    case 2: return a < b;
    case 3: return a <= b;
    case 4: return a == b;
    default: return a != b;
  }
}

SHP_HD inline Val java_cmp(const Instr& in, const Val& x, const Val& y) {
  Val r{T_BOOL, 0};
  if (x.tag == T_NULL || y.tag == T_NULL) return r;
  bool b;
  switch (in.b) {
    case T_DOUBLE: b = cmp_op<double>(in.a, asD(x), asD(y)); break;
    case T_FLOAT: b = cmp_op<float>(in.a, asF(x), asF(y)); break;
    case T_LONG: b = cmp_op<int64_t>(in.a, asL(x), asL(y)); break;
    case T_INT: b = cmp_op<int32_t>(in.a, (int32_t)x.bits, (int32_t)y.bits); break;
    default: {  // string ids / bools: equality only
      bool eq = x.bits == y.bits;
      b = in.a == 4 ? eq : !eq;
    }
  }
  r.bits = b;
  return r;
}

// core/executor/math/{add,subtract,multiply,divide,mod}/*: null on /0 for every type
SHP_HD inline Val java_arith(const Instr& in, const Val& x, const Val& y) {
  Val r{T_NULL, 0};
  if (x.tag == T_NULL || y.tag == T_NULL) return r;
  int op = in.a;
  switch (in.b) {
    case T_DOUBLE: {
      double a = asD(x), b = asD(y), o;
      if (op >= 3 && b == 0.0) return r;
      o = op == 0 ? a + b : op == 1 ? a - b : op == 2 ? a * b : op == 3 ? a / b : fmod(a, b);
      r.tag = T_DOUBLE;
      r.bits = d_bits(o);
      return r;
    }
    case T_FLOAT: {
      float a = asF(x), b = asF(y), o;
      if (op >= 3 && b == 0.0f) return r;
      o = op == 0 ? a + b : op == 1 ? a - b : op == 2 ? a * b : op == 3 ? a / b : fmodf(a, b);
      r.tag = T_FLOAT;
      r.bits = f_bits(o);
      return r;
    }
    case T_LONG: {
      int64_t a = asL(x), b = asL(y);
      if (op >= 3 && b == 0) return r;
      uint64_t ua = (uint64_t)a, ub = (uint64_t)b;
      int64_t o;
      if (op == 0) o = (int64_t)(ua + ub);
      else if (op == 1) o = (int64_t)(ua - ub);
      else if (op == 2) o = (int64_t)(ua * ub);
      else if (op == 3) o = (b == -1) ? (int64_t)(0 - ua) : a / b;
      else o = (b == -1) ? 0 : a % b;
      r.tag = T_LONG;
      r.bits = o;
      return r;
    }
    default: {
      int32_t a = (int32_t)asL(x), b = (int32_t)asL(y);
      if (op >= 3 && b == 0) return r;
      uint32_t ua = (uint32_t)a, ub = (uint32_t)b;
      int32_t o;
      if (op == 0) o = (int32_t)(ua + ub);
      else if (op == 1) o = (int32_t)(ua - ub);
      else if (op == 2) o = (int32_t)(ua * ub);
      else if (op == 3) o = (b == -1) ? (int32_t)(0u - ua) : a / b;
      else o = (b == -1) ? 0 : a % b;
      r.tag = T_INT;
      r.bits = o;
      return r;
    }
  }
}

// Predicate VM. `Res` resolves (state, index) to an event handle and reads its values.
template <class Res>
SHP_HD inline bool run_filter(const DevProg& P, int pc, const Res& res) {
  Val st[MAXSTACK];
  int sp = 0;
  for (;;) {
    const Instr& in = P.code[pc];
    switch (in.op) {
      case OP_END:
        return sp > 0 && st[sp - 1].tag == T_BOOL && st[sp - 1].bits != 0;
      case OP_CONST:
        st[sp++] = Val{(int8_t)in.a, in.imm};
        break;
      case OP_VAR:
        st[sp++] = res.value((int)in.a, (int)(int8_t)in.b, (int)in.c);
        break;
      case OP_ISNULLSTATE:
        st[sp++] = Val{T_BOOL, res.isnull_state((int)in.a, (int)(int8_t)in.b) ? 1 : 0};
        break;
      case OP_AND: {
        Val x = st[--sp];
        if (!(x.tag == T_BOOL && x.bits)) {
          st[sp++] = Val{T_BOOL, 0};
          pc = in.d;
          continue;
        }
        break;
      }
      case OP_OR: {
        Val x = st[--sp];
        if (x.tag == T_BOOL && x.bits) {
          st[sp++] = Val{T_BOOL, 1};
          pc = in.d;
          continue;
        }
        break;
      }
      case OP_ANDEND:
      case OP_OREND: {
        Val y = st[--sp];
        st[sp++] = Val{T_BOOL, (y.tag == T_BOOL && y.bits) ? 1 : 0};
        break;
      }
      case OP_NOT: {
        Val x = st[--sp];
        st[sp++] = Val{T_BOOL, (x.tag == T_BOOL && x.bits) ? 0 : 1};
        break;
      }
      case OP_ISNULL: {
        Val x = st[--sp];
        st[sp++] = Val{T_BOOL, x.tag == T_NULL ? 1 : 0};
        break;
      }
      case OP_CMP: {
        Val y = st[--sp];
        Val x = st[--sp];
        st[sp++] = java_cmp(in, x, y);
        break;
      }
      case OP_ARITH: {
        Val y = st[--sp];
        Val x = st[--sp];
        st[sp++] = java_arith(in, x, y);
        break;
      }
      case OP_IFTE: {  // IfThenElseFunctionExecutor.execute (all three arguments evaluated)
        Val b = st[--sp];
        Val a = st[--sp];
        Val c = st[--sp];
        st[sp++] = (c.tag == T_BOOL && c.bits) ? a : b;
        break;
      }
      case OP_COALESCE: {  // CoalesceFunctionExecutor.execute
        const int n = in.a;
        sp -= n;
        Val r{T_NULL, 0};
        for (int i = n - 1; i >= 0; i--)
          if (st[sp + i].tag != T_NULL) r = st[sp + i];
        st[sp++] = r;
        break;
      }
      case OP_INSTOF: {  // InstanceOf*FunctionExecutor.execute: data instanceof <Type>
        Val x = st[--sp];
        st[sp++] = Val{T_BOOL, (x.tag == (int8_t)in.a && x.tag != T_NULL) ? 1 : 0};
        break;
      }
      default:
        return false;
    }
    pc++;
  }
}

SHP_HD inline Val load_col(const BatchView& B, const DevProg& P, int col, int64_t g) {
  Val v{T_NULL, 0};
  if (B.nulls[col] && B.nulls[col][g]) return v;
  v.tag = P.colTag[col];
  switch (v.tag) {
    case T_LONG: v.bits = ((const int64_t*)B.cols[col])[g]; break;
    case T_DOUBLE: v.bits = ((const int64_t*)B.cols[col])[g]; break;
    case T_FLOAT: v.bits = (int64_t)((const uint32_t*)B.cols[col])[g]; break;
    case T_BOOL: v.bits = ((const uint8_t*)B.cols[col])[g]; break;
    default: v.bits = (int64_t)((const int32_t*)B.cols[col])[g]; break;
  }
  return v;
}

// ---------------------------------------------------------------------------
// The lane.  AS = address space of the state arena on the device: 1 = global (HBM), 3 = LDS,
// 0 = generic (host builds).  Every state access goes through at(), which derives the element
// pointer from an AS-qualified base, so the compiler emits global_* / ds_* instructions instead
// of flat ones (flat accesses count against both the LDS and the memory wait counters).
// ---------------------------------------------------------------------------
template <int AS>
struct LaneAS {
  typedef char type;
};
#if defined(__HIP_DEVICE_COMPILE__)
template <>
struct LaneAS<1> {
  typedef __attribute__((address_space(1))) char type;
};
template <>
struct LaneAS<3> {
  typedef __attribute__((address_space(3))) char type;
};
#endif

template <int AS, int TIER = 0>
struct LaneT {
  using C = LaneCaps<TIER>;
  static constexpr int NSE = C::NSE, NN = C::NN, LCAP = C::LCAP, QCAP = C::QCAP;
  static constexpr int GC_SE_RESERVE = C::GC_SE_RESERVE, GC_ND_RESERVE = C::GC_ND_RESERVE;
  const DevProg& P;
  const LaneLayout& Y;
  char* base;
  int64_t lane;
  int32_t key;
  const BatchView& B;
  const MatchOut& O;
  int64_t clock;      // TimestampGenerator.currentTime() while this lane runs
  int64_t emit_pos;   // global seq stamped on emitted matches
  int32_t err = 0;
  uint32_t ret;       // PostStateProcessor.isEventReturned bits (per key here)

  SHP_HD LaneT(const DevProg& p, const LaneLayout& y, char* b, int64_t l, int32_t k, const BatchView& bv,
              const MatchOut& o)
      : P(p), Y(y), base(b), lane(l), key(k), B(bv), O(o), clock(0), emit_pos(0) {
    ret = at<uint32_t>(Y.o_ret, 0);
  }
  SHP_HD void flush_ret() { at<uint32_t>(Y.o_ret, 0) = ret; }

  template <class T>
  SHP_HD T& at(int64_t off, int64_t i) const {
    typedef typename LaneAS<AS>::type C;
    C* q = (C*)base + off + (i * Y.L + lane) * (int64_t)sizeof(T);
    return *(T*)q;
  }

  // ------------------------------------------------------------ pools
  SHP_HD int16_t& slot(int se, int s) const { return at<int16_t>(Y.o_se_slot, se * MAXS + s); }
  SHP_HD int64_t& sets(int se) const { return at<int64_t>(Y.o_se_ts, se); }
  SHP_HD uint8_t& setype(int se) const { return at<uint8_t>(Y.o_se_type, se); }
  SHP_HD int16_t& nnext(int nd) const { return at<int16_t>(Y.o_nd_next, nd); }
  SHP_HD int64_t& nseq(int nd) const { return at<int64_t>(Y.o_nd_seq, nd); }
  SHP_HD int64_t& nts(int nd) const { return at<int64_t>(Y.o_nd_ts, nd); }
  SHP_HD uint8_t& pflags(int p) const { return at<uint8_t>(Y.o_pflags, p); }
  SHP_HD int64_t& lsched(int p) const { return at<int64_t>(Y.o_lsched, p); }
  SHP_HD int64_t& larr(int p) const { return at<int64_t>(Y.o_larr, p); }
  SHP_HD bool flag(int p, uint8_t f) const { return (pflags(p) & f) != 0; }
  SHP_HD void setf(int p, uint8_t f, bool on) const {
    uint8_t& x = pflags(p);
    x = on ? (uint8_t)(x | f) : (uint8_t)(x & ~f);
  }

  SHP_HD int alloc_bit(int64_t off, int words, int32_t errbit) {
    for (int w = 0; w < words; w++) {
      uint64_t& u = at<uint64_t>(off, w);
      if (~u) {
        int b = 0;
        uint64_t free = ~u;
        while (!((free >> b) & 1ull)) b++;
        u |= 1ull << b;
        return w * 64 + b;
      }
    }
    err |= errbit;
    return -1;
  }
  SHP_HD int free_count(int64_t off, int words) const {
    int c = 0;
    for (int w = 0; w < words; w++) {
      uint64_t u = at<uint64_t>(off, w);
      for (int b = 0; b < 64; b++) c += !((u >> b) & 1ull);
    }
    return c;
  }

  // StateEventFactory.newInstance: all slots null, ts -1, CURRENT
  SHP_HD int new_se() {
    int s = alloc_bit(Y.o_se_used, NSE / 64, E_SE);
    if (s < 0) return -1;
    for (int i = 0; i < P.nstates; i++) slot(s, i) = -1;
    sets(s) = -1;
    setype(s) = 0;
    return s;
  }
  // StateEventCloner.copyStateEvent: shallow slot copy
  SHP_HD int copy_se(int src) {
    int s = alloc_bit(Y.o_se_used, NSE / 64, E_SE);
    if (s < 0) return -1;
    for (int i = 0; i < P.nstates; i++) slot(s, i) = slot(src, i);
    sets(s) = sets(src);
    setype(s) = setype(src);
    return s;
  }
  // StreamEventCloner.copyStreamEvent of batch event g (captures predicate columns)
  SHP_HD int node_of_event(int64_t g) {
    int nd = alloc_bit(Y.o_nd_used, NN / 64, E_ND);
    if (nd < 0) return -1;
    nseq(nd) = bseq(B, g);
    nts(nd) = B.ts[g];
    nnext(nd) = -1;
    int st = B.stream[g];
    uint8_t nul = 0;
    for (int j = 0; j < P.streamNcol[st]; j++) {
      int c = P.streamCols[st][j];
      Val v = load_col(B, P, c, g);
      at<int64_t>(Y.o_nd_val, nd * NV + j) = v.bits;
      if (v.tag == T_NULL) nul |= (uint8_t)(1u << j);
    }
    at<uint8_t>(Y.o_nd_null, nd) = nul;
    return nd;
  }
  // StreamEventFactory.newInstance(): empty event (ts -1, all attributes null)
  SHP_HD int empty_node() {
    int nd = alloc_bit(Y.o_nd_used, NN / 64, E_ND);
    if (nd < 0) return -1;
    nseq(nd) = -1;
    nts(nd) = -1;
    nnext(nd) = -1;
    at<uint8_t>(Y.o_nd_null, nd) = 0xff;
    return nd;
  }

  // mark-sweep over everything reachable from the lists (the only roots at event boundaries)
  SHP_HD void gc() {
    uint64_t mse[NSE / 64] = {0};
    uint64_t mnd[NN / 64] = {0};
    for (int l = 0; l < 2 * MAXP; l++) {
      int n = at<int16_t>(Y.o_lst_len, l);
      for (int i = 0; i < n; i++) {
        int s = at<int16_t>(Y.o_lst, l * LCAP + i);
        if (s < 0) continue;
        if ((mse[s >> 6] >> (s & 63)) & 1ull) continue;
        mse[s >> 6] |= 1ull << (s & 63);
        for (int k = 0; k < P.nstates; k++) {
          for (int nd = slot(s, k); nd >= 0; nd = nnext(nd)) {
            if ((mnd[nd >> 6] >> (nd & 63)) & 1ull) break;
            mnd[nd >> 6] |= 1ull << (nd & 63);
          }
        }
      }
    }
    for (int w = 0; w < NSE / 64; w++) at<uint64_t>(Y.o_se_used, w) = mse[w];
    for (int w = 0; w < NN / 64; w++) at<uint64_t>(Y.o_nd_used, w) = mnd[w];
  }
  SHP_HD void maybe_gc() {
    if (free_count(Y.o_se_used, NSE / 64) < GC_SE_RESERVE || free_count(Y.o_nd_used, NN / 64) < GC_ND_RESERVE)
      gc();
  }

  // ------------------------------------------------------------ lists
  SHP_HD int16_t& llen(int p, int which) const { return at<int16_t>(Y.o_lst_len, which * MAXP + p); }
  SHP_HD int16_t& litem(int p, int which, int i) const {
    return at<int16_t>(Y.o_lst, (which * MAXP + p) * LCAP + i);
  }
  SHP_HD void lpush(int p, int which, int se) {
    int16_t& n = llen(p, which);
    if (n >= LCAP) {
      err |= E_LIST;
      return;
    }
    litem(p, which, n) = (int16_t)se;
    n++;
  }
  SHP_HD void lerase(int p, int which, int i) {
    int16_t& n = llen(p, which);
    for (int k = i; k + 1 < n; k++) litem(p, which, k) = litem(p, which, k + 1);
    n--;
  }
  SHP_HD void lremove_obj(int p, int which, int se) {
    int n = llen(p, which);
    for (int i = 0; i < n; i++)
      if (litem(p, which, i) == se) {
        lerase(p, which, i);
        return;
      }
  }
  static constexpr int PEND = 0, NEW = 1;

  // ------------------------------------------------------------ chains
  SHP_HD int chain_len(int nd) const {
    int c = 0;
    for (; nd >= 0; nd = nnext(nd)) c++;
    return c;
  }
  // StateEvent.getStreamEvent(int[]) (core/event/state/StateEvent.java:138-189)
  SHP_HD int get_event(int se, int state, int index) const {
    int nd = slot(se, state);
    if (nd < 0) return -1;
    if (index >= 0) {
      for (int i = 1; i <= index; i++) {
        nd = nnext(nd);
        if (nd < 0) return -1;
      }
      return nd;
    }
    if (index == -1) {
      while (nnext(nd) >= 0) nd = nnext(nd);
      return nd;
    }
    if (index == -2) {
      if (nnext(nd) < 0) return -1;
      while (nnext(nnext(nd)) >= 0) nd = nnext(nd);
      return nd;
    }
    int len = chain_len(nd);
    int idx = len + index;
    if (idx < 0) return -1;
    for (int i = 0; i < idx; i++) nd = nnext(nd);
    return nd;
  }
  // StateEvent.addEvent :212-222
  SHP_HD void add_event(int se, int pos, int nd) {
    int a = slot(se, pos);
    if (a < 0) {
      slot(se, pos) = (int16_t)nd;
      return;
    }
    while (nnext(a) >= 0) a = nnext(a);
    nnext(a) = (int16_t)nd;
  }
  // StateEvent.removeLastEvent :224-236
  SHP_HD void remove_last_event(int se, int pos) {
    int a = slot(se, pos);
    if (a >= 0) {
      while (nnext(a) >= 0) {
        if (nnext(nnext(a)) < 0) {
          nnext(a) = -1;
          return;
        }
        a = nnext(a);
      }
      slot(se, pos) = -1;
    }
  }

  // ------------------------------------------------------------ filter
  struct Res {
    const LaneT* L;
    int se;
    SHP_HD Val value(int state, int index, int col) const {
      Val v{T_NULL, 0};
      int nd = L->get_event(se, state, index);
      if (nd < 0 || L->nseq(nd) < 0) return v;
      int pos = L->P.colPos[col];
      if ((L->at<uint8_t>(L->Y.o_nd_null, nd) >> pos) & 1) return v;
      v.tag = L->P.colTag[col];
      v.bits = L->at<int64_t>(L->Y.o_nd_val, nd * NV + pos);
      return v;
    }
    SHP_HD bool isnull_state(int state, int index) const { return L->get_event(se, state, index) < 0; }
  };

  // ------------------------------------------------------------ emit
  SHP_HD void emit(int se) {
    unsigned long long mi, ri;
    int lens[MAXS];
    int tot = 0;
    for (int s = 0; s < P.nstates; s++) {
      lens[s] = chain_len(slot(se, s));
      tot += lens[s];
    }
#if defined(__HIP_DEVICE_COMPILE__)
    mi = atomicAdd(&O.count[0], 1ull);
    ri = atomicAdd(&O.count[1], (unsigned long long)tot);
#else
    mi = O.count[0]++;
    ri = O.count[1];
    O.count[1] += tot;
#endif
    if ((int64_t)mi >= O.cap || (int64_t)(ri + tot) > O.refcap) {
      err |= E_OUT;
      return;
    }
    O.key[mi] = key;
    O.ts[mi] = sets(se);
    O.type[mi] = (int8_t)setype(se);
    O.pos[mi] = emit_pos;
    O.ref_off[mi] = (int64_t)ri;
    int64_t r = (int64_t)ri;
    for (int s = 0; s < P.nstates; s++) {
      O.slot_len[mi * MAXS + s] = (int16_t)lens[s];
      for (int nd = slot(se, s); nd >= 0; nd = nnext(nd)) O.refs[r++] = nseq(nd);
    }
    if (P.aggFn && O.agg) O.agg[mi] = aggregate(se);
  }

  // The selector's running aggregate of this key over its matches in emission order
  // (QuerySelector.processInBatchNoGroupBy :271-313, one output per match; per partition key
  // its own state, AttributeAggregatorExecutor.initAggregator :43-60), folded as the match is
  // emitted: AvgAttributeAggregatorExecutor (`value += x; count++`, value / count), Sum, Count,
  // Min / MaxAttributeAggregatorExecutor (first value, then `if (value > x) value = x`).  A null
  // argument leaves the state and returns the current value (processAdd :110-115); a result that
  // is itself null (no value yet) flags E_AGGNULL and the push fails, as on the sweep.
  SHP_HD double aggregate(int se) {
    double& a = at<double>(Y.o_agg, 0);  // avg / sum: the sum; min / max: the value (NaN: first was NaN)
    double& c = at<double>(Y.o_agg, 1);  // values folded (count: matches)
    const int fn = P.aggFn;
    if (fn == 3) {
      c += 1.0;
      return c;
    }
    Res R{this, se};
    const Val v = R.value(P.aggState, 0, P.aggCol);
    if (v.tag != T_NULL) {
      double x;
      if (v.tag == T_FLOAT) x = (double)bits_f(v.bits);
      else if (v.tag == T_DOUBLE) x = bits_d(v.bits);
      else x = (double)v.bits;  // int / long (exact to 2^53, as the sweep's double state)
      if (fn <= 2) {
        a += x;
      } else if (c == 0.0) {
        a = x;
      } else if (!(a != a) && x == x) {
        a = fn == 4 ? (a > x ? x : a) : (a < x ? x : a);
      }
      c += 1.0;
    }
    if (c == 0.0) {
      err |= E_AGGNULL;
      return 0.0;
    }
    return fn == 1 ? a / c : a;
  }

  // ------------------------------------------------------------ timers
  SHP_HD void notify_at(int sched, int64_t t) {
    int16_t& h = at<int16_t>(Y.o_qhead, sched);
    int16_t& n = at<int16_t>(Y.o_qlen, sched);
    if (n >= QCAP) {
      err |= E_Q;
      return;
    }
    at<int64_t>(Y.o_q, sched * QCAP + (h + n) % QCAP) = t;
    n++;
  }

  // =================================================================
  // PreStateProcessor family (state/*PreStateProcessor.java)
  // =================================================================
  SHP_HD bool is_absent(int p) const { return P.pre[p].kind == K_ABSENT_STREAM || P.pre[p].kind == K_ABSENT_LOGICAL; }

  // StreamPreStateProcessor.init :178-194
  SHP_HD void init(int p) {
    const DPre& d = P.pre[p];
    const DPost& q = P.post[d.thisPost];
    if (d.isStart && (!flag(p, F_INIT) || q.nextEvery >= 0 ||
                      (P.type == SEQUENCE && q.nextState >= 0 && is_absent(q.nextState)))) {
      int se = new_se();
      if (se < 0) return;
      add_state(p, se);
      setf(p, F_INIT, true);
    }
  }

  // LogicalPreStateProcessor.addState :43-62
  SHP_HD void logical_add_state(int p, int se) {
    const DPre& d = P.pre[p];
    if (d.isStart || P.type == SEQUENCE) {
      if (llen(p, NEW) == 0) lpush(p, NEW, se);
      if (d.partner >= 0 && llen(d.partner, NEW) == 0) lpush(d.partner, NEW, se);
    } else {
      lpush(p, NEW, se);
      if (d.partner >= 0) lpush(d.partner, NEW, se);
    }
  }

  SHP_HD void add_state(int p, int se) {
    const DPre& d = P.pre[p];
    switch (d.kind) {
      case K_STREAM:  // StreamPreStateProcessor.addState :214-227
        if (P.type == SEQUENCE) {
          if (llen(p, NEW) == 0) lpush(p, NEW, se);
        } else {
          lpush(p, NEW, se);
        }
        break;
      case K_COUNT:  // CountPreStateProcessor.addState :114-138
        if (P.type == SEQUENCE) {
          if (llen(p, NEW) == 0) lpush(p, NEW, se);
        } else {
          lpush(p, NEW, se);
        }
        if (d.minCount == 0 && slot(se, d.stateId) < 0) min_count_reached(d.countPost, se);
        break;
      case K_LOGICAL:
        logical_add_state(p, se);
        break;
      case K_ABSENT_STREAM:  // AbsentStreamPreStateProcessor.addState :80-103
        if (flag(p, F_INACTIVE)) return;
        if (P.type == SEQUENCE) llen(p, NEW) = 0;
        lpush(p, NEW, se);
        if (!d.isStart) {
          lsched(p) = sets(se) + d.waiting;
          notify_at(d.sched, lsched(p));
        }
        break;
      case K_ABSENT_LOGICAL:  // AbsentLogicalPreStateProcessor.addState :77-97
        if (flag(p, F_INACTIVE)) return;
        logical_add_state(p, se);
        if (!d.isStart && d.waiting != -1) {
          notify_at(d.sched, sets(se) + d.waiting);
          const DPre& pp = P.pre[d.partner];
          if (pp.kind == K_ABSENT_LOGICAL) notify_at(pp.sched, sets(se) + pp.waiting);
        }
        break;
    }
  }

  SHP_HD void add_every_state(int p, int se) {
    const DPre& d = P.pre[p];
    int c = copy_se(se);
    if (c < 0) return;
    setype(c) = 0;
    switch (d.kind) {
      case K_STREAM:
      case K_COUNT:  // StreamPreStateProcessor.addEveryState :230-247
        for (int i = d.stateId; i < P.nstates; i++) slot(c, i) = -1;
        lpush(p, NEW, c);
        break;
      case K_LOGICAL:  // LogicalPreStateProcessor.addEveryState :65-84
        for (int i = d.stateId; i < P.nstates; i++) slot(c, i) = -1;
        lpush(p, NEW, c);
        if (d.partner >= 0) {
          slot(c, P.pre[d.partner].stateId) = -1;
          lpush(d.partner, NEW, c);
        }
        break;
      case K_ABSENT_STREAM:  // AbsentStreamPreStateProcessor.addEveryState :106-123
        for (int i = d.stateId; i < P.nstates; i++) slot(c, i) = -1;
        lpush(p, NEW, c);
        lsched(p) = sets(se) + d.waiting;
        notify_at(d.sched, lsched(p));
        break;
      case K_ABSENT_LOGICAL:  // AbsentLogicalPreStateProcessor.addEveryState :100-118
        if (slot(c, d.stateId) >= 0) sets(c) = nts(slot(c, d.stateId));
        slot(c, d.stateId) = -1;
        slot(c, P.pre[d.partner].stateId) = -1;
        lpush(p, NEW, c);
        lpush(d.partner, NEW, c);
        break;
    }
  }

  SHP_HD bool next_pending_nonempty(int p) const {
    int ns = P.post[P.pre[p].thisPost].nextState;
    return ns >= 0 && llen(ns, PEND) > 0;
  }

  SHP_HD void reset_state(int p) {
    const DPre& d = P.pre[p];
    const DPost& q = P.post[d.thisPost];
    switch (d.kind) {
      case K_STREAM:
      case K_COUNT:  // StreamPreStateProcessor.resetState :288-305
        llen(p, PEND) = 0;
        if (d.isStart && llen(p, NEW) == 0) {
          if (P.type == SEQUENCE && q.nextEvery < 0 && next_pending_nonempty(p)) return;
          init(p);
        }
        break;
      case K_LOGICAL:
      case K_ABSENT_LOGICAL:  // LogicalPreStateProcessor.resetState :87-110
        if (d.logical == L_OR || llen(p, PEND) == llen(d.partner, PEND)) {
          llen(p, PEND) = 0;
          llen(d.partner, PEND) = 0;
          if (d.isStart && llen(p, NEW) == 0) {
            if (P.type == SEQUENCE && q.nextEvery < 0 && next_pending_nonempty(p)) return;
            init(p);
          }
        }
        break;
      case K_ABSENT_STREAM:  // AbsentStreamPreStateProcessor.resetState :126-148
        llen(p, PEND) = 0;
        if (d.isStart) {
          if (P.type == SEQUENCE && q.nextEvery < 0 && next_pending_nonempty(p)) return;
          init(p);
        }
        break;
    }
  }

  // newAndEvery.sort(eventTimeComparator) (ts -1 last, stable) then pending.addAll
  SHP_HD void sort_move(int p) {
    int n = llen(p, NEW);
    for (int i = 1; i < n; i++) {  // stable insertion sort
      int16_t x = litem(p, NEW, i);
      int64_t tx = sets(x);
      int j = i - 1;
      while (j >= 0) {
        int64_t tj = sets(litem(p, NEW, j));
        bool gt = (tx == -1) ? false : (tj == -1 ? true : tj > tx);
        if (!gt) break;
        litem(p, NEW, j + 1) = litem(p, NEW, j);
        j--;
      }
      litem(p, NEW, j + 1) = x;
    }
    for (int i = 0; i < n; i++) lpush(p, PEND, litem(p, NEW, i));
    llen(p, NEW) = 0;
  }

  SHP_HD void update_state(int p) {
    const DPre& d = P.pre[p];
    switch (d.kind) {
      case K_STREAM:
      case K_ABSENT_STREAM:  // StreamPreStateProcessor.updateState :308-323
        sort_move(p);
        break;
      case K_COUNT:  // CountPreStateProcessor.updateState :182-193
        if (flag(p, F_SSRESET)) {
          setf(p, F_SSRESET, false);
          init(p);
        }
        sort_move(p);
        break;
      case K_LOGICAL:
      case K_ABSENT_LOGICAL:  // LogicalPreStateProcessor.updateState :113-125
        sort_move(p);
        sort_move(d.partner);
        break;
    }
  }

  // StreamPreStateProcessor.isExpired :118-129
  SHP_HD bool is_expired(int se, int64_t now) const {
    if (P.within == -1) return false;
    for (int i = 0; i < P.nstart; i++) {
      int nd = slot(se, P.startIds[i]);
      if (nd >= 0) {
        int64_t dlt = nts(nd) - now;
        if (dlt < 0) dlt = -dlt;
        if (dlt > P.within) return true;
      }
    }
    return false;
  }

  // StreamPreStateProcessor.expireEvents :326-361
  SHP_HD void expire_events(int p, int64_t ts) {
    int expired = -1;
    while (llen(p, PEND) > 0) {
      int se = litem(p, PEND, 0);
      if (!is_expired(se, ts)) break;
      lerase(p, PEND, 0);
      if (setype(se) != 1) {
        setype(se) = 1;
        expired = se;
      }
    }
    for (int i = 0; i < llen(p, NEW);) {
      int se = litem(p, NEW, i);
      if (is_expired(se, ts)) {
        lerase(p, NEW, i);
        if (setype(se) != 1) {
          setype(se) = 1;
          expired = se;
        }
      } else {
        i++;
      }
    }
    int we = P.pre[p].withinEvery;
    if (expired >= 0 && we >= 0) {
      add_every_state(we, expired);
      update_state(we);
    }
  }

  // StreamPreStateProcessor.process(StateEvent) :131-142 + FilterProcessor.process
  SHP_HD void process(int p, int se) {
    setf(p, F_CHANGED, false);
    const DPre& d = P.pre[p];
    if (d.filterPc >= 0) {
      Res r{this, se};
      if (!run_filter(P, d.filterPc, r)) return;
    }
    post_process(d.thisPost, se);
  }

  SHP_HD bool take_returned(int p) {
    int tl = P.pre[p].thisLast;
    if ((ret >> tl) & 1u) {
      ret &= ~(1u << tl);
      return true;
    }
    return false;
  }

  // returns the number of StateEvents placed in out[] (emitted by the receiver)
  SHP_HD int process_and_return(int p, int64_t g, int* out) {
    const DPre& d = P.pre[p];
    int nret = 0;
    switch (d.kind) {
      case K_STREAM:
        return stream_par(p, g, true, out);
      case K_ABSENT_STREAM:  // AbsentStreamPreStateProcessor.processAndReturn :257-274
        if (flag(p, F_INACTIVE)) return 0;
        stream_par(p, g, false, out);
        return 0;
      case K_COUNT: {  // CountPreStateProcessor.processAndReturn :53-95
        for (int i = 0; i < llen(p, PEND);) {
          int se = litem(p, PEND, i);
          if ((P.nstates > d.stateId + 1 && slot(se, d.stateId + 1) >= 0) ||
              (P.nstates > d.stateId + 2 && slot(se, d.stateId + 2) >= 0)) {
            lerase(p, PEND, i);
            continue;
          }
          int nd = node_of_event(g);
          if (nd < 0) return nret;
          add_event(se, d.stateId, nd);
          setf(p, F_SUCCESS, false);
          process(p, se);
          if (take_returned(p)) out[nret++] = se;
          bool removed = false;
          if (flag(p, F_CHANGED)) {
            lerase(p, PEND, i);
            removed = true;
          }
          if (!flag(p, F_SUCCESS)) {
            remove_last_event(se, d.stateId);
            if (P.type == SEQUENCE && !removed) {
              lerase(p, PEND, i);
              removed = true;
            }
          }
          if (!removed) i++;
        }
        return nret;
      }
      case K_LOGICAL: {  // LogicalPreStateProcessor.processAndReturn :128-167
        for (int i = 0; i < llen(p, PEND);) {
          int se = litem(p, PEND, i);
          if (d.logical == L_OR && slot(se, P.pre[d.partner].stateId) >= 0) {
            lerase(p, PEND, i);
            continue;
          }
          int nd = node_of_event(g);
          if (nd < 0) return nret;
          slot(se, d.stateId) = (int16_t)nd;
          process(p, se);
          if (take_returned(p)) out[nret++] = se;
          if (flag(p, F_CHANGED)) {
            lerase(p, PEND, i);
          } else {
            slot(se, d.stateId) = -1;
            if (P.type == SEQUENCE) lerase(p, PEND, i);
            else i++;
          }
        }
        return nret;
      }
      case K_ABSENT_LOGICAL: {  // AbsentLogicalPreStateProcessor.processAndReturn :262-319
        if (flag(p, F_INACTIVE)) return 0;
        for (int i = 0; i < llen(p, PEND);) {
          int se = litem(p, PEND, i);
          if (d.logical == L_OR && slot(se, P.pre[d.partner].stateId) >= 0) {
            lerase(p, PEND, i);
            continue;
          }
          int cur = slot(se, d.stateId);
          int nd = node_of_event(g);
          if (nd < 0) return 0;
          slot(se, d.stateId) = (int16_t)nd;
          process(p, se);
          if (d.waiting != -1 ||
              (P.type == SEQUENCE && d.logical == L_AND && P.post[d.thisPost].nextEvery >= 0))
            slot(se, d.stateId) = (int16_t)cur;
          bool removed = false;
          if (take_returned(p)) {
            lerase(p, PEND, i);
            removed = true;
            if (P.type == SEQUENCE) lremove_obj(d.partner, PEND, se);
          }
          if (!flag(p, F_CHANGED)) {
            slot(se, d.stateId) = (int16_t)cur;
            if (P.type == SEQUENCE && !removed) {
              lerase(p, PEND, i);
              removed = true;
            }
          }
          if (!removed) i++;
        }
        return 0;
      }
    }
    return nret;
  }

  // StreamPreStateProcessor.processAndReturn :364-403
  SHP_HD int stream_par(int p, int64_t g, bool removeOnNoChange, int* out) {
    const DPre& d = P.pre[p];
    int nret = 0;
    for (int i = 0; i < llen(p, PEND);) {
      int se = litem(p, PEND, i);
      int nd = node_of_event(g);
      if (nd < 0) return nret;
      slot(se, d.stateId) = (int16_t)nd;
      process(p, se);
      if (take_returned(p)) out[nret++] = se;
      if (flag(p, F_CHANGED)) {
        lerase(p, PEND, i);
      } else {
        slot(se, d.stateId) = -1;
        if (P.type == SEQUENCE) {
          int cb = P.post[d.thisPost].callbackPre;
          if (cb >= 0) setf(cb, F_SSRESET, true);
          if (removeOnNoChange) {
            lerase(p, PEND, i);
            continue;
          }
        }
        i++;
      }
    }
    return nret;
  }

  SHP_HD void update_last_arrival(int p, int64_t ts) {
    const DPre& d = P.pre[p];
    if (d.kind == K_ABSENT_STREAM) {  // AbsentStreamPreStateProcessor.updateLastArrivalTime :68-78
      lsched(p) = ts + d.waiting;
      notify_at(d.sched, lsched(p));
    } else {  // AbsentLogicalPreStateProcessor.updateLastArrivalTime :66-75
      larr(p) = ts;
    }
  }

  // =================================================================
  // PostStateProcessor family
  // =================================================================
  SHP_HD void set_returned(int q) { ret |= 1u << q; }

  // StreamPostStateProcessor.process :64-83
  SHP_HD void stream_post(int qi, int se) {
    const DPost& q = P.post[qi];
    setf(q.thisPre, F_CHANGED, true);
    sets(se) = nts(slot(se, q.stateId));
    if (q.hasNext) set_returned(qi);
    if (q.nextState >= 0) add_state(q.nextState, se);
    if (q.nextEvery >= 0) add_every_state(q.nextEvery, se);
    if (q.callbackPre >= 0) setf(q.callbackPre, F_SSRESET, true);
  }

  // CountPostStateProcessor.processMinCountReached :67-79
  SHP_HD void min_count_reached(int qi, int se) {
    const DPost& q = P.post[qi];
    if (q.hasNext) {
      setf(q.thisPre, F_CHANGED, true);
      set_returned(qi);
    }
    if (q.nextState >= 0) add_state(q.nextState, se);
    if (q.nextEvery >= 0) add_every_state(q.nextEvery, se);
  }

  // AbsentLogicalPreStateProcessor.partnerCanProceed :353-388
  SHP_HD bool partner_can_proceed(int p, int se) {
    const DPre& d = P.pre[p];
    const DPost& q = P.post[d.thisPost];
    if (P.type == SEQUENCE && q.nextEvery < 0 && larr(p) > 0) return false;
    if (d.waiting == -1) {
      if (q.nextEvery < 0) return slot(se, d.stateId) < 0;
      if (larr(p) > 0) {
        larr(p) = 0;
        init(p);
        return false;
      }
      return true;
    }
    return slot(se, d.stateId) >= 0;
  }

  SHP_HD void post_process(int qi, int se) {
    const DPost& q = P.post[qi];
    switch (q.kind) {
      case K_STREAM:
        stream_post(qi, se);
        break;
      case K_COUNT: {  // CountPostStateProcessor.process :39-65
        int nd = slot(se, q.stateId);
        int n = 1;
        while (nnext(nd) >= 0) {
          n++;
          nd = nnext(nd);
        }
        setf(q.thisPre, F_SUCCESS, true);
        sets(se) = nts(nd);
        if (n >= q.minCount) {
          if (P.type == SEQUENCE) {
            if (q.nextState >= 0) add_state(q.nextState, se);
            if (n != q.maxCount) add_state(q.thisPre, se);
          } else if (n == q.minCount) {
            min_count_reached(qi, se);
          }
          if (n == q.maxCount) setf(q.thisPre, F_CHANGED, true);
        }
        break;
      }
      case K_LOGICAL: {  // LogicalPostStateProcessor.process :59-87
        if (q.logical == L_AND) {
          bool proc;
          if (P.pre[q.partnerPre].kind == K_ABSENT_LOGICAL) proc = partner_can_proceed(q.partnerPre, se);
          else proc = slot(se, P.pre[q.partnerPre].stateId) >= 0;
          if (proc) stream_post(qi, se);
          else setf(q.thisPre, F_CHANGED, true);
        } else {
          stream_post(qi, se);
          if (P.post[q.partnerPost].hasNext && P.pre[q.thisPre].thisLast == q.partnerPost) set_returned(q.partnerPost);
        }
        break;
      }
      case K_ABSENT_STREAM: {  // AbsentStreamPostStateProcessor.process :36-56
        setf(q.thisPre, F_CHANGED, true);
        int nd = slot(se, q.stateId);
        sets(se) = nts(nd);
        set_returned(qi);
        if (P.pre[q.thisPre].isStart && q.nextEvery >= 0 && q.nextEvery == q.thisPre) add_every_state(q.nextEvery, se);
        update_last_arrival(q.thisPre, nts(nd));
        break;
      }
      case K_ABSENT_LOGICAL: {  // AbsentLogicalPostStateProcessor.process :37-49
        setf(q.thisPre, F_CHANGED, true);
        int nd = slot(se, q.stateId);
        set_returned(qi);
        update_last_arrival(q.thisPre, nts(nd));
        break;
      }
    }
  }

  // =================================================================
  // absent timers
  // =================================================================
  // AbsentStreamPreStateProcessor.sendEvent :238-254
  SHP_HD void absent_stream_send(int p, int se) {
    const DPre& d = P.pre[p];
    const DPost& q = P.post[d.thisPost];
    if (q.hasNext) emit(se);
    if (q.nextState >= 0) add_state(q.nextState, se);
    if (q.nextEvery >= 0) add_every_state(q.nextEvery, se);
    else if (d.isStart) setf(p, F_INACTIVE, true);
    if (q.callbackPre >= 0) setf(q.callbackPre, F_SSRESET, true);
  }

  // AbsentStreamPreStateProcessor.process(ComplexEventChunk) :151-227
  SHP_HD void absent_stream_timer(int p, int64_t now) {
    const DPre& d = P.pre[p];
    const DPost& q = P.post[d.thisPost];
    if (flag(p, F_INACTIVE)) return;
    int rets[LCAP];
    int nr = 0;
    bool initialize = d.isStart && llen(p, NEW) == 0 && llen(p, PEND) == 0;
    if (initialize && P.type == SEQUENCE && q.nextEvery < 0 && lsched(p) > 0) initialize = false;
    if (initialize) {
      int se = new_se();
      if (se >= 0) add_state(p, se);
    } else if (P.type == SEQUENCE && llen(p, NEW) > 0) {
      reset_state(p);
    }
    update_state(p);
    for (int i = 0; i < llen(p, PEND);) {
      int ev = litem(p, PEND, i);
      if (is_expired(ev, now)) {
        lerase(p, PEND, i);
        if (d.withinEvery >= 0 && q.nextEvery != p && q.nextEvery >= 0) add_every_state(q.nextEvery, ev);
        continue;
      }
      if ((sets(ev) == -1 && now >= lsched(p)) || (sets(ev) != -1 && now >= sets(ev) + d.waiting)) {
        lerase(p, PEND, i);
        sets(ev) = now;
        if (nr < LCAP) rets[nr++] = ev;
        else err |= E_LIST;
        continue;
      }
      i++;
    }
    if (d.withinEvery >= 0) update_state(d.withinEvery);
    bool notProcessed = nr == 0;
    for (int i = 0; i < nr; i++) absent_stream_send(p, rets[i]);
    if (clock > d.waiting + now) lsched(p) = clock + d.waiting;
    if (notProcessed && lsched(p) < now) {
      lsched(p) = now + d.waiting;
      notify_at(d.sched, lsched(p));
    }
  }

  // AbsentLogicalPreStateProcessor.sendEvent :230-250
  SHP_HD void absent_logical_send(int p, int se) {
    const DPre& d = P.pre[p];
    const DPost& q = P.post[d.thisPost];
    if (q.hasNext) emit(se);
    if (q.nextState >= 0) add_state(q.nextState, se);
    if (q.nextEvery >= 0) {
      add_every_state(q.nextEvery, se);
    } else if (d.isStart) {
      setf(p, F_INACTIVE, true);
      if (d.logical == L_OR && P.pre[d.partner].kind == K_ABSENT_LOGICAL) setf(d.partner, F_INACTIVE, true);
    }
    if (q.callbackPre >= 0) setf(q.callbackPre, F_SSRESET, true);
  }

  // AbsentLogicalPreStateProcessor.process(ComplexEventChunk) :121-209
  SHP_HD void absent_logical_timer(int p, int64_t now) {
    const DPre& d = P.pre[p];
    const DPost& q = P.post[d.thisPost];
    if (flag(p, F_INACTIVE)) return;
    bool notProcessed = true;
    if (now >= larr(p) + d.waiting) {
      int rets[LCAP];
      int nr = 0;
      if (d.isStart && P.type == SEQUENCE && llen(p, NEW) == 0 && llen(p, PEND) == 0) {
        int se = new_se();
        if (se >= 0) add_state(p, se);
      } else if (P.type == SEQUENCE && llen(p, NEW) > 0) {
        reset_state(p);
      }
      update_state(p);
      int expired = -1;
      int pst = P.pre[d.partner].stateId;
      for (int i = 0; i < llen(p, PEND);) {
        int se = litem(p, PEND, i);
        if (is_expired(se, now)) {
          expired = se;
          lerase(p, PEND, i);
          continue;
        }
        int mine = slot(se, d.stateId);
        bool passed = mine < 0 ? now >= sets(se) + d.waiting : now >= nts(mine) + d.waiting;
        if (passed) {
          lerase(p, PEND, i);
          bool pf = slot(se, pst) >= 0;
          if (d.logical == L_OR && !pf) {
            int nd = empty_node();
            if (nd >= 0) add_event(se, d.stateId, nd);
            if (nr < LCAP) rets[nr++] = se;
          } else if (d.logical == L_AND && pf) {
            if (nr < LCAP) rets[nr++] = se;
          } else if (d.logical == L_AND && !pf) {
            int nd = empty_node();
            if (nd >= 0) add_event(se, d.stateId, nd);
          }
          continue;
        }
        i++;
      }
      if (expired >= 0 && d.withinEvery >= 0) {
        add_every_state(d.withinEvery, expired);
        update_state(d.withinEvery);
      }
      notProcessed = nr == 0;
      for (int i = 0; i < nr; i++) {
        sets(rets[i]) = now;
        absent_logical_send(p, rets[i]);
      }
      larr(p) = 0;
    }
    if (q.nextEvery >= 0 || (notProcessed && d.isStart)) {
      int64_t nb = larr(p) == 0 ? clock + d.waiting : larr(p) + d.waiting;
      notify_at(d.sched, nb);
    }
  }

  // partitionCreated (AbsentStream :291-308, AbsentLogical :332-351)
  SHP_HD void partition_created(int p) {
    const DPre& d = P.pre[p];
    if (!flag(p, F_STARTED)) {
      setf(p, F_STARTED, true);
      if (d.isStart && d.waiting != -1 && !flag(p, F_INACTIVE)) {
        if (d.kind == K_ABSENT_STREAM) {
          lsched(p) = clock + d.waiting;
          notify_at(d.sched, lsched(p));
        } else {
          notify_at(d.sched, clock + d.waiting);
        }
      }
    }
  }

  // StateStreamRuntime.initPartition :90-97
  SHP_HD void init_partition() {
    for (int i = 0; i < P.ninit; i++) init(P.initOrder[i]);
    for (int i = 0; i < P.nstartup; i++) partition_created(P.startup[i]);
    at<uint8_t>(Y.o_kinit, 0) = 1;
  }

  SHP_HD void fire_one(int s, int64_t due) {
    int p = P.schedPre[s];
    if (P.pre[p].kind == K_ABSENT_STREAM) absent_stream_timer(p, due);
    else absent_logical_timer(p, due);
  }

  SHP_HD bool q_head(int s, int64_t* h) const {
    if (at<int16_t>(Y.o_qlen, s) == 0) return false;
    *h = at<int64_t>(Y.o_q, s * QCAP + at<int16_t>(Y.o_qhead, s));
    return true;
  }
  SHP_HD void q_pop(int s) const {
    int16_t& h = at<int16_t>(Y.o_qhead, s);
    h = (int16_t)((h + 1) % QCAP);
    at<int16_t>(Y.o_qlen, s)--;
  }

  SHP_HD int64_t clock_before(int64_t g) const { return g == 0 ? B.clock0 : B.rmax[g - 1]; }
  SHP_HD bool is_call(int64_t g) const { return !P.playback || B.tclk[g] >= clock_before(g); }

  // first global event index c in [lo, hi] at which a timer due at `due` fires:
  // playback: a call point whose clock (= ts[c]) >= due; live: first event with ts >= due.
  SHP_HD int64_t first_fire(int64_t lo, int64_t hi, int64_t due) const {
    if (lo > hi) return -1;
    if (clock_before(lo) < due) {
      // rmax is monotone: lower_bound(rmax[lo..hi] >= due); that event raised the clock -> a call
      const int64_t rh = B.rmax[hi];
      if (rh < due) return -1;
      const int64_t rl = B.rmax[lo];
      if (rl >= due) return lo;
      // lower bound in (a, b] with rmax[a] < due <= rmax[b]: interpolation steps (event-time
      // clocks are close to linear in the index, so this takes a few dependent loads, not
      // log2(range)), alternating with bisection for the worst case
      int64_t a = lo, b = hi, ra = rl, rb = rh;
      bool interp = true;
      while (b - a > 1) {
        int64_t m;
        if (interp && rb > ra) {
          const double f = (double)(due - ra) / (double)(rb - ra);
          m = a + (int64_t)(f * (double)(b - a));
          m = m <= a ? a + 1 : (m >= b ? b - 1 : m);
        } else {
          m = a + (b - a) / 2;
        }
        interp = !interp;
        const int64_t rm = B.rmax[m];
        if (rm >= due) {
          b = m;
          rb = rm;
        } else {
          a = m;
          ra = rm;
        }
      }
      return b;
    }
    for (int64_t c = lo; c <= hi; c++) {
      if (P.playback ? is_call(c) : (B.ts[c] >= due)) return c;
    }
    return -1;
  }

  // Emulate Scheduler.onTimeChange for this key over global events [lo, hi]
  // (core/util/Scheduler.java:71-103, 171-209): listeners in scheduler order, FIFO queues.
  SHP_HD void timers(int64_t lo, int64_t hi) {
    if (P.nsched == 0) return;
    while (lo <= hi && !err) {
      int64_t best = -1;
      if (P.playback) {
        for (int s = 0; s < P.nsched; s++) {
          int64_t h;
          if (!q_head(s, &h)) continue;
          int64_t c = first_fire(lo, hi, h);
          if (c >= 0 && (best < 0 || c < best)) best = c;
        }
        if (best < 0) return;
        clock = B.tclk[best];
        emit_pos = bseq(B, best);
        for (int s = 0; s < P.nsched; s++) {
          int64_t h;
          while (q_head(s, &h) && h <= clock) {
            q_pop(s);
            fire_one(s, h);
            if (err) return;
          }
        }
        lo = best + 1;
      } else {
        // live scheduler emulation: earliest due head first (scheduler order on ties)
        int bs = -1;
        int64_t bh = 0;
        for (int s = 0; s < P.nsched; s++) {
          int64_t h;
          if (q_head(s, &h) && (bs < 0 || h < bh)) {
            bs = s;
            bh = h;
          }
        }
        if (bs < 0) return;
        int64_t c = first_fire(lo, hi, bh);
        if (c < 0) return;
        int64_t cb = clock_before(c);
        clock = cb > bh ? cb : bh;
        emit_pos = bseq(B, c);
        // Scheduler.sendTimerEvents for (bs, this key): drain every head <= clock
        int64_t h;
        while (q_head(bs, &h) && h <= clock) {
          q_pop(bs);
          fire_one(bs, h);
          if (err) return;
        }
        lo = c;  // more timers may fire before the same event
      }
    }
  }

  // One InputHandler.send of batch event g on this key (after its timers).
  SHP_HD void on_event(int64_t g) {
    clock = B.rmax[g];
    emit_pos = bseq(B, g);
    if (!at<uint8_t>(Y.o_kinit, 0)) init_partition();
    int st = B.stream[g];
    if (st < 0 || st >= P.nstream || P.recvCount[st] == 0) return;
    maybe_gc();
    int64_t ts = B.ts[g];
    // stabilizeStates (state/receiver/*.java)
    for (int i = 0; i < P.nexpire; i++) expire_events(P.expireOrder[i], ts);
    if (P.type == SEQUENCE) {
      for (int i = 0; i < P.nreset; i++) reset_state(P.resetOrder[i]);
      for (int i = 0; i < P.nupdate; i++) update_state(P.updateOrder[i]);
    } else if (P.recvMulti[st]) {
      for (int i = 0; i < P.recvCount[st]; i++) update_state(P.recvPre[st][i]);
    } else {
      update_state(P.recvPre[st][0]);
    }
    int out[LCAP];
    if (P.recvMulti[st]) {
      for (int i = P.recvCount[st] - 1; i >= 0; i--) {
        int n = process_and_return(P.recvPre[st][i], g, out);
        if (P.recvSelector[st])
          for (int k = 0; k < n; k++) emit(out[k]);
      }
    } else {
      int n = process_and_return(P.recvPre[st][0], g, out);
      if (P.recvSelector[st])
        for (int k = 0; k < n; k++) emit(out[k]);
    }
  }
};

using Lane = LaneT<0>;

}  // namespace shp
