// siddhi-hip: the "sweep" path — the 2-state `every e1=S[f1] -> e2=S[f2] within W`
// query as two HBM passes (partition, then an LDS-resident per-owner sweep).
//
// Semantics (StreamPreStateProcessor.processAndReturn/expireEvents
// :326-403 and the last-state-first order of PatternMultiProcessStreamReceiver :32-39):
// per partition key, with non-decreasing timestamps, every event i with f1(i) opens
// candidate i; candidate i closes at the first later event j of the key with
// ts_j - ts_i <= W and f2(i, j), and expires at the first later event with ts_j - ts_i > W.
// Matches are emitted in (j, i) order per key.  Candidates are independent of each other.
//
// Layout and passes:
//   keys are hashed onto NOWN "owners" (host-built map key -> owner | local key << 16,
//   <= SW_LK local keys per owner).
//   k_sw_count    super-tile x owner histogram            reads key (+stream)      4 B/event
//   exclusive scan of the NOWN x NST counts (owner-major)  -> stable owner regions
//   k_sw_scatter  stable multisplit by owner (wave ballot ranks, no atomics), writes a
//                 16-byte record {ts|local key, batch index, value} per event
//                                                          reads 16 B, writes 16 B
//   k_sw_solve    one workgroup per owner walks its region in chunks of SWS_CHUNK records:
//                 carried open candidates + chunk -> stable split by local key in LDS ->
//                 per-candidate forward scan -> per-closer counts -> block scan ->
//                 (i, j) pairs written in (key, j, i) order -> open candidates carried.
//                                                          reads 16 B, writes 16 B/match
// Per-key emission order is exact; across keys the order is unspecified (as the ABI says).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>
#include <cstring>
#include <rocprim/rocprim.hpp>
#include <utility>
#include <stdexcept>
#include <vector>

#include "fast_core.h"
#include "fastpath.h"
#include "nfa_lane.h"
#include "prog.h"
#include "wave_dpp.h"

namespace shp {

#ifndef SWS_THREADS_CFG
#define SWS_THREADS_CFG 512
#endif
#ifndef SWS_CHUNK_CFG
#define SWS_CHUNK_CFG 1984
#endif
#ifndef SWS_CCAP_CFG
#define SWS_CCAP_CFG 512
#endif
#ifndef SWS_OWN_MIN
#define SWS_OWN_MIN 512
#endif
constexpr int SW_THREADS = 256;
constexpr int SW_WAVES = SW_THREADS / 64;
constexpr int SW_LK = 255;          // local keys per owner; bin 255 = "no item"
constexpr int SW_MAXOWN = 2048;     // owners (partition bins)
constexpr int SW_PREF_OWN = 1024;   // owner count the map stops at unless keys would crowd them
constexpr int SW_MIN_OWN = SWS_OWN_MIN;     // owner count the map grows to while owners keep ~2 keys (fill the CUs)
constexpr int SW_LKTAB = 65536;     // scatter LDS bound: its counters + the key -> local key table
// partition
#ifndef SWP_THREADS_CFG
#define SWP_THREADS_CFG 512
#endif
constexpr int SWP_THREADS = SWP_THREADS_CFG;  // scatter workgroup
constexpr int SWP_WAVES = SWP_THREADS / 64;
#ifndef SWP_PER_LANE_CFG
#define SWP_PER_LANE_CFG 8
#endif
constexpr int SWP_ROUND = SWP_THREADS * SWP_PER_LANE_CFG;  // events ranked per round: 8 per lane
constexpr int SWP_SEG = SWP_ROUND / SWP_WAVES;
constexpr int SWP_SUB = SWP_SEG / 64;
// solve
constexpr int SWS_CHUNK = SWS_CHUNK_CFG;  // records per chunk: with ~<64 carried, E <= 2048 = 4 per thread
constexpr int SWS_CCAP = SWS_CCAP_CFG;  // carried open candidates per owner
constexpr int SWS_EMAX = SWS_CHUNK + SWS_CCAP;
constexpr int SWS_SEG = SWS_EMAX / SW_WAVES;
constexpr int SWS_SUB = SWS_SEG / 64;
constexpr int SW_PROBE = 8;  // probe window (emit back-search, sentinel padding)
constexpr int SW_P1 = 4;     // first-round probes per position
constexpr int SW_P2 = 8;     // probes per worklist round

// error bits (engine.hip maps them to status codes)
constexpr int SWE_KEYS = 1 << 20;   // key id outside [0, max_keys)
constexpr int SWE_MONO = 1 << 21;   // ts decreases within a key (scan kernels only; the sweep is exact)
constexpr int SWE_RANGE = 1 << 23;  // ts outside base +- 2^49 ms
constexpr int SWE_AGGNULL = 1 << 24; // SHP_LAYOUT_AGG: a closing event's aggregated value is null
constexpr int SWE_P32 = 1 << 25;     // SHP_LAYOUT_PAIRS32: e2 seq - e1 seq >= 2^32
constexpr int SWE_LEAN = 1 << 26;    // k_sw_lean handed the push to k_sw_solve (not an error)
constexpr int SWE_SPILL = 1 << 19;   // an owner's carry outgrew SWS_CCAP: it moves to k_sw_spill (re-run)
constexpr int SWE_BOUND = 1 << 30;   // a match pair names an event outside the push (a broken
                                     // invariant: the expansion skips it and the push fails)

// 16-byte record.  kt: [63:56] local key (0xFF = none), [55] carried, [54] null,
// [49:0] ts - base + 2^49.  ref: batch index (events) or carry slot (carried).
struct __attribute__((aligned(16))) SwRec {
  uint64_t kt;
  uint32_t ref;
  uint32_t v;
};

// 12-byte record (round 5) for pushes the lean solve takes (one stream column, no nulls): kt = local
// key << 24 | e1's filter << 23 | ts - base (23 bits, signed).  A push whose ts leave base +- 2^22 ms
// raises the scatter's overflow flag (D.tsmax[1] bit 1) and re-runs with the 16-byte records.
struct SwRec12 {
  uint32_t kt;
  uint32_t ref;
  uint32_t v;
};
constexpr int64_t SW_R12_SPAN = 1ll << 22;
__device__ __forceinline__ uint32_t sw_rec_lk(const SwRec& r) { return (uint32_t)(r.kt >> 56); }
__device__ __forceinline__ int32_t sw_rec_ts32(const SwRec& r) { return (int32_t)(uint32_t)r.kt; }
__device__ __forceinline__ bool sw_rec_f1(const SwRec& r) { return (r.kt & (1ull << 53)) != 0; }
__device__ __forceinline__ uint32_t sw_rec_lk(const SwRec12& r) { return r.kt >> 24; }
__device__ __forceinline__ int32_t sw_rec_ts32(const SwRec12& r) { return ((int32_t)(r.kt << 9)) >> 9; }
__device__ __forceinline__ bool sw_rec_f1(const SwRec12& r) { return ((r.kt >> 23) & 1u) != 0; }
// a record held in registers across a loop: the 12-byte form in a 4-register tuple, so a prefetch
// lands where the loop reads it (a 3-register load result copied into the loop's tuple waited for
// the load: tools/isa_check.py)
template <class R>
struct SwRecReg {
  using T = R;
  static __device__ __forceinline__ T load(const R* p, int64_t i) { return p[i]; }
};
struct __attribute__((aligned(16))) SwRec12R {
  uint32_t kt, ref, v, pad;
};
template <>
struct SwRecReg<SwRec12> {
  using T = SwRec12R;
  static __device__ __forceinline__ T load(const SwRec12* p, int64_t i) {
    T t;
    t.kt = p[i].kt;
    t.ref = p[i].ref;
    t.v = p[i].v;
    t.pad = 0;
    return t;
  }
};
__device__ __forceinline__ uint32_t sw_rec_lk(const SwRec12R& r) { return r.kt >> 24; }
__device__ __forceinline__ int32_t sw_rec_ts32(const SwRec12R& r) { return ((int32_t)(r.kt << 9)) >> 9; }
__device__ __forceinline__ bool sw_rec_f1(const SwRec12R& r) { return ((r.kt >> 23) & 1u) != 0; }

constexpr uint64_t SW_TSBIAS = 1ull << 49;
constexpr uint64_t SW_TSMASK = (1ull << 50) - 1;
constexpr uint64_t SW_CARRIED = 1ull << 55;
constexpr uint64_t SW_NULL = 1ull << 54;
constexpr uint64_t SW_F1 = 1ull << 53;  // the event satisfies e1's filter (evaluated by the scatter)

__device__ __forceinline__ uint32_t sw_lk(uint64_t kt) { return (uint32_t)(kt >> 56); }
__device__ __forceinline__ int64_t sw_ts(uint64_t kt) { return (int64_t)(kt & SW_TSMASK) - (int64_t)SW_TSBIAS; }
__device__ __forceinline__ uint64_t sw_kt(uint32_t lk, int64_t rel, uint64_t flags) {
  return ((uint64_t)lk << 56) | flags | ((uint64_t)(rel + (int64_t)SW_TSBIAS) & SW_TSMASK);
}
__device__ __forceinline__ bool sw_rel_ok(int64_t rel) {
  return rel >= -(int64_t)SW_TSBIAS && rel < (int64_t)SW_TSBIAS;
}

struct SwTerm {
  int32_t mask;  // outcomes that make the term true: 1 A<B, 2 A==B, 4 A>B, 8 unordered (NaN)
  int8_t ak, bk; // operand kind: 0 const, 1 e1.v, 2 e2.v
  int8_t flt;    // int column promoted to float: round through float
  int8_t pad;
  double ac, bc;
};
struct SwPred {
  int32_t n, combine;  // terms (0: no filter), 0 AND / 1 OR
  SwTerm t[2];
};

// Diagnostic build only (-DSHP_SW_STAMPS): per-owner cycle counts of the solve phases.
#ifdef SHP_SW_STAMPS
#define SW_STAMP(k)                          \
  do {                                       \
    __syncthreads();                         \
    if (tid == 0) {                          \
      uint64_t t_ = clock64();               \
      st_acc[k] += t_ - st_prev;             \
      st_prev = t_;                          \
    }                                        \
  } while (0)
#else
#define SW_STAMP(k) \
  do {              \
  } while (0)
#endif

struct SweepDev {
  SwPred f1, f2;
  int64_t within;
  int32_t vtag;  // tag of the predicate column, T_NULL when the query reads none
  int32_t fstream;
  int32_t nown, own_bits, nst, maxkeys;
  int32_t lk_bits;       // bits of the largest local key id
  int32_t maybe_null;    // some pushed batch carried a null bitmap (sticky; the carry may hold nulls)
  int64_t st_len;
  int32_t cur;           // which copy of the double-buffered per-owner state the next push reads
  int32_t f1ct;          // e1's filter in the scatter: typed compare class (1 float, 2 int; 0 generic doubles)
  int32_t r12;           // this push's records are SwRec12 (set per push by SweepState::run)
  const uint8_t* lk8;    // unused since round 4 (the local key is sw_local(key)); kept null
  int32_t lk_lds;
  uint32_t* cnt;         // nown * nst + 1: counts, scanned into off
  uint32_t* off;
  SwRec* recs;           // batch capacity, plus one record the scatter's unused lanes write
  int64_t trash;         // (that record's index)
  // per-owner state carried across pushes, double-buffered: a push reads copy `cur` and writes
  // copy cur ^ 1, and the engine flips `cur` only when the push succeeded (a failed push leaves
  // the engine's state as it was)
  int32_t* c_n[2];       // nown
  int64_t* c_ts[2];      // nown * SWS_CCAP, absolute ts
  int64_t* c_seq[2];
  uint32_t* c_v[2];
  uint8_t* c_lk[2];
  uint8_t* c_null[2];
  uint8_t* lastc[2];     // nown * SW_LK: the key's latest event opened a candidate (it is then the
                         // key's last carried candidate, still on the new-and-every list)
  unsigned long long* tsmax;  // [0] max of ts over the push, as ts ^ 2^63 (0: no event); [1] some ts
                              // lies beyond base +- 2^30 (k_sw_lean does not apply); reset per push
  // SHP_LAYOUT_AGG: selector aggregate over e2's value (1 avg, 2 sum, 3 count, 4 min, 5 max; 0 off), its
  // running per-key state (sum, count as doubles: exact integers to 2^53) and the owner-local
  // key -> partition key map for the output rows
  int32_t agg;
  int32_t p32;           // SHP_LAYOUT_PAIRS32: (e2 index in the batch, e2 seq - e1 seq) as two u32
  double* agg_s[2];      // nown * SW_LK
  double* agg_c[2];
  int32_t* inv;          // nown * SW_LK
  unsigned long long* stamps;  // diagnostic build: nown * 8 phase cycle counts (else unused)
  // spilled owners (sweep_spill.h): solved by k_sw_spill with their open candidates in HBM
  int32_t spill_on;      // some owner is spilled: the LDS solves skip spilled owners
  uint8_t* spilled[2];   // nown, double-buffered like the carry
  int32_t* sp_n[2];      // nown: the owner's carry in the pool (-1: still in the c_* arrays)
  int64_t* sp_base[2];   // nown: its segment of pool copy c
  int64_t* p_ts[2];      // the pool, per copy: ts, seq, value, local key, null
  int64_t* p_seq[2];
  uint32_t* p_v[2];
  uint8_t* p_lk[2];
  uint8_t* p_null[2];
  uint8_t* ovf;          // nown: k_sw_solve's carry overflowed for this owner in this push
  int32_t* sp_active;    // owners still spilled after a push (k_sw_spill counts them)
  int64_t* scr_base;     // nown: the owner's scratch segment for this push
  uint32_t* s_idx;       // scratch: record positions grouped by key
  int64_t* s_ts;         // scratch: per-key candidate lists
  int64_t* s_seq;
  uint32_t* s_v;
  uint8_t* s_st;
  // k_sw_win (sweep_win.h): unit tickets, per-unit look-back status, per (unit, owner) segment
  // presence masks of local keys, the initial halo of a unit and of an owner's tail (records)
  uint32_t* w_ticket;
  unsigned long long* w_stat;
  uint32_t* w_pres;
  int32_t w_halo, w_tail;
};

// Predicate terms lowered for the sweep (host, SweepState::lower): with one 4-byte column, every
// operand of a compare is a constant, e1.v or e2.v, and Java's binary numeric promotion
// (JLS 5.6.2, as CompareConditionExpressionExecutor*Float/Int/... apply it) is exact in double
// once an int operand promoted to float has been rounded to float first.  A term is therefore
// (op, A, B) over doubles; string ids compare by equality only (java_cmp's default branch).
__device__ __forceinline__ bool sw_term(const SwTerm t, double c1f, double c1i, bool n1, double c2f, double c2i,
                                        bool n2) {
  const double c1 = t.flt ? c1f : c1i, c2 = t.flt ? c2f : c2i;
  const double c12a = t.ak == 1 ? c1 : c2, c12b = t.bk == 1 ? c1 : c2;
  const double A = t.ak == 0 ? t.ac : c12a;
  const double B = t.bk == 0 ? t.bc : c12b;
  const bool nul = (t.ak == 1 && n1) || (t.ak == 2 && n2) || (t.bk == 1 && n1) || (t.bk == 2 && n2);
  // branch-free IEEE compare: gt {4}, ge {2,4}, lt {1}, le {1,2}, eq {2}, ne {1,4,8}
  const int o3 = (A < B ? 1 : 0) | (A == B ? 2 : 0) | (A > B ? 4 : 0);
  const bool r = ((o3 | (o3 == 0 ? 8 : 0)) & t.mask) != 0;
  return !nul && r;  // CompareConditionExpressionExecutor: a null operand -> false
}
// NT: number of terms (template, so the probe loop is straight-line code); AND/OR without
// short-circuit (terms have no side effects; And/OrConditionExpressionExecutor give the same value)
template <int NT>
__device__ __forceinline__ bool sw_pred(const SwPred& p, double c1f, double c1i, bool n1, double c2f, double c2i,
                                        bool n2) {
  if constexpr (NT == 0) {
    return true;
  } else if constexpr (NT == 1) {
    return sw_term(p.t[0], c1f, c1i, n1, c2f, c2i, n2);
  } else {
    const bool a = sw_term(p.t[0], c1f, c1i, n1, c2f, c2i, n2);
    const bool b = sw_term(p.t[1], c1f, c1i, n1, c2f, c2i, n2);
    return p.combine ? (a || b) : (a && b);
  }
}
// f2 in canonical form (SweepState::lower): every term is `e2.v OP B` with B a constant or e1.v,
// so B is resolved once per candidate and a probe costs one compare per term.  CT is the type
// the compares run in: 0 double (always exact, see SwTerm), 1 float (float column, constants
// exactly representable), 2 int32 (int / string-id column, integral constants in range) —
// chosen on the host where it gives the same answer as the promoted Java compare.
template <int CT> struct SwTy { using T = double; };
template <> struct SwTy<1> { using T = float; };
template <> struct SwTy<2> { using T = int32_t; };

template <int CT>
struct SwCand {
  typename SwTy<CT>::T b[2];
  bool bn[2];
};
template <class T>
__device__ __forceinline__ bool sw_cmp(int32_t mask, T A, T B) {
  const bool lt = A < B, eq = A == B, gt = A > B;
  const bool un = !(lt || eq || gt);
  return (lt & ((mask & 1) != 0)) | (eq & ((mask & 2) != 0)) | (gt & ((mask & 4) != 0)) | (un & ((mask & 8) != 0));
}
// The standard comparison masks as single compares (Java semantics: false on NaN, except !=).
// OPC 0 is the generic mask form; the solve picks OPC once per launch (uniform branch).
__host__ __device__ inline int sw_opclass(int32_t mask) {
  switch (mask) {
    case 1: return 1;   // <
    case 2: return 2;   // ==
    case 3: return 3;   // <=
    case 4: return 4;   // >
    case 6: return 5;   // >=
    case 13: return 6;  // !=
    default: return 0;
  }
}
template <int OPC, class T>
__device__ __forceinline__ bool sw_cmp_op(int32_t mask, T A, T B) {
  if constexpr (OPC == 1) return A < B;
  else if constexpr (OPC == 2) return A == B;
  else if constexpr (OPC == 3) return A <= B;
  else if constexpr (OPC == 4) return A > B;
  else if constexpr (OPC == 5) return A >= B;
  else if constexpr (OPC == 6) return !(A == B);
  else return sw_cmp(mask, A, B);
}
template <int CT>
__device__ __forceinline__ typename SwTy<CT>::T sw_val(uint32_t v, double f, double i, bool flt) {
  if constexpr (CT == 1) return __uint_as_float(v);
  else if constexpr (CT == 2) return (int32_t)v;
  else return flt ? f : i;
}
template <int NT, int CT>
__device__ __forceinline__ SwCand<CT> sw_cand(const SwPred& p, uint32_t av, double af, double ai, bool an) {
  SwCand<CT> c{};
#pragma unroll
  for (int t = 0; t < NT; t++) {
    const SwTerm& x = p.t[t];
    c.b[t] = x.bk == 0 ? (typename SwTy<CT>::T)x.bc : sw_val<CT>(av, af, ai, x.flt);
    c.bn[t] = x.bk == 1 && an;
  }
  return c;
}
template <int NT, int CT, int OPC = 0>
__device__ __forceinline__ bool sw_close(const SwPred& p, const SwCand<CT>& c, uint32_t ev, double ef, double ei,
                                         bool en) {
  if constexpr (NT == 0) {
    return true;
  } else if constexpr (NT == 1) {
    return !en & !c.bn[0] & sw_cmp_op<OPC>(p.t[0].mask, sw_val<CT>(ev, ef, ei, p.t[0].flt), c.b[0]);
  } else {
    const bool a = !en & !c.bn[0] & sw_cmp(p.t[0].mask, sw_val<CT>(ev, ef, ei, p.t[0].flt), c.b[0]);
    const bool b = !en & !c.bn[1] & sw_cmp(p.t[1].mask, sw_val<CT>(ev, ef, ei, p.t[1].flt), c.b[1]);
    return p.combine ? (a | b) : (a & b);
  }
}

// f1 in canonical form: every term is `e1.v OP constant` (typed compares as for f2)
template <int NT, int CT>
__device__ __forceinline__ bool sw_open(const SwPred& p, uint32_t v, bool n) {
  if constexpr (NT == 0) {
    return true;
  } else if constexpr (NT == 1) {
    return !n & sw_cmp(p.t[0].mask, sw_val<CT>(v, 0.0, 0.0, false), (typename SwTy<CT>::T)p.t[0].bc);
  } else {
    const bool a = !n & sw_cmp(p.t[0].mask, sw_val<CT>(v, 0.0, 0.0, false), (typename SwTy<CT>::T)p.t[0].bc);
    const bool b = !n & sw_cmp(p.t[1].mask, sw_val<CT>(v, 0.0, 0.0, false), (typename SwTy<CT>::T)p.t[1].bc);
    return p.combine ? (a | b) : (a & b);
  }
}

// the column value as the two promoted doubles (float path / exact int path)
__device__ __forceinline__ void sw_conv(uint32_t v, bool isfloat, double& f, double& i) {
  if (isfloat) {
    f = i = (double)__uint_as_float(v);
  } else {
    const int32_t x = (int32_t)v;
    f = (double)(float)x;
    i = (double)x;
  }
}

// key -> owner: the low bits of the dense dictionary id, and the local key its high bits (round 4;
// rounds 1-3 hashed the id onto the owner and looked the local key up in a table, a byte load per
// event that the 100k-key C5 took from L2).  Dictionary ids are dense (shp_dict, and k / N on rank
// k % N of a key-sharded group), so every owner gets max_keys / nown keys, one more at most.
// shp_push_batch_device callers that bring their own ids must keep them dense for speed: strided
// ids (all even, multiples of nown) put every event on a few owners, whose solves then run
// serially and overflow to the spill path -- results stay exact, throughput drops.
__host__ __device__ __forceinline__ uint32_t sw_owner(uint32_t k, int bits) {
  return bits == 0 ? 0u : (k & ((1u << bits) - 1u));
}
__host__ __device__ __forceinline__ uint32_t sw_local(uint32_t k, int bits) { return k >> bits; }

__device__ __forceinline__ uint64_t sw_match_peers(uint32_t bin, int bits, bool valid) {
  uint64_t peers = __ballot(valid);
  for (int b = 0; b < bits; b++) {
    bool bit = (bin >> b) & 1u;
    uint64_t m = __ballot(bit);
    peers &= bit ? m : ~m;
  }
  return peers;
}

__device__ __forceinline__ uint64_t sw_lanemask_lt() {
  uint32_t lane = __lane_id();
  return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// exclusive block scan of one value per thread (SW_THREADS threads); wtot: SW_WAVES words of LDS
__device__ __forceinline__ uint32_t sw_block_scan(uint32_t v, uint32_t* wtot, uint32_t& total) {
  uint32_t lane = __lane_id(), w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t y = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) wtot[w] = x;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < SW_WAVES; i++) {
    uint32_t t = wtot[i];
    pre += (uint32_t)i < w ? t : 0u;
    tot += t;
  }
  total = tot;
  __syncthreads();
  return pre + x - v;
}

// Owner histogram of the count passes in lane-banked copies (round 4): lane l adds to copy l % C of
// its owner's counters, word o * C + l % C.  With C = 32 the 32 lanes of a half-wave (the LDS
// atomic's lane group) land on 32 different banks whatever their owners -- one LDS-array cycle per
// group, where a single counter array took ~3 (random owners: SQ_LDS_BANK_CONFLICT 71 % of the
// kernel's LDS cycles).  C = SW_HCAP / nown, at most 32 (32 up to 512 owners, 16 at 1024).  The
// reduction reads copy (c + o) % C at step c, again one bank per lane.
constexpr int SW_HCAP = 16384;  // words (64 KB)
constexpr int SW_CNT_THREADS = 512;  // (two workgroups per CU with the 64 KB of copies: 16 waves)
struct SwHist {
  uint32_t* h;
  uint32_t C, sel;
  __device__ __forceinline__ SwHist(uint32_t* lds, int nown, int nthreads) : h(lds) {
    const int c = SW_HCAP / nown;
    C = c >= 32 ? 32u : (uint32_t)c;
    sel = __lane_id() & (C - 1u);
    for (int b = threadIdx.x; b < nown * (int)C / 4; b += nthreads) reinterpret_cast<uint4*>(h)[b] = make_uint4(0, 0, 0, 0);
  }
  __device__ __forceinline__ void add(uint32_t o) { atomicAdd(&h[o * C + sel], 1u); }
  __device__ __forceinline__ uint32_t total(uint32_t o) const {
    uint32_t s = 0;
    for (uint32_t c = 0; c < C; c++) s += h[o * C + ((c + o) & (C - 1u))];
    return s;
  }
};
static_assert(SW_HCAP / SW_MAXOWN >= 1, "every owner needs one counter");

// ------------------------------------------------------------------ pass 1: count
static __global__ __launch_bounds__(SW_CNT_THREADS) __attribute__((amdgpu_waves_per_eu(4))) void k_sw_count(SweepDev D, BatchView B, const int32_t* __restrict__ key,
                                                         int* err) {
  __shared__ __attribute__((aligned(16))) uint32_t hl[SW_HCAP];
  // super-tiles in reverse launch order: the workgroups that run last (three rounds of two per CU)
  // leave the first super-tiles' keys in the caches for the scatter, which starts there
  const int st = D.nst - 1 - (int)blockIdx.x;
  SwHist H(hl, D.nown, SW_CNT_THREADS);
  __syncthreads();
  const int64_t lo = (int64_t)st * D.st_len, hi = min(B.n, lo + D.st_len);
  int e = 0;
  if (!B.stream && B.partitioned && ((uintptr_t)key & 15) == 0 && (lo & 3) == 0) {
    // one stream, aligned keys: 16-byte loads, 4 in flight per thread
    constexpr int U = 4;
    const int4* k4 = (const int4*)key;
    const int64_t q0 = lo >> 2, q1 = hi >> 2;
    for (int64_t i0 = q0 + threadIdx.x; i0 < q1; i0 += (int64_t)SW_CNT_THREADS * U) {
      int4 kv[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int64_t i = i0 + (int64_t)u * SW_CNT_THREADS;
        kv[u] = i < q1 ? k4[i] : make_int4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        if (i0 + (int64_t)u * SW_CNT_THREADS >= q1) continue;
        const int32_t kq[4] = {kv[u].x, kv[u].y, kv[u].z, kv[u].w};
#pragma unroll
        for (int c = 0; c < 4; c++) {
          if (kq[c] < 0 || kq[c] >= D.maxkeys) e |= SWE_KEYS;
          else if (D.fstream == 0) H.add(sw_owner((uint32_t)kq[c], D.own_bits));
        }
      }
    }
    for (int64_t i = q1 * 4 + threadIdx.x; i < hi; i += SW_CNT_THREADS) {
      const int32_t k = key[i];
      if (k < 0 || k >= D.maxkeys) e |= SWE_KEYS;
      else if (D.fstream == 0) H.add(sw_owner((uint32_t)k, D.own_bits));
    }
  } else {
  constexpr int U = 8;  // loads of U events in flight per thread before the LDS adds
  for (int64_t i0 = lo + threadIdx.x; i0 < hi; i0 += (int64_t)SW_CNT_THREADS * U) {
    int32_t kk[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t i = i0 + (int64_t)u * SW_CNT_THREADS;
      int32_t k = -1;
      if (i < hi) {
        const int s = B.stream ? B.stream[i] : 0;
        if (s >= 0) {
          k = B.partitioned ? key[i] : 0;
          if (k < 0 || k >= D.maxkeys) {
            e |= SWE_KEYS;
            k = -1;
          } else if (s != D.fstream) {
            k = -1;
          }
        }
      }
      kk[u] = k;
    }
#pragma unroll
    for (int u = 0; u < U; u++)
      if (kk[u] >= 0) H.add(sw_owner((uint32_t)kk[u], D.own_bits));
  }
  }
  if (e) atomicOr(err, e);
  __syncthreads();
  for (int b = threadIdx.x; b < D.nown; b += SW_CNT_THREADS) D.cnt[(int64_t)b * D.nst + st] = H.total((uint32_t)b);
  if (st == 0 && threadIdx.x == 0) D.cnt[(int64_t)D.nown * D.nst] = 0;
}

// ------------------------------------------------------------------ pass 2: stable scatter by owner
// A/B: SHP_SCATTER_NOPF=1 keeps the round-start loads on every push
inline bool getenv_flag_scatter_nopf() {
  static const bool v = getenv("SHP_SCATTER_NOPF") != nullptr;
  return v;
}

// PF (one stream, no null bytes: the common push): the next round's key / ts / value are loaded
// into registers as soon as this round's are consumed, so they are in flight while this round is
// ranked and its scattered stores drain (tools/scatter_micro.hip: 1.44 -> 1.21 ms on 100M events
// over 512 owners, even at one workgroup per CU)
// STG (PF + R12 only, round 5, A/B): the round's records are placed in LDS in owner order first and
// then written out by position, so one store instruction covers whole owner runs (consecutive
// lanes, consecutive addresses) instead of 64 scattered 12-byte records.  Extra LDS: the round-local
// owner starts [nown] and the stage, SWP_ROUND x (kt, ref, v, destination) words.
template <bool PF, bool R12, bool STG = false>
static __global__ __launch_bounds__(SWP_THREADS) void k_sw_scatter(SweepDev D, BatchView B, const int32_t* __restrict__ key,
                                                           int* err) {
  static_assert(!STG || (PF && R12), "the staged scatter is built for the prefetched 12-byte form");
  // dynamic LDS: per-wave counts (then write cursors) [SWP_WAVES][nown] and the running owner
  // offsets [nown] (STG: then lofs [nown] and the stage)
  extern __shared__ uint32_t sw_dyn[];
  const int nown = D.nown;
  uint32_t* grun = sw_dyn + SWP_WAVES * nown;
  const int st = blockIdx.x;
  const uint32_t lane = __lane_id(), w = threadIdx.x >> 6;
  uint32_t* wcw = sw_dyn + w * nown;
  const uint64_t lt = sw_lanemask_lt();
  for (int b = threadIdx.x; b < nown; b += SWP_THREADS) grun[b] = D.off[(int64_t)b * D.nst + st];
  const int64_t lo = (int64_t)st * D.st_len, hi = min(B.n, lo + D.st_len);
  const int64_t base = B.n > 0 ? B.ts[0] : 0;
  const uint32_t* vcol = (const uint32_t*)B.cols[0];
  const uint8_t* ncol = B.nulls[0];
  const bool vnull = D.vtag == T_NULL, vflt = D.vtag == T_FLOAT;
  int e = 0;
  bool wide = false;  // some ts beyond base +- 2^30: the lean solve's 32-bit ts do not hold
  bool r12o = false;  // R12: some ts beyond base +- 2^22 (the 12-byte record's 23 bits)
  int64_t tmax = INT64_MIN;
  int32_t pk[PF ? SWP_SUB : 1];  // PF: the next round's raw key / ts / value
  int64_t pt[PF ? SWP_SUB : 1];
  uint32_t pv[PF ? SWP_SUB : 1];
  auto load_round = [&](int64_t r0) {
#pragma unroll
    for (int s = 0; s < (PF ? SWP_SUB : 0); s++) {
      const int64_t i = r0 + (int64_t)w * SWP_SEG + s * 64 + lane;
      pk[s] = i < hi ? (B.partitioned ? key[i] : 0) : -1;
      pt[s] = i < hi ? B.ts[i] : 0;
      pv[s] = (i < hi && vcol) ? vcol[i] : 0u;
    }
  };
  if (PF) load_round(lo);
  for (int64_t r0 = lo; r0 < hi; r0 += SWP_ROUND) {
    SwRec rec[SWP_SUB];
    uint32_t own[SWP_SUB];
    uint32_t rk[SWP_SUB], pc[SWP_SUB], ld[SWP_SUB];
    // all loads of the round first (independent, so they are in flight together), then the
    // key-map lookups, then the ranking
    int32_t kk[SWP_SUB];
#pragma unroll
    for (int s = 0; s < SWP_SUB; s++) {
      const int64_t i = r0 + (int64_t)w * SWP_SEG + s * 64 + lane;
      int32_t k = -1;
      if constexpr (PF) {
        k = pk[s];
        if (k >= D.maxkeys || D.fstream != 0) k = -1;
        rec[s].ref = (uint32_t)i;
        rec[s].kt = (uint64_t)pt[s];
        rec[s].v = pv[s];
      } else if (i < hi) {
        const int sid = B.stream ? B.stream[i] : 0;
        k = B.partitioned ? key[i] : 0;
        if (sid != D.fstream || k >= D.maxkeys) k = -1;
        rec[s].ref = (uint32_t)i;
        rec[s].kt = (uint64_t)B.ts[i];
        rec[s].v = vcol ? vcol[i] : 0u;
        if (k >= 0 && ncol && ncol[i]) k |= 0x40000000;  // null flag rides in the key for now
      }
      kk[s] = k;
    }
    if (PF && r0 + SWP_ROUND < hi) load_round(r0 + SWP_ROUND);
    for (int b = lane; b < nown; b += 64) wcw[b] = 0;
    __syncthreads();
    uint32_t lk[SWP_SUB];
#pragma unroll
    for (int s = 0; s < SWP_SUB; s++) lk[s] = kk[s] >= 0 ? sw_local((uint32_t)(kk[s] & 0x3fffffff), D.own_bits) : 0u;
#pragma unroll
    for (int s = 0; s < SWP_SUB; s++) {
      const bool valid = kk[s] >= 0;
      const uint32_t o = valid ? sw_owner((uint32_t)(kk[s] & 0x3fffffff), D.own_bits) : 0u;
      if (valid) {
        const int64_t t = (int64_t)rec[s].kt;
        tmax = max(tmax, t);
        const int64_t rel = t - base;
        if (!sw_rel_ok(rel)) e |= SWE_RANGE;
        wide |= rel >= (1ll << 30) || rel < -(1ll << 30);
        if (R12) r12o |= rel >= SW_R12_SPAN || rel < -SW_R12_SPAN;
        const bool nl = (kk[s] & 0x40000000) != 0;
        double af = 0.0, ai = 0.0;
        if (D.f1ct == 0) sw_conv(rec[s].v, vflt, af, ai);
        const bool an = vnull || nl;
        bool c1 = true;  // e1's filter: typed where the solve's is (exact for Java's promotion), else doubles
        if (D.f1ct == 1) {
          c1 = D.f1.n == 1 ? sw_open<1, 1>(D.f1, rec[s].v, an) : (D.f1.n == 2 ? sw_open<2, 1>(D.f1, rec[s].v, an) : true);
        } else if (D.f1ct == 2) {
          c1 = D.f1.n == 1 ? sw_open<1, 2>(D.f1, rec[s].v, an) : (D.f1.n == 2 ? sw_open<2, 2>(D.f1, rec[s].v, an) : true);
        } else if (D.f1.n == 1) {
          c1 = sw_term(D.f1.t[0], af, ai, an, 0.0, 0.0, true);
        } else if (D.f1.n == 2) {
          const bool x = sw_term(D.f1.t[0], af, ai, an, 0.0, 0.0, true);
          const bool y = sw_term(D.f1.t[1], af, ai, an, 0.0, 0.0, true);
          c1 = D.f1.combine ? (x || y) : (x && y);
        }
        rec[s].kt = sw_kt(lk[s], rel, (nl ? SW_NULL : 0ull) | (c1 ? SW_F1 : 0ull));
      }
      const uint64_t peers = sw_match_peers(o, D.own_bits, valid);
      rk[s] = (uint32_t)__popcll(peers & lt);
      own[s] = valid ? o : 0xffffffffu;
      pc[s] = (valid && (peers & lt) == 0) ? (uint32_t)__popcll(peers) : 0u;  // leader: group size
      ld[s] = peers ? (uint32_t)__ffsll((unsigned long long)peers) - 1u : 0u;    // leader lane
    }
    // per-wave running counts: the leaders' LDS adds of all sub-rounds issue back to back (LDS
    // keeps a wave's operations in order, so sub-round s sees s-1's add), one wait, then each
    // lane takes its leader's old count
    uint32_t old[SWP_SUB];
#pragma unroll
    for (int s = 0; s < SWP_SUB; s++) old[s] = pc[s] ? atomicAdd(&wcw[own[s]], pc[s]) : 0u;
#pragma unroll
    for (int s = 0; s < SWP_SUB; s++) rk[s] += __shfl(old[s], (int)ld[s], 64);
    __syncthreads();
    if constexpr (STG) {
      __shared__ uint32_t stg_w[SWP_WAVES];
      uint32_t* lofs = grun + nown;  // round-local start of each owner's records
      uint32_t* skt = lofs + nown;
      uint32_t* sref = skt + SWP_ROUND;
      uint32_t* sv = sref + SWP_ROUND;
      uint32_t* sdst = sv + SWP_ROUND;
      // round totals per owner (thread t: owners [t * per, t * per + per)), block exclusive scan
      const int per = (nown + SWP_THREADS - 1) / SWP_THREADS;
      const int b0 = min(nown, (int)threadIdx.x * per), b1 = min(nown, b0 + per);
      uint32_t tsum = 0;
      for (int b = b0; b < b1; b++)
#pragma unroll
        for (int ww = 0; ww < SWP_WAVES; ww++) tsum += sw_dyn[ww * nown + b];
      const uint32_t inc = dpp_incl_add(tsum, lane);
      if (lane == 63) stg_w[w] = inc;
      __syncthreads();
      uint32_t tot = 0, wpre = 0;
#pragma unroll
      for (int ww = 0; ww < SWP_WAVES; ww++) {
        const uint32_t t = stg_w[ww];
        wpre += ww < (int)w ? t : 0u;
        tot += t;
      }
      uint32_t g = wpre + inc - tsum;
      for (int b = b0; b < b1; b++) {
        lofs[b] = g;
#pragma unroll
        for (int ww = 0; ww < SWP_WAVES; ww++) {
          const uint32_t c = sw_dyn[ww * nown + b];
          sw_dyn[ww * nown + b] = g;
          g += c;
        }
      }
      __syncthreads();
#pragma unroll
      for (int s = 0; s < SWP_SUB; s++)
        if (own[s] != 0xffffffffu) {
          const uint32_t o = own[s];
          const uint32_t p = wcw[o] + rk[s];  // round-local, owner order
          skt[p] = (uint32_t)(rec[s].kt >> 56) << 24 | ((rec[s].kt & SW_F1) ? 1u << 23 : 0u) |
                   ((uint32_t)(int32_t)sw_ts(rec[s].kt) & 0x7FFFFFu);
          sref[p] = rec[s].ref;
          sv[p] = rec[s].v;
          sdst[p] = grun[o] + (p - lofs[o]);
        }
      __syncthreads();
      // a fixed store count per lane (positions past the round's records go to the trash slot), as
      // in the unstaged form, so the next round's start waits for the prefetched loads only
#pragma unroll
      for (int q = 0; q < SWP_PER_LANE_CFG; q++) {
        const uint32_t p = (uint32_t)(q * SWP_THREADS) + threadIdx.x;
        const bool ok = p < tot;
        SwRec12 r;
        r.kt = skt[p];
        r.ref = sref[p];
        r.v = sv[p];
        reinterpret_cast<SwRec12*>(D.recs)[ok ? (int64_t)sdst[p] : D.trash] = r;
      }
      for (int b = b0; b < b1; b++) grun[b] += (b + 1 < nown ? lofs[b + 1] : tot) - lofs[b];
      __syncthreads();
      continue;
    }
    for (int b = threadIdx.x; b < nown; b += SWP_THREADS) {
      uint32_t g = grun[b];
#pragma unroll
      for (int ww = 0; ww < SWP_WAVES; ww++) {
        uint32_t c = sw_dyn[ww * nown + b];
        sw_dyn[ww * nown + b] = g;
        g += c;
      }
      grun[b] = g;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < SWP_SUB; s++)
#ifdef SHP_SCATTER_DIAG  // diagnostics only: coalesced stores at the event's own index (wrong output)
      if (own[s] != 0xffffffffu) D.recs[rec[s].ref] = rec[s];
#else
    {
      // every lane stores (lanes without a record into the trash slot): a store count the same on
      // every path lets the compiler wait for the prefetched loads alone at the next round's start
      // (vmcnt(8)), not for these stores too
      const bool ok = own[s] != 0xffffffffu;
      const int64_t dst = ok ? (int64_t)wcw[ok ? own[s] : 0u] + rk[s] : D.trash;
      if constexpr (R12) {
        SwRec12 r;
        r.kt = (uint32_t)(rec[s].kt >> 56) << 24 | ((rec[s].kt & SW_F1) ? 1u << 23 : 0u) |
               ((uint32_t)(int32_t)sw_ts(rec[s].kt) & 0x7FFFFFu);
        r.ref = rec[s].ref;
        r.v = rec[s].v;
        reinterpret_cast<SwRec12*>(D.recs)[dst] = r;
      } else {
        D.recs[dst] = rec[s];
      }
    }
#endif
    __syncthreads();
  }
  if (e) atomicOr(err, e);
  if (wide || r12o) atomicOr(D.tsmax + 1, (wide ? 1ull : 0ull) | (r12o ? 2ull : 0ull));
  // running max of ts (the engine clock after the push)
  for (int d = 32; d > 0; d >>= 1) tmax = max(tmax, (int64_t)__shfl_xor((long long)tmax, d, 64));
  if (lane == 0 && tmax != INT64_MIN) atomicMax(D.tsmax, (unsigned long long)tmax ^ (1ull << 63));
}

// ------------------------------------------------------------------ pass 3: per-owner sweep
// One 512-thread workgroup per owner walks the owner's region (arrival order) in chunks of
// SWS_CHUNK records.  Per chunk, all in LDS:
//   rank     records (prefetched into registers during the previous chunk) are ranked by local
//            key with wave ballots; carried open candidates are already in key order
//   place    sorted position p -> (ts relative to the chunk base, value), key|flags, ref
//   probe    every candidate tests the next SW_PROBE events of its key unconditionally
//            (straight-line code); a loop finishes the rare longer scans
//   emit     each closing event finds its candidates (backward probe of m), a block scan gives
//            the output offsets, (e1 seq, e2 seq) pairs are written in (key, j, i) order
//   carry    still-open candidates (key order) become the next chunk's carry
#define SWM(p) S.m_[8 + (p)]
constexpr int SWS_THREADS = SWS_THREADS_CFG;
constexpr int SWS_WAVES = SWS_THREADS / 64;
constexpr int SWS_RPT = (SWS_CHUNK + SWS_THREADS - 1) / SWS_THREADS;  // prefetch slots per thread
constexpr int SWS_PER = (SWS_EMAX + SWS_THREADS - 1) / SWS_THREADS;
constexpr int SWS_WLCAP = 64 * SWS_PER;  // a wave's positions
constexpr uint32_t SW_LKF_CAR = 1u << 8, SW_LKF_NULL = 1u << 9, SW_LKF_F1 = 1u << 10, SW_LKF_NONE = 0xFFu;
constexpr int32_t SW_TS_FLOOR = -(1 << 30) - 1;  // carried ts below this are clamped (all expired)
constexpr int64_t SW_TS_SPAN = 1ll << 29;        // |event ts - chunk base| bound

// One straight-line batch of P probes for a candidate (ts a_ts, resolved values cbv) starting at
// sorted position qb of its key run ending at `end`: -2 run ended (open), -1 expired, q closing
// event, -4 unresolved.  `res` carries an earlier resolution through unchanged.
template <int NT2, int CT, int P, int OPC>
__device__ __forceinline__ int sw_probe(const int2* tv, const uint16_t* lkf, int qb, int end, int32_t a_ts, int32_t W,
                                        const SwPred& f2, const SwCand<CT>& cbv, bool vflt, bool vnull, bool maybe_null,
                                        int res) {
  int2 b[P];
  uint32_t bf[P];
#pragma unroll
  for (int d = 0; d < P; d++) {
    b[d] = tv[qb + d];
    bf[d] = 0;
  }
  if (maybe_null) {
#pragma unroll
    for (int d = 0; d < P; d++) bf[d] = lkf[qb + d];
  }
#pragma unroll
  for (int d = 0; d < P; d++) {
    double ef = 0, ei = 0;
    if constexpr (CT == 0) sw_conv((uint32_t)b[d].y, vflt, ef, ei);
    const bool inrun = qb + d < end;
    const bool expired = b[d].x - a_ts > W;
    const bool hit = sw_close<NT2, CT, OPC>(f2, cbv, (uint32_t)b[d].y, ef, ei, vnull || (bf[d] & SW_LKF_NULL) != 0);
    const int r = !inrun ? -2 : (expired ? -1 : (hit ? qb + d : -4));
    res = res == -4 ? r : res;
  }
  return res;
}

// probe call specialised on the f2 comparison (single-term f2 only; uniform branch)
#define SW_PROBE_OPC(CALL, P, ARGS)                     \
  switch (opc) {                                        \
    case 1: CALL<NT2, CT, P, 1> ARGS; break;            \
    case 2: CALL<NT2, CT, P, 2> ARGS; break;            \
    case 3: CALL<NT2, CT, P, 3> ARGS; break;            \
    case 4: CALL<NT2, CT, P, 4> ARGS; break;            \
    case 5: CALL<NT2, CT, P, 5> ARGS; break;            \
    case 6: CALL<NT2, CT, P, 6> ARGS; break;            \
    default: CALL<NT2, CT, P, 0> ARGS; break;           \
  }

struct SwSolveSmem {
  int2 tv[SWS_EMAX + 2 * SW_PROBE];   // (ts - chunk base, value) by sorted position, then sentinels
  uint16_t lkf[SWS_EMAX + 2 * SW_PROBE];  // local key | carried | null
  uint32_t ref[SWS_EMAX];             // batch index, or carry slot (carried)
  uint32_t cnt2[SWS_EMAX / 2 + 1];    // closes per position, two 16-bit counters per word
  int16_t m_[8 + SWS_EMAX + 8];       // m(p) = m_[8 + p]: >=0 closing position, -1 expired, -2 open,
                                      // -3 not a candidate (8 guard entries each side)
  uint16_t wc[SWS_WAVES][SW_LK + 1];  // per-wave record counts per key, then write cursors
  uint32_t binoff[SW_LK + 2];
  uint32_t ncar[SW_LK + 1];           // carried candidates per key
  uint16_t cstart[SW_LK + 1], fe[SW_LK + 1];  // carry index / sorted position of a key's first event
  uint64_t ckt[2][SWS_CCAP];          // carry: key | null | ts50 (batch-relative)
  uint32_t cv[2][SWS_CCAP];
  int64_t cseq[2][SWS_CCAP];
  uint8_t slow[SW_LK + 1];            // key solved by the exact sequential replay in this chunk
  uint8_t lastc[SW_LK + 1];           // the key's latest event opened a candidate (SweepDev::lastc)
  int32_t anyslow;
  uint32_t wtot[SWS_WAVES];
  unsigned long long gbase;
  union {
    uint16_t wl[SWS_WAVES * SWS_WLCAP];  // per-wave probe worklists (unresolved candidates)
    double ainit[2 * SW_LK];             // after the probe, AGG: per-key (sum, count) carried in
  };
  double aws[SWS_WAVES], awn[SWS_WAVES];  // AGG: segmented-scan wave totals
  uint32_t awf[SWS_WAVES];
  int32_t ainv[SW_LK];                    // AGG: local key -> partition key of this owner
};

// exclusive segmented block scan (head flags) of one (sum, count) pair per thread; in: the
// thread's inclusive aggregate and whether a segment starts in it; out: the sum and count the
// thread's first position continues from (0 after a segment start in an earlier thread...
// combined in order)
__device__ __forceinline__ void sw_block_segscan(double& s, double& n, bool f, double* ws, double* wn, uint32_t* wf) {
  const uint32_t lane = __lane_id(), w = threadIdx.x >> 6;
  double is = s, in = n;
  bool inf = f;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const double ys = __shfl_up(is, d, 64), yn = __shfl_up(in, d, 64);
    const int yf = __shfl_up((int)inf, d, 64);
    if (lane >= (uint32_t)d) {
      if (!inf) {
        is += ys;
        in += yn;
      }
      inf = inf || yf;
    }
  }
  double es = __shfl_up(is, 1, 64), en = __shfl_up(in, 1, 64);
  int ef = __shfl_up((int)inf, 1, 64);
  if (lane == 0) {
    es = 0;
    en = 0;
    ef = 0;
  }
  if (lane == 63) {
    ws[w] = is;
    wn[w] = in;
    wf[w] = inf ? 1u : 0u;
  }
  __syncthreads();
  double as = 0, an = 0;
  for (uint32_t i = 0; i < w; i++) {
    if (wf[i]) {
      as = ws[i];
      an = wn[i];
    } else {
      as += ws[i];
      an += wn[i];
    }
  }
  s = ef ? es : as + es;
  n = ef ? en : an + en;
}

// min / max aggregates (MinAttributeAggregatorExecutor / MaxAttributeAggregatorExecutor,
// core/query/selector/attribute/aggregator/, non-sliding: no deque): value = first value, then
// `if (value > x) value = x` (min; `<` for max).  A NaN first value therefore stays, and a NaN
// later one never replaces.  Fold state: the best non-NaN value (keeps the earlier one on ties),
// the count, and whether the first value was NaN; combining two folds is associative.
template <bool MAX>
__device__ __forceinline__ double sw_mm_best(double a, double b) {  // a folded first
  if constexpr (MAX) return a < b ? b : a;
  else return a > b ? b : a;
}
template <bool MAX>
__device__ __forceinline__ double sw_mm_ident() {
  return MAX ? -INFINITY : INFINITY;
}
// exclusive segmented block scan of one (best, count, first-NaN) fold per thread (see
// sw_block_segscan): out = the fold the thread's first position continues from
template <bool MAX>
__device__ __forceinline__ void sw_block_segscan_mm(double& m, double& n, bool& fn, bool f, double* wm, double* wn,
                                                    uint32_t* wf) {
  const uint32_t lane = __lane_id(), w = threadIdx.x >> 6;
  double im = m, in = n;
  int ifn = fn, inf = f;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const double ym = __shfl_up(im, d, 64), yn = __shfl_up(in, d, 64);
    const int yfn = __shfl_up(ifn, d, 64), yf = __shfl_up(inf, d, 64);
    if (lane >= (uint32_t)d) {
      if (!inf) {
        im = sw_mm_best<MAX>(ym, im);
        ifn = yn > 0 ? yfn : ifn;
        in = yn + in;
      }
      inf = inf || yf;
    }
  }
  double em = __shfl_up(im, 1, 64), en = __shfl_up(in, 1, 64);
  int efn = __shfl_up(ifn, 1, 64), ef = __shfl_up(inf, 1, 64);
  if (lane == 0) {
    em = sw_mm_ident<MAX>();
    en = 0;
    efn = 0;
    ef = 0;
  }
  if (lane == 63) {
    wm[w] = im;
    wn[w] = in;
    wf[w] = (inf ? 1u : 0u) | (ifn ? 2u : 0u);
  }
  __syncthreads();
  double am = sw_mm_ident<MAX>(), an = 0;
  int afn = 0;
  for (uint32_t i = 0; i < w; i++) {
    if (wf[i] & 1u) {
      am = wm[i];
      an = wn[i];
      afn = (wf[i] & 2u) != 0;
    } else {
      am = sw_mm_best<MAX>(am, wm[i]);
      afn = an > 0 ? afn : ((wf[i] & 2u) != 0);
      an += wn[i];
    }
  }
  if (ef) {
    m = em;
    n = en;
    fn = efn != 0;
  } else {
    m = sw_mm_best<MAX>(am, em);
    fn = (an > 0 ? afn : efn) != 0;
    n = an + en;
  }
}

// SHP_LAYOUT_AGG with min / max: every match a closing event q makes outputs the fold after q's
// value (adding the same value again does not change a min / max); the key's state (value: NaN
// when the first value was NaN, count) is seeded from the carry and written at each run end.
template <bool MAX>
__device__ __forceinline__ void sw_agg_minmax(SwSolveSmem& S, const SweepDev& D, const MatchOut& O, int E,
                                              const uint32_t* cq, uint32_t so, bool vflt, int o, int wr) {
  const uint32_t tid = threadIdx.x;
  auto seed = [&](uint32_t lk, double& m, double& n, bool& fn) {
    const double v = S.ainit[lk];
    n = S.ainit[SW_LK + lk];
    fn = n > 0 && v != v;
    m = (n > 0 && !fn) ? v : sw_mm_ident<MAX>();
  };
  auto fold = [&](double v, double& m, double& n, bool& fn) {
    if (n == 0) {
      fn = v != v;
      m = fn ? sw_mm_ident<MAX>() : v;
    } else if (v == v) {
      m = sw_mm_best<MAX>(m, v);
    }
  };
  double m = sw_mm_ident<MAX>(), n = 0;
  bool fn = false, tf = false;
#pragma unroll
  for (int k = 0; k < SWS_PER; k++) {
    const int q = (int)tid * SWS_PER + k;
    if (q < E) {
      const uint32_t lk = S.lkf[q] & 0xFFu;
      if ((uint32_t)q == S.binoff[lk]) {
        seed(lk, m, n, fn);
        tf = true;
      }
      if (cq[k]) {
        const double v = vflt ? (double)__uint_as_float((uint32_t)S.tv[q].y) : (double)S.tv[q].y;
        fold(v, m, n, fn);
        n += (double)cq[k];
      }
    }
  }
  sw_block_segscan_mm<MAX>(m, n, fn, tf, S.aws, S.awn, S.awf);
  const unsigned long long gb = S.gbase;
#pragma unroll
  for (int k = 0; k < SWS_PER; k++) {
    const int q = (int)tid * SWS_PER + k;
    if (q < E) {
      const uint32_t lk = S.lkf[q] & 0xFFu;
      if ((uint32_t)q == S.binoff[lk]) seed(lk, m, n, fn);
      const uint32_t c = cq[k];
      if (c) {
        const double v = vflt ? (double)__uint_as_float((uint32_t)S.tv[q].y) : (double)S.tv[q].y;
        fold(v, m, n, fn);
        n += (double)c;
        const double val = fn ? __longlong_as_double(0x7ff8000000000000ll) : m;
        const int32_t kid = S.ainv[lk];
        for (uint32_t r = 0; r < c; r++) {
          const uint64_t slot = gb + so + r;
          if (slot < (uint64_t)O.cap) {
            O.key[slot] = kid;
            O.agg[slot] = val;
          }
        }
      }
      so += c;
      if ((uint32_t)q + 1 == S.binoff[lk + 1]) {  // run end: the key's state after this chunk
        D.agg_s[wr][(int64_t)o * SW_LK + lk] = n == 0 ? 0.0 : (fn ? __longlong_as_double(0x7ff8000000000000ll) : m);
        D.agg_c[wr][(int64_t)o * SW_LK + lk] = n;
      }
    }
  }
}

template <int NW>
__device__ __forceinline__ uint32_t sw_block_scan_n(uint32_t v, uint32_t* wtot, uint32_t& total) {
  const uint32_t lane = __lane_id(), w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) wtot[w] = x;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NW; i++) {
    const uint32_t t = wtot[i];
    pre += (uint32_t)i < w ? t : 0u;
    tot += t;
  }
  total = tot;
  __syncthreads();
  return pre + x - v;
}

// Exact replay of one key's run of the chunk (one thread), for keys whose timestamps are not
// non-decreasing over [carried candidates..., events...] or lie beyond the chunk's 32-bit span.
// There the closed form does not hold: StreamPreStateProcessor.expireEvents (:326-361) expires
// the pending list only from its head while |ts - now| > within (it stops at the first live
// partial, which may keep expired ones behind it) and the new-and-every list (the candidate the
// previous event opened) whole; processAndReturn (:364-403) then tries every pending partial in
// list order without any expiry test.  The results go to the same m(p) / close counts the
// parallel probe produces (whose own results for the key are undone first), so the offsets,
// carry and emission steps need no change.
template <int NT2, int CT>
__device__ __forceinline__ void sw_seq_key(SwSolveSmem& S, int b, int cur, const BatchView& B, int64_t base, int32_t W,
                                        const SwPred& f2, bool vflt, bool vnull) {
  const int beg = (int)S.binoff[b], fe = (int)S.fe[b], end = (int)S.binoff[b + 1];
  for (int p = beg; p < end; p++) {
    const int q = SWM(p);
    if (q >= 0) atomicSub(&S.cnt2[q >> 1], 1u << ((q & 1) * 16));
  }
  auto ts_of = [&](int p) -> int64_t {  // exact, batch-relative
    const uint32_t r = S.ref[p];
    return (S.lkf[p] & SW_LKF_CAR) ? sw_ts(S.ckt[cur][r]) : B.ts[r] - base;
  };
  for (int p = beg; p < fe; p++) SWM(p) = -2;  // carried candidates: the pending list, in order
  int head = beg;
  int prevc = (fe > beg && S.lastc[b]) ? fe - 1 : -1;  // on the new-and-every list
  for (int q = fe; q < end; q++) {
    const int64_t tq = ts_of(q);
    for (int p = head; p < q; p++) {  // expireEvents: pending list from the head
      if (SWM(p) != -2) continue;
      if (p == prevc) break;
      const int64_t d = ts_of(p) - tq;
      if (d > W || d < -W) SWM(p) = -1;
      else break;
    }
    if (prevc >= 0 && SWM(prevc) == -2) {  // ... and the new-and-every list, whole
      const int64_t d = ts_of(prevc) - tq;
      if (d > W || d < -W) SWM(prevc) = -1;
    }
    const uint32_t fq = S.lkf[q];
    const uint32_t ev = (uint32_t)S.tv[q].y;
    double ef = 0, ei = 0;
    if constexpr (CT == 0) sw_conv(ev, vflt, ef, ei);
    const bool en = vnull || (fq & SW_LKF_NULL) != 0;
    for (int p = head; p < q; p++) {  // processAndReturn: every pending partial, in list order
      if (SWM(p) != -2) continue;
      const uint32_t av = (uint32_t)S.tv[p].y;
      double af = 0, ai = 0;
      if constexpr (CT == 0) sw_conv(av, vflt, af, ai);
      const bool an = vnull || (S.lkf[p] & SW_LKF_NULL) != 0;
      const SwCand<CT> c = sw_cand<NT2, CT>(f2, av, af, ai, an);
      if (sw_close<NT2, CT, 0>(f2, c, ev, ef, ei, en)) {
        SWM(p) = (int16_t)q;
        atomicAdd(&S.cnt2[q >> 1], 1u << ((q & 1) * 16));
      }
    }
    if (fq & SW_LKF_F1) {  // e1 matched: a new partial on the new-and-every list
      SWM(q) = -2;
      prevc = q;
    } else {
      SWM(q) = -3;
      prevc = -1;
    }
    while (head <= q && SWM(head) != -2) head++;
  }
}

template <int NT1, int NT2, int CT>
__global__ __launch_bounds__(SWS_THREADS, 4) void k_sw_solve(SweepDev D, BatchView B, MatchOut O, int* err) {
  __shared__ SwSolveSmem S;
  const int o = blockIdx.x;
  const uint32_t tid0 = threadIdx.x;
  const uint32_t tid = tid0, lane = __lane_id(), w = tid >> 6;
  const uint64_t lt = sw_lanemask_lt();
  const int64_t rb = D.off[(int64_t)o * D.nst], re = D.off[(int64_t)(o + 1) * D.nst];
  const int rd = D.cur, wr = D.cur ^ 1;  // double-buffered per-owner state: read rd, write wr
  if (D.spill_on && D.spilled[rd][o]) return;  // k_sw_spill solves this owner
  if (rb == re) {  // no events for this owner: its state passes through unchanged
    const int n0 = D.c_n[rd][o];
    for (int i = tid; i < n0; i += SWS_THREADS) {
      const int64_t c = (int64_t)o * SWS_CCAP + i;
      D.c_ts[wr][c] = D.c_ts[rd][c];
      D.c_seq[wr][c] = D.c_seq[rd][c];
      D.c_v[wr][c] = D.c_v[rd][c];
      D.c_lk[wr][c] = D.c_lk[rd][c];
      D.c_null[wr][c] = D.c_null[rd][c];
    }
    for (int i = tid; i < SW_LK; i += SWS_THREADS) {
      const int64_t k = (int64_t)o * SW_LK + i;
      D.lastc[wr][k] = D.lastc[rd][k];
      if (D.agg) {
        D.agg_s[wr][k] = D.agg_s[rd][k];
        D.agg_c[wr][k] = D.agg_c[rd][k];
      }
    }
    if (tid == 0) D.c_n[wr][o] = n0;
    return;
  }
  const int64_t base = B.ts[0];
  const int32_t W = (int32_t)D.within;  // <= SW_TS_SPAN = 2^29 (SweepState::shape_ok)
  const SwPred f1 = D.f1, f2 = D.f2;
  const bool vnull = D.vtag == T_NULL;
  const bool vflt = D.vtag == T_FLOAT;
  const bool maybe_null = D.maybe_null != 0;
  const int lkbits = D.lk_bits;
  const int opc = NT2 == 1 ? sw_opclass(f2.t[0].mask) : 0;
  int e = 0;
  // carry from the previous push
  int nc = D.c_n[rd][o];
  for (int i = tid; i <= SW_LK; i += SWS_THREADS) S.ncar[i] = 0;
  if (tid < 8) S.m_[tid] = -3;
  __syncthreads();
  for (int i = tid; i < nc; i += SWS_THREADS) {
    const int64_t c = (int64_t)o * SWS_CCAP + i;
    const int64_t rel = D.c_ts[rd][c] - base;
    if (!sw_rel_ok(rel)) e |= SWE_RANGE;
    S.ckt[0][i] = sw_kt(D.c_lk[rd][c], rel, D.c_null[rd][c] ? SW_NULL : 0ull);
    S.cv[0][i] = D.c_v[rd][c];
    S.cseq[0][i] = D.c_seq[rd][c];
    atomicAdd(&S.ncar[D.c_lk[rd][c]], 1u);
  }
  for (int i = tid; i < SW_LK; i += SWS_THREADS) {
    const int64_t k = (int64_t)o * SW_LK + i;
    S.lastc[i] = D.lastc[rd][k];
    if (D.agg) {  // the chunks below read and update copy wr
      D.agg_s[wr][k] = D.agg_s[rd][k];
      D.agg_c[wr][k] = D.agg_c[rd][k];
    }
  }
  if (D.agg)
    for (int i = tid; i < SW_LK; i += SWS_THREADS) S.ainv[i] = D.inv[(int64_t)o * SW_LK + i];
  int cur = 0;
  // prefetch chunk 0: record j of a chunk = w * (64 * SWS_RPT) + s * 64 + lane
  SwRec pf[SWS_RPT];
#pragma unroll
  for (int s = 0; s < SWS_RPT; s++) {
    const int jj = (int)w * (64 * SWS_RPT) + s * 64 + (int)lane;
    const int64_t j = rb + jj;
    if (jj < SWS_CHUNK && j < re) pf[s] = D.recs[j];
  }
  uint64_t tbk = D.recs[rb].kt;
  for (int i = tid; i < SWS_WAVES * (SW_LK + 1); i += SWS_THREADS) (&S.wc[0][0])[i] = 0;
  __syncthreads();
#ifdef SHP_SW_STAMPS
  unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t st_prev = clock64();
  unsigned long long dbg_steps = 0, dbg_cands = 0, dbg_chunks = 0, dbg_nc = 0;
  __shared__ unsigned long long dbg_sum[2];
  if (tid == 0) dbg_sum[0] = dbg_sum[1] = 0;
#endif
  for (int64_t cb = rb; cb < re; cb += SWS_CHUNK) {
    uint32_t tid_o = tid0;
    asm volatile("" : "+v"(tid_o));  // keep per-thread LDS addresses out of loop-invariant registers
    const uint32_t tid = tid_o, lane = tid_o & 63u, w = __builtin_amdgcn_readfirstlane(tid_o >> 6);
    const int nchunk = (int)min((int64_t)SWS_CHUNK, re - cb);
    const int E = nc + nchunk;
    const int64_t tb = sw_ts(tbk);  // chunk base: batch-relative ts of the chunk's first record
#ifdef SHP_SW_STAMPS
    dbg_chunks++;
    dbg_nc += nc;
#endif
    // 1. rank the chunk's records by local key (stable: wave-major, then sub-round, then lane);
    //    S.wc was zeroed during the previous chunk's probe (or before the first chunk)
    for (int i = tid; i <= SW_LK; i += SWS_THREADS) S.slow[i] = 0;
    if (tid == 0) S.anyslow = 0;
    uint32_t rk[SWS_RPT], bin[SWS_RPT];
    const uint32_t nonebin = lkbits >= 8 ? SW_LKF_NONE : (1u << lkbits);
    const int rbits = lkbits >= 8 ? 8 : lkbits + 1;
#pragma unroll
    for (int s = 0; s < SWS_RPT; s++) {
      const int j = (int)w * (64 * SWS_RPT) + s * 64 + (int)lane;
      const uint32_t bn = j < nchunk ? sw_lk(pf[s].kt) : nonebin;
      bin[s] = bn;
      const uint64_t peers = sw_match_peers(bn, rbits, true);
      const uint32_t before = S.wc[w][bn];
      rk[s] = before + (uint32_t)__popcll(peers & lt);
      if ((peers & lt) == 0) S.wc[w][bn] = (uint16_t)(before + (uint32_t)__popcll(peers));
    }
    __syncthreads();
    {  // key offsets (carried first within each key), per-wave write cursors
      const uint32_t b = tid;
      uint32_t c[SWS_WAVES], t = 0, nk = 0;
      if (b <= (uint32_t)SW_LK && b != nonebin) {
        nk = S.ncar[b];
#pragma unroll
        for (int ww = 0; ww < SWS_WAVES; ww++) {
          c[ww] = S.wc[ww][b];
          t += c[ww];
        }
      }
      uint32_t total;
      const uint32_t pre = sw_block_scan_n<SWS_WAVES>(((t + nk) << 16) | nk, S.wtot, total);
      if (b <= (uint32_t)SW_LK && b != nonebin) {
        uint32_t g = (pre >> 16) + nk;
        S.binoff[b] = pre >> 16;
        S.cstart[b] = (uint16_t)(pre & 0xffffu);
        S.fe[b] = (uint16_t)((pre >> 16) + nk);
#pragma unroll
        for (int ww = 0; ww < SWS_WAVES; ww++) {
          S.wc[ww][b] = (uint16_t)g;
          g += c[ww];
        }
      }
      if (b <= (uint32_t)SW_LK && b == nonebin) {
        S.binoff[b] = pre >> 16;
        S.cstart[b] = (uint16_t)(pre & 0xffffu);
        S.fe[b] = (uint16_t)(pre >> 16);
      }
      if (tid == 0) S.binoff[SW_LK + 1] = total >> 16;
    }
    __syncthreads();
    // 2. place records and carried candidates by sorted position
#pragma unroll
    for (int s = 0; s < SWS_RPT; s++) {
      if (bin[s] == nonebin) continue;
      const uint32_t p = S.wc[w][bin[s]] + rk[s];
      int64_t rel = sw_ts(pf[s].kt) - tb;
      if (rel >= SW_TS_SPAN || rel <= -SW_TS_SPAN) {  // beyond the 32-bit probe: exact replay
        S.slow[bin[s]] = 1;
        S.anyslow = 1;
        rel = rel > 0 ? SW_TS_SPAN : -SW_TS_SPAN;
      }
      S.tv[p] = make_int2((int32_t)rel, (int32_t)pf[s].v);
      S.lkf[p] = (uint16_t)(bin[s] | ((pf[s].kt & SW_NULL) ? SW_LKF_NULL : 0u) | ((pf[s].kt & SW_F1) ? SW_LKF_F1 : 0u));
      S.ref[p] = pf[s].ref;
    }
    for (int x = tid; x < nc; x += SWS_THREADS) {
      const uint64_t kt = S.ckt[cur][x];
      const uint32_t lk = sw_lk(kt);
      const uint32_t p = S.binoff[lk] + (uint32_t)x - S.cstart[lk];
      const int64_t rel = sw_ts(kt) - tb;
      if (rel > SW_TS_SPAN) {  // a carried candidate later than the chunk's span: exact replay
        S.slow[lk] = 1;
        S.anyslow = 1;
      }
      const int64_t crel = rel < SW_TS_FLOOR ? SW_TS_FLOOR : (rel > SW_TS_SPAN ? SW_TS_SPAN : rel);
      S.tv[p] = make_int2((int32_t)crel, (int32_t)S.cv[cur][x]);
      S.lkf[p] = (uint16_t)(lk | SW_LKF_CAR | ((kt & SW_NULL) ? SW_LKF_NULL : 0u));
      S.ref[p] = (uint32_t)x;
    }
    if (tid < 2 * SW_PROBE) {
      S.tv[E + tid] = make_int2(0, 0);
      S.lkf[E + tid] = (uint16_t)SW_LKF_NONE;
    }
    if (tid < 8) SWM(E + tid) = -3;
    for (int i = tid; i <= SWS_EMAX / 2; i += SWS_THREADS) S.cnt2[i] = 0;
    // prefetch the next chunk while this one is solved
    {
      const int64_t nb = cb + SWS_CHUNK;
#pragma unroll
      for (int s = 0; s < SWS_RPT; s++) {
        const int jj = (int)w * (64 * SWS_RPT) + s * 64 + (int)lane;
        const int64_t j = nb + jj;
        if (jj < SWS_CHUNK && j < re) pf[s] = D.recs[j];
      }
      if (nb < re) tbk = D.recs[nb].kt;
    }
    __syncthreads();
    SW_STAMP(0);
    // 3. probe.  Round 1: every position tests whether it is a candidate and probes the first
    //    SW_P1 events of its key (straight-line code, no per-lane loop).  Candidates still
    //    unresolved go to a worklist; each later round gives every worklist entry SW_P2 more
    //    events, so lanes stay busy on the few long scans instead of idling in divergent loops.
    for (int i = tid; i < SWS_WAVES * (SW_LK + 1); i += SWS_THREADS) (&S.wc[0][0])[i] = 0;  // next rank
    uint16_t* wlw = S.wl + w * SWS_WLCAP;  // this wave's worklist
    uint32_t nwl = 0;                      // wave-uniform (ballot counts)
    for (int k = 0; k < SWS_PER; k++) {
      if ((int)(w * 64) + k * SWS_THREADS >= E) break;  // wave-uniform
      const int p = (int)tid + k * SWS_THREADS;
      int res = -3;
      if (p < E) {
        const uint32_t f = S.lkf[p];
        const int2 a = S.tv[p];
        const bool an = vnull || (f & SW_LKF_NULL) != 0;
        double af = 0, ai = 0;
        if constexpr (CT == 0) sw_conv((uint32_t)a.y, vflt, af, ai);
        const bool cand = (f & (SW_LKF_CAR | SW_LKF_F1)) != 0;  // carried, or e1's filter (scatter)
        const uint32_t lk = f & 0xFFu;
        const int end = (int)S.binoff[lk + 1];
        // the closed form needs non-decreasing ts over the key's [carried..., events...]
#ifndef SHP_AB_NOSLOW
        if (p > (int)S.binoff[lk] && S.tv[p - 1].x > a.x) {
          S.slow[lk] = 1;
          S.anyslow = 1;
        }
#endif
        const int q0 = max(p + 1, (int)S.fe[lk]);  // carried candidates are not events
        const SwCand<CT> cbv = sw_cand<NT2, CT>(f2, (uint32_t)a.y, af, ai, an);
        res = cand ? -4 : -3;  // -4: unresolved
        SW_PROBE_OPC(res = sw_probe, SW_P1, (S.tv, S.lkf, q0, end, a.x, W, f2, cbv, vflt, vnull, maybe_null, res));
      }
      const bool unres = res == -4;
      const uint64_t um = __ballot(unres);
      if (unres) {
        wlw[nwl + (uint32_t)__popcll(um & lt)] = (uint16_t)p;
      } else if (p < E) {
        SWM(p) = (int16_t)res;
        if (res >= 0) atomicAdd(&S.cnt2[res >> 1], 1u << ((res & 1) * 16));
      }
      nwl += (uint32_t)__popcll(um);
    }
    // Later rounds, per wave (no block barrier): every worklist entry gets SW_P2 more events;
    // still-unresolved entries are compacted in place (an entry moves only to a lower index,
    // already read: the wave's LDS operations complete in order)
    for (int round = 0; nwl > 0; round++) {
      uint32_t nn = 0;
      for (uint32_t b0 = 0; b0 < nwl; b0 += 64) {
        const uint32_t idx = b0 + lane;
        int p = 0, res = -3;
        if (idx < nwl) {
          p = (int)wlw[idx];
          const uint32_t f = S.lkf[p];
          const int2 a = S.tv[p];
          const bool an = vnull || (f & SW_LKF_NULL) != 0;
          double af = 0, ai = 0;
          if constexpr (CT == 0) sw_conv((uint32_t)a.y, vflt, af, ai);
          const uint32_t lk = f & 0xFFu;
          const int end = (int)S.binoff[lk + 1];
          const int qn = max(p + 1, (int)S.fe[lk]) + SW_P1 + round * SW_P2;
          const SwCand<CT> cbv = sw_cand<NT2, CT>(f2, (uint32_t)a.y, af, ai, an);
          SW_PROBE_OPC(res = sw_probe, SW_P2, (S.tv, S.lkf, qn, end, a.x, W, f2, cbv, vflt, vnull, maybe_null, -4));
          if (res == -4 && qn + SW_P2 >= end) res = -2;  // key run exhausted: still open
        }
        const bool unres = res == -4;
        const uint64_t um = __ballot(unres);
        if (unres) {
          wlw[nn + (uint32_t)__popcll(um & lt)] = (uint16_t)p;
        } else if (idx < nwl) {
          SWM(p) = (int16_t)res;
          if (res >= 0) atomicAdd(&S.cnt2[res >> 1], 1u << ((res & 1) * 16));
        }
        nn += (uint32_t)__popcll(um);
      }
      nwl = nn;
#ifdef SHP_SW_STAMPS
      if (lane == 0) {
        dbg_steps += nwl;
        dbg_cands++;
      }
#endif
    }
    __syncthreads();
    if (S.anyslow) {  // rare: keys the closed form does not cover, replayed exactly
      for (int b = tid; b < (int)min(nonebin, (uint32_t)SW_LK); b += SWS_THREADS)
        if (S.slow[b]) sw_seq_key<NT2, CT>(S, b, cur, B, base, W, f2, vflt, vnull);
      __syncthreads();
    }
    SW_STAMP(1);
    // 4. one block scan gives both the output offsets (closes per closing event, counted by the
    //    probe; 16-bit, in place of the counts) and the carry slots of still-open candidates
    //    (packed: closes << 16 | opens; both totals are at most E)
    uint16_t* off16 = reinterpret_cast<uint16_t*>(S.cnt2);
    const int nx = cur ^ 1;
    {
      uint32_t cq[SWS_PER], tot = 0, open = 0;
#pragma unroll
      for (int k = 0; k < SWS_PER; k++) {
        const int q = (int)tid * SWS_PER + k;
        cq[k] = q < E ? off16[q] : 0u;
        tot += cq[k];
        open += (q < E && SWM(q) == -2) ? 1u : 0u;
      }
      for (int i = tid; i <= SW_LK; i += SWS_THREADS) S.ncar[i] = 0;  // recounted below
      if (D.agg) {  // per-key aggregate state carried in (read before any run end rewrites it)
        for (int b = tid; b < (int)min(nonebin, (uint32_t)SW_LK); b += SWS_THREADS) {
          S.ainit[b] = D.agg_s[wr][(int64_t)o * SW_LK + b];
          S.ainit[SW_LK + b] = D.agg_c[wr][(int64_t)o * SW_LK + b];
        }
      }
      uint32_t total;
      const uint32_t pk = sw_block_scan_n<SWS_WAVES>((tot << 16) | open, S.wtot, total);
      uint32_t off = pk >> 16, pre = pk & 0xffffu;
      const uint32_t ctot = total >> 16;
      uint32_t ntot = total & 0xffffu;
#pragma unroll
      for (int k = 0; k < SWS_PER; k++) {
        const int q = (int)tid * SWS_PER + k;
        if (q < E) off16[q] = (uint16_t)off;
        off += cq[k];
      }
      if (tid == 0) {
        off16[E] = (uint16_t)ctot;
        const unsigned long long g = ctot ? atomicAdd(O.count, (unsigned long long)ctot) : 0ull;
        if (g + ctot > (unsigned long long)O.cap) e |= E_OUT;
        S.gbase = g;
      }
      if (D.agg >= 4) {
        if (D.agg == 4) sw_agg_minmax<false>(S, D, O, E, cq, pk >> 16, vflt, o, wr);
        else sw_agg_minmax<true>(S, D, O, E, cq, pk >> 16, vflt, o, wr);
        for (int k = 0; k < SWS_PER; k++) {
          const int q = (int)tid * SWS_PER + k;
          if (q < E && cq[k] && ((S.lkf[q] & SW_LKF_NULL) || vnull)) e |= SWE_AGGNULL;
        }
      } else if (D.agg) {
        // SHP_LAYOUT_AGG: the selector's running aggregate per match, in place of the pairs.
        // Per closing event q (c closes, value v): the r-th match adds v once more, so its
        // output is (S + (r+1) v) / (N + r + 1) for avg, where (S, N) is the key's state before
        // q: a segmented scan over positions (key runs) seeded with the carried-in state.
        double ts_ = 0, tn_ = 0;
        bool tf = false;
#pragma unroll
        for (int k = 0; k < SWS_PER; k++) {
          const int q = (int)tid * SWS_PER + k;
          if (q < E) {
            const uint32_t f = S.lkf[q];
            const uint32_t lk = f & 0xFFu;
            const double v = vflt ? (double)__uint_as_float((uint32_t)S.tv[q].y) : (double)S.tv[q].y;
            if (cq[k] && ((f & SW_LKF_NULL) || vnull)) e |= SWE_AGGNULL;
            if ((uint32_t)q == S.binoff[lk]) {
              ts_ = S.ainit[lk];
              tn_ = S.ainit[SW_LK + lk];
              tf = true;
            }
            ts_ += (double)cq[k] * v;
            tn_ += (double)cq[k];
          }
        }
        sw_block_segscan(ts_, tn_, tf, S.aws, S.awn, S.awf);
        const unsigned long long gb = S.gbase;
        uint32_t so = pk >> 16;
        double ps = ts_, pn = tn_;
#pragma unroll
        for (int k = 0; k < SWS_PER; k++) {
          const int q = (int)tid * SWS_PER + k;
          if (q < E) {
            const uint32_t f = S.lkf[q];
            const uint32_t lk = f & 0xFFu;
            const double v = vflt ? (double)__uint_as_float((uint32_t)S.tv[q].y) : (double)S.tv[q].y;
            if ((uint32_t)q == S.binoff[lk]) {
              ps = S.ainit[lk];
              pn = S.ainit[SW_LK + lk];
            }
            const uint32_t c = cq[k];
            if (c) {
              const int32_t kid = S.ainv[lk];
              for (uint32_t r = 0; r < c; r++) {
                const double sr = ps + (double)(r + 1) * v, nr = pn + (double)(r + 1);
                const double val = D.agg == 1 ? sr / nr : (D.agg == 2 ? sr : nr);
                const uint64_t slot = gb + so + r;
                if (slot < (uint64_t)O.cap) {
                  O.key[slot] = kid;
                  O.agg[slot] = val;
                }
              }
            }
            ps += (double)c * v;
            pn += (double)c;
            so += c;
            if ((uint32_t)q + 1 == S.binoff[lk + 1]) {  // run end: the key's state after this chunk
              D.agg_s[wr][(int64_t)o * SW_LK + lk] = ps;
              D.agg_c[wr][(int64_t)o * SW_LK + lk] = pn;
            }
          }
        }
      }
      // 5. still-open candidates become the next carry (sorted order = key, then i); a key whose
      //    latest event opened a candidate has it on the new-and-every list (sw_seq_key)
      for (int b = tid; b < (int)min(nonebin, (uint32_t)SW_LK); b += SWS_THREADS) {
        const int fe = (int)S.fe[b], end = (int)S.binoff[b + 1];
        if (fe < end) S.lastc[b] = (S.lkf[end - 1] & SW_LKF_F1) ? 1 : 0;
      }
#pragma unroll
      for (int k = 0; k < SWS_PER; k++) {
        const int p = (int)tid * SWS_PER + k;
        if (p < E && SWM(p) == -2) {
          if (pre < (uint32_t)SWS_CCAP) {
            const uint32_t f = S.lkf[p];
            const uint32_t r = S.ref[p];
            const uint32_t lk = f & 0xFFu;
            if (f & SW_LKF_CAR) {
              S.ckt[nx][pre] = S.ckt[cur][r];
              S.cv[nx][pre] = S.cv[cur][r];
              S.cseq[nx][pre] = S.cseq[cur][r];
            } else {
              // a slow key's tv.x may be clamped to the chunk span: take the exact ts instead
              const int64_t ts = S.slow[lk] ? B.ts[r] - base : tb + S.tv[p].x;
              S.ckt[nx][pre] = sw_kt(lk, ts, (f & SW_LKF_NULL) ? SW_NULL : 0ull);
              S.cv[nx][pre] = (uint32_t)S.tv[p].y;
              S.cseq[nx][pre] = bseq(B, r);
            }
            atomicAdd(&S.ncar[lk], 1u);
          }
          pre++;
        }
      }
      if (ntot > (uint32_t)SWS_CCAP) {  // the owner moves to k_sw_spill (the push re-runs)
        e |= SWE_SPILL;
        if (tid == 0) D.ovf[o] = 1;
        ntot = SWS_CCAP;
      }
      nc = (int)ntot;
    }
    __syncthreads();
    SW_STAMP(2);
    // 6. every matched candidate writes its own pair: its slot among the candidates of its
    //    closing event q is fixed by how many later candidates q also closed.  No barrier after
    //    it: the next chunk's rank step touches only S.wc, and its first barrier comes before
    //    anything this step reads is rewritten.
    if (!D.agg) {
      const unsigned long long gb = S.gbase;
      for (int k = 0; k < SWS_PER; k++) {
        const int p = (int)tid + k * SWS_THREADS;
        if (p >= E) break;
        const int q = SWM(p);
        if (q < 0) continue;
        const uint32_t c = (uint32_t)off16[q + 1] - off16[q];
        // the next SW_PROBE entries are read unconditionally (guard entries past E), so the
        // reads issue back to back instead of one branch and wait per entry
        int16_t mm[SW_PROBE];
#pragma unroll
        for (int d = 0; d < SW_PROBE; d++) mm[d] = SWM(p + 1 + d);
        uint32_t later = 0;
#pragma unroll
        for (int d = 0; d < SW_PROBE; d++) later += ((p + 1 + d < q) & (mm[d] == q)) ? 1u : 0u;
        for (int p2 = p + SW_PROBE + 1; p2 < q; p2++) later += SWM(p2) == q ? 1u : 0u;
        const uint32_t r = S.ref[p];
        const int64_t si = (S.lkf[p] & SW_LKF_CAR) ? S.cseq[cur][r] : bseq(B, r);
        const int64_t sq = bseq(B, S.ref[q]);
        const uint64_t slot = gb + off16[q] + (c - 1 - later);
        if (slot < (uint64_t)O.cap) {
          if (D.p32) {
            const int64_t dq = sq - si;  // >= 1
            if (dq >= (1ll << 32)) e |= SWE_P32;
            reinterpret_cast<uint2*>(O.refs)[slot] = make_uint2(S.ref[q], (uint32_t)dq);
          } else if (B.seq) {  // a seq column: keep e2's batch index for k_sw_expand (FULL layout)
            *(longlong2*)(O.refs + 2 * slot) = make_longlong2(si, (int64_t)S.ref[q]);
          } else {
            *(longlong2*)(O.refs + 2 * slot) = make_longlong2(si, sq);
          }
        }
      }
    }
    cur = nx;
    SW_STAMP(3);
    SW_STAMP(4);
    SW_STAMP(5);
    SW_STAMP(6);
    SW_STAMP(7);
  }
  __syncthreads();
#ifdef SHP_SW_STAMPS
  atomicAdd(&dbg_sum[0], dbg_steps);
  atomicAdd(&dbg_sum[1], dbg_cands);
  __syncthreads();
  if (tid == 0 && D.stamps) {
    for (int k = 0; k < 6; k++) D.stamps[(int64_t)o * 8 + k] = st_acc[k];
    D.stamps[(int64_t)o * 8 + 7] = (dbg_sum[0] << 24) | (dbg_sum[1] & 0xffffff);
    D.stamps[(int64_t)o * 8 + 6] = (dbg_chunks << 40) | (dbg_nc & 0xffffffffffull);
  }
#endif
  // write back the carry and the per-key flags (copy wr)
  for (int i = tid; i < nc; i += SWS_THREADS) {
    const int64_t c = (int64_t)o * SWS_CCAP + i;
    const uint64_t kt = S.ckt[cur][i];
    D.c_ts[wr][c] = base + sw_ts(kt);
    D.c_seq[wr][c] = S.cseq[cur][i];
    D.c_v[wr][c] = S.cv[cur][i];
    D.c_lk[wr][c] = (uint8_t)sw_lk(kt);
    D.c_null[wr][c] = (kt & SW_NULL) ? 1 : 0;
  }
  for (int i = tid; i < SW_LK; i += SWS_THREADS) D.lastc[wr][(int64_t)o * SW_LK + i] = S.lastc[i];
  if (tid == 0) D.c_n[wr][o] = nc;
  if (e) atomicOr(err, e);
}

// full match records from the (i, j) pairs (shp_push_batch / shp_fetch_matches).  p32: the
// pairs are SHP_LAYOUT_PAIRS32 (e2 batch index, e2 seq - e1 seq), staged by the caller in O.pos
// (8 bytes per match); thread i reads its pair before it writes O.pos[i].
//
// Round-2 fault (tests/test_lean_sweep.py::test_fallback_and_back_keeps_state_exact, "illegal
// memory access"): this kernel used to run right after a k_sw_lean push that handed back with
// SWE_LEAN.  The lean kernel had already reserved output slots (O.count) it never wrote, so the
// expansion read stale pair words as batch indices g and loaded B.ts[g] / key[g] far out of
// bounds.  Now a handed-back push is not expanded (the exact re-run expands its own output), and
// any pair whose index falls outside the push sets SWE_BOUND instead of being dereferenced.
static __global__ void k_sw_expand(BatchView B, const int32_t* __restrict__ key, MatchOut O, int p32, int* err) {
  // a push k_sw_lean handed back has reserved slots it never wrote: the exact re-run expands
  if (*err & SWE_LEAN) return;
  int bad = 0;
  const int64_t m = min((int64_t)*O.count, O.cap);
  if (blockIdx.x == 0 && threadIdx.x == 0) O.count[1] = 2ull * (unsigned long long)m;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t j, g;
    if (p32) {  // (e2's batch index, e2 seq - e1 seq)
      const uint2 pr = reinterpret_cast<const uint2*>(O.pos)[i];
      g = (int64_t)pr.x;
      if (g >= B.n) {
        bad = SWE_BOUND;
        continue;
      }
      j = bseq(B, g);
      O.refs[2 * i] = j - (int64_t)pr.y;
      O.refs[2 * i + 1] = j;
    } else if (B.seq) {  // (e1 seq, e2's batch index): the FULL layout with a seq column
      g = O.refs[2 * i + 1];
      if (g < 0 || g >= B.n) {
        bad = SWE_BOUND;
        continue;
      }
      j = B.seq[g];
      O.refs[2 * i + 1] = j;
    } else {  // (e1 seq, e2 seq)
      j = O.refs[2 * i + 1];
      g = j - B.seq0;
    }
    if (g < 0 || g >= B.n) {  // not a pair of this push (never written)
      bad = SWE_BOUND;
      continue;
    }
    O.key[i] = B.partitioned ? key[g] : 0;
    O.ts[i] = B.ts[g];
    O.type[i] = 0;
    O.pos[i] = j;
    O.ref_off[i] = 2 * i;
    O.slot_len[i * MAXS] = 1;
    O.slot_len[i * MAXS + 1] = 1;
  }
  if (bad) atomicOr(err, bad);
}

static __global__ void k_sw_init(SweepDev D) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < D.nown) D.c_n[0][i] = D.c_n[1][i] = 0;
  if (i < (int64_t)D.nown * SW_LK) D.lastc[0][i] = D.lastc[1][i] = 0;
}

}  // namespace shp

#include "sweep_lean.h"
#include "sweep_spill.h"
#include "sweep_win.h"

// ------------------------------------------------------------------ host side
namespace shp {

// The solve kernels' template instantiations live in units of their own (sweep_solve.hip, built
// once per NT1, and sweep_lean.hip), so the library's units build in parallel.
void sw_launch_solve(int nt1, int nt2, int ct, unsigned grid, hipStream_t s, const SweepDev& D, const BatchView& B,
                     const MatchOut& O, int* err);
void sw_launch_lean(int ct, int opc, unsigned grid, hipStream_t s, const SweepDev& D, const BatchView& B,
                    const MatchOut& O, int* err);
void sw_launch_lean_agg(int ct, int opc, unsigned grid, hipStream_t s, const SweepDev& D, const BatchView& B,
                        const MatchOut& O, int* err);
void sw_launch_spill(int nt2, int ct, unsigned grid, hipStream_t s, const SweepDev& D, const BatchView& B,
                     const MatchOut& O, int* err);
void sw_launch_win(int ct, int opc, unsigned grid, hipStream_t s, const SweepDev& D, const BatchView& B,
                   const MatchOut& O, int* err);
void sw_launch_win_tail(int ct, int opc, unsigned grid, hipStream_t s, const SweepDev& D, const BatchView& B,
                        int* err);

struct SweepState {
  SweepDev D{};
  int64_t pool_cap[2] = {0, 0};  // entries of each pool copy (spilled owners' carries)
  int64_t scr_cap = 0;           // entries of the spill scratch
  int64_t* sizes = nullptr;      // k_sw_spill_sizes output (3 x nown)
  int ct = 0;  // compare type of the probe loop (see SwCand)
  int lean_opc = 0;  // > 0: k_sw_lean applies to the query (its f2 comparison class)
  int64_t w_units = 0;  // k_sw_win: units the status array holds
  bool win_off = true;  // k_sw_win is opt-in: SHP_WIN=1 (tests/test_win_sweep.py, A/B)
  bool last_win = false;  // the last run() launched k_sw_win
  // events per super-tile (one scatter workgroup).  Pushes of 64M events and more take 131072: 37.6
  // against 37.3 G events/s at 65536 on C2, 29.75 against 29.6 G on C5 (fewer tiles, a smaller count
  // pass and scan; profiles/r06_stlen_ab.txt).  Smaller pushes keep 65536, which is also the
  // allocation's granularity: at 12.5M events 131072 leaves 95 workgroups for 256 CUs (scatter 0.20 ->
  // 0.34 ms).  SHP_SW_STLEN sets both, for diagnostics.
  int64_t st_len = 65536;
  int64_t st_len_big = 131072;
  int32_t nst_max = 1;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;

  static uint32_t hash32(uint32_t x) {  // murmur3 finaliser
    x ^= x >> 16;
    x *= 0x85ebca6bu;
    x ^= x >> 13;
    x *= 0xc2b2ae35u;
    x ^= x >> 16;
    return x;
  }

  // Is the program a sweep shape? One 4-byte predicate column (int / float / string id) or none,
  // filters over slot 0/1 attributes of that column only, lowerable to SwPred.
  static bool shape_ok(const DevProg& P, const FastShape& f) {
    // `within` must fit the probe's 32-bit chunk-relative timestamps (and the carried-candidate
    // floor, SW_TS_FLOOR): longer windows take the scan kernels (64-bit timestamps)
    if (!f.ok || P.ncol > 1 || f.within > SW_TS_SPAN) return false;
    if (P.ncol == 1 && !(P.colTag[0] == T_INT || P.colTag[0] == T_FLOAT || P.colTag[0] == T_STR)) return false;
    SwPred a, b;
    int8_t vt = P.ncol == 1 ? P.colTag[0] : T_NULL;
    return lower(f.f1, vt, a) && lower(f.f2, vt, b) && canonical_e2(b);
  }

  static bool lower_operand(const FOperand& o, int8_t ptype, int8_t vtag, int8_t& kind, double& c) {
    kind = 0;
    c = 0;
    if (o.kind == 1) {
      if (o.pos != 0 || vtag == T_NULL) return false;
      kind = (int8_t)(o.state + 1);
      return o.state == 0 || o.state == 1;
    }
    switch (o.tag) {
      case T_INT: {
        int32_t x = (int32_t)o.imm;
        c = ptype == T_FLOAT ? (double)(float)x : (double)x;
        return true;
      }
      case T_LONG: {
        // exact against 32-bit column values whatever the rounding, unless equal-compared
        // beyond 2^53 (left to the scan path)
        if (o.imm > (1ll << 53) || o.imm < -(1ll << 53)) return false;
        c = ptype == T_FLOAT ? (double)(float)o.imm : (double)o.imm;
        return true;
      }
      case T_FLOAT: {
        uint32_t u = (uint32_t)o.imm;
        float f;
        memcpy(&f, &u, 4);
        c = (double)f;
        return true;
      }
      case T_DOUBLE: memcpy(&c, &o.imm, 8); return true;
      case T_STR: c = (double)(int32_t)o.imm; return true;
      default: return false;
    }
  }

  // narrowest compare type that is exact for every term of the canonical f2 (see SwCand)
  static int compare_type(const SwPred& p, int8_t vtag) {
    bool f = vtag == T_FLOAT, i = vtag == T_INT || vtag == T_STR;
    for (int k = 0; k < p.n; k++) {
      const SwTerm& t = p.t[k];
      if (t.bk == 0) {
        double c = t.bc;
        if (f && !(c != c) && (double)(float)c != c) f = false;
        if (i && !(c >= -2147483648.0 && c <= 2147483647.0 && c == std::floor(c))) i = false;
      }
      if (t.flt) i = false;
    }
    return f ? 1 : (i ? 2 : 0);
  }

  // f1 as `e1.v OP constant` terms (needed for the typed compare paths)
  static bool canonical_e1(SwPred& p) {
    for (int i = 0; i < p.n; i++) {
      SwTerm& t = p.t[i];
      if (t.ak == 0 && t.bk == 1) {
        std::swap(t.ak, t.bk);
        std::swap(t.ac, t.bc);
        t.mask = (t.mask & 0xA) | ((t.mask & 1) << 2) | ((t.mask & 4) >> 2);
      }
      if (!(t.ak == 1 && t.bk == 0)) return false;
    }
    return true;
  }

  // rewrite every term of f2 as `e2.v OP B` (B const or e1.v), mirroring the operator on a swap
  static bool canonical_e2(SwPred& p) {
    for (int i = 0; i < p.n; i++) {
      SwTerm& t = p.t[i];
      if (t.ak != 2 && t.bk == 2) {
        std::swap(t.ak, t.bk);
        std::swap(t.ac, t.bc);
        t.mask = (t.mask & 0xA) | ((t.mask & 1) << 2) | ((t.mask & 4) >> 2);  // lt <-> gt
      }
      if (t.ak != 2 || t.bk == 2) return false;
    }
    return true;
  }

  static bool lower(const FPred& p, int8_t vtag, SwPred& out) {
    out = SwPred{};
    out.n = p.n;
    out.combine = p.combine;
    for (int i = 0; i < p.n; i++) {
      const FTerm& t = p.t[i];
      SwTerm& o = out.t[i];
      if (t.ptype == T_BOOL || t.ptype == T_NULL) return false;
      if (t.a.kind == 0 && t.b.kind == 0) return false;
      static const int32_t masks[6] = {4, 6, 1, 3, 2, 13};  // gt ge lt le eq ne
      // string ids (java_cmp's default branch): == for eq, != for every other operator
      o.mask = t.ptype == T_STR ? (t.cmp == 4 ? 2 : 13) : masks[t.cmp < 6 ? t.cmp : 5];
      o.flt = vtag == T_INT && t.ptype == T_FLOAT;
      if (!lower_operand(t.a, t.ptype, vtag, o.ak, o.ac) || !lower_operand(t.b, t.ptype, vtag, o.bk, o.bc))
        return false;
    }
    return true;
  }

  // host key map: key -> owner | local key << 16; false when keys cannot be spread under the caps
  static bool build_map(int32_t max_keys, int32_t& nown, std::vector<uint32_t>& kmap) {
    nown = 1;
    static const int kpo = getenv("SHP_SW_KPO") ? std::max(1, atoi(getenv("SHP_SW_KPO"))) : 20;  // diagnostics
    // about kpo keys per owner, but at most SW_PREF_OWN owners while an owner stays under
    // ~200 keys: fewer, longer per-owner runs per scatter round (full-line writes), and 1024
    // owners already give every CU its workgroups
    // ... and at least SW_MIN_OWN owners (two solve workgroups per CU) while an owner keeps
    // about two keys: one rank of a key-sharded job holds K/N keys (1250 of C2's 10k at N=8),
    // and K/N/20 owners would leave most CUs without a solve workgroup
    static const int minown = getenv("SHP_SW_MINOWN") ? std::max(1, atoi(getenv("SHP_SW_MINOWN"))) : SW_MIN_OWN;
    static const int prefown = getenv("SHP_SW_PREFOWN") ? std::max(1, atoi(getenv("SHP_SW_PREFOWN"))) : SW_PREF_OWN;
    while (nown < SW_MAXOWN &&
           (((int64_t)nown * kpo < max_keys && (nown < prefown || (int64_t)nown * 200 < max_keys)) ||
            (nown < minown && (int64_t)nown * 2 <= max_keys)))
      nown *= 2;
    for (;;) {
      std::vector<int32_t> nloc(nown, 0);
      kmap.assign(max_keys, 0);
      int32_t mx = 0;
      int bits = 0;
      while ((1 << bits) < nown) bits++;
      for (int32_t k = 0; k < max_keys; k++) {
        const uint32_t o = sw_owner((uint32_t)k, bits);
        const int32_t lk = (int32_t)sw_local((uint32_t)k, bits);
        nloc[o]++;
        mx = std::max(mx, lk + 1);
        kmap[k] = o | ((uint32_t)lk << 16);
      }
      if (mx <= SW_LK) return true;
      if (nown >= SW_MAXOWN) return false;
      nown *= 2;
    }
  }

  template <class T>
  static void al(T*& p, int64_t n) {
    if (hipMalloc((void**)&p, std::max<int64_t>(n, 1) * sizeof(T)) != hipSuccess)
      throw std::runtime_error("hipMalloc failed (sweep path)");
  }

  void create(const DevProg& P, const FastShape& f, int32_t max_keys, int64_t cap, int32_t nown,
              const std::vector<uint32_t>& kmap, hipStream_t s) {
    D.vtag = P.ncol == 1 ? P.colTag[0] : T_NULL;
    if (!lower(f.f1, (int8_t)D.vtag, D.f1) || !lower(f.f2, (int8_t)D.vtag, D.f2) || !canonical_e2(D.f2))
      throw std::runtime_error("sweep: predicate not lowerable");
    D.within = f.within;
    D.fstream = f.stream;
    {
      SwPred c1 = D.f1;
      if (canonical_e1(c1)) {
        D.f1 = c1;
        int a = compare_type(D.f1, (int8_t)D.vtag), b = compare_type(D.f2, (int8_t)D.vtag);
        ct = a == b ? a : 0;
      } else {
        ct = 0;  // f1 evaluated by the generic double path
      }
    }
    D.nown = nown;
    D.own_bits = 0;
    while ((1 << D.own_bits) < nown) D.own_bits++;
    D.maxkeys = max_keys;
    {
      uint32_t mx = 0;
      for (uint32_t km : kmap) mx = std::max(mx, km >> 16);
      D.lk_bits = 0;
      while ((1u << D.lk_bits) <= mx) D.lk_bits++;
    }
    if (getenv("SHP_SW_STLEN")) st_len = st_len_big = std::max<int64_t>(4096, atoll(getenv("SHP_SW_STLEN")));
    nst_max = (int32_t)std::max<int64_t>(1, (cap + st_len - 1) / st_len);
    D.st_len = st_len;
    {
      for (int32_t k = 0; k < max_keys; k++)
        if ((kmap[k] & 0xffffu) != sw_owner((uint32_t)k, D.own_bits) ||
            (kmap[k] >> 16) != sw_local((uint32_t)k, D.own_bits))
          throw std::runtime_error("sweep: key map disagrees with sw_owner / sw_local");
      D.lk8 = nullptr;
      D.lk_lds = 0;
      const size_t lds = (size_t)(SWP_WAVES + 1) * nown * 4;
      // the staged scatter's LDS (> 64 KB at every owner count): counters, lofs and the stage
      if (hipFuncSetAttribute((const void*)k_sw_scatter<true, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)stg_lds(nown)) != hipSuccess)
        throw std::runtime_error("sweep: staged scatter LDS request refused");
      if (lds > 65536) {
        const void* fs[4] = {(const void*)k_sw_scatter<false, false>, (const void*)k_sw_scatter<true, false>,
                             (const void*)k_sw_scatter<false, true>, (const void*)k_sw_scatter<true, true>};
        for (const void* f : fs)
          if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            throw std::runtime_error("sweep: scatter LDS request refused");
      }
    }
    int64_t nc = (int64_t)nown * nst_max + 1;
    al(D.cnt, nc);
    al(D.off, nc);
    al(D.recs, cap + 1);
    D.trash = cap;
    for (int c = 0; c < 2; c++) {
      al(D.c_n[c], nown);
      al(D.c_ts[c], (int64_t)nown * SWS_CCAP);
      al(D.c_seq[c], (int64_t)nown * SWS_CCAP);
      al(D.c_v[c], (int64_t)nown * SWS_CCAP);
      al(D.c_lk[c], (int64_t)nown * SWS_CCAP);
      al(D.c_null[c], (int64_t)nown * SWS_CCAP);
      al(D.lastc[c], (int64_t)nown * SW_LK);
    }
    al(D.tsmax, 2);
    for (int c = 0; c < 2; c++) {
      al(D.spilled[c], nown);
      al(D.sp_n[c], nown);
      al(D.sp_base[c], nown);
      if (hipMemsetAsync(D.spilled[c], 0, nown, s) != hipSuccess ||
          hipMemsetAsync(D.sp_n[c], 0, (size_t)nown * 4, s) != hipSuccess)
        throw std::runtime_error("sweep: spill state");
    }
    al(D.ovf, nown);
    al(D.sp_active, 1);
    al(D.scr_base, nown);
    if (hipMemsetAsync(D.ovf, 0, nown, s) != hipSuccess) throw std::runtime_error("sweep: spill state");
    D.spill_on = 0;
    D.cur = 0;
    (void)rocprim::exclusive_scan(nullptr, tmp_bytes, D.cnt, D.off, 0u, (size_t)nc, rocprim::plus<uint32_t>(), s);
    if (hipMalloc(&tmp, std::max<size_t>(tmp_bytes, 16)) != hipSuccess)
      throw std::runtime_error("hipMalloc failed (sweep scan scratch)");
    // k_sw_lean: one f2 term `e2.v OP B` in the column's own type (float / int32), one of the six
    // standard comparisons; the pair layouts without nulls are checked per push (run)
    D.f1ct = ct != 0 && !getenv("SHP_SCATTER_GENERIC") ? ct : 0;
    lean_opc = 0;
    // (batch indices below 2^31: e1's filter rides in the index's top bit)
    if (D.f2.n == 1 && (ct == 1 || ct == 2) && !D.f2.t[0].flt && D.vtag != T_NULL && cap < (1ll << 31) &&
        !getenv("SHP_NO_LEAN"))
      lean_opc = sw_opclass(D.f2.t[0].mask);
    // k_sw_win: units of SWW_U records; a halo of about 16 events per local key of an owner
    // opt-in (SHP_WIN=1): measured 4.8 ms against k_sw_lean's 1.57 ms on C2
    win_off = getenv("SHP_WIN") == nullptr || getenv("SHP_NO_WIN") != nullptr;
    w_units = win_off ? 0 : (cap + SWW_U - 1) / SWW_U + 1;
    if (!win_off) {
      al(D.w_ticket, 1);
      al(D.w_stat, w_units);
      al(D.w_pres, (w_units + nown) * 8);
    }
    {
      const int64_t kpo = (max_keys + nown - 1) / nown;
      int64_t h = std::max<int64_t>((16 * kpo + 63) / 64 * 64, 64);
      if (getenv("SHP_WIN_HALO")) h = std::max<int64_t>(1, atoll(getenv("SHP_WIN_HALO")));  // tests, diagnostics
      D.w_halo = (int32_t)std::min<int64_t>(h, 1 << 24);
      D.w_tail = std::max<int32_t>(D.w_halo, 256);
    }
    int64_t ninit = std::max<int64_t>(nown, (int64_t)nown * SW_LK);
    k_sw_init<<<(unsigned)((ninit + 255) / 256), 256, 0, s>>>(D);
  }

  // SHP_LAYOUT_AGG: per-key aggregate state (zero) and the (owner, local key) -> key map
  void enable_agg(int fn, int32_t max_keys, const std::vector<uint32_t>& kmap, hipStream_t s) {
    const int64_t nk = (int64_t)D.nown * SW_LK;
    std::vector<int32_t> inv(nk, -1);
    for (int32_t k = 0; k < max_keys; k++) inv[(int64_t)(kmap[k] & 0xffffu) * SW_LK + (kmap[k] >> 16)] = k;
    al(D.inv, nk);
    if (hipMemcpy(D.inv, inv.data(), nk * 4, hipMemcpyHostToDevice) != hipSuccess)
      throw std::runtime_error("sweep: aggregate state");
    for (int c = 0; c < 2; c++) {
      al(D.agg_s[c], nk);
      al(D.agg_c[c], nk);
      if (hipMemsetAsync(D.agg_s[c], 0, nk * 8, s) != hipSuccess || hipMemsetAsync(D.agg_c[c], 0, nk * 8, s) != hipSuccess)
        throw std::runtime_error("sweep: aggregate state");
    }
    D.agg = fn;
  }

  // the push succeeded: the state it wrote becomes the state the next push reads
  void commit() { D.cur ^= 1; }

  void release() {
    void* ps[] = {(void*)D.lk8, D.inv, D.cnt, D.off, D.recs, D.tsmax, tmp, D.ovf, D.sp_active, D.scr_base,
                  D.s_idx, D.s_ts, D.s_seq, D.s_v, D.s_st, sizes, D.w_ticket, D.w_stat, D.w_pres};
    for (void* p : ps)
      if (p) (void)hipFree(p);
    for (int c = 0; c < 2; c++) {
      void* qs[] = {D.agg_s[c], D.agg_c[c], D.c_n[c], D.c_ts[c], D.c_seq[c], D.c_v[c], D.c_lk[c], D.c_null[c], D.lastc[c],
                    D.spilled[c], D.sp_n[c], D.sp_base[c], D.p_ts[c], D.p_seq[c], D.p_v[c], D.p_lk[c], D.p_null[c]};
      for (void* q : qs)
        if (q) (void)hipFree(q);
    }
    pool_cap[0] = pool_cap[1] = scr_cap = 0;
    sizes = nullptr;
    D = SweepDev{};
    tmp = nullptr;
  }

  // the three passes over one batch; matches (i, j) go to O.refs in per-key emission order
  void run(const BatchView& B, const int32_t* key, const MatchOut& O, int* err, hipStream_t s, KTimer& kt) {
    if (B.n <= 0) return;
    if (B.nulls[0]) D.maybe_null = 1;
    D.st_len = B.n >= (64ll << 20) ? st_len_big : st_len;
    D.nst = (int32_t)((B.n + D.st_len - 1) / D.st_len);
    (void)hipMemsetAsync(D.tsmax, 0, 2 * sizeof(unsigned long long), s);
    // overflow flags describe this push only: flags a failed push left must not be promoted to
    // spilled owners by a later push's SWE_SPILL re-run
    (void)hipMemsetAsync(D.ovf, 0, (size_t)D.nown, s);
    size_t nc = (size_t)D.nown * D.nst + 1;
    kt.mark("sw_count", s);
    k_sw_count<<<D.nst, SW_CNT_THREADS, 0, s>>>(D, B, key, err);
    kt.mark("sw_scan", s);
    size_t tb = tmp_bytes;
    (void)rocprim::exclusive_scan(tmp, tb, D.cnt, D.off, 0u, nc, rocprim::plus<uint32_t>(), s);
    kt.mark("sw_scatter", s);
    const bool win = win_push_for(B);
    // 12-byte records when the lean solve takes the push (k_sw_win, k_sw_solve and k_sw_spill read
    // the 16-byte form: a push the lean solve hands back is scattered again, rescatter16)
    D.r12 = !win && lean_push_for(B) && !D.spill_on && !r16_env() ? 1 : 0;
    scatter(B, key, err, s);
    last_win = false;
    if (win) {
      const int64_t units = (B.n + SWW_U - 1) / SWW_U;
      if (units > w_units) throw std::runtime_error("sweep: k_sw_win units beyond the batch capacity");
      (void)hipMemsetAsync(D.w_ticket, 0, sizeof(uint32_t), s);
      (void)hipMemsetAsync(D.w_stat, 0, (size_t)units * sizeof(unsigned long long), s);
      kt.mark("sw_win", s);
      sw_launch_win(ct, lean_opc, (unsigned)units, s, D, B, O, err);
      kt.mark("sw_win_tail", s);
      sw_launch_win_tail(ct, lean_opc, (unsigned)D.nown, s, D, B, err);
      kt.mark(nullptr, s);
      last_win = true;
    } else if (lean_push()) {
      kt.mark("sw_lean", s);
      launch_lean(B, O, err, s);
      kt.mark(nullptr, s);
    } else {
      solve(B, O, err, s, kt);
    }
  }

  static bool r16_env() {
    static const bool v = getenv("SHP_SW_R16") != nullptr;  // A/B: the 16-byte records on every push
    return v;
  }
  static size_t stg_lds(int nown) { return (size_t)(SWP_WAVES + 2) * nown * 4 + (size_t)4 * SWP_ROUND * 4; }
  static bool stg_env() {
    static const bool v = getenv("SHP_SCATTER_STAGE") != nullptr;  // A/B: the LDS-staged 12-byte scatter
    return v;
  }
  void scatter(const BatchView& B, const int32_t* key, int* err, hipStream_t s) {
    const size_t lds = (size_t)(SWP_WAVES + 1) * D.nown * 4;
    const bool pf = !B.stream && !B.nulls[0] && !getenv_flag_scatter_nopf();
    if (pf && D.r12 && stg_env()) k_sw_scatter<true, true, true><<<D.nst, SWP_THREADS, stg_lds(D.nown), s>>>(D, B, key, err);
    else if (pf && D.r12) k_sw_scatter<true, true><<<D.nst, SWP_THREADS, lds, s>>>(D, B, key, err);
    else if (pf) k_sw_scatter<true, false><<<D.nst, SWP_THREADS, lds, s>>>(D, B, key, err);
    else if (D.r12) k_sw_scatter<false, true><<<D.nst, SWP_THREADS, lds, s>>>(D, B, key, err);
    else k_sw_scatter<false, false><<<D.nst, SWP_THREADS, lds, s>>>(D, B, key, err);
  }
  // the push's records again in the 16-byte form, for the solves that read it (same counts and
  // offsets; the overflow flags of the 12-byte pass are cleared, the wide flag set again if so)
  bool rescatter16(const BatchView& B, const int32_t* key, int* err, hipStream_t s, KTimer& kt) {
    if (!D.r12) return false;
    D.r12 = 0;
    (void)hipMemsetAsync(D.tsmax, 0, 2 * sizeof(unsigned long long), s);
    kt.mark("sw_scatter16", s);
    scatter(B, key, err, s);
    kt.mark(nullptr, s);
    return true;
  }

  // does this push run k_sw_lean (so SWE_LEAN may come back and ask for solve())?
  // (SHP_LAYOUT_AGG: every selector aggregate -- avg / sum / count / min / max -- folds in k_sw_lean)
  bool lean_push() const { return lean_opc && D.agg <= 5 && !D.maybe_null; }
  bool lean_push_for(const BatchView& B) const { return lean_push() && !B.nulls[0]; }
  // k_sw_win (sweep_win.h): the pair layouts of the lean shape, no spilled owner
  bool win_push_for(const BatchView& B) const {
    return !win_off && lean_push_for(B) && D.agg == 0 && !D.spill_on && B.n > 0;
  }

  void launch_lean(const BatchView& B, const MatchOut& O, int* err, hipStream_t s) {
    if (D.agg) sw_launch_lean_agg(ct, lean_opc, (unsigned)D.nown, s, D, B, O, err);
    else sw_launch_lean(ct, lean_opc, (unsigned)D.nown, s, D, B, O, err);
  }

  // the exact solve (k_sw_solve) over the partition the scatter left; also the re-run of a push
  // k_sw_lean handed back with SWE_LEAN (the per-owner state it read is unchanged)
  void solve(const BatchView& B, const MatchOut& O, int* err, hipStream_t s, KTimer& kt) {
    kt.mark("sw_solve", s);
    sw_launch_solve(D.f1.n, D.f2.n, ct, (unsigned)D.nown, s, D, B, O, err);
    kt.mark(nullptr, s);
  }

  // ---- spilled owners (sweep_spill.h)
  void ensure_pool(int c, int64_t n) {
    if (n <= pool_cap[c]) return;
    const int64_t cap = std::max<int64_t>(n, pool_cap[c] * 2);
    int64_t *ts = nullptr, *seq = nullptr;
    uint32_t* v = nullptr;
    uint8_t *lk = nullptr, *nl = nullptr;
    al(ts, cap);
    al(seq, cap);
    al(v, cap);
    al(lk, cap);
    al(nl, cap);
    // keep what the copy holds (a committed copy may be grown too: restore)
    if (pool_cap[c] > 0) {
      const size_t m = (size_t)pool_cap[c];
      if (hipMemcpy(ts, D.p_ts[c], m * 8, hipMemcpyDeviceToDevice) != hipSuccess ||
          hipMemcpy(seq, D.p_seq[c], m * 8, hipMemcpyDeviceToDevice) != hipSuccess ||
          hipMemcpy(v, D.p_v[c], m * 4, hipMemcpyDeviceToDevice) != hipSuccess ||
          hipMemcpy(lk, D.p_lk[c], m, hipMemcpyDeviceToDevice) != hipSuccess ||
          hipMemcpy(nl, D.p_null[c], m, hipMemcpyDeviceToDevice) != hipSuccess)
        throw std::runtime_error("sweep: spill pool copy");
    }
    for (void* q : {(void*)D.p_ts[c], (void*)D.p_seq[c], (void*)D.p_v[c], (void*)D.p_lk[c], (void*)D.p_null[c]})
      if (q) (void)hipFree(q);
    D.p_ts[c] = ts;
    D.p_seq[c] = seq;
    D.p_v[c] = v;
    D.p_lk[c] = lk;
    D.p_null[c] = nl;
    pool_cap[c] = cap;
  }
  void ensure_scratch(int64_t n) {
    if (n <= scr_cap) return;
    const int64_t cap = std::max<int64_t>(n, scr_cap * 2);
    for (void* q : {(void*)D.s_idx, (void*)D.s_ts, (void*)D.s_seq, (void*)D.s_v, (void*)D.s_st})
      if (q) (void)hipFree(q);
    D.s_idx = nullptr;
    D.s_ts = D.s_seq = nullptr;
    D.s_v = nullptr;
    D.s_st = nullptr;
    al(D.s_idx, cap);
    al(D.s_ts, cap);
    al(D.s_seq, cap);
    al(D.s_v, cap);
    al(D.s_st, cap);
    scr_cap = cap;
  }
  // restore: pool copy c with exactly n entries (contents follow from the snapshot)
  void pool_exact(int c, int64_t n) {
    if (n == pool_cap[c]) return;
    for (void* q : {(void*)D.p_ts[c], (void*)D.p_seq[c], (void*)D.p_v[c], (void*)D.p_lk[c], (void*)D.p_null[c]})
      if (q) (void)hipFree(q);
    D.p_ts[c] = D.p_seq[c] = nullptr;
    D.p_v[c] = nullptr;
    D.p_lk[c] = D.p_null[c] = nullptr;
    pool_cap[c] = 0;
    if (n > 0) {
      al(D.p_ts[c], n);
      al(D.p_seq[c], n);
      al(D.p_v[c], n);
      al(D.p_lk[c], n);
      al(D.p_null[c], n);
      pool_cap[c] = n;
    }
  }
  // owners spilled in the committed state (host read-back)
  int64_t count_spilled() const {
    std::vector<uint8_t> f((size_t)D.nown);
    if (hipMemcpy(f.data(), D.spilled[D.cur], f.size(), hipMemcpyDeviceToHost) != hipSuccess) return -1;
    int64_t n = 0;
    for (uint8_t x : f) n += x ? 1 : 0;
    return n;
  }
  // the push's overflowing owners become spilled in the committed state (the push then re-runs).
  // If the re-run fails, they stay marked: that changes no state a later push or a snapshot reads
  // (sp_n = -1 keeps their carry in the c_* arrays, where describe() and every solve read it), only
  // which kernel solves them -- k_sw_spill, exact for every owner -- until spill_settle clears it
  void mark_spilled(hipStream_t s) {
    k_sw_mark_spilled<<<(unsigned)((D.nown + 255) / 256), 256, 0, s>>>(D);
    D.spill_on = 1;
  }
  // k_sw_spill over the spilled owners of this push: size their scratch and pool segments on the
  // host (one small read-back), then solve them
  void spill(const BatchView& B, const MatchOut& O, int* err, hipStream_t s, KTimer& kt) {
    if (!D.spill_on) return;
    const int rd = D.cur, wr = D.cur ^ 1;
    if (!sizes) al(sizes, (int64_t)D.nown * 3);
    k_sw_spill_sizes<<<(unsigned)((D.nown + 255) / 256), 256, 0, s>>>(D, sizes);
    std::vector<int64_t> h((size_t)D.nown * 3);
    if (hipMemcpyAsync(h.data(), sizes, h.size() * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      throw std::runtime_error("sweep: spill sizes");
    std::vector<int64_t> scr((size_t)D.nown, 0), pb((size_t)D.nown, 0);
    int64_t tot = 0;
    for (int32_t o = 0; o < D.nown; o++) {
      if (!h[3 * o]) continue;
      scr[o] = pb[o] = tot;
      tot += h[3 * o + 1] + h[3 * o + 2];  // records + carried: bounds the carry out too
    }
    ensure_scratch(tot + 1);
    ensure_pool(wr, tot + 1);
    if (hipMemcpyAsync(D.scr_base, scr.data(), scr.size() * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(D.sp_base[wr], pb.data(), pb.size() * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemsetAsync(D.sp_active, 0, 4, s) != hipSuccess)
      throw std::runtime_error("sweep: spill sizes");
    (void)rd;
    kt.mark("sw_spill", s);
    sw_launch_spill(D.f2.n, ct, (unsigned)D.nown, s, D, B, O, err);
    kt.mark(nullptr, s);
  }
  // after a committed push: are owners still spilled?  When none is, the spill state is cleared
  // in both copies and the LDS solves stop checking it
  void spill_settle(hipStream_t s) {
    if (!D.spill_on) return;
    int32_t act = 0;
    if (hipMemcpyAsync(&act, D.sp_active, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      throw std::runtime_error("sweep: spill state");
    if (act) return;
    for (int c = 0; c < 2; c++)
      if (hipMemsetAsync(D.spilled[c], 0, D.nown, s) != hipSuccess ||
          hipMemsetAsync(D.sp_n[c], 0, (size_t)D.nown * 4, s) != hipSuccess)
        throw std::runtime_error("sweep: spill state");
    D.spill_on = 0;
  }

  void expand(const BatchView& B, const int32_t* key, const MatchOut& O, int* err, hipStream_t s, KTimer& kt,
              int64_t m_host = -1) {
    if (D.p32 && m_host > 0)  // stage the 8-byte pairs where k_sw_expand reads them
      (void)hipMemcpyAsync(O.pos, O.refs, (size_t)m_host * 8, hipMemcpyDeviceToDevice, s);
    kt.mark("sw_expand", s);
    k_sw_expand<<<2048, 256, 0, s>>>(B, key, O, D.p32, err);
    kt.mark(nullptr, s);
  }
};

}  // namespace shp
