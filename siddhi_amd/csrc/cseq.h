// siddhi-hip: the count-sequence path, `every e1=S[f1]<1:M>, e2=S[f2]` (SURVEY.md §8d C3').
//
// For this sequence shape the Pre/PostStateProcessor chain (CountPreStateProcessor.processAndReturn
// :53-95, CountPostStateProcessor.process :39-65, StreamPreStateProcessor.processAndReturn
// :364-403 with the SEQUENCE removal rules, and the `every` re-arm of addEveryState :230-247)
// reduces, per partition key, to an automaton over L = the length of e1's chain.  The chain is
// always the key's last L events (an event that neither extends nor closes it ends it), so
// e1[last] is the key's previous event.  On each event x of the key (p = the previous event):
//   L > 0 and f2(p, x)           -> emit (chain, x); L = (L == M and f1(x)) ? 1 : 0
//                                   (a full chain left e1's every-partial re-armed: x opens it)
//   0 < L < M and f1(x)          -> L = L + 1
//   f1(x)                        -> L = 1   (L == 0, or a full chain that x did not close)
//   otherwise                    -> L = 0
// The rule was derived from, and is checked against, the oracle's object-level restatement of
// those processors (oracle/oracle.cpp): tests/test_cseq.py runs both on random streams for every
// M in 1..8 and every comparison, with NaN and null values, whole and split batches.
//
// Kernels (round 3, the default): k_cs_pack packs each event into a 16-byte record (ts, value,
// batch index | null) and rocPRIM's stable radix sort moves the records with their keys, so every
// later read is coalesced; k_cs2 then runs the automaton data-parallel over the key-sorted records:
// per event the transition is a function on L in 0..M (a table of M+1 nibbles: f1(x) = 0 -> 0;
// f1(x) and f2 -> T11; f1(x) alone -> T10), and L before each event is a segmented wave scan of
// their composition, seeded at each key's run start with the stored L (every prefix is then a
// constant).  One wave per key-aligned range of ~CS2_P events: a count pass, a scan over the waves,
// an emit pass writing each wave's records contiguously (per key in emission order).
//
// Kernels (round 2, kept as the reference form of the rule): the batch is partitioned by key with the
// engine's stable radix sort (as for the general lanes); k_cseq runs one thread per key over the key's
// events in arrival order, with
// the automaton, the previous value and the last M events' (seq, ts) in registers.  It runs
// twice: the first pass counts each key's records and refs, an exclusive scan over the keys
// places them, the second pass writes them (per key contiguous, in emission order) and the
// state.  One pair of same-address atomics per wave and event step measured 45 ms per 100M
// events at 1M keys: they serialise.  Per-key state (L, previous value and null flag, last M seqs and ts) lives in
// HBM, double-buffered: a push reads copy `cur`, writes `cur ^ 1`, and the engine flips `cur`
// only when the push succeeded.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <type_traits>
#include <stdexcept>

#include <rocprim/rocprim.hpp>

#include "nfa_lane.h"
#include "prog.h"
#include "sweep.h"

namespace shp {

// one event of the round-3 form: packed in arrival order, sorted with its key
struct __attribute__((aligned(16))) CsRec {
  int64_t ts;
  uint32_t v;
  uint32_t g;  // batch index | null << 31
};
// the narrow form (the default): ts relative to the push's first ts (B.ts[0]), 12 bytes, so the
// sort moves 32 instead of 40 bytes per event and pass; a push whose ts leave +-2^31 ms of that base
// sets CS_WIDE and re-runs in the 16-byte form
struct CsRec12 {
  int32_t tr;
  uint32_t v;
  uint32_t g;
};
constexpr int CS_WIDE = 1 << 26;
__device__ __forceinline__ int64_t cs_ts(const CsRec& r, int64_t) { return r.ts; }
__device__ __forceinline__ int64_t cs_ts(const CsRec12& r, int64_t base) { return base + r.tr; }
__device__ __forceinline__ void cs_set_ts(CsRec& r, int64_t t, int64_t, bool&) { r.ts = t; }
__device__ __forceinline__ void cs_set_ts(CsRec12& r, int64_t t, int64_t base, bool& wide) {
  const int64_t d = t - base;
  wide |= d != (int64_t)(int32_t)d;
  r.tr = (int32_t)d;
}

struct CseqDev {
  SwPred f1, f2;     // f1: e1 slot = the arriving event; f2: e1 slot = e1[last], e2 slot = the arriving event
  int32_t M, vtag, nk, cur;
  int32_t ch32;       // SHP_LAYOUT_CHAIN32: k_cs3's emit writes one word per match (cseq_own.h)
  int32_t mode;       // CS_EVERY1 .. CS_ONCEN (cs_tables)
  uint8_t* len[2];   // nk: L
  uint32_t* prev[2]; // nk: the previous event's value bits
  uint8_t* pnull[2]; // nk: ... and whether it was null
  int64_t* hseq[2];  // M * nk: seq of the key's last M events (slot M-1 = the latest), -1 none
  int64_t* hts[2];   // M * nk: their ts
  unsigned long long* tsmax;  // max ts of the push as ts ^ 2^63 (0: no event)
  uint32_t *cm, *cr;  // nk: records and refs per key (pass 1), then their exclusive scans
  uint32_t *om, *orf;
  // round-3 form: the packed records, sorted with their keys; per wave range starts, counts, offsets
  uint32_t *pk, *sk;
  CsRec *pr, *sr;
  unsigned long long* kend;  // nk: epoch << 32 | sorted position of the key's last event in the push (k_cs3)
  uint32_t epoch;            // this push's (k_cs_state tells a key with events from one without)
  int64_t* ws;
  uint32_t *wcm, *wcr, *wom, *wor;
};

// history slot s of key k (s = M-1 the key's latest event, M-2 the one before, ...): a key's M
// slots are contiguous, so the run end that rewrites them writes one span (slot-major arrays,
// s * nk + k, measured 0.8 ms of C3''s 2.5 ms emit in scattered 8-byte writes)
__host__ __device__ __forceinline__ int64_t cs_hslot(int s, int64_t k, int M) { return k * M + s; }

// ---- round-3 data-parallel form (see the header)
#ifndef CS2_P_CFG
#define CS2_P_CFG 2048
#endif
constexpr int CS2_P = CS2_P_CFG;  // nominal events per wave range (ranges start at key runs)

// pack: the sort key (key id; `nokey` for clock-only events and keys out of range) and the record,
// plus the push's max ts
template <class R>
__global__ void k_cs_pack(const int64_t* __restrict__ ts, const int32_t* __restrict__ key,
                          const int32_t* __restrict__ stream, const uint32_t* __restrict__ vcol,
                          const uint8_t* __restrict__ ncol, int64_t n, int partitioned, uint32_t nokey,
                          uint32_t* __restrict__ okey, R* __restrict__ orec, unsigned long long* tsmax, int* err) {
  int e = 0;
  int64_t mx = INT64_MIN;
  const int64_t base = ts[0];
  bool wide = false;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t k = 0;
    const int64_t t = ts[i];
    if (stream && stream[i] < 0) {  // (no stream column: every event on the query's stream)
      k = nokey;
    } else {
      mx = max(mx, t);
      if (partitioned) {
        const int32_t x = key[i];
        if (x < 0 || (uint32_t)x >= nokey) {
          e = 1 << 20;
          k = nokey;
        } else {
          k = (uint32_t)x;
        }
      }
    }
    okey[i] = k;
    R r;
    bool w = false;  // (clock-only events are never read back: their ts may lie anywhere)
    cs_set_ts(r, t, base, w);
    wide |= w && k != nokey;
    r.v = vcol ? vcol[i] : 0u;
    r.g = (uint32_t)i | ((ncol && ncol[i]) ? 0x80000000u : 0u);
    orec[i] = r;
  }
  for (int d = 32; d > 0; d >>= 1) mx = max(mx, (int64_t)__shfl_xor((long long)mx, d, 64));
  if (__lane_id() == 0 && mx != INT64_MIN) atomicMax(tsmax, (unsigned long long)mx ^ (1ull << 63));
  if (wide) e |= CS_WIDE;
  if (e) atomicOr(err, e);
}

// transition tables: entry i (4 bits at 4 i) = L after the event from L = i, for L in 0..CS_NL-1
// (0..M, and M + 1 the dead state of a once-armed start)
constexpr int CS_NL = CSEQ_MAXM + 2;
__device__ __forceinline__ uint64_t cs_tab_const(uint32_t c) { return 0x1111111111ull * (uint64_t)c; }
__device__ __forceinline__ uint32_t cs_at(uint64_t f, uint32_t i) { return (uint32_t)(f >> (4 * i)) & 15u; }
__device__ __forceinline__ uint64_t cs_comp(uint64_t g, uint64_t f) {  // g after f
  uint64_t h = 0;
#pragma unroll
  for (int i = 0; i < CS_NL; i++) h |= (uint64_t)cs_at(g, cs_at(f, i)) << (4 * i);
  return h;
}
// The shape's modes (CseqShape: `every` and min of e1's <min:M>), and per mode the tables T0
// (not f1(x)), T10 (f1(x) without f2), T11 (f1(x) and f2) on L in 0..M+1 (tests/test_cseq.py checks
// the rule against the oracle for every <min:M>, M <= 8, with and without `every`):
//   0 every, min 1   T0: -> 0; T10: 0 -> 1, L -> L + 1 (0 < L < M), M -> 1; T11: 0 -> 1, M -> 1, else 0
//   1 no every, min 1  (D = M + 1: the start state is armed once, CountPreStateProcessor.init
//                    :178-194 / resetState :288-305) T0: -> D; T10: 0 -> 1, L -> L + 1, M -> D;
//                    T11: 0 -> 1, L -> D; D -> D
//   2 every, min >= 2 / 3 no every, min >= 2: a chain never passes 1 (it reaches e1's new-and-every
//                    list only from min on, and the sequence's per-event reset clears the pending
//                    one) -- nothing is ever emitted.  L = 1 is the count-1 partial of the key's last
//                    event, alive until the key's next event: every: T10 = T11 -> 1, T0 -> 0; no
//                    every: T10 = T11: 0 -> 1, else D; T0 -> D (tests/test_cseq.py checks the live
//                    partials against the oracle's oldest live event)
// A match closes at an event with f2 when L before it is in 1..M (modes 0, 1).
constexpr int CS_EVERY1 = 0, CS_ONCE1 = 1, CS_EVERYN = 2, CS_ONCEN = 3;
__device__ __forceinline__ void cs_tables(int M, int mode, uint64_t& t0, uint64_t& t10, uint64_t& t11) {
  const uint64_t D = (uint64_t)M + 1u;
  t0 = t10 = t11 = 0;
  for (int i = 0; i < CS_NL; i++) {
    uint64_t a, b, z;
    if (mode == CS_EVERY1) {
      z = 0;
      a = (i == 0 || i >= M) ? 1u : (uint64_t)(i + 1);
      b = (i == 0 || i >= M) ? 1u : 0u;
    } else if (mode == CS_ONCE1) {
      z = D;
      a = i == 0 ? 1u : (i < M ? (uint64_t)(i + 1) : D);
      b = i == 0 ? 1u : D;
    } else if (mode == CS_EVERYN) {
      z = 0;
      a = b = 1;
    } else {
      z = D;
      a = b = i == 0 ? 1u : D;
    }
    t0 |= z << (4 * i);
    t10 |= a << (4 * i);
    t11 |= b << (4 * i);
  }
}
__device__ __forceinline__ bool cs_emits(int mode, uint32_t Lb, int M) {
  return mode <= CS_ONCE1 && Lb >= 1u && Lb <= (uint32_t)M;
}

// the first key-run start at or after position j of the sorted keys (n if none): a 64-ary search
// by the whole wave (every lane gets the result)
__device__ __forceinline__ int64_t cs_run_start(const uint32_t* __restrict__ sk, int64_t n, int64_t j) {
  if (j <= 0) return 0;
  if (j >= n) return n;
  const uint32_t k = sk[j];
  if (sk[j - 1] != k) return j;
  const uint32_t lane = __lane_id();
  // gallop: [lo, hi) with sk[lo] == k and sk[hi] != k (or hi == n)
  int64_t lo = j, hi = -1, stride = 1;
  while (hi < 0) {
    const int64_t p = lo + (int64_t)(lane + 1) * stride;
    const bool past = p >= n || sk[p] != k;
    const uint64_t m = __ballot(past);
    if (m) {
      const int f = __ffsll((unsigned long long)m) - 1;
      hi = min(n, lo + (int64_t)(f + 1) * stride);
      lo = lo + (int64_t)f * stride;
    } else {
      lo += 64 * stride;
      stride *= 64;
    }
  }
  while (hi - lo > 1) {  // refine: 64 probes per round
    const int64_t st = (hi - lo + 63) / 64;
    const int64_t p = lo + (int64_t)(lane + 1) * st;
    const bool past = p >= hi || sk[p] != k;
    const uint64_t m = __ballot(past);
    const int f = __ffsll((unsigned long long)m) - 1;  // m != 0: lane 63 probes >= hi
    const int64_t nh = min(hi, lo + (int64_t)(f + 1) * st);
    lo = lo + (int64_t)f * st;
    hi = nh;
  }
  return hi;
}

// per wave: its range start (ws[w], the count pass) -- the count and emit passes share them
static __global__ void k_cs2_ranges(const uint32_t* __restrict__ sk, int64_t n, int64_t nw, int64_t* ws) {
  const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (w > nw) return;
  const int64_t s = cs_run_start(sk, n, w * (int64_t)CS2_P);
  if (__lane_id() == 0) ws[w] = s;
}

template <int NT1, int NT2, bool EMIT, class R>
__global__ __launch_bounds__(256) void k_cs2(CseqDev C, BatchView B, MatchOut O, const uint32_t* __restrict__ sk,
                                             const R* __restrict__ sv, const int64_t* __restrict__ ws, int64_t nw,
                                             int* err) {
  const int64_t wv = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (wv >= nw) return;  // whole waves
  const uint32_t lane = __lane_id();
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  const int rd = C.cur, wr = C.cur ^ 1;
  const int M = C.M;
  const uint32_t nk = (uint32_t)C.nk;
  const int64_t S = ws[wv], E = ws[wv + 1];
  const bool vnull = C.vtag == T_NULL, vflt = C.vtag == T_FLOAT;
  const int64_t tbase = B.ts[0];  // the narrow records' ts base (k_cs_pack)
  uint64_t t0, t10, t11;
  cs_tables(M, C.mode, t0, t10, t11);
  // carried from the previous 64 events (lane 63's): L after it, its value, its run's start
  uint32_t cL = 0, cpv = 0;
  bool cpn = true;
  int64_t crs = S;
  uint32_t nm = 0, nr = 0;
  int64_t mo = 0, ro = 0;  // EMIT: the wave's next record / ref slot
  if (EMIT) {
    mo = C.wom[wv];
    ro = C.wor[wv];
    if (wv == nw - 1 && lane == 0) {  // the push's totals
      O.count[0] = (unsigned long long)(mo + C.wcm[wv]);
      O.count[1] = (unsigned long long)(ro + C.wcr[wv]);
    }
  }
  int e = 0;
  for (int64_t p0 = S; p0 < E; p0 += 64) {
    const int64_t j = p0 + lane;
    const uint32_t k = j < E ? sk[j] : 0xFFFFFFFFu;
    const bool v = j < E && k < nk;  // clock-only events sort last (nokey) and are skipped
    const uint32_t kprev = (j > S && j < E) ? sk[j - 1] : 0xFFFFFFFEu;
    const bool head = v && (j == S || kprev != k);
    R r{};
    if (v) r = sv[j];
    const uint32_t x = r.v;
    const bool xn = vnull || (r.g >> 31) != 0;
    uint32_t L0 = 0, spv = 0;
    bool spn = true;
    if (head) {  // the key's stored state (the previous push)
      L0 = C.len[rd][k];
      spv = C.prev[rd][k];
      spn = C.pnull[rd][k] != 0;
    }
    // the previous event of the key: lane - 1, or (lane 0) the carried one, or (a run start) stored
    uint32_t pv = __shfl_up(x, 1, 64);
    bool pn = __shfl_up((int)xn, 1, 64) != 0;
    if (lane == 0) {
      pv = cpv;
      pn = cpn;
    }
    if (head) {
      pv = spv;
      pn = spn;
    }
    double xf, xi, pf, pi;
    sw_conv(x, vflt, xf, xi);
    sw_conv(pv, vflt, pf, pi);
    const bool a = v && sw_pred<NT1>(C.f1, xf, xi, xn, 0.0, 0.0, true);
    const bool b = v && sw_pred<NT2>(C.f2, pf, pi, pn, xf, xi, xn);
    const uint64_t F = a ? (b ? t11 : t10) : t0;
    // seeded elements: a run start composes F with its stored L, lane 0 with the carried L
    const bool seeded = head || lane == 0;
    const uint32_t Lseed = head ? L0 : cL;
    uint64_t val = seeded ? cs_tab_const(cs_at(F, Lseed)) : F;
    int fl = seeded ? 1 : 0;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {  // segmented inclusive scan of the compositions
      const uint64_t y = __shfl_up(val, d, 64);
      const int yf = __shfl_up(fl, d, 64);
      if (lane >= (uint32_t)d && !fl) val = cs_comp(val, y);
      if (lane >= (uint32_t)d) fl |= yf;
    }
    const uint32_t La = cs_at(val, 0);  // L after this event (every prefix is a constant)
    uint32_t Lb = __shfl_up(La, 1, 64);  // L before it
    if (lane == 0) Lb = cL;
    if (head) Lb = L0;
    const bool em = v && cs_emits(C.mode, Lb, M) && b;
    const uint32_t rfs = em ? Lb + 1u : 0u;
    // this event's run start (for the chain refs and the history): the latest head at or before it
    int64_t rs = head ? j : -1;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int64_t y = __shfl_up(rs, d, 64);
      if (lane >= (uint32_t)d && rs < 0) rs = y;
    }
    if (rs < 0) rs = crs;
    if (!EMIT) {
      nm += em ? 1u : 0u;
      nr += rfs;
    } else {
      // offsets: wave exclusive scans of the records and refs
      uint32_t xm = em ? 1u : 0u, xr = rfs;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t ym = __shfl_up(xm, d, 64), yr = __shfl_up(xr, d, 64);
        if (lane >= (uint32_t)d) {
          xm += ym;
          xr += yr;
        }
      }
      const int64_t mi = mo + xm - (em ? 1 : 0), ri = ro + xr - rfs;
      if (em) {
        if (mi >= O.cap || ri + rfs > O.refcap) {
          e |= E_OUT;
        } else {
          const int64_t sg = bseq(B, r.g & 0x7FFFFFFFu);
          O.key[mi] = B.partitioned ? (int32_t)k : 0;
          O.ts[mi] = cs_ts(r, tbase);  // StateEvent ts = e2's (StreamPostStateProcessor.process :64-83)
          O.type[mi] = 0;
          O.pos[mi] = sg;
          O.ref_off[mi] = ri;
          O.slot_len[mi * MAXS] = (int16_t)Lb;
          O.slot_len[mi * MAXS + 1] = 1;
          // e1's chain: the key's Lb events before this one, oldest first; then e2
          for (uint32_t t = 1; t <= Lb; t++) {
            const int64_t pp = j - (int64_t)t;
            int64_t q;
            if (pp >= rs) q = bseq(B, sv[pp].g & 0x7FFFFFFFu);
            else q = C.hseq[rd][cs_hslot(M - (int)(rs - pp), k, M)];  // before the push
            O.refs[ri + (Lb - t)] = q;
          }
          O.refs[ri + Lb] = sg;
        }
      }
      mo += __shfl(xm, 63, 64);
      ro += __shfl(xr, 63, 64);
      // the key's state after its run in the push (the run's last event)
      const uint32_t knext = j + 1 < E ? sk[j + 1] : 0xFFFFFFFDu;
      if (v && knext != k) {
        C.len[wr][k] = (uint8_t)La;
        C.prev[wr][k] = x;
        C.pnull[wr][k] = xn ? 1 : 0;
        for (int s2 = 0; s2 < M; s2++) {  // slot M-1 = this event, M-2 the one before, ...
          const int64_t pp = j - (int64_t)(M - 1 - s2);
          int64_t hs, ht;
          if (pp >= rs) {
            const R q = pp == j ? r : sv[pp];
            hs = bseq(B, q.g & 0x7FFFFFFFu);
            ht = cs_ts(q, tbase);
          } else {
            const int64_t so = cs_hslot(M - (int)(rs - pp), k, M);
            hs = C.hseq[rd][so];
            ht = C.hts[rd][so];
          }
          C.hseq[wr][cs_hslot(s2, k, M)] = hs;
          C.hts[wr][cs_hslot(s2, k, M)] = ht;
        }
      }
    }
    cL = __shfl(La, 63, 64);
    cpv = __shfl(x, 63, 64);
    cpn = __shfl((int)xn, 63, 64) != 0;
    crs = __shfl(rs, 63, 64);
    (void)lt;
  }
  if (!EMIT) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
      nm += __shfl_xor(nm, d, 64);
      nr += __shfl_xor(nr, d, 64);
    }
    if (lane == 0) {
      C.wcm[wv] = nm;
      C.wcr[wv] = nr;
    }
  }
  if (e) atomicOr(err, e);
}

// The lane-sequential form (the default; k_cs2 kept for A/B, SHP_CSEQ_SCAN64): a wave's range is
// walked in tiles of 64 x CS3_Q sorted positions, each lane a contiguous CS3_Q of them.  A lane
// composes its events' transitions itself (seeded at a run start with the stored L), so the wave
// scans once per tile instead of once per 64 events: one segmented scan of the lanes' compositions
// (lane 0 seeded with the carried L, so every prefix is a constant), one max-scan of the latest run
// start, and (emit) one scan of the lanes' record / ref counts.  Then each lane re-walks its events
// with a concrete L: the same rule as k_cs2, event for event.
#ifndef CS3_QC_CFG
#define CS3_QC_CFG 4
#endif
#ifndef CS3_QE_CFG
#define CS3_QE_CFG 2
#endif
constexpr int CS3_QC = CS3_QC_CFG;  // events per lane per tile, count pass
constexpr int CS3_QE = CS3_QE_CFG;  // ... emit pass (measured: 4 and 2 fastest, 8 / 16 slower)

template <int NT1, int NT2, bool EMIT, class R, int CS3_Q = EMIT ? CS3_QE : CS3_QC>
__global__ __launch_bounds__(256) void k_cs3(CseqDev C, BatchView B, MatchOut O, const uint32_t* __restrict__ sk,
                                             const R* __restrict__ sv, const int64_t* __restrict__ ws, int64_t nw,
                                             int* err) {
  static_assert(CS3_Q == 1 || CS3_Q == 2 || CS3_Q == 4 || CS3_Q == 8 || CS3_Q == 16,
                "a lane's events: 4 flag fields of CS3_Q bits in one word");
  using Cs3W = typename std::conditional<(CS3_Q > 8), uint64_t, uint32_t>::type;
  const int64_t wv = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (wv >= nw) return;  // whole waves
  const uint32_t lane = __lane_id();
  const int rd = C.cur, wr = C.cur ^ 1;
  const int M = C.M;
  const uint32_t nk = (uint32_t)C.nk;
  const int64_t S = ws[wv], E = ws[wv + 1];
  const bool vnull = C.vtag == T_NULL, vflt = C.vtag == T_FLOAT;
  const int64_t tbase = B.ts[0];  // the narrow records' ts base (k_cs_pack)
  uint64_t t0, t10, t11;
  cs_tables(M, C.mode, t0, t10, t11);
  uint64_t ident = 0;
#pragma unroll
  for (int i = 0; i < CS_NL; i++) ident |= (uint64_t)i << (4 * i);
  // carried from the previous tile (its last event): L after it, its value and null flag, its run start
  uint32_t cL = 0, cpv = 0;
  bool cpn = true;
  int64_t crs = S;
  uint32_t nm = 0, nr = 0;
  int64_t mo = 0, ro = 0;  // EMIT: the wave's next record / ref slot
  if (EMIT) {
    mo = C.wom[wv];
    ro = C.wor[wv];
    if (wv == nw - 1 && lane == 0) {  // the push's totals
      O.count[0] = (unsigned long long)(mo + C.wcm[wv]);
      O.count[1] = (unsigned long long)(ro + C.wcr[wv]);
    }
  }
  int e = 0;
  for (int64_t p0 = S; p0 < E; p0 += 64 * CS3_Q) {
    const int64_t j0 = p0 + (int64_t)lane * CS3_Q;
    uint32_t kq[CS3_Q];
    R rq[CS3_Q];
#pragma unroll
    for (int q = 0; q < CS3_Q; q++) {
      const int64_t j = j0 + q;
      kq[q] = j < E ? sk[j] : 0xFFFFFFFFu;
      rq[q] = j < E ? sv[j] : R{};
    }
    const uint32_t kbefore = (j0 > S && j0 < E) ? sk[j0 - 1] : 0xFFFFFFFEu;
    // the previous event's value for the lane's first event: lane - 1's last, or (lane 0) the carried
    const bool xnl = vnull || (rq[CS3_Q - 1].g >> 31) != 0;
    uint32_t px = __shfl_up(rq[CS3_Q - 1].v, 1, 64);
    bool pxn = __shfl_up((int)xnl, 1, 64) != 0;
    if (lane == 0) {
      px = cpv;
      pxn = cpn;
    }
    // walk 1: per event f1 / f2 / head / valid bits (and the stored L at heads); the lane's composition
    uint32_t hb = 0, ab = 0, bb = 0, vb = 0;
    uint64_t L0q = 0;
    uint64_t G = ident;
    int gs = 0;
    int64_t lh = -1;  // the lane's latest run start
#pragma unroll
    for (int q = 0; q < CS3_Q; q++) {
      const int64_t j = j0 + q;
      const uint32_t k = kq[q];
      const bool v = j < E && k < nk;  // clock-only events sort last (nokey) and are skipped
      const uint32_t kp = q == 0 ? kbefore : kq[q - 1];
      const bool head = v && (j == S || kp != k);
      const uint32_t x = rq[q].v;
      const bool xn = vnull || (rq[q].g >> 31) != 0;
      uint32_t L0 = 0;
      if (head) {  // the key's stored state (the previous push)
        L0 = C.len[rd][k];
        px = C.prev[rd][k];
        pxn = C.pnull[rd][k] != 0;
        L0q |= (uint64_t)L0 << (4 * q);
        lh = j;
      }
      double xf, xi, pf, pi;
      sw_conv(x, vflt, xf, xi);
      sw_conv(px, vflt, pf, pi);
      const bool a = v && sw_pred<NT1>(C.f1, xf, xi, xn, 0.0, 0.0, true);
      const bool b = v && sw_pred<NT2>(C.f2, pf, pi, pxn, xf, xi, xn);
      const uint64_t F = a ? (b ? t11 : t10) : t0;
      hb |= (head ? 1u : 0u) << q;
      ab |= (a ? 1u : 0u) << q;
      bb |= (b ? 1u : 0u) << q;
      vb |= (v ? 1u : 0u) << q;
      if (head) {
        G = cs_tab_const(cs_at(F, L0));
        gs = 1;
      } else {
        G = cs_comp(F, G);
      }
      px = x;
      pxn = xn;
    }
    // the wave's scans: L into each lane, and the run start in force at its first event
    uint64_t val = G;
    int fl = gs;
    if (lane == 0 && !gs) {
      val = cs_tab_const(cs_at(G, cL));
      fl = 1;
    }
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint64_t y = __shfl_up(val, d, 64);
      const int yf = __shfl_up(fl, d, 64);
      if (lane >= (uint32_t)d && !fl) val = cs_comp(val, y);
      if (lane >= (uint32_t)d) fl |= yf;
    }
    uint32_t Lin = cs_at(__shfl_up(val, 1, 64), 0);
    if (lane == 0) Lin = cL;
    int64_t rsc = lh;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int64_t y = __shfl_up(rsc, d, 64);
      if (lane >= (uint32_t)d && y > rsc) rsc = y;
    }
    int64_t rs_in = __shfl_up(rsc, 1, 64);
    if (lane == 0 || rs_in < crs) rs_in = crs;
    // walk 2: the lane's records and refs; per event L before it (a nibble) and the flags
    // (emits | run start << Q | valid << 2Q | f1(x) << 3Q) for the event-major emit
    uint32_t L = Lin, lm = 0, lr = 0;
    Cs3W lbw = 0, fw = 0;
#pragma unroll
    for (int q = 0; q < CS3_Q; q++) {
      const bool head = (hb >> q) & 1u;
      const uint32_t Lb = head ? (uint32_t)(L0q >> (4 * q)) & 15u : L;
      const bool a = (ab >> q) & 1u, b = (bb >> q) & 1u, v = (vb >> q) & 1u;
      L = cs_at(a ? (b ? t11 : t10) : t0, Lb);
      const bool em = v && cs_emits(C.mode, Lb, M) && b;
      lm += em ? 1u : 0u;
      lr += em ? Lb + 1u : 0u;
      lbw |= (Cs3W)Lb << (4 * q);
      fw |= (Cs3W)(em ? 1u : 0u) << q;
    }
    fw |= ((Cs3W)hb << CS3_Q) | ((Cs3W)vb << (2 * CS3_Q)) | ((Cs3W)ab << (3 * CS3_Q));
    const uint32_t Lend = L;
    const int64_t rs_end = max(rs_in, lh);
    const uint32_t xlast = rq[CS3_Q - 1].v;
    if (!EMIT) {
      nm += lm;
      nr += lr;
    } else {
      uint32_t xm = lm, xr = lr;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t ym = __shfl_up(xm, d, 64), yr = __shfl_up(xr, d, 64);
        if (lane >= (uint32_t)d) {
          xm += ym;
          xr += yr;
        }
      }
      const uint32_t m0 = xm - lm, r0 = xr - lr;        // the lane's first record / ref, from mo / ro
      const int32_t rs0 = (int32_t)(rs_in - S);          // its run start in force, from S
      // event-major: in step s lane l takes event p0 + 64 s + l (coalesced loads and stores), which
      // lane 8 s + l / 8 walked; that lane's words give L before it and its record / ref slots
#pragma unroll 1
      for (int st = 0; st < CS3_Q; st++) {
        const int src = st * (64 / CS3_Q) + (int)(lane / CS3_Q);
        const int q = (int)(lane % CS3_Q);
        const Cs3W LbW = __shfl(lbw, src, 64), FW = __shfl(fw, src, 64);
        const uint32_t M0 = __shfl(m0, src, 64), R0 = __shfl(r0, src, 64);
        const int32_t RS = __shfl(rs0, src, 64);
        const int64_t j = p0 + (int64_t)st * 64 + lane;
        // the next event's key (a run end: it differs): lane + 1's, lane 63 reads it
        const uint32_t kl = j < E ? sk[j] : 0xFFFFFFFDu;
        uint32_t knext = __shfl_down(kl, 1, 64);
        if (lane == 63) knext = j + 1 < E ? sk[j + 1] : 0xFFFFFFFDu;
        if (!((FW >> (2 * CS3_Q + q)) & 1u)) continue;  // not a valid event (past E, or clock-only)
        const uint32_t emw = (uint32_t)(FW & ((1u << CS3_Q) - 1u)), hw = (uint32_t)(FW >> CS3_Q) & ((1u << CS3_Q) - 1u);
        const uint32_t below = (1u << q) - 1u;
        uint32_t rb = 0;
#pragma unroll
        for (int q2 = 0; q2 < CS3_Q; q2++)
          rb += ((emw >> q2) & 1u) && q2 < q ? (uint32_t)((LbW >> (4 * q2)) & 15u) + 1u : 0u;
        const int64_t mi = mo + M0 + (uint32_t)__popc(emw & below), ri = ro + R0 + rb;
        const uint32_t hm = hw & ((2u << q) - 1u);  // run starts at or before this event
        const int64_t rs = hm ? p0 + (int64_t)src * CS3_Q + (31 - __clz(hm)) : S + RS;
        const uint32_t Lb = (uint32_t)(LbW >> (4 * q)) & 15u;
        const bool em = (emw >> q) & 1u, a = (FW >> (3 * CS3_Q + q)) & 1u;
        const uint32_t La = cs_at(a ? (em ? t11 : t10) : t0, Lb);  // (no emission: T11 and T10 agree)
        const uint32_t k = kl;
        const R rj = sv[j];
        if (em && C.ch32) {  // CHAIN32: e2's batch index | L << 28 (the chain is implied)
          if (mi >= O.cap) e |= E_OUT;
          else reinterpret_cast<uint32_t*>(O.refs)[mi] = (rj.g & 0x7FFFFFFFu) | (Lb << 28);
        } else if (em) {
          const uint32_t rfs = Lb + 1u;
          if (mi >= O.cap || ri + rfs > O.refcap) {
            e |= E_OUT;
          } else {
            const int64_t sg = bseq(B, rj.g & 0x7FFFFFFFu);
            O.key[mi] = B.partitioned ? (int32_t)k : 0;
            O.ts[mi] = cs_ts(rj, tbase);  // StateEvent ts = e2's (StreamPostStateProcessor.process :64-83)
            O.type[mi] = 0;
            O.pos[mi] = sg;
            O.ref_off[mi] = ri;
            O.slot_len[mi * MAXS] = (int16_t)Lb;
            O.slot_len[mi * MAXS + 1] = 1;
            // e1's chain: the key's Lb events before this one, oldest first; then e2
#ifndef CS_DIAG_NOREFS  // diagnostics only (wrong output): the emit without its chain refs
            for (uint32_t t = 1; t <= Lb; t++) {
              const int64_t pp = j - (int64_t)t;
              int64_t qs;
              if (pp >= rs) qs = bseq(B, sv[pp].g & 0x7FFFFFFFu);
              else qs = C.hseq[rd][cs_hslot(M - (int)(rs - pp), k, M)];  // before the push
              O.refs[ri + (Lb - t)] = qs;
            }
            O.refs[ri + Lb] = sg;
#endif
          }
        }
        // the key's state after its run in the push (the run's last event)
        if (knext != k) {  // the run's last event: L after it, and where it is (k_cs_state does the rest)
          C.len[wr][k] = (uint8_t)La;
          C.kend[k] = ((unsigned long long)C.epoch << 32) | (uint32_t)j;
        }
      }
      mo += __shfl(xm, 63, 64);
      ro += __shfl(xr, 63, 64);
    }
    cL = __shfl(Lend, 63, 64);
    cpv = __shfl(xlast, 63, 64);
    cpn = __shfl((int)xnl, 63, 64) != 0;
    crs = __shfl(rs_end, 63, 64);
  }
  if (!EMIT) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
      nm += __shfl_xor(nm, d, 64);
      nr += __shfl_xor(nr, d, 64);
    }
    if (lane == 0) {
      C.wcm[wv] = nm;
      C.wcr[wv] = nr;
    }
  }
  if (e) atomicOr(err, e);
}

// per key, after k_cs3's emit: a key with events in the push takes its previous value and null
// flag and its last M events' (seq, ts) from the sorted records at its run end (the slots before the
// run from its stored history); a key without passes its state through.  One thread per key, each
// key's M slots contiguous: coalesced where the emit's per-run-end writes were not (0.8 ms of 2.5)
template <class R>
__global__ __launch_bounds__(256) void k_cs_state(CseqDev C, BatchView B, const uint32_t* __restrict__ sk,
                                                  const R* __restrict__ sv) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= C.nk) return;
  const int rd = C.cur, wr = C.cur ^ 1;
  const int M = C.M;
  const unsigned long long ke = C.kend[k];
  if ((uint32_t)(ke >> 32) != C.epoch) {
    C.len[wr][k] = C.len[rd][k];
    C.prev[wr][k] = C.prev[rd][k];
    C.pnull[wr][k] = C.pnull[rd][k];
    for (int s2 = 0; s2 < M; s2++) {
      C.hseq[wr][cs_hslot(s2, k, M)] = C.hseq[rd][cs_hslot(s2, k, M)];
      C.hts[wr][cs_hslot(s2, k, M)] = C.hts[rd][cs_hslot(s2, k, M)];
    }
    return;
  }
  const int64_t j = (int64_t)(uint32_t)ke;
  const int64_t tbase = B.ts[0];
  const R rj = sv[j];
  C.prev[wr][k] = rj.v;
  C.pnull[wr][k] = (C.vtag == T_NULL || (rj.g >> 31) != 0) ? 1 : 0;
  // the run start, as far back as the history reaches
  int64_t rs = j;
  while (rs > j - (M - 1) && rs > 0 && sk[rs - 1] == (uint32_t)k) rs--;
  for (int s2 = 0; s2 < M; s2++) {  // slot M-1 = the last event, M-2 the one before, ...
    const int64_t pp = j - (int64_t)(M - 1 - s2);
    int64_t hs, ht;
    if (pp >= rs) {
      const R qv = pp == j ? rj : sv[pp];
      hs = bseq(B, qv.g & 0x7FFFFFFFu);
      ht = cs_ts(qv, tbase);
    } else {
      const int64_t so = cs_hslot(M - (int)(rs - pp), k, M);
      hs = C.hseq[rd][so];
      ht = C.hts[rd][so];
    }
    C.hseq[wr][cs_hslot(s2, k, M)] = hs;
    C.hts[wr][cs_hslot(s2, k, M)] = ht;
  }
}

template <int NT1, int NT2, bool EMIT>
__global__ __launch_bounds__(256) void k_cseq(CseqDev C, BatchView B, MatchOut O, const uint32_t* __restrict__ perm,
                                              const uint32_t* __restrict__ kbeg, const uint32_t* __restrict__ kcnt,
                                              int* err) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  const bool live = k < C.nk;
  const int rd = C.cur, wr = C.cur ^ 1;
  const int M = C.M;
  int L = 0;
  uint32_t pv = 0;
  bool pn = true;
  int64_t hs[CSEQ_MAXM], ht[CSEQ_MAXM];
#pragma unroll
  for (int i = 0; i < CSEQ_MAXM; i++) {
    hs[i] = -1;
    ht[i] = -1;
  }
  uint32_t beg = 0, cnt = 0;
  if (live) {
    L = C.len[rd][k];
    pv = C.prev[rd][k];
    pn = C.pnull[rd][k] != 0;
#pragma unroll
    for (int i = 0; i < CSEQ_MAXM; i++) {
      const int s = i - (CSEQ_MAXM - M);  // history slot s of the stored M
      if (s >= 0) {
        hs[i] = C.hseq[rd][cs_hslot(s, k, M)];
        ht[i] = C.hts[rd][cs_hslot(s, k, M)];
      }
    }
    beg = kbeg[k];
    cnt = kcnt[k];
  }
  const uint32_t* vcol = (const uint32_t*)B.cols[0];
  const uint8_t* ncol = B.nulls[0];
  const bool vnull = C.vtag == T_NULL, vflt = C.vtag == T_FLOAT;
  int64_t tmax = INT64_MIN;
  int e = 0;
  uint32_t nm = 0, nr = 0;  // this key's records and refs so far
  int64_t mi = 0, ri = 0;
  if (EMIT && live) {
    mi = C.om[k];
    ri = C.orf[k];
    if (k == C.nk - 1) {  // the push's totals
      O.count[0] = (unsigned long long)(mi + C.cm[k]);
      O.count[1] = (unsigned long long)(ri + C.cr[k]);
    }
  }
  for (uint32_t j = 0; j < cnt; j++) {
    const bool act = true;
    bool em = false;
    int nL = 0;
    int64_t tsg = 0, sg = 0;
    uint32_t x = 0;
    bool xn = true;
    if (act) {
      const int64_t g = perm[beg + j];
      tsg = B.ts[g];
      tmax = max(tmax, tsg);
      sg = bseq(B, g);
      x = vcol ? vcol[g] : 0u;
      xn = vnull || (ncol && ncol[g]);
      double xf, xi, pf, pi;
      sw_conv(x, vflt, xf, xi);
      sw_conv(pv, vflt, pf, pi);
      const bool f1x = sw_pred<NT1>(C.f1, xf, xi, xn, 0.0, 0.0, true);
      em = L > 0 && sw_pred<NT2>(C.f2, pf, pi, pn, xf, xi, xn);
      if (em) nL = (L == M && f1x) ? 1 : 0;
      else if (L > 0 && L < M && f1x) nL = L + 1;
      else nL = f1x ? 1 : 0;
    }
    if (em) {
      nm++;
      nr += (uint32_t)L + 1u;
      if (EMIT) {
        if (mi >= O.cap || ri + L + 1 > O.refcap) {
          e |= E_OUT;
        } else {
          O.key[mi] = B.partitioned ? k : 0;
          O.ts[mi] = tsg;  // StateEvent ts = e2's (StreamPostStateProcessor.process :64-83)
          O.type[mi] = 0;
          O.pos[mi] = sg;
          O.ref_off[mi] = ri;
          O.slot_len[mi * MAXS] = (int16_t)L;
          O.slot_len[mi * MAXS + 1] = 1;
          // e1's chain: the key's last L events, oldest first; then e2
          int64_t r = ri;
#pragma unroll
          for (int i = 0; i < CSEQ_MAXM; i++)
            if (i >= CSEQ_MAXM - L) O.refs[r++] = hs[i];
          O.refs[r] = sg;
        }
        mi++;
        ri += L + 1;
      }
    }
    if (act) {
#pragma unroll
      for (int i = 0; i + 1 < CSEQ_MAXM; i++) {
        hs[i] = hs[i + 1];
        ht[i] = ht[i + 1];
      }
      hs[CSEQ_MAXM - 1] = sg;
      ht[CSEQ_MAXM - 1] = tsg;
      L = nL;
      pv = x;
      pn = xn;
    }
  }
  if (!EMIT) {
    if (live) {
      C.cm[k] = nm;
      C.cr[k] = nr;
    }
    return;
  }
  if (live) {
    C.len[wr][k] = (uint8_t)L;
    C.prev[wr][k] = pv;
    C.pnull[wr][k] = pn ? 1 : 0;
#pragma unroll
    for (int i = 0; i < CSEQ_MAXM; i++) {
      const int s = i - (CSEQ_MAXM - M);
      if (s >= 0) {
        C.hseq[wr][cs_hslot(s, k, M)] = hs[i];
        C.hts[wr][cs_hslot(s, k, M)] = ht[i];
      }
    }
  }
  for (int d = 32; d > 0; d >>= 1) tmax = max(tmax, (int64_t)__shfl_xor((long long)tmax, d, 64));
  if (__lane_id() == 0 && tmax != INT64_MIN) atomicMax(C.tsmax, (unsigned long long)tmax ^ (1ull << 63));
  if (e) atomicOr(err, e);
}

static __global__ void k_cseq_init(CseqDev C) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int c = 0; c < 2; c++) {
    if (i < C.nk) {
      C.len[c][i] = 0;
      C.prev[c][i] = 0;
      C.pnull[c][i] = 1;
    }
    if (i < (int64_t)C.M * C.nk) {
      C.hseq[c][i] = -1;
      C.hts[c][i] = -1;
    }
  }
}

}  // namespace shp

#include "cseq_own.h"

namespace shp {

struct CseqState {
  CseqDev D{};

  template <class T>
  static void al(T*& p, int64_t n) {
    if (hipMalloc((void**)&p, std::max<int64_t>(n, 1) * sizeof(T)) != hipSuccess)
      throw std::runtime_error("hipMalloc failed (count-sequence path)");
  }

  int64_t cap = 0;
  bool scan64 = getenv("SHP_CSEQ_SCAN64") != nullptr;  // A/B: k_cs2 (a wave scan per 64 events)
  void* tmp = nullptr;  // the record sort's rocPRIM scratch
  size_t tmp_bytes = 0;

  // the records sorted with their keys (stable); CS_RADIX_BITS > 8: a onesweep config with that many
  // bits per pass (fewer passes over the 20 key bits of 1M keys)
  template <class R>
  void sort_records(void* t, size_t& tb, int64_t n, int key_bits, hipStream_t s) {
    R* pr = reinterpret_cast<R*>(D.pr);
    R* sr = reinterpret_cast<R*>(D.sr);
#if defined(CS_RADIX_BITS) && CS_RADIX_BITS != 8
    using Cfg = rocprim::radix_sort_config<
        rocprim::default_config, rocprim::default_config,
        rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 8>, rocprim::kernel_config<1024, 8>,
                                            CS_RADIX_BITS, rocprim::block_radix_rank_algorithm::match>>;
    (void)rocprim::radix_sort_pairs<Cfg>(t, tb, D.pk, D.sk, pr, sr, (size_t)n, 0, key_bits + 1, s);
#else
    (void)rocprim::radix_sort_pairs(t, tb, D.pk, D.sk, pr, sr, (size_t)n, 0, key_bits + 1, s);
#endif
  }

  // the owner path (cseq_own.h): CHAIN32 pushes whose keys and M fit its per-owner LDS state
  CoDev P{};
  bool own = false;
  uint32_t* ch = nullptr;  // CHAIN32 words staged for the expansion (mcap)
  bool ch_saved = false;   // this push's words are in `ch` (set by the first expansion, reset per push)
  int64_t mcap = 0;

  // owners and local keys for nk keys with M history slots: false when they do not fit
  static int mode_of(const CseqShape& s) {
    return s.every ? (s.minc <= 1 ? CS_EVERY1 : CS_EVERYN) : (s.minc <= 1 ? CS_ONCE1 : CS_ONCEN);
  }
  bool own_plan(int M, int mode, int32_t nk) {
    // without `every` (CS_ONCE1 and CS_ONCEN) a used once-armed start is the dead state D = M + 1,
    // which k_co_run's 8-byte tables hold only for M + 1 <= CO_MAXM
    if (M > CO_MAXM || ((mode == CS_ONCE1 || mode == CS_ONCEN) && M + 1 > CO_MAXM)) return false;
    const int per = 8 + 4 * M;  // value, L / null / ring head / ring fill, the ring
    int kmax = 1;
    while (kmax * 2 <= CO_KPO_MAX && kmax * 2 * per <= CO_KEY_LDS) kmax *= 2;
    const int64_t need = ((int64_t)nk + kmax - 1) / kmax;
    int64_t nown = 1, pk = 1;
    while (nown < need) nown *= 2;
    while (pk < nk) pk *= 2;
    nown = std::max<int64_t>(nown, std::min<int64_t>(CO_MINOWN, pk));
    if (const char* o = getenv("SHP_CO_OWN")) {  // A/B: a fixed owner count (a power of two)
      const int64_t x = atoll(o);
      if (x > 0 && (x & (x - 1)) == 0 && x * kmax >= nk) nown = x;
    }
    if (nown > CO_MAXOWN) return false;
    P.nown = (int32_t)nown;
    P.bits = 0;
    while ((1 << P.bits) < nown) P.bits++;
    P.kpo = (int32_t)(((int64_t)nk + nown - 1) >> P.bits);
    P.lkbits = 0;
    while ((1 << P.lkbits) < P.kpo) P.lkbits++;
    return true;
  }

  void create(const DevProg& Pg, const CseqShape& s, int32_t max_keys, int64_t batch_cap, int key_bits,
              hipStream_t st, bool chain32 = false, int64_t match_cap = 0) {
    cap = std::max<int64_t>(batch_cap, 1);
    al(D.pk, cap);
    al(D.sk, cap);
    al(D.pr, cap);
    al(D.sr, cap);
    const int64_t nwmax = cap / CS2_P + 2;
    al(D.ws, nwmax + 1);
    al(D.kend, std::max<int64_t>(max_keys, 1));
    (void)hipMemsetAsync(D.kend, 0, sizeof(unsigned long long) * std::max<int64_t>(max_keys, 1), st);
    D.epoch = 0;
    al(D.wcm, nwmax);
    al(D.wcr, nwmax);
    al(D.wom, nwmax);
    al(D.wor, nwmax);
    size_t b1 = 0, b2 = 0, b3 = 0;
    sort_records<CsRec>(nullptr, b1, cap, key_bits, st);
    sort_records<CsRec12>(nullptr, b3, cap, key_bits, st);
    (void)rocprim::exclusive_scan(nullptr, b2, D.wcm, D.wom, 0u, (size_t)nwmax, rocprim::plus<uint32_t>(), st);
    tmp_bytes = std::max<size_t>(std::max(std::max(b1, b2), b3), 16);
    D.ch32 = chain32 ? 1 : 0;
    if (chain32) {
      mcap = std::max<int64_t>(match_cap, 1);
      al(ch, mcap);
      size_t b4 = 0;
      (void)rocprim::exclusive_scan(nullptr, b4, rocprim::make_transform_iterator((const uint32_t*)ch, ChRefs{}),
                                    (int64_t*)nullptr, (int64_t)0, (size_t)mcap, rocprim::plus<int64_t>(), st);
      tmp_bytes = std::max(tmp_bytes, b4);
    }
    // the owner path takes CHAIN32 words and FULL rows alike (k_co_run); SHP_CO_OFF: the sorted records
    own = getenv("SHP_CO_OFF") == nullptr && (chain32 || getenv("SHP_CO_FULL_OFF") == nullptr) &&
          own_plan(s.M, mode_of(s), max_keys);
    {
      if (own) {
        const int64_t nst_max = (cap + CO_STLEN - 1) / CO_STLEN;
        const int64_t nc = (int64_t)P.nown * nst_max + 1;
        al(P.cnt, nc);
        al(P.off, nc);
        al(P.recs, cap);
        size_t b5 = 0;
        (void)rocprim::exclusive_scan(nullptr, b5, P.cnt, P.off, 0u, (size_t)nc, rocprim::plus<uint32_t>(), st);
        tmp_bytes = std::max(tmp_bytes, b5);
        const int dyn = (int)co_dyn_bytes(P.kpo, s.M);
        const void* runs[6] = {(const void*)k_co_run<0, false>, (const void*)k_co_run<1, false>,
                               (const void*)k_co_run<2, false>, (const void*)k_co_run<0, true>,
                               (const void*)k_co_run<1, true>,  (const void*)k_co_run<2, true>};
        for (const void* f : runs)
          if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, dyn) != hipSuccess)
            throw std::runtime_error("count-sequence owner path: LDS request refused");
      }
    }
    if (hipMalloc(&tmp, tmp_bytes) != hipSuccess) throw std::runtime_error("hipMalloc failed (count-sequence sort)");
    create_state(Pg, s, max_keys, st);
  }

  void create_state(const DevProg& P, const CseqShape& s, int32_t max_keys, hipStream_t st) {
    D.vtag = P.ncol == 1 ? P.colTag[0] : T_NULL;
    if (!SweepState::lower(s.f1, (int8_t)D.vtag, D.f1) || !SweepState::lower(s.f2, (int8_t)D.vtag, D.f2))
      throw std::runtime_error("count-sequence: predicate not lowerable");
    D.M = s.M;
    D.mode = mode_of(s);
    D.nk = max_keys;
    D.cur = 0;
    for (int c = 0; c < 2; c++) {
      al(D.len[c], max_keys);
      al(D.prev[c], max_keys);
      al(D.pnull[c], max_keys);
      al(D.hseq[c], (int64_t)s.M * max_keys);
      al(D.hts[c], (int64_t)s.M * max_keys);
    }
    al(D.tsmax, 1);
    al(D.cm, max_keys);
    al(D.cr, max_keys);
    al(D.om, max_keys);
    al(D.orf, max_keys);
    const int64_t n = (int64_t)s.M * max_keys;
    k_cseq_init<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(D);
  }

  // can the lowered predicates run here (f1 and f2 each at most two terms)?
  static bool shape_ok(const DevProg& P, const CseqShape& s) {
    if (!s.ok) return false;
    if (P.ncol == 1 && !(P.colTag[0] == T_INT || P.colTag[0] == T_FLOAT || P.colTag[0] == T_STR)) return false;
    SwPred a, b;
    const int8_t vt = P.ncol == 1 ? P.colTag[0] : T_NULL;
    return SweepState::lower(s.f1, vt, a) && SweepState::lower(s.f2, vt, b);
  }

  template <bool EMIT>
  void pass(const BatchView& B, const MatchOut& O, const uint32_t* perm, const uint32_t* kbeg, const uint32_t* kcnt,
            int* err, hipStream_t s) {
    const unsigned g = (unsigned)((D.nk + 255) / 256);
    switch (D.f1.n * 3 + D.f2.n) {
#define CS_CASE(a, b) \
  case a * 3 + b: k_cseq<a, b, EMIT><<<g, 256, 0, s>>>(D, B, O, perm, kbeg, kcnt, err); break;
      CS_CASE(0, 0) CS_CASE(0, 1) CS_CASE(0, 2) CS_CASE(1, 0) CS_CASE(1, 1) CS_CASE(1, 2)
      CS_CASE(2, 0) CS_CASE(2, 1) CS_CASE(2, 2)
#undef CS_CASE
      default: break;
    }
  }

  // count pass, placement scan over the keys (tmp: rocPRIM scratch of the engine), emit pass
  void run(const BatchView& B, const MatchOut& O, const uint32_t* perm, const uint32_t* kbeg, const uint32_t* kcnt,
           int* err, void* tmp, size_t tmp_bytes, hipStream_t s, KTimer& kt) {
    (void)hipMemsetAsync(D.tsmax, 0, sizeof(unsigned long long), s);
    kt.mark("cseq_count", s);
    pass<false>(B, O, perm, kbeg, kcnt, err, s);
    kt.mark("cseq_scan", s);
    size_t tb = tmp_bytes;
    (void)rocprim::exclusive_scan(tmp, tb, D.cm, D.om, 0u, (size_t)D.nk, rocprim::plus<uint32_t>(), s);
    tb = tmp_bytes;
    (void)rocprim::exclusive_scan(tmp, tb, D.cr, D.orf, 0u, (size_t)D.nk, rocprim::plus<uint32_t>(), s);
    kt.mark("cseq", s);
    pass<true>(B, O, perm, kbeg, kcnt, err, s);
    kt.mark(nullptr, s);
  }

  template <bool EMIT, class R>
  void pass2(const BatchView& B, const MatchOut& O, int64_t nw, int* err, hipStream_t s) {
    const unsigned g = (unsigned)((nw * 64 + 255) / 256);
    const R* sr = reinterpret_cast<const R*>(D.sr);
    switch (D.f1.n * 3 + D.f2.n) {
#define CS2_CASE(a, b) \
  case a * 3 + b:                                                                                \
    if (scan64)                                                                                  \
      k_cs2<a, b, EMIT, R><<<g, 256, 0, s>>>(D, B, O, D.sk, sr, D.ws, nw, err);                  \
    else                                                                                         \
      k_cs3<a, b, EMIT, R><<<g, 256, 0, s>>>(D, B, O, D.sk, sr, D.ws, nw, err);                  \
    break;
      CS2_CASE(0, 0) CS2_CASE(0, 1) CS2_CASE(0, 2) CS2_CASE(1, 0) CS2_CASE(1, 1) CS2_CASE(1, 2)
      CS2_CASE(2, 0) CS2_CASE(2, 1) CS2_CASE(2, 2)
#undef CS2_CASE
      default: break;
    }
  }

  // the round-3 form over one push (device columns): pack, sort the records with their keys,
  // wave ranges, count pass, scan over the waves, the state carried to copy wr, emit pass
  // narrow: the 12-byte records (a push beyond their ts range sets CS_WIDE; the engine re-runs it wide)
  void run2(const BatchView& B, const int32_t* key, const int32_t* stream, int key_bits, const MatchOut& O, int* err,
            hipStream_t s, KTimer& kt, bool narrow) {
    if (own && B.n > 0)
      run_own(B, key, stream, O, err, s, kt);
    else if (narrow)
      run2t<CsRec12>(B, key, stream, key_bits, O, err, s, kt);
    else
      run2t<CsRec>(B, key, stream, key_bits, O, err, s, kt);
  }

  template <class R>
  void run2t(const BatchView& B, const int32_t* key, const int32_t* stream, int key_bits, const MatchOut& O, int* err,
             hipStream_t s, KTimer& kt) {
    const int64_t n = B.n;
    (void)hipMemsetAsync(D.tsmax, 0, sizeof(unsigned long long), s);
    // the state of keys without events in this push passes to copy wr unchanged
    const int rd = D.cur, wr = D.cur ^ 1;
    const size_t nk = (size_t)D.nk, hm = (size_t)D.M * nk * 8;
    if (scan64 || n <= 0) {  // (k_cs3: k_cs_state passes the state of keys without events)
      (void)hipMemcpyAsync(D.len[wr], D.len[rd], nk, hipMemcpyDeviceToDevice, s);
      (void)hipMemcpyAsync(D.prev[wr], D.prev[rd], nk * 4, hipMemcpyDeviceToDevice, s);
      (void)hipMemcpyAsync(D.pnull[wr], D.pnull[rd], nk, hipMemcpyDeviceToDevice, s);
      (void)hipMemcpyAsync(D.hseq[wr], D.hseq[rd], hm, hipMemcpyDeviceToDevice, s);
      (void)hipMemcpyAsync(D.hts[wr], D.hts[rd], hm, hipMemcpyDeviceToDevice, s);
    }
    D.epoch++;
    if (D.epoch == 0) {  // (2^32 pushes) no stale run end may carry the new epoch
      (void)hipMemsetAsync(D.kend, 0, sizeof(unsigned long long) * nk, s);
      D.epoch = 1;
    }
    if (n <= 0) {
      (void)hipMemsetAsync(O.count, 0, 2 * sizeof(unsigned long long), s);
      return;
    }
    kt.mark("cs_pack", s);
    const unsigned gp = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
    k_cs_pack<R><<<gp, 256, 0, s>>>(B.ts, key, stream, (const uint32_t*)B.cols[0], B.nulls[0], n, B.partitioned,
                                    (uint32_t)D.nk, D.pk, reinterpret_cast<R*>(D.pr), D.tsmax, err);
    kt.mark("cs_sort", s);
    size_t tb = tmp_bytes;
    sort_records<R>(tmp, tb, n, key_bits, s);
    kt.mark("cs_count", s);
    const int64_t nw = (n + CS2_P - 1) / CS2_P;
    k_cs2_ranges<<<(unsigned)(((nw + 1) * 64 + 255) / 256), 256, 0, s>>>(D.sk, n, nw, D.ws);
    pass2<false, R>(B, O, nw, err, s);
    kt.mark("cs_scan", s);
    tb = tmp_bytes;
    (void)rocprim::exclusive_scan(tmp, tb, D.wcm, D.wom, 0u, (size_t)nw, rocprim::plus<uint32_t>(), s);
    tb = tmp_bytes;
    (void)rocprim::exclusive_scan(tmp, tb, D.wcr, D.wor, 0u, (size_t)nw, rocprim::plus<uint32_t>(), s);
    kt.mark("cs_emit", s);
    pass2<true, R>(B, O, nw, err, s);
    if (!scan64) {
      kt.mark("cs_state", s);
      k_cs_state<R><<<(unsigned)((D.nk + 255) / 256), 256, 0, s>>>(D, B, D.sk, reinterpret_cast<const R*>(D.sr));
    }
    kt.mark(nullptr, s);
  }

  // the owner path over one push (cseq_own.h): count, scan, scatter, per-owner run
  bool stg_attr = false;  // the staged scatter's LDS limit is set (once per engine)
  void run_own(const BatchView& B, const int32_t* key, const int32_t* stream, const MatchOut& O, int* err,
               hipStream_t s, KTimer& kt) {
    const int64_t n = B.n;
    P.nst = (int32_t)((n + CO_STLEN - 1) / CO_STLEN);
    if ((int64_t)P.nst * CO_STLEN < n || n > cap) throw std::runtime_error("count-sequence owner path: batch beyond capacity");
    (void)hipMemsetAsync(D.tsmax, 0, sizeof(unsigned long long), s);
    kt.mark("co_count", s);
    k_co_count<<<(unsigned)P.nst, CO_CNT_THREADS, 0, s>>>(P, B, key, stream, (uint32_t)D.nk, D.tsmax, err);
    kt.mark("co_scan", s);
    size_t tb = tmp_bytes;
    (void)rocprim::exclusive_scan(tmp, tb, P.cnt, P.off, 0u, (size_t)P.nown * P.nst + 1, rocprim::plus<uint32_t>(), s);
    kt.mark("co_scatter", s);
    const size_t lds = (size_t)(CO_SCT_WAVES + 1) * P.nown * 4;
    const bool pf = !stream && !B.nulls[0] && !getenv_flag_scatter_nopf();
    // the LDS-staged scatter (round 5: co_scatter 1.21 -> 1.08 ms on C3', profiles/r05_scatter_stage_ab.txt);
    // SHP_SCATTER_NOSTAGE=1 is the A/B back to the direct scattered stores
    static const bool nostage = getenv("SHP_SCATTER_NOSTAGE") != nullptr;
    const bool stg = pf && !nostage;
    const size_t stg_lds = (size_t)(CO_SCT_WAVES + 2) * P.nown * 4 + (size_t)4 * CO_SCT_ROUND * 4;
    if (stg && !stg_attr) {
      const void* fs[3] = {(const void*)k_co_scatter<0, true, true>, (const void*)k_co_scatter<1, true, true>,
                           (const void*)k_co_scatter<2, true, true>};
      for (const void* f : fs)
        if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)((size_t)(CO_SCT_WAVES + 2) * CO_MAXOWN * 4 + (size_t)4 * CO_SCT_ROUND * 4)) !=
            hipSuccess)
          throw std::runtime_error("count-sequence: staged scatter LDS request refused");
      stg_attr = true;
    }
#define CO_SCT(N)                                                                              \
  if (stg) {                                                                                   \
    k_co_scatter<N, true, true><<<(unsigned)P.nst, CO_SCT_THREADS, stg_lds, s>>>(P, D, B, key, stream); \
  } else if (pf) k_co_scatter<N, true><<<(unsigned)P.nst, CO_SCT_THREADS, lds, s>>>(P, D, B, key, stream); \
  else k_co_scatter<N, false><<<(unsigned)P.nst, CO_SCT_THREADS, lds, s>>>(P, D, B, key, stream);
    switch (D.f1.n) {
      case 0: CO_SCT(0) break;
      case 1: CO_SCT(1) break;
      default: CO_SCT(2) break;
    }
#undef CO_SCT
    kt.mark("co_run", s);
    const size_t dyn = co_dyn_bytes(P.kpo, D.M);
    switch (D.f2.n) {
#define CO_RUN(N)                                                                           \
  if (D.ch32) k_co_run<N, false><<<(unsigned)P.nown, CO_THREADS, dyn, s>>>(P, D, B, O, err); \
  else k_co_run<N, true><<<(unsigned)P.nown, CO_THREADS, dyn, s>>>(P, D, B, O, err);
      case 0: CO_RUN(0) break;
      case 1: CO_RUN(1) break;
      default: CO_RUN(2) break;
#undef CO_RUN
    }
    kt.mark(nullptr, s);
  }

  // CHAIN32 -> FULL for the last push's m words (in O.refs), after its commit: the push's events
  // sorted by key again (the 16-byte records), each match's refs placed by a scan of L + 1
  void expand(const BatchView& B, const int32_t* key, const int32_t* stream, int key_bits, const MatchOut& O, int64_t m,
              int* err, hipStream_t s, KTimer& kt) {
    if (m <= 0 || B.n <= 0) {
      (void)hipMemsetAsync(O.count + 1, 0, sizeof(unsigned long long), s);
      return;
    }
    if (m > mcap) throw std::runtime_error("count-sequence expansion: more matches than the staging buffer");
    const int64_t n = B.n;
    kt.mark("cs_expand", s);
    // the words move to `ch` once per push: an expansion that failed (and overwrote part of O.refs
    // with FULL refs) re-runs from `ch`
    if (!ch_saved) (void)hipMemcpyAsync(ch, O.refs, (size_t)m * 4, hipMemcpyDeviceToDevice, s);
    ch_saved = true;
    const unsigned gp = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
    k_cs_pack<CsRec><<<gp, 256, 0, s>>>(B.ts, key, stream, (const uint32_t*)B.cols[0], B.nulls[0], n, B.partitioned,
                                        (uint32_t)D.nk, D.pk, D.pr, D.tsmax, err);
    size_t tb = tmp_bytes;
    sort_records<CsRec>(tmp, tb, n, key_bits, s);
    tb = tmp_bytes;
    (void)rocprim::exclusive_scan(tmp, tb, rocprim::make_transform_iterator((const uint32_t*)ch, ChRefs{}), O.ref_off,
                                  (int64_t)0, (size_t)m, rocprim::plus<int64_t>(), s);
    const unsigned ge = (unsigned)std::min<int64_t>((m + 255) / 256, 4096);
    k_cs_expand<CsRec><<<ge, 256, 0, s>>>(D, B, key, D.sk, D.sr, ch, m, D.cur ^ 1, O, err);
    kt.mark(nullptr, s);
  }

  void commit() { D.cur ^= 1; }

  void release() {
    for (int c = 0; c < 2; c++) {
      void* ps[] = {D.len[c], D.prev[c], D.pnull[c], D.hseq[c], D.hts[c]};
      for (void* p : ps)
        if (p) (void)hipFree(p);
    }
    void* qs[] = {D.tsmax, D.cm, D.cr, D.om, D.orf, D.pk, D.sk, D.pr, D.sr, D.ws, D.wcm, D.wcr, D.wom, D.wor, D.kend, tmp,
                  ch, P.cnt, P.off, P.recs};
    for (void* p : qs)
      if (p) (void)hipFree(p);
    D = CseqDev{};
    P = CoDev{};
    tmp = nullptr;
    ch = nullptr;
    own = false;
  }
};

}  // namespace shp
