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
// Kernels: the batch is partitioned by key with the engine's stable radix sort (as for the
// general lanes); k_cseq runs one thread per key over the key's events in arrival order, with
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

#include <stdexcept>

#include "nfa_lane.h"
#include "prog.h"
#include "sweep.h"

namespace shp {

struct CseqDev {
  SwPred f1, f2;     // f1: e1 slot = the arriving event; f2: e1 slot = e1[last], e2 slot = the arriving event
  int32_t M, vtag, nk, cur;
  uint8_t* len[2];   // nk: L
  uint32_t* prev[2]; // nk: the previous event's value bits
  uint8_t* pnull[2]; // nk: ... and whether it was null
  int64_t* hseq[2];  // M * nk: seq of the key's last M events (slot M-1 = the latest), -1 none
  int64_t* hts[2];   // M * nk: their ts
  unsigned long long* tsmax;  // max ts of the push as ts ^ 2^63 (0: no event)
  uint32_t *cm, *cr;  // nk: records and refs per key (pass 1), then their exclusive scans
  uint32_t *om, *orf;
};

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
        hs[i] = C.hseq[rd][(int64_t)s * C.nk + k];
        ht[i] = C.hts[rd][(int64_t)s * C.nk + k];
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
        C.hseq[wr][(int64_t)s * C.nk + k] = hs[i];
        C.hts[wr][(int64_t)s * C.nk + k] = ht[i];
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

struct CseqState {
  CseqDev D{};

  template <class T>
  static void al(T*& p, int64_t n) {
    if (hipMalloc((void**)&p, std::max<int64_t>(n, 1) * sizeof(T)) != hipSuccess)
      throw std::runtime_error("hipMalloc failed (count-sequence path)");
  }

  void create(const DevProg& P, const CseqShape& s, int32_t max_keys, hipStream_t st) {
    D.vtag = P.ncol == 1 ? P.colTag[0] : T_NULL;
    if (!SweepState::lower(s.f1, (int8_t)D.vtag, D.f1) || !SweepState::lower(s.f2, (int8_t)D.vtag, D.f2))
      throw std::runtime_error("count-sequence: predicate not lowerable");
    D.M = s.M;
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

  void commit() { D.cur ^= 1; }

  void release() {
    for (int c = 0; c < 2; c++) {
      void* ps[] = {D.len[c], D.prev[c], D.pnull[c], D.hseq[c], D.hts[c]};
      for (void* p : ps)
        if (p) (void)hipFree(p);
    }
    void* qs[] = {D.tsmax, D.cm, D.cr, D.om, D.orf};
    for (void* p : qs)
      if (p) (void)hipFree(p);
    D = CseqDev{};
  }
};

}  // namespace shp
