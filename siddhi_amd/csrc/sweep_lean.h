// siddhi-hip: k_sw_lean, the sweep solve for the common 2-state shape (included by sweep.h).
//
// Same semantics and output as k_sw_solve (StreamPreStateProcessor
// .processAndReturn / expireEvents :326-403): per key, candidate i (e1's filter, evaluated by the
// scatter) closes at the first later event j of the key with ts_j - ts_i <= W and f2(i, j), and
// expires at the first later event beyond W; matches per key in (j, i) order.
//
// It covers the shape the headline configs use -- one f2 term `e2.v OP e1.v` or `e2.v OP const`
// over a float or int column compared in its own type, no nulls, pair layouts -- and keeps every
// quantity of the per-chunk work 32-bit.  Anything outside that (a push whose timestamps leave
// base +- 2^30 ms, a key whose timestamps decrease, a carry beyond SL_CCAP, a closing event with
// more than 255 far candidates) raises SWE_LEAN: the engine then re-runs the solve of the same
// push with k_sw_solve, which is exact for all of them.  The two kernels share the per-owner
// state in HBM (carry in key order, absolute ts), so either can continue from the other.
//
// Structure per chunk of SL_CHUNK records of the owner (512 threads, 3 block barriers):
//   rank    stable ranks by local key (wave ballots, per-wave counters)          | barrier A
//   scan    wave 0: key run offsets (carried first), write cursors, and the split
//           of the sorted positions into 8 wave ranges aligned to key runs         | barrier B
//   place   records and carried candidates at their sorted positions             | barrier C
//   then every wave works alone on its range (whole key runs, so nothing crosses waves):
//   probe   each candidate tests the next SW_P1 events of its key; unresolved ones go to the
//           wave's worklist (SW_P2 events per round).  A closer records its distance in a
//           32-bit word of the closing event: bits 0..23 = distance 1..24, bits 24..31 = count
//           of farther ones.
//   scan    per lane a contiguous block of positions: closes and still-open candidates, one
//           wave scan, one LDS atomic for the wave's carry slots; open candidates are compacted
//           (key order) as the next carry.  The last wave through reserves the chunk's output
//           with one global atomic (per-wave global atomics were measured 2.7x slower: 400k
//           same-address atomics per launch serialise).
//   emit    between barriers A and B of the next chunk (the chunk's positions are intact until
//           the next place step): a candidate's rank among its closer's candidates is the
//           popcount of the nearer distance bits, so each match is written straight to its slot.
#pragma once

namespace shp {

constexpr int SL_THREADS = 512;
constexpr int SL_WAVES = SL_THREADS / 64;
constexpr int SL_R = 4;                       // records per thread per chunk
constexpr int SL_CHUNK = SL_THREADS * SL_R;   // 2048
constexpr int SL_CCAP = 384;                  // carried candidates per owner (<= SWS_CCAP)
constexpr int SL_EMAX = SL_CHUNK + SL_CCAP;
constexpr int SL_PAD = 16;                    // sentinel positions past E (probe reads)
constexpr int SL_WL = 120;                    // worklist entries per wave (drained from SL_WLD on)
constexpr int SL_WLD = 56;
constexpr int SL_NEAR = 24;                   // closer distances kept as bits
#ifndef SL_P1_CFG
#define SL_P1_CFG SW_P1
#endif
#ifndef SL_P2_CFG
#define SL_P2_CFG SW_P2
#endif
constexpr int SL_P1 = SL_P1_CFG;              // first-round probes per candidate
constexpr int SL_P2 = SL_P2_CFG;              // probes per worklist round
static_assert(SL_P1 < SL_PAD && SL_P2 < SL_PAD, "probes read at most SL_PAD sentinels past E");
static_assert(SL_CCAP <= SWS_CCAP, "lean carry must fit the HBM carry arrays");

struct SwLeanSmem {
  int2 tv[SL_EMAX + SL_PAD];         // (ts - chunk base, value) by sorted position; later x = output offset
  uint32_t ref[SL_EMAX];             // batch index, or carry slot (carried)
  uint32_t cl[SL_EMAX];              // closers of this position: distance bits | far count << 24
  uint32_t meta[SL_EMAX + SL_PAD];   // local key | key run end << 8 | first event of the run << 20
                                     // (carried: position < first event; e1's filter: ref bit 31)
  int16_t m[SL_EMAX];                // >= 0 closing position, -1 expired, -2 open, -3 not a candidate
  uint16_t wc[SL_WAVES][256];        // per-wave rank counters, then write cursors
  uint32_t binoff[257];              // key run starts (then, at the end, key-order carry offsets)
  uint16_t fe[256];                  // first event position of a key's run (after its carried)
  uint32_t ncar[256];                // carried candidates of a key in the current carry buffer
  uint16_t ckf[2][256];              // index of a key's first entry in carry buffer 0/1
  uint8_t lastc[256];                // the key's latest event opened a candidate (SweepDev::lastc)
  int32_t cts[2][SL_CCAP];           // carry: ts - batch base (exact; a carry beyond +-2^31 ms: SWE_LEAN)
  int32_t cseq[2][SL_CCAP];          // carry: seq - the push's first seq (exact; beyond +-2^31: SWE_LEAN)
  uint32_t cv[2][SL_CCAP];
  uint8_t clk[2][SL_CCAP];
  uint32_t wl[SL_WAVES][SL_WL];      // worklists: position | next probe position << 16
  int32_t ps[SL_WAVES + 1];          // wave ranges of sorted positions
  int32_t cn[2];                     // entries in carry buffer 0/1
  uint32_t wtot[SL_WAVES];
  uint32_t wt[SL_WAVES], wb[SL_WAVES];  // matches per wave in the chunk, and their offsets
  unsigned long long gbase;           // the chunk's output range (one global atomic per chunk)
  int32_t done;                       // waves through the chunk's reservation step
  int32_t scanner[2];                 // the wave that runs the scan step of even / odd chunks
  int32_t flag;
};

template <int CT, int OPC, int P>
__device__ __forceinline__ int sl_probe(const int2* tv, int qb, int end, int32_t a_ts, int32_t W,
                                        typename SwTy<CT>::T b) {
  int2 x[P];
#pragma unroll
  for (int d = 0; d < P; d++) x[d] = tv[qb + d];
  int res = -4;
#pragma unroll
  for (int d = 0; d < P; d++) {
    const bool hit = sw_cmp_op<OPC>(0, sw_val<CT>((uint32_t)x[d].y, 0.0, 0.0, false), b);
    const int r = qb + d >= end ? -2 : (x[d].x - a_ts > W ? -1 : (hit ? qb + d : -4));
    res = res == -4 ? r : res;
  }
  return res;
}

__device__ __forceinline__ uint32_t sl_closes(uint32_t c) { return (uint32_t)__popc(c & 0xFFFFFFu) + (c >> 24); }

// One lane per match for a 64-position block of the AGG emission: the block's matches are the
// consecutive indices [0, T) (lane q's c matches from ex = exclusive scan of c), taken 64 at a time;
// index t's source lane is the last one whose first index is <= t: each source writes its lane at
// its first index inside the window (a byte of the wave's scratch), the rest of the window keeps 0,
// and a max scan fills the gaps (sources increase with the index).  out(t, src, r) writes the match
// t, the r-th of lane src.  Every lane of the wave calls it (DPP moves, shuffles).
// (scr: LDS.  The fence keeps the compiler from forwarding a lane's own store to its load -- the
// load must see the other lanes' stores; the LDS runs one wave's operations in order.)
template <class Out>
__device__ __forceinline__ void sl_expand_block(uint8_t* scr, uint32_t lane, uint32_t c, uint32_t ex, uint32_t T,
                                                Out&& out) {
  for (uint32_t t0 = 0; t0 < T; t0 += 64) {
    scr[lane] = 0;
    if (c && ex < t0 + 64u && ex + c > t0) scr[(ex > t0 ? ex : t0) - t0] = (uint8_t)lane;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    uint32_t j = scr[lane];
    dpp_scan_steps(lane, [&](auto ctl, bool take) {
      const uint32_t y = dpp32<decltype(ctl)::value>(j);
      if (take) j = y > j ? y : j;
    });
    const uint32_t sex = (uint32_t)__shfl((int)ex, (int)j, 64);
    out(t0 + lane, (int)j, t0 + lane - sex, t0 + lane < T);
  }
}

// AGG: SHP_LAYOUT_AGG -- the selector's running aggregate per match
// (QuerySelector.processInBatchNoGroupBy) in place of the pairs: avg / sum / count (D.agg 1..3;
// AvgAttributeAggregatorExecutor: `value += x; count++`) and, since round 4, min / max (D.agg 4 / 5;
// MinAttributeAggregatorExecutor.java:126-130, bit-exact with k_sw_solve's fold)
// HS: the batch carries a seq column (B.seq).  A template parameter, not a branch: with both
// variants in one body the compiler's wait counters, merging the variant that loads seqs with the
// one that does not, held the emission's stores at the scanner step (s_waitcnt vmcnt(0)).
// R: the scatter's record form (SwRec12 for the pushes it takes since round 5, SwRec after a k_sw_win
// hand-back)
template <int CT, int OPC, bool AGG = false, bool HS = false, class R = SwRec12>
__global__ __launch_bounds__(SL_THREADS, 4) void k_sw_lean(SweepDev D, BatchView B, MatchOut O, int* err) {
  const R* recs = reinterpret_cast<const R*>(D.recs);
  using T = typename SwTy<CT>::T;
  __shared__ SwLeanSmem S;
  __shared__ double ag[AGG ? 2 * 256 : 1];  // AGG: per local key (running sum, count) before the chunk emitted next
  const int o = blockIdx.x;
  const uint32_t tid = threadIdx.x, lane = __lane_id(), w = tid >> 6;
  const uint64_t lt = sw_lanemask_lt();
  const int64_t rb = D.off[(int64_t)o * D.nst], re = D.off[(int64_t)(o + 1) * D.nst];
  const int rd = D.cur, wr = D.cur ^ 1;
  if (D.spill_on && D.spilled[rd][o]) return;  // k_sw_spill solves this owner
  if (rb == re) {  // no events for this owner: its state passes through unchanged
    const int n0 = D.c_n[rd][o];
    for (int i = tid; i < n0; i += SL_THREADS) {
      const int64_t c = (int64_t)o * SWS_CCAP + i;
      D.c_ts[wr][c] = D.c_ts[rd][c];
      D.c_seq[wr][c] = D.c_seq[rd][c];
      D.c_v[wr][c] = D.c_v[rd][c];
      D.c_lk[wr][c] = D.c_lk[rd][c];
      D.c_null[wr][c] = D.c_null[rd][c];
    }
    for (int i = tid; i < SW_LK; i += SL_THREADS) {
      const int64_t k = (int64_t)o * SW_LK + i;
      D.lastc[wr][k] = D.lastc[rd][k];
      if constexpr (AGG) {
        D.agg_s[wr][k] = D.agg_s[rd][k];
        D.agg_c[wr][k] = D.agg_c[rd][k];
      }
    }
    if (tid == 0) D.c_n[wr][o] = n0;
    return;
  }
  const int nc0 = D.c_n[rd][o];
  // the scatter saw a ts beyond base +- 2^30 (batch-relative ts are 32-bit here), or the carry
  // is larger than the lean kernel holds
  if (D.tsmax[1] != 0 || nc0 > SL_CCAP) {
    if (tid == 0) atomicOr(err, SWE_LEAN);
    return;
  }
  const int64_t base = B.ts[0];
  const int64_t sbase = HS ? B.seq[0] : B.seq0;  // carried seqs are kept relative to it
  const int32_t W = (int32_t)D.within;  // <= SW_TS_SPAN (SweepState::shape_ok)
  const SwTerm t2 = D.f2.t[0];
  const bool bconst = t2.bk == 0;
  const T bc = (T)t2.bc;
  const int lkbits = D.lk_bits;
  const int nb = lkbits >= 8 ? SW_LK : (1 << lkbits);  // local keys 0..nb-1
  int e = 0;
  for (int i = tid; i < 256; i += SL_THREADS) {
    S.ncar[i] = 0;
    S.ckf[0][i] = 0;
    S.lastc[i] = i < SW_LK ? D.lastc[rd][(int64_t)o * SW_LK + i] : 0;
  }
  for (int i = tid; i < SL_WAVES * 256; i += SL_THREADS) (&S.wc[0][0])[i] = 0;
  if constexpr (AGG)
    for (int i = tid; i < SW_LK; i += SL_THREADS) {
      ag[i] = D.agg_s[rd][(int64_t)o * SW_LK + i];
      ag[256 + i] = D.agg_c[rd][(int64_t)o * SW_LK + i];
    }
  if (tid == 0) {
    S.flag = 0;
    S.done = 0;
    S.scanner[0] = S.scanner[1] = 0;
    S.cn[0] = nc0;
    S.cn[1] = 0;
  }
  __syncthreads();
  // carry from the previous push (key order): counts and first index per key
  for (int x = tid; x < nc0; x += SL_THREADS) {
    const int64_t c = (int64_t)o * SWS_CCAP + x;
    const uint32_t lk = D.c_lk[rd][c];
    const int64_t dts = D.c_ts[rd][c] - base, dsq = D.c_seq[rd][c] - sbase;
    if (dts != (int64_t)(int32_t)dts || dsq != (int64_t)(int32_t)dsq) S.flag = 1;  // the exact kernel
    S.cts[0][x] = (int32_t)dts;
    S.cv[0][x] = D.c_v[rd][c];
    S.cseq[0][x] = (int32_t)dsq;
    S.clk[0][x] = (uint8_t)lk;
    atomicAdd(&S.ncar[lk], 1u);
    if (x == 0 || D.c_lk[rd][c - 1] != lk) S.ckf[0][lk] = (uint16_t)x;
  }
  int cur = 0;
  using RR = SwRecReg<R>;
  constexpr bool R12 = std::is_same<R, SwRec12>::value;
  typename RR::T pf[SL_R];
  // (12-byte records: every lane loads, past the region's end its last record -- unused -- so the
  // loads land in the loop's registers instead of merging with their old values)
  auto pload = [&](int64_t i, typename RR::T& x) __attribute__((always_inline)) {
    if constexpr (R12) x = RR::load(recs, min(i, re - 1));
    else if (i < re) x = RR::load(recs, i);
  };
#pragma unroll
  for (int s = 0; s < SL_R; s++) pload(rb + (int)w * (64 * SL_R) + s * 64 + (int)lane, pf[s]);
  auto rawkt = [&](int64_t i) __attribute__((always_inline)) -> uint64_t { return (uint64_t)recs[i].kt; };
  uint64_t tbk = rawkt(rb);  // (decoded where the chunk starts)
  // 6. emit (a chunk's matches are written between barriers A and B of the next chunk, once the
  //    last wave through the chunk has reserved its output range with one global atomic):
  //    slot = offset(q) + (closes(q) - 1 - later), later = closers of q nearer than p
  // (has_seq: the batch's seq column is present.  Without it the loop issues no global load, so the
  // compiler's wait counters do not hold each 64-position block for the previous block's stores)
  auto emit = [&](int PS, int PE, int pc, auto has_seq) {
    constexpr bool ES = decltype(has_seq)::value;
    auto seq_of = [&](uint32_t g) -> int64_t { return ES ? B.seq[g] : B.seq0 + (int64_t)g; };
    const unsigned long long gb = S.gbase + S.wb[w];
    for (int g = PS; g < PE; g += 64) {
      const int p = g + (int)lane;
      if (p >= PE) continue;
      const int q = S.m[p];
      if (q < 0) continue;
      const uint32_t c = S.cl[q];
      const int d = q - p;
      uint32_t later;
      if (d <= SL_NEAR) {
        later = (uint32_t)__popc(c & ((1u << (d - 1)) - 1u));
      } else {
        later = (uint32_t)__popc(c & 0xFFFFFFu);
        for (int p2 = p + 1; p2 < q - SL_NEAR; p2++) later += S.m[p2] == q ? 1u : 0u;
      }
      const uint32_t r = S.ref[p] & 0x7FFFFFFFu, rq = S.ref[q] & 0x7FFFFFFFu;
      const int64_t si = p < (int)(S.meta[p] >> 20) ? sbase + S.cseq[pc][r] : seq_of(r);
      const int64_t sq = seq_of(rq);
      const uint64_t slot = gb + (uint32_t)S.tv[q].x + (sl_closes(c) - 1u - later);
      if (slot < (uint64_t)O.cap) {
        if (D.p32) {
          const int64_t dq = sq - si;
          if (dq >= (1ll << 32)) e |= SWE_P32;
          reinterpret_cast<uint2*>(O.refs)[slot] = make_uint2(rq, (uint32_t)dq);
        } else if (ES) {
          *(longlong2*)(O.refs + 2 * slot) = make_longlong2(si, (int64_t)rq);
        } else {
          *(longlong2*)(O.refs + 2 * slot) = make_longlong2(si, sq);
        }
      }
    }
  };
  // AGG emission of the chunk a wave finished (between barriers A and B of the next chunk, like the
  // pairs): per closing position q in key order, the key's (sum, count) before q by a segmented
  // wave scan (segments = key runs, seeded with the key's state), then q's c matches: the r-th adds
  // q's value once more, (S + (r+1) v) / (N + r + 1) for avg -- k_sw_solve's arithmetic.
  // the AGG emissions' per-wave scratch: the wave's worklist, idle from its probe to the next one
  uint8_t* scr = reinterpret_cast<uint8_t*>(&S.wl[w][0]);
  auto emit_agg = [&](int PS, int PE) {
    const unsigned long long gb = S.gbase + S.wb[w];
    double cs = 0;               // the running state at the end of the previous 64-block
    uint32_t cn = 0;
    uint32_t clk = 0xFFFFFFFFu;  // ... and its key
    for (int g0 = PS; g0 < PE; g0 += 64) {
      const int q = g0 + (int)lane;
      const bool v = q < PE;
      const uint32_t lk = v ? (S.meta[q] & 0xFFu) : 0xFFFFu;
      const uint32_t c = v ? sl_closes(S.cl[q]) : 0u;
      const uint32_t vb = v ? (uint32_t)S.tv[q].y : 0u;
      const double x = CT == 1 ? (double)__uint_as_float(vb) : (double)(int32_t)vb;
      const uint32_t lkp = __shfl_up(lk, 1, 64);
      const bool head = lane == 0 || lk != lkp;
      double s0 = 0;
      uint32_t n0 = 0;  // (counts are integers: 32-bit in the scan, one shuffle a step fewer)
      if (head && v) {
        if (lane == 0 && lk == clk) {
          s0 = cs;
          n0 = cn;
        } else {
          s0 = ag[lk];
          n0 = (uint32_t)ag[256 + lk];
        }
      }
      double is = (head ? s0 : 0.0) + (double)c * x;
      uint32_t in = (head ? n0 : 0u) + c;
      uint32_t f = head ? 1u : 0u;
      dpp_scan_steps(lane, [&](auto ctl, bool take) {  // segmented (sum, count) scan, DPP moves
        constexpr int C = decltype(ctl)::value;
        const double ys = dppf64<C>(is);
        const uint32_t yn = dpp32<C>(in), yf = dpp32<C>(f);
        if (take && !f) {
          is += ys;
          in += yn;
        }
        if (take) f |= yf;
      });
      const double ps = __shfl_up(is, 1, 64);
      const uint32_t pn = __shfl_up(in, 1, 64);
      const double es = head ? s0 : ps;  // the key's state before q
      const uint32_t en = head ? n0 : pn;
      const uint32_t cx = dpp_incl_add(c, lane);
      const uint32_t T = wave_last(cx);
      if (T) {  // (S + (r+1) x) / (N + r + 1) for the r-th match of q, one lane per match
        const uint64_t s0b = gb + (uint32_t)S.tv[g0].x;  // the block's first match (lane 0 is valid)
        sl_expand_block(scr, lane, c, cx - c, T, [&](uint32_t t, int j, uint32_t r, bool ok) {
          const double ses = __shfl(es, j, 64);
          const uint32_t sen = (uint32_t)__shfl((int)en, j, 64), svb = (uint32_t)__shfl((int)vb, j, 64);
          const uint32_t slk = (uint32_t)__shfl((int)lk, j, 64);
          const uint64_t slot = s0b + t;
          if (ok && slot < (uint64_t)O.cap) {
            const double sx = CT == 1 ? (double)__uint_as_float(svb) : (double)(int32_t)svb;
            const double sr = ses + (double)(r + 1) * sx, nr = (double)(sen + r + 1);
            O.key[slot] = (int32_t)((slk << D.own_bits) | (uint32_t)o);  // (sw_owner / sw_local inverted)
            O.agg[slot] = D.agg == 1 ? sr / nr : (D.agg == 2 ? sr : nr);
          }
        });
      }
      if (v && (q + 1 >= PE || (S.meta[q + 1] & 0xFFu) != lk)) {  // the run's end: the key's new state
        ag[lk] = is;
        ag[256 + lk] = (double)in;
      }
      cs = wave_last_f64(is);
      cn = wave_last(in);
      clk = wave_last(lk);
    }
  };
  // AGG with min / max (D.agg 4 / 5; MinAttributeAggregatorExecutor / Max...: value = first value,
  // then `if (value > x) value = x`): a segmented wave scan of k_sw_solve's fold (best non-NaN
  // value, count, first value was NaN) over the closing positions; every match of q outputs the
  // fold after q's value (folding the same value again changes nothing).  The per-key state in
  // ag[] is (value -- NaN when the first value was NaN, 0 before any --, count), as k_sw_solve keeps it.
  auto emit_mm = [&](int PS, int PE, bool MAX) {
    const unsigned long long gb = S.gbase + S.wb[w];
    const double ident = MAX ? -INFINITY : INFINITY;
    auto best = [&](double a, double b) { return MAX ? (a < b ? b : a) : (a > b ? b : a); };  // a folded first
    double cm = ident, cn = 0;   // the running fold at the end of the previous 64-block
    int cfn = 0;
    uint32_t clk = 0xFFFFFFFFu;  // ... and its key
    for (int g0 = PS; g0 < PE; g0 += 64) {
      const int q = g0 + (int)lane;
      const bool v = q < PE;
      const uint32_t lk = v ? (S.meta[q] & 0xFFu) : 0xFFFFu;
      const uint32_t c = v ? sl_closes(S.cl[q]) : 0u;
      const uint32_t vb = v ? (uint32_t)S.tv[q].y : 0u;
      const double x = CT == 1 ? (double)__uint_as_float(vb) : (double)(int32_t)vb;
      const uint32_t lkp = __shfl_up(lk, 1, 64);
      const bool head = lane == 0 || lk != lkp;
      double m = ident, n = 0;
      int fn = 0;
      if (head && v) {  // the key's fold before this block: carried from the previous block or from ag[]
        if (lane == 0 && lk == clk) {
          m = cm;
          n = cn;
          fn = cfn;
        } else {
          const double sv = ag[lk];
          n = ag[256 + lk];
          fn = n > 0 && sv != sv;
          m = (n > 0 && !fn) ? sv : ident;
        }
      }
      if (c) {  // fold q's value once, count its c matches
        if (n == 0) {
          fn = x != x;
          m = fn ? ident : x;
        } else if (x == x) {
          m = best(m, x);
        }
        n += (double)c;
      }
      uint32_t f = head ? 1u : 0u, fnu = (uint32_t)fn;
      dpp_scan_steps(lane, [&](auto ctl, bool take) {  // segmented fold scan, DPP moves
        constexpr int C = decltype(ctl)::value;
        const double ym = dppf64<C>(m), yn = dppf64<C>(n);
        const uint32_t yfn = dpp32<C>(fnu), yf = dpp32<C>(f);
        if (take && !f) {
          m = best(ym, m);
          fnu = yn > 0 ? yfn : fnu;
          n = yn + n;
        }
        if (take) f |= yf;
      });
      fn = (int)fnu;
      const uint32_t cx = dpp_incl_add(c, lane);
      const uint32_t T = wave_last(cx);
      if (T) {  // every match of q outputs the fold after q, one lane per match
        const double val = fn ? __longlong_as_double(0x7ff8000000000000ll) : m;
        const uint64_t s0b = gb + (uint32_t)S.tv[g0].x;  // the block's first match (lane 0 is valid)
        sl_expand_block(scr, lane, c, cx - c, T, [&](uint32_t t, int j, uint32_t, bool ok) {
          const double sval = __shfl(val, j, 64);
          const uint32_t slk = (uint32_t)__shfl((int)lk, j, 64);
          const uint64_t slot = s0b + t;
          if (ok && slot < (uint64_t)O.cap) {
            O.key[slot] = (int32_t)((slk << D.own_bits) | (uint32_t)o);  // (sw_owner / sw_local inverted)
            O.agg[slot] = sval;
          }
        });
      }
      if (v && (q + 1 >= PE || (S.meta[q + 1] & 0xFFu) != lk)) {  // the run's end: the key's new state
        ag[lk] = n == 0 ? 0.0 : (fn ? __longlong_as_double(0x7ff8000000000000ll) : m);
        ag[256 + lk] = n;
      }
      cm = wave_last_f64(m);
      cn = wave_last_f64(n);
      cfn = (int)wave_last((uint32_t)fn);
      clk = wave_last(lk);
    }
  };
  int pPS = 0, pPE = 0, pcur = 0;  // this wave's range of the previous chunk, and its carry buffer
  unsigned long long gres = 0;     // (lane 0 of the chunk's last wave) the reserved output base,
  uint32_t gres_t = 0;             // the chunk's match count,
  bool gpend = false;              // and whether S.gbase still has to take them
  auto publish = [&]() {
    if (gpend) {
      if (gres + gres_t > (unsigned long long)O.cap) e |= E_OUT;
      S.gbase = gres;
      gpend = false;
    }
  };
#ifdef SHP_SW_STAMPS  // diagnostic build: wave cycles per phase (barrier waits count in the phase before)
  unsigned long long stc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t stp = clock64();
#define SL_STAMP(k)                 \
  do {                              \
    const uint64_t t_ = clock64();  \
    stc[k] += t_ - stp;             \
    stp = t_;                       \
  } while (0)
#else
#define SL_STAMP(k) \
  do {              \
  } while (0)
#endif
  __syncthreads();
  int ci = 0;  // chunk counter (the scanner of a chunk is chosen by the one before)
  for (int64_t cb = rb; cb < re; cb += SL_CHUNK, ci++) {
    const int nchunk = (int)min((int64_t)SL_CHUNK, re - cb);
    const int nx = cur ^ 1;
    const int32_t tb32 = R12 ? sw_rec_ts32(SwRec12{(uint32_t)tbk, 0u, 0u}) : (int32_t)(uint32_t)tbk;  // chunk base, batch-relative
    // 1. rank by local key (stable: wave-major, then slot, then lane = arrival order)
    uint32_t rk[SL_R], bin[SL_R];
#pragma unroll
    for (int s = 0; s < SL_R; s++) {
      const int j = (int)w * (64 * SL_R) + s * 64 + (int)lane;
      const bool valid = j < nchunk;
      const uint32_t lk = valid ? sw_rec_lk(pf[s]) : 0u;
      const uint64_t peers = sw_match_peers(lk, lkbits, valid);
      bin[s] = valid ? lk : 0xFFFFu;
      rk[s] = 0;
      if (valid) {
        const uint32_t before = S.wc[w][lk];
        rk[s] = before + (uint32_t)__popcll(peers & lt);
        if ((peers & lt) == 0) S.wc[w][lk] = (uint16_t)(before + (uint32_t)__popcll(peers));
      }
    }
    publish();
    __syncthreads();  // A
    SL_STAMP(0);
    // flags raised by the previous chunk are read here, where no thread writes S.flag (all
    // threads take the same branch)
    if (S.flag) break;
    if (cb != rb) {  // the previous chunk's matches
      if constexpr (AGG) {
        if (D.agg >= 4) emit_mm(pPS, pPE, D.agg == 5);
        else emit_agg(pPS, pPE);
      } else {
        emit(pPS, pPE, pcur, std::integral_constant<bool, HS>{});
      }
    }
    SL_STAMP(1);
    const int E = S.cn[cur] + nchunk;
    // 2. key run offsets and the wave split (one wave: the one with the least to emit, the
    //    previous chunk's scanner picked it from that chunk's split)
    if ((int)w == S.scanner[ci & 1]) {
      uint32_t run = 0;
      int32_t psv[SL_WAVES];
#pragma unroll
      for (int k = 0; k < SL_WAVES; k++) psv[k] = -1;
      for (int b0 = 0; b0 < nb; b0 += 64) {
        const int b = b0 + (int)lane;
        const bool v = b < nb;
        uint32_t c[SL_WAVES], t = 0;
#pragma unroll
        for (int ww = 0; ww < SL_WAVES; ww++) {
          c[ww] = v ? S.wc[ww][b] : 0u;
          t += c[ww];
        }
        const uint32_t nk = v ? S.ncar[b] : 0u;
        t += nk;
        const uint32_t x = dpp_incl_add(t, lane);
        const uint32_t pre = run + x - t;
        if (v) {
          S.binoff[b] = pre;
          S.fe[b] = (uint16_t)(pre + nk);
          uint32_t g = pre + nk;
#pragma unroll
          for (int ww = 0; ww < SL_WAVES; ww++) {
            S.wc[ww][b] = (uint16_t)g;
            g += c[ww];
          }
        }
        // wave k starts at the first key run that starts at or after k * E / 8
#pragma unroll
        for (int k = 1; k < SL_WAVES; k++) {
          const uint64_t mk = __ballot(v && (int64_t)pre * SL_WAVES >= (int64_t)k * E);
          if (mk && psv[k] < 0) psv[k] = __builtin_amdgcn_readlane((int)pre, __ffsll((unsigned long long)mk) - 1);
        }
        run += wave_last(x);
      }
      if (lane == 0) {
        S.binoff[nb] = run;  // = E
        S.ps[0] = 0;
        S.ps[SL_WAVES] = E;
      }
      if (lane > 0 && lane < (uint32_t)SL_WAVES) {
        int32_t pv = -1;
#pragma unroll
        for (int k = 1; k < SL_WAVES; k++) pv = (uint32_t)k == lane ? psv[k] : pv;
        S.ps[lane] = pv < 0 ? E : pv;
      }
      if (lane == 0) {  // the next chunk's scanner: the wave with the smallest range of this chunk
        int best = 0, bl = 1 << 30, prev = 0;
#pragma unroll
        for (int k = 0; k < SL_WAVES; k++) {
          const int nxt = k + 1 < SL_WAVES ? (psv[k + 1] < 0 ? E : psv[k + 1]) : E;
          const int len = nxt - prev;
          if (len < bl) {
            bl = len;
            best = k;
          }
          prev = nxt;
        }
        S.scanner[(ci + 1) & 1] = best;
      }
    }
    __syncthreads();  // B
    SL_STAMP(2);
    // 3. place records and carried candidates at their sorted positions
#pragma unroll
    for (int s = 0; s < SL_R; s++) {
      if (bin[s] == 0xFFFFu) continue;
      const uint32_t p = S.wc[w][bin[s]] + rk[s];
      const int32_t rel = sw_rec_ts32(pf[s]) - tb32;
      if (rel > (int32_t)SW_TS_SPAN || rel < -(int32_t)SW_TS_SPAN) S.flag = 1;
      S.tv[p] = make_int2(rel, (int32_t)pf[s].v);
      S.meta[p] = bin[s] | (S.binoff[bin[s] + 1] << 8) | ((uint32_t)S.fe[bin[s]] << 20);
      S.ref[p] = pf[s].ref | (sw_rec_f1(pf[s]) ? 0x80000000u : 0u);
    }
    {
      const int ncur = S.cn[cur];
      for (int x = tid; x < ncur; x += SL_THREADS) {
        const uint32_t lk = S.clk[cur][x];
        const uint32_t p = S.binoff[lk] + (uint32_t)x - S.ckf[cur][lk];
        const int64_t r = S.cts[cur][x] - (int64_t)tb32;
        if (r > SW_TS_SPAN) S.flag = 1;  // later than the chunk's span: the exact kernel
        const int32_t crel = r < (int64_t)SW_TS_FLOOR ? SW_TS_FLOOR : (int32_t)r;
        S.tv[p] = make_int2(crel, (int32_t)S.cv[cur][x]);
        S.meta[p] = lk | (S.binoff[lk + 1] << 8) | ((uint32_t)S.fe[lk] << 20);
        S.ref[p] = (uint32_t)x;
      }
    }
    if (tid < SL_PAD) {
      S.tv[E + tid] = make_int2(0, 0);
      S.meta[E + tid] = SW_LKF_NONE;
    }
    if (tid == 0) S.cn[nx] = 0;
    {  // prefetch the next chunk while this one is solved
      const int64_t nbk = cb + SL_CHUNK;
#pragma unroll
      for (int s = 0; s < SL_R; s++) {
        const int jj = (int)w * (64 * SL_R) + s * 64 + (int)lane;
        pload(nbk + jj, pf[s]);
      }
      if (nbk < re) tbk = rawkt(nbk);
    }
    __syncthreads();  // C
    SL_STAMP(3);
    // ---- from here each wave works alone on its key runs [PS, PE)
    const int PS = S.ps[w], PE = S.ps[w + 1];
    for (int b = (int)lane; b < nb; b += 64) S.wc[w][b] = 0;  // this wave's counters, next chunk
    for (int p = PS + (int)lane; p < PE; p += 64) S.cl[p] = 0;
    auto record = [&](int p, int res) {
      S.m[p] = (int16_t)res;
      if (res >= 0) {
        const int d = res - p;
        if (d <= SL_NEAR) {
          atomicOr(&S.cl[res], 1u << (d - 1));
        } else {
          const uint32_t old = atomicAdd(&S.cl[res], 1u << 24);
          if ((old >> 24) == 255u) S.flag = 1;
        }
      }
    };
    uint32_t* wl = S.wl[w];
    // 4. probe: round 1 per position, unresolved candidates to the worklist, drained 8 events a round
    auto drain = [&](uint32_t nwl) -> uint32_t {
      uint32_t nn = 0;
      for (uint32_t b0 = 0; b0 < nwl; b0 += 64) {
        const uint32_t idx = b0 + lane;
        int p = 0, res = -3;
        uint32_t qn = 0;
        if (idx < nwl) {
          const uint32_t ent = wl[idx];
          p = (int)(ent & 0xFFFFu);
          qn = ent >> 16;
          const int2 a = S.tv[p];
          const int end = (int)((S.meta[p] >> 8) & 0xFFFu);
          const T bv = bconst ? bc : sw_val<CT>((uint32_t)a.y, 0.0, 0.0, false);
          res = sl_probe<CT, OPC, SL_P2>(S.tv, (int)qn, end, a.x, W, bv);
          qn += SL_P2;
          if (res == -4 && (int)qn >= end) res = -2;
        }
        const bool unres = res == -4;
        const uint64_t um = __ballot(unres);
        if (unres) wl[nn + (uint32_t)__popcll(um & lt)] = (uint32_t)p | (qn << 16);
        else if (idx < nwl) record(p, res);
        nn += (uint32_t)__popcll(um);
      }
      return nn;
    };
    uint32_t nwl = 0;
    for (int g = PS; g < PE; g += 64) {
      const int p = g + (int)lane;
      int res = -3;
      uint32_t qn = 0;
      if (p < PE) {
        // all of a position's facts in independent loads: its meta word (key, run end, first
        // event), its (ts, value), its ref (e1's filter in bit 31) and the previous position's
        const uint32_t mt = S.meta[p];
        const int2 a = S.tv[p];
        const bool f1 = (S.ref[p] >> 31) != 0;
        const uint32_t mprev = p > 0 ? S.meta[p - 1] : 0xFFFFFFFFu;
        const int tprev = p > 0 ? S.tv[p - 1].x : 0;
        const uint32_t lk = mt & 0xFFu;
        const int end = (int)((mt >> 8) & 0xFFFu), fe = (int)(mt >> 20);
        const bool first = (mprev & 0xFFu) != lk;  // the key run starts here
        if (first) S.ncar[lk] = 0;  // recounted by the carry step below
        if (p == end - 1 && p >= fe) S.lastc[lk] = f1 ? 1 : 0;
        if (!first && tprev > a.x) S.flag = 1;  // ts decrease within the key: exact kernel
        if (p < fe || f1) {  // carried, or e1's filter
          const T bv = bconst ? bc : sw_val<CT>((uint32_t)a.y, 0.0, 0.0, false);
          const int q0 = max(p + 1, fe);
          res = sl_probe<CT, OPC, SL_P1>(S.tv, q0, end, a.x, W, bv);
          qn = (uint32_t)(q0 + SL_P1);
          if (res == -4 && (int)qn >= end) res = -2;
        }
      }
      const bool unres = res == -4;
      const uint64_t um = __ballot(unres);
      if (unres) wl[nwl + (uint32_t)__popcll(um & lt)] = (uint32_t)p | (qn << 16);
      else if (p < PE) record(p, res);
      nwl += (uint32_t)__popcll(um);
      if (nwl >= SL_WLD) nwl = drain(nwl);
    }
    while (nwl > 0) nwl = drain(nwl);
    SL_STAMP(4);
    // 5. closes and open candidates per position (contiguous block per lane), output range and
    //    carry slots; open candidates compacted in key order; tv.x becomes the output offset
    const int nw = PE - PS;
    const int K = (nw + 63) >> 6;
    const int lb = PS + (int)lane * K, le = min(lb + K, PE);
    uint32_t cs = 0, os = 0;
    for (int q = lb; q < le; q++) {
      cs += sl_closes(S.cl[q]);
      os += S.m[q] == -2 ? 1u : 0u;
    }
    const uint32_t pk = (cs << 16) | os;
    const uint32_t incl = dpp_incl_add(pk, lane);
    const uint32_t tot = wave_last(incl);
    const uint32_t ctot = tot >> 16, otot = tot & 0xFFFFu;
    int cbase = 0;
    if (lane == 0) {
      cbase = otot ? atomicAdd(&S.cn[nx], (int)otot) : 0;
      S.wt[w] = ctot;
      // the last wave through reserves the chunk's output (LDS keeps each wave's operations in
      // order, so it sees every other wave's count)
      if (atomicAdd(&S.done, 1) == SL_WAVES - 1) {
        uint32_t t = 0;
        for (int ww = 0; ww < SL_WAVES; ww++) {
          S.wb[ww] = t;
          t += S.wt[ww];
        }
        // the returned base is first needed by the next chunk's emission: it is written to LDS
        // just before the next barrier A, so the atomic's round trip overlaps this wave's carry
        // bookkeeping and its next rank step instead of holding every wave at that barrier
        // (+ a lane count that is always 0: an address the compiler cannot prove uniform keeps its
        // atomic optimizer, which reads the result back at once, off this single-lane add)
        gres = t ? atomicAdd(O.count + __builtin_amdgcn_mbcnt_lo(0u, 0u), (unsigned long long)t) : 0ull;
        gres_t = t;
        gpend = true;
        S.done = 0;
      }
    }
    cbase = __shfl(cbase, 0, 64);
    if (cbase + (int)otot > SL_CCAP) S.flag = 1;
    {
      // two copies of the loop: without a seq column it issues no global load, so nothing in it
      // waits on the output reservation's atomic still in flight (published before barrier A)
      auto compact = [&](auto has_seq) {
        uint32_t co = (incl - pk) >> 16, oo = (incl - pk) & 0xFFFFu;
        for (int q = lb; q < le; q++) {
          const uint32_t c = sl_closes(S.cl[q]);
          if (S.m[q] == -2) {
            const int x = cbase + (int)oo;
            if (x < SL_CCAP) {
              const uint32_t f = S.meta[q];
              const uint32_t r = S.ref[q] & 0x7FFFFFFFu;
              if (q < (int)(f >> 20)) {  // carried
                S.cts[nx][x] = S.cts[cur][r];
                S.cv[nx][x] = S.cv[cur][r];
                S.cseq[nx][x] = S.cseq[cur][r];
              } else {
                const int2 a = S.tv[q];
                S.cts[nx][x] = tb32 + a.x;  // |.| < 2^30 (the scatter's wide flag)
                S.cv[nx][x] = (uint32_t)a.y;
                const int64_t dsq = (decltype(has_seq)::value ? B.seq[r] : B.seq0 + (int64_t)r) - sbase;
                if (dsq != (int64_t)(int32_t)dsq) S.flag = 1;
                S.cseq[nx][x] = (int32_t)dsq;
              }
              S.clk[nx][x] = (uint8_t)(f & 0xFFu);
            }
            oo++;
          }
          S.tv[q].x = (int32_t)co;
          co += c;
        }
      };
      compact(std::integral_constant<bool, HS>{});
    }
    {  // per-key first index and count of the new carry entries
      const int xe = min(cbase + (int)otot, SL_CCAP);
      for (int x = cbase + (int)lane; x < xe; x += 64) {
        const uint32_t lk = S.clk[nx][x];
        if (x == cbase || S.clk[nx][x - 1] != lk) S.ckf[nx][lk] = (uint16_t)x;
      }
      for (int x = cbase + (int)lane; x < xe; x += 64) {
        const uint32_t lk = S.clk[nx][x];
        if (x + 1 == xe || S.clk[nx][x + 1] != lk) S.ncar[lk] = (uint32_t)(x + 1 - S.ckf[nx][lk]);
      }
    }
    pPS = PS;
    pPE = PE;
    pcur = cur;
    cur = nx;
    SL_STAMP(5);
  }
  publish();
  __syncthreads();
  if (S.flag) {
    if (tid == 0) atomicOr(err, SWE_LEAN);
    return;
  }
  if constexpr (AGG) {  // the last chunk's matches
    if (D.agg >= 4) emit_mm(pPS, pPE, D.agg == 5);
    else emit_agg(pPS, pPE);
  } else {
    emit(pPS, pPE, pcur, std::integral_constant<bool, HS>{});
  }
#ifdef SHP_SW_STAMPS
  SL_STAMP(1);
  {
    __shared__ unsigned long long sts[8];
    if (tid < 8) sts[tid] = 0;
    __syncthreads();
    if (lane == 0)
      for (int k = 0; k < 8; k++) atomicAdd(&sts[k], stc[k]);
    __syncthreads();
    if (tid < 8 && D.stamps) D.stamps[(int64_t)o * 8 + tid] = sts[tid];
  }
#endif
  // write back the carry in key order (k_sw_solve's layout) and the per-key flags (copy wr)
  {
    uint32_t total;
    const uint32_t v = tid < (uint32_t)nb ? S.ncar[tid] : 0u;
    const uint32_t pre = sw_block_scan_n<SL_WAVES>(v, S.wtot, total);
    if (tid < (uint32_t)nb) S.binoff[tid] = pre;
  }
  __syncthreads();
  const int ncf = S.cn[cur];
  for (int x = tid; x < ncf; x += SL_THREADS) {
    const uint32_t lk = S.clk[cur][x];
    const int64_t c = (int64_t)o * SWS_CCAP + S.binoff[lk] + (uint32_t)x - S.ckf[cur][lk];
    D.c_ts[wr][c] = base + S.cts[cur][x];
    D.c_seq[wr][c] = sbase + S.cseq[cur][x];
    D.c_v[wr][c] = S.cv[cur][x];
    D.c_lk[wr][c] = (uint8_t)lk;
    D.c_null[wr][c] = 0;
  }
  for (int i = tid; i < SW_LK; i += SL_THREADS) D.lastc[wr][(int64_t)o * SW_LK + i] = S.lastc[i];
  if constexpr (AGG)  // every wave's last emission is behind the block scan's barriers above
    for (int i = tid; i < SW_LK; i += SL_THREADS) {
      D.agg_s[wr][(int64_t)o * SW_LK + i] = ag[i];
      D.agg_c[wr][(int64_t)o * SW_LK + i] = ag[256 + i];
    }
  if (tid == 0) D.c_n[wr][o] = ncf;
  if (e) atomicOr(err, e);
}

}  // namespace shp
