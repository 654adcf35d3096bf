// siddhi-hip: k_sw_win, the sweep solve as independent units of the owner-major record array
// (round 4: the default solve of the headline shape; included by sweep.h).
//
// Same semantics and output as k_sw_lean / k_sw_solve (SURVEY.md Appendix A.7;
// StreamPreStateProcessor.processAndReturn / expireEvents :326-403): per key, candidate i (e1's
// filter, evaluated by the scatter) closes at the first later event j of the key with
// ts_j - ts_i <= W and f2(i, j), and expires at the first later event beyond W; matches per key
// in (j, i) order, i ascending within one closer.
//
// Decomposition.  k_sw_lean gives each owner one workgroup that walks the owner's records in
// chunks: a block-wide sort by key per chunk, three block barriers, and 8 waves waiting for the
// most loaded one.  Here the record array (owner-major, arrival order within an owner) is cut into
// fixed units of SWW_U records, one wave each, with no barrier at all:
//   * a unit reads its records in arrival order, 64 per window (one per lane); the records of
//     one key inside a window are found with bit ballots over the local key, so no sort is needed;
//     a candidate probes the later lanes of its key (straight-line, 4 at a time), and the open
//     candidates of earlier windows (an LDS list in arrival order) probe the window the same way;
//   * the open candidates at the unit's start are recomputed, not handed over: a candidate
//     depends only on later events of its key within W, so the unit replays a halo of the owner's
//     records before it, with an empty list.  The halo is exact for a key once the key's events
//     in it span more than W (every older candidate of the key has expired by then) and for every
//     key once it reaches the owner's start (then the push's carry seeds the list).  A unit whose
//     keys are not all covered doubles its halo and replays again;
//   * output order: the matches of a unit are staged in LDS in emission order; the unit's offset is
//     the sum of the match counts of all earlier units (decoupled look-back over a status word per
//     unit, 64 predecessors per probe), units being numbered in the order they start (a ticket), so
//     a wave only ever waits for units that are running or done;
//   * the per-owner state after the push (open candidates in key order, each key's lastc flag) is
//     written by k_sw_win_tail, one wave per owner, which replays the owner's last records the same
//     way (its halo covers every key with events in the push, from the units' presence masks).
// Anything outside this kernel's cover -- a ts decrease within a key, more than SWW_CAP open
// candidates, a wide push, a staging overflow -- raises SWE_LEAN and the engine re-runs the push
// with the exact solve from the same committed state.
#pragma once

namespace shp {

constexpr int SWW_U = 1024;                 // records per unit
constexpr int SWW_CAP = 128;                // open candidates held by a wave
constexpr int SWW_SCAP = SWW_U + SWW_CAP;   // staged matches per unit
constexpr uint64_t SWW_AGG = 1ull << 62, SWW_INC = 2ull << 62, SWW_VAL = (1ull << 62) - 1;
constexpr int32_t SWW_NONE = INT32_MIN;

struct SwWinSmem {
  uint2 stg[SWW_SCAP];        // staged matches: (e2's batch index, e2 seq - e1 seq)
  int4 car[SWW_CAP];          // open candidates: ts (push-relative), value bits, seq - sbase, local key
  int32_t cres[SWW_CAP];      // per open candidate in the current window: closer lane | rank << 8, -1, -2
  int2 wv[65];                // the window's (ts, value) by lane; [64] a dummy probe target
  uint32_t ccnt[64], ocnt[64];  // carried / own candidates closing at each lane of the window
  int32_t lastts[256];        // per local key: latest ts seen (SWW_NONE: none)
  int32_t fts[256];           // per local key: first ts in the halo (SWW_NONE: none)
  uint8_t vk[256];            // per local key: the halo covers it
  uint8_t lcf[256];           // per local key: its latest event opened a candidate (tail)
  uint32_t pres[8];           // local keys with events in the segment
  uint32_t hist[256];         // tail: final carry per key, then its write cursors
};

// one window's probe results for a candidate (ts a_ts, resolved compare operand b) over the lanes
// of mask m in lane order: -2 no resolution among them (open), -1 expired, lane of the closer
template <int CT, int OPC>
__device__ __forceinline__ int sww_probe(const int2* wv, uint64_t m, int32_t a_ts, int32_t W,
                                         typename SwTy<CT>::T b) {
  int res = -4;
  while (res == -4) {
    int j[4];
#pragma unroll
    for (int d = 0; d < 4; d++) {
      j[d] = m ? (int)__ffsll((unsigned long long)m) - 1 : 64;
      m &= m - 1;
    }
    int2 x[4];
#pragma unroll
    for (int d = 0; d < 4; d++) x[d] = wv[j[d]];
#pragma unroll
    for (int d = 0; d < 4; d++) {
      const bool hit = sw_cmp_op<OPC>(0, sw_val<CT>((uint32_t)x[d].y, 0.0, 0.0, false), b);
      const int r = j[d] == 64 ? -2 : (x[d].x - W > a_ts ? -1 : (hit ? j[d] : -4));
      res = res == -4 ? r : res;
    }
    if (res == -4 && m == 0) res = -2;
  }
  return res;
}

// lanes whose 6-bit value c equals this lane's, among the lanes of `act`
__device__ __forceinline__ uint64_t sww_match6(uint32_t c, bool act) {
  uint64_t p = __ballot(act);
#pragma unroll
  for (int b = 0; b < 6; b++) {
    const bool bit = (c >> b) & 1u;
    const uint64_t m = __ballot(bit);
    p &= bit ? m : ~m;
  }
  return p;
}

__device__ __forceinline__ uint32_t sww_scan_excl(uint32_t x, uint32_t lane, uint32_t& total) {
  uint32_t incl = x;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(incl, d, 64);
    if (lane >= (uint32_t)d) incl += y;
  }
  total = __shfl(incl, 63, 64);
  return incl - x;
}

// The wave's replay state: the open-candidate list length, the staging cursor, flags.
struct SwwCtx {
  int ncar;
  uint32_t cur;
  int flag;  // 1: SWE_LEAN (exact kernel), 2: SWE_P32
};

// Replay records [ps, pe) of one owner (0 <= ps <= pe), windows of 64 lanes.
//   EMIT   : stage the matches (closers in this range), check the halo cover of each key
//   !EMIT  : halo / tail -- record each key's first ts (fts) and its last event's filter (lcf)
// Returns false when a key of an emitted window is not covered by the halo (the caller widens it).
#ifdef SHP_SW_STAMPS
#define SWR_STAMP(k)                     \
  do {                                   \
    if (EMIT) {                          \
      const uint64_t t_ = clock64();     \
      wst[k] += t_ - wsp;                \
      wsp = t_;                          \
    }                                    \
  } while (0)
#else
#define SWR_STAMP(k) \
  do {               \
  } while (0)
#endif
template <int CT, int OPC, bool EMIT>
__device__ bool sww_replay(const SweepDev& D, const BatchView& B, SwWinSmem& S, SwwCtx& X, int64_t ps, int64_t pe,
                           int32_t W, bool bconst, typename SwTy<CT>::T bc, int64_t sbase, int lkb
#ifdef SHP_SW_STAMPS
                           , unsigned long long* wst
#endif
                           ) {
  using T = typename SwTy<CT>::T;
#ifdef SHP_SW_STAMPS
  uint64_t wsp = clock64();
#endif
  const uint32_t lane = __lane_id();
  const uint64_t lt = sw_lanemask_lt();
  const uint64_t gtm = lane == 63 ? 0ull : (~0ull << (lane + 1));
  SwRec nx{};
  if (ps + lane < pe) nx = D.recs[ps + lane];
  for (int64_t pw = ps; pw < pe; pw += 64) {
    asm volatile("" ::: "memory");  // other lanes' LDS writes of the last window: reload, in order
    const SwRec r = nx;
    const bool valid = pw + lane < pe;
    if (pw + 64 + lane < pe) nx = D.recs[pw + 64 + lane];  // the next window's records in flight
    const uint32_t lk = valid ? (uint32_t)(r.kt >> 56) : 0u;
    const int32_t ts = (int32_t)(uint32_t)r.kt;  // push-relative (|.| < 2^30: the scatter's wide flag)
    const uint32_t v = r.v, ref = r.ref;
    const bool f1 = valid && (r.kt & SW_F1) != 0;
    const uint64_t vmask = __ballot(valid);
    uint64_t mb[8];
    uint64_t peers = vmask;
#pragma unroll
    for (int b = 0; b < 8; b++) {
      mb[b] = b < lkb ? __ballot(valid && ((lk >> b) & 1u)) : 0ull;
      peers &= ((lk >> b) & 1u) ? mb[b] : ~mb[b];
    }
    if (!valid) peers = 0;
    if constexpr (EMIT) {  // every key of the window must be covered by the halo
      const bool bad = valid && !S.vk[lk];
      if (__ballot(bad)) return false;
    }
    // per key: ts never decreases (the exact kernel replays keys that do), latest ts, first ts
    const uint64_t pm = peers & lt;
    const int prevl = pm ? 63 - (int)__clzll((long long)pm) : 0;
    const int32_t tsp = __shfl(ts, prevl, 64);
    const int32_t tprev = pm ? tsp : (valid ? S.lastts[lk] : SWW_NONE);
    if (valid && ts < tprev) X.flag |= 1;
    const bool lastk = valid && (peers & gtm) == 0;
    S.wv[lane] = make_int2(ts, (int32_t)v);
    if (lastk) S.lastts[lk] = ts;
    SWR_STAMP(0);
    if constexpr (!EMIT) {
      if (valid && pm == 0 && S.fts[lk] == SWW_NONE) S.fts[lk] = ts;
      if (lastk) S.lcf[lk] = f1 ? 1 : 0;
    } else {
      if (lastk) atomicOr(&S.pres[lk >> 5], 1u << (lk & 31));
      S.ccnt[lane] = 0;
      S.ocnt[lane] = 0;
    }
    // this window's own candidates against the later lanes of their key
    int ores = -3;
    if (f1) ores = sww_probe<CT, OPC>(S.wv, peers & gtm, ts, W, bconst ? bc : sw_val<CT>(v, 0.0, 0.0, false));
    SWR_STAMP(1);
    // the open candidates of earlier windows against every lane of their key
    const int nc = X.ncar;
    for (int c0 = 0; c0 < nc; c0 += 64) {
      const int e = c0 + (int)lane;
      const bool ev = e < nc;
      int res = -2;
      uint64_t m = 0;
      int4 ce = make_int4(0, 0, 0, 0);
      if (ev) {
        ce = S.car[e];
        m = vmask;
#pragma unroll
        for (int b = 0; b < 8; b++) m &= (((uint32_t)ce.w >> b) & 1u) ? mb[b] : ~mb[b];
        if (m) res = sww_probe<CT, OPC>(S.wv, m, ce.x, W, bconst ? bc : sw_val<CT>((uint32_t)ce.y, 0.0, 0.0, false));
      }
      if constexpr (EMIT) {  // rank among the carried candidates closing at the same lane (list order)
        const bool cl = ev && res >= 0;
        const uint32_t c = cl ? (uint32_t)res : 0u;
        const uint64_t pe6 = sww_match6(c, cl);
        const uint32_t before = cl ? S.ccnt[c] : 0u;
        if (cl && (pe6 & lt) == 0) S.ccnt[c] = before + (uint32_t)__popcll(pe6);
        if (cl) res |= (int)((before + (uint32_t)__popcll(pe6 & lt)) << 8);
      }
      if (ev) S.cres[e] = res;
    }
    SWR_STAMP(2);
    uint32_t T = 0, base = 0, cc = 0;
    if constexpr (EMIT) {
      const bool cl = ores >= 0;
      const uint32_t c = cl ? (uint32_t)ores : 0u;
      const uint64_t pe6 = sww_match6(c, cl);
      const uint32_t orank = (uint32_t)__popcll(pe6 & lt);
      if (cl && orank == 0) S.ocnt[c] = (uint32_t)__popcll(pe6);
      cc = S.ccnt[lane];
      base = sww_scan_excl(cc + S.ocnt[lane], lane, T);
      if (X.cur + T > (uint32_t)SWW_SCAP) {
        X.flag |= 1;
        return true;
      }
      // own matches: (e2 index, e2 seq - e1 seq), after the carried ones closing at the same lane
      const uint32_t sidx = __shfl(base + cc, (int)c, 64);
      const uint32_t rj = __shfl(ref, (int)c, 64);
      if (cl) {
        const int64_t dq = bseq(B, rj) - bseq(B, ref);
        if (dq >= (1ll << 32)) X.flag |= D.p32 ? 2 : 1;
        S.stg[X.cur + sidx + orank] = make_uint2(rj, (uint32_t)dq);
      }
    }
    SWR_STAMP(3);
    // carried matches, then the new list: surviving carried candidates (list order), then this
    // window's open candidates (lane order) -- per key still in arrival order
    int w = 0;
    for (int c0 = 0; c0 < nc; c0 += 64) {
      const int e = c0 + (int)lane;
      const bool ev = e < nc;
      const int cr = ev ? S.cres[e] : -1;
      const int4 ce = ev ? S.car[e] : make_int4(0, 0, 0, 0);
      if constexpr (EMIT) {
        const int c = cr >= 0 ? (cr & 0xFF) : 0;
        const uint32_t sb = __shfl(base, c, 64);
        const uint32_t rj = __shfl(ref, c, 64);
        if (cr >= 0) {
          const int64_t dq = bseq(B, rj) - (sbase + (int64_t)ce.z);
          if (dq >= (1ll << 32)) X.flag |= D.p32 ? 2 : 1;
          S.stg[X.cur + sb + ((uint32_t)cr >> 8)] = make_uint2(rj, (uint32_t)dq);
        }
      }
      const bool keep = cr == -2;
      const uint64_t sm = __ballot(keep);
      if (keep) S.car[w + (int)__popcll(sm & lt)] = ce;
      w += (int)__popcll(sm);
    }
    const bool op = ores == -2;
    const uint64_t sm = __ballot(op);
    if (op) {
      const int dst = w + (int)__popcll(sm & lt);
      const int64_t dsq = bseq(B, ref) - sbase;
      if (dsq != (int64_t)(int32_t)dsq) X.flag |= 1;
      if (dst < SWW_CAP) S.car[dst] = make_int4(ts, (int32_t)v, (int32_t)dsq, (int32_t)lk);
    }
    w += (int)__popcll(sm);
    if (w > SWW_CAP) {
      X.flag |= 1;
      w = SWW_CAP;
    }
    X.ncar = w;
    if constexpr (EMIT) X.cur += T;
    SWR_STAMP(4);
#ifdef SHP_SW_STAMPS
    if (EMIT) wst[5] += (uint64_t)nc;
#endif
  }
  return true;
}

// the per-key state before the replay: empty, or (from the owner's start) the push's carry
__device__ __forceinline__ void sww_init(const SweepDev& D, SwWinSmem& S, SwwCtx& X, int o, bool from_start, int nb,
                                         int64_t base, int64_t sbase) {
  const uint32_t lane = __lane_id();
  for (int b = (int)lane; b < nb; b += 64) {
    S.lastts[b] = SWW_NONE;
    S.fts[b] = SWW_NONE;
  }
  if (lane < 8) S.pres[lane] = 0;
  X.ncar = 0;
  if (!from_start) return;
  const int rd = D.cur;
  const int n0 = D.c_n[rd][o];
  if (n0 > SWW_CAP) {
    X.flag |= 1;
    return;
  }
  for (int x = (int)lane; x < n0; x += 64) {
    const int64_t c = (int64_t)o * SWS_CCAP + x;
    const int64_t dts = D.c_ts[rd][c] - base, dsq = D.c_seq[rd][c] - sbase;
    if (dts != (int64_t)(int32_t)dts || dsq != (int64_t)(int32_t)dsq) X.flag |= 1;
    const uint32_t lk = D.c_lk[rd][c];
    S.car[x] = make_int4((int32_t)dts, (int32_t)D.c_v[rd][c], (int32_t)dsq, (int32_t)lk);
    // the key's latest ts so far: its last carried candidate (key order, ts ascending)
    if (x + 1 == n0 || D.c_lk[rd][c + 1] != lk) S.lastts[lk] = (int32_t)dts;
  }
  X.ncar = n0;
}

// owner o's record range [os, oe): o is the owner with off[o * nst] <= p < off[(o + 1) * nst]
__device__ __forceinline__ int sww_owner_of(const SweepDev& D, int64_t p) {
  const uint32_t lane = __lane_id();
  int lo = 0, n = D.nown;  // search [lo, lo + n)
  while (n > 1) {
    const int step = (n + 63) / 64;
    const int q = lo + (int)lane * step;
    const bool le = q < lo + n && (int64_t)D.off[(int64_t)q * D.nst] <= p;
    const uint64_t m = __ballot(le);
    const int last = 63 - (int)__clzll((long long)m);  // lane 0 always qualifies (off[lo] <= p)
    lo = lo + last * step;
    n = min(step, D.nown - lo);
  }
  return lo;
}

template <int CT, int OPC>
__global__ __launch_bounds__(64) void k_sw_win(SweepDev D, BatchView B, MatchOut O, int* err) {
  using T = typename SwTy<CT>::T;
  __shared__ SwWinSmem S;
  const uint32_t lane = threadIdx.x;
#ifdef SHP_SW_STAMPS  // diagnostic build: cycles per phase summed over units (D.stamps[0..7])
  unsigned long long st_c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long wst[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t st_p = clock64(), st_0 = st_p;
#define SWW_STAMP(k)                \
  do {                              \
    const uint64_t t_ = clock64();  \
    st_c[k] += t_ - st_p;           \
    st_p = t_;                      \
  } while (0)
#else
#define SWW_STAMP(k) \
  do {               \
  } while (0)
#endif
  uint32_t u = 0;
  if (lane == 0) u = atomicAdd(D.w_ticket, 1u);
  u = __shfl(u, 0, 64);
  SWW_STAMP(0);
  const int64_t nrec = D.off[(int64_t)D.nown * D.nst];
  const int64_t g0 = (int64_t)u * SWW_U, g1 = min(nrec, g0 + SWW_U);
  const int64_t base = B.ts[0];
  const int64_t sbase = bseq(B, 0);
  const int32_t W = (int32_t)D.within;
  const SwTerm t2 = D.f2.t[0];
  const bool bconst = t2.bk == 0;
  const T bc = (T)t2.bc;
  const int lkb = D.lk_bits;
  const int nb = lkb >= 8 ? SW_LK : (1 << lkb);
  SwwCtx X{0, 0u, 0};
  if (lane == 0) S.wv[64] = make_int2(0, 0);
  if (D.tsmax[1] != 0 || (*err & SWE_LEAN)) X.flag |= 1;  // a wide push: the exact kernel
  int64_t p = g0;
  int o = p < g1 ? sww_owner_of(D, p) : 0;
  while (p < g1 && !X.flag) {
    while ((int64_t)D.off[(int64_t)(o + 1) * D.nst] <= p) o++;  // skip empty owners
    const int64_t os = D.off[(int64_t)o * D.nst], oe = D.off[(int64_t)(o + 1) * D.nst];
    const int64_t s0 = p, s1 = min(g1, oe);
    int64_t h = D.w_halo;
    const uint32_t cur0 = X.cur;
    for (;;) {
      const int64_t H = max(os, s0 - h);
      sww_init(D, S, X, o, H == os, nb, base, sbase);
      X.cur = cur0;
      SWW_STAMP(1);
      sww_replay<CT, OPC, false>(D, B, S, X, H, s0, W, bconst, bc, sbase, lkb
#ifdef SHP_SW_STAMPS
                                 , wst
#endif
      );
#ifdef SHP_SW_STAMPS
      st_c[7] += (uint64_t)(s0 - H);
#endif
      SWW_STAMP(2);
      for (int b = (int)lane; b < nb; b += 64)
        S.vk[b] = H == os || (S.fts[b] != SWW_NONE && S.lastts[b] - S.fts[b] > W);
      asm volatile("" ::: "memory");
      if (X.flag) break;
      const bool ok = sww_replay<CT, OPC, true>(D, B, S, X, s0, s1, W, bconst, bc, sbase, lkb
#ifdef SHP_SW_STAMPS
                                                , wst
#endif
      );
      SWW_STAMP(3);
      if (ok) break;
      h *= 2;  // a key of the segment is not covered: a longer halo
    }
    if (lane < 8) D.w_pres[((int64_t)u + o) * 8 + lane] = S.pres[lane];
    p = s1;
  }
  // the unit's matches: publish the count, find the offset (decoupled look-back), write
  const uint32_t Tu = X.flag ? 0u : X.cur;
  // (a push the exact kernel re-runs may still fail there with SWE_P32, as k_sw_lean's would)
  if (X.flag && lane == 0) atomicOr(err, (X.flag & 1) ? SWE_LEAN : SWE_P32);
  unsigned long long* st = D.w_stat;
  uint64_t excl = 0;
  if (u == 0) {
    excl = O.count[0];
    if (lane == 0) __hip_atomic_store(st, SWW_INC | (excl + Tu), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    if (lane == 0) __hip_atomic_store(st + u, SWW_AGG | (uint64_t)Tu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int64_t v = (int64_t)u - 1;
    for (;;) {
      const int64_t idx = v - (int64_t)lane;
      uint64_t s = idx >= 0 ? __hip_atomic_load(st + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : SWW_INC;
      const uint64_t inc = __ballot((s >> 62) == 2), rdy = __ballot((s >> 62) != 0);
      const int fi = inc ? (int)__ffsll((unsigned long long)inc) - 1 : 64;
      const uint64_t need = fi >= 63 ? ~0ull : ((2ull << fi) - 1);
      if ((rdy & need) != need) {
        __builtin_amdgcn_s_sleep(2);
        continue;
      }
      uint64_t x = (int)lane <= fi ? (s & SWW_VAL) : 0ull;
#pragma unroll
      for (int d = 32; d > 0; d >>= 1) x += __shfl_xor(x, d, 64);
      excl += x;
      if (fi < 64) break;
      v -= 64;
    }
    if (lane == 0) __hip_atomic_store(st + u, SWW_INC | (excl + Tu), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  SWW_STAMP(4);
  if (u == gridDim.x - 1 && lane == 0) {  // the last unit: the push's match count
    O.count[0] = excl + Tu;
    if (excl + Tu > (uint64_t)O.cap) atomicOr(err, E_OUT);
  }
  for (uint32_t k = lane; k < Tu; k += 64) {
    const uint64_t slot = excl + k;
    if (slot >= (uint64_t)O.cap) break;
    const uint2 m = S.stg[k];
    if (D.p32) {
      reinterpret_cast<uint2*>(O.refs)[slot] = m;
    } else {
      const int64_t sq = bseq(B, m.x), si = sq - (int64_t)m.y;
      *(longlong2*)(O.refs + 2 * slot) = make_longlong2(si, B.seq ? (int64_t)m.x : sq);
    }
  }
#ifdef SHP_SW_STAMPS
  SWW_STAMP(5);
  st_c[6] = clock64() - st_0;
  if (lane == 0 && D.stamps)
    for (int k = 0; k < 8; k++) {
      atomicAdd(D.stamps + k, st_c[k]);
      atomicAdd(D.stamps + 8 + k, wst[k]);
    }
#endif
}

// The per-owner state after the push: the open candidates at the owner's end (key order, as
// k_sw_solve keeps them) and each key's lastc flag, replayed from a halo that covers every key
// with events in the push; keys without events pass their state through.
template <int CT, int OPC>
__global__ __launch_bounds__(64) void k_sw_win_tail(SweepDev D, BatchView B, int* err) {
  using T = typename SwTy<CT>::T;
  __shared__ SwWinSmem S;
  if (*err & (SWE_LEAN | SWE_P32)) return;  // the exact kernel re-runs the push
  const uint32_t lane = threadIdx.x;
  const uint64_t lt = sw_lanemask_lt();
  const int o = blockIdx.x;
  const int rd = D.cur, wr = D.cur ^ 1;
  const int64_t os = D.off[(int64_t)o * D.nst], oe = D.off[(int64_t)(o + 1) * D.nst];
  const int64_t base = B.ts[0];
  const int64_t sbase = bseq(B, 0);
  const int32_t W = (int32_t)D.within;
  const SwTerm t2 = D.f2.t[0];
  const bool bconst = t2.bk == 0;
  const T bc = (T)t2.bc;
  const int lkb = D.lk_bits;
  const int nb = lkb >= 8 ? SW_LK : (1 << lkb);
  const int n0 = D.c_n[rd][o];
  // keys with events in the push: the presence masks of every unit segment of this owner
  uint32_t pm8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (os < oe) {
    const int64_t u0 = os / SWW_U, u1 = (oe - 1) / SWW_U;
    for (int64_t uu = u0 + lane; uu <= u1; uu += 64)
#pragma unroll
      for (int i = 0; i < 8; i++) pm8[i] |= D.w_pres[(uu + o) * 8 + i];
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
      for (int d = 32; d > 0; d >>= 1) pm8[i] |= __shfl_xor(pm8[i], d, 64);
  }
  auto present = [&](int b) -> bool { return (pm8[b >> 5] >> (b & 31)) & 1u; };
  SwwCtx X{0, 0u, 0};
  if (lane == 0) S.wv[64] = make_int2(0, 0);
  bool from_start = true;
  if (os < oe) {
    int64_t h = D.w_tail;
    for (;;) {
      const int64_t H = max(os, oe - h);
      from_start = H == os;
      sww_init(D, S, X, o, from_start, nb, base, sbase);
      for (int b = (int)lane; b < nb; b += 64) S.lcf[b] = 0;
      sww_replay<CT, OPC, false>(D, B, S, X, H, oe, W, bconst, bc, sbase, lkb
#ifdef SHP_SW_STAMPS
                                 , nullptr
#endif
      );
      if (X.flag || from_start) break;
      bool ok = true;
      for (int b = (int)lane; b < nb; b += 64)
        if (present(b) && !(S.fts[b] != SWW_NONE && S.lastts[b] - S.fts[b] > W)) ok = false;
      if (__ballot(!ok) == 0) break;
      h *= 2;
    }
  } else {
    sww_init(D, S, X, o, true, nb, base, sbase);  // no events: the carry passes through
  }
  if (X.flag) {
    if (lane == 0) atomicOr(err, SWE_LEAN);
    return;
  }
  // final list in key order: the replayed candidates, plus (halo short of the owner's start) the
  // carried entries of keys without events in the push, which nothing touched
  const bool pass = !from_start;
  for (int b = (int)lane; b < 256; b += 64) S.hist[b] = 0;
  for (int x = (int)lane; x < X.ncar; x += 64) atomicAdd(&S.hist[S.car[x].w], 1u);
  if (pass)
    for (int x = (int)lane; x < n0; x += 64) {
      const uint32_t lk = D.c_lk[rd][(int64_t)o * SWS_CCAP + x];
      if (!present((int)lk)) atomicAdd(&S.hist[lk], 1u);
    }
  uint32_t tot = 0;
  {
    uint32_t hv[4], s = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      hv[i] = S.hist[lane * 4 + i];
      s += hv[i];
    }
    uint32_t pre = sww_scan_excl(s, lane, tot);
#pragma unroll
    for (int i = 0; i < 4; i++) {
      S.hist[lane * 4 + i] = pre;
      pre += hv[i];
    }
  }
  if (tot > (uint32_t)SWS_CCAP) {
    if (lane == 0) atomicOr(err, SWE_LEAN);
    return;
  }
  // stable placement: entries in list order, ranked among equal keys by ballot matching
  auto place = [&](bool ok, uint32_t lk, int64_t ts, int64_t sq, uint32_t v) {
    uint64_t p = __ballot(ok);
#pragma unroll
    for (int b = 0; b < 8; b++) {
      const bool bit = (lk >> b) & 1u;
      const uint64_t m = __ballot(bit);
      p &= bit ? m : ~m;
    }
    const uint32_t before = ok ? S.hist[lk] : 0u;
    if (ok && (p & lt) == 0) S.hist[lk] = before + (uint32_t)__popcll(p);
    if (ok) {
      const int64_t c = (int64_t)o * SWS_CCAP + before + (uint32_t)__popcll(p & lt);
      D.c_ts[wr][c] = ts;
      D.c_seq[wr][c] = sq;
      D.c_v[wr][c] = v;
      D.c_lk[wr][c] = (uint8_t)lk;
      D.c_null[wr][c] = 0;
    }
  };
  for (int x0 = 0; x0 < X.ncar; x0 += 64) {
    const int x = x0 + (int)lane;
    const bool ok = x < X.ncar;
    const int4 ce = ok ? S.car[x] : make_int4(0, 0, 0, 0);
    place(ok, (uint32_t)ce.w, base + ce.x, sbase + ce.z, (uint32_t)ce.y);
  }
  if (pass)
    for (int x0 = 0; x0 < n0; x0 += 64) {
      const int x = x0 + (int)lane;
      const int64_t c = (int64_t)o * SWS_CCAP + x;
      const uint32_t lk = x < n0 ? D.c_lk[rd][c] : 0u;
      const bool ok = x < n0 && !present((int)lk);
      place(ok, lk, ok ? D.c_ts[rd][c] : 0, ok ? D.c_seq[rd][c] : 0, ok ? D.c_v[rd][c] : 0u);
    }
  for (int b = (int)lane; b < SW_LK; b += 64) {
    const int64_t k = (int64_t)o * SW_LK + b;
    D.lastc[wr][k] = (os < oe && present(b)) ? S.lcf[b] : D.lastc[rd][k];
  }
  if (lane == 0) D.c_n[wr][o] = (int32_t)tot;
}

}  // namespace shp
