// siddhi-hip: k_sw_spill, the sweep path's unbounded per-owner form (included by sweep.h).
//
// The reference keeps every pending partial of a state in an unbounded LinkedList
// (StreamPreStateProcessor.java:437-438): one key whose price falls for a whole `within` window at
// 1 event/ms holds ~1000 open e1 candidates.  The LDS solves (k_sw_lean / k_sw_solve)
// carry at most SWS_CCAP = 512 open candidates per owner.  An owner whose carry would outgrow that
// is "spilled": from then on it is solved by this kernel, with its open candidates in HBM, until
// its carry falls back to SWS_CCAP / 2 (hysteresis), when it returns to the LDS solves.
//
// Per spilled owner, one 256-thread workgroup:
//   1. group   the owner's records of the push (arrival order, from the scatter) by local key:
//              a count per key, a scan, and a stable scatter of record positions into per-key
//              index lists (wave ballots per round of 64, one wave: rounds stay in order);
//   2. replay  one thread per local key walks its carried candidates, then its records, with the
//              exact rules of the sequential replay sw_seq_key -- StreamPreStateProcessor
//              .expireEvents (:326-361: the pending list expires from its head and stops at the
//              first live partial; the new-and-every list, i.e. the candidate the key's previous
//              event opened, whole) and processAndReturn (:364-403: every pending partial tried in
//              list order) -- over a candidate list in HBM (capacity: carried + records of the
//              key, since each event opens at most one candidate).  The matches of one closing
//              event are reserved with one atomic and written in list order, so each key's
//              records keep the reference's (j, i) order.  SHP_LAYOUT_AGG folds the selector's
//              aggregate per match in emission order, as the Java aggregator does;
//   3. carry   the open candidates, in key order, back to the LDS solves' carry arrays when they
//              fit SWS_CCAP / 2, else to this owner's segment of the HBM pool.
// Any ts order and span are exact here (64-bit timestamps throughout).
#pragma once

namespace shp {

constexpr int SP_THREADS = 256;

template <int NT2, int CT>
__global__ __launch_bounds__(SP_THREADS) void k_sw_spill(SweepDev D, BatchView B, MatchOut O, int* err) {
  __shared__ uint32_t nrec[SW_LK + 1], rbase[SW_LK + 1], cur[SW_LK + 1];
  __shared__ uint32_t ncar[SW_LK + 1], cbase[SW_LK + 1];
  __shared__ uint32_t wt[SP_THREADS / 64];
  __shared__ uint32_t tot_out;
  const int o = blockIdx.x;
  const uint32_t tid = threadIdx.x, lane = __lane_id();
  const int rd = D.cur, wr = D.cur ^ 1;
  if (!D.spilled[rd][o]) {  // an owner of the LDS solves: its spill state stays empty
    if (tid == 0) {
      D.spilled[wr][o] = 0;
      D.sp_n[wr][o] = 0;
    }
    return;
  }
  const int64_t rb = D.off[(int64_t)o * D.nst], re = D.off[(int64_t)(o + 1) * D.nst];
  const int64_t nr = re - rb;
  const int64_t base = B.n > 0 ? B.ts[0] : 0;
  const int64_t W = D.within;
  const SwPred f2 = D.f2;
  const bool vnull = D.vtag == T_NULL, vflt = D.vtag == T_FLOAT;
  // the carry in: the LDS solves' arrays (sp_n < 0: spilled by this push's re-run) or the pool
  const bool from_pool = D.sp_n[rd][o] >= 0;
  const int64_t nin = from_pool ? D.sp_n[rd][o] : D.c_n[rd][o];
  const int64_t pin = from_pool ? D.sp_base[rd][o] : (int64_t)o * SWS_CCAP;
  const int64_t* in_ts = from_pool ? D.p_ts[rd] : D.c_ts[rd];
  const int64_t* in_seq = from_pool ? D.p_seq[rd] : D.c_seq[rd];
  const uint32_t* in_v = from_pool ? D.p_v[rd] : D.c_v[rd];
  const uint8_t* in_lk = from_pool ? D.p_lk[rd] : D.c_lk[rd];
  const uint8_t* in_null = from_pool ? D.p_null[rd] : D.c_null[rd];
  const int64_t sb = D.scr_base[o];  // this owner's scratch: nin + nr entries
  for (uint32_t k = tid; k <= (uint32_t)SW_LK; k += SP_THREADS) {
    nrec[k] = 0;
    ncar[k] = 0;
    cur[k] = 0;
  }
  __syncthreads();
  // 1. counts per key (records of the push, carried candidates)
  for (int64_t i = tid; i < nr; i += SP_THREADS) atomicAdd(&nrec[sw_lk(D.recs[rb + i].kt)], 1u);
  for (int64_t i = tid; i < nin; i += SP_THREADS) atomicAdd(&ncar[in_lk[pin + i]], 1u);
  __syncthreads();
  if (tid < 64) {  // scans over the keys: record lists (after the carry entries) and carry starts
    uint32_t rrun = 0, crun = 0;
    for (int b0 = 0; b0 <= SW_LK; b0 += 64) {
      const int b = b0 + (int)lane;
      const uint32_t r = b <= SW_LK ? nrec[b] : 0u, c = b <= SW_LK ? ncar[b] : 0u;
      uint32_t xr = r, xc = c;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t yr = __shfl_up(xr, d, 64), yc = __shfl_up(xc, d, 64);
        if (lane >= (uint32_t)d) {
          xr += yr;
          xc += yc;
        }
      }
      if (b <= SW_LK) {
        rbase[b] = rrun + xr - r;
        cbase[b] = crun + xc - c;
      }
      rrun += __shfl(xr, 63, 64);
      crun += __shfl(xc, 63, 64);
    }
  }
  __syncthreads();
  // stable scatter of record positions into per-key lists (one wave: rounds stay in arrival order)
  uint32_t* idx = D.s_idx + sb;  // nr entries, key-grouped
  if (tid < 64) {
    const uint64_t lt = sw_lanemask_lt();
    for (int64_t r0 = 0; r0 < nr; r0 += 64) {
      const int64_t i = r0 + lane;
      const bool v = i < nr;
      const uint32_t lk = v ? sw_lk(D.recs[rb + i].kt) : 0u;
      const uint64_t peers = sw_match_peers(lk, 8, v);
      if (v) {
        const uint32_t before = cur[lk];
        idx[rbase[lk] + before + (uint32_t)__popcll(peers & lt)] = (uint32_t)i;
        if ((peers & lt) == 0) cur[lk] = before + (uint32_t)__popcll(peers);
      }
    }
  }
  __syncthreads();
  // 2. replay, one thread per local key
  uint32_t nopen = 0, nlist = 0;  // this key's open candidates, and its list's length
  int64_t lbase = 0;
  if (tid < (uint32_t)SW_LK) {
    const uint32_t k = tid;
    const uint32_t nc = ncar[k], nk = nrec[k];
    // this key's candidate list: [lbase, lbase + nc + nk) of the scratch list arrays
    lbase = sb + (int64_t)cbase[k] + rbase[k];
    int64_t* L_ts = D.s_ts + lbase;
    int64_t* L_seq = D.s_seq + lbase;
    uint32_t* L_v = D.s_v + lbase;
    uint8_t* L_st = D.s_st + lbase;  // 1 pending, 2 null value
    uint32_t nl = 0;
    for (uint32_t j = 0; j < nc; j++) {
      const int64_t c = pin + cbase[k] + j;
      L_ts[nl] = in_ts[c];
      L_seq[nl] = in_seq[c];
      L_v[nl] = in_v[c];
      L_st[nl] = (uint8_t)(1u | (in_null[c] ? 2u : 0u));
      nl++;
    }
    uint8_t lastc = D.lastc[rd][(int64_t)o * SW_LK + k];
    int64_t prevc = (nc > 0 && lastc) ? (int64_t)nc - 1 : -1;  // on the new-and-every list
    uint32_t head = 0;
    double as = 0, an = 0;
    bool afn = false;
    if (D.agg) {
      as = D.agg_s[rd][(int64_t)o * SW_LK + k];
      an = D.agg_c[rd][(int64_t)o * SW_LK + k];
      afn = (D.agg == 4 || D.agg == 5) && an > 0 && as != as;
    }
    const int32_t kid = D.agg ? D.inv[(int64_t)o * SW_LK + k] : 0;
    for (uint32_t q = 0; q < nk; q++) {
      const SwRec rec = D.recs[rb + idx[rbase[k] + q]];
      const int64_t tq = base + sw_ts(rec.kt);
      // expireEvents: the pending list from its head (stops at the first live partial), then the
      // new-and-every list whole
      for (uint32_t p = head; p < nl; p++) {
        if (!(L_st[p] & 1u)) continue;
        if ((int64_t)p == prevc) break;
        const int64_t d = L_ts[p] - tq;
        if (d > W || d < -W) L_st[p] &= ~1u;
        else break;
      }
      if (prevc >= 0 && (L_st[prevc] & 1u)) {
        const int64_t d = L_ts[prevc] - tq;
        if (d > W || d < -W) L_st[prevc] &= ~1u;
      }
      const uint32_t ev = rec.v;
      double ef = 0, ei = 0;
      if constexpr (CT == 0) sw_conv(ev, vflt, ef, ei);
      const bool en = vnull || (rec.kt & SW_NULL) != 0;
      // processAndReturn: every pending partial in list order; count first, then one reservation
      uint32_t nm = 0;
      for (uint32_t p = head; p < nl; p++) {
        if (!(L_st[p] & 1u)) continue;
        const uint32_t av = L_v[p];
        double af = 0, ai = 0;
        if constexpr (CT == 0) sw_conv(av, vflt, af, ai);
        const bool an2 = vnull || (L_st[p] & 2u) != 0;
        const SwCand<CT> cd = sw_cand<NT2, CT>(f2, av, af, ai, an2);
        if (sw_close<NT2, CT, 0>(f2, cd, ev, ef, ei, en)) {
          L_st[p] |= 4u;  // closes at this event
          nm++;
        }
      }
      if (nm) {
        const unsigned long long gb = atomicAdd(O.count, (unsigned long long)nm);
        if (gb + nm > (unsigned long long)O.cap) atomicOr(err, E_OUT);
        const uint32_t rq = rec.ref;
        const int64_t sq = bseq(B, rq);
        uint32_t r = 0;
        double vq = 0;
        if (D.agg) {
          if (en && D.agg != 3) atomicOr(err, SWE_AGGNULL);
          vq = vflt ? (double)__uint_as_float(ev) : (double)(int32_t)ev;
        }
        for (uint32_t p = head; p < nl && r < nm; p++) {
          if (!(L_st[p] & 4u)) continue;
          L_st[p] &= ~5u;
          const uint64_t slot = gb + r++;
          if (slot >= (uint64_t)O.cap) continue;
          if (D.agg) {  // QuerySelector.processInBatchNoGroupBy per match (AvgAttributeAggregatorExecutor etc.)
            double val;
            if (D.agg == 4 || D.agg == 5) {  // min / max: first value, then `if (value > x) value = x`
              if (an == 0) {
                afn = vq != vq;
                as = vq;
              } else if (!afn && vq == vq) {
                as = D.agg == 4 ? (as > vq ? vq : as) : (as < vq ? vq : as);
              }
              an += 1;
              val = as;
            } else {
              as += vq;
              an += 1;
              val = D.agg == 1 ? as / an : (D.agg == 2 ? as : an);
            }
            O.key[slot] = kid;
            O.agg[slot] = val;
          } else if (D.p32) {
            const int64_t dq = sq - L_seq[p];
            if (dq >= (1ll << 32)) atomicOr(err, SWE_P32);
            reinterpret_cast<uint2*>(O.refs)[slot] = make_uint2(rq, (uint32_t)dq);
          } else if (B.seq) {
            *(longlong2*)(O.refs + 2 * slot) = make_longlong2(L_seq[p], (int64_t)rq);
          } else {
            *(longlong2*)(O.refs + 2 * slot) = make_longlong2(L_seq[p], sq);
          }
        }
      }
      if (rec.kt & SW_F1) {  // e1 matched: a new partial on the new-and-every list
        L_ts[nl] = tq;
        L_seq[nl] = bseq(B, rec.ref);
        L_v[nl] = ev;
        L_st[nl] = (uint8_t)(1u | ((rec.kt & SW_NULL) ? 2u : 0u));
        prevc = nl;
        nl++;
        lastc = 1;
      } else {
        prevc = -1;
        lastc = 0;
      }
      while (head < nl && !(L_st[head] & 1u)) head++;
    }
    if (D.agg) {
      D.agg_s[wr][(int64_t)o * SW_LK + k] = (D.agg == 4 || D.agg == 5) && afn ? __longlong_as_double(0x7ff8000000000000ll) : as;
      D.agg_c[wr][(int64_t)o * SW_LK + k] = an;
    }
    D.lastc[wr][(int64_t)o * SW_LK + k] = lastc;
    for (uint32_t p = 0; p < nl; p++) nopen += (L_st[p] & 1u) ? 1u : 0u;
    nlist = nl;
  }
  // 3. the carry out, key order: a block scan of the open counts
  uint32_t x = nopen;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) wt[tid >> 6] = x;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
  for (uint32_t i = 0; i < SP_THREADS / 64; i++) {
    pre += i < (tid >> 6) ? wt[i] : 0u;
    tot += wt[i];
  }
  pre += x - nopen;
  if (tid == 0) tot_out = tot;
  const bool back = tot <= (uint32_t)(SWS_CCAP / 2);  // back to the LDS solves
  if (tid < (uint32_t)SW_LK && nopen) {
    const int64_t* L_ts = D.s_ts + lbase;
    const int64_t* L_seq = D.s_seq + lbase;
    const uint32_t* L_v = D.s_v + lbase;
    const uint8_t* L_st = D.s_st + lbase;
    // the list as the replay left it: entries past nlist were never written (scratch garbage)
    const uint32_t nl = nlist;
    int64_t c = back ? (int64_t)o * SWS_CCAP + pre : D.sp_base[wr][o] + pre;
    int64_t* o_ts = back ? D.c_ts[wr] : D.p_ts[wr];
    int64_t* o_seq = back ? D.c_seq[wr] : D.p_seq[wr];
    uint32_t* o_v = back ? D.c_v[wr] : D.p_v[wr];
    uint8_t* o_lk = back ? D.c_lk[wr] : D.p_lk[wr];
    uint8_t* o_null = back ? D.c_null[wr] : D.p_null[wr];
    for (uint32_t p = 0; p < nl; p++) {
      if (!(L_st[p] & 1u)) continue;
      o_ts[c] = L_ts[p];
      o_seq[c] = L_seq[p];
      o_v[c] = L_v[p];
      o_lk[c] = (uint8_t)tid;
      o_null[c] = (L_st[p] & 2u) ? 1 : 0;
      c++;
    }
  }
  if (tid == 0) {
    D.spilled[wr][o] = back ? 0 : 1;
    D.sp_n[wr][o] = back ? 0 : (int32_t)tot;
    D.c_n[wr][o] = back ? (int32_t)tot : 0;
    if (!back) atomicAdd(D.sp_active, 1);
  }
}

// the owners whose carry overflowed in a push become spilled in the committed state (their carry
// stays in the LDS solves' arrays: sp_n = -1), for the re-run of that push
static __global__ void k_sw_mark_spilled(SweepDev D) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= D.nown) return;
  if (D.ovf[o]) {
    D.spilled[D.cur][o] = 1;
    D.sp_n[D.cur][o] = -1;
    D.ovf[o] = 0;
  }
}

// per owner: first record offset, record count, carry-in count (host sizing of the spill scratch)
static __global__ void k_sw_spill_sizes(SweepDev D, int64_t* out) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= D.nown) return;
  const int rd = D.cur;
  const int64_t rb = D.off[(int64_t)o * D.nst], re = D.off[(int64_t)(o + 1) * D.nst];
  out[3 * o] = D.spilled[rd][o];
  out[3 * o + 1] = re - rb;
  out[3 * o + 2] = D.sp_n[rd][o] >= 0 ? D.sp_n[rd][o] : D.c_n[rd][o];
}

}  // namespace shp
