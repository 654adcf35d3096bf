// siddhi-hip: k_sw_bal, the balanced form of k_sw_lean (included by sweep.h after sweep_lean.h).
//
// Same semantics, shape and hand-back rules as k_sw_lean (SURVEY.md Appendix A.7;
// StreamPreStateProcessor.processAndReturn / expireEvents :326-403): per key, candidate i closes at
// the first later event j of its key with ts_j - ts_i <= W and f2(i, j), expires at the first later
// event beyond W; matches per key in (j, i) order.  What changes is how a chunk's work is split
// over the 8 waves.  k_sw_lean gives each wave whole key runs, so with the ~20 keys an owner holds
// at C2 a wave gets 2 or 3 runs and every barrier waits for the most loaded one.  Here every wave
// takes exactly E / 8 sorted positions, wherever the key runs fall:
//   rank    stable ranks by local key (wave ballots, per-wave counters)            | barrier A
//   emit    the previous chunk's matches (its positions are intact until the place step)
//   scan    one wave: key run offsets (carried first) and per-wave write cursors    | barrier B
//   place   records and carried candidates at their sorted positions              | barrier C
//   probe   each wave's E / 8 positions: a candidate tests the next SW_P1 events of its key, then
//           the wave's worklist; a probe may read, and a closer may count into, positions of
//           another wave (LDS atomics on the closing position's distance bits)     | barrier D
//   offsets per lane a contiguous block of the wave's positions: closes and still-open
//           candidates, a wave scan, the wave totals                              | barrier E
//           then block offsets: each closing position's output offset (chunk-relative), and the
//           open candidates compacted in position order -- which is key order -- as the next
//           carry; one thread reserves the chunk's output with one global atomic.
// The carry therefore stays in key order without a per-key gather, and the final write-back is a
// straight copy.
#pragma once

namespace shp {

struct SwBalSmem {
  int2 tv[SL_EMAX + SL_PAD];         // (ts - chunk base, value) by sorted position; later x = output offset
  uint32_t ref[SL_EMAX];             // batch index (e1's filter in bit 31), or carry slot (carried)
  uint32_t cl[SL_EMAX];              // closers of this position: distance bits | far count << 24
  uint32_t meta[SL_EMAX + SL_PAD];   // local key | key run end << 8 | first event of the run << 20
  int16_t m[SL_EMAX];                // >= 0 closing position, -1 expired, -2 open, -3 not a candidate
  uint16_t wc[SL_WAVES][256];        // per-wave rank counters, then write cursors
  uint32_t binoff[257];              // key run starts
  uint16_t fe[256];                  // first event position of a key's run (after its carried)
  uint16_t cst[256], cen[256];       // carry prefix at a key's run start / after its run end
  uint16_t ckf[2][256];              // index of a key's first entry in carry buffer 0/1
  uint32_t ncar[256];                // carried candidates of a key in the current carry buffer
  uint8_t lastc[256];                // the key's latest event opened a candidate (SweepDev::lastc)
  uint8_t run[256];                  // the key has a run in the chunk being finished
  int64_t cts[2][SL_CCAP];           // carry: ts - batch base (exact)
  int64_t cseq[2][SL_CCAP];
  uint32_t cv[2][SL_CCAP];
  uint8_t clk[2][SL_CCAP];
  uint32_t wl[SL_WAVES][SL_WL];      // worklists: position | next probe position << 16
  uint32_t wt[SL_WAVES];             // per wave: closes << 16 | opens
  int32_t cn[2];                     // entries in carry buffer 0/1
  unsigned long long gbase;          // the chunk's output range (one global atomic per chunk)
  int32_t flag;
};

template <int CT, int OPC>
__global__ __launch_bounds__(SL_THREADS, 4) void k_sw_bal(SweepDev D, BatchView B, MatchOut O, int* err) {
  using T = typename SwTy<CT>::T;
  __shared__ SwBalSmem S;
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
    }
    if (tid == 0) D.c_n[wr][o] = n0;
    return;
  }
  const int nc0 = D.c_n[rd][o];
  if (D.tsmax[1] != 0 || nc0 > SL_CCAP) {  // a ts beyond base +- 2^30, or a carry larger than held here
    if (tid == 0) atomicOr(err, SWE_LEAN);
    return;
  }
  const int64_t base = B.ts[0];
  const int32_t W = (int32_t)D.within;
  const SwTerm t2 = D.f2.t[0];
  const bool bconst = t2.bk == 0;
  const T bc = (T)t2.bc;
  const int lkbits = D.lk_bits;
  const int nb = lkbits >= 8 ? SW_LK : (1 << lkbits);
  int e = 0;
  for (int i = tid; i < 256; i += SL_THREADS) {
    S.ncar[i] = 0;
    S.ckf[0][i] = 0;
    S.lastc[i] = i < SW_LK ? D.lastc[rd][(int64_t)o * SW_LK + i] : 0;
  }
  for (int i = tid; i < SL_WAVES * 256; i += SL_THREADS) (&S.wc[0][0])[i] = 0;
  if (tid == 0) {
    S.flag = 0;
    S.cn[0] = nc0;
    S.cn[1] = 0;
  }
  __syncthreads();
  // carry from the previous push (key order, as both solves write it): counts and first index per key
  for (int x = tid; x < nc0; x += SL_THREADS) {
    const int64_t c = (int64_t)o * SWS_CCAP + x;
    const uint32_t lk = D.c_lk[rd][c];
    S.cts[0][x] = D.c_ts[rd][c] - base;
    S.cv[0][x] = D.c_v[rd][c];
    S.cseq[0][x] = D.c_seq[rd][c];
    S.clk[0][x] = (uint8_t)lk;
    atomicAdd(&S.ncar[lk], 1u);
    if (x == 0 || D.c_lk[rd][c - 1] != lk) S.ckf[0][lk] = (uint16_t)x;
  }
  int cur = 0;
  SwRec pf[SL_R];
#pragma unroll
  for (int s = 0; s < SL_R; s++) {
    const int jj = (int)w * (64 * SL_R) + s * 64 + (int)lane;
    if (rb + jj < re) pf[s] = D.recs[rb + jj];
  }
  uint64_t tbk = D.recs[rb].kt;
  // emit a finished chunk's matches (this wave's positions of it): slot = offset(q) + (closes(q)
  // - 1 - later), later = closers of q nearer than p
  auto emit = [&](int PS, int PE, int pc) {
    const unsigned long long gb = S.gbase;
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
      const int64_t si = p < (int)(S.meta[p] >> 20) ? S.cseq[pc][r] : bseq(B, r);
      const int64_t sq = bseq(B, rq);
      const uint64_t slot = gb + (uint32_t)S.tv[q].x + (sl_closes(c) - 1u - later);
      if (slot < (uint64_t)O.cap) {
        if (D.p32) {
          const int64_t dq = sq - si;
          if (dq >= (1ll << 32)) e |= SWE_P32;
          reinterpret_cast<uint2*>(O.refs)[slot] = make_uint2(rq, (uint32_t)dq);
        } else if (B.seq) {
          *(longlong2*)(O.refs + 2 * slot) = make_longlong2(si, (int64_t)rq);
        } else {
          *(longlong2*)(O.refs + 2 * slot) = make_longlong2(si, sq);
        }
      }
    }
  };
  int pPS = 0, pPE = 0, pcur = 0;
  __syncthreads();
  for (int64_t cb = rb; cb < re; cb += SL_CHUNK) {
    const int nchunk = (int)min((int64_t)SL_CHUNK, re - cb);
    const int nx = cur ^ 1;
    const int32_t tb32 = (int32_t)(uint32_t)tbk;
    // 1. rank by local key (stable: wave-major, then slot, then lane = arrival order)
    uint32_t rk[SL_R], bin[SL_R];
#pragma unroll
    for (int s = 0; s < SL_R; s++) {
      const int j = (int)w * (64 * SL_R) + s * 64 + (int)lane;
      const bool valid = j < nchunk;
      const uint32_t lk = valid ? (uint32_t)(pf[s].kt >> 56) : 0u;
      const uint64_t peers = sw_match_peers(lk, lkbits, valid);
      bin[s] = valid ? lk : 0xFFFFu;
      rk[s] = 0;
      if (valid) {
        const uint32_t before = S.wc[w][lk];
        rk[s] = before + (uint32_t)__popcll(peers & lt);
        if ((peers & lt) == 0) S.wc[w][lk] = (uint16_t)(before + (uint32_t)__popcll(peers));
      }
    }
    __syncthreads();  // A
    if (S.flag) break;
    if (cb != rb) emit(pPS, pPE, pcur);  // the previous chunk's matches
    const int E = S.cn[cur] + nchunk;
    // 2. key run offsets and write cursors (wave 0); the previous chunk's per-key carry counts
    if (w == 0) {
      uint32_t run = 0;
      for (int b0 = 0; b0 < nb; b0 += 64) {
        const int b = b0 + (int)lane;
        const bool v = b < nb;
        uint32_t c[SL_WAVES], t = 0;
#pragma unroll
        for (int ww = 0; ww < SL_WAVES; ww++) {
          c[ww] = v ? S.wc[ww][b] : 0u;
          t += c[ww];
        }
        uint32_t nk = 0;
        if (v) {
          if (cb != rb) {  // the carry the previous chunk left: [cst, cen) of keys that had a run
            const bool had = S.run[b] != 0;
            nk = had ? (uint32_t)(S.cen[b] - S.cst[b]) : 0u;
            S.ckf[cur][b] = had ? S.cst[b] : (uint16_t)0;
            S.ncar[b] = nk;
          } else {
            nk = S.ncar[b];
          }
        }
        t += nk;
        uint32_t x = t;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const uint32_t y = __shfl_up(x, d, 64);
          if (lane >= (uint32_t)d) x += y;
        }
        const uint32_t pre = run + x - t;
        if (v) {
          S.binoff[b] = pre;
          S.fe[b] = (uint16_t)(pre + nk);
          S.run[b] = t ? 1 : 0;
          uint32_t g = pre + nk;
#pragma unroll
          for (int ww = 0; ww < SL_WAVES; ww++) {
            S.wc[ww][b] = (uint16_t)g;
            g += c[ww];
          }
        }
        run += __shfl(x, 63, 64);
      }
      if (lane == 0) S.binoff[nb] = run;  // = E
    }
    __syncthreads();  // B
    // 3. place records and carried candidates at their sorted positions
#pragma unroll
    for (int s = 0; s < SL_R; s++) {
      if (bin[s] == 0xFFFFu) continue;
      const uint32_t p = S.wc[w][bin[s]] + rk[s];
      const int32_t rel = (int32_t)(uint32_t)pf[s].kt - tb32;
      if (rel > (int32_t)SW_TS_SPAN || rel < -(int32_t)SW_TS_SPAN) S.flag = 1;
      S.tv[p] = make_int2(rel, (int32_t)pf[s].v);
      S.meta[p] = bin[s] | (S.binoff[bin[s] + 1] << 8) | ((uint32_t)S.fe[bin[s]] << 20);
      S.ref[p] = pf[s].ref | ((pf[s].kt & SW_F1) ? 0x80000000u : 0u);
    }
    {
      const int ncur = S.cn[cur];
      for (int x = tid; x < ncur; x += SL_THREADS) {
        const uint32_t lk = S.clk[cur][x];
        const uint32_t p = S.binoff[lk] + (uint32_t)x - S.ckf[cur][lk];
        const int64_t r = S.cts[cur][x] - (int64_t)tb32;
        if (r > SW_TS_SPAN) S.flag = 1;
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
    for (int p = tid; p < E; p += SL_THREADS) S.cl[p] = 0;
    {  // prefetch the next chunk while this one is solved
      const int64_t nbk = cb + SL_CHUNK;
#pragma unroll
      for (int s = 0; s < SL_R; s++) {
        const int jj = (int)w * (64 * SL_R) + s * 64 + (int)lane;
        if (nbk + jj < re) pf[s] = D.recs[nbk + jj];
      }
      if (nbk < re) tbk = D.recs[nbk].kt;
    }
    __syncthreads();  // C
    // ---- balanced: wave w takes sorted positions [PS, PE), E / 8 of them, across key runs
    const int PS = (int)(((int64_t)E * w) >> 3), PE = (int)(((int64_t)E * (w + 1)) >> 3);
    for (int b = (int)lane; b < nb; b += 64) S.wc[w][b] = 0;  // this wave's counters, next chunk
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
          res = sl_probe<CT, OPC, SW_P2>(S.tv, (int)qn, end, a.x, W, bv);
          qn += SW_P2;
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
    // 4. probe
    uint32_t nwl = 0;
    for (int g = PS; g < PE; g += 64) {
      const int p = g + (int)lane;
      int res = -3;
      uint32_t qn = 0;
      if (p < PE) {
        const uint32_t mt = S.meta[p];
        const int2 a = S.tv[p];
        const bool f1 = (S.ref[p] >> 31) != 0;
        const uint32_t mprev = p > 0 ? S.meta[p - 1] : 0xFFFFFFFFu;
        const int tprev = p > 0 ? S.tv[p - 1].x : 0;
        const uint32_t lk = mt & 0xFFu;
        const int end = (int)((mt >> 8) & 0xFFFu), fe = (int)(mt >> 20);
        const bool first = (mprev & 0xFFu) != lk;
        if (p == end - 1 && p >= fe) S.lastc[lk] = f1 ? 1 : 0;
        if (!first && tprev > a.x) S.flag = 1;  // ts decrease within the key: exact kernel
        if (p < fe || f1) {
          const T bv = bconst ? bc : sw_val<CT>((uint32_t)a.y, 0.0, 0.0, false);
          const int q0 = max(p + 1, fe);
          res = sl_probe<CT, OPC, SW_P1>(S.tv, q0, end, a.x, W, bv);
          qn = (uint32_t)(q0 + SW_P1);
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
    __syncthreads();  // D: every closer has been counted
    // 5. closes and open candidates per position (contiguous block per lane)
    const int nw = PE - PS;
    const int K = (nw + 63) >> 6;
    const int lb = PS + (int)lane * K, le = min(lb + K, PE);
    uint32_t cs = 0, os = 0;
    for (int q = lb; q < le; q++) {
      cs += sl_closes(S.cl[q]);
      os += S.m[q] == -2 ? 1u : 0u;
    }
    const uint32_t pk = (cs << 16) | os;
    uint32_t incl = pk;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(incl, d, 64);
      if (lane >= (uint32_t)d) incl += y;
    }
    if (lane == 63) S.wt[w] = incl;
    __syncthreads();  // E
    uint32_t wbase = 0, tot = 0;
#pragma unroll
    for (int ww = 0; ww < SL_WAVES; ww++) {
      const uint32_t t = S.wt[ww];
      wbase += (uint32_t)ww < w ? t : 0u;
      tot += t;
    }
    const uint32_t ctot = tot >> 16, otot = tot & 0xFFFFu;
    if (otot > (uint32_t)SL_CCAP) S.flag = 1;
    if (tid == 0) {
      const unsigned long long g0 = ctot ? atomicAdd(O.count, (unsigned long long)ctot) : 0ull;
      if (g0 + ctot > (unsigned long long)O.cap) e |= E_OUT;
      S.gbase = g0;
      S.cn[nx] = (int32_t)min(otot, (uint32_t)SL_CCAP);
    }
    {
      const uint32_t ex = wbase + incl - pk;
      uint32_t co = ex >> 16, oo = ex & 0xFFFFu;
      for (int q = lb; q < le; q++) {
        const uint32_t c = sl_closes(S.cl[q]);
        const uint32_t f = S.meta[q];
        const uint32_t lk = f & 0xFFu;
        if (q == 0 || (S.meta[q - 1] & 0xFFu) != lk) S.cst[lk] = (uint16_t)oo;  // the key's run starts here
        if (S.m[q] == -2) {
          const int x = (int)oo;
          if (x < SL_CCAP) {
            const uint32_t r = S.ref[q] & 0x7FFFFFFFu;
            if (q < (int)(f >> 20)) {  // carried
              S.cts[nx][x] = S.cts[cur][r];
              S.cv[nx][x] = S.cv[cur][r];
              S.cseq[nx][x] = S.cseq[cur][r];
            } else {
              const int2 a = S.tv[q];
              S.cts[nx][x] = (int64_t)tb32 + a.x;
              S.cv[nx][x] = (uint32_t)a.y;
              S.cseq[nx][x] = bseq(B, r);
            }
            S.clk[nx][x] = (uint8_t)lk;
          }
          oo++;
        }
        if (q + 1 == (int)((f >> 8) & 0xFFFu)) S.cen[lk] = (uint16_t)oo;  // the key's run ends here
        S.tv[q].x = (int32_t)co;
        co += c;
      }
    }
    pPS = PS;
    pPE = PE;
    pcur = cur;
    cur = nx;
  }
  __syncthreads();
  if (S.flag) {
    if (tid == 0) atomicOr(err, SWE_LEAN);
    return;
  }
  emit(pPS, pPE, pcur);  // the last chunk's matches
  // write back the carry: already in key order (position order)
  const int ncf = S.cn[cur];
  for (int x = tid; x < ncf; x += SL_THREADS) {
    const int64_t c = (int64_t)o * SWS_CCAP + x;
    D.c_ts[wr][c] = base + S.cts[cur][x];
    D.c_seq[wr][c] = S.cseq[cur][x];
    D.c_v[wr][c] = S.cv[cur][x];
    D.c_lk[wr][c] = S.clk[cur][x];
    D.c_null[wr][c] = 0;
  }
  for (int i = tid; i < SW_LK; i += SL_THREADS) D.lastc[wr][(int64_t)o * SW_LK + i] = S.lastc[i];
  if (tid == 0) D.c_n[wr][o] = ncf;
  if (e) atomicOr(err, e);
}

}  // namespace shp
