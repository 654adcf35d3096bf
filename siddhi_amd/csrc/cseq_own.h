// siddhi-hip: the count-sequence path by owners (round 4; C3' with SHP_LAYOUT_CHAIN32).
//
// Same rule as k_cs3 (cseq.h; CountPreStateProcessor.java:53-95, CountPostStateProcessor.java:
// 39-79 for `every e1=S[f1]<1:M>, e2=S[f2(e1[last], e2)]` in a partition): per key, L in 0..M
// before each event, f1(x) without f2 -> T10, f1(x) and f2 -> T11, neither -> 0; an event with
// L > 0 and f2 closes a match whose e1 chain is the key's L events just before it.  Instead of a
// global key sort (three rocPRIM onesweep passes over 21 key bits, 2.9 of C3''s 6.6 ms), the push
// is partitioned the way the sweep partitions C2 (sweep.h), and each owner's events are put in key
// order chunk by chunk in LDS:
//   k_co_count    super-tile x owner histogram, the push's max ts       reads key (+stream), ts
//   exclusive scan of the NOWN x NST counts (owner-major)
//   k_co_scatter  stable multisplit by owner (wave ballot ranks); evaluates f1; writes a 12-byte
//                 record {value, batch index | null, local key | f1}     reads key, value, writes 12 B
//   k_co_run      one workgroup per owner walks its region in chunks of CO_CHUNK records: stable
//                 split by local key in LDS, the transition tables composed along each key run
//                 (block segmented scan, seeded with the key's L from LDS), then each closing event
//                 writes its CHAIN32 word (e2's batch index | L << 28) at an offset reserved with one
//                 atomic per chunk (a key's matches stay in emission order: a workgroup's chunks run
//                 in order).  Per key in LDS across chunks: L, the previous value and null flag and a
//                 ring of the batch indices of its last M events; written back to the key state (copy
//                 wr, as k_cs_state's) when the owner ends.
// The e1 chains are implied by the words (the key's L events before e2); shp_fetch_matches and the
// group gather materialise FULL records from them (CseqState::expand: the push's events sorted by
// key, each word's e2 found by binary search, chain events before the push from the stored history).
// (Included by cseq.h after its kernels: uses CseqDev, the transition tables and sw_* helpers.)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace shp {

constexpr int CO_THREADS = 512;
constexpr int CO_WAVES = CO_THREADS / 64;
constexpr int CO_PER = 4;                       // sorted positions per thread per chunk
constexpr int CO_CHUNK = CO_THREADS * CO_PER;   // records per chunk
constexpr int CO_SEG = CO_CHUNK / CO_WAVES;     // a wave's records of the chunk, in arrival order
constexpr int CO_SUB = CO_SEG / 64;
constexpr int CO_KPO_MAX = 1024;                // local keys per owner
constexpr int CO_KEY_LDS = 32768;               // per-key state budget (L, value, null, ring of M)
constexpr int CO_MAXOWN = 1024;
constexpr int CO_MINOWN = 256;
constexpr int CO_CNT_THREADS = 256;
#ifndef CO_SCT_PER_CFG
#define CO_SCT_PER_CFG 8
#endif
constexpr int CO_SCT_THREADS = 512;
constexpr int CO_SCT_WAVES = CO_SCT_THREADS / 64;
constexpr int CO_SCT_ROUND = CO_SCT_THREADS * CO_SCT_PER_CFG;  // events ranked per round
constexpr int CO_SCT_SEG = CO_SCT_ROUND / CO_SCT_WAVES;
constexpr int CO_SCT_SUB = CO_SCT_SEG / 64;
constexpr int64_t CO_STLEN = 65536;             // events per super-tile
constexpr uint32_t CH32_G = (1u << 28) - 1u;    // CHAIN32 word: e2's batch index | L << 28
constexpr uint32_t CO_F1 = 1u << 15;            // LDS local-key word: e1's filter holds

struct CoRec {
  uint32_t v;   // the value column's bits
  uint32_t g;   // batch index | null << 31
  uint32_t lk;  // local key | f1 << 31
};

struct CoDev {
  int32_t nown, bits, kpo, lkbits, nst, pad;
  uint32_t* cnt;  // nown * nst + 1: counts, scanned into off
  uint32_t* off;
  CoRec* recs;    // cap: owner-major, arrival order within an owner
};

// ------------------------------------------------------------------ pass 1: count (and the max ts)
static __global__ __launch_bounds__(CO_CNT_THREADS) void k_co_count(CoDev P, BatchView B, const int32_t* __restrict__ key,
                                                                 const int32_t* __restrict__ stream, uint32_t nk,
                                                                 unsigned long long* tsmax, int* err) {
  __shared__ uint32_t h[CO_MAXOWN];
  const int st = blockIdx.x;
  for (int b = threadIdx.x; b < P.nown; b += CO_CNT_THREADS) h[b] = 0;
  __syncthreads();
  const int64_t lo = (int64_t)st * CO_STLEN, hi = min(B.n, lo + CO_STLEN);
  const uint32_t mask = (uint32_t)P.nown - 1u;
  int e = 0;
  int64_t mx = INT64_MIN;
  constexpr int U = 4;  // loads in flight per thread
  for (int64_t i0 = lo + threadIdx.x; i0 < hi; i0 += (int64_t)CO_CNT_THREADS * U) {
    int32_t kk[U];
    int64_t tt[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t i = i0 + (int64_t)u * CO_CNT_THREADS;
      kk[u] = -2;
      tt[u] = INT64_MIN;
      if (i < hi && (!stream || stream[i] >= 0)) {  // (stream < 0: a clock-only event)
        kk[u] = B.partitioned ? key[i] : 0;
        tt[u] = B.ts[i];
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      mx = max(mx, tt[u]);
      if (kk[u] == -2) continue;
      if (kk[u] < 0 || (uint32_t)kk[u] >= nk) e |= SWE_KEYS;
      else atomicAdd(&h[(uint32_t)kk[u] & mask], 1u);
    }
  }
  if (e) atomicOr(err, e);
  for (int d = 32; d > 0; d >>= 1) mx = max(mx, (int64_t)__shfl_xor((long long)mx, d, 64));
  if (__lane_id() == 0 && mx != INT64_MIN) atomicMax(tsmax, (unsigned long long)mx ^ (1ull << 63));
  __syncthreads();
  for (int b = threadIdx.x; b < P.nown; b += CO_CNT_THREADS) P.cnt[(int64_t)b * P.nst + st] = h[b];
  if (st == 0 && threadIdx.x == 0) P.cnt[(int64_t)P.nown * P.nst] = 0;
}

// ------------------------------------------------------------------ pass 2: stable scatter by owner
// dynamic LDS: per-wave counts, then write cursors [CO_SCT_WAVES][nown], and the running owner
// offsets [nown]
// PF (no stream column, no null bytes): the next round's keys and values are loaded as soon as this
// round's are consumed (as k_sw_scatter's PF path)
// STG (PF only, round 5, the default for PF): the round's records placed in LDS in owner order, then
// written out by position, so a store instruction covers whole owner runs (k_sw_scatter's STG form);
// extra LDS: lofs [nown] and the stage, CO_SCT_ROUND x 4 words (104 KB at 1024 owners).  Measured
// 1.21 -> 1.08 ms on C3' (profiles/r05_scatter_stage_ab.txt); the sweep's 12-byte scatter lost with it.
template <int NT1, bool PF, bool STG = false>
__global__ __launch_bounds__(CO_SCT_THREADS) void k_co_scatter(CoDev P, CseqDev C, BatchView B,
                                                               const int32_t* __restrict__ key,
                                                               const int32_t* __restrict__ stream) {
  static_assert(!STG || PF, "the staged scatter is built for the prefetched form");
  extern __shared__ uint32_t co_dyn[];
  const int nown = P.nown;
  uint32_t* grun = co_dyn + CO_SCT_WAVES * nown;
  const int st = blockIdx.x;
  const uint32_t lane = __lane_id(), w = threadIdx.x >> 6;
  uint32_t* wcw = co_dyn + w * nown;
  const uint64_t lt = sw_lanemask_lt();
  for (int b = threadIdx.x; b < nown; b += CO_SCT_THREADS) grun[b] = P.off[(int64_t)b * P.nst + st];
  const int64_t lo = (int64_t)st * CO_STLEN, hi = min(B.n, lo + CO_STLEN);
  const uint32_t* vcol = (const uint32_t*)B.cols[0];
  const uint8_t* ncol = B.nulls[0];
  const bool vnull = C.vtag == T_NULL, vflt = C.vtag == T_FLOAT;
  const uint32_t nk = (uint32_t)C.nk, mask = (uint32_t)nown - 1u;
  int32_t pk[PF ? CO_SCT_SUB : 1];
  uint32_t pv[PF ? CO_SCT_SUB : 1];
  auto load_round = [&](int64_t r0) {
#pragma unroll
    for (int s = 0; s < (PF ? CO_SCT_SUB : 0); s++) {
      const int64_t i = r0 + (int64_t)w * CO_SCT_SEG + s * 64 + lane;
      pk[s] = i < hi ? (B.partitioned ? key[i] : 0) : -1;
      pv[s] = (i < hi && vcol) ? vcol[i] : 0u;
    }
  };
  if (PF) load_round(lo);
  for (int64_t r0 = lo; r0 < hi; r0 += CO_SCT_ROUND) {
    CoRec rec[CO_SCT_SUB];
    int32_t kk[CO_SCT_SUB];
    uint8_t nl[CO_SCT_SUB];
#pragma unroll
    for (int s = 0; s < CO_SCT_SUB; s++) {  // every load of the round first
      const int64_t i = r0 + (int64_t)w * CO_SCT_SEG + s * 64 + lane;
      kk[s] = -1;
      nl[s] = 0;
      rec[s].v = 0;
      if constexpr (PF) {
        kk[s] = (pk[s] >= 0 && (uint32_t)pk[s] < nk) ? pk[s] : -1;
        rec[s].v = pv[s];
      } else if (i < hi && (!stream || stream[i] >= 0)) {
        const int32_t k = B.partitioned ? key[i] : 0;
        kk[s] = (k >= 0 && (uint32_t)k < nk) ? k : -1;  // (out of range: k_co_count flagged it)
        rec[s].v = vcol ? vcol[i] : 0u;
        nl[s] = ncol ? ncol[i] : 0;
      }
      rec[s].g = (uint32_t)i;
    }
    if (PF && r0 + CO_SCT_ROUND < hi) load_round(r0 + CO_SCT_ROUND);
    for (int b = lane; b < nown; b += 64) wcw[b] = 0;
    __syncthreads();
    uint32_t own[CO_SCT_SUB], rk[CO_SCT_SUB], pc[CO_SCT_SUB], ld[CO_SCT_SUB];
#pragma unroll
    for (int s = 0; s < CO_SCT_SUB; s++) {
      const bool valid = kk[s] >= 0;
      const uint32_t o = valid ? ((uint32_t)kk[s] & mask) : 0u;
      if (valid) {
        const bool xn = vnull || nl[s] != 0;
        double xf, xi;
        sw_conv(rec[s].v, vflt, xf, xi);
        const bool a = sw_pred<NT1>(C.f1, xf, xi, xn, 0.0, 0.0, true);
        rec[s].g |= nl[s] ? 0x80000000u : 0u;
        rec[s].lk = ((uint32_t)kk[s] >> P.bits) | (a ? 0x80000000u : 0u);
      }
      const uint64_t peers = sw_match_peers(o, P.bits, valid);
      rk[s] = (uint32_t)__popcll(peers & lt);
      own[s] = valid ? o : 0xffffffffu;
      pc[s] = (valid && (peers & lt) == 0) ? (uint32_t)__popcll(peers) : 0u;  // leader: group size
      ld[s] = peers ? (uint32_t)__ffsll((unsigned long long)peers) - 1u : 0u;
    }
    // the leaders' LDS adds of all sub-rounds back to back (a wave's LDS operations stay in order)
    uint32_t old[CO_SCT_SUB];
#pragma unroll
    for (int s = 0; s < CO_SCT_SUB; s++) old[s] = pc[s] ? atomicAdd(&wcw[own[s]], pc[s]) : 0u;
#pragma unroll
    for (int s = 0; s < CO_SCT_SUB; s++) rk[s] += __shfl(old[s], (int)ld[s], 64);
    __syncthreads();
    if constexpr (STG) {
      __shared__ uint32_t stg_w[CO_SCT_WAVES];
      uint32_t* lofs = grun + nown;
      uint32_t* sv = lofs + nown;
      uint32_t* sg = sv + CO_SCT_ROUND;
      uint32_t* slk = sg + CO_SCT_ROUND;
      uint32_t* sdst = slk + CO_SCT_ROUND;
      const int per = (nown + CO_SCT_THREADS - 1) / CO_SCT_THREADS;
      const int b0 = min(nown, (int)threadIdx.x * per), b1 = min(nown, b0 + per);
      uint32_t tsum = 0;
      for (int b = b0; b < b1; b++)
#pragma unroll
        for (int ww = 0; ww < CO_SCT_WAVES; ww++) tsum += co_dyn[ww * nown + b];
      const uint32_t inc = dpp_incl_add(tsum, lane);
      if (lane == 63) stg_w[w] = inc;
      __syncthreads();
      uint32_t tot = 0, wpre = 0;
#pragma unroll
      for (int ww = 0; ww < CO_SCT_WAVES; ww++) {
        const uint32_t t = stg_w[ww];
        wpre += ww < (int)w ? t : 0u;
        tot += t;
      }
      uint32_t g = wpre + inc - tsum;
      for (int b = b0; b < b1; b++) {
        lofs[b] = g;
#pragma unroll
        for (int ww = 0; ww < CO_SCT_WAVES; ww++) {
          const uint32_t c = co_dyn[ww * nown + b];
          co_dyn[ww * nown + b] = g;
          g += c;
        }
      }
      __syncthreads();
#pragma unroll
      for (int s = 0; s < CO_SCT_SUB; s++)
        if (own[s] != 0xffffffffu) {
          const uint32_t o = own[s];
          const uint32_t p = wcw[o] + rk[s];
          sv[p] = rec[s].v;
          sg[p] = rec[s].g;
          slk[p] = rec[s].lk;
          sdst[p] = grun[o] + (p - lofs[o]);
        }
      __syncthreads();
      // only the round's records are stored (the recs array has no trash slot)
#pragma unroll
      for (int q = 0; q < CO_SCT_PER_CFG; q++) {
        const uint32_t p = (uint32_t)(q * CO_SCT_THREADS) + threadIdx.x;
        if (p < tot) {
          CoRec r;
          r.v = sv[p];
          r.g = sg[p];
          r.lk = slk[p];
          P.recs[sdst[p]] = r;
        }
      }
      for (int b = b0; b < b1; b++) grun[b] += (b + 1 < nown ? lofs[b + 1] : tot) - lofs[b];
      __syncthreads();
      continue;
    }
    for (int b = threadIdx.x; b < nown; b += CO_SCT_THREADS) {
      uint32_t g = grun[b];
#pragma unroll
      for (int ww = 0; ww < CO_SCT_WAVES; ww++) {
        const uint32_t c = co_dyn[ww * nown + b];
        co_dyn[ww * nown + b] = g;
        g += c;
      }
      grun[b] = g;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < CO_SCT_SUB; s++)
      if (own[s] != 0xffffffffu) P.recs[wcw[own[s]] + rk[s]] = rec[s];
    __syncthreads();
  }
}

// exclusive scan of one value per thread over the CO_THREADS threads (sc: CO_WAVES words of LDS)
__device__ __forceinline__ uint32_t co_block_scan(uint32_t v, uint32_t* sc, uint32_t& total) {
  const uint32_t lane = __lane_id(), w = threadIdx.x >> 6;
  const uint32_t x = dpp_incl_add(v, lane);
  if (lane == 63) sc[w] = x;
  __syncthreads();
  uint32_t pre = 0;
  total = 0;
#pragma unroll
  for (int i = 0; i < CO_WAVES; i++) {
    const uint32_t t = sc[i];
    pre += (uint32_t)i < w ? t : 0u;
    total += t;
  }
  __syncthreads();
  return pre + x - v;
}

// Transition tables as 8 bytes (byte i = L after, from L = i), composed with two byte permutes.
// The tables (cs_tables' modes) on L in 0..7: a state past M is either M (every: T* map it like 0)
// or the dead state M + 1 (no every), so inputs 0..7 cover M <= 7 (M <= 6 without every) and every
// output value is a valid selector of the next composition; larger M run on the sorted records.
__device__ __forceinline__ uint64_t co_const(uint32_t c) { return 0x0101010101010101ull * (uint64_t)c; }
__device__ __forceinline__ uint32_t co_at(uint64_t f, uint32_t i) { return (uint32_t)(f >> (8 * i)) & 0xffu; }
__device__ __forceinline__ uint64_t co_comp(uint64_t g, uint64_t f) {  // g after f
  const uint32_t gl = (uint32_t)g, gh = (uint32_t)(g >> 32);
  const uint32_t lo = __builtin_amdgcn_perm(gh, gl, (uint32_t)f);
  const uint32_t hi = __builtin_amdgcn_perm(gh, gl, (uint32_t)(f >> 32));
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ void co_tables(int M, int mode, uint64_t& t0, uint64_t& t10, uint64_t& t11) {
  uint64_t n0, n10, n11;  // cs_tables' nibbles, widened to bytes
  cs_tables(M, mode, n0, n10, n11);
  t0 = t10 = t11 = 0;
  for (int i = 0; i < 8; i++) {
    t0 |= ((n0 >> (4 * i)) & 15u) << (8 * i);
    t10 |= ((n10 >> (4 * i)) & 15u) << (8 * i);
    t11 |= ((n11 >> (4 * i)) & 15u) << (8 * i);
  }
}
constexpr uint64_t CO_IDENT = 0x0706050403020100ull;
constexpr int CO_MAXM = 7;

struct CoSmem {
  uint32_t cv[CO_CHUNK];       // the chunk in key order: value
  uint32_t cg[CO_CHUNK];       // batch index | null << 31
  uint16_t cl[CO_CHUNK + 2];   // local key | f1 (CO_F1)
  uint64_t wt[CO_WAVES];       // a wave's composed transition table
  int32_t wf[CO_WAVES];        // ... whether it holds a run start
  int32_t wh[CO_WAVES];        // ... its latest run start
  uint32_t sc[CO_WAVES];
  uint32_t base;
  unsigned long long fb[2];    // FULL rows: the chunk's first match and first ref
};

// dynamic LDS after CoSmem: wc[CO_WAVES][kpo + 1] (uint16, per-wave counts then cursors), then per
// key: sP[kpo] (uint32), sH[M][kpo] (uint32 ring), sL, sN, sRh, sRf [kpo] (uint8)
__host__ __device__ inline size_t co_wc_stride(int kpo) { return (size_t)((kpo + 2) & ~1); }
__host__ __device__ inline size_t co_dyn_bytes(int kpo, int M) {
  return (size_t)CO_WAVES * co_wc_stride(kpo) * 2 + (size_t)kpo * (4 + 4 * (size_t)M + 4);
}

// (<= 128 VGPRs: two 512-thread workgroups per CU, as their LDS allows)
// FR: FULL rows (else CHAIN32 words) -- a template parameter, so the words' variant keeps the wait
// counters it had (the rows' gathers wait on their loads; tools/isa_check.py)
template <int NT2, bool FR>
__global__ __launch_bounds__(CO_THREADS) __attribute__((amdgpu_waves_per_eu(4))) void k_co_run(CoDev P, CseqDev C, BatchView B, MatchOut O, int* err) {
  __shared__ CoSmem S;
  extern __shared__ uint8_t co_key[];
  const int kpo = P.kpo, M = C.M;
  const size_t wst = co_wc_stride(kpo);
  uint16_t* wc = reinterpret_cast<uint16_t*>(co_key);
  uint32_t* sP = reinterpret_cast<uint32_t*>(co_key + (size_t)CO_WAVES * wst * 2);
  uint32_t* sH = sP + kpo;
  uint8_t* sL = reinterpret_cast<uint8_t*>(sH + (size_t)M * kpo);
  uint8_t* sN = sL + kpo;
  uint8_t* sRh = sN + kpo;
  uint8_t* sRf = sRh + kpo;
  const int o = blockIdx.x;
  const int tid = threadIdx.x;
  const uint32_t lane = __lane_id(), w = (uint32_t)tid >> 6;
  const int rd = C.cur, wr = C.cur ^ 1;
  const uint32_t nk = (uint32_t)C.nk;
  const bool vnull = C.vtag == T_NULL, vflt = C.vtag == T_FLOAT;
  uint64_t t0, t10, t11;
  co_tables(M, C.mode, t0, t10, t11);
  const uint64_t ident = CO_IDENT;
  // the owner's keys' state (the previous push)
  for (int lk = tid; lk < kpo; lk += CO_THREADS) {
    const uint32_t k = ((uint32_t)lk << P.bits) | (uint32_t)o;
    const bool in = k < nk;
    sL[lk] = in ? C.len[rd][k] : 0;
    sP[lk] = in ? C.prev[rd][k] : 0u;
    sN[lk] = in ? C.pnull[rd][k] : 1;
    sRh[lk] = 0;
    sRf[lk] = 0;
  }
  const int64_t rb = P.off[(int64_t)o * P.nst], re = P.off[(int64_t)(o + 1) * P.nst];
  const uint64_t lt = sw_lanemask_lt();
  uint32_t* words = reinterpret_cast<uint32_t*>(O.refs);
  int e = 0;
  // a chunk's words are written during the next chunk, after its rank step: the output
  // reservation's atomic (tid 0) is then published to LDS at the next chunk's first barrier instead
  // of being waited on at once, and the stores are no longer the last memory operations before the
  // wait for the prefetched records (which, with stores in flight, waits for them too)
  uint32_t pw[CO_PER];        // the previous chunk's words of this thread (positions with pem bits)
  uint32_t pem = 0, pmo = 0;  // ... which positions emitted, and the thread's offset in the chunk
  unsigned long long pres = 0;  // (tid 0) the previous chunk's reserved base
  bool ppend = false;
#pragma unroll
  for (int q = 0; q < CO_PER; q++) pw[q] = 0;
  auto flush_words = [&]() {
    if (pem) {
      const int64_t base = (int64_t)S.base;
#pragma unroll
      for (int q = 0; q < CO_PER; q++)
        if ((pem >> q) & 1u) {
          const int64_t mi = base + pmo + __popc(pem & ((1u << q) - 1u));
          if (mi >= O.cap) e |= E_OUT;
          else words[mi] = pw[q];
        }
      pem = 0;
    }
  };
  // the chunk's records, loaded one chunk ahead (in flight while the previous chunk is solved)
  CoRec r[CO_SUB];
#pragma unroll
  for (int s = 0; s < CO_SUB; s++) {
    const int64_t i = rb + (int64_t)w * CO_SEG + s * 64 + lane;
    r[s] = i < re ? P.recs[i] : CoRec{0u, 0u, 0u};
  }
  for (int64_t c0 = rb; c0 < re; c0 += CO_CHUNK) {
    const int nc = (int)min((int64_t)CO_CHUNK, re - c0);
    {
      uint32_t* z = reinterpret_cast<uint32_t*>(wc + w * wst);  // (wst is even)
      for (int i = lane; i < (int)(wst >> 1); i += 64) z[i] = 0;
    }
    if (ppend) {  // (tid 0; the whole 64-bit result, so its registers stay reserved until here)
      if (pres >> 32) e |= E_OUT;
      S.base = (uint32_t)pres;
      ppend = false;
    }
    __syncthreads();
    // rank: stable within the chunk (waves own consecutive segments, sub-rounds in order)
    uint32_t lkq[CO_SUB], rk[CO_SUB];
#pragma unroll
    for (int s = 0; s < CO_SUB; s++) {
      const int i = (int)w * CO_SEG + s * 64 + (int)lane;
      const bool valid = i < nc;
      lkq[s] = r[s].lk & 0x7fffffffu;
      const uint64_t peers = sw_match_peers(lkq[s], P.lkbits, valid);
      const uint32_t below = (uint32_t)__popcll(peers & lt);
      const bool lead = valid && (peers & lt) == 0;
      const uint32_t ldl = peers ? (uint32_t)__ffsll((unsigned long long)peers) - 1u : 0u;
      uint32_t old = 0;
      if (lead) {
        old = wc[w * wst + lkq[s]];
        wc[w * wst + lkq[s]] = (uint16_t)(old + (uint32_t)__popcll(peers));
      }
      rk[s] = below + __shfl(old, (int)ldl, 64);
    }
    flush_words();  // the previous chunk's (S.base published before the barrier above)
    __syncthreads();
    // per-key totals -> key offsets -> per-wave cursors (a thread takes consecutive local keys)
    {
      const int per = (kpo + CO_THREADS - 1) / CO_THREADS;
      const int l0 = tid * per;
      uint32_t sum = 0;
      for (int l = l0; l < min(kpo, l0 + per); l++)
        for (int ww = 0; ww < CO_WAVES; ww++) sum += wc[ww * wst + l];
      uint32_t tot;
      uint32_t g = co_block_scan(sum, S.sc, tot);
      for (int l = l0; l < min(kpo, l0 + per); l++)
        for (int ww = 0; ww < CO_WAVES; ww++) {
          const uint32_t c = wc[ww * wst + l];
          wc[ww * wst + l] = (uint16_t)g;
          g += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < CO_SUB; s++) {
      const int i = (int)w * CO_SEG + s * 64 + (int)lane;
      if (i < nc) {
        const uint32_t p = wc[w * wst + lkq[s]] + rk[s];
        S.cv[p] = r[s].v;
        S.cg[p] = r[s].g;
        S.cl[p] = (uint16_t)(lkq[s] | ((r[s].lk >> 31) ? CO_F1 : 0u));
      }
    }
    if (tid == 0) S.cl[nc] = 0xffffu;  // run-end sentinel
#pragma unroll
    for (int s = 0; s < CO_SUB; s++) {  // the next chunk's records
      const int64_t i = c0 + CO_CHUNK + (int64_t)w * CO_SEG + s * 64 + lane;
      r[s] = i < re ? P.recs[i] : CoRec{0u, 0u, 0u};
    }
    __syncthreads();
    // walk 1: per position f1 / f2 / run start bits, the key's stored L at a run start, and the
    // thread's composed transition table
    const int p0 = tid * CO_PER;
    uint32_t hb = 0, ab = 0, bb = 0, vb = 0;
    uint32_t L0q = 0;
    uint64_t G = ident;
    int gs = 0, lh = -1;
    uint32_t px = 0;
    bool pxn = true;
    if (p0 > 0 && p0 < nc) {
      px = S.cv[p0 - 1];
      pxn = vnull || (S.cg[p0 - 1] >> 31) != 0;
    }
    uint32_t kprev = p0 > 0 && p0 <= nc ? (S.cl[p0 - 1] & 0x7fffu) : 0xffffu;
    // the thread's positions in one 16-byte (values, batch indices) and 8-byte (keys) LDS read each
    static_assert(CO_PER == 4, "vector LDS reads of 4 positions");
    const uint4 xv4 = reinterpret_cast<const uint4*>(S.cv)[tid];
    const uint4 xg4 = reinterpret_cast<const uint4*>(S.cg)[tid];
    const uint2 xl2 = reinterpret_cast<const uint2*>(S.cl)[tid];
    const uint32_t xv[4] = {xv4.x, xv4.y, xv4.z, xv4.w};
    const uint32_t xg[4] = {xg4.x, xg4.y, xg4.z, xg4.w};
    const uint32_t xl[4] = {xl2.x & 0xffffu, xl2.x >> 16, xl2.y & 0xffffu, xl2.y >> 16};
#pragma unroll
    for (int q = 0; q < CO_PER; q++) {
      const int p = p0 + q;
      if (p >= nc) break;
      const uint32_t cl = xl[q], lk = cl & 0x7fffu;
      const bool head = p == 0 || lk != kprev;
      kprev = lk;
      const uint32_t x = xv[q];
      const bool xn = vnull || (xg[q] >> 31) != 0;
      uint32_t L0 = 0;
      if (head) {
        L0 = sL[lk];
        px = sP[lk];
        pxn = sN[lk] != 0;
        L0q |= L0 << (4 * q);
        lh = p;
      }
      double xf, xi, pf, pi;
      sw_conv(x, vflt, xf, xi);
      sw_conv(px, vflt, pf, pi);
      const bool a = (cl & CO_F1) != 0;
      const bool b = sw_pred<NT2>(C.f2, pf, pi, pxn, xf, xi, xn);
      const uint64_t F = a ? (b ? t11 : t10) : t0;
      hb |= (head ? 1u : 0u) << q;
      ab |= (a ? 1u : 0u) << q;
      bb |= (b ? 1u : 0u) << q;
      vb |= 1u << q;
      if (head) {
        G = co_const(co_at(F, L0));
        gs = 1;
      } else {
        G = co_comp(F, G);
      }
      px = x;
      pxn = xn;
    }
    // block segmented scan of the tables (every prefix holding a run start is a constant) and max
    // scan of the run starts
    uint64_t val = G;
    int fl = gs, hmax = lh;
    dpp_scan_steps(lane, [&](auto ctl, bool take) {  // DPP moves, no LDS round trips
      constexpr int C = decltype(ctl)::value;
      const uint64_t y = dpp64<C>(val);
      const int yf = (int)dpp32<C>((uint32_t)fl), yh = (int)dpp32<C>((uint32_t)hmax);
      if (take) {
        if (!fl) val = co_comp(val, y);
        fl |= yf;
        hmax = max(hmax, yh);
      }
    });
    if (lane == 63) {
      S.wt[w] = val;
      S.wf[w] = fl;
      S.wh[w] = hmax;
    }
    __syncthreads();
    uint64_t cin = ident;
    int cfl = 0, chm = -1;
    for (uint32_t ww = 0; ww < w; ww++) {
      cin = S.wf[ww] ? S.wt[ww] : co_comp(S.wt[ww], cin);
      cfl |= S.wf[ww];
      chm = max(chm, S.wh[ww]);
    }
    uint64_t ev = __shfl_up(val, 1, 64);
    const int ef = __shfl_up(fl, 1, 64);
    int rs_in = __shfl_up(hmax, 1, 64);
    if (lane == 0) {
      ev = cin;
      rs_in = chm;
    } else {
      if (!ef) ev = co_comp(ev, cin);
      rs_in = max(rs_in, chm);
    }
    const uint32_t Lin = co_at(ev, 0);
    // walk 2: L before each position, the closing ones
    uint32_t L = Lin, lm = 0, lr = 0, lbw = 0, law = 0, emw = 0;
#pragma unroll
    for (int q = 0; q < CO_PER; q++) {
      if (!((vb >> q) & 1u)) break;
      const bool head = (hb >> q) & 1u;
      const uint32_t Lb = head ? (L0q >> (4 * q)) & 15u : L;
      const bool a = (ab >> q) & 1u, b = (bb >> q) & 1u;
      L = co_at(a ? (b ? t11 : t10) : t0, Lb);
      const bool em = cs_emits(C.mode, Lb, M) && b;
      lm += em ? 1u : 0u;
      lr += em ? Lb + 1u : 0u;
      lbw |= Lb << (4 * q);
      law |= L << (4 * q);
      emw |= (em ? 1u : 0u) << q;
    }
    uint32_t tot;
    if constexpr (FR) {  // FULL rows: matches (low 16 bits: <= 2048 a chunk) and refs (high: <= 9 * 2048)
      const uint32_t mr = co_block_scan(lm | (lr << 16), S.sc, tot);
      if (tid == 0) {
        const uint32_t tm = tot & 0xffffu, tr = tot >> 16;
        S.fb[0] = tm ? atomicAdd(O.count, (unsigned long long)tm) : 0ull;
        S.fb[1] = tr ? atomicAdd(O.count + 1, (unsigned long long)tr) : 0ull;
      }
      __syncthreads();
      // e1's chain of each closing position: the key's Lb events before it -- in the chunk from its
      // run start rs, before that from the ring of the key's events in earlier chunks, and before
      // those from the history the push started from (copy rd).  Read before walk 3 moves the ring.
      const int64_t mb = (int64_t)S.fb[0] + (mr & 0xffffu), rbase = (int64_t)S.fb[1] + (mr >> 16);
      int64_t mi = mb, ri = rbase;
      int rs = rs_in;
      int64_t tq[CO_PER];  // e2's ts, loaded for every closing position before any row is stored
#pragma unroll
      for (int q = 0; q < CO_PER; q++) tq[q] = ((emw >> q) & 1u) ? B.ts[xg[q] & 0x7fffffffu] : 0;
#pragma unroll
      for (int q = 0; q < CO_PER; q++) {
        if (!((vb >> q) & 1u)) break;
        const int p = p0 + q;
        if ((hb >> q) & 1u) rs = p;
        if (!((emw >> q) & 1u)) continue;
        const uint32_t Lb = (lbw >> (4 * q)) & 15u;
        const uint32_t g = xg[q] & 0x7fffffffu, lk = xl[q] & 0x7fffu;
        const uint32_t k = (lk << P.bits) | (uint32_t)o;
        if (mi >= O.cap || ri + (int64_t)Lb + 1 > O.refcap) {
          e |= E_OUT;
        } else {
          const int64_t sg = bseq(B, g);
          O.key[mi] = B.partitioned ? (int32_t)k : 0;
          O.ts[mi] = tq[q];  // StateEvent ts = e2's (StreamPostStateProcessor.process :64-83)
          O.type[mi] = 0;
          O.pos[mi] = sg;
          O.ref_off[mi] = ri;
          O.slot_len[mi * MAXS] = (int16_t)Lb;
          O.slot_len[mi * MAXS + 1] = 1;
          const int h = sRh[lk], f = sRf[lk];
          for (uint32_t t = 1; t <= Lb; t++) {
            const int pp = p - (int)t;
            int64_t qs;
            if (pp >= rs) {
              qs = bseq(B, S.cg[pp] & 0x7fffffffu);
            } else {
              const int d = rs - pp - 1;  // 0: the key's latest event before this chunk
              qs = d < f ? bseq(B, sH[(size_t)((h + M - 1 - d) % M) * kpo + lk])
                         : C.hseq[rd][cs_hslot(M - 1 - (d - f), (int64_t)k, M)];
            }
            O.refs[ri + (Lb - t)] = qs;
          }
          O.refs[ri + Lb] = sg;
        }
        mi++;
        ri += Lb + 1;
      }
      emw = 0;  // (no words)
      __syncthreads();
    } else {
      const uint32_t mo = co_block_scan(lm, S.sc, tot);
      pmo = mo;
      if (tid == 0) {  // (+ a lane count that is always 0: keeps the atomic optimizer, which reads the
                       // result back at once, off this one-lane add)
        pres = tot ? atomicAdd(O.count + __builtin_amdgcn_mbcnt_lo(0u, 0u), (unsigned long long)tot) : 0ull;
        ppend = true;
      }
      __syncthreads();
    }
    // walk 3: the words (written during the next chunk), and at each run end the key's state after
    // the run
    pem = emw;
    int rs = rs_in;
    const uint32_t lnext = p0 + CO_PER <= nc ? (S.cl[p0 + CO_PER] & 0x7fffu) : 0xffffu;
#pragma unroll
    for (int q = 0; q < CO_PER; q++) {
      if (!((vb >> q) & 1u)) break;
      const int p = p0 + q;
      if ((hb >> q) & 1u) rs = p;
      const uint32_t Lb = (lbw >> (4 * q)) & 15u;
      const uint32_t gq = xg[q];
      if ((emw >> q) & 1u) pw[q] = (gq & 0x7fffffffu) | (Lb << 28);
      const uint32_t lk = xl[q] & 0x7fffu;
      const uint32_t ln = q + 1 < CO_PER ? (p + 1 < nc ? (xl[q + 1 < CO_PER ? q + 1 : q] & 0x7fffu) : 0xffffu) : lnext;
      if (ln != lk) {  // the key's run ends here
        const int n = p - rs + 1;
        sL[lk] = (uint8_t)((law >> (4 * q)) & 15u);
        sP[lk] = xv[q];
        sN[lk] = (vnull || (gq >> 31) != 0) ? 1 : 0;
        const int h = sRh[lk];
        const int c = min(M, n);
        int slot = (h + n - c) % M;  // the ring slot of the run's (n - c)-th event
        for (int i = n - c; i < n; i++) {
          sH[(size_t)slot * kpo + lk] = S.cg[rs + i] & 0x7fffffffu;
          slot = slot + 1 == M ? 0 : slot + 1;
        }
        sRh[lk] = (uint8_t)slot;
        sRf[lk] = (uint8_t)min(M, (int)sRf[lk] + n);
      }
    }
    __syncthreads();
  }
  if (ppend) {  // the last chunk's words
    if (pres >> 32) e |= E_OUT;
    S.base = (uint32_t)pres;
  }
  __syncthreads();
  flush_words();
  // the keys' state after the push (copy wr): L, value, null, and the last M events' (seq, ts) --
  // the push's from the ring, the older ones from the stored history
  for (int lk = tid; lk < kpo; lk += CO_THREADS) {
    const uint32_t k = ((uint32_t)lk << P.bits) | (uint32_t)o;
    if (k >= nk) continue;
    C.len[wr][k] = sL[lk];
    C.prev[wr][k] = sP[lk];
    C.pnull[wr][k] = sN[lk];
    const int f = sRf[lk], h = sRh[lk];
    for (int s2 = 0; s2 < M; s2++) {
      const int d = M - 1 - s2;  // 0: the key's latest event
      int64_t hs, ht;
      if (d < f) {
        const uint32_t g = sH[(size_t)((h + M - 1 - d) % M) * kpo + lk];
        hs = bseq(B, g);
        ht = B.ts[g];
      } else {
        const int64_t so = cs_hslot(M - 1 - (d - f), k, M);
        hs = C.hseq[rd][so];
        ht = C.hts[rd][so];
      }
      C.hseq[wr][cs_hslot(s2, k, M)] = hs;
      C.hts[wr][cs_hslot(s2, k, M)] = ht;
    }
  }
  if (e) atomicOr(err, e);
}

// ------------------------------------------------------------------ CHAIN32 -> FULL
struct ChRefs {  // refs of a CHAIN32 match: its L e1 events and e2
  __host__ __device__ int64_t operator()(uint32_t w) const { return (int64_t)(w >> 28) + 1; }
};

// one thread per match: e2's sorted position (the push's events sorted by key, batch index
// ascending within a key) by binary search, the chain from the positions before it or, before the
// key's first event in the push, from the history the push started from (copy pre)
template <class R>
__global__ void k_cs_expand(CseqDev C, BatchView B, const int32_t* __restrict__ key, const uint32_t* __restrict__ sk,
                            const R* __restrict__ sr, const uint32_t* __restrict__ ch, int64_t m, int pre, MatchOut O,
                            int* err) {
  int bad = 0;
  const int M = C.M;
  const int64_t n = B.n;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t wd = ch[i];
    const int64_t g = wd & CH32_G;
    const int L = (int)(wd >> 28);
    if (g >= n || L < 1 || L > M) {
      bad |= SWE_BOUND;
      continue;
    }
    const uint32_t k = B.partitioned ? (uint32_t)key[g] : 0u;
    int64_t a = 0, b = n;
    while (a < b) {
      const int64_t mid = (a + b) >> 1;
      if (sk[mid] < k) a = mid + 1;
      else b = mid;
    }
    const int64_t lo = a;
    b = n;
    while (a < b) {
      const int64_t mid = (a + b) >> 1;
      if (sk[mid] == k && (int64_t)(sr[mid].g & 0x7fffffffu) < g) a = mid + 1;
      else b = mid;
    }
    const int64_t j = a;
    if (j >= n || sk[j] != k || (int64_t)(sr[j].g & 0x7fffffffu) != g) {
      bad |= SWE_BOUND;
      continue;
    }
    const int64_t ri = O.ref_off[i];
    if (ri + L + 1 > O.refcap) {
      bad |= E_OUT;
      continue;
    }
    const int64_t sg = bseq(B, g);
    O.key[i] = B.partitioned ? (int32_t)k : 0;
    O.ts[i] = B.ts[g];  // StateEvent ts = e2's (StreamPostStateProcessor.process :64-83)
    O.type[i] = 0;
    O.pos[i] = sg;
    O.slot_len[i * MAXS] = (int16_t)L;
    O.slot_len[i * MAXS + 1] = 1;
    for (int t = 1; t <= L; t++) {
      const int64_t pp = j - t;
      O.refs[ri + (L - t)] = pp >= lo ? bseq(B, sr[pp].g & 0x7fffffffu)
                                      : C.hseq[pre][cs_hslot(M - (int)(lo - pp), (int64_t)k, M)];
    }
    O.refs[ri + L] = sg;
    if (i == m - 1) O.count[1] = (unsigned long long)(ri + L + 1);
  }
  if (bad) atomicOr(err, bad);
}

}  // namespace shp
