// Diagnostic microbenchmark (not product code): where the owner scatter's time goes.
// Standalone: hipcc --offload-arch=gfx950 -O3 -o tools/scatter_micro tools/scatter_micro.hip
//   tools/scatter_micro <events> <owners <= 2048> <keys>
// Variants of one stable multisplit of N 16-byte records into NOWN owner regions (the structure of
// k_sw_scatter / k_co_scatter: rounds of 512 x PER events, per-wave ballot ranks, per-wave LDS
// counters, a cursor pass, scattered stores):
//   0 full            the scatter as built
//   1 no stores       ranks and cursors, the records folded into a checksum instead of stored
//   2 own index       full ranking, records stored at their own index (coalesced)
//   3 copy            loads and coalesced stores only (no ranking, no LDS)
//   4 prefetch early  full, the next round's loads issued as soon as this round's are consumed
//   5 LDS-staged      full ranking; records and their destinations placed in LDS in owner order,
//                     then written out by position (a wave's store covers whole owner runs)
//   6 staged+prefetch 5 with the loads of 4
//   7 window          full ranking, but each super-tile's records land in its own 1 MB window of the
//                     output, grouped by owner inside it (owner segments within the window)
//   8 window+prefetch 7 with the loads of 4
// Variants 5 / 6 run with PER 8 (4096-event rounds) and PER 4 (2048).  The staged variants are
// checked against variant 0 (same record at every position).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int T = 512, W = T / 64, MAXOWN = 2048;
constexpr int64_t STLEN = 65536;

struct __attribute__((aligned(16))) Rec {
  uint64_t kt;
  uint32_t ref, v;
};

__device__ __forceinline__ uint64_t peers_of(uint32_t bin, int bits, bool valid) {
  uint64_t p = __ballot(valid);
  for (int b = 0; b < bits; b++) {
    const bool bit = (bin >> b) & 1u;
    const uint64_t m = __ballot(bit);
    p &= bit ? m : ~m;
  }
  return p;
}

__global__ void k_count(const int32_t* key, int64_t n, int nown, int nst, uint32_t* cnt) {
  __shared__ uint32_t h[MAXOWN];
  for (int b = threadIdx.x; b < nown; b += blockDim.x) h[b] = 0;
  __syncthreads();
  const int64_t lo = (int64_t)blockIdx.x * STLEN, hi = min(n, lo + STLEN);
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) atomicAdd(&h[key[i] & (nown - 1)], 1u);
  __syncthreads();
  for (int b = threadIdx.x; b < nown; b += blockDim.x) cnt[(int64_t)b * nst + blockIdx.x] = h[b];
}

template <int ROUND>
constexpr size_t stage_bytes() {
  return (size_t)ROUND * (sizeof(Rec) + 4);
}

template <int V, int PER>
__global__ __launch_bounds__(T) void k_scatter(const int32_t* __restrict__ key, const int64_t* __restrict__ ts,
                                               const uint32_t* __restrict__ val, int64_t n, int nown, int bits,
                                               int nst, const uint32_t* __restrict__ off, Rec* __restrict__ out,
                                               unsigned long long* sink) {
  constexpr int ROUND = T * PER, SEG = ROUND / W, SUB = SEG / 64;
  constexpr bool STAGED = V == 5 || V == 6, PREFETCH = V == 4 || V == 6 || V == 8, WINDOW = V == 7 || V == 8;
  extern __shared__ uint32_t dyn[];
  __shared__ uint32_t sc[T];
  uint32_t* grun = dyn + W * nown;
  uint32_t* lofs = grun + nown;  // staged: round-local start of each owner
  uint32_t* wcw = dyn + (threadIdx.x >> 6) * nown;
  Rec* stage = reinterpret_cast<Rec*>(dyn + ((W + 2) * nown + 3) / 4 * 4);
  uint32_t* sdst = reinterpret_cast<uint32_t*>(stage + ROUND);
  const int st = blockIdx.x;
  const uint32_t lane = __lane_id(), w = threadIdx.x >> 6;
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  const int64_t lo = (int64_t)st * STLEN, hi = min(n, lo + STLEN);
  const int per = (nown + T - 1) / T;  // owners per thread in the staged offset pass
  if (WINDOW) {  // the tile's owner segments inside its own window [lo, hi): a scan of its counts
    const int b0 = (int)threadIdx.x * per, b1 = min(nown, b0 + per);
    uint32_t tsum = 0;
    for (int b = b0; b < b1; b++) tsum += off[(int64_t)b * nst + st + 1] - off[(int64_t)b * nst + st];
    sc[threadIdx.x] = tsum;
    __syncthreads();
    for (int d = 1; d < T; d <<= 1) {
      const uint32_t y = threadIdx.x >= (unsigned)d ? sc[threadIdx.x - d] : 0u;
      __syncthreads();
      sc[threadIdx.x] += y;
      __syncthreads();
    }
    uint32_t g = (uint32_t)lo + sc[threadIdx.x] - tsum;
    for (int b = b0; b < b1; b++) {
      grun[b] = g;
      g += off[(int64_t)b * nst + st + 1] - off[(int64_t)b * nst + st];
    }
    __syncthreads();
  } else {
    for (int b = threadIdx.x; b < nown; b += T) grun[b] = off[(int64_t)b * nst + st];
  }
  unsigned long long acc = 0;
  int32_t pk[SUB];
  int64_t pt[SUB];
  uint32_t pv[SUB];
  auto load = [&](int64_t r0) {
#pragma unroll
    for (int s = 0; s < SUB; s++) {
      const int64_t i = r0 + (int64_t)w * SEG + s * 64 + lane;
      pk[s] = i < hi ? key[i] : -1;
      pt[s] = i < hi ? ts[i] : 0;
      pv[s] = i < hi ? val[i] : 0;
    }
  };
  load(lo);
  for (int64_t r0 = lo; r0 < hi; r0 += ROUND) {
    if (r0 != lo && !PREFETCH) load(r0);
    Rec rec[SUB];
    int32_t kk[SUB];
#pragma unroll
    for (int s = 0; s < SUB; s++) {
      kk[s] = pk[s];
      rec[s].kt = (uint64_t)pt[s] ^ ((uint64_t)(pk[s] >> bits) << 56);
      rec[s].ref = (uint32_t)(r0 + (int64_t)w * SEG + s * 64 + lane);
      rec[s].v = pv[s];
    }
    if (V == 3) {
#pragma unroll
      for (int s = 0; s < SUB; s++)
        if (kk[s] >= 0) out[rec[s].ref] = rec[s];
      continue;
    }
    if (PREFETCH && r0 + ROUND < hi) load(r0 + ROUND);
    for (int b = lane; b < nown; b += 64) wcw[b] = 0;
    __syncthreads();
    uint32_t own[SUB], rk[SUB], pc[SUB], ld[SUB];
#pragma unroll
    for (int s = 0; s < SUB; s++) {
      const bool valid = kk[s] >= 0;
      const uint32_t o = valid ? ((uint32_t)kk[s] & (uint32_t)(nown - 1)) : 0u;
      const uint64_t peers = peers_of(o, bits, valid);
      rk[s] = (uint32_t)__popcll(peers & lt);
      own[s] = valid ? o : 0xffffffffu;
      pc[s] = (valid && (peers & lt) == 0) ? (uint32_t)__popcll(peers) : 0u;
      ld[s] = peers ? (uint32_t)__ffsll((unsigned long long)peers) - 1u : 0u;
    }
    uint32_t old[SUB];
#pragma unroll
    for (int s = 0; s < SUB; s++) old[s] = pc[s] ? atomicAdd(&wcw[own[s]], pc[s]) : 0u;
#pragma unroll
    for (int s = 0; s < SUB; s++) rk[s] += __shfl(old[s], (int)ld[s], 64);
    __syncthreads();
    if (STAGED) {
      // round-local owner offsets: thread t takes owners [t * per, t * per + per)
      const int b0 = (int)threadIdx.x * per, b1 = min(nown, b0 + per);
      uint32_t tsum = 0;
      for (int b = b0; b < b1; b++)
        for (int ww = 0; ww < W; ww++) tsum += dyn[ww * nown + b];
      sc[threadIdx.x] = tsum;
      __syncthreads();
      for (int d = 1; d < T; d <<= 1) {
        const uint32_t y = threadIdx.x >= (unsigned)d ? sc[threadIdx.x - d] : 0u;
        __syncthreads();
        sc[threadIdx.x] += y;
        __syncthreads();
      }
      uint32_t g = sc[threadIdx.x] - tsum;
      for (int b = b0; b < b1; b++) {
        lofs[b] = g;
        for (int ww = 0; ww < W; ww++) {
          const uint32_t c = dyn[ww * nown + b];
          dyn[ww * nown + b] = g;
          g += c;
        }
      }
      __syncthreads();
#pragma unroll
      for (int s = 0; s < SUB; s++)
        if (own[s] != 0xffffffffu) {
          const uint32_t p = wcw[own[s]] + rk[s];  // round-local, in owner order
          stage[p] = rec[s];
          sdst[p] = grun[own[s]] + (p - lofs[own[s]]);
        }
      __syncthreads();
      const uint32_t nr = (uint32_t)min((int64_t)ROUND, hi - r0);
      for (uint32_t p = threadIdx.x; p < nr; p += T) out[sdst[p]] = stage[p];
      // the owners' running offsets past this round
      for (int b = b0; b < b1; b++) grun[b] += (b + 1 < nown ? lofs[b + 1] : nr) - lofs[b];
      __syncthreads();
      continue;
    }
    for (int b = threadIdx.x; b < nown; b += T) {
      uint32_t g = grun[b];
#pragma unroll
      for (int ww = 0; ww < W; ww++) {
        const uint32_t c = dyn[ww * nown + b];
        dyn[ww * nown + b] = g;
        g += c;
      }
      grun[b] = g;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < SUB; s++) {
      if (own[s] == 0xffffffffu) continue;
      if (V == 1) acc += rec[s].kt + wcw[own[s]] + rk[s];
      else if (V == 2) out[rec[s].ref] = rec[s];
      else out[wcw[own[s]] + rk[s]] = rec[s];
    }
    __syncthreads();
  }
  if (V == 1 && acc == 0x1234567ull) *sink = acc;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 100000000;
  const int nown = argc > 2 ? atoi(argv[2]) : 512;
  const int keys = argc > 3 ? atoi(argv[3]) : 10000;
  if (nown < 1 || nown > MAXOWN || (nown & (nown - 1)) != 0 || keys < nown || n < 1 || n > (1ll << 31)) {
    fprintf(stderr, "owners: a power of two <= %d, keys >= owners, 1 <= events < 2^31\n", MAXOWN);
    return 2;
  }
  int bits = 0;
  while ((1 << bits) < nown) bits++;
  std::vector<int32_t> hk(n);
  std::vector<int64_t> ht(n);
  std::vector<uint32_t> hv(n);
  uint64_t x = 88172645463325252ull;
  for (int64_t i = 0; i < n; i++) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    hk[i] = (int32_t)(x % (uint64_t)keys);
    ht[i] = 1000000 + i / 10;
    hv[i] = (uint32_t)(x >> 40);
  }
  int32_t* key;
  int64_t* ts;
  uint32_t *val, *cnt, *off;
  Rec* out;
  unsigned long long* sink;
  const int nst = (int)((n + STLEN - 1) / STLEN);
  CK(hipMalloc(&key, n * 4));
  CK(hipMalloc(&ts, n * 8));
  CK(hipMalloc(&val, n * 4));
  CK(hipMalloc(&out, n * sizeof(Rec)));
  CK(hipMalloc(&cnt, ((size_t)nown * nst + 1) * 4));
  CK(hipMalloc(&off, ((size_t)nown * nst + 1) * 4));
  CK(hipMalloc(&sink, 8));
  CK(hipMemcpy(key, hk.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(ts, ht.data(), n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(val, hv.data(), n * 4, hipMemcpyHostToDevice));
  k_count<<<nst, 256>>>(key, n, nown, nst, cnt);
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> hc((size_t)nown * nst), ho((size_t)nown * nst + 1);
  CK(hipMemcpy(hc.data(), cnt, hc.size() * 4, hipMemcpyDeviceToHost));
  uint32_t run = 0;
  for (size_t i = 0; i < hc.size(); i++) {
    ho[i] = run;
    run += hc[i];
  }
  ho[hc.size()] = run;
  if ((int64_t)run != n) {
    fprintf(stderr, "count mismatch\n");
    return 1;
  }
  CK(hipMemcpy(off, ho.data(), ho.size() * 4, hipMemcpyHostToDevice));
  const size_t lds_base = ((size_t)(W + 2) * nown + 3) / 4 * 4 * 4;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct Var {
    const char* name;
    const void* fn;
    size_t lds;
  };
#define KV(V, P) (const void*)k_scatter<V, P>
  const Var vars[] = {{"full", KV(0, 8), lds_base},
                      {"no stores", KV(1, 8), lds_base},
                      {"own index", KV(2, 8), lds_base},
                      {"copy", KV(3, 8), lds_base},
                      {"prefetch early", KV(4, 8), lds_base},
                      {"staged 4096", KV(5, 8), lds_base + stage_bytes<4096>()},
                      {"staged 2048", KV(5, 4), lds_base + stage_bytes<2048>()},
                      {"staged+prefetch 4096", KV(6, 8), lds_base + stage_bytes<4096>()},
                      {"staged+prefetch 2048", KV(6, 4), lds_base + stage_bytes<2048>()},
                      {"window", KV(7, 8), lds_base},
                      {"window+prefetch", KV(8, 8), lds_base}};
  auto launch = [&](const Var& v) {
    void* args[] = {&key, &ts, &val, (void*)&n, (void*)&nown, &bits, (void*)&nst, &off, &out, &sink};
    CK(hipLaunchKernel(v.fn, dim3(nst), dim3(T), args, v.lds, 0));
  };
  for (const Var& v : vars)
    if (v.lds > 65536) CK(hipFuncSetAttribute(v.fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)v.lds));
  for (int rep = 0; rep < 2; rep++) {
    for (const Var& v : vars) {
      launch(v);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      for (int it = 0; it < 5; it++) launch(v);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("rep %d %-22s lds %6zu B  %.3f ms\n", rep, v.name, v.lds, ms / 5);
      fflush(stdout);
    }
  }
  std::vector<Rec> a(n), b(n);
  CK(hipMemset(out, 0, n * sizeof(Rec)));
  launch(vars[0]);
  CK(hipMemcpy(a.data(), out, n * sizeof(Rec), hipMemcpyDeviceToHost));
  for (int i : {4, 5, 6, 7, 8}) {
    CK(hipMemset(out, 0, n * sizeof(Rec)));
    launch(vars[i]);
    CK(hipMemcpy(b.data(), out, n * sizeof(Rec), hipMemcpyDeviceToHost));
    int64_t bad = 0;
    for (int64_t j = 0; j < n; j++) bad += a[j].ref != b[j].ref;
    printf("%-22s vs full: %lld records differ\n", vars[i].name, (long long)bad);
  }
  for (int i : {9, 10}) {  // window layout: a permutation, owner-grouped and stable inside each tile's window
    CK(hipMemset(out, 0, n * sizeof(Rec)));
    launch(vars[i]);
    CK(hipMemcpy(b.data(), out, n * sizeof(Rec), hipMemcpyDeviceToHost));
    std::vector<uint8_t> seen(n, 0);
    int64_t bad = 0;
    for (int64_t j = 0; j < n; j++) {
      const uint32_t r = b[j].ref;
      if (r >= (uint64_t)n || seen[r]) {
        bad++;
        continue;
      }
      seen[r] = 1;
      if (r / STLEN != (uint64_t)j / STLEN) bad++;  // stays in its tile's window
      if (j % STLEN != 0) {
        const uint32_t p = b[j - 1].ref;
        const uint32_t op = (uint32_t)hk[p] & (nown - 1), oc = (uint32_t)hk[r] & (nown - 1);
        if (op > oc || (op == oc && p >= r)) bad++;
      }
    }
    printf("%-22s layout check: %lld bad\n", vars[i].name, (long long)bad);
  }
  return 0;
}
