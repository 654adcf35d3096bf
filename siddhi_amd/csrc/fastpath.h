// siddhi-hip: HIP kernels of the specialised 2-state path (bodies in fast_core.h).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <rocprim/rocprim.hpp>
#include <string>
#include <utility>
#include <vector>

#include "fast_core.h"

namespace shp {

// Per-kernel device time of the last push, from HIP events on the engine stream
// (enabled by shp_config.profile_kernels; bench.py reads it for the roofline line).
struct KTimer {
  bool enabled = false;
  static constexpr int N = 32;
  hipEvent_t ev[N + 1] = {};
  const char* names[N] = {};
  int used = 0;
  const char* cur = nullptr;
  std::vector<std::pair<std::string, double>> last;
  void begin_push() { used = 0; cur = nullptr; }
  int debug = -1;  // SHP_DEBUG_SYNC=1: synchronise after every kernel and name the failing one
  void mark(const char* next, hipStream_t s) {
    if (debug < 0) debug = getenv("SHP_DEBUG_SYNC") ? 1 : 0;
    if (debug) {
      hipError_t e = hipStreamSynchronize(s);
      if (e == hipSuccess) e = hipGetLastError();
      if (e != hipSuccess) fprintf(stderr, "SHP_DEBUG_SYNC: error after kernel '%s': %s\n", cur ? cur : "?",
                                   hipGetErrorString(e));
      else if (cur) fprintf(stderr, "SHP_DEBUG_SYNC: ok after '%s'\n", cur);
      if (!enabled) cur = next;
    }
    if (!enabled) return;
    if (!ev[0]) for (int i = 0; i <= N; i++) (void)hipEventCreate(&ev[i]);
    if (used >= N) return;
    (void)hipEventRecord(ev[used], s);
    if (cur) names[used - 1] = cur;
    cur = next;
    used++;
    if (!next) cur = nullptr;
  }
  void collect() {
    last.clear();
    if (!enabled) return;
    for (int i = 0; i + 1 < used; i++) {
      if (!names[i]) continue;
      float ms = 0;
      (void)hipEventElapsedTime(&ms, ev[i], ev[i + 1]);
      last.emplace_back(names[i], ms);
    }
    for (int i = 0; i < N; i++) names[i] = nullptr;
  }
  double get(const std::string& n) const {
    double t = 0;
    for (auto& p : last)
      if (p.first == n) t += p.second;
    return t;
  }
  void release() {
    for (int i = 0; i <= N; i++)
      if (ev[i]) (void)hipEventDestroy(ev[i]);
  }
};

static __global__ void k_fast_gather(const DevProg* __restrict__ Pp, BatchView B, FastDev F, const uint32_t* __restrict__ perm,
                              const uint32_t* __restrict__ skey, int64_t n, int* err) {
  int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; p < n; p += (int64_t)gridDim.x * blockDim.x) fast_gather_item(*Pp, B, F, perm, skey, p, err);
}

static __global__ void k_fast_search(const DevProg* __restrict__ Pp, BatchView B, FastDev F, const uint32_t* __restrict__ perm,
                              const uint32_t* __restrict__ skey, const uint32_t* __restrict__ kbeg,
                              const uint32_t* __restrict__ kcnt, int64_t n, int fstream) {
  int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  (void)Pp;
  for (int64_t i = p; i < n; i += stride) fast_search_item(B, F, perm, skey, kbeg, kcnt, i, fstream);
  for (int64_t c = p; c < (int64_t)F.nk * FCC; c += stride) fast_search_carry_item(B, F, perm, kbeg, kcnt, c, fstream);
}

static __global__ void k_fast_seq(FastDev F, BatchView B, const uint32_t* __restrict__ perm, const uint32_t* __restrict__ kbeg,
                           const uint32_t* __restrict__ kcnt, int fstream) {
  int32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < F.nk) fast_seq_item(F, B, perm, kbeg, kcnt, k, fstream);
}

static __global__ void k_fast_emit(FastDev F, BatchView B, MatchOut O, const uint32_t* __restrict__ perm,
                            const uint32_t* __restrict__ skey, const uint32_t* __restrict__ kbeg, int64_t n,
                            const unsigned long long* total, int* err) {
  int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q == 0) {
    O.count[0] = *total;
    O.count[1] = 2 * *total;
    if ((int64_t)*total > O.cap || (int64_t)(2 * *total) > O.refcap) atomicOr(err, E_OUT);
  }
  for (; q < n; q += (int64_t)gridDim.x * blockDim.x) fast_emit_item(F, B, O, perm, skey, kbeg, q);
}

static __global__ void k_fast_carry(FastDev F, BatchView B, const uint32_t* __restrict__ perm,
                             const uint32_t* __restrict__ kbeg, const uint32_t* __restrict__ kcnt, int* err) {
  int32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < F.nk) fast_carry_item(F, B, perm, kbeg, kcnt, k, err);
}

static __global__ void k_fast_init(FastDev F) {
  int32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= F.nk) return;
  F.c_n[k] = 0;
  F.last_ts[k] = INT64_MIN;
  F.slow[k] = 0;
  F.last_cand[k] = 0;
  F.first_open[k] = 0xffffffffu;
}

static __global__ void k_fast_total(const uint32_t* nclose, const uint32_t* moff, int64_t n, unsigned long long* total) {
  *total = n > 0 ? (unsigned long long)moff[n - 1] + nclose[n - 1] : 0ull;
}

struct FastState {
  FastDev F{};
  int stream_ = 0;
  unsigned long long* d_total = nullptr;

  void release() {
    void* ps[] = {F.c_seq, F.c_ts, F.c_val, F.c_null, F.c_n, F.c_match, F.last_ts, F.slow, F.last_cand, F.s_ts,
                  F.s_val, F.s_null, F.match, F.nclose, F.moff, F.first_open, d_total};
    for (void* p : ps)
      if (p) (void)hipFree(p);
    F = FastDev{};
    d_total = nullptr;
  }

  size_t scratch_bytes(int64_t cap, int32_t, hipStream_t s) {
    size_t b = 0;
    (void)rocprim::exclusive_scan(nullptr, b, (uint32_t*)nullptr, (uint32_t*)nullptr, 0u, (size_t)cap,
                                  rocprim::plus<uint32_t>(), s);
    return b;
  }

  // debug-only (SHP_DEBUG_VALIDATE): check the partition step's outputs on the host before
  // the search kernel trusts them as indices
  bool validate(const DevProg& P, int64_t n, int32_t nk, const uint32_t* perm, const uint32_t* skey,
                const uint32_t* kbeg, const uint32_t* kcnt, const DevProg* dprog, size_t tmp_bytes, hipStream_t s) {
    (void)hipStreamSynchronize(s);
    std::vector<uint32_t> hp(n), hk(n), hb(nk + 1), hc(nk + 1);
    DevProg dp;
    (void)hipMemcpy(hp.data(), perm, n * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hk.data(), skey, n * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hb.data(), kbeg, (nk + 1) * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hc.data(), kcnt, (nk + 1) * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&dp, dprog, sizeof(DevProg), hipMemcpyDeviceToHost);
    bool ok = true;
    if (memcmp(&dp, &P, sizeof(DevProg)) != 0) { fprintf(stderr, "VALIDATE: device DevProg differs\n"); ok = false; }
    std::vector<char> seen(n, 0);
    for (int64_t i = 0; i < n; i++) {
      if (hp[i] >= (uint32_t)n || seen[hp[i]]) { fprintf(stderr, "VALIDATE: perm[%ld]=%u bad\n", (long)i, hp[i]); ok = false; break; }
      seen[hp[i]] = 1;
      if (i && hk[i] < hk[i - 1]) { fprintf(stderr, "VALIDATE: skey not sorted at %ld\n", (long)i); ok = false; break; }
    }
    uint64_t tot = 0;
    for (int k = 0; k < nk; k++) {
      if (hb[k] != tot) { fprintf(stderr, "VALIDATE: kbeg[%d]=%u expected %lu\n", k, hb[k], (unsigned long)tot); ok = false; break; }
      tot += hc[k];
    }
    if (tot > (uint64_t)n) { fprintf(stderr, "VALIDATE: kcnt sum %lu > n %ld\n", (unsigned long)tot, (long)n); ok = false; }
    size_t need = 0;
    (void)rocprim::radix_sort_pairs(nullptr, need, (uint32_t*)nullptr, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                    (uint32_t*)nullptr, (size_t)n, 0, 16, s);
    fprintf(stderr, "VALIDATE: n=%ld nk=%d tmp_bytes=%zu sort_need(n,16b)=%zu ok=%d\n", (long)n, nk, tmp_bytes, need, (int)ok);
    return ok;
  }

  template <class T>
  static void al(T*& p, int64_t n) {
    if (hipMalloc((void**)&p, std::max<int64_t>(n, 1) * sizeof(T)) != hipSuccess)
      throw std::runtime_error("hipMalloc failed (fast path)");
  }

  void create(const DevProg& P, const FastShape& fsh, int32_t nk, int64_t cap, int64_t, hipStream_t s) {
    F.within = fsh.within;
    F.f1 = fsh.f1;
    F.f2 = fsh.f2;
    F.nk = nk;
    F.nv = P.ncol;
    stream_ = fsh.stream;
    F.fstream = fsh.stream;
    al(F.c_seq, (int64_t)nk * FCC);
    al(F.c_ts, (int64_t)nk * FCC);
    al(F.c_val, (int64_t)nk * FCC * 2);
    al(F.c_null, (int64_t)nk * FCC * 2);
    al(F.c_n, nk);
    al(F.c_match, (int64_t)nk * FCC);
    al(F.last_ts, nk);
    al(F.slow, nk);
    al(F.last_cand, nk);
    al(F.s_ts, cap);
    al(F.s_val, cap * 2);
    al(F.s_null, cap * 2);
    al(F.match, cap);
    al(F.nclose, cap);
    al(F.moff, cap + 1);
    al(F.first_open, nk);
    al(d_total, 1);
    k_fast_init<<<(nk + 255) / 256, 256, 0, s>>>(F);
  }

  // skey: sorted keys from the partition step are not kept by the engine; recover from perm
  void run(const DevProg& P, const BatchView& B, const MatchOut& O, const uint32_t* perm, const uint32_t* kbeg,
           const uint32_t* kcnt, int32_t nk, void* tmp, size_t tmp_bytes, int* err, hipStream_t s,
           const uint32_t* skey, const DevProg* dprog, KTimer& kt) {
    int64_t n = B.n;
    int gb = (int)std::min<int64_t>((n + 255) / 256, 8192);
    if (gb < 1) gb = 1;
    kt.mark("fast_gather", s);
    k_fast_gather<<<gb, 256, 0, s>>>(dprog, B, F, perm, skey, n, err);
    int gs = (int)std::min<int64_t>((std::max<int64_t>(n, (int64_t)nk * FCC) + 255) / 256, 8192);
    if (getenv("SHP_DEBUG_VALIDATE")) {  // debug: validate inputs, never launch the search
      validate(P, n, nk, perm, skey, kbeg, kcnt, dprog, tmp_bytes, s);
      int bad = 1 << 22;
      (void)hipMemcpyAsync(err, &bad, sizeof(int), hipMemcpyHostToDevice, s);
      (void)hipStreamSynchronize(s);
      return;
    }
    kt.mark("fast_search", s);
    k_fast_search<<<gs, 256, 0, s>>>(dprog, B, F, perm, skey, kbeg, kcnt, n, stream_);
    kt.mark("fast_seq", s);
    k_fast_seq<<<(nk + 255) / 256, 256, 0, s>>>(F, B, perm, kbeg, kcnt, stream_);
    size_t tb = tmp_bytes;
    kt.mark("nclose_scan", s);
    (void)rocprim::exclusive_scan(tmp, tb, F.nclose, F.moff, 0u, (size_t)n, rocprim::plus<uint32_t>(), s);
    kt.mark("fast_total", s);
    k_fast_total<<<1, 1, 0, s>>>(F.nclose, F.moff, n, d_total);
    kt.mark("fast_emit", s);
    k_fast_emit<<<gb, 256, 0, s>>>(F, B, O, perm, skey, kbeg, n, d_total, err);
    kt.mark("fast_carry", s);
    k_fast_carry<<<(nk + 255) / 256, 256, 0, s>>>(F, B, perm, kbeg, kcnt, err);
    kt.mark(nullptr, s);
  }
};

}  // namespace shp
