// siddhi-hip: specialised kernels for `every e1=S[f1] -> e2=S[f2] within W`.
//
// For this shape the processor chain (derived from
// StreamPreStateProcessor.processAndReturn/expireEvents :326-403 and the
// reversed same-stream order of PatternMultiProcessStreamReceiver :32-39)
// reduces, per key with non-decreasing timestamps, to:
//   every event i with f1(i) opens candidate i; candidate i closes at the first
//   later event j of the key with f2(i, j) and ts_j - ts_i <= W, else it expires;
//   matches are emitted ordered by j, then i.
// Candidates are independent, so the kernels are data-parallel over events:
//   k_fast_gather  key-sorted SoA (ts, predicate columns) + per-key ts monotonicity check
//   k_fast_search  one thread per candidate: forward scan to its closing event
//   k_fast_emit    one thread per closing event: backward scan emits (j, i) in order
//   k_fast_carry   open candidates at the batch end -> per-key carry (next batch)
// The general lane kernel (nfa_lane.h) remains the reference for this shape.
#pragma once
#include <hip/hip_runtime.h>

#include <rocprim/rocprim.hpp>
#include <string>
#include <utility>
#include <vector>

#include "nfa_lane.h"
#include "prog.h"

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
  void mark(const char* next, hipStream_t s) {
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

constexpr int FCC = 64;  // carried open candidates per key

struct FastDev {
  int64_t within;
  int32_t nk;            // keys
  int32_t nv;            // predicate columns (<= 2)
  // carry (per key)
  int64_t* c_seq;        // nk * FCC
  int64_t* c_ts;
  int64_t* c_val;        // nk * FCC * 2  (value bits)
  uint8_t* c_null;       // nk * FCC * 2
  int32_t* c_n;          // nk
  int32_t* c_match;      // nk * FCC : matched sorted position, -1 dead, -2 open
  int64_t* last_ts;      // nk, INT64_MIN when unseen
  // batch scratch
  int64_t* s_ts;         // n (key-sorted)
  int64_t* s_val;        // n * 2
  uint8_t* s_null;       // n * 2
  int32_t* match;        // n : sorted position of closing event, -1 none/dead, -2 open, -3 not a candidate
  uint32_t* nclose;      // n
  uint32_t* moff;        // n (exclusive scan of nclose)
  uint32_t* first_open;  // nk : lowest sorted position of a still-open batch candidate
};

// values of one event for the predicate VM: slot 0 = candidate, slot 1 = closing event
struct FastRes {
  const DevProg* P;
  int64_t v[2][2];
  uint8_t nul[2][2];
  bool has[2];
  SHP_HD Val value(int state, int index, int col) const {
    Val r{T_NULL, 0};
    if (state < 0 || state > 1 || !has[state]) return r;
    if (!(index == 0 || index == -1)) return r;  // single-event slots
    int pos = P->colPos[col];
    if (nul[state][pos]) return r;
    r.tag = P->colTag[col];
    r.bits = v[state][pos];
    return r;
  }
  SHP_HD bool isnull_state(int state, int index) const {
    return !(state >= 0 && state <= 1 && has[state] && (index == 0 || index == -1));
  }
};

__device__ inline void fast_load(const DevProg& P, const BatchView& B, int64_t g, int64_t* v, uint8_t* nul) {
  int st = B.stream[g];
  for (int j = 0; j < 2; j++) {
    v[j] = 0;
    nul[j] = 1;
  }
  if (st < 0) return;
  for (int j = 0; j < P.streamNcol[st]; j++) {
    Val x = load_col(B, P, P.streamCols[st][j], g);
    v[j] = x.bits;
    nul[j] = x.tag == T_NULL;
  }
}

__global__ void k_fast_gather(const DevProg* __restrict__ Pp, BatchView B, FastDev F, const uint32_t* __restrict__ perm,
                              const uint32_t* __restrict__ skey, int64_t n, int fstream, int* err) {
  const DevProg& P = *Pp;
  int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; p < n; p += (int64_t)gridDim.x * blockDim.x) {
    uint32_t g = perm[p];
    int64_t t = B.ts[g];
    F.s_ts[p] = t;
    int64_t v[2];
    uint8_t nul[2];
    fast_load(P, B, g, v, nul);
    F.s_val[2 * p] = v[0];
    F.s_val[2 * p + 1] = v[1];
    F.s_null[2 * p] = nul[0];
    F.s_null[2 * p + 1] = nul[1];
    F.nclose[p] = 0;
    uint32_t k = skey[p];
    if (k < (uint32_t)F.nk) {
      int64_t prev = (p > 0 && skey[p - 1] == k) ? B.ts[perm[p - 1]] : F.last_ts[k];
      if (t < prev) atomicOr(err, 1 << 21);
    }
  }
}

// forward scan from `from` (sorted position) to `end` for the closing event of a candidate
__device__ inline int32_t fast_scan(const DevProg& P, const FastDev& F, FastRes& r, int64_t ti, int64_t from,
                                    int64_t end, int fstream, const BatchView& B, const uint32_t* perm) {
  const int pc2 = P.pre[1].filterPc;
  for (int64_t q = from; q < end; q++) {
    uint32_t g = perm[q];
    if (B.stream[g] != fstream) continue;  // other partition streams never reach this query
    int64_t tq = F.s_ts[q];
    if (tq - ti > F.within) return -1;  // expired (expireEvents before processAndReturn)
    r.has[1] = true;
    r.v[1][0] = F.s_val[2 * q];
    r.v[1][1] = F.s_val[2 * q + 1];
    r.nul[1][0] = F.s_null[2 * q];
    r.nul[1][1] = F.s_null[2 * q + 1];
    if (pc2 < 0 || run_filter(P, pc2, r)) return (int32_t)q;
  }
  return -2;  // still open at the batch end
}

__global__ void k_fast_search(const DevProg* __restrict__ Pp, BatchView B, FastDev F, const uint32_t* __restrict__ perm,
                              const uint32_t* __restrict__ skey, const uint32_t* __restrict__ kbeg,
                              const uint32_t* __restrict__ kcnt, int64_t n, int fstream) {
  const DevProg& P = *Pp;
  int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  // batch candidates
  for (int64_t i = p; i < n; i += stride) {
    uint32_t k = skey[i];
    if (k >= (uint32_t)F.nk || B.stream[perm[i]] != fstream) {
      F.match[i] = -3;
      continue;
    }
    FastRes r;
    r.P = &P;
    r.has[0] = true;
    r.has[1] = false;
    r.v[0][0] = F.s_val[2 * i];
    r.v[0][1] = F.s_val[2 * i + 1];
    r.nul[0][0] = F.s_null[2 * i];
    r.nul[0][1] = F.s_null[2 * i + 1];
    int pc1 = P.pre[0].filterPc;
    if (pc1 >= 0 && !run_filter(P, pc1, r)) {
      F.match[i] = -3;
      continue;
    }
    int64_t end = (int64_t)kbeg[k] + kcnt[k];
    int32_t q = fast_scan(P, F, r, F.s_ts[i], i + 1, end, fstream, B, perm);
    F.match[i] = q;
    if (q >= 0) atomicAdd(&F.nclose[q], 1u);
    if (q == -2) atomicMin(&F.first_open[k], (uint32_t)i);
  }
  // carried candidates
  for (int64_t c = p; c < (int64_t)F.nk * FCC; c += stride) {
    int32_t k = (int32_t)(c / FCC);
    int32_t j = (int32_t)(c % FCC);
    if (j >= F.c_n[k]) continue;
    if (kcnt[k] == 0) {
      F.c_match[c] = -2;
      continue;
    }
    FastRes r;
    r.P = &P;
    r.has[0] = true;
    r.has[1] = false;
    r.v[0][0] = F.c_val[2 * c];
    r.v[0][1] = F.c_val[2 * c + 1];
    r.nul[0][0] = F.c_null[2 * c];
    r.nul[0][1] = F.c_null[2 * c + 1];
    int64_t b = kbeg[k];
    int32_t q = fast_scan(P, F, r, F.c_ts[c], b, b + kcnt[k], fstream, B, perm);
    F.c_match[c] = q;
    if (q >= 0) atomicAdd(&F.nclose[q], 1u);
  }
}

__global__ void k_fast_emit(FastDev F, BatchView B, MatchOut O, const uint32_t* __restrict__ perm,
                            const uint32_t* __restrict__ skey, const uint32_t* __restrict__ kbeg, int64_t n,
                            const unsigned long long* total, int* err) {
  int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q == 0) {
    O.count[0] = *total;
    O.count[1] = 2 * *total;
    if ((int64_t)*total > O.cap || (int64_t)(2 * *total) > O.refcap) atomicOr(err, E_OUT);
  }
  for (; q < n; q += (int64_t)gridDim.x * blockDim.x) {
    uint32_t cnt = F.nclose[q];
    if (!cnt) continue;
    uint32_t k = skey[q];
    int64_t base = F.moff[q];
    if (base + cnt > O.cap) continue;
    int64_t tq = F.s_ts[q];
    int64_t seqq = B.seq0 + perm[q];
    uint32_t w = 0;
    auto put = [&](int64_t seqi, uint32_t slot) {
      int64_t m = base + slot;
      O.key[m] = (int32_t)k;
      O.ts[m] = tq;
      O.type[m] = 0;
      O.pos[m] = seqq;
      O.ref_off[m] = 2 * m;
      O.slot_len[m * MAXS] = 1;
      O.slot_len[m * MAXS + 1] = 1;
      O.refs[2 * m] = seqi;
      O.refs[2 * m + 1] = seqq;
    };
    // carried (older) candidates first, in carry order
    int cn = F.c_n[k];
    for (int j = 0; j < cn && w < cnt; j++)
      if (F.c_match[(int64_t)k * FCC + j] == (int32_t)q) put(F.c_seq[(int64_t)k * FCC + j], w++);
    // batch candidates closed by q lie in (kbeg, q) within W of ts_q: collect backwards,
    // place forwards (ascending i)
    uint32_t nb = cnt - w;
    uint32_t placed = 0;
    for (int64_t i = q - 1; i >= (int64_t)kbeg[k] && placed < nb; i--) {
      if (tq - F.s_ts[i] > F.within) break;
      if (F.match[i] == (int32_t)q) {
        put(B.seq0 + perm[i], w + nb - 1 - placed);
        placed++;
      }
    }
  }
}

__global__ void k_fast_carry(FastDev F, BatchView B, const uint32_t* __restrict__ perm,
                             const uint32_t* __restrict__ kbeg, const uint32_t* __restrict__ kcnt, int* err) {
  int32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= F.nk) return;
  uint32_t cnt = kcnt[k];
  if (cnt == 0) return;
  int64_t b = kbeg[k], e = b + cnt;
  F.last_ts[k] = F.s_ts[e - 1];
  int64_t first_open = F.first_open[k] == 0xffffffffu ? e : (int64_t)F.first_open[k];
  F.first_open[k] = 0xffffffffu;
  int64_t base = (int64_t)k * FCC;
  int w = 0;
  int cn = F.c_n[k];
  for (int j = 0; j < cn; j++) {
    int64_t c = base + j;
    if (F.c_match[c] == -2) {
      if (w != j) {
        F.c_seq[base + w] = F.c_seq[c];
        F.c_ts[base + w] = F.c_ts[c];
        F.c_val[2 * (base + w)] = F.c_val[2 * c];
        F.c_val[2 * (base + w) + 1] = F.c_val[2 * c + 1];
        F.c_null[2 * (base + w)] = F.c_null[2 * c];
        F.c_null[2 * (base + w) + 1] = F.c_null[2 * c + 1];
      }
      w++;
    }
  }
  for (int64_t i = first_open; i < e; i++) {
    if (F.match[i] != -2) continue;
    if (w >= FCC) {
      atomicOr(err, E_LIST);
      break;
    }
    int64_t c = base + w;
    F.c_seq[c] = B.seq0 + perm[i];
    F.c_ts[c] = F.s_ts[i];
    F.c_val[2 * c] = F.s_val[2 * i];
    F.c_val[2 * c + 1] = F.s_val[2 * i + 1];
    F.c_null[2 * c] = F.s_null[2 * i];
    F.c_null[2 * c + 1] = F.s_null[2 * i + 1];
    w++;
  }
  F.c_n[k] = w;
}

__global__ void k_fast_init(FastDev F) {
  int32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= F.nk) return;
  F.c_n[k] = 0;
  F.last_ts[k] = INT64_MIN;
  F.first_open[k] = 0xffffffffu;
}

__global__ void k_fast_total(const uint32_t* nclose, const uint32_t* moff, int64_t n, unsigned long long* total) {
  *total = n > 0 ? (unsigned long long)moff[n - 1] + nclose[n - 1] : 0ull;
}

struct FastState {
  FastDev F{};
  int stream_ = 0;
  unsigned long long* d_total = nullptr;

  void release() {
    void* ps[] = {F.c_seq, F.c_ts, F.c_val, F.c_null, F.c_n, F.c_match, F.last_ts, F.s_ts,
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

  template <class T>
  static void al(T*& p, int64_t n) {
    if (hipMalloc((void**)&p, std::max<int64_t>(n, 1) * sizeof(T)) != hipSuccess)
      throw std::runtime_error("hipMalloc failed (fast path)");
  }

  void create(const DevProg& P, const FastShape& fsh, int32_t nk, int64_t cap, int64_t, hipStream_t s) {
    F.within = fsh.within;
    F.nk = nk;
    F.nv = P.ncol;
    stream_ = fsh.stream;
    al(F.c_seq, (int64_t)nk * FCC);
    al(F.c_ts, (int64_t)nk * FCC);
    al(F.c_val, (int64_t)nk * FCC * 2);
    al(F.c_null, (int64_t)nk * FCC * 2);
    al(F.c_n, nk);
    al(F.c_match, (int64_t)nk * FCC);
    al(F.last_ts, nk);
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
    k_fast_gather<<<gb, 256, 0, s>>>(dprog, B, F, perm, skey, n, stream_, err);
    int gs = (int)std::min<int64_t>((std::max<int64_t>(n, (int64_t)nk * FCC) + 255) / 256, 8192);
    kt.mark("fast_search", s);
    k_fast_search<<<gs, 256, 0, s>>>(dprog, B, F, perm, skey, kbeg, kcnt, n, stream_);
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
