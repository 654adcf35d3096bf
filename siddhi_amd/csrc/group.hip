// siddhi-hip: key-sharded engine groups — multi-GPU behind the C-ABI ("Multi-GPU
// is internal to the engine, which owns the RCCL communicator"; §8e).
//
// A partitioned query's per-key state is isolated (PartitionStateHolder.java:43-48), so `world`
// engines split the keys: key k lives on rank k % world, as the dense id k / world there (the
// reference's own precedent for spreading by key is PartitionedDistributionStrategy.java:99-110).
// A push hands every rank one slice of the global stream (consecutive pieces, in rank order).
// Per push:
//   1. split   each rank splits its slice by destination rank, stable (HIP, k_gs_count +
//              k_gs_scatter below), into destination-grouped columns: ts, key / world, the
//              predicate columns, stream, and when the query needs them the global playback
//              clock (absent-state timers) and the events' global sequence numbers (match
//              records that name events);
//   2. counts  every rank learns every rank's counts, slice length and largest ts (the global
//              clock seed and sequence base): RCCL all-gather between processes, a host read
//              within one process;
//   3. exchange the columns go to their owners: grouped ncclSend / ncclRecv over xGMI between
//              processes, device-to-device copies within one process.  A rank receives its
//              events ordered by source rank, then arrival, i.e. in global order, so each key
//              sees its events in the reference's order;
//   4. run     each rank's engine processes what it received (shp_push_batch_device), plus one
//              clock-only event at the push's global clock so timers due before the end of the
//              global batch fire in this push as they do in one process.
// Clock-only events of the slices (stream -1) are not moved: the global clock column carries
// their effect.  Sharded absent-state timers are exact when every rank sees one of its own events
// at least every `waitingTime` of global clock (true for SURVEY §8d C4's dense stream): a timer
// then fires late on a rank by less than waitingTime, which leaves lastScheduledTime as in one
// process (AbsentStreamPreStateProcessor.java:216-223).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include <rocprim/rocprim.hpp>

#include "../../include/siddhi_hip.h"
#include "compile.h"

namespace {

constexpr int GS_THREADS = 512;  // split workgroup: 8 waves
constexpr int GS_TILE = 65536;  // events per split workgroup
constexpr int GS_MAXG = 16;
constexpr int GS_MAXCOL = 20;

// columns moved by the split: in[c] (4 or 8 bytes per event) -> out[c] grouped by destination
struct GsCols {
  int32_t n;
  int32_t sz[GS_MAXCOL];
  const void* in[GS_MAXCOL];
  void* out[GS_MAXCOL];
};

// per tile: events per destination (clock-only events go nowhere) and the tile's largest ts
__global__ __launch_bounds__(GS_THREADS) void k_gs_count(const int32_t* __restrict__ key,
                                                         const int32_t* __restrict__ stream,
                                                         const int64_t* __restrict__ ts, int64_t n, int G,
                                                         int ntiles, uint32_t* cnt, unsigned long long* tsmax) {
  __shared__ uint32_t h[GS_MAXG];
  if (threadIdx.x < GS_MAXG) h[threadIdx.x] = 0;
  __syncthreads();
  const int t = blockIdx.x;
  const int64_t lo = (int64_t)t * GS_TILE, hi = min(n, lo + GS_TILE);
  uint32_t c[GS_MAXG] = {};
  int64_t mx = INT64_MIN;
  for (int64_t i = lo + threadIdx.x; i < hi; i += GS_THREADS) {
    mx = max(mx, ts[i]);
    if (stream && stream[i] < 0) continue;
    const uint32_t d = (uint32_t)key[i] % (uint32_t)G;
#pragma unroll
    for (int g = 0; g < GS_MAXG; g++) c[g] += d == (uint32_t)g ? 1u : 0u;
  }
  for (int g = 0; g < G; g++)
    if (c[g]) atomicAdd(&h[g], c[g]);
  for (int d = 32; d > 0; d >>= 1) mx = max(mx, (int64_t)__shfl_xor((long long)mx, d, 64));
  if (__lane_id() == 0 && mx != INT64_MIN) atomicMax(tsmax, (unsigned long long)mx ^ (1ull << 63));
  __syncthreads();
  if (threadIdx.x < G) cnt[(int64_t)threadIdx.x * ntiles + t] = h[threadIdx.x];
}

// exclusive scan of the G x ntiles counts (destination-major), one workgroup; total per
// destination to tot[g]
__global__ __launch_bounds__(1024) void k_gs_scan(const uint32_t* cnt, uint32_t* off, int64_t m, int G, int ntiles,
                                                  int64_t* tot) {
  __shared__ uint32_t part[1024];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int64_t b = 0; b < m; b += 1024) {
    const int64_t i = b + threadIdx.x;
    const uint32_t v = i < m ? cnt[i] : 0u;
    part[threadIdx.x] = v;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
      const uint32_t y = threadIdx.x >= (unsigned)d ? part[threadIdx.x - d] : 0u;
      __syncthreads();
      part[threadIdx.x] += y;
      __syncthreads();
    }
    if (i < m) off[i] = carry + part[threadIdx.x] - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry += part[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) off[m] = carry;
  __syncthreads();
  if (threadIdx.x < G) tot[threadIdx.x] = (int64_t)off[(int64_t)(threadIdx.x + 1) * ntiles] - off[(int64_t)threadIdx.x * ntiles];
}

// stable split: per tile, rounds of 64 * SUB events per wave ranked by destination with wave
// ballots; per-wave running cursors.  Columns are written at their destination-grouped slot, one
// column at a time with the round's SUB loads of a lane issued before its SUB stores (a load ->
// store chain per element leaves one load in flight per lane).  Derived columns: key -> key / G;
// gclk -> max(seed, running max of ts) (the global clock); gseq -> seq_base + index.
template <int SUB>
__global__ __launch_bounds__(GS_THREADS) void k_gs_scatter(const int32_t* __restrict__ key,
                                                           const int32_t* __restrict__ stream,
                                                           const int64_t* __restrict__ ts,
                                                           const int64_t* __restrict__ rmax, int64_t n, int G,
                                                           int gbits, int ntiles, const uint32_t* __restrict__ off,
                                                           GsCols cols, int32_t* okey, int64_t* oclk, int64_t seed,
                                                           int64_t* oseq, int64_t seq_base) {
  constexpr int NW = GS_THREADS / 64;
  __shared__ uint32_t wc[NW][GS_MAXG];
  __shared__ uint32_t run[GS_MAXG];
  const int t = blockIdx.x;
  const uint32_t lane = __lane_id(), w = threadIdx.x >> 6;
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  if (threadIdx.x < G) run[threadIdx.x] = off[(int64_t)threadIdx.x * ntiles + t];
  const int64_t lo = (int64_t)t * GS_TILE, hi = min(n, lo + GS_TILE);
  constexpr int ROUND = GS_THREADS * SUB;
  for (int64_t r0 = lo; r0 < hi; r0 += ROUND) {
    if (threadIdx.x < NW * GS_MAXG) (&wc[0][0])[threadIdx.x] = 0;
    __syncthreads();
    uint32_t dst[SUB], rk[SUB], kq[SUB];
#pragma unroll
    for (int s = 0; s < SUB; s++) {
      const int64_t i = r0 + (int64_t)w * (64 * SUB) + s * 64 + lane;
      dst[s] = GS_MAXG;
      kq[s] = 0;
      if (i < hi && !(stream && stream[i] < 0)) {
        kq[s] = (uint32_t)key[i];
        dst[s] = kq[s] % (uint32_t)G;
      }
    }
#pragma unroll
    for (int s = 0; s < SUB; s++) {
      const bool valid = dst[s] < GS_MAXG;
      uint64_t peers = __ballot(valid);
      for (int b = 0; b < gbits; b++) {
        const bool bit = (dst[s] >> b) & 1u;
        const uint64_t m = __ballot(bit);
        peers &= bit ? m : ~m;
      }
      const uint32_t before = valid ? wc[w][dst[s]] : 0u;
      rk[s] = before + (uint32_t)__popcll(peers & lt);
      if (valid && (peers & lt) == 0) wc[w][dst[s]] = before + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    if (threadIdx.x < (unsigned)G) {  // wave cursors of destination d: its run, then the waves in order
      const int d = (int)threadIdx.x;
      uint32_t g = run[d];
#pragma unroll
      for (int ww = 0; ww < NW; ww++) {
        const uint32_t c = wc[ww][d];
        wc[ww][d] = g;
        g += c;
      }
      run[d] = g;
    }
    __syncthreads();
    uint32_t o[SUB];
#pragma unroll
    for (int s = 0; s < SUB; s++) o[s] = dst[s] < GS_MAXG ? wc[w][dst[s]] + rk[s] : 0u;
    const int64_t i0 = r0 + (int64_t)w * (64 * SUB) + lane;
#pragma unroll
    for (int s = 0; s < SUB; s++)
      if (dst[s] < GS_MAXG) okey[o[s]] = (int32_t)(kq[s] / (uint32_t)G);
    for (int c = 0; c < cols.n; c++) {
      if (cols.sz[c] == 8) {
        const int64_t* in = (const int64_t*)cols.in[c];
        int64_t v[SUB];
#pragma unroll
        for (int s = 0; s < SUB; s++) v[s] = dst[s] < GS_MAXG ? in[i0 + s * 64] : 0;
#pragma unroll
        for (int s = 0; s < SUB; s++)
          if (dst[s] < GS_MAXG) ((int64_t*)cols.out[c])[o[s]] = v[s];
      } else if (cols.sz[c] == 4) {
        const int32_t* in = (const int32_t*)cols.in[c];
        int32_t v[SUB];
#pragma unroll
        for (int s = 0; s < SUB; s++) v[s] = dst[s] < GS_MAXG ? in[i0 + s * 64] : 0;
#pragma unroll
        for (int s = 0; s < SUB; s++)
          if (dst[s] < GS_MAXG) ((int32_t*)cols.out[c])[o[s]] = v[s];
      } else {  // null bytes
        const uint8_t* in = (const uint8_t*)cols.in[c];
        uint8_t v[SUB];
#pragma unroll
        for (int s = 0; s < SUB; s++) v[s] = dst[s] < GS_MAXG ? in[i0 + s * 64] : 0;
#pragma unroll
        for (int s = 0; s < SUB; s++)
          if (dst[s] < GS_MAXG) ((uint8_t*)cols.out[c])[o[s]] = v[s];
      }
    }
    if (oclk) {
      int64_t v[SUB];
#pragma unroll
      for (int s = 0; s < SUB; s++) v[s] = dst[s] < GS_MAXG ? rmax[i0 + s * 64] : 0;
#pragma unroll
      for (int s = 0; s < SUB; s++)
        if (dst[s] < GS_MAXG) oclk[o[s]] = max(seed, v[s]);
    }
    if (oseq)
#pragma unroll
      for (int s = 0; s < SUB; s++)
        if (dst[s] < GS_MAXG) oseq[o[s]] = seq_base + i0 + s * 64;
    __syncthreads();
  }
}

__global__ void k_gs_fill_tail(int64_t* ts, int32_t* key, int32_t* stream, int64_t* clk, int64_t* seq, int64_t at,
                               int64_t clock, int64_t seqv) {
  ts[at] = clock;
  key[at] = 0;
  stream[at] = -1;
  if (clk) clk[at] = clock;
  if (seq) seq[at] = seqv;
}

// ---- device gather of the matches (shp_group_gather_matches): each rank's records of the last push
// move to the root in HBM (RCCL send / recv between processes, peer copies within one process);
// the per-record work (global key ids, slot stride, ref offsets) runs on the device and the host
// takes the gathered columns with one copy each
__global__ void k_gm_nref(const int16_t* __restrict__ slot, int64_t m, int S, int64_t* __restrict__ nref) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t t = 0;
    for (int s = 0; s < S; s++) t += slot[i * shp::MAXS + s];
    nref[i] = t;
  }
}
// global key ids, slot lengths at stride S, and the refs in record order (the engine appends a
// record's refs wherever its reservation fell): noff = exclusive scan of the records' ref counts
__global__ void k_gm_pack(const int32_t* __restrict__ key, const int16_t* __restrict__ slot,
                          const int64_t* __restrict__ off, const int64_t* __restrict__ refs, int64_t m, int S,
                          int world, int rank, int32_t* __restrict__ okey, int16_t* __restrict__ oslot,
                          const int64_t* __restrict__ noff, int64_t* __restrict__ orefs) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    okey[i] = (int32_t)((int64_t)key[i] * world + rank);  // rank-local dense id -> global key
    if (slot) {
      int64_t o = off[i], d = noff[i];
      for (int s = 0; s < S; s++) {
        const int l = slot[i * shp::MAXS + s];
        oslot[i * S + s] = (int16_t)l;
        for (int t = 0; t < l; t++) orefs[d++] = refs[o++];
      }
    }
  }
}
__global__ void k_gm_rebase(int64_t* __restrict__ off, int64_t m, int64_t base) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
    off[i] += base;
}

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  void ensure(size_t b) {
    if (b <= bytes) return;
    if (p) (void)hipFree(p);
    p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(b, 256)) != hipSuccess) throw std::runtime_error("hipMalloc failed (group)");
    bytes = std::max<size_t>(b, 256);
  }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

int col_bytes(int8_t tag) { return (tag == shp::T_LONG || tag == shp::T_DOUBLE) ? 8 : (tag == shp::T_BOOL ? 1 : 4); }

}  // namespace

// engine.hip (internal): the last push's records in HBM, pair layouts expanded to full records
extern "C" int shp_engine_device_records(shp_engine* e, shp_matches* out, int64_t* nrefs);

struct shp_group {
  int world = 1;
  int rank0 = 0;  // rank of local slot 0
  int nlocal = 1;
  bool rccl = false;
  ncclComm_t comm = nullptr;
  shp_config cfg{};
  shp::ProgramCompiler comp;
  bool need_clock = false, need_seq = false, has_stream_col = false;
  int ncol = 0;
  std::vector<int8_t> ctag;
  struct Local {
    int dev = 0;
    int rank = 0;
    shp_engine* eng = nullptr;
    hipStream_t s = nullptr;
    hipEvent_t split_done = nullptr;
    // split workspace
    DevBuf cnt, off, tot, tsmax, rmax, scan_tmp;
    // send (destination-grouped) columns: ts, key, stream, clock, seq, predicate columns
    DevBuf s_ts, s_key, s_stream, s_clk, s_seq;
    DevBuf s_col[shp::MAXCOL], s_null[shp::MAXCOL];
    DevBuf zero;                    // zero bytes: the null column of a slice without one
    int64_t n_slice = 0;
    int64_t max_ts = INT64_MIN;
    uint32_t null_mask = 0;         // columns this rank's slice carries a null array for
    std::vector<int64_t> send_cnt;  // per destination
    // three receive slots: batch i + 2 can be exchanged while the engines run batch i
    struct Slot {
      DevBuf r_ts, r_key, r_stream, r_clk, r_seq;
      DevBuf r_col[shp::MAXCOL], r_null[shp::MAXCOL];
      uint32_t null_cols = 0;         // columns whose null bytes this batch exchanges
      std::vector<int64_t> recv_cnt;  // per source
      int64_t n_recv = 0;
      int64_t push_clock = INT64_MIN, next_seq = 0;
      hipEvent_t done = nullptr;      // the exchange into this slot has landed
    } slot[3];
    int64_t last_m = 0;
    DevBuf p_key, p_slot, p_off, p_refs, p_tmp;  // gather: this rank's records, global key ids, S-stride slots,
                                                 // refs in record order
  };
  std::atomic<int64_t> staged{0}, ran{0};  // batches exchanged / run (at most three staged ahead)
  std::vector<Local> L;
  int64_t seq = 0;              // global sequence number of the next push's first event
  int64_t clock = INT64_MIN;    // global playback clock
  std::string err;
  // host copies of the last fetch
  std::vector<int32_t> h_key;
  std::vector<int64_t> h_ts, h_pos, h_off, h_refs;
  std::vector<int8_t> h_type;
  std::vector<int16_t> h_slot;
  std::vector<double> h_agg;
  // gather: the root's device columns (key, ts, type, pos, ref_off, slot_len, refs, agg)
  DevBuf g_key, g_ts, g_type, g_pos, g_off, g_slot, g_refs, g_agg;

  int fail(int code, const std::string& m) {
    err = m;
    return code;
  }
};

namespace {

#define GH(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)
#define GN(x)                                                                                \
  do {                                                                                       \
    ncclResult_t r_ = (x);                                                                   \
    if (r_ != ncclSuccess) throw std::runtime_error(std::string(#x) + ": " + ncclGetErrorString(r_)); \
  } while (0)

// step 1a: per-destination counts, slice length and largest ts (device -> host)
void split_count(shp_group& g, shp_group::Local& l, const shp_batch& b) {
  GH(hipSetDevice(l.dev));
  const int G = g.world;
  const int64_t n = b.n;
  const int ntiles = (int)std::max<int64_t>(1, (n + GS_TILE - 1) / GS_TILE);
  l.cnt.ensure((size_t)G * ntiles * 4 + 4);
  l.off.ensure(((size_t)G * ntiles + 1) * 4);
  l.tot.ensure(GS_MAXG * 8);
  l.tsmax.ensure(8);
  GH(hipMemsetAsync(l.tsmax.p, 0, 8, l.s));
  GH(hipMemsetAsync(l.cnt.p, 0, (size_t)G * ntiles * 4, l.s));
  if (n > 0)
    k_gs_count<<<ntiles, GS_THREADS, 0, l.s>>>(b.key, b.stream, b.ts, n, G, ntiles, (uint32_t*)l.cnt.p,
                                               (unsigned long long*)l.tsmax.p);
  k_gs_scan<<<1, 1024, 0, l.s>>>((const uint32_t*)l.cnt.p, (uint32_t*)l.off.p, (int64_t)G * ntiles, G, ntiles,
                                 (int64_t*)l.tot.p);
  GH(hipGetLastError());
  std::vector<int64_t> tot(GS_MAXG);
  unsigned long long mx = 0;
  GH(hipMemcpyAsync(tot.data(), l.tot.p, GS_MAXG * 8, hipMemcpyDeviceToHost, l.s));
  GH(hipMemcpyAsync(&mx, l.tsmax.p, 8, hipMemcpyDeviceToHost, l.s));
  GH(hipStreamSynchronize(l.s));
  l.send_cnt.assign(tot.begin(), tot.begin() + G);
  l.n_slice = n;
  l.null_mask = 0;
  for (int c = 0; c < g.ncol; c++)
    if (b.nulls && b.nulls[c]) l.null_mask |= 1u << c;
  l.max_ts = mx ? (int64_t)(mx ^ (1ull << 63)) : INT64_MIN;
}

// step 1b: the scatter into destination-grouped send columns
void split_scatter(shp_group& g, shp_group::Local& l, const shp_batch& b, int64_t clock_seed, int64_t seq_base,
                   uint32_t null_cols) {
  GH(hipSetDevice(l.dev));
  const int G = g.world;
  const int64_t n = b.n;
  const int ntiles = (int)std::max<int64_t>(1, (n + GS_TILE - 1) / GS_TILE);
  const size_t cap = (size_t)std::max<int64_t>(n, 1);
  l.s_ts.ensure(cap * 8);
  l.s_key.ensure(cap * 4);
  GsCols cols{};
  cols.n = 0;
  auto add = [&](const void* in, DevBuf& out, int sz) {
    out.ensure(cap * sz);
    cols.in[cols.n] = in;
    cols.out[cols.n] = out.p;
    cols.sz[cols.n] = sz;
    cols.n++;
  };
  add(b.ts, l.s_ts, 8);
  if (g.has_stream_col) add(b.stream, l.s_stream, 4);
  for (int c = 0; c < g.ncol; c++) {
    const int sz = col_bytes(g.ctag[c]);
    if (sz == 1) throw std::runtime_error("group: bool columns are not exchanged");
    add(b.cols[c], l.s_col[c], sz);
  }
  // null bytes travel as 1-byte columns for every column some rank's slice has nulls in (the
  // same set on every rank: the masks are all-gathered); a slice without them sends zeros
  for (int c = 0; c < g.ncol; c++) {
    if (!((null_cols >> c) & 1u)) continue;
    const uint8_t* in = (b.nulls && b.nulls[c]) ? b.nulls[c] : nullptr;
    if (!in) {
      if (l.zero.bytes < cap) {
        l.zero.ensure(cap);
        GH(hipMemsetAsync(l.zero.p, 0, l.zero.bytes, l.s));
      }
      in = (const uint8_t*)l.zero.p;
    }
    add(in, l.s_null[c], 1);
  }
  int64_t* oclk = nullptr;
  if (g.need_clock && n > 0) {  // the global clock after each event: running max of ts, seeded
    l.rmax.ensure(cap * 8);
    size_t tb = 0;
    GH(rocprim::inclusive_scan(nullptr, tb, b.ts, (int64_t*)l.rmax.p, (size_t)n, rocprim::maximum<int64_t>(), l.s));
    l.scan_tmp.ensure(tb);
    GH(rocprim::inclusive_scan(l.scan_tmp.p, tb, b.ts, (int64_t*)l.rmax.p, (size_t)n, rocprim::maximum<int64_t>(),
                               l.s));
    l.s_clk.ensure(cap * 8);
    oclk = (int64_t*)l.s_clk.p;
  }
  int64_t* oseq = nullptr;
  if (g.need_seq) {
    l.s_seq.ensure(cap * 8);
    oseq = (int64_t*)l.s_seq.p;
  }
  int gbits = 0;
  while ((1 << gbits) < G) gbits++;
  if (n > 0)
    k_gs_scatter<8><<<ntiles, GS_THREADS, 0, l.s>>>(b.key, b.stream, b.ts, (const int64_t*)l.rmax.p, n, G, gbits,
                                                   ntiles, (const uint32_t*)l.off.p, cols, (int32_t*)l.s_key.p, oclk,
                                                   clock_seed, oseq, seq_base);
  GH(hipGetLastError());
  GH(hipEventRecord(l.split_done, l.s));
}

void ensure_recv(shp_group& g, shp_group::Local::Slot& r, int64_t n) {
  const size_t cap = (size_t)n + 1;  // + the end-of-push clock event
  r.r_ts.ensure(cap * 8);
  r.r_key.ensure(cap * 4);
  r.r_stream.ensure(cap * 4);
  if (g.need_clock) r.r_clk.ensure(cap * 8);
  if (g.need_seq) r.r_seq.ensure(cap * 8);
  for (int c = 0; c < g.ncol; c++) r.r_col[c].ensure(cap * col_bytes(g.ctag[c]));
  for (int c = 0; c < g.ncol; c++)
    if ((r.null_cols >> c) & 1u) r.r_null[c].ensure(cap);
}

// the columns exchanged, as (send buffer, receive buffer, bytes per event)
std::vector<std::tuple<void*, void*, int>> column_pairs(shp_group& g, shp_group::Local& src,
                                                        shp_group::Local::Slot& dst) {
  std::vector<std::tuple<void*, void*, int>> v = {{src.s_ts.p, dst.r_ts.p, 8}, {src.s_key.p, dst.r_key.p, 4}};
  if (g.has_stream_col) v.emplace_back(src.s_stream.p, dst.r_stream.p, 4);
  if (g.need_clock) v.emplace_back(src.s_clk.p, dst.r_clk.p, 8);
  if (g.need_seq) v.emplace_back(src.s_seq.p, dst.r_seq.p, 8);
  for (int c = 0; c < g.ncol; c++) v.emplace_back(src.s_col[c].p, dst.r_col[c].p, col_bytes(g.ctag[c]));
  for (int c = 0; c < g.ncol; c++)
    if ((dst.null_cols >> c) & 1u) v.emplace_back(src.s_null[c].p, dst.r_null[c].p, 1);
  return v;
}

// step 4: one engine push of what a rank received (slot r), plus the end-of-push clock event
int run_local(shp_group& g, shp_group::Local& l, shp_group::Local::Slot& r) {
  GH(hipSetDevice(l.dev));
  GH(hipEventSynchronize(r.done));
  const int64_t push_clock = r.push_clock, next_seq = r.next_seq;
  const int64_t m = r.n_recv;
  const bool tail = g.need_clock && push_clock != INT64_MIN;
  std::vector<const void*> colp(std::max(1, g.ncol));
  for (int c = 0; c < g.ncol; c++) colp[c] = r.r_col[c].p;
  shp_batch b{};
  b.n = m + (tail ? 1 : 0);
  b.ts = (const int64_t*)r.r_ts.p;
  b.key = (const int32_t*)r.r_key.p;
  b.stream = (const int32_t*)r.r_stream.p;
  b.cols = colp.data();
  std::vector<const uint8_t*> nullp(std::max(1, g.ncol), nullptr);
  for (int c = 0; c < g.ncol; c++)
    if ((r.null_cols >> c) & 1u) nullp[c] = (const uint8_t*)r.r_null[c].p;
  b.nulls = r.null_cols ? nullp.data() : nullptr;
  b.clock = g.need_clock ? (const int64_t*)r.r_clk.p : nullptr;
  b.seq = g.need_seq ? (const int64_t*)r.r_seq.p : nullptr;
  (void)next_seq;
  if (b.n == 0) {
    l.last_m = 0;
    return SHP_OK;
  }
  shp_matches mt{};
  const int rc = shp_push_batch_device(l.eng, &b, &mt);
  if (rc != SHP_OK) {
    g.err = std::string("rank ") + std::to_string(l.rank) + ": " + shp_last_error(l.eng);
    return rc;
  }
  l.last_m = mt.m;
  return SHP_OK;
}

// steps 1-3 for one batch into the next receive slot (asynchronous once the counts are known)
int stage_impl(shp_group& g, const shp_batch* slices) {
  const int G = g.world;
  if (g.staged - g.ran >= 3) return g.fail(SHP_ERR_ARG, "three batches are staged already (run one first)");
  const int sl = (int)(g.staged % 3);
  if (!g.rccl && g.staged > 0) {  // the previous batch's copies read the send columns this split rewrites
    const int prev = (int)((g.staged - 1) % 3);
    for (auto& a : g.L) {
      GH(hipSetDevice(a.dev));
      for (auto& b : g.L) GH(hipStreamWaitEvent(a.s, b.slot[prev].done, 0));
    }
  }
  // 1a + 2: counts, slice lengths, largest ts of every rank
  for (int i = 0; i < g.nlocal; i++) split_count(g, g.L[i], slices[i]);
  constexpr int X = 3;  // per rank: counts[G], n, maxts, null-column mask
  std::vector<int64_t> all((size_t)G * (G + X));
  if (g.rccl) {
    shp_group::Local& l = g.L[0];
    DevBuf mine, gath;
    mine.ensure((G + X) * 8);
    gath.ensure((size_t)G * (G + X) * 8);
    std::vector<int64_t> v(l.send_cnt);
    v.push_back(l.n_slice);
    v.push_back(l.max_ts);
    v.push_back((int64_t)l.null_mask);
    GH(hipMemcpyAsync(mine.p, v.data(), (G + X) * 8, hipMemcpyHostToDevice, l.s));
    GN(ncclAllGather(mine.p, gath.p, (size_t)(G + X), ncclInt64, g.comm, l.s));
    GH(hipMemcpyAsync(all.data(), gath.p, all.size() * 8, hipMemcpyDeviceToHost, l.s));
    GH(hipStreamSynchronize(l.s));
  } else {
    for (int i = 0; i < g.nlocal; i++) {
      shp_group::Local& l = g.L[i];
      for (int d = 0; d < G; d++) all[(size_t)l.rank * (G + X) + d] = l.send_cnt[d];
      all[(size_t)l.rank * (G + X) + G] = l.n_slice;
      all[(size_t)l.rank * (G + X) + G + 1] = l.max_ts;
      all[(size_t)l.rank * (G + X) + G + 2] = (int64_t)l.null_mask;
    }
  }
  auto cnt = [&](int s, int d) { return all[(size_t)s * (G + X) + d]; };
  std::vector<int64_t> base(G + 1, g.seq), seed(G + 1, g.clock);
  uint32_t null_cols = 0;
  for (int r = 0; r < G; r++) {
    base[r + 1] = base[r] + all[(size_t)r * (G + X) + G];
    seed[r + 1] = std::max(seed[r], all[(size_t)r * (G + X) + G + 1]);
    null_cols |= (uint32_t)all[(size_t)r * (G + X) + G + 2];
  }
  // every rank's receive total from the all-gathered counts (identical on every rank): if any
  // rank would overflow, every rank fails here, before any exchange is posted (a rank that failed
  // alone would leave its peers blocked in ncclSend / ncclRecv to it)
  for (int d = 0; d < G; d++) {
    int64_t tot = 0;
    for (int s = 0; s < G; s++) tot += cnt(s, d);
    if (tot + 1 > g.cfg.max_batch)
      return g.fail(SHP_ERR_CAPACITY, "rank " + std::to_string(d) + " would receive " + std::to_string(tot) +
                                          " events (> max_batch)");
  }
  for (int i = 0; i < g.nlocal; i++) {
    shp_group::Local::Slot& r = g.L[i].slot[sl];
    r.recv_cnt.assign(G, 0);
    r.n_recv = 0;
    for (int s = 0; s < G; s++) {
      r.recv_cnt[s] = cnt(s, g.L[i].rank);
      r.n_recv += r.recv_cnt[s];
    }
    if (r.n_recv + 1 > g.cfg.max_batch)
      return g.fail(SHP_ERR_CAPACITY, "rank " + std::to_string(g.L[i].rank) + " would receive " +
                                          std::to_string(r.n_recv) + " events (> max_batch)");
    r.push_clock = seed[G];
    r.next_seq = base[G];
    r.null_cols = null_cols;
  }
  // 1b: scatter
  for (int i = 0; i < g.nlocal; i++)
    split_scatter(g, g.L[i], slices[i], seed[g.L[i].rank], base[g.L[i].rank], null_cols);
  for (int i = 0; i < g.nlocal; i++) ensure_recv(g, g.L[i].slot[sl], g.L[i].slot[sl].n_recv);
  // 3: exchange
  if (g.rccl) {
    shp_group::Local& l = g.L[0];
    shp_group::Local::Slot& r = l.slot[sl];
    GH(hipSetDevice(l.dev));
    auto cols = column_pairs(g, l, r);
    GN(ncclGroupStart());
    for (auto& c : cols) {
      void* sb = std::get<0>(c);
      void* rb = std::get<1>(c);
      const int sz = std::get<2>(c);
      int64_t so = 0, ro = 0;
      for (int p = 0; p < G; p++) {
        const int64_t sn = l.send_cnt[p], rn = r.recv_cnt[p];
        if (sn) GN(ncclSend((char*)sb + so * sz, (size_t)sn * sz, ncclChar, p, g.comm, l.s));
        if (rn) GN(ncclRecv((char*)rb + ro * sz, (size_t)rn * sz, ncclChar, p, g.comm, l.s));
        so += sn;
        ro += rn;
      }
    }
    GN(ncclGroupEnd());
  } else {
    for (int di = 0; di < g.nlocal; di++) {
      shp_group::Local& dst = g.L[di];
      shp_group::Local::Slot& r = dst.slot[sl];
      GH(hipSetDevice(dst.dev));
      int64_t ro = 0;
      for (int si = 0; si < g.nlocal; si++) {
        shp_group::Local& src = g.L[si];
        GH(hipStreamWaitEvent(dst.s, src.split_done, 0));
        int64_t so = 0;
        for (int d = 0; d < dst.rank; d++) so += src.send_cnt[d];
        const int64_t k = src.send_cnt[dst.rank];
        if (k)
          for (auto& c : column_pairs(g, src, r)) {
            const int sz = std::get<2>(c);
            GH(hipMemcpyPeerAsync((char*)std::get<1>(c) + ro * sz, dst.dev, (char*)std::get<0>(c) + so * sz, src.dev,
                                  (size_t)k * sz, dst.s));
          }
        ro += k;
      }
    }
  }
  // the received batch's stream column (when the query reads one stream) and its end-of-push
  // clock event, then the slot is ready
  for (int i = 0; i < g.nlocal; i++) {
    shp_group::Local& l = g.L[i];
    shp_group::Local::Slot& r = l.slot[sl];
    GH(hipSetDevice(l.dev));
    if (!g.has_stream_col) GH(hipMemsetAsync(r.r_stream.p, 0, (size_t)r.n_recv * 4, l.s));
    for (int c = 0; c < g.ncol; c++)
      if ((r.null_cols >> c) & 1u) GH(hipMemsetAsync((uint8_t*)r.r_null[c].p + r.n_recv, 0, 1, l.s));
    if (g.need_clock && r.push_clock != INT64_MIN)
      k_gs_fill_tail<<<1, 1, 0, l.s>>>((int64_t*)r.r_ts.p, (int32_t*)r.r_key.p, (int32_t*)r.r_stream.p,
                                       (int64_t*)r.r_clk.p, g.need_seq ? (int64_t*)r.r_seq.p : nullptr, r.n_recv,
                                       r.push_clock, r.next_seq);
    GH(hipGetLastError());
    GH(hipEventRecord(r.done, l.s));
  }
  g.seq = base[G];
  if (seed[G] != INT64_MIN) g.clock = std::max(g.clock, seed[G]);
  g.staged++;
  return SHP_OK;
}

// step 4 for the oldest staged batch: every local engine runs what it received (one host thread
// per engine, so the GPUs of an in-process group overlap)
int run_impl(shp_group& g, int64_t* counts) {
  if (g.ran == g.staged) return g.fail(SHP_ERR_ARG, "no staged batch to run");
  const int sl = (int)(g.ran % 3);
  std::vector<int> rcs(g.nlocal, SHP_OK);
  std::vector<std::string> errs(g.nlocal);
  auto one = [&](int i) {
    try {
      rcs[i] = run_local(g, g.L[i], g.L[i].slot[sl]);
    } catch (std::exception& ex) {
      errs[i] = ex.what();
      rcs[i] = SHP_ERR_DEVICE;
    }
  };
  if (g.nlocal == 1) {
    one(0);
  } else {
    std::vector<std::thread> th;
    for (int i = 0; i < g.nlocal; i++) th.emplace_back(one, i);
    for (auto& t : th) t.join();
  }
  g.ran++;
  for (int i = 0; i < g.nlocal; i++) {
    if (!errs[i].empty()) return g.fail(rcs[i], errs[i]);
    if (rcs[i] != SHP_OK) return rcs[i];
  }
  if (counts)
    for (int i = 0; i < g.nlocal; i++) counts[i] = g.L[i].last_m;
  return SHP_OK;
}

// shp_group_gather_matches: every rank's records of the last push to `root` (a collective call
// between processes).  Per rank r: m_r records and n_r refs, all-gathered; the root's columns hold
// rank 0's records, then rank 1's, ...; each rank's keep their engine's per-key order.
int gather_impl(shp_group& g, int root, shp_matches* out) {
  const int G = g.world;
  if (root < 0 || root >= G) return g.fail(SHP_ERR_ARG, "root outside the group");
  const int S = shp_engine_num_states(g.L[0].eng);
  std::vector<shp_matches> dm(g.nlocal);
  // per local rank: records, refs, layout, and its status -- a rank whose records cannot be
  // prepared reports it through the all-gather instead of returning early, so no rank is left
  // waiting in the collectives below: every rank sees every status and all fail together
  std::vector<int64_t> mine(4 * (size_t)g.nlocal);
  std::string why;
  for (int i = 0; i < g.nlocal; i++) {
    int64_t nr = 0;
    const int rc = shp_engine_device_records(g.L[i].eng, &dm[i], &nr);
    if (rc != SHP_OK && why.empty()) why = "rank " + std::to_string(g.L[i].rank) + ": " + shp_last_error(g.L[i].eng);
    mine[4 * i] = rc == SHP_OK ? dm[i].m : 0;
    mine[4 * i + 1] = rc == SHP_OK ? nr : 0;
    mine[4 * i + 2] = rc == SHP_OK ? dm[i].layout : 0;
    mine[4 * i + 3] = rc;
  }
  std::vector<int64_t> all4(4 * (size_t)G);
  if (g.rccl) {
    shp_group::Local& l = g.L[0];
    GH(hipSetDevice(l.dev));
    DevBuf a, b;
    a.ensure(4 * 8);
    b.ensure((size_t)G * 4 * 8);
    GH(hipMemcpyAsync(a.p, mine.data(), 4 * 8, hipMemcpyHostToDevice, l.s));
    GN(ncclAllGather(a.p, b.p, 4, ncclInt64, g.comm, l.s));
    GH(hipMemcpyAsync(all4.data(), b.p, all4.size() * 8, hipMemcpyDeviceToHost, l.s));
    GH(hipStreamSynchronize(l.s));
  } else {
    all4 = mine;
  }
  for (int r = 0; r < G; r++)
    if (all4[4 * r + 3] != SHP_OK)
      return g.fail((int)all4[4 * r + 3], why.empty() ? "rank " + std::to_string(r) + " could not prepare its matches" : why);
  std::vector<int64_t> all(3 * (size_t)G);
  for (int r = 0; r < G; r++)
    for (int k = 0; k < 3; k++) all[3 * r + k] = all4[4 * r + k];
  for (int i = 0; i < g.nlocal; i++) {
    mine[3 * i] = mine[4 * i];
    mine[3 * i + 1] = mine[4 * i + 1];
    mine[3 * i + 2] = mine[4 * i + 2];
  }
  const bool agg = all[2] == SHP_LAYOUT_AGG;
  std::vector<int64_t> mb(G + 1, 0), rb(G + 1, 0);
  for (int r = 0; r < G; r++) {
    mb[r + 1] = mb[r] + all[3 * r];
    rb[r + 1] = rb[r] + all[3 * r + 1];
  }
  const int64_t M = mb[G], R = rb[G];
  // pack: global key ids, slot lengths at stride S, refs in record order with their new offsets
  for (int i = 0; i < g.nlocal; i++) {
    shp_group::Local& l = g.L[i];
    const int64_t m = dm[i].m, nr = mine[3 * i + 1];
    GH(hipSetDevice(l.dev));
    const unsigned gb = (unsigned)std::min<int64_t>((m + 255) / 256, 4096);
    l.p_key.ensure((size_t)std::max<int64_t>(m, 1) * 4);
    if (!agg) {
      l.p_slot.ensure((size_t)std::max<int64_t>(m, 1) * S * 2);
      l.p_off.ensure((size_t)std::max<int64_t>(m, 1) * 8);
      l.p_refs.ensure((size_t)std::max<int64_t>(nr, 1) * 8);
      l.rmax.ensure((size_t)std::max<int64_t>(m, 1) * 8);  // scratch: the records' ref counts
    }
    if (m > 0 && !agg) {
      k_gm_nref<<<gb, 256, 0, l.s>>>(dm[i].slot_len, m, S, (int64_t*)l.rmax.p);
      size_t tb = 0;
      GH(rocprim::exclusive_scan(nullptr, tb, (const int64_t*)l.rmax.p, (int64_t*)l.p_off.p, (int64_t)0, (size_t)m,
                                 rocprim::plus<int64_t>(), l.s));
      l.p_tmp.ensure(tb);
      GH(rocprim::exclusive_scan(l.p_tmp.p, tb, (const int64_t*)l.rmax.p, (int64_t*)l.p_off.p, (int64_t)0, (size_t)m,
                                 rocprim::plus<int64_t>(), l.s));
    }
    if (m > 0)
      k_gm_pack<<<gb, 256, 0, l.s>>>(dm[i].key, agg ? nullptr : dm[i].slot_len, dm[i].ref_off, dm[i].refs, m, S, G,
                                     l.rank, (int32_t*)l.p_key.p, agg ? nullptr : (int16_t*)l.p_slot.p,
                                     (const int64_t*)l.p_off.p, (int64_t*)l.p_refs.p);
    GH(hipGetLastError());
  }
  // the root's local slot (an in-process group: local index = rank)
  int ri = -1;
  for (int i = 0; i < g.nlocal; i++)
    if (g.L[i].rank == root) ri = i;
  struct Col {
    DevBuf* dst;
    int sz;
  };
  std::vector<Col> cols = agg ? std::vector<Col>{{&g.g_key, 4}, {&g.g_agg, 8}}
                              : std::vector<Col>{{&g.g_key, 4}, {&g.g_ts, 8}, {&g.g_type, 1}, {&g.g_pos, 8},
                                                 {&g.g_off, 8}, {&g.g_slot, 2 * S}};
  auto src_of = [&](int i, int c) -> const void* {  // local rank i's device column c (and refs: c = -1)
    const shp_matches& d = dm[i];
    if (c < 0) return g.L[i].p_refs.p;
    if (c == 0) return g.L[i].p_key.p;
    if (agg) return d.agg;
    switch (c) {
      case 1: return d.ts;
      case 2: return d.type;
      case 3: return d.pos;
      case 4: return g.L[i].p_off.p;
      default: return g.L[i].p_slot.p;
    }
  };
  if (ri >= 0) {
    GH(hipSetDevice(g.L[ri].dev));
    for (auto& c : cols) c.dst->ensure((size_t)std::max<int64_t>(M, 1) * c.sz);
    if (!agg) g.g_refs.ensure((size_t)std::max<int64_t>(R, 1) * 8);
  }
  if (g.rccl) {
    shp_group::Local& l = g.L[0];
    GH(hipSetDevice(l.dev));
    GN(ncclGroupStart());
    for (size_t c = 0; c < cols.size() + (agg ? 0 : 1); c++) {
      const bool refs = c == cols.size();
      const int sz = refs ? 8 : cols[c].sz;
      const int64_t mm = refs ? mine[1] : mine[0];  // this rank's records / refs
      if (mm > 0) GN(ncclSend(src_of(0, refs ? -1 : (int)c), (size_t)mm * sz, ncclChar, root, g.comm, l.s));
      if (l.rank == root)
        for (int r = 0; r < G; r++) {
          const int64_t n = refs ? all[3 * r + 1] : all[3 * r];
          const int64_t o = refs ? rb[r] : mb[r];
          void* dst = refs ? g.g_refs.p : cols[c].dst->p;
          if (n > 0) GN(ncclRecv((char*)dst + o * sz, (size_t)n * sz, ncclChar, r, g.comm, l.s));
        }
    }
    GN(ncclGroupEnd());
  } else {
    shp_group::Local& rl = g.L[ri];
    for (int i = 0; i < g.nlocal; i++) {
      GH(hipSetDevice(g.L[i].dev));
      GH(hipStreamSynchronize(g.L[i].s));
    }
    GH(hipSetDevice(rl.dev));
    for (int i = 0; i < g.nlocal; i++) {
      const int r = g.L[i].rank;
      for (size_t c = 0; c < cols.size() + (agg ? 0 : 1); c++) {
        const bool refs = c == cols.size();
        const int sz = refs ? 8 : cols[c].sz;
        const int64_t n = refs ? all[3 * r + 1] : all[3 * r];
        const int64_t o = refs ? rb[r] : mb[r];
        void* dst = refs ? g.g_refs.p : cols[c].dst->p;
        if (n > 0)
          GH(hipMemcpyPeerAsync((char*)dst + o * sz, rl.dev, src_of(i, refs ? -1 : (int)c), g.L[i].dev, (size_t)n * sz,
                                rl.s));
      }
    }
  }
  *out = shp_matches{};
  out->num_states = S;
  out->layout = agg ? SHP_LAYOUT_AGG : SHP_LAYOUT_FULL;
  if (ri < 0) {  // not the root: its records went there
    out->m = 0;
    return SHP_OK;
  }
  shp_group::Local& rl = g.L[ri];
  GH(hipSetDevice(rl.dev));
  if (!agg)  // each source's ref offsets continue after the refs of the ranks before it
    for (int r = 1; r < G; r++)
      if (all[3 * r] > 0)
        k_gm_rebase<<<(unsigned)std::min<int64_t>((all[3 * r] + 255) / 256, 4096), 256, 0, rl.s>>>(
            (int64_t*)g.g_off.p + mb[r], all[3 * r], rb[r]);
  GH(hipGetLastError());
  g.h_key.resize(M);
  GH(hipMemcpyAsync(g.h_key.data(), g.g_key.p, (size_t)M * 4, hipMemcpyDeviceToHost, rl.s));
  if (agg) {
    g.h_agg.resize(M);
    GH(hipMemcpyAsync(g.h_agg.data(), g.g_agg.p, (size_t)M * 8, hipMemcpyDeviceToHost, rl.s));
  } else {
    g.h_ts.resize(M);
    g.h_type.resize(M);
    g.h_pos.resize(M);
    g.h_off.resize(M);
    g.h_slot.resize((size_t)M * S);
    g.h_refs.resize(R);
    GH(hipMemcpyAsync(g.h_ts.data(), g.g_ts.p, (size_t)M * 8, hipMemcpyDeviceToHost, rl.s));
    GH(hipMemcpyAsync(g.h_type.data(), g.g_type.p, (size_t)M, hipMemcpyDeviceToHost, rl.s));
    GH(hipMemcpyAsync(g.h_pos.data(), g.g_pos.p, (size_t)M * 8, hipMemcpyDeviceToHost, rl.s));
    GH(hipMemcpyAsync(g.h_off.data(), g.g_off.p, (size_t)M * 8, hipMemcpyDeviceToHost, rl.s));
    GH(hipMemcpyAsync(g.h_slot.data(), g.g_slot.p, (size_t)M * S * 2, hipMemcpyDeviceToHost, rl.s));
    GH(hipMemcpyAsync(g.h_refs.data(), g.g_refs.p, (size_t)R * 8, hipMemcpyDeviceToHost, rl.s));
  }
  GH(hipStreamSynchronize(rl.s));
  out->m = M;
  out->key = g.h_key.data();
  if (agg) {
    out->agg = g.h_agg.data();
    return SHP_OK;
  }
  out->ts = g.h_ts.data();
  out->type = g.h_type.data();
  out->pos = g.h_pos.data();
  out->ref_off = g.h_off.data();
  out->slot_len = g.h_slot.data();
  out->refs = g.h_refs.data();
  return SHP_OK;
}

int create_impl(shp_group* g, const char* json, const shp_config* cfg, int world, const int32_t* devices, int rank,
                const void* comm_id) {
  if (world < 1 || world > GS_MAXG) return g->fail(SHP_ERR_ARG, "world must be in [1, 16]");
  g->world = world;
  g->cfg = *cfg;
  g->comp.compile(json);
  const shp::DevProg& P = g->comp.P;
  if (!P.partitioned && world > 1) return g->fail(SHP_ERR_UNSUPPORTED, "only partitioned queries shard by key");
  g->need_clock = P.nsched > 0 && P.playback;  // absent-state timers read the playback clock
  // global sequence numbers travel with the events where the records name events by seq: FULL, and
  // CHAIN32 (its words name batch indices; the expansion on fetch / gather maps them through seq)
  g->need_seq = cfg->match_layout == SHP_LAYOUT_FULL || cfg->match_layout == SHP_LAYOUT_CHAIN32;
  g->has_stream_col = P.nstream > 1;
  g->ncol = P.ncol;
  g->ctag.assign(P.colTag, P.colTag + P.ncol);
  shp_config ec = *cfg;
  ec.max_keys = (int32_t)((cfg->max_keys + world - 1) / world);
  g->nlocal = comm_id ? 1 : world;
  g->rank0 = comm_id ? rank : 0;
  g->L.resize(g->nlocal);
  g->clock = cfg->start_clock;
  for (int i = 0; i < g->nlocal; i++) {
    shp_group::Local& l = g->L[i];
    l.rank = g->rank0 + i;
    l.dev = comm_id ? cfg->device : devices[i];
    ec.device = l.dev;
    GH(hipSetDevice(l.dev));
    GH(hipStreamCreateWithFlags(&l.s, hipStreamNonBlocking));
    GH(hipEventCreateWithFlags(&l.split_done, hipEventDisableTiming));
    for (auto& r : l.slot) GH(hipEventCreateWithFlags(&r.done, hipEventDisableTiming));
    const int rc = shp_engine_create(json, &ec, &l.eng);
    if (rc != SHP_OK) return g->fail(rc, "engine creation failed on rank " + std::to_string(l.rank));
  }
  if (comm_id) {  // (world 1 too: a one-rank communicator runs the same RCCL calls, sends to itself)
    g->rccl = true;
    ncclUniqueId id;
    std::memcpy(&id, comm_id, sizeof id);
    GH(hipSetDevice(g->L[0].dev));
    GN(ncclCommInitRank(&g->comm, world, id, rank));
  }
  return SHP_OK;
}

void destroy_impl(shp_group* g) {
  if (g->comm) (void)ncclCommDestroy(g->comm);
  for (auto& l : g->L) {
    (void)hipSetDevice(l.dev);
    if (l.eng) shp_engine_destroy(l.eng);
    if (l.split_done) (void)hipEventDestroy(l.split_done);
    for (auto& r : l.slot)
      if (r.done) (void)hipEventDestroy(r.done);
    if (l.s) (void)hipStreamDestroy(l.s);
  }
}

template <class F>
int guarded(shp_group* g, F&& f) {
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  int rc;
  try {
    rc = f();
  } catch (shp::CompileError& ce) {
    g->err = ce.what();
    rc = ce.code == -2 ? SHP_ERR_UNSUPPORTED : SHP_ERR_ARG;
  } catch (std::exception& ex) {
    g->err = ex.what();
    rc = SHP_ERR_DEVICE;
  }
  if (prev >= 0) (void)hipSetDevice(prev);
  return rc;
}

}  // namespace

extern "C" {

int shp_comm_id(void* id, size_t len) {
  if (!id || len < sizeof(ncclUniqueId)) return SHP_ERR_ARG;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return SHP_ERR_DEVICE;
  std::memcpy(id, &u, sizeof u);
  return SHP_OK;
}

int shp_group_create(const char* json, const shp_config* cfg, int32_t world, const int32_t* devices,
                     shp_group** out) {
  if (!json || !cfg || !devices || !out) return SHP_ERR_ARG;
  auto* g = new shp_group();
  const int rc = guarded(g, [&]() { return create_impl(g, json, cfg, world, devices, 0, nullptr); });
  if (rc != SHP_OK) {
    fprintf(stderr, "shp_group_create: %s\n", g->err.c_str());
    destroy_impl(g);
    delete g;
    *out = nullptr;
    return rc;
  }
  *out = g;
  return SHP_OK;
}

int shp_group_create_rank(const char* json, const shp_config* cfg, int32_t world, int32_t rank, const void* comm_id,
                          shp_group** out) {
  if (!json || !cfg || !comm_id || !out || rank < 0 || rank >= world) return SHP_ERR_ARG;
  auto* g = new shp_group();
  const int rc = guarded(g, [&]() { return create_impl(g, json, cfg, world, nullptr, rank, comm_id); });
  if (rc != SHP_OK) {
    fprintf(stderr, "shp_group_create_rank: %s\n", g->err.c_str());
    destroy_impl(g);
    delete g;
    *out = nullptr;
    return rc;
  }
  *out = g;
  return SHP_OK;
}

int shp_group_push(shp_group* g, const shp_batch* slices, int64_t* matches) {
  if (!g || !slices) return SHP_ERR_ARG;
  return guarded(g, [&]() {
    if (g->staged != g->ran) return g->fail(SHP_ERR_ARG, "staged batches pending (shp_group_run them first)");
    const int rc = stage_impl(*g, slices);
    return rc != SHP_OK ? rc : run_impl(*g, matches);
  });
}

int shp_group_stage(shp_group* g, const shp_batch* slices) {
  if (!g || !slices) return SHP_ERR_ARG;
  return guarded(g, [&]() { return stage_impl(*g, slices); });
}

int shp_group_run(shp_group* g, int64_t* matches) {
  if (!g) return SHP_ERR_ARG;
  return guarded(g, [&]() { return run_impl(*g, matches); });
}

int shp_group_local_engines(const shp_group* g) { return g ? g->nlocal : 0; }

shp_engine* shp_group_engine(shp_group* g, int32_t i) {
  return (g && i >= 0 && i < g->nlocal) ? g->L[i].eng : nullptr;
}

int shp_group_fetch_matches(shp_group* g, shp_matches* out) {
  if (!g || !out) return SHP_ERR_ARG;
  return guarded(g, [&]() {
    g->h_key.clear();
    g->h_ts.clear();
    g->h_pos.clear();
    g->h_off.clear();
    g->h_refs.clear();
    g->h_type.clear();
    g->h_slot.clear();
    g->h_agg.clear();
    int layout = SHP_LAYOUT_FULL, S = shp_engine_num_states(g->L[0].eng);
    for (auto& l : g->L) {
      shp_matches m{};
      const int rc = shp_fetch_matches(l.eng, &m);
      if (rc != SHP_OK) return g->fail(rc, std::string("rank ") + std::to_string(l.rank) + ": " + shp_last_error(l.eng));
      layout = m.layout;
      for (int64_t i = 0; i < m.m; i++)  // rank-local dense key ids -> the global ones
        g->h_key.push_back((int32_t)((int64_t)m.key[i] * g->world + l.rank));
      if (m.layout == SHP_LAYOUT_AGG) {
        g->h_agg.insert(g->h_agg.end(), m.agg, m.agg + m.m);
        continue;
      }
      const int64_t r0 = (int64_t)g->h_refs.size();
      int64_t nr = 0;
      for (int64_t i = 0; i < m.m * S; i++) nr += m.slot_len[i];
      g->h_ts.insert(g->h_ts.end(), m.ts, m.ts + m.m);
      g->h_pos.insert(g->h_pos.end(), m.pos, m.pos + m.m);
      g->h_type.insert(g->h_type.end(), m.type, m.type + m.m);
      g->h_slot.insert(g->h_slot.end(), m.slot_len, m.slot_len + m.m * S);
      for (int64_t i = 0; i < m.m; i++) g->h_off.push_back(r0 + m.ref_off[i]);
      g->h_refs.insert(g->h_refs.end(), m.refs, m.refs + nr);
    }
    *out = shp_matches{};
    out->m = (int64_t)g->h_key.size();
    out->num_states = S;
    out->layout = layout;
    out->key = g->h_key.data();
    if (layout == SHP_LAYOUT_AGG) {
      out->agg = g->h_agg.data();
      return SHP_OK;
    }
    out->ts = g->h_ts.data();
    out->type = g->h_type.data();
    out->pos = g->h_pos.data();
    out->ref_off = g->h_off.data();
    out->slot_len = g->h_slot.data();
    out->refs = g->h_refs.data();
    return SHP_OK;
  });
}

int shp_group_gather_matches(shp_group* g, int32_t root, shp_matches* out) {
  if (!g || !out) return SHP_ERR_ARG;
  return guarded(g, [&]() { return gather_impl(*g, root, out); });
}

const char* shp_group_last_error(const shp_group* g) { return g ? g->err.c_str() : "null group"; }

void shp_group_destroy(shp_group* g) {
  if (!g) return;
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  destroy_impl(g);
  delete g;
  if (prev >= 0) (void)hipSetDevice(prev);
}
}
