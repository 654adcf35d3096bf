// siddhi-hip: key-owner exchange helpers for multi-GPU runs.
// Utilities around the boundary (like synth.hip), not part of the reference interface:
//   shp_shard_partition  stable split of a batch by destination rank (key % G) into packed
//                        16-byte records {ts:int64, stream<<24 | key/G : u32, value:u32},
//                        grouped by destination, arrival order kept within each destination
//   shp_shard_unpack     packed records -> the engine's SoA columns (ts, key, stream, value)
//   shp_shard_partition_soa  the same split into destination-grouped SoA columns: one
//                        all-to-all per column lands the owner's engine input, no unpack pass
// siddhi_amd/shard.py uses the SoA form (one all-to-all per column; RCCL); the packed form
// (one all-to-all of 16-byte records, then an unpack) is kept for the parity test.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <rocprim/rocprim.hpp>

namespace {

constexpr int SH_THREADS = 256;
constexpr int SH_TILE = 65536;  // events per super-tile (one workgroup)
#ifndef SH_ROUND_EVENTS
#define SH_ROUND_EVENTS 2048
#endif
constexpr int SH_ROUND = SH_ROUND_EVENTS;
constexpr int SH_SUB = SH_ROUND / SH_THREADS;
constexpr int SH_MAXG = 16;

struct __attribute__((aligned(16))) ShRec {
  int64_t ts;
  uint32_t key;  // packed form: stream << 24 | key / G; SoA form: key / G (full 32 bits)
  uint32_t v;
};

__global__ __launch_bounds__(SH_THREADS) void k_shard_count(const int32_t* __restrict__ key, int64_t n, int G,
                                                            int ntiles, uint32_t* cnt) {
  __shared__ uint32_t h[SH_MAXG];
  if (threadIdx.x < SH_MAXG) h[threadIdx.x] = 0;
  __syncthreads();
  const int t = blockIdx.x;
  const int64_t lo = (int64_t)t * SH_TILE, hi = min(n, lo + SH_TILE);
  uint32_t c[SH_MAXG] = {};
  for (int64_t i = lo + threadIdx.x; i < hi; i += SH_THREADS) {
    const uint32_t d = (uint32_t)key[i] % (uint32_t)G;
#pragma unroll
    for (int g = 0; g < SH_MAXG; g++) c[g] += d == (uint32_t)g ? 1u : 0u;
  }
  for (int g = 0; g < G; g++) atomicAdd(&h[g], c[g]);
  __syncthreads();
  if (threadIdx.x < G) cnt[(int64_t)threadIdx.x * ntiles + t] = h[threadIdx.x];
  if (t == 0 && threadIdx.x == 0) cnt[(int64_t)G * ntiles] = 0;
}

// SoA destination columns (shp_shard_partition_soa): the received buffers of one all-to-all
// per column are the engine's input columns as they stand, with no unpack pass
struct ShSoa {
  int64_t* ts;
  int32_t* key;
  uint32_t* val;
  int32_t* stream;
};

// Per round of SH_ROUND events: rank by destination (wave ballots), stage the records in LDS
// grouped by destination, then write each destination's run with consecutive lanes on
// consecutive addresses (full-line stores, not 8-way scattered ones).
template <bool SOA>
__global__ __launch_bounds__(SH_THREADS) void k_shard_scatter(const int64_t* __restrict__ ts,
                                                              const int32_t* __restrict__ key,
                                                              const uint32_t* __restrict__ val,
                                                              const int32_t* __restrict__ stream, int64_t n, int G,
                                                              int gbits, int ntiles, const uint32_t* __restrict__ off,
                                                              ShRec* out, ShSoa so) {
  constexpr int NW = SH_THREADS / 64;
  __shared__ uint32_t wc[NW][SH_MAXG];   // per-wave counts, then the wave's LDS slot base
  __shared__ uint32_t run[SH_MAXG];      // next global position per destination
  __shared__ uint32_t gst[SH_MAXG];      // this round's global start per destination
  __shared__ uint32_t lst[SH_MAXG + 1];  // this round's LDS start per destination
  __shared__ ShRec srec[SH_ROUND];
  __shared__ uint8_t sdst[SH_ROUND];
  __shared__ int32_t sstp[SOA ? SH_ROUND : 1];   // SoA: stream id by destination-grouped slot
  const int t = blockIdx.x;
  const uint32_t lane = __lane_id(), w = threadIdx.x >> 6;
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  if (threadIdx.x < G) run[threadIdx.x] = off[(int64_t)threadIdx.x * ntiles + t];
  const int64_t lo = (int64_t)t * SH_TILE, hi = min(n, lo + SH_TILE);
  for (int64_t r0 = lo; r0 < hi; r0 += SH_ROUND) {
    if (threadIdx.x < NW * SH_MAXG) (&wc[0][0])[threadIdx.x] = 0;
    __syncthreads();
    ShRec rec[SH_SUB];
    uint32_t dst[SH_SUB], rk[SH_SUB];
    int32_t sid[SH_SUB];
#pragma unroll
    for (int s = 0; s < SH_SUB; s++) {  // wave w owns items [w*SEG, (w+1)*SEG) of the round
      const int64_t i = r0 + (int64_t)w * (SH_ROUND / NW) + s * 64 + lane;
      if (i < hi) {
        const uint32_t k = (uint32_t)key[i];
        rec[s].ts = ts[i];
        // the SoA form carries the stream id in its own LDS column (no 24-bit packing)
        rec[s].key = SOA ? k / (uint32_t)G : (k / (uint32_t)G) | (stream ? ((uint32_t)stream[i] << 24) : 0u);
        rec[s].v = val ? val[i] : 0u;
        sid[s] = (SOA && stream) ? stream[i] : 0;
        dst[s] = k % (uint32_t)G;
      } else {
        dst[s] = SH_MAXG;
      }
    }
#pragma unroll
    for (int s = 0; s < SH_SUB; s++) {
      const bool valid = dst[s] < SH_MAXG;
      uint64_t peers = __ballot(valid);
      for (int b = 0; b < gbits; b++) {
        const bool bit = (dst[s] >> b) & 1u;
        const uint64_t m = __ballot(bit);
        peers &= bit ? m : ~m;
      }
      uint32_t before = valid ? wc[w][dst[s]] : 0u;
      rk[s] = before + (uint32_t)__popcll(peers & lt);
      if (valid && (peers & lt) == 0) wc[w][dst[s]] = before + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // G <= 16 destinations x NW waves: one thread
      uint32_t l = 0;
      for (int d = 0; d < G; d++) {
        lst[d] = l;
        gst[d] = run[d];
        for (int ww = 0; ww < NW; ww++) {
          const uint32_t c = wc[ww][d];
          wc[ww][d] = l;
          l += c;
        }
        run[d] += l - lst[d];
      }
      lst[G] = l;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < SH_SUB; s++) {
      if (dst[s] >= SH_MAXG) continue;
      const uint32_t slot = wc[w][dst[s]] + rk[s];
      srec[slot] = rec[s];
      sdst[slot] = (uint8_t)dst[s];
      if (SOA && stream) sstp[slot] = sid[s];
    }
    __syncthreads();
    const int nv = (int)lst[G];
    for (int x = threadIdx.x; x < nv; x += SH_THREADS) {
      const uint32_t d = sdst[x];
      const uint32_t o = gst[d] + ((uint32_t)x - lst[d]);
      const ShRec r = srec[x];
      if constexpr (SOA) {
        so.ts[o] = r.ts;
        so.key[o] = (int32_t)r.key;
        if (so.stream) so.stream[o] = sstp[x];
        if (so.val) so.val[o] = r.v;
      } else {
        out[o] = r;
      }
    }
    __syncthreads();
  }
}

__global__ void k_shard_check(const int32_t* __restrict__ key, const int32_t* __restrict__ stream, int64_t n, int G,
                              int* bad) {
  int b = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if ((uint32_t)key[i] / (uint32_t)G >= (1u << 24)) b = 1;
    if (stream && (stream[i] < 0 || stream[i] > 255)) b = 1;
  }
  if (b) atomicOr(bad, 1);
}

__global__ void k_shard_unpack(const ShRec* __restrict__ in, int64_t m, int64_t* ts, int32_t* key, uint32_t* val,
                               int32_t* stream) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    const ShRec r = in[i];
    ts[i] = r.ts;
    key[i] = (int32_t)(r.key & 0xffffffu);
    if (stream) stream[i] = (int32_t)(r.key >> 24);
    if (val) val[i] = r.v;
  }
}

}  // namespace

static size_t scan_bytes(size_t nc) {
  size_t tb = 0;
  (void)rocprim::exclusive_scan(nullptr, tb, (uint32_t*)nullptr, (uint32_t*)nullptr, 0u, nc,
                                rocprim::plus<uint32_t>(), (hipStream_t)0);
  return tb;
}

// device workspace bytes shp_shard_partition needs for n events over G ranks
extern "C" int64_t shp_shard_workspace_bytes(int64_t n, int G) {
  const size_t ntiles = (size_t)((n + SH_TILE - 1) / SH_TILE);
  const size_t nc = (size_t)G * ntiles + 1;
  return (int64_t)(2 * ((nc * 4 + 255) / 256 * 256) + scan_bytes(nc) + 256);
}

// n events (device SoA) -> out: n packed records grouped by destination rank key % G (stable);
// counts[g] (host) = records for rank g.  Packed form: keys must be < 2^24 * G and stream ids in
// [0, 255] (shp_shard_partition checks both); the SoA form carries full 32-bit keys and streams.
// ws: device workspace of shp_shard_workspace_bytes(n, G) bytes.
static int shard_partition(int64_t n, const int64_t* ts, const int32_t* key, const void* value,
                           const int32_t* stream, int G, void* out, const ShSoa* so, int64_t* counts, void* ws,
                           void* hip_stream) {
  if (G < 1 || G > SH_MAXG || n < 0 || !ws) return -1;
  hipStream_t s = (hipStream_t)hip_stream;
  const int ntiles = (int)((n + SH_TILE - 1) / SH_TILE);
  const size_t nc = (size_t)G * ntiles + 1;
  const size_t cb = (nc * 4 + 255) / 256 * 256;
  uint32_t* cnt = (uint32_t*)ws;
  uint32_t* off = (uint32_t*)((char*)ws + cb);
  void* tmp = (char*)ws + 2 * cb;
  size_t tb = scan_bytes(nc);
  if (ntiles == 0) {
    for (int g = 0; g < G; g++) counts[g] = 0;
    return 0;
  }
  int gbits = 0;
  while ((1 << gbits) < G) gbits++;
  k_shard_count<<<ntiles, SH_THREADS, 0, s>>>(key, n, G, ntiles, cnt);
  if (rocprim::exclusive_scan(tmp, tb, cnt, off, 0u, nc, rocprim::plus<uint32_t>(), s) != hipSuccess) return -5;
  if (so)
    k_shard_scatter<true><<<ntiles, SH_THREADS, 0, s>>>(ts, key, (const uint32_t*)value, stream, n, G, gbits, ntiles,
                                                        off, nullptr, *so);
  else
    k_shard_scatter<false><<<ntiles, SH_THREADS, 0, s>>>(ts, key, (const uint32_t*)value, stream, n, G, gbits, ntiles,
                                                         off, (ShRec*)out, ShSoa{});
  uint32_t h[SH_MAXG + 1];
  for (int g = 0; g <= G; g++)
    if (hipMemcpyAsync(&h[g], off + (size_t)g * ntiles, 4, hipMemcpyDeviceToHost, s) != hipSuccess) return -5;
  if (hipStreamSynchronize(s) != hipSuccess || hipGetLastError() != hipSuccess) return -5;
  for (int g = 0; g < G; g++) counts[g] = (int64_t)h[g + 1] - h[g];
  return 0;
}

extern "C" int shp_shard_partition(int64_t n, const int64_t* ts, const int32_t* key, const void* value,
                                   const int32_t* stream, int G, void* out, int64_t* counts, void* ws,
                                   void* hip_stream) {
  if (!out && n > 0) return -1;
  if (n > 0 && G >= 1 && G <= SH_MAXG) {  // the packed record's limits: key / G < 2^24, stream in [0, 255]
    int* bad = (int*)((char*)ws + shp_shard_workspace_bytes(n, G) - 256);
    hipStream_t s = (hipStream_t)hip_stream;
    if (hipMemsetAsync(bad, 0, 4, s) != hipSuccess) return -5;
    int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
    k_shard_check<<<blocks, 256, 0, s>>>(key, stream, n, G, bad);
    int hb = 0;
    if (hipMemcpyAsync(&hb, bad, 4, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
      return -5;
    if (hb) return -1;
  }
  return shard_partition(n, ts, key, value, stream, G, out, nullptr, counts, ws, hip_stream);
}

// The same stable split into destination-grouped SoA columns: out_ts/out_key(key / G)/out_value
// (NULL when value is NULL)/out_stream (NULL when stream is NULL), each of n elements.  One
// all-to-all per column then delivers the owner's engine input directly (no unpack).
extern "C" int shp_shard_partition_soa(int64_t n, const int64_t* ts, const int32_t* key, const void* value,
                                       const int32_t* stream, int G, int64_t* out_ts, int32_t* out_key,
                                       void* out_value, int32_t* out_stream, int64_t* counts, void* ws,
                                       void* hip_stream) {
  if (n > 0 && (!out_ts || !out_key || (value && !out_value) || (stream && !out_stream))) return -1;
  const ShSoa so{out_ts, out_key, value ? (uint32_t*)out_value : nullptr, stream ? out_stream : nullptr};
  return shard_partition(n, ts, key, value, stream, G, nullptr, &so, counts, ws, hip_stream);
}

extern "C" int shp_shard_unpack(int64_t m, const void* in, int64_t* ts, int32_t* key, void* value, int32_t* stream,
                                void* hip_stream) {
  if (m <= 0) return 0;
  int blocks = (int)((m + 255) / 256);
  if (blocks > 8192) blocks = 8192;
  k_shard_unpack<<<blocks, 256, 0, (hipStream_t)hip_stream>>>((const ShRec*)in, m, ts, key, (uint32_t*)value, stream);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
