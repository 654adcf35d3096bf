// siddhi-hip: the general NFA lanes' kernels (one lane per partition key replays the processor
// chain, nfa_lane.h), a translation unit of their own so the library's units build in parallel.
// engine.hip launches them through lanes_launch / lanes_launch_lds.
#include <hip/hip_runtime.h>

#include "nfa_lane.h"

using namespace shp;

// SHP_LANES_WPE: waves per EU requested from the compiler for the lane kernels (diagnostic A/B:
// fewer VGPRs and more waves to hide the lanes' dependent memory latency, against more spills)
#ifdef SHP_LANES_WPE
#define SHP_LANES_ATTR __attribute__((amdgpu_waves_per_eu(SHP_LANES_WPE, SHP_LANES_WPE)))
#else
#define SHP_LANES_ATTR
#endif

template <int T>
__global__ __launch_bounds__(64) SHP_LANES_ATTR void k_nfa_lanes(const DevProg* __restrict__ Pp, LaneLayout Y, char* arena,
                                                  BatchView B, MatchOut O, const uint32_t* __restrict__ perm,
                                                  const uint32_t* __restrict__ kbeg,
                                                  const uint32_t* __restrict__ kcnt, int32_t nlanes, int* err) {
  int32_t k = blockIdx.x * blockDim.x + threadIdx.x;
#ifdef SHP_LANES_PLDS  // A/B: the program in LDS (the lanes' field reads at LDS latency)
  __shared__ DevProg sP;
  for (int i = threadIdx.x; i < (int)(sizeof(DevProg) / 4); i += blockDim.x)
    ((uint32_t*)&sP)[i] = ((const uint32_t*)Pp)[i];
  __syncthreads();
  if (k >= nlanes) return;
  const DevProg& P = sP;
#else
  if (k >= nlanes) return;
  const DevProg& P = *Pp;
#endif
  LaneT<1, T> ln(P, Y, arena, k, k, B, O);
  if (!B.partitioned && !ln.template at<uint8_t>(Y.o_kinit, 0)) {
    ln.clock = B.init_clock;
    ln.emit_pos = B.seq0;
    ln.init_partition();
  }
  int64_t lo = 0;
  uint32_t b = kbeg[k], e = b + kcnt[k];
  for (uint32_t p = b; p < e && !ln.err; p++) {
    int64_t g = perm[p];
    ln.maybe_gc();
    ln.timers(lo, g);
    ln.on_event(g);
    lo = g + 1;
  }
  if (!ln.err) {
    ln.maybe_gc();
    ln.timers(lo, B.n - 1);
  }
  ln.flush_ret();
  if (ln.err) {
    ln.template at<int32_t>(Y.o_err, 0) |= ln.err;
    atomicOr(err, ln.err);
  }
}

// copy one lane's state between two arena layouts (element i of lane l at field[i * L + l])
__device__ inline void lane_copy(const LaneLayout& Yd, char* dst, int64_t ld, const LaneLayout& Ys, const char* src,
                                 int64_t ls) {
  for (int f = 0; f < Ys.nf; f++) {
    const int sz = Ys.f_sz[f];
    for (int i = 0; i < Ys.f_elems[f]; i++) {
      char* d = dst + Yd.f_off[f] + ((int64_t)i * Yd.L + ld) * sz;
      const char* s = src + Ys.f_off[f] + ((int64_t)i * Ys.L + ls) * sz;
      switch (sz) {
        case 8: *(uint64_t*)d = *(const uint64_t*)s; break;
        case 4: *(uint32_t*)d = *(const uint32_t*)s; break;
        case 2: *(uint16_t*)d = *(const uint16_t*)s; break;
        default: *d = *s; break;
      }
    }
  }
}

#if SHP_LANE_TIER == 0
// Few keys: the lanes' state lives in LDS for the batch (copied in and out of the HBM arena),
// so the per-event chain of dependent state accesses runs at LDS latency instead of HBM
// latency.  Same Lane code, one lane per thread, blockDim lanes per workgroup.
__global__ __launch_bounds__(64) SHP_LANES_ATTR void k_nfa_lanes_lds(const DevProg* __restrict__ Pp, LaneLayout Y,
                                const char* arena, char* arena_out, LaneLayout Yl,
                                BatchView B, MatchOut O, const uint32_t* __restrict__ perm,
                                const uint32_t* __restrict__ kbeg, const uint32_t* __restrict__ kcnt, int32_t nlanes,
                                int* err) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int32_t t = threadIdx.x;
  const int32_t k = blockIdx.x * blockDim.x + t;
  if (k >= nlanes) return;
  lane_copy(Yl, lds, t, Y, (char*)arena, k);
  const DevProg& P = *Pp;
  LaneT<3> ln(P, Yl, lds, t, k, B, O);
  if (!B.partitioned && !ln.at<uint8_t>(Yl.o_kinit, 0)) {
    ln.clock = B.init_clock;
    ln.emit_pos = B.seq0;
    ln.init_partition();
  }
  int64_t lo = 0;
  uint32_t b = kbeg[k], e = b + kcnt[k];
  for (uint32_t p = b; p < e && !ln.err; p++) {
    int64_t g = perm[p];
    ln.maybe_gc();
    ln.timers(lo, g);
    ln.on_event(g);
    lo = g + 1;
  }
  if (!ln.err) {
    ln.maybe_gc();
    ln.timers(lo, B.n - 1);
  }
  ln.flush_ret();
  if (ln.err) {
    ln.at<int32_t>(Yl.o_err, 0) |= ln.err;
    atomicOr(err, ln.err);
  }
  lane_copy(Y, arena_out, k, Yl, lds, t);
}


#endif  // SHP_LANE_TIER == 0

#ifndef SHP_LANE_TIER
#error "lanes.hip is built once per capacity tier (-DSHP_LANE_TIER=0..4)"
#endif
// this unit's tier; tier 0's unit also holds the LDS-resident form
#define LN_FN_(t) lanes_launch_t##t
#define LN_FN(t) LN_FN_(t)
void LN_FN(SHP_LANE_TIER)(unsigned grid, hipStream_t s, const DevProg* P, const LaneLayout& Y, char* arena,
                          const BatchView& B, const MatchOut& O, const uint32_t* perm, const uint32_t* kbeg,
                          const uint32_t* kcnt, int32_t nlanes, int* err) {
  k_nfa_lanes<SHP_LANE_TIER><<<grid, 64, 0, s>>>(P, Y, arena, B, O, perm, kbeg, kcnt, nlanes, err);
}

#if SHP_LANE_TIER == 0
void lanes_launch_lds(unsigned grid, unsigned block, hipStream_t s, const DevProg* P, const LaneLayout& Y,
                      const char* arena, char* arena_out, const LaneLayout& Yl, const BatchView& B, const MatchOut& O,
                      const uint32_t* perm, const uint32_t* kbeg, const uint32_t* kcnt, int32_t nlanes, int* err) {
  k_nfa_lanes_lds<<<grid, block, (size_t)Yl.bytes, s>>>(P, Y, arena, arena_out, Yl, B, O, perm, kbeg, kcnt, nlanes, err);
}
#endif
