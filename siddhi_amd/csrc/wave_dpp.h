// siddhi-hip: wave-wide inclusive scans over DPP lane moves (round 4).
//
// A Hillis-Steele step through __shfl_up is a ds_bpermute per 32-bit word (the LDS crossbar, one
// LDS round trip of latency each); the same network through DPP moves is plain VALU: row_shr 1, 2,
// 4, 8 inside each row of 16 lanes, then row_bcast:15 (lane 15 of a row into the next row, taken by
// lanes 16-31 and 48-63) and row_bcast:31 (lane 31 into lanes 32-63).  Any associative combine
// works on it -- segmented ones included, (a, fa) then (b, fb) -> (fb ? b : a (+) b, fa | fb).
// GFX9 encodings (gfx950 keeps the row broadcasts that GFX10+ dropped).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace shp {

template <int CTRL>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
  return ((uint64_t)dpp32<CTRL>((uint32_t)(v >> 32)) << 32) | dpp32<CTRL>((uint32_t)v);
}
template <int CTRL>
__device__ __forceinline__ double dppf64(double v) {
  return __longlong_as_double((long long)dpp64<CTRL>((uint64_t)__double_as_longlong(v)));
}

// step(ctrl, take): one scan step; `ctrl` is a std::integral_constant holding the DPP control (use
// decltype(ctrl)::value), `take` whether this lane combines the moved value into its own
template <class Step>
__device__ __forceinline__ void dpp_scan_steps(uint32_t lane, Step&& step) {
  const uint32_t rl = lane & 15u;
  step(std::integral_constant<int, 0x111>{}, rl >= 1);            // row_shr:1
  step(std::integral_constant<int, 0x112>{}, rl >= 2);            // row_shr:2
  step(std::integral_constant<int, 0x114>{}, rl >= 4);            // row_shr:4
  step(std::integral_constant<int, 0x118>{}, rl >= 8);            // row_shr:8
  step(std::integral_constant<int, 0x142>{}, (lane & 31u) >= 16); // row_bcast:15
  step(std::integral_constant<int, 0x143>{}, lane >= 32);         // row_bcast:31
}

// inclusive wave scan of a 32-bit sum
__device__ __forceinline__ uint32_t dpp_incl_add(uint32_t x, uint32_t lane) {
  dpp_scan_steps(lane, [&](auto ctl, bool take) {
    const uint32_t y = dpp32<decltype(ctl)::value>(x);
    if (take) x += y;
  });
  return x;
}

// lane 63's value (an SGPR read; every lane of the wave must be active)
__device__ __forceinline__ uint32_t wave_last(uint32_t x) { return (uint32_t)__builtin_amdgcn_readlane((int)x, 63); }
__device__ __forceinline__ double wave_last_f64(double x) {
  const uint64_t b = (uint64_t)__double_as_longlong(x);
  return __longlong_as_double((long long)(((uint64_t)wave_last((uint32_t)(b >> 32)) << 32) | wave_last((uint32_t)b)));
}

}  // namespace shp
