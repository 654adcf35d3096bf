// Device-side generator of the SURVEY.md §8d synthetic streams (bench/test utility,
// not part of the reference boundary). Bit-identical to siddhi_amd/synth.py:
// PCG32(seed = 0x51DD1 + config, stream 1); per event draws key, price, volume[, stream].
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr uint64_t PCG_MULT = 6364136223846793005ull;
constexpr int64_t T0 = 1544512385000ll;

__host__ __device__ inline void pcg_seed(uint64_t initstate, uint64_t initseq, uint64_t* state, uint64_t* inc) {
  *inc = (initseq << 1u) | 1u;
  *state = 0;
  *state = *state * PCG_MULT + *inc;
  *state += initstate;
  *state = *state * PCG_MULT + *inc;
}

__host__ __device__ inline uint64_t pcg_advance(uint64_t state, uint64_t inc, uint64_t delta) {
  uint64_t acc_mult = 1, acc_plus = 0, cur_mult = PCG_MULT, cur_plus = inc;
  while (delta > 0) {
    if (delta & 1) {
      acc_mult *= cur_mult;
      acc_plus = acc_plus * cur_mult + cur_plus;
    }
    cur_plus = (cur_mult + 1) * cur_plus;
    cur_mult *= cur_mult;
    delta >>= 1;
  }
  return acc_mult * state + acc_plus;
}

__device__ inline uint32_t pcg_next(uint64_t* state, uint64_t inc) {
  uint64_t old = *state;
  *state = old * PCG_MULT + inc;
  uint32_t xorshifted = (uint32_t)(((old >> 18u) ^ old) >> 27u);
  uint32_t rot = (uint32_t)(old >> 59u);
  return (xorshifted >> rot) | (xorshifted << ((-rot) & 31));
}

constexpr int EV_PER_THREAD = 64;

__global__ void k_synth(uint64_t state0, uint64_t inc, int64_t start, int64_t count, int64_t keys, int n_streams,
                        int dense, int64_t* ts, int32_t* key, float* price, int64_t* volume, int32_t* stream) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t first = t * EV_PER_THREAD;
  if (first >= count) return;
  int per = n_streams > 1 ? 4 : 3;
  uint64_t st = pcg_advance(state0, inc, (uint64_t)(start + first) * per);
  int64_t div = keys / 100 > 1 ? keys / 100 : 1;
  for (int64_t j = first; j < first + EV_PER_THREAD && j < count; j++) {
    uint32_t u = pcg_next(&st, inc);
    uint32_t p = pcg_next(&st, inc);
    uint32_t v = pcg_next(&st, inc);
    int32_t s = 0;
    if (per == 4) s = (int32_t)(pcg_next(&st, inc) % (uint32_t)n_streams);
    int64_t i = start + j;
    if (key) key[j] = (int32_t)(u % (uint32_t)keys);
    if (price) price[j] = (float)(p % 10000u) / 100.0f;
    if (volume) volume[j] = (int64_t)(v % 1000u);
    if (stream) stream[j] = s;
    if (ts) ts[j] = dense ? T0 + i : T0 + i / div;
  }
}

}  // namespace

extern "C" int shp_synth_fill(int config, int64_t start, int64_t count, int64_t keys, int n_streams, int dense,
                              int64_t* ts, int32_t* key, float* price, int64_t* volume, int32_t* stream,
                              void* hip_stream) {
  uint64_t st, inc;
  pcg_seed(0x51DD1ull + (uint64_t)config, 1, &st, &inc);
  int64_t threads = (count + EV_PER_THREAD - 1) / EV_PER_THREAD;
  int blocks = (int)((threads + 255) / 256);
  if (blocks < 1) return 0;
  k_synth<<<blocks, 256, 0, (hipStream_t)hip_stream>>>(st, inc, start, count, keys, n_streams, dense, ts, key, price,
                                                       volume, stream);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// Bench/test utilities: device buffers without a second HIP runtime in the process.
extern "C" void* shp_dev_alloc(int64_t bytes) {
  void* p = nullptr;
  return hipMalloc(&p, bytes > 0 ? bytes : 1) == hipSuccess ? p : nullptr;
}
extern "C" int shp_dev_free(void* p) { return hipFree(p) == hipSuccess ? 0 : -5; }
extern "C" int shp_dev_to_host(void* dst, const void* src, int64_t bytes) {
  return hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -5;
}
// Page-locked host memory for match payloads: a D2H copy into it runs at the DMA engine's rate
// instead of through a pageable bounce buffer.  (A Java host would pin its receive segment once
// with shp_host_register, which wraps hipHostRegister.)
extern "C" void* shp_host_alloc(int64_t bytes) {
  void* p = nullptr;
  return hipHostMalloc(&p, bytes > 0 ? bytes : 1, hipHostMallocDefault) == hipSuccess ? p : nullptr;
}
extern "C" int shp_host_free(void* p) { return hipHostFree(p) == hipSuccess ? 0 : -5; }
extern "C" int shp_host_register(void* p, int64_t bytes) {
  return hipHostRegister(p, (size_t)bytes, hipHostRegisterDefault) == hipSuccess ? 0 : -5;
}
extern "C" int shp_host_unregister(void* p) { return hipHostUnregister(p) == hipSuccess ? 0 : -5; }
