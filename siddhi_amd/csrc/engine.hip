// siddhi-hip engine: libsiddhi_hip.so (gfx950).
//
// Per push (shp_push_batch / shp_push_batch_device):
//   1. clock:     rmax = inclusive max-scan of ts seeded with the carried clock
//                 (TimestampGeneratorImpl.setCurrentTimestamp, playback)
//   2. partition: stable radix sort of (key, seq) -> perm; per-key [kbeg, kbeg+kcnt)
//                 (PartitionStreamReceiver routes each event to its key's state, and a
//                 key's events keep arrival order)
//   3a. general:  k_nfa_lanes — one lane per key replays the processor chain (nfa_lane.h)
//   3b. fast:     k_fast_* — the closed form of `every e1=S[f1] -> e2=S[f2] within W`
//                 (fastpath.h), chosen at create time when the program has that shape
//   4. matches are appended to an HBM match table; host pushes copy them back.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <memory>
#include <numeric>
#include <rocprim/rocprim.hpp>
#include <string>
#include <vector>

#include "../../include/siddhi_hip.h"
#include "compile.h"
#include "fastpath.h"
#include "nfa_lane.h"
#include "sweep.h"
#include "cseq.h"
#include "labs.h"

using namespace shp;

#define HIP_OK(x)                                                                          \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) throw DevError(std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

struct DevError : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct OutputError : std::runtime_error {  // a capacity found short after the push (SHP_ERR_OUTPUT)
  using std::runtime_error::runtime_error;
};

// ---------------------------------------------------------------- kernels
__global__ void k_iota(uint32_t* v, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (int64_t)gridDim.x * blockDim.x) v[i] = (uint32_t)i;
}

// per-key event counts.  Up to KEY_HIST_LDS keys the block counts in LDS and adds its nonzero
// bins once (few keys would otherwise serialise every event on one global atomic: C1 has one)
constexpr int KEY_HIST_LDS = 8192;
__global__ void k_key_hist(const int32_t* key, const int32_t* stream, int64_t n, uint32_t* cnt, int32_t max_keys,
                           int partitioned, int* err) {
  extern __shared__ uint32_t h[];
  const bool lds = max_keys <= KEY_HIST_LDS;
  if (lds) {
    for (int b = threadIdx.x; b < max_keys; b += blockDim.x) h[b] = 0;
    __syncthreads();
  }
  int e = 0;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int32_t k = partitioned ? key[i] : 0;
    if (stream[i] < 0) continue;  // clock-only event (advance)
    if (k < 0 || k >= max_keys) {
      e = 1 << 20;
      continue;
    }
    if (lds) atomicAdd(&h[k], 1u);
    else atomicAdd(&cnt[k], 1u);
  }
  if (e) atomicOr(err, e);
  if (lds) {
    __syncthreads();
    for (int b = threadIdx.x; b < max_keys; b += blockDim.x)
      if (h[b]) atomicAdd(&cnt[b], h[b]);
  }
}

__global__ void k_sort_keys(const int32_t* key, const int32_t* stream, int64_t n, uint32_t* out, int partitioned,
                            uint32_t nokey) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = stream[i] < 0 ? nokey : (partitioned ? (uint32_t)key[i] : 0u);
}

// the same sort key with the key range checked here (paths without k_key_hist): invalid keys
// sort past every valid one and fail the push
__global__ void k_sort_keys_chk(const int32_t* key, const int32_t* stream, int64_t n, uint32_t* out, int partitioned,
                                uint32_t nokey, int* err) {
  int e = 0;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t k = 0;
    if (stream[i] < 0) {
      k = nokey;
    } else if (partitioned) {
      const int32_t x = key[i];
      if (x < 0 || (uint32_t)x >= nokey) {
        e = 1 << 20;
        k = nokey;
      } else {
        k = (uint32_t)x;
      }
    }
    out[i] = k;
  }
  if (e) atomicOr(err, e);
}

// each key's run in the key-sorted batch: kbeg = its first position, kcnt = its length (a key
// without events starts where it would: kbeg = lower bound, kcnt = 0, so per-key output regions
// derived from kbeg -- the logical-absent path -- stay disjoint).  One thread per key, two binary
// searches over the sorted keys: a push touching few keys of a large key range costs O(keys log n),
// not a serial fill of the missing keys' bounds by the threads at key boundaries.
__device__ __forceinline__ uint32_t key_lower_bound(const uint32_t* __restrict__ sk, int64_t n, uint32_t k) {
  int64_t a = 0, b = n;
  while (a < b) {
    const int64_t m = a + ((b - a) >> 1);
    if (sk[m] < k) a = m + 1;
    else b = m;
  }
  return (uint32_t)a;
}
__global__ void k_key_bounds(const uint32_t* __restrict__ sk, int64_t n, uint32_t* kbeg, uint32_t* kcnt, uint32_t nk) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nk) return;
  const uint32_t a = key_lower_bound(sk, n, (uint32_t)k), b = key_lower_bound(sk, n, (uint32_t)k + 1u);
  kbeg[k] = a;
  kcnt[k] = b - a;
}

__global__ void k_clamp_clock(int64_t* rmax, int64_t n, int64_t clock0) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (rmax[i] < clock0) rmax[i] = clock0;
}

// shp_stage_batch_ts32: the narrow ingest form (4-byte ts offsets from the batch's base) widened
// in HBM before the run -- 4 B read + 8 B written per event, against 4 B saved on the host link
__global__ void k_widen_ts(const int32_t* __restrict__ d, int64_t base, int64_t* __restrict__ ts, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (int64_t)gridDim.x * blockDim.x) ts[i] = base + d[i];
}

// shp_stage_batch_narrow: 2-byte key ids (max_keys <= 65536) widened in HBM
__global__ void k_widen_key(const uint16_t* __restrict__ d, int32_t* __restrict__ key, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (int64_t)gridDim.x * blockDim.x) key[i] = (int32_t)d[i];
}

// Capacity growth: the committed arena of layout Ys (tier t) into layout Yd (tier >= t), every
// lane.  Fields keep their order and element sizes across tiers; element indices that embed a
// capacity are re-indexed: list items ((which * MAXP + p) * LCAP + i) and the timer rings
// (s * QCAP + (head + i) % QCAP, linearised so the new head is 0).  The new arena is zeroed first
// (free pool bits, empty lists).
__global__ __launch_bounds__(256) void k_lane_migrate(LaneLayout Yd, char* dst, LaneLayout Ys, const char* src) {
  const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= Ys.L) return;
  auto sp = [&](int64_t off, int64_t i, int sz) { return src + off + (i * Ys.L + l) * sz; };
  auto dp = [&](int64_t off, int64_t i, int sz) { return dst + off + (i * Yd.L + l) * sz; };
  auto cp = [&](char* d, const char* s_, int sz) {
    for (int b = 0; b < sz; b++) d[b] = s_[b];
  };
  for (int f = 0; f < Ys.nf; f++) {
    const int64_t so = Ys.f_off[f], d_o = Yd.f_off[f];
    const int sz = Ys.f_sz[f];
    if (so == Ys.o_lst) {
      for (int li = 0; li < 2 * MAXP; li++)
        for (int i = 0; i < Ys.lcap; i++) cp(dp(d_o, (int64_t)li * Yd.lcap + i, sz), sp(so, (int64_t)li * Ys.lcap + i, sz), sz);
    } else if (so == Ys.o_q) {
      for (int q = 0; q < MAXQ; q++) {
        const int16_t h = *(const int16_t*)sp(Ys.o_qhead, q, 2), n = *(const int16_t*)sp(Ys.o_qlen, q, 2);
        for (int i = 0; i < n; i++)
          cp(dp(d_o, (int64_t)q * Yd.qcap + i, sz), sp(so, (int64_t)q * Ys.qcap + (h + i) % Ys.qcap, sz), sz);
      }
    } else if (so == Ys.o_qhead) {
      for (int q = 0; q < MAXQ; q++) *(int16_t*)dp(d_o, q, 2) = 0;
    } else {
      for (int i = 0; i < Ys.f_elems[f]; i++) cp(dp(d_o, i, sz), sp(so, i, sz), sz);
    }
  }
}

// the general lanes' kernels (k_nfa_lanes<tier>, k_nfa_lanes_lds) live in lanes.hip, a unit of
// their own (the library's units build in parallel)
#define LN_DECL(t)                                                                                        \
  void lanes_launch_t##t(unsigned grid, hipStream_t s, const DevProg* P, const LaneLayout& Y, char* arena,   \
                         const BatchView& B, const MatchOut& O, const uint32_t* perm, const uint32_t* kbeg, \
                         const uint32_t* kcnt, int32_t nlanes, int* err);
LN_DECL(0)
LN_DECL(1)
LN_DECL(2)
LN_DECL(3)
LN_DECL(4)
#undef LN_DECL
static void lanes_launch(int tier, unsigned grid, hipStream_t s, const DevProg* P, const LaneLayout& Y, char* arena,
                         const BatchView& B, const MatchOut& O, const uint32_t* perm, const uint32_t* kbeg,
                         const uint32_t* kcnt, int32_t nlanes, int* err) {
  static_assert(LANE_TIERS == 5, "one lanes unit per tier");
  switch (tier) {
    case 0: lanes_launch_t0(grid, s, P, Y, arena, B, O, perm, kbeg, kcnt, nlanes, err); break;
    case 1: lanes_launch_t1(grid, s, P, Y, arena, B, O, perm, kbeg, kcnt, nlanes, err); break;
    case 2: lanes_launch_t2(grid, s, P, Y, arena, B, O, perm, kbeg, kcnt, nlanes, err); break;
    case 3: lanes_launch_t3(grid, s, P, Y, arena, B, O, perm, kbeg, kcnt, nlanes, err); break;
    default: lanes_launch_t4(grid, s, P, Y, arena, B, O, perm, kbeg, kcnt, nlanes, err); break;
  }
}
void lanes_launch_lds(unsigned grid, unsigned block, hipStream_t s, const DevProg* P, const LaneLayout& Y,
                      const char* arena, char* arena_out, const LaneLayout& Yl, const BatchView& B, const MatchOut& O,
                      const uint32_t* perm, const uint32_t* kbeg, const uint32_t* kcnt, int32_t nlanes, int* err);

// ---------------------------------------------------------------- engine
constexpr int32_t SWEEP_MIN_KEYS = 256;
constexpr int32_t LDS_LANES_MAX_KEYS = 8192;  // general lanes with state in LDS up to this many keys

struct shp_engine {
  KTimer kt;
  ProgramCompiler comp;
  DevProg* dprog = nullptr;
  shp_config cfg{};
  LaneLayout Y{};
  // general lanes: the committed arena and the one a push writes (the committed state copied in
  // first); the push swaps them only when it succeeded
  char* arena = nullptr;
  char* arena2 = nullptr;
  int tier = 0;  // LaneCaps tier of Y
  int fast = 0;   // 1: specialised scan kernels (fastpath.h), 2: sweep (sweep.h), 3: count sequence (cseq.h)
  FastState fs{};
  SweepState sw{};
  CseqState cs{};
  LabsState la{};
  bool expanded = true;  // sweep matches materialised as full records
  BatchView lastB{};
  const int32_t* lastKey = nullptr;
  const int32_t* lastStream = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
  std::string err;

  // batch buffers
  int64_t cap = 0;
  int64_t* d_ts = nullptr;
  int64_t *d_clk = nullptr, *d_seq = nullptr;  // staged optional columns (host pushes)
  int32_t* d_key = nullptr;
  int32_t* d_stream = nullptr;
  void* d_cols[MAXCOL] = {};
  uint8_t* d_nulls[MAXCOL] = {};
  bool staged_null[MAXCOL] = {};  // the last staged (host) push carried a null bitmap for column c
  int64_t* d_rmax = nullptr;
  uint32_t *d_skey = nullptr, *d_skey2 = nullptr, *d_idx = nullptr, *d_perm = nullptr;
  uint32_t *d_kcnt = nullptr, *d_kbeg = nullptr;
  void* d_tmp = nullptr;
  size_t tmp_bytes = 0;
  int* d_err = nullptr;  // = d_status + 2
  // per-push status block on the device (match counts [0..1], error bits [2]) and its
  // page-locked host mirror (+ the engine clock [3]): one memset and two small DMA reads per push
  unsigned long long* d_status = nullptr;
  unsigned long long* h_status = nullptr;
  // match table
  int64_t mcap = 0, rcap = 0;
  unsigned long long* d_mcount = nullptr;  // = d_status
  int32_t* d_mkey = nullptr;
  int64_t *d_mts = nullptr, *d_mpos = nullptr, *d_moff = nullptr, *d_refs = nullptr;
  int8_t* d_mtype = nullptr;
  int16_t* d_mslot = nullptr;
  double* d_magg = nullptr;
  std::vector<double> h_agg;
  // host copies
  std::vector<int32_t> h_key;
  std::vector<int64_t> h_ts, h_pos, h_off, h_refs;
  std::vector<int8_t> h_type;
  std::vector<int16_t> h_slot;
  int64_t h_m = 0;
  // run state
  int64_t seq = 0;
  int64_t clock = 0;
  int key_bits = 1;
  const bool cseq_v1 = getenv("SHP_CSEQ_V1") != nullptr;  // A/B: the round-2 count-sequence kernels
  const bool cseq_wide = getenv("SHP_CSEQ_WIDE") != nullptr;  // A/B: the 16-byte records on every push
  int64_t cseq_wide_reruns = 0;
  const bool labs_v1 = getenv("SHP_LABS_V1") != nullptr;  // A/B: logical-absent batch by key sort + gather
  LaneLayout Yl{};     // per-workgroup LDS layout of the lanes (lds_lanes > 0)
  int lds_lanes = 0;
  double last_ms_part = 0, last_ms_nfa = 0, last_ms_total = 0;
  int64_t last_m = 0;
  int64_t pushes = 0, lean_pushes = 0, lean_fallbacks = 0, labs_fallbacks = 0, labs_segmiss = 0;  // shp_engine_stat
  int64_t win_pushes = 0, win_fallbacks = 0, r16_reruns = 0;
  int64_t spill_reruns = 0;

  // ---- pipelined host ingest (shp_stage_batch / shp_run_staged): two device slots
  // filled from host columns on a copy stream while the compute stream runs the previous batch, and
  // the compact records copied back into page-locked memory.  Allocated at the first stage.
  struct Slot {
    int64_t n = 0;
    int64_t* ts = nullptr;
    int32_t* ts32 = nullptr;  // shp_stage_batch_ts32: ts = ts_base + ts32[i], widened on the device
    uint16_t* k16 = nullptr;  // shp_stage_batch_narrow: 2-byte key ids, widened on the device
    int64_t ts_base = 0;
    bool narrow = false, nkey = false;
    int32_t* key = nullptr;
    int32_t* strm = nullptr;
    int64_t *clk = nullptr, *sq = nullptr;
    void* cols[MAXCOL] = {};
    uint8_t* nulls[MAXCOL] = {};
    bool has_stream = false, has_clk = false, has_seq = false, has_null[MAXCOL] = {};
    hipEvent_t ready = nullptr;     // its H2D copies are done (copy stream)
    hipEvent_t consumed = nullptr;  // the run that read it is done (compute stream)
  };
  Slot slots[2];
  int slot_head = 0, slot_count = 0;
  bool slots_ready = false;
  hipStream_t cstream = nullptr;
  uint32_t* h_wpin = nullptr;  // page-locked compact records of the last shp_run_staged
  int64_t h_wpin_words = 0;

  ~shp_engine() { release(); }

  void release() {
    auto F = [](void* p) {
      if (p) (void)hipFree(p);
    };
    F(dprog);
    F(arena);
    F(arena2);
    F(d_ts);
    F(d_clk);
    F(d_seq);
    F(d_key);
    F(d_stream);
    for (int c = 0; c < MAXCOL; c++) {
      F(d_cols[c]);
      F(d_nulls[c]);
    }
    F(d_rmax);
    F(d_skey);
    F(d_skey2);
    F(d_idx);
    F(d_perm);
    F(d_kcnt);
    F(d_kbeg);
    F(d_tmp);
    F(d_status);
    if (h_status) (void)hipHostFree(h_status);
    F(d_mkey);
    F(d_mts);
    F(d_mpos);
    F(d_moff);
    F(d_refs);
    F(d_mtype);
    F(d_mslot);
    F(d_magg);
    fs.release();
    sw.release();
    cs.release();
    la.release();
    kt.release();
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
    if (ev2) (void)hipEventDestroy(ev2);
    for (Slot& sl : slots) {
      F(sl.ts);
      F(sl.ts32);
      F(sl.k16);
      F(sl.key);
      F(sl.strm);
      F(sl.clk);
      F(sl.sq);
      for (int c = 0; c < MAXCOL; c++) {
        F(sl.cols[c]);
        F(sl.nulls[c]);
      }
      if (sl.ready) (void)hipEventDestroy(sl.ready);
      if (sl.consumed) (void)hipEventDestroy(sl.consumed);
    }
    if (h_wpin) (void)hipHostFree(h_wpin);
    if (cstream) (void)hipStreamDestroy(cstream);
    if (stream) (void)hipStreamDestroy(stream);
  }

  template <class T>
  void alloc(T*& p, int64_t elems) {
    HIP_OK(hipMalloc((void**)&p, std::max<int64_t>(elems, 1) * sizeof(T)));
  }

  static int colBytes(int8_t tag) {
    switch (tag) {
      case T_LONG:
      case T_DOUBLE: return 8;
      case T_BOOL: return 1;
      default: return 4;
    }
  }

  void create(const char* json, const shp_config* c) {
    cfg = *c;
    if (cfg.max_keys < 1) cfg.max_keys = 1;
    if (cfg.max_batch < 1) cfg.max_batch = 1 << 16;
    if (cfg.max_matches < 1) cfg.max_matches = std::max<int64_t>(cfg.max_batch, 1 << 16);
    comp.compile(json);
    program = json;
    if (!comp.P.partitioned) cfg.max_keys = 1;
    HIP_OK(hipSetDevice(cfg.device));
    HIP_OK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    HIP_OK(hipEventCreate(&ev0));
    HIP_OK(hipEventCreate(&ev1));
    HIP_OK(hipEventCreate(&ev2));
    alloc(dprog, 1);
    HIP_OK(hipMemcpy(dprog, &comp.P, sizeof(DevProg), hipMemcpyHostToDevice));
    clock = cfg.start_clock;
    while ((1ll << key_bits) <= cfg.max_keys) key_bits++;  // + one sentinel key for clock-only events
    fast = comp.fast.ok && cfg.force_general != 1;
    int32_t nown = 0;
    std::vector<uint32_t> kmap;
    // the sweep needs enough keys to spread over workgroups (one owner region is sequential);
    // below SWEEP_MIN_KEYS the scan kernels are parallel over candidates instead
    const bool want_sweep = cfg.force_general == 3 || (cfg.force_general == 0 && cfg.max_keys >= SWEEP_MIN_KEYS);
    if (fast && want_sweep && SweepState::shape_ok(comp.P, comp.fast) &&
        SweepState::build_map(cfg.max_keys, nown, kmap))
      fast = 2;
    if (!fast && cfg.force_general != 1 && CseqState::shape_ok(comp.P, comp.cseq) &&
        !(cseq_v1 && CseqState::mode_of(comp.cseq) != CS_EVERY1))  // (the round-2 kernels: every, min 1)
      fast = 3;
    // the logical-absent automaton (labs.h): exact for any timestamp order, the default for its shape
    if (!fast && cfg.force_general == 4 && !LabsState::shape_ok(comp.P, comp.labs))
      throw CompileError(-2, "force_general 4: the query is not `every (x=X and y=Y) -> not Z for T` in playback");
    if (!fast && (cfg.force_general == 0 || cfg.force_general == 4) && LabsState::shape_ok(comp.P, comp.labs) &&
        !getenv("SHP_NO_LABS"))
      fast = 4;
    if (cfg.match_layout == SHP_LAYOUT_COMPACT)  // the path's own compact form (a host that decodes all)
      cfg.match_layout = fast == 2 ? SHP_LAYOUT_PAIRS32
                                   : (fast == 3 && !cseq_v1 && cfg.max_batch <= (int64_t)CH32_G ? SHP_LAYOUT_CHAIN32
                                                                                                 : SHP_LAYOUT_FULL);
    if ((cfg.match_layout == SHP_LAYOUT_PAIRS || cfg.match_layout == SHP_LAYOUT_PAIRS32) && fast != 2)
      throw CompileError(-2, "match_layout PAIRS / PAIRS32 needs the sweep path");
    if (cfg.match_layout == SHP_LAYOUT_CHAIN32) {
      if (fast != 3 || cseq_v1) throw CompileError(-2, "match_layout CHAIN32 needs the count-sequence path");
      if (cfg.max_batch > (int64_t)CH32_G) throw CompileError(-1, "match_layout CHAIN32: max_batch must be below 2^28");
    }
    if (cfg.match_layout == SHP_LAYOUT_AGG) {
      // the sweep folds an aggregate of e2's value (its single predicate column; count: none);
      // the general lanes fold one over any state's column at emission (nfa_lane.h aggregate()),
      // so every other shape -- the count-sequence and logical-absent ones included -- runs its
      // aggregate there
      if (!comp.agg_fn) throw CompileError(-2, "match_layout AGG: the query's select has no device aggregate");
      const bool arg_ok = comp.agg_fn == 3 || (comp.agg_state >= 0 && comp.agg_state < comp.P.nstates &&
                                               comp.agg_col >= 0 && comp.agg_col < comp.P.ncol);
      if (!arg_ok) throw CompileError(-2, "match_layout AGG: the aggregate's argument is not a state's column");
      const bool sweep_ok = comp.agg_fn == 3 || (comp.agg_state == 1 && comp.agg_col == 0 && comp.P.ncol == 1);
      if (fast != 2 || !sweep_ok) fast = 0;
    } else if (cfg.match_layout != SHP_LAYOUT_FULL && cfg.match_layout != SHP_LAYOUT_PAIRS &&
               cfg.match_layout != SHP_LAYOUT_PAIRS32 && cfg.match_layout != SHP_LAYOUT_CHAIN32) {
      throw CompileError(-1, "unknown match_layout");
    }
    kt.enabled = cfg.profile_kernels != 0;
    cap = cfg.max_batch + 1;
    alloc(d_ts, cap);
    alloc(d_clk, cap);
    alloc(d_seq, cap);
    alloc(d_key, cap);
    alloc(d_stream, cap);
    for (int i = 0; i < comp.P.ncol; i++) {
      HIP_OK(hipMalloc(&d_cols[i], cap * colBytes(comp.P.colTag[i])));
      alloc(d_nulls[i], cap);
    }
    alloc(d_rmax, cap);
    alloc(d_skey, cap);
    alloc(d_skey2, cap);
    alloc(d_idx, cap);
    alloc(d_perm, cap);
    alloc(d_kcnt, cfg.max_keys + 1);
    alloc(d_kbeg, cfg.max_keys + 1);
    alloc(d_status, 4);
    d_err = reinterpret_cast<int*>(d_status + 2);
    d_mcount = d_status;
    HIP_OK(hipHostMalloc((void**)&h_status, 4 * sizeof(unsigned long long), hipHostMallocDefault));
    mcap = cfg.max_matches;
    rcap = mcap * comp.P.nstates * 2 + 64;
    // CHAIN32: a committed push must always expand to FULL (shp_fetch_matches, the group gather come
    // after the commit), so the refs hold the longest chains: L + 1 <= M + 1 per match
    if (cfg.match_layout == SHP_LAYOUT_CHAIN32) rcap = std::max<int64_t>(rcap, mcap * (comp.cseq.M + 1) + 64);
    alloc(d_mkey, mcap);
    alloc(d_mts, mcap);
    alloc(d_mpos, mcap);
    alloc(d_moff, mcap);
    alloc(d_refs, rcap);
    alloc(d_mtype, mcap);
    alloc(d_mslot, mcap * MAXS);
    if (cfg.match_layout == SHP_LAYOUT_AGG) alloc(d_magg, mcap);
    // scratch for rocPRIM
    size_t b1 = 0, b2 = 0, b3 = 0;
    HIP_OK(rocprim::radix_sort_pairs(nullptr, b1, d_skey, d_skey2, d_idx, d_perm, (size_t)cap, 0, key_bits + 1,
                                     stream));
    HIP_OK(rocprim::inclusive_scan(nullptr, b2, d_ts, d_rmax, (size_t)cap, rocprim::maximum<int64_t>(), stream));
    HIP_OK(rocprim::exclusive_scan(nullptr, b3, d_kcnt, d_kbeg, 0u, (size_t)cfg.max_keys, rocprim::plus<uint32_t>(),
                                   stream));
    tmp_bytes = std::max(b1, std::max(b2, b3));
    if (fast == 1) tmp_bytes = std::max(tmp_bytes, fs.scratch_bytes(cap, cfg.max_keys, stream));
    HIP_OK(hipMalloc(&d_tmp, tmp_bytes));
    if (fast == 2) {
      sw.create(comp.P, comp.fast, cfg.max_keys, cap, nown, kmap, stream);
      if (cfg.match_layout == SHP_LAYOUT_AGG) sw.enable_agg(comp.agg_fn, cfg.max_keys, kmap, stream);
      sw.D.p32 = cfg.match_layout == SHP_LAYOUT_PAIRS32;
#ifdef SHP_SW_STAMPS
      HIP_OK(hipMalloc((void**)&sw.D.stamps, (size_t)nown * 8 * sizeof(unsigned long long)));
      HIP_OK(hipMemset(sw.D.stamps, 0, (size_t)nown * 8 * sizeof(unsigned long long)));
#endif
    } else if (fast == 1) {
      fs.create(comp.P, comp.fast, cfg.max_keys, cap, mcap, stream);
    } else if (fast == 3) {
      cs.create(comp.P, comp.cseq, cfg.max_keys, cfg.max_batch, key_bits, stream,
                cfg.match_layout == SHP_LAYOUT_CHAIN32, mcap);
    } else if (fast == 4) {
      la.create(comp.P, comp.labs, cfg.max_keys, mcap, cap, stream);
      if (!labs_v1) la.sort_scratch(cap, key_bits, stream);
    } else {
      Y.build(cfg.max_keys);
      // few keys: lanes in LDS, as many per workgroup as fit 64 KB (at most 16)
      lds_lanes = 0;
      if (cfg.max_keys <= LDS_LANES_MAX_KEYS && !getenv("SHP_NO_LDS_LANES")) {
        for (int lw = 16; lw >= 1; lw /= 2) {
          Yl.build(lw);
          if (Yl.bytes <= 65536) {
            lds_lanes = lw;
            break;
          }
        }
      }
      HIP_OK(hipMalloc((void**)&arena, Y.bytes));
      HIP_OK(hipMalloc((void**)&arena2, Y.bytes));
      HIP_OK(hipMemsetAsync(arena, 0, Y.bytes, stream));
    }
    HIP_OK(hipStreamSynchronize(stream));
  }

  // runs the pipeline over n events at device pointers `in` (engine buffers after stage(), or
  // the caller's HBM columns for shp_push_batch_device); leaves matches in HBM
  int run(int64_t n, bool clock_only = false, const shp_batch* in = nullptr, bool staged_clk = false,
          bool staged_seq = false) {
    cs.ch_saved = false;  // a new push: its CHAIN32 words are in O.refs
    const DevProg& P = comp.P;
    const int64_t* x_ts = in ? in->ts : d_ts;
    const int64_t* x_clk = in ? in->clock : (staged_clk ? d_clk : nullptr);
    const int64_t* x_seq = in ? in->seq : (staged_seq ? d_seq : nullptr);
    if (x_seq && cfg.match_layout == SHP_LAYOUT_PAIRS)
      return fail(SHP_ERR_ARG, "a seq column needs match layout FULL, PAIRS32 or AGG");
    const int32_t* x_key = in ? (P.partitioned ? in->key : d_key) : d_key;
    const int32_t* x_stream = in ? in->stream : d_stream;
    if (in && !P.partitioned && fast != 2) HIP_OK(hipMemsetAsync(d_key, 0, n * 4, stream));
    if (!x_stream && fast != 2 && !(fast == 3 && !cseq_v1)) {  // NULL stream column: every event on stream 0
      HIP_OK(hipMemsetAsync(d_stream, 0, n * 4, stream));
      x_stream = d_stream;
    }
    HIP_OK(hipMemsetAsync(d_status, 0, 3 * sizeof(unsigned long long), stream));  // counts + error bits
    pushes++;
    kt.begin_push();
    HIP_OK(hipEventRecord(ev0, stream));
    BatchView B{};
    B.n = n;
    B.seq0 = seq;
    B.clock0 = clock;
    B.init_clock = cfg.start_clock;
    B.partitioned = P.partitioned;
    B.ts = x_ts;
    B.tclk = x_clk ? x_clk : x_ts;
    B.seq = x_seq;
    B.stream = x_stream;
    B.rmax = d_rmax;
    for (int c = 0; c < P.ncol; c++) {
      B.cols[c] = in ? in->cols[c] : d_cols[c];
      B.nulls[c] = in ? (in->nulls ? in->nulls[c] : nullptr) : (staged_null[c] ? d_nulls[c] : nullptr);
    }
    MatchOut O{mcap, rcap, d_mcount, d_mkey, d_mts, d_mtype, d_mpos, d_moff, d_mslot, d_refs, d_magg};
    int64_t* h_tsmax = reinterpret_cast<int64_t*>(h_status + 3);
    *h_tsmax = INT64_MIN;  // the previous push has completed (stream synchronised)
    if (fast == 2) {
      // sweep: no clock scan, no global sort (the engine clock is the running max of ts)
      HIP_OK(hipEventRecord(ev1, stream));
      if (!clock_only && n > 0 && sw.lean_push_for(B)) lean_pushes++;
      if (!clock_only) sw.run(B, x_key, O, d_err, stream, kt);
      if (!clock_only && sw.last_win) win_pushes++;
      if (!clock_only && n > 0) sw.spill(B, O, d_err, stream, kt);  // spilled owners (none: no launch)
      lastB = B;
      lastKey = x_key;
      expanded = false;
      if (cfg.match_layout == SHP_LAYOUT_FULL) {
        sw.expand(B, x_key, O, d_err, stream, kt);
        expanded = true;
      }
      HIP_OK(hipMemcpyAsync(h_tsmax, sw.D.tsmax, sizeof(int64_t), hipMemcpyDeviceToHost, stream));
    } else if (fast == 3 && !cseq_v1) {  // count sequence: its own record sort (cseq.h, run2)
      kt.mark(nullptr, stream);
      HIP_OK(hipEventRecord(ev1, stream));
      cs.run2(B, x_key, x_stream, key_bits, O, d_err, stream, kt, !cseq_wide);
      HIP_OK(hipMemcpyAsync(h_tsmax, cs.D.tsmax, sizeof(int64_t), hipMemcpyDeviceToHost, stream));
      lastB = B;
      lastKey = x_key;
      lastStream = x_stream;
      expanded = cfg.match_layout != SHP_LAYOUT_CHAIN32;  // CHAIN32: materialised on demand
    } else {
      int gb = (int)std::min<int64_t>((n + 255) / 256, 2048);
      if (gb < 1) gb = 1;
      // 1. clock (the count-sequence path has no timers: its kernel keeps the push's max ts; the
      // logical-absent multisplit computes it in its own passes, labs.h k_la_seg_clock)
      size_t tb = tmp_bytes;
      la.fuse_clock = fast == 4 && !labs_v1 && n > 0 && la.fuses_clock();
      la.rmax_out = d_rmax;
      if (fast != 3 && !la.fuse_clock) {
        kt.mark("clock_scan", stream);
        HIP_OK(rocprim::inclusive_scan(d_tmp, tb, B.tclk, d_rmax, (size_t)n, rocprim::maximum<int64_t>(), stream));
        kt.mark("clamp_clock", stream);
        k_clamp_clock<<<gb, 256, 0, stream>>>(d_rmax, n, clock);
      }
      // 2. partition by key (stable)
      HIP_OK(hipMemsetAsync(d_kcnt, 0, (cfg.max_keys + 1) * sizeof(uint32_t), stream));
      const bool bounds = fast != 1;  // key runs from the sorted keys (the scan kernels keep the histogram)
      la.sorted = false;
      bool la_v1 = labs_v1;
      if (fast == 4 && !la_v1) {  // the logical-absent records sorted with their keys (labs.h)
        HIP_OK(hipMemsetAsync(d_kbeg, 0, (cfg.max_keys + 1) * sizeof(uint32_t), stream));
        la.sort_events(B, x_key, d_skey, d_skey2, key_bits, d_err, stream, kt, d_kbeg, d_kcnt);
        int e0 = 0;  // a push beyond the 16-byte records' ranges: the 32-byte form (pack + gather)
        HIP_OK(hipMemcpyAsync(&e0, d_err, sizeof(int), hipMemcpyDeviceToHost, stream));
        HIP_OK(hipStreamSynchronize(stream));
        if (e0 & LA_WIDE) {
          const int keep = e0 & ~LA_WIDE;
          HIP_OK(hipMemcpyAsync(d_err, &keep, sizeof(int), hipMemcpyHostToDevice, stream));
          HIP_OK(hipStreamSynchronize(stream));
          la.sorted = false;
          la.steps_done = false;
          la_v1 = true;
        }
      }
      if (fast == 4 && !la_v1) {
      } else if (!bounds) {
        kt.mark("key_hist", stream);
        k_key_hist<<<gb, 256, cfg.max_keys <= KEY_HIST_LDS ? (size_t)cfg.max_keys * 4 : 0, stream>>>(
            x_key, x_stream, n, d_kcnt, cfg.max_keys, P.partitioned, d_err);
        tb = tmp_bytes;
        kt.mark("key_scan", stream);
        HIP_OK(rocprim::exclusive_scan(d_tmp, tb, d_kcnt, d_kbeg, 0u, (size_t)cfg.max_keys, rocprim::plus<uint32_t>(),
                                       stream));
        kt.mark("sort_keys", stream);
        k_sort_keys<<<gb, 256, 0, stream>>>(x_key, x_stream, n, d_skey, P.partitioned, (uint32_t)cfg.max_keys);
      } else {
        HIP_OK(hipMemsetAsync(d_kbeg, 0, (cfg.max_keys + 1) * sizeof(uint32_t), stream));
        kt.mark("sort_keys", stream);
        k_sort_keys_chk<<<gb, 256, 0, stream>>>(x_key, x_stream, n, d_skey, P.partitioned, (uint32_t)cfg.max_keys,
                                                 d_err);
      }
      if (!la.sorted) {
        kt.mark("iota", stream);
        k_iota<<<gb, 256, 0, stream>>>(d_idx, n);
        tb = tmp_bytes;
        kt.mark("radix_sort", stream);
        HIP_OK(rocprim::radix_sort_pairs(d_tmp, tb, d_skey, d_skey2, d_idx, d_perm, (size_t)n, 0, key_bits + 1, stream));
      }
      if (bounds && !(fast == 4 && !la_v1 && la.bounds)) {  // (the logical-absent multisplit set them)
        kt.mark("key_bounds", stream);
        k_key_bounds<<<(unsigned)((cfg.max_keys + 255) / 256), 256, 0, stream>>>(d_skey2, n, d_kbeg, d_kcnt,
                                                                                (uint32_t)cfg.max_keys);
      }
      kt.mark(nullptr, stream);
      HIP_OK(hipEventRecord(ev1, stream));
      // 3. NFA
      if (fast == 1) {
        fs.run(P, B, O, d_perm, d_kbeg, d_kcnt, cfg.max_keys, d_tmp, tmp_bytes, d_err, stream, d_skey2, dprog, kt);
      } else if (fast == 3) {
        cs.run(B, O, d_perm, d_kbeg, d_kcnt, d_err, d_tmp, tmp_bytes, stream, kt);
      } else if (fast == 4) {
        la.run(B, O, d_perm, d_kbeg, d_kcnt, d_err, d_tmp, tmp_bytes, stream, kt);
      } else {
        int L = cfg.max_keys;
        kt.mark("nfa_lanes", stream);
        if (lds_lanes > 0 && tier == 0) {  // reads the committed arena, writes arena2
          lanes_launch_lds((unsigned)((L + lds_lanes - 1) / lds_lanes), (unsigned)lds_lanes, stream, dprog, Y, arena,
                           arena2, Yl, B, O, d_perm, d_kbeg, d_kcnt, L, d_err);
        } else {
          HIP_OK(hipMemcpyAsync(arena2, arena, Y.bytes, hipMemcpyDeviceToDevice, stream));
          const unsigned gl = (unsigned)((L + 63) / 64);
          lanes_launch(tier, gl, stream, dprog, Y, arena2, B, O, d_perm, d_kbeg, d_kcnt, L, d_err);
        }
        kt.mark(nullptr, stream);
      }
      if (fast == 3)
        HIP_OK(hipMemcpyAsync(h_tsmax, cs.D.tsmax, sizeof(int64_t), hipMemcpyDeviceToHost, stream));
      else if (n > 0)
        HIP_OK(hipMemcpyAsync(h_tsmax, d_rmax + (n - 1), sizeof(int64_t), hipMemcpyDeviceToHost, stream));
    }
    HIP_OK(hipEventRecord(ev2, stream));
    HIP_OK(hipGetLastError());
    HIP_OK(hipMemcpyAsync(h_status, d_status, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost, stream));
    HIP_OK(hipStreamSynchronize(stream));
    int herr = 0;
    std::memcpy(&herr, h_status + 2, sizeof(int));
    if (fast == 2 && sw.last_win && (herr & SWE_LEAN) && !(herr & (SWE_KEYS | SWE_RANGE))) {
      // k_sw_win handed the push back (a ts decrease within a key, more open candidates than a
      // wave holds, a wide push): k_sw_lean re-runs it from the same committed state, and hands
      // it on to the exact solve below if it does not cover it either
      win_fallbacks++;
      HIP_OK(hipMemsetAsync(d_status, 0, 3 * sizeof(unsigned long long), stream));
      kt.mark("sw_lean", stream);
      sw.launch_lean(B, O, d_err, stream);
      kt.mark(nullptr, stream);
      if (cfg.match_layout == SHP_LAYOUT_FULL) sw.expand(B, x_key, O, d_err, stream, kt);
      HIP_OK(hipEventRecord(ev2, stream));
      HIP_OK(hipGetLastError());
      HIP_OK(hipMemcpyAsync(h_status, d_status, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost, stream));
      HIP_OK(hipStreamSynchronize(stream));
      std::memcpy(&herr, h_status + 2, sizeof(int));
    }
    if (fast == 2 && (herr & SWE_LEAN) && !(herr & (SWE_KEYS | SWE_RANGE)) && sw.D.r12) {
      // k_sw_lean handed back a push scattered in 12-byte records (ts beyond base +- 2^22 ms, or a
      // reason the 16-byte form shares): the push is scattered again in the 16-byte form and the
      // lean solve re-runs; what it hands back again goes to the exact solve below
      r16_reruns++;
      HIP_OK(hipMemsetAsync(d_status, 0, 3 * sizeof(unsigned long long), stream));
      sw.rescatter16(B, x_key, d_err, stream, kt);
      kt.mark("sw_lean", stream);
      sw.launch_lean(B, O, d_err, stream);
      kt.mark(nullptr, stream);
      if (cfg.match_layout == SHP_LAYOUT_FULL) sw.expand(B, x_key, O, d_err, stream, kt);
      HIP_OK(hipEventRecord(ev2, stream));
      HIP_OK(hipGetLastError());
      HIP_OK(hipMemcpyAsync(h_status, d_status, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost, stream));
      HIP_OK(hipStreamSynchronize(stream));
      std::memcpy(&herr, h_status + 2, sizeof(int));
    }
    if (fast == 2 && (herr & SWE_LEAN) && !(herr & (SWE_KEYS | SWE_RANGE))) {
      // k_sw_lean handed the push back (a ts decrease within a key, a wide ts span, a large
      // carry): the exact solve re-runs it over the same partition from the same committed state
      lean_fallbacks++;
      HIP_OK(hipMemsetAsync(d_status, 0, 3 * sizeof(unsigned long long), stream));
      sw.solve(B, O, d_err, stream, kt);
      sw.spill(B, O, d_err, stream, kt);
      if (cfg.match_layout == SHP_LAYOUT_FULL) sw.expand(B, x_key, O, d_err, stream, kt);
      HIP_OK(hipEventRecord(ev2, stream));
      HIP_OK(hipGetLastError());
      HIP_OK(hipMemcpyAsync(h_status, d_status, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost, stream));
      HIP_OK(hipStreamSynchronize(stream));
      std::memcpy(&herr, h_status + 2, sizeof(int));
    }
    if (fast == 2 && (herr & SWE_SPILL) && !(herr & (SWE_KEYS | SWE_RANGE))) {
      // an owner's open candidates outgrew the LDS solves' carry (the reference's lists are
      // unbounded): it becomes a spilled owner (sweep_spill.h) and the push re-runs from the same
      // committed state, the spilled owners on k_sw_spill
      spill_reruns++;
      HIP_OK(hipMemsetAsync(d_status, 0, 3 * sizeof(unsigned long long), stream));
      sw.mark_spilled(stream);
      sw.solve(B, O, d_err, stream, kt);
      sw.spill(B, O, d_err, stream, kt);
      if (cfg.match_layout == SHP_LAYOUT_FULL) sw.expand(B, x_key, O, d_err, stream, kt);
      HIP_OK(hipEventRecord(ev2, stream));
      HIP_OK(hipGetLastError());
      HIP_OK(hipMemcpyAsync(h_status, d_status, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost, stream));
      HIP_OK(hipStreamSynchronize(stream));
      std::memcpy(&herr, h_status + 2, sizeof(int));
    }
    if (fast == 3 && !cseq_v1 && !cseq_wide && (herr & CS_WIDE)) {
      // the push's ts leave the narrow records' range (+-2^31 ms of its first ts): the 16-byte
      // form re-runs it from the same committed state
      cseq_wide_reruns++;
      HIP_OK(hipMemsetAsync(d_status, 0, 3 * sizeof(unsigned long long), stream));
      cs.run2(B, x_key, x_stream, key_bits, O, d_err, stream, kt, false);
      HIP_OK(hipMemcpyAsync(h_tsmax, cs.D.tsmax, sizeof(int64_t), hipMemcpyDeviceToHost, stream));
      HIP_OK(hipEventRecord(ev2, stream));
      HIP_OK(hipGetLastError());
      HIP_OK(hipMemcpyAsync(h_status, d_status, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost, stream));
      HIP_OK(hipStreamSynchronize(stream));
      std::memcpy(&herr, h_status + 2, sizeof(int));
    }
    if (fast == 4 && (herr & LA_SEGMISS) && !(herr & (LA_SLOW | SWE_KEYS))) {
      // a warmed-up segment of k_labs_w started from another state than its predecessor ended
      // with: the push re-runs unsegmented from the same committed state
      labs_segmiss++;
      HIP_OK(hipMemsetAsync(d_status, 0, 3 * sizeof(unsigned long long), stream));
      la.noseg = true;
      la.run(B, O, d_perm, d_kbeg, d_kcnt, d_err, d_tmp, tmp_bytes, stream, kt);
      la.noseg = false;
      HIP_OK(hipEventRecord(ev2, stream));
      HIP_OK(hipGetLastError());
      HIP_OK(hipMemcpyAsync(h_status, d_status, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost, stream));
      HIP_OK(hipStreamSynchronize(stream));
      std::memcpy(&herr, h_status + 2, sizeof(int));
    }
    if (fast == 4 && (herr & LA_SLOW) && !(herr & SWE_KEYS)) {
      // k_labs_w handed the push back (a key with more than 64 pairs waiting at once): k_labs
      // re-runs it over the same partition from the same committed state
      labs_fallbacks++;
      HIP_OK(hipMemsetAsync(d_status, 0, 3 * sizeof(unsigned long long), stream));
      la.slow = true;
      la.run(B, O, d_perm, d_kbeg, d_kcnt, d_err, d_tmp, tmp_bytes, stream, kt);
      la.slow = false;
      HIP_OK(hipEventRecord(ev2, stream));
      HIP_OK(hipGetLastError());
      HIP_OK(hipMemcpyAsync(h_status, d_status, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost, stream));
      HIP_OK(hipStreamSynchronize(stream));
      std::memcpy(&herr, h_status + 2, sizeof(int));
    }
    const unsigned long long cnt[2] = {h_status[0], h_status[1]};
    int64_t tsmax = *h_tsmax;
    if (fast == 2 || fast == 3) {  // the per-push max is kept as ts ^ 2^63 (0: no event)
      const unsigned long long raw = h_status[3];
      tsmax = raw ? (int64_t)(raw ^ (1ull << 63)) : INT64_MIN;
    }
    float a = 0, b = 0;
    HIP_OK(hipEventElapsedTime(&a, ev0, ev1));
    HIP_OK(hipEventElapsedTime(&b, ev1, ev2));
    last_ms_part = a;
    last_ms_nfa = b;
    last_ms_total = a + b;
    kt.collect();
    last_m = std::min<int64_t>((int64_t)cnt[0], mcap);
    if (!herr) {
      // carry the clock (running max of ts, playback) and the sequence numbers: only a push that
      // succeeded advances them (a failed push leaves the sweep path's state as it was)
      if (tsmax != INT64_MIN && tsmax > clock) clock = tsmax;
      if (!clock_only) seq += n;
      if (fast == 2) {
        sw.commit();
        sw.spill_settle(stream);
      }
      if (fast == 3) cs.commit();
      if (fast == 4) la.commit();
      if (fast == 0) std::swap(arena, arena2);
    } else {
      last_m = 0;
      // a lane's pools or lists overflowed: re-run the push from the committed state at the next
      // capacity tier (the reference's lists are unbounded)
      const int lane_cap = E_SE | E_ND | E_LIST | E_Q;
      if (fast == 0 && (herr & lane_cap) && !(herr & ~lane_cap) && tier + 1 < LANE_TIERS && grow(tier + 1))
        return run(n, clock_only, in, staged_clk, staged_seq);
      // a key's ring of pairs waiting on the absent state overflowed: the next capacity tier
      if (fast == 4 && herr == E_LIST && la.tier + 1 < LA_TIERS && la.set_tier(la.tier + 1, true, stream))
        return run(n, clock_only, in, staged_clk, staged_seq);
      if (herr & SWE_KEYS) return fail(SHP_ERR_KEYS, "partition key id >= max_keys");
      if (herr & SWE_BOUND) return fail(SHP_ERR_DEVICE, "internal: a match pair names an event outside its push (SWE_BOUND)");
      if (fast == 4 && (herr & LA_BOUND)) return fail(SHP_ERR_DEVICE, "logical-absent path: a key's records overflowed its region");
      if (herr & E_OUT) return fail(SHP_ERR_OUTPUT, "match buffer too small for this batch (max_matches)");
      if (herr & SWE_MONO) return fail(SHP_ERR_UNSUPPORTED, "timestamps decrease within a key on the 2-state scan kernels");
      if (herr & SWE_RANGE)
        return fail(SHP_ERR_UNSUPPORTED, "timestamps of one push (and the carried candidates) span 2^49 ms or more");
      if ((herr & SWE_AGGNULL) || (fast == 0 && (herr & E_AGGNULL)))
        return fail(SHP_ERR_UNSUPPORTED, "null value in the aggregated column (match_layout AGG)");
      if (herr & SWE_P32)
        return fail(SHP_ERR_UNSUPPORTED, "a match spans 2^32 or more events (match_layout PAIRS32; use PAIRS)");
      return fail(SHP_ERR_CAPACITY, "per-key table capacity exceeded (code " + std::to_string(herr) + ")");
    }
    return SHP_OK;
  }

  // the general lanes at capacity tier t: new arenas of layout LaneLayout(max_keys, t); with
  // migrate, the committed state is carried over (else the caller overwrites it).  False when
  // the two arenas would not fit in free device memory (the engine is then unchanged).
  bool set_tier(int t, bool migrate) {
    LaneLayout Yn{};
    Yn.build(cfg.max_keys, t);
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) return false;
    if ((size_t)Yn.bytes * 2 + (256u << 20) > fr + (migrate ? 0 : (size_t)Y.bytes * 2)) return false;
    HIP_OK(hipStreamSynchronize(stream));
    char *a = nullptr, *b = nullptr;
    if (hipMalloc((void**)&a, Yn.bytes) != hipSuccess) return false;
    if (hipMalloc((void**)&b, Yn.bytes) != hipSuccess) {
      (void)hipFree(a);
      return false;
    }
    HIP_OK(hipMemsetAsync(a, 0, Yn.bytes, stream));
    if (migrate) k_lane_migrate<<<(unsigned)((Y.L + 255) / 256), 256, 0, stream>>>(Yn, a, Y, arena);
    HIP_OK(hipGetLastError());
    HIP_OK(hipStreamSynchronize(stream));
    (void)hipFree(arena);
    (void)hipFree(arena2);
    arena = a;
    arena2 = b;
    Y = Yn;
    tier = t;
    return true;
  }
  bool grow(int t) { return set_tier(t, true); }

  // ---- snapshot / restore (State.snapshot/restore, core/util/snapshot/state/State.java:25-36):
  // the device buffers that carry per-key state across pushes, for the engine's path
  struct Section {
    void* p;
    size_t bytes;
  };
  std::vector<Section> state_sections() {
    std::vector<Section> v;
    const int64_t nk = cfg.max_keys;
    if (fast == 2) {
      const SweepDev& D = sw.D;
      const int64_t no = D.nown, cc = (int64_t)no * SWS_CCAP;
      const int c = D.cur;  // the committed copy
      v = {{D.c_n[c], (size_t)no * 4}, {D.c_ts[c], (size_t)cc * 8}, {D.c_seq[c], (size_t)cc * 8},
           {D.c_v[c], (size_t)cc * 4}, {D.c_lk[c], (size_t)cc}, {D.c_null[c], (size_t)cc},
           {D.lastc[c], (size_t)no * SW_LK}};
      if (D.agg) {
        v.push_back({D.agg_s[c], (size_t)no * SW_LK * 8});
        v.push_back({D.agg_c[c], (size_t)no * SW_LK * 8});
      }
      // spilled owners: flags, their pool segments, and the pool copy (its current capacity)
      const size_t pc = (size_t)sw.pool_cap[c];
      v.push_back({D.spilled[c], (size_t)no});
      v.push_back({D.sp_n[c], (size_t)no * 4});
      v.push_back({D.sp_base[c], (size_t)no * 8});
      v.push_back({D.p_ts[c], pc * 8});
      v.push_back({D.p_seq[c], pc * 8});
      v.push_back({D.p_v[c], pc * 4});
      v.push_back({D.p_lk[c], pc});
      v.push_back({D.p_null[c], pc});
    } else if (fast == 4) {
      const LabsDev& L = la.D;
      v = {{L.pend[L.cur], (size_t)nk * sizeof(LaPend)}, {L.wq[L.cur], (size_t)nk * L.wcap * sizeof(LaWait)},
           {L.fq[L.cur], (size_t)nk * L.wcap * sizeof(LaEnt)}};
    } else if (fast == 3) {
      const CseqDev& C = cs.D;
      const int c = C.cur;
      const size_t hm = (size_t)C.M * nk * 8;
      v = {{C.len[c], (size_t)nk}, {C.prev[c], (size_t)nk * 4}, {C.pnull[c], (size_t)nk}, {C.hseq[c], hm}, {C.hts[c], hm}};
    } else if (fast == 1) {
      const FastDev& F = fs.F;
      v = {{F.c_seq, (size_t)nk * FCC * 8}, {F.c_ts, (size_t)nk * FCC * 8}, {F.c_val, (size_t)nk * FCC * 16},
           {F.c_null, (size_t)nk * FCC * 2}, {F.c_n, (size_t)nk * 4}, {F.c_match, (size_t)nk * FCC * 4},
           {F.last_ts, (size_t)nk * 8}, {F.first_open, (size_t)nk * 4}, {F.last_cand, (size_t)nk}};
    } else {
      v = {{arena, (size_t)Y.bytes}};
    }
    return v;
  }

  static uint64_t fnv1a(const std::string& t) {
    uint64_t h = 1469598103934665603ull;
    for (unsigned char c : t) h = (h ^ c) * 1099511628211ull;
    return h;
  }

  std::vector<char> snap;
  std::string program;
  struct SnapHeader {
    char magic[8];
    int32_t version, path;
    int64_t max_keys, seq, clock, sections, payload;
    uint64_t program_hash;
    int32_t maybe_null, pad;
  };

  void snapshot(void** buf, size_t* len) { snapshot_into(snap, buf, len); }

  void snapshot_into(std::vector<char>& snap, void** buf, size_t* len) {
    HIP_OK(hipStreamSynchronize(stream));
    auto secs = state_sections();
    size_t payload = 0;
    for (auto& x : secs) payload += 8 + x.bytes;
    snap.assign(sizeof(SnapHeader) + payload, 0);
    SnapHeader h{};
    memcpy(h.magic, "SHPSNAP1", 8);
    h.version = 4;  // 4: round 4's owner map (sw_owner / sw_local: low / high bits of the key id)
    h.path = fast;
    h.max_keys = cfg.max_keys;
    h.seq = seq;
    h.clock = clock;
    h.sections = (int64_t)secs.size();
    h.payload = (int64_t)payload;
    h.program_hash = fnv1a(program);
    h.maybe_null = fast == 2 ? sw.D.maybe_null : 0;
    h.pad = fast == 0 ? tier : (fast == 4 ? la.tier : 0);  // lanes / logical-absent: capacity tier
    memcpy(snap.data(), &h, sizeof h);
    char* q = snap.data() + sizeof h;
    for (auto& x : secs) {
      uint64_t b = x.bytes;
      memcpy(q, &b, 8);
      q += 8;
      HIP_OK(hipMemcpy(q, x.p, x.bytes, hipMemcpyDeviceToHost));
      q += x.bytes;
    }
    *buf = snap.data();
    *len = snap.size();
  }

  int restore(const void* buf, size_t len) {
    SnapHeader h;
    if (!buf || len < sizeof h) return fail(SHP_ERR_ARG, "snapshot too short");
    memcpy(&h, buf, sizeof h);
    if (memcmp(h.magic, "SHPSNAP1", 8) != 0 || h.version != 4) return fail(SHP_ERR_ARG, "not a snapshot (or of another version)");
    if (h.path != fast || h.max_keys != cfg.max_keys || h.program_hash != fnv1a(program))
      return fail(SHP_ERR_ARG, "snapshot is of a different query, path or key capacity");
    if (fast == 0 && (h.pad < 0 || h.pad >= LANE_TIERS)) return fail(SHP_ERR_ARG, "snapshot capacity tier unknown");
    if (fast == 4 && h.pad != la.tier) {  // the waits rings of the snapshot's tier
      if (h.pad < 0 || h.pad >= LA_TIERS) return fail(SHP_ERR_ARG, "snapshot capacity tier unknown");
      const size_t need = sizeof h + 24 + (size_t)cfg.max_keys * sizeof(LaPend) +
                          (size_t)cfg.max_keys * LA_CAPS[h.pad] * (sizeof(LaWait) + sizeof(LaEnt));
      if (need != len) return fail(SHP_ERR_ARG, "snapshot layout mismatch");
      if (!la.set_tier(h.pad, false, stream)) return fail(SHP_ERR_CAPACITY, "no device memory for the snapshot's tier");
    }
    if (fast == 0 && h.pad != tier) {  // the arena layout of the snapshot's tier (contents copied below)
      LaneLayout Yn{};
      Yn.build(cfg.max_keys, h.pad);
      if (sizeof h + 8 + (size_t)Yn.bytes != len) return fail(SHP_ERR_ARG, "snapshot layout mismatch");
      if (!set_tier(h.pad, false)) return fail(SHP_ERR_CAPACITY, "no device memory for the snapshot's capacity tier");
    }
    if (fast == 2) {  // the blob's pool capacity (the 5th-last section holds its ts column)
      const char* q0 = (const char*)buf + sizeof h;
      std::vector<uint64_t> sz;
      for (int64_t i = 0; i < h.sections && (size_t)(q0 - (const char*)buf) + 8 <= len; i++) {
        uint64_t b;
        memcpy(&b, q0, 8);
        sz.push_back(b);
        q0 += 8 + b;
      }
      if (sz.size() < 5) return fail(SHP_ERR_ARG, "snapshot layout mismatch");
      const int64_t pc = (int64_t)(sz[sz.size() - 5] / 8);
      // validate the whole blob against the layout it implies before anything changes: a
      // rejected blob leaves the committed pool (and everything else) as it was
      auto want = state_sections();
      if ((size_t)h.sections != want.size() || sizeof h + (size_t)h.payload != len || sz.size() != want.size())
        return fail(SHP_ERR_ARG, "snapshot layout mismatch");
      static const size_t pool_elem[5] = {8, 8, 4, 1, 1};  // the pool's ts, seq, value, local key, null
      for (size_t i = 0; i < want.size(); i++) {
        const size_t exp = i + 5 >= want.size() ? (size_t)pc * pool_elem[i + 5 - want.size()] : want[i].bytes;
        if (sz[i] != exp) return fail(SHP_ERR_ARG, "snapshot section size mismatch");
      }
      HIP_OK(hipStreamSynchronize(stream));
      sw.pool_exact(sw.D.cur, pc);
    }
    auto secs = state_sections();
    if ((size_t)h.sections != secs.size() || sizeof h + (size_t)h.payload != len)
      return fail(SHP_ERR_ARG, "snapshot layout mismatch");
    const char* q = (const char*)buf + sizeof h;
    for (auto& x : secs) {
      uint64_t b;
      memcpy(&b, q, 8);
      q += 8;
      if (b != x.bytes) return fail(SHP_ERR_ARG, "snapshot section size mismatch");
      q += b;
    }
    q = (const char*)buf + sizeof h;
    HIP_OK(hipStreamSynchronize(stream));
    for (auto& x : secs) {
      q += 8;
      HIP_OK(hipMemcpy(x.p, q, x.bytes, hipMemcpyHostToDevice));
      q += x.bytes;
    }
    seq = h.seq;
    clock = h.clock;
    last_m = 0;  // the last push's records belong to the state the restore replaced
    expanded = true;
    if (fast == 2) {
      sw.D.maybe_null = h.maybe_null;
      sw.D.spill_on = sw.count_spilled() > 0;
    }
    return SHP_OK;
  }

  // ---- the snapshot in the reference's State.snapshot() key names (shp_snapshot_describe):
  // per partition key and state, what StreamPreState.snapshot (StreamPreStateProcessor.java:
  // 450-469) and its Count / Absent / Scheduler subclasses would hold.  Events are named by
  // {seq, ts}: the host rebuilds StreamEvents from the sequence numbers, as for match records.
  static void jnum(std::string& o, int64_t v) { o += std::to_string(v); }
  static void jbool(std::string& o, bool b) { o += b ? "true" : "false"; }

  std::string describe(const void* buf, size_t len) {
    SnapHeader h;
    if (!buf || len < sizeof h) throw std::runtime_error("snapshot too short");
    memcpy(&h, buf, sizeof h);
    if (memcmp(h.magic, "SHPSNAP1", 8) != 0 || h.version != 4 || h.path != fast || h.max_keys != cfg.max_keys ||
        h.program_hash != fnv1a(program))
      throw std::runtime_error("not a snapshot of this engine's query, path and key capacity");
    LaneLayout Yb = Y;  // lanes: the layout of the snapshot's capacity tier
    if (fast == 0) {
      if (h.pad < 0 || h.pad >= LANE_TIERS) throw std::runtime_error("snapshot capacity tier unknown");
      Yb.build(cfg.max_keys, h.pad);
    }
    auto secs = state_sections();
    if (fast == 0) secs[0].bytes = (size_t)Yb.bytes;
    if (fast == 4) {
      if (h.pad < 0 || h.pad >= LA_TIERS) throw std::runtime_error("snapshot capacity tier unknown");
      secs[1].bytes = (size_t)cfg.max_keys * LA_CAPS[h.pad] * sizeof(LaWait);
      secs[2].bytes = (size_t)cfg.max_keys * LA_CAPS[h.pad] * sizeof(LaEnt);
    }
    std::vector<const char*> sp(secs.size());
    const char* q = (const char*)buf + sizeof h;
    for (size_t i = 0; i < secs.size(); i++) {
      uint64_t b;
      memcpy(&b, q, 8);
      if (fast == 2 && i + 5 >= secs.size()) secs[i].bytes = b;  // the pool: the blob's capacity
      if (b != secs[i].bytes || (size_t)(q + 8 + b - (const char*)buf) > len)
        throw std::runtime_error("snapshot layout mismatch");
      sp[i] = q + 8;
      q += 8 + b;
    }
    const DevProg& P = comp.P;
    std::string o = "{\"engine\":{\"path\":";
    jnum(o, fast);
    o += ",\"seq\":";
    jnum(o, h.seq);
    o += ",\"clock\":";
    jnum(o, h.clock);
    if (fast == 0 || fast == 4) {  // lanes: the tier of the pools and lists (LaneCaps); labs: of the rings
      o += ",\"tier\":";
      jnum(o, h.pad);
    }
    o += "},\"keys\":{";
    bool firstKey = true;
    auto ev = [&](std::string& s, int64_t seqv, int64_t tsv) {
      if (live_min && seqv >= 0 && seqv < *live_min) *live_min = seqv;
      s += "{\"seq\":";
      jnum(s, seqv);
      s += ",\"ts\":";
      jnum(s, tsv);
      s += "}";
    };
    if (fast == 4) {
      // logical-absent: the logical partial (x / y slots), the pairs on the absent state's pending and
      // new-and-every lists, its lastScheduledTime and the key's Scheduler queue
      const LaPend* pd = (const LaPend*)sp[0];
      const LaWait* wq = (const LaWait*)sp[1];
      const LaEnt* fq = (const LaEnt*)sp[2];
      const LabsDev& L = la.D;
      const int64_t wcap = LA_CAPS[h.pad >= 0 && h.pad < LA_TIERS ? h.pad : 0];
      for (int32_t k = 0; k < cfg.max_keys; k++) {
        const LaPend& s = pd[k];
        if (s.last == INT64_MIN) continue;
        o += firstKey ? "\"" : ",\"";
        firstKey = false;
        jnum(o, k);
        o += "\":{\"logical\":{\"PendingStateEventList\":[{\"slots\":{";
        o += "\"e" + std::to_string(L.sid[0] + 1) + "\":[";
        if (s.xseq >= 0) ev(o, s.xseq, s.xts);
        o += "],\"e" + std::to_string(L.sid[1] + 1) + "\":[";
        if (s.yseq >= 0) ev(o, s.yseq, s.yts);
        o += "]}}]},\"absent\":{\"PendingStateEventList\":[";
        for (int i = 0; i < s.nw; i++) {
          const LaWait& w = wq[(int64_t)k * wcap + ((s.wh + i) & (wcap - 1))];
          if (i == s.nw - s.nae) o += "],\"NewAndEveryStateEventList\":[";
          else if (i) o += ",";
          o += "{\"ts\":";
          jnum(o, w.due - L.wait);
          o += ",\"due\":";
          jnum(o, w.due);
          o += ",\"slots\":[";
          ev(o, w.xseq, w.xts);
          o += ",";
          ev(o, w.yseq, w.yts);
          o += "]}";
        }
        if (s.nae == 0) o += "],\"NewAndEveryStateEventList\":[";
        o += "],\"LastScheduledTime\":";
        jnum(o, s.lst);
        o += "},\"scheduler0\":{\"ToNotifyQueue\":[";
        for (int i = 0; i < s.ne; i++) {
          if (i) o += ",";
          const int64_t t = fq[(int64_t)k * wcap + ((s.eh + i) & (wcap - 1))].t;
          if (due_min && i == 0 && t < *due_min) *due_min = t;  // the key's FIFO head
          jnum(o, t);
        }
        o += "]}}";
      }
    } else if (fast == 3) {
      // count sequence: e1's chain is the partial CountPreStateProcessor holds (its e1 slot, the
      // key's last L events); with L == 0 only the re-armed start partial (no events) is pending
      const CseqDev& C = cs.D;
      const uint8_t* len = (const uint8_t*)sp[0];
      const int64_t* hseq = (const int64_t*)sp[3];
      const int64_t* hts = (const int64_t*)sp[4];
      for (int32_t k = 0; k < cfg.max_keys; k++) {
        const int64_t last = hseq[cs_hslot(C.M - 1, k, C.M)];
        if (last < 0) continue;  // no event of this key yet
        o += firstKey ? "\"" : ",\"";
        firstKey = false;
        jnum(o, k);
        const int L = len[k] > C.M ? 0 : len[k];  // (M + 1: the once-armed start has been used)
        o += "\":{\"e1\":{\"Count\":";
        jnum(o, L);
        o += ",\"PendingStateEventList\":[{\"ts\":";
        jnum(o, L ? hts[cs_hslot(C.M - 1, k, C.M)] : -1);
        o += ",\"slots\":[[";
        for (int i = C.M - L; i < C.M; i++) {
          if (i > C.M - L) o += ",";
          ev(o, hseq[cs_hslot(i, k, C.M)], hts[cs_hslot(i, k, C.M)]);
        }
        o += "],[]]}]},\"LastEvent\":";
        int64_t* const keep = live_min;  // the key's last event: history, not a partial's event
        live_min = nullptr;
        ev(o, last, hts[cs_hslot(C.M - 1, k, C.M)]);
        live_min = keep;
        o += "}";
      }
    } else if (fast == 2 || fast == 1) {
      // 2-state `every e1 -> e2 within`: e1's start partial, e2's open candidates (partials
      // holding e1); the key's latest event, when it opened a candidate, left that one (and
      // e1's re-armed partial) on the new-and-every lists
      std::vector<std::vector<std::pair<int64_t, int64_t>>> open(cfg.max_keys);  // (seq, ts) per key
      std::vector<uint8_t> lastc(cfg.max_keys, 0), seen(cfg.max_keys, 0);
      if (fast == 2) {
        int32_t nown = 0;
        std::vector<uint32_t> kmap;
        SweepState::build_map(cfg.max_keys, nown, kmap);
        std::vector<int32_t> inv((size_t)nown * SW_LK, -1);
        for (int32_t k = 0; k < cfg.max_keys; k++) inv[(size_t)(kmap[k] & 0xffffu) * SW_LK + (kmap[k] >> 16)] = k;
        const int32_t* c_n = (const int32_t*)sp[0];
        const int64_t* c_ts = (const int64_t*)sp[1];
        const int64_t* c_seq = (const int64_t*)sp[2];
        const uint8_t* c_lk = (const uint8_t*)sp[4];
        const uint8_t* lc = (const uint8_t*)sp[6];
        const size_t s0 = sw.D.agg ? 9 : 7;  // spill sections: spilled, sp_n, sp_base, pool ts / seq / v / lk / null
        const uint8_t* spl = (const uint8_t*)sp[s0];
        const int32_t* spn = (const int32_t*)sp[s0 + 1];
        const int64_t* spb = (const int64_t*)sp[s0 + 2];
        const int64_t* p_ts = (const int64_t*)sp[s0 + 3];
        const int64_t* p_seq = (const int64_t*)sp[s0 + 4];
        const uint8_t* p_lk = (const uint8_t*)sp[s0 + 6];
        const int64_t npool = (int64_t)(secs[s0 + 3].bytes / 8);
        for (int32_t ow = 0; ow < nown; ow++) {
          if (spl[ow] && spn[ow] >= 0) {  // a spilled owner: its open candidates are in the pool
            if (spb[ow] < 0 || spb[ow] + spn[ow] > npool) throw std::runtime_error("snapshot pool segment out of range");
            for (int64_t i = 0; i < spn[ow]; i++) {
              const int64_t c = spb[ow] + i;
              const int32_t k = inv[(size_t)ow * SW_LK + p_lk[c]];
              if (k >= 0) open[k].push_back({p_seq[c], p_ts[c]});
            }
          } else {
            if (c_n[ow] < 0 || c_n[ow] > SWS_CCAP) throw std::runtime_error("snapshot carry count out of range");
            for (int i = 0; i < c_n[ow]; i++) {
              const int64_t c = (int64_t)ow * SWS_CCAP + i;
              const int32_t k = inv[(size_t)ow * SW_LK + c_lk[c]];
              if (k >= 0) open[k].push_back({c_seq[c], c_ts[c]});
            }
          }
          for (int l = 0; l < SW_LK; l++) {
            const int32_t k = inv[(size_t)ow * SW_LK + l];
            if (k >= 0) lastc[k] = lc[(size_t)ow * SW_LK + l];
          }
        }
      } else {
        const int64_t* c_seq = (const int64_t*)sp[0];
        const int64_t* c_ts = (const int64_t*)sp[1];
        const int32_t* c_n = (const int32_t*)sp[4];
        const int64_t* last_ts = (const int64_t*)sp[6];
        const uint8_t* lc = (const uint8_t*)sp[8];
        for (int32_t k = 0; k < cfg.max_keys; k++) {
          for (int i = 0; i < c_n[k]; i++) open[k].push_back({c_seq[(int64_t)k * FCC + i], c_ts[(int64_t)k * FCC + i]});
          lastc[k] = lc[k];
          seen[k] = last_ts[k] != INT64_MIN;
        }
      }
      for (int32_t k = 0; k < cfg.max_keys; k++) {
        if (open[k].empty() && !lastc[k] && !seen[k]) continue;
        o += firstKey ? "\"" : ",\"";
        firstKey = false;
        jnum(o, k);
        o += "\":{\"e1\":{\"FirstEvent\":null,\"PendingStateEventList\":[";
        const char* empty = "{\"ts\":-1,\"slots\":[[],[]]}";
        if (!lastc[k]) o += empty;
        o += "],\"NewAndEveryStateEventList\":[";
        if (lastc[k]) o += empty;
        o += "],\"Initialized\":true,\"Started\":false},\"e2\":{\"FirstEvent\":null,\"PendingStateEventList\":[";
        const size_t np = open[k].size() - ((lastc[k] && !open[k].empty()) ? 1 : 0);
        for (size_t i = 0; i < open[k].size(); i++) {
          if (i == np) o += "],\"NewAndEveryStateEventList\":[";
          else if (i) o += ",";
          o += "{\"ts\":";
          jnum(o, open[k][i].second);
          o += ",\"slots\":[[";
          ev(o, open[k][i].first, open[k][i].second);
          o += "],[]]}";
        }
        if (np == open[k].size()) o += "],\"NewAndEveryStateEventList\":[";
        o += "],\"Initialized\":false,\"Started\":false}}";
      }
    } else {
      // general lanes: decode each key's arena (lane-interleaved SoA, LaneLayout)
      const char* a = sp[0];
      auto at = [&](int64_t off, int64_t i, int64_t k, int sz) -> const char* {
        return a + off + (i * Yb.L + k) * sz;
      };
      auto i16 = [&](int64_t off, int64_t i, int64_t k) { int16_t v; memcpy(&v, at(off, i, k, 2), 2); return v; };
      auto i64 = [&](int64_t off, int64_t i, int64_t k) { int64_t v; memcpy(&v, at(off, i, k, 8), 8); return v; };
      auto u8 = [&](int64_t off, int64_t i, int64_t k) { return *(const uint8_t*)at(off, i, k, 1); };
      for (int64_t k = 0; k < Yb.L; k++) {
        if (!u8(Yb.o_kinit, 0, k)) continue;
        o += firstKey ? "\"" : ",\"";
        firstKey = false;
        jnum(o, k);
        o += "\":{";
        auto partial = [&](std::string& s, int se) {
          s += "{\"ts\":";
          jnum(s, i64(Yb.o_se_ts, se, k));
          s += ",\"type\":\"";
          s += u8(Yb.o_se_type, se, k) ? "EXPIRED" : "CURRENT";
          s += "\",\"slots\":[";
          for (int st = 0; st < P.nstates; st++) {
            s += st ? ",[" : "[";
            int guard = 0;
            for (int nd = i16(Yb.o_se_slot, (int64_t)se * MAXS + st, k); nd >= 0 && guard < Yb.nn;
                 nd = i16(Yb.o_nd_next, nd, k), guard++) {
              if (guard) s += ",";
              ev(s, i64(Yb.o_nd_seq, nd, k), i64(Yb.o_nd_ts, nd, k));
            }
            s += "]";
          }
          s += "]}";
        };
        for (int p = 0; p < P.npre; p++) {
          const DPre& d = P.pre[p];
          o += p ? ",\"" : "\"";
          o += "pre" + std::to_string(p) + "(e" + std::to_string(d.stateId + 1) + ")\":{\"FirstEvent\":null";
          for (int which = 0; which < 2; which++) {
            o += which == 0 ? ",\"PendingStateEventList\":[" : ",\"NewAndEveryStateEventList\":[";
            const int n = i16(Yb.o_lst_len, which * MAXP + p, k);
            for (int i = 0; i < n; i++) {
              if (i) o += ",";
              partial(o, i16(Yb.o_lst, (int64_t)(which * MAXP + p) * Yb.lcap + i, k));
            }
            o += "]";
          }
          const uint8_t f = u8(Yb.o_pflags, p, k);
          o += ",\"Initialized\":";
          jbool(o, f & F_INIT);
          o += ",\"Started\":";
          jbool(o, f & F_STARTED);
          if (d.kind == K_COUNT) {
            o += ",\"SuccessCondition\":";
            jbool(o, f & F_SUCCESS);
            o += ",\"StartStateReset\":";
            jbool(o, f & F_SSRESET);
          }
          if (d.kind == K_ABSENT_STREAM || d.kind == K_ABSENT_LOGICAL) {
            o += ",\"IsActive\":";
            jbool(o, !(f & F_INACTIVE));
            o += ",\"LastScheduledTime\":";
            jnum(o, i64(Yb.o_lsched, p, k));
            o += ",\"LastArrivalTime\":";
            jnum(o, i64(Yb.o_larr, p, k));
          }
          o += "}";
        }
        for (int s = 0; s < P.nsched; s++) {  // Scheduler.SchedulerState: ToNotifyQueue (FIFO)
          o += ",\"scheduler" + std::to_string(s) + "\":{\"ToNotifyQueue\":[";
          const int hd = i16(Yb.o_qhead, s, k), n = i16(Yb.o_qlen, s, k);
          for (int i = 0; i < n; i++) {
            if (i) o += ",";
            const int64_t t = i64(Yb.o_q, (int64_t)s * Yb.qcap + (hd + i) % Yb.qcap, k);
            if (due_min && i == 0 && t < *due_min) *due_min = t;  // the key's FIFO head
            jnum(o, t);
          }
          o += "]}";
        }
        o += "}";
      }
    }
    o += "}}";
    return o;
  }

  // ---- the oldest event sequence number the committed state still names (shp_engine_oldest_live_seq):
  // every event of an open partial -- a pending / new-and-every list entry of any state, a count
  // chain, a logical slot, a pair waiting on an absent timer, a sweep carry or spill-pool entry.  A
  // later push's matches name only these events and the later pushes' own, so a host that rebuilds
  // match events from its own rows (ColumnarBatch) may drop every row below it.  The walk is the
  // snapshot decoder's (describe), so it covers exactly what a snapshot would restore.
  int64_t* live_min = nullptr;
  std::vector<char> live_snap;
  int64_t oldest_live_seq() {
    void* b = nullptr;
    size_t n = 0;
    snapshot_into(live_snap, &b, &n);
    int64_t m = seq;  // nothing open: every later match names only later events
    live_min = &m;
    try {
      (void)describe(b, n);
    } catch (...) {
      live_min = nullptr;
      throw;
    }
    live_min = nullptr;
    return m;
  }

  // ---- the earliest due time of any key's timer queue (shp_engine_next_due): the head of each
  // key's Scheduler FIFO (Scheduler.java:113-127, 332) -- the EventCaller of a live-mode Scheduler
  // is scheduled at the head's due time (Scheduler.schedule :129-155, EventCaller.run :287-326).
  // INT64_MAX when no timer is pending (the 2-state, count-sequence paths have none).
  int64_t* due_min = nullptr;
  int64_t next_due() {
    if (fast != 0 && fast != 4) return INT64_MAX;
    if (fast == 0 && comp.P.nsched == 0) return INT64_MAX;
    void* b = nullptr;
    size_t n = 0;
    snapshot_into(live_snap, &b, &n);
    int64_t m = INT64_MAX;
    due_min = &m;
    try {
      (void)describe(b, n);
    } catch (...) {
      due_min = nullptr;
      throw;
    }
    due_min = nullptr;
    return m;
  }

  // sweep path, PAIRS layout: materialise the full records of the last push on demand
  void ensure_expanded() {
    if (expanded || cfg.match_layout == SHP_LAYOUT_AGG || (fast != 2 && fast != 3)) return;
    MatchOut O{mcap, rcap, d_mcount, d_mkey, d_mts, d_mtype, d_mpos, d_moff, d_mslot, d_refs, d_magg};
    HIP_OK(hipMemsetAsync(d_err, 0, sizeof(int), stream));
    if (fast == 2) sw.expand(lastB, lastKey, O, d_err, stream, kt, last_m);
    else cs.expand(lastB, lastKey, lastStream, key_bits, O, last_m, d_err, stream, kt);
    int herr = 0;
    HIP_OK(hipMemcpyAsync(&herr, d_err, sizeof(int), hipMemcpyDeviceToHost, stream));
    HIP_OK(hipStreamSynchronize(stream));
    if (herr & SWE_BOUND) throw DevError("internal: a match pair names an event outside its push (SWE_BOUND)");
    if (herr & E_OUT)  // (unreachable: rcap holds M + 1 refs per match for CHAIN32 engines)
      throw OutputError("CHAIN32 expansion beyond the ref capacity (raise max_matches)");
    expanded = true;
  }

  int fail(int code, const std::string& m) {
    err = m;
    return code;
  }

  void stage(const shp_batch* in, hipMemcpyKind kind) {
    const DevProg& P = comp.P;
    int64_t n = in->n;
    HIP_OK(hipMemcpyAsync(d_ts, in->ts, n * 8, kind, stream));
    if (in->clock) HIP_OK(hipMemcpyAsync(d_clk, in->clock, n * 8, kind, stream));
    if (in->seq) HIP_OK(hipMemcpyAsync(d_seq, in->seq, n * 8, kind, stream));
    if (P.partitioned) HIP_OK(hipMemcpyAsync(d_key, in->key, n * 4, kind, stream));
    else HIP_OK(hipMemsetAsync(d_key, 0, n * 4, stream));
    if (in->stream) HIP_OK(hipMemcpyAsync(d_stream, in->stream, n * 4, kind, stream));
    else HIP_OK(hipMemsetAsync(d_stream, 0, n * 4, stream));
    for (int c = 0; c < P.ncol; c++) {
      HIP_OK(hipMemcpyAsync(d_cols[c], in->cols[c], n * colBytes(P.colTag[c]), kind, stream));
      // a column without nulls is run with no null bitmap (as a device push without one)
      staged_null[c] = in->nulls && in->nulls[c];
      if (staged_null[c]) HIP_OK(hipMemcpyAsync(d_nulls[c], in->nulls[c], n, kind, stream));
    }
  }

  // ---- pipelined host ingest
  void slots_alloc() {
    if (slots_ready) return;
    const DevProg& P = comp.P;
    HIP_OK(hipStreamCreateWithFlags(&cstream, hipStreamNonBlocking));
    for (Slot& sl : slots) {
      alloc(sl.ts, cap);
      alloc(sl.ts32, cap);
      alloc(sl.k16, cap);
      alloc(sl.key, cap);
      alloc(sl.strm, cap);
      alloc(sl.clk, cap);
      alloc(sl.sq, cap);
      for (int c = 0; c < P.ncol; c++) {
        HIP_OK(hipMalloc(&sl.cols[c], std::max<int64_t>(cap, 1) * colBytes(P.colTag[c])));
        alloc(sl.nulls[c], cap);
      }
      HIP_OK(hipEventCreateWithFlags(&sl.ready, hipEventDisableTiming));
      HIP_OK(hipEventCreateWithFlags(&sl.consumed, hipEventDisableTiming));
      HIP_OK(hipEventRecord(sl.consumed, stream));
    }
    slots_ready = true;
  }

  // H2D of one host batch into the next free slot on the copy stream; returns once enqueued
  int stage_slot(const shp_batch* in, const int32_t* ts32, int64_t ts_base, const uint16_t* key16 = nullptr) {
    const DevProg& P = comp.P;
    if (in->n > cfg.max_batch) return fail(SHP_ERR_ARG, "batch larger than max_batch");
    if (in->n > 0 && !ts32 && !in->ts) return fail(SHP_ERR_ARG, "no ts column");
    if (P.partitioned && in->n > 0 && !in->key && !key16) return fail(SHP_ERR_ARG, "no key column");
    if (key16 && cfg.max_keys > 65536) return fail(SHP_ERR_ARG, "2-byte key ids need max_keys <= 65536");
    if (slot_count == 2) return fail(SHP_ERR_CAPACITY, "two batches staged: run one first (shp_run_staged)");
    slots_alloc();
    Slot& sl = slots[(slot_head + slot_count) % 2];
    const int64_t n = in->n;
    const hipMemcpyKind k = hipMemcpyHostToDevice;
    HIP_OK(hipStreamWaitEvent(cstream, sl.consumed, 0));  // the run that read this slot is done
    sl.n = n;
    sl.narrow = ts32 != nullptr;
    sl.nkey = P.partitioned && key16 != nullptr;
    sl.ts_base = ts_base;
    if (n > 0) {
      if (ts32) HIP_OK(hipMemcpyAsync(sl.ts32, ts32, n * 4, k, cstream));
      else HIP_OK(hipMemcpyAsync(sl.ts, in->ts, n * 8, k, cstream));
      if (sl.nkey) HIP_OK(hipMemcpyAsync(sl.k16, key16, n * 2, k, cstream));
      else if (P.partitioned) HIP_OK(hipMemcpyAsync(sl.key, in->key, n * 4, k, cstream));
      sl.has_stream = in->stream != nullptr;
      if (sl.has_stream) HIP_OK(hipMemcpyAsync(sl.strm, in->stream, n * 4, k, cstream));
      sl.has_clk = in->clock != nullptr;
      if (sl.has_clk) HIP_OK(hipMemcpyAsync(sl.clk, in->clock, n * 8, k, cstream));
      sl.has_seq = in->seq != nullptr;
      if (sl.has_seq) HIP_OK(hipMemcpyAsync(sl.sq, in->seq, n * 8, k, cstream));
      for (int c = 0; c < P.ncol; c++) {
        HIP_OK(hipMemcpyAsync(sl.cols[c], in->cols[c], n * colBytes(P.colTag[c]), k, cstream));
        sl.has_null[c] = in->nulls && in->nulls[c];
        if (sl.has_null[c]) HIP_OK(hipMemcpyAsync(sl.nulls[c], in->nulls[c], n, k, cstream));
      }
    }
    HIP_OK(hipEventRecord(sl.ready, cstream));
    slot_count++;
    return SHP_OK;
  }

  // the oldest staged batch through the engine; compact records to page-locked host memory
  int run_slot(shp_matches* out) {
    if (slot_count == 0) return fail(SHP_ERR_ARG, "no staged batch (shp_stage_batch first)");
    const DevProg& P = comp.P;
    Slot& sl = slots[slot_head];
    slot_head = (slot_head + 1) % 2;
    slot_count--;
    HIP_OK(hipStreamWaitEvent(stream, sl.ready, 0));
    const int64_t n = sl.n;
    if (sl.narrow && n > 0) {
      const int gb = (int)std::min<int64_t>((n + 255) / 256, 8192);
      k_widen_ts<<<gb, 256, 0, stream>>>(sl.ts32, sl.ts_base, sl.ts, n);
    }
    if (sl.nkey && n > 0) {
      const int gb = (int)std::min<int64_t>((n + 255) / 256, 8192);
      k_widen_key<<<gb, 256, 0, stream>>>(sl.k16, sl.key, n);
    }
    const void* cp[MAXCOL];
    const uint8_t* np[MAXCOL];
    for (int c = 0; c < P.ncol; c++) {
      cp[c] = sl.cols[c];
      np[c] = sl.has_null[c] ? sl.nulls[c] : nullptr;
    }
    shp_batch b{n, sl.ts, sl.key, sl.has_stream ? sl.strm : nullptr, cp, np, sl.has_clk ? sl.clk : nullptr,
                sl.has_seq ? sl.sq : nullptr};
    const int rc = run(n, false, &b);
    HIP_OK(hipEventRecord(sl.consumed, stream));
    if (rc != SHP_OK) return rc;
    const int lay = cfg.match_layout;
    const bool compact = !expanded && ((fast == 2 && (lay == SHP_LAYOUT_PAIRS32 || lay == SHP_LAYOUT_PAIRS)) ||
                                       (fast == 3 && lay == SHP_LAYOUT_CHAIN32));
    if (!compact) {
      fetch(out);
      return SHP_OK;
    }
    const int64_t m = last_m;
    const int64_t words = lay == SHP_LAYOUT_PAIRS ? 4 * m : (lay == SHP_LAYOUT_PAIRS32 ? 2 * m : m);
    if (words > h_wpin_words) {
      if (h_wpin) HIP_OK(hipHostFree(h_wpin));
      h_wpin = nullptr;
      h_wpin_words = std::max<int64_t>(words, h_wpin_words * 2);
      HIP_OK(hipHostMalloc((void**)&h_wpin, (size_t)h_wpin_words * 4, hipHostMallocDefault));
    }
    if (m) {
      HIP_OK(hipMemcpyAsync(h_wpin, d_refs, (size_t)words * 4, hipMemcpyDeviceToHost, stream));
      HIP_OK(hipStreamSynchronize(stream));
    }
    *out = shp_matches{};
    out->layout = lay;
    out->m = m;
    out->num_states = P.nstates;
    out->refs = (int64_t*)h_wpin;
    return SHP_OK;
  }

  void fill_device(shp_matches* out) {
    out->agg = nullptr;
    if (cfg.match_layout == SHP_LAYOUT_AGG) {
      *out = shp_matches{};
      out->layout = SHP_LAYOUT_AGG;
      out->m = last_m;
      out->num_states = comp.P.nstates;
      out->key = d_mkey;
      out->agg = d_magg;
      return;
    }
    out->layout = expanded ? SHP_LAYOUT_FULL : cfg.match_layout;
    out->m = last_m;
    out->num_states = comp.P.nstates;
    out->key = d_mkey;
    out->ts = d_mts;
    out->type = d_mtype;
    out->pos = d_mpos;
    out->ref_off = d_moff;
    out->slot_len = d_mslot;
    out->refs = d_refs;
  }

  // copy to host and order by (pos, per-lane order) so callbacks follow reference emission order
  void fetch(shp_matches* out) {
    if (cfg.match_layout == SHP_LAYOUT_AGG) {  // per-key emission order as produced
      const int64_t m = last_m;
      h_key.resize(m);
      h_agg.resize(m);
      if (m) {
        HIP_OK(hipMemcpy(h_key.data(), d_mkey, m * 4, hipMemcpyDeviceToHost));
        HIP_OK(hipMemcpy(h_agg.data(), d_magg, m * 8, hipMemcpyDeviceToHost));
      }
      *out = shp_matches{};
      out->layout = SHP_LAYOUT_AGG;
      out->m = m;
      out->num_states = comp.P.nstates;
      out->key = h_key.data();
      out->agg = h_agg.data();
      return;
    }
    ensure_expanded();
    out->layout = SHP_LAYOUT_FULL;
    int64_t m = last_m;
    int S = comp.P.nstates;
    std::vector<int32_t> k(m);
    std::vector<int64_t> ts(m), pos(m), off(m);
    std::vector<int8_t> ty(m);
    std::vector<int16_t> sl(m * MAXS);
    unsigned long long cnt[2];
    HIP_OK(hipMemcpy(cnt, d_mcount, sizeof(cnt), hipMemcpyDeviceToHost));
    int64_t r = (int64_t)cnt[1];
    std::vector<int64_t> refs(r);
    if (m) {
      HIP_OK(hipMemcpy(k.data(), d_mkey, m * 4, hipMemcpyDeviceToHost));
      HIP_OK(hipMemcpy(ts.data(), d_mts, m * 8, hipMemcpyDeviceToHost));
      HIP_OK(hipMemcpy(pos.data(), d_mpos, m * 8, hipMemcpyDeviceToHost));
      HIP_OK(hipMemcpy(off.data(), d_moff, m * 8, hipMemcpyDeviceToHost));
      HIP_OK(hipMemcpy(ty.data(), d_mtype, m, hipMemcpyDeviceToHost));
      HIP_OK(hipMemcpy(sl.data(), d_mslot, m * MAXS * 2, hipMemcpyDeviceToHost));
      if (r) HIP_OK(hipMemcpy(refs.data(), d_refs, r * 8, hipMemcpyDeviceToHost));
    }
    // per-key order is the append order; stable-sort by (pos, key-append-order)
    std::vector<int64_t> idx(m);
    std::iota(idx.begin(), idx.end(), 0);
    std::stable_sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) {
      if (pos[a] != pos[b]) return pos[a] < pos[b];
      if (k[a] != k[b]) return k[a] < k[b];
      return a < b;
    });
    h_key.resize(m);
    h_ts.resize(m);
    h_pos.resize(m);
    h_off.resize(m);
    h_type.resize(m);
    h_slot.resize(m * S);
    h_refs.clear();
    for (int64_t i = 0; i < m; i++) {
      int64_t j = idx[i];
      h_key[i] = k[j];
      h_ts[i] = ts[j];
      h_pos[i] = pos[j];
      h_type[i] = ty[j];
      h_off[i] = (int64_t)h_refs.size();
      int64_t o = off[j];
      for (int s = 0; s < S; s++) {
        int16_t l = sl[j * MAXS + s];
        h_slot[i * S + s] = l;
        for (int t = 0; t < l; t++) h_refs.push_back(refs[o++]);
      }
    }
    h_m = m;
    out->m = m;
    out->num_states = S;
    out->key = h_key.data();
    out->ts = h_ts.data();
    out->type = h_type.data();
    out->pos = h_pos.data();
    out->ref_off = h_off.data();
    out->slot_len = h_slot.data();
    out->refs = h_refs.data();
    out->agg = nullptr;
  }

  // shp_push_batch_compact: the last push's records in the compact layout the engine produced them in
  // (PAIRS32 / PAIRS on the sweep path, CHAIN32 on the count-sequence path, AGG rows), copied to
  // the host as they are -- no expansion.  On a path that emits full records this is
  // shp_fetch_matches: the caller reads out->layout.  The compact words keep the engine's per-key emission order; across
  // keys they are in owner order, so a host that needs the reference's global order sorts them by
  // e2's batch index (stable).
  std::vector<uint32_t> h_words;
  int fetch_compact(shp_matches* out) {
    const int lay = cfg.match_layout;
    const bool compact = !expanded && ((fast == 2 && (lay == SHP_LAYOUT_PAIRS32 || lay == SHP_LAYOUT_PAIRS)) ||
                                       (fast == 3 && lay == SHP_LAYOUT_CHAIN32));
    if (!compact) {
      fetch(out);
      return SHP_OK;
    }
    const int64_t m = last_m;
    const int64_t words = lay == SHP_LAYOUT_PAIRS ? 4 * m : (lay == SHP_LAYOUT_PAIRS32 ? 2 * m : m);
    h_words.resize((size_t)std::max<int64_t>(words, 1));
    if (m) HIP_OK(hipMemcpy(h_words.data(), d_refs, (size_t)words * 4, hipMemcpyDeviceToHost));
    *out = shp_matches{};
    out->layout = lay;
    out->m = m;
    out->num_states = comp.P.nstates;
    out->refs = (int64_t*)h_words.data();
    return SHP_OK;
  }
};

// ---------------------------------------------------------------- C-ABI
extern "C" {

int shp_engine_create(const char* json, const shp_config* cfg, shp_engine** out) {
  if (!json || !cfg || !out) return SHP_ERR_ARG;
  // create binds the engine's device for its allocations; the caller's current device is restored
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  struct Restore {
    int d;
    ~Restore() {
      if (d >= 0) (void)hipSetDevice(d);
    }
  } restore{prev};
  auto* e = new shp_engine();
  try {
    e->create(json, cfg);
  } catch (CompileError& ce) {
    fprintf(stderr, "shp_engine_create: %s\n", ce.what());
    delete e;
    *out = nullptr;
    return ce.code == -2 ? SHP_ERR_UNSUPPORTED : SHP_ERR_ARG;
  } catch (DevError& de) {
    fprintf(stderr, "shp_engine_create: %s\n", de.what());
    delete e;
    *out = nullptr;
    return SHP_ERR_DEVICE;
  } catch (std::exception& ex) {
    fprintf(stderr, "shp_engine_create: %s\n", ex.what());
    delete e;
    *out = nullptr;
    return SHP_ERR_ARG;
  }
  *out = e;
  return SHP_OK;
}

int shp_engine_create_siddhiql(const char* app_text, const char* query_name, shp_dict* dict, const shp_config* cfg,
                               shp_engine** out) {
  if (!app_text || !dict || !cfg || !out) return SHP_ERR_ARG;
  const int64_t n = shp_compile_siddhiql(app_text, query_name, dict, nullptr, 0);
  if (n < 0) {
    fprintf(stderr, "shp_engine_create_siddhiql: %s\n", shp_compile_last_error());
    *out = nullptr;
    return (int)n;
  }
  std::string prog((size_t)n + 1, '\0');
  // the dictionary already holds this query's constants: the second lowering interns nothing new
  if (shp_compile_siddhiql(app_text, query_name, dict, &prog[0], prog.size()) != n) return SHP_ERR_ARG;
  prog.resize((size_t)n);
  return shp_engine_create(prog.c_str(), cfg, out);
}

// The engine's HIP calls run on its own device whatever thread calls in: HIP's current device
// is per thread (a Java host, or bench.py's worker thread, may call from a thread whose
// current device is another GPU).  The caller's current device is restored on return.
struct DeviceScope {
  int prev = -1;
  explicit DeviceScope(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  int restore_to(int dev) const { return prev >= 0 && prev != dev ? prev : -1; }
};

static int guarded(shp_engine* e, const std::function<int()>& f) {
  const DeviceScope ds(e->cfg.device);
  struct Restore {
    int d;
    ~Restore() {
      if (d >= 0) (void)hipSetDevice(d);
    }
  } restore{ds.restore_to(e->cfg.device)};
  try {
    return f();
  } catch (DevError& de) {
    e->err = de.what();
    return SHP_ERR_DEVICE;
  } catch (OutputError& oe) {
    e->err = oe.what();
    return SHP_ERR_OUTPUT;
  } catch (std::exception& ex) {
    e->err = ex.what();
    return SHP_ERR_ARG;
  }
}

int shp_push_batch(shp_engine* e, const shp_batch* in, shp_matches* out) {
  if (!e || !in || !out) return SHP_ERR_ARG;
  return guarded(e, [&]() {
    int64_t done = 0;
    std::vector<int32_t> keys;
    // one device batch per max_batch events
    int64_t n = in->n;
    if (n > e->cfg.max_batch) return e->fail(SHP_ERR_ARG, "batch larger than max_batch");
    e->stage(in, hipMemcpyHostToDevice);
    int rc = e->run(n, false, nullptr, in->clock != nullptr, in->seq != nullptr);
    if (rc != SHP_OK) return rc;
    e->fetch(out);
    (void)done;
    return SHP_OK;
  });
}

int shp_push_batch_device(shp_engine* e, const shp_batch* in, shp_matches* out) {
  if (!e || !in || !out) return SHP_ERR_ARG;
  return guarded(e, [&]() {
    if (in->n > e->cfg.max_batch) return e->fail(SHP_ERR_ARG, "batch larger than max_batch");
    int rc = e->run(in->n, false, in);  // zero-copy: the kernels read the caller's HBM columns
    if (rc != SHP_OK) return rc;
    e->fill_device(out);
    return SHP_OK;
  });
}

// internal (group.hip's device gather): the last push's records in HBM -- expanded to full records
// for the pair layouts -- and the number of refs; slot_len has stride MAXS on the device
extern "C" int shp_engine_device_records(shp_engine* e, shp_matches* out, int64_t* nrefs) {
  if (!e || !out || !nrefs) return SHP_ERR_ARG;
  return guarded(e, [&]() {
    e->ensure_expanded();
    e->fill_device(out);
    *nrefs = 0;
    if (out->layout != SHP_LAYOUT_AGG && out->m > 0) {
      unsigned long long cnt[2];
      HIP_OK(hipMemcpy(cnt, e->d_mcount, sizeof(cnt), hipMemcpyDeviceToHost));
      *nrefs = (int64_t)cnt[1];
    }
    return SHP_OK;
  });
}

int shp_engine_oldest_live_seq(shp_engine* e, int64_t* out) {
  if (!e || !out) return SHP_ERR_ARG;
  return guarded(e, [&]() {
    *out = e->oldest_live_seq();
    return SHP_OK;
  });
}

int shp_engine_next_due(shp_engine* e, int64_t* out) {
  if (!e || !out) return SHP_ERR_ARG;
  return guarded(e, [&]() {
    const int64_t t = e->next_due();
    if (t == INT64_MAX) return 0;
    *out = t;
    return 1;
  });
}

int shp_push_batch_compact(shp_engine* e, const shp_batch* in, shp_matches* out) {
  if (!e || !in || !out) return SHP_ERR_ARG;
  return guarded(e, [&]() {
    if (in->n > e->cfg.max_batch) return e->fail(SHP_ERR_ARG, "batch larger than max_batch");
    e->stage(in, hipMemcpyHostToDevice);
    int rc = e->run(in->n, false, nullptr, in->clock != nullptr, in->seq != nullptr);
    if (rc != SHP_OK) return rc;
    return e->fetch_compact(out);
  });
}

int shp_stage_batch(shp_engine* e, const shp_batch* in) {
  if (!e || !in) return SHP_ERR_ARG;
  return guarded(e, [&]() { return e->stage_slot(in, nullptr, 0); });
}

int shp_stage_batch_ts32(shp_engine* e, const shp_batch* in, int64_t ts_base, const int32_t* ts_delta) {
  if (!e || !in || (in->n > 0 && !ts_delta)) return SHP_ERR_ARG;
  return guarded(e, [&]() { return e->stage_slot(in, ts_delta, ts_base); });
}

int shp_stage_batch_narrow(shp_engine* e, const shp_batch* in, int64_t ts_base, const int32_t* ts_delta,
                           const uint16_t* key16) {
  if (!e || !in || (in->n > 0 && !ts_delta)) return SHP_ERR_ARG;
  return guarded(e, [&]() { return e->stage_slot(in, ts_delta, ts_base, key16); });
}

int shp_run_staged(shp_engine* e, shp_matches* out) {
  if (!e || !out) return SHP_ERR_ARG;
  return guarded(e, [&]() { return e->run_slot(out); });
}

int shp_fetch_matches(shp_engine* e, shp_matches* out) {
  if (!e || !out) return SHP_ERR_ARG;
  return guarded(e, [&]() {
    e->fetch(out);
    return SHP_OK;
  });
}

int shp_advance_clock(shp_engine* e, int64_t now, shp_matches* out) {
  if (!e || !out) return SHP_ERR_ARG;
  return guarded(e, [&]() {
    // a clock-only event: stream -1, no key; lanes see it as a (possible) onTimeChange call
    int64_t ts = now;
    int32_t st = -1, k = 0;
    std::vector<const void*> cols(MAXCOL, nullptr);
    std::vector<std::vector<uint8_t>> zero(e->comp.P.ncol, std::vector<uint8_t>(8, 0));
    for (int c = 0; c < e->comp.P.ncol; c++) cols[c] = zero[c].data();
    shp_batch b{1, &ts, &k, &st, cols.data(), nullptr};
    e->stage(&b, hipMemcpyHostToDevice);
    int rc = e->run(1, true);
    if (rc != SHP_OK) return rc;
    if (e->fast == 2 && now > e->clock) e->clock = now;
    e->fetch(out);
    return SHP_OK;
  });
}

int64_t shp_snapshot_describe(shp_engine* e, const void* blob, size_t len, char* out, size_t cap) {
  if (!e || !blob) return SHP_ERR_ARG;
  std::string s;
  const int rc = guarded(e, [&]() {
    s = e->describe(blob, len);
    return SHP_OK;
  });
  if (rc != SHP_OK) return rc;
  if (out && cap) {
    const size_t n = std::min(cap - 1, s.size());
    memcpy(out, s.data(), n);
    out[n] = 0;
  }
  return (int64_t)s.size();
}

int shp_engine_num_states(const shp_engine* e) { return e ? e->comp.P.nstates : 0; }
int shp_engine_state_stream(const shp_engine* e, int state) {
  if (!e || state < 0 || state >= e->comp.P.nstates) return -1;
  const DevProg& P = e->comp.P;
  for (int p = 0; p < P.npre; p++)
    if (P.pre[p].stateId == state) return P.pre[p].stream;
  return -1;
}
int shp_engine_path(const shp_engine* e) { return e ? e->fast : -1; }

int64_t shp_engine_stat(const shp_engine* e, const char* which) {
  if (!e || !which) return -1;
  const std::string w = which;
  if (w == "pushes") return e->pushes;
  if (w == "lean_pushes") return e->lean_pushes;
  if (w == "lean_fallbacks") return e->lean_fallbacks;
  if (w == "win_pushes") return e->win_pushes;
  if (w == "win_fallbacks") return e->win_fallbacks;
  if (w == "cseq_wide_reruns") return e->cseq_wide_reruns;
  if (w == "cseq_owner") return e->fast == 3 && e->cs.own ? 1 : 0;  // CHAIN32 pushes on the owner kernels
  if (w == "labs_fallbacks") return e->labs_fallbacks;
  if (w == "labs_segmiss") return e->labs_segmiss;
  if (w == "sweep_r16_reruns") return e->r16_reruns;
  if (w == "match_layout") return e->cfg.match_layout;  // as resolved at create (SHP_LAYOUT_COMPACT)
  if (w == "spill_reruns") return e->spill_reruns;
  if (w == "spilled_owners") return e->fast == 2 ? e->sw.count_spilled() : 0;
  return -1;
}

double shp_last_kernel_ms(const shp_engine* e, const char* which) {
  if (!e) return -1;
  std::string w = which ? which : "total";
  if (w == "partition") return e->last_ms_part;
  if (w == "nfa") return e->last_ms_nfa;
  if (w == "total") return e->last_ms_total;
  return e->kt.get(w);
}

#ifdef SHP_SW_STAMPS
// diagnostic build only: per-owner solve phase cycles of the last push (nown * 8)
int shp_debug_la_stamps(shp_engine* e, unsigned long long* host, int64_t n) {
  if (!e || e->fast != 4 || !e->la.D.stamps) return SHP_ERR_ARG;
  int64_t k = std::min<int64_t>(n, (int64_t)e->la.D.nk * e->la.D.seg * LA_NSTAMP);
  return hipMemcpy(host, e->la.D.stamps, k * 8, hipMemcpyDeviceToHost) == hipSuccess ? (int)(k / LA_NSTAMP)
                                                                                    : SHP_ERR_DEVICE;
}
int shp_debug_sw_stamps(shp_engine* e, unsigned long long* host, int64_t n) {
  if (!e || e->fast != 2 || !e->sw.D.stamps) return SHP_ERR_ARG;
  int64_t k = std::min<int64_t>(n, (int64_t)e->sw.D.nown * 8);
  return hipMemcpy(host, e->sw.D.stamps, k * 8, hipMemcpyDeviceToHost) == hipSuccess ? (int)(k / 8) : SHP_ERR_DEVICE;
}
#endif

int shp_snapshot(shp_engine* e, void** buf, size_t* len) {
  if (!e || !buf || !len) return SHP_ERR_ARG;
  return guarded(e, [&]() {
    e->snapshot(buf, len);
    return SHP_OK;
  });
}

int shp_restore(shp_engine* e, const void* buf, size_t len) {
  if (!e) return SHP_ERR_ARG;
  return guarded(e, [&]() { return e->restore(buf, len); });
}

const char* shp_last_error(const shp_engine* e) { return e ? e->err.c_str() : "null engine"; }

void shp_engine_destroy(shp_engine* e) {
  if (!e) return;
  const DeviceScope ds(e->cfg.device);
  const int back = ds.restore_to(e->cfg.device);
  delete e;
  if (back >= 0) (void)hipSetDevice(back);
}
}
