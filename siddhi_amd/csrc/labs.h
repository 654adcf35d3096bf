// siddhi-hip: the logical-absent path, the playback pattern
//   every (x=X[fx] and y=Y[fy]) -> not Z[fz] for T [within W]        
// over three distinct streams (engine path 4, the default for this shape).
//
// For this shape the LogicalPre/PostStateProcessor pair (LogicalPreStateProcessor.java
// processAndReturn :128-167, addEveryState :65-84), the AbsentStreamPre/PostStateProcessor
// (AbsentStreamPreStateProcessor.java addState :80-103, processAndReturn :257-274, the timer
// process(ComplexEventChunk) :151-227) and the playback Scheduler (Scheduler.java :71-103, 113-127,
// 171-209) reduce, per partition key, to:
//   pend    the one logical partial: an x slot and a y slot (StateEvent with e1 / e2);
//   pairs   completed (x, y) pairs on the absent state's lists, in list order, the last `nae` of
//           them on its new-and-every list;
//   queue   the key's Scheduler queue, a FIFO of notify times, and lastScheduledTime.
// k_labs runs that state event by event for ANY timestamp order (the rule is stated and checked
// against the oracle in tests/labs_exact.py): a queue entry fires at the first send whose clock
// reaches it and sets the clock, behind the entries ahead of it; its timer emits the pending pairs
// at least T old (ts = the entry), drops the expired ones, and re-arms when it emitted nothing.
// k_labs_w runs the ordered special case (a key's events do not go back in time, no event lags the
// clock by T, no clock step beyond T: then the queue stays sorted and a pair fires at its due time)
// a wave per key segment, 64 events a step, and leaves the same state.  Since round 6 a block of a
// key that breaks the ordered case (a ts going back, an event lagging the clock by T) runs the exact
// rule inside k_labs_w, on the whole wave, and the key returns to the ordered formulation once its
// state is regular again; only more than 64 pairs / entries or a clock step beyond T raise LA_SLOW
// (k_labs re-runs the push from the committed state).  Cross-key ties of the playback scheduler's
// TreeMultimap (one state per due time per onTimeChange) are not modelled, as on the general lanes
// (parity-unpinned).  The rings (pairs, queue) start at 8 per key and grow x16 per
// tier in HBM when a push overflows them (the push then re-runs from the committed state).
//
// Batch order: since round 5 a stable multisplit by key (k_la_ms_count, one scan, k_la_ms_scatter:
// one wave per 16k-event segment writes each event's 16-byte record at its key-order position), so
// each key's events are contiguous; up to 4096 keys (LA_MS_BINS), else the 16-byte records are
// sorted with their keys (k_labs_pack2 + one rocPRIM radix sort).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdexcept>

#include "nfa_lane.h"
#include "prog.h"
#include "sweep.h"

namespace shp {

constexpr int LA_WCAP = 8;                       // waiting pairs per key held in LDS (tier 0)
// the reference's per-key timer queue is unbounded (Scheduler.java: a LinkedBlockingQueue): the
// rings grow x16 per tier while device memory lasts (set_tier fails, and the push with it, only
// when the next tier's rings do not fit)
constexpr int LA_TIERS = 6;
constexpr int32_t LA_CAPS[LA_TIERS] = {8, 256, 4096, 65536, 1 << 20, 1 << 24};
constexpr int LA_SB = 16;                        // events of a key staged in LDS per refill

struct __attribute__((aligned(16))) LaEv {  // one event: packed (32 B, one sector), key order, LDS staging
  int64_t ts, clk;
  uint32_t g, v;
  int32_t role;  // its stream's state: 0 x, 1 y, 2 z, -1 none (clock-only, or a stream the query does not read)
  uint32_t n;    // 1: its value is null; 2: its own filter holds (fx for x, fy for y: la_pack_q)
};
constexpr int LA_WIDE = 1 << 26;       // a push's ts / clock leave base +- 2^31 ms or its batch index 2^27:
                                        // the push re-runs with the 32-byte records (not an error)

// the sorted form of LaEv (round 3): 16 bytes, so rocPRIM moves 20-byte (key, record) pairs; ts and
// clock relative to the push's first ts, role + 1, the filter flag and the null flag above the index
struct __attribute__((aligned(16))) LaEv16 {
  int32_t ts, clk;
  uint32_t gs;  // batch index (27 bits) | role + 1 << 27 (2 bits) | filter << 29 | null << 31
  uint32_t v;
};

struct LaTermD {
  int32_t mask;      // outcomes that make the term true: 1 A<B, 2 A==B, 4 A>B, 8 unordered
  int8_t ak, bk;     // operand: 0 const, 1 x, 2 y, 3 z
  int8_t aflt, bflt; // int column promoted to float
  double ac, bc;
};
struct LaPredD {
  int32_t n, combine;
  LaTermD t[2];
};

struct __attribute__((aligned(8))) LaWait {
  int64_t due, xseq, xts, yseq, yts;
  uint32_t xv, yv;
  uint32_t fl;  // 1 x null, 2 y null
  uint32_t pad;
};

// one record of k_labs_w, in the key's region of LabsDev::rec (ceil(kbeg / 2) + 65 k: a key's
// push completes at most ceil(cnt / 2) pairs, and at most 64 were waiting before it)
struct __attribute__((aligned(8))) LaRec {
  int64_t due, xseq, yseq;
  uint32_t flo, fhi;  // the fire event is the first batch index in [flo, fhi] whose clock reaches thr
  int64_t thr;        // (due for the ordered formulation's records; a record of an exactly stepped block
                      // fires where an earlier entry of the same window crossed, or at flo: thr = INT64_MIN)
};

// one timer entry of the key's Scheduler queue (ToNotifyQueue, a FIFO: Scheduler.java:113-127, 332)
struct __attribute__((aligned(8))) LaEnt {
  int64_t t;    // notify time
  int32_t i0;   // the first batch index of the current push it may fire at (0 for carried entries)
  int32_t pad;  // (k_labs_w's exact blocks keep their entries in registers, with the same fields)
};

struct LaPend {
  int64_t xseq, xts, yseq, yts;  // seq -1: slot empty
  uint32_t xv, yv;
  uint32_t fl;    // 1 x null, 2 y null
  int32_t nw;     // pairs held on the absent state's lists
  int32_t wh;     // ring head of the pairs
  int32_t nae;    // the last nae of them are on its new-and-every list (the rest pending)
  int64_t last;   // ts of the key's latest event (INT64_MIN: none)
  int64_t lst;    // AbsentStreamPreStateProcessor's lastScheduledTime
  int32_t ne;     // timer entries queued
  int32_t eh;     // ring head of the entries
  int32_t reg;    // 1: regular -- k_labs_w may run from this state (la_regular)
  int32_t pad;
};

struct LabsDev {
  LaPredD fx, fy, fz;
  int8_t tag[3];     // column tags of x, y, z (T_NULL: no column)
  int8_t pad0;
  int32_t st[3];     // streams of x, y, z
  int32_t col[3];    // their columns (-1 none)
  int32_t sid[3];    // their state ids (slot order of the records)
  int64_t wait, within;
  int32_t nk, cur;
  int32_t wcap, pad1;  // waits ring per key (LA_CAPS[tier])
  LaPend* pend[2];   // nk
  LaWait* wq[2];     // nk * wcap: the pairs on the absent state's lists
  LaWait* wtmp;      // nk * wcap: the count pass's working rings
  LaEnt* fq[2];      // nk * wcap: the timer entries (Scheduler queue)
  LaEnt* ftmp;       // nk * wcap: the count pass's working entry rings
  unsigned long long* maxstep;  // the push's largest clock step after its first event (k_labs_steps)
  uint32_t *cm, *om; // nk: records per key (count pass), their exclusive scan
  // the batch in key order (k_labs_gather): one thread per key then reads its events
  // contiguously; random gathers from 16 waves were bound by address translation (5 us an event)
  LaEv* p_ev;        // the batch's events in arrival order, packed (k_labs_pack: one sector each)
  LaEv* s_ev;        // ... in key order (k_labs_gather)
  int32_t ev16;      // this push's key-order batch is LaEv16 records in s_ev's memory (sort_events)
  int32_t seg;       // k_labs_w segments per key (LA_H; 1: none) -- the slot stride of cm / om / rec
  uint32_t warm;     // warm-up events before a cut (LA_WARM; SHP_LABS_WARM for tests)
  struct LaSnap* snap[2];  // segment boundary states: [0] warmed-up start of segment h, [1] end of h - 1
  int64_t* rc;             // the push's clock at the end of each 64-event block (k_labs_out's coarse search)
  int64_t* segclk;         // multisplit segments: [0, nseg) each one's max clock column, [nseg, 2 nseg) the
                           // clock before it (k_la_seg_clock) -- the fused clock scan
  int32_t pad2;
  unsigned long long* stamps;  // diagnostic build (SHP_SW_STAMPS): k_labs_w phase cycles per key
  LaRec* rec;        // k_labs_w's records, per key region (la_region)
};

// key-order event i of the push, whichever record form the push sorted
// (the 16-byte form's times are relative to the push's first ts, B.ts[0])
__device__ __forceinline__ LaEv la_ev_at(const LabsDev& D, const BatchView& B, int64_t i) {
  if (!D.ev16) return D.s_ev[i];
  const LaEv16 r = reinterpret_cast<const LaEv16*>(D.s_ev)[i];
  const int64_t base = B.ts[0];
  LaEv x;
  x.ts = base + r.ts;
  x.clk = base + r.clk;
  x.g = r.gs & 0x7FFFFFFu;
  x.role = (int32_t)((r.gs >> 27) & 3u) - 1;
  x.n = (r.gs >> 31) | (((r.gs >> 29) & 1u) << 1);
  x.v = r.v;
  return x;
}

// the event's role, and whether its own filter holds (the x / y filters of a k_labs_w shape read only
// their own event: LabsState::wave_ok; for other shapes the flag is unused)
__device__ __forceinline__ int la_pack_role(const LabsDev& D, int st) {
  return st == D.st[0] ? 0 : (st == D.st[1] ? 1 : (st == D.st[2] ? 2 : -1));
}
__device__ __forceinline__ bool la_pack_q(const LabsDev& D, int role, uint32_t v, bool nl);

// event g in arrival order (coalesced reads): ts, clock, batch index, the value of its stream's
// column, stream, null -- one 32-byte record, so the key-order gather reads one sector per event
// (the five columns gathered separately cost five: 9.0 ms per 100M events)
static __global__ void k_labs_pack(LabsDev D, BatchView B, int64_t n) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n; g += (int64_t)gridDim.x * blockDim.x) {
    const int st = B.stream ? B.stream[g] : 0;
    const int role = la_pack_role(D, st);
    const int c = role == 0 ? D.col[0] : (role == 1 ? D.col[1] : (role == 2 ? D.col[2] : -1));
    LaEv x;
    x.ts = B.ts[g];
    x.clk = B.rmax[g];
    x.g = (uint32_t)g;
    x.v = c >= 0 ? ((const uint32_t*)B.cols[c])[g] : 0u;
    x.role = role;
    const bool nl = c < 0 || (B.nulls[c] && B.nulls[c][g]);
    x.n = (nl ? 1u : 0u) | (la_pack_q(D, role, x.v, nl) ? 2u : 0u);
    D.p_ev[g] = x;
  }
}
// the same records with their sort keys (round 3): key id, or `nokey` for clock-only events and
// keys out of range (SWE_KEYS); rocPRIM's radix sort then moves the records with the keys, so the
// key-order batch costs one sort of 36-byte pairs instead of a key sort plus a random gather
static __global__ void k_labs_pack2(LabsDev D, BatchView B, const int32_t* __restrict__ key, int64_t n,
                                    uint32_t nokey, uint32_t* __restrict__ okey, int* err) {
  int e = 0;
  LaEv16* out = reinterpret_cast<LaEv16*>(D.p_ev);
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n; g += (int64_t)gridDim.x * blockDim.x) {
    const int st = B.stream ? B.stream[g] : 0;
    const int role = la_pack_role(D, st);
    const int c = role == 0 ? D.col[0] : (role == 1 ? D.col[1] : (role == 2 ? D.col[2] : -1));
    uint32_t k = 0;
    if (st < 0) {
      k = nokey;
    } else if (B.partitioned) {
      const int32_t x = key[g];
      if (x < 0 || (uint32_t)x >= nokey) {
        e |= 1 << 20;
        k = nokey;
      } else {
        k = (uint32_t)x;
      }
    }
    okey[g] = k;
    const int64_t base = B.ts[0];
    const int64_t dt = B.ts[g] - base, dc = B.rmax[g] - base;
    if (dt != (int64_t)(int32_t)dt || dc != (int64_t)(int32_t)dc || g >= (1ll << 27)) e |= LA_WIDE;
    LaEv16 x;
    x.ts = (int32_t)dt;
    x.clk = (int32_t)dc;
    const bool nl = c < 0 || (B.nulls[c] && B.nulls[c][g]);
    x.v = c >= 0 ? ((const uint32_t*)B.cols[c])[g] : 0u;
    x.gs = ((uint32_t)g & 0x7FFFFFFu) | (uint32_t)(role + 1) << 27 | (la_pack_q(D, role, x.v, nl) ? 1u << 29 : 0u) |
           (nl ? 0x80000000u : 0u);
    out[g] = x;
  }
  if (e) atomicOr(err, e);
}

// ---- the key-order batch by a stable multisplit (round 5), for up to LA_MS_BINS keys: per segment
// of LA_MS_SEG events a key histogram (k_la_ms_count), one scan of the bin-major counts, then one
// wave per segment packs each event's 16-byte record straight to its key-order position
// (k_la_ms_scatter) -- in place of k_labs_pack2 + a radix sort of (key, record) pairs
constexpr int LA_MS_SEG = 16384;
constexpr int LA_MS_BINS = 4096;
__device__ __forceinline__ uint32_t la_bin(const BatchView& B, const int32_t* __restrict__ key, int64_t g, int st,
                                           uint32_t nokey, int& e) {
  if (st < 0) return nokey;
  if (!B.partitioned) return 0u;
  const int32_t x = key[g];
  if (x < 0 || (uint32_t)x >= nokey) {
    e |= 1 << 20;  // SWE_KEYS
    return nokey;
  }
  return (uint32_t)x;
}
// FC (the fused clock): the segment's running clock from its own events (segment-local: without the
// clock carried in from earlier segments) to rmax, and its last value to segmax[seg] for
// k_la_seg_clock.  Event g = lo + 1024 r + 256 w + 64 u + lane (round r, wave w, chunk u): lane-
// contiguous loads, a DPP max-scan per chunk, the waves' totals combined through LDS.
template <bool FC>
static __global__ __launch_bounds__(256) void k_la_ms_count(BatchView B, const int32_t* __restrict__ key, int64_t n,
                                                            uint32_t nokey, int32_t nseg, uint32_t* __restrict__ cnt,
                                                            int* err, int64_t* __restrict__ segmax,
                                                            int64_t* __restrict__ rloc) {
  __shared__ uint32_t h[LA_MS_BINS];
  __shared__ int64_t wtot[4];
  const uint32_t nb = nokey + 1u;
  for (uint32_t b = threadIdx.x; b < nb; b += 256) h[b] = 0;
  __syncthreads();
  int e = 0;
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  int64_t carry = INT64_MIN;  // FC: the segment's clock before this round
  const int64_t lo = (int64_t)blockIdx.x * LA_MS_SEG, hi = min(n, lo + LA_MS_SEG);
  // four events a thread per round, their loads issued before the first LDS add
  for (int64_t g = lo + (FC ? 256 * w + lane : threadIdx.x); g < hi + (FC ? 256 * w + lane : threadIdx.x);
       g += 1024) {
    int st[4], kx[4];
    int64_t c[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int64_t x = g + (FC ? 64 : 256) * u;
      const bool in = x < hi;
      st[u] = in ? (B.stream ? B.stream[x] : 0) : -2;
      kx[u] = in && B.partitioned ? key[x] : 0;
      c[u] = FC && in ? B.tclk[x] : INT64_MIN;
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      if (st[u] == -2) continue;
      uint32_t bin = nokey;
      if (st[u] >= 0) {
        if (!B.partitioned) bin = 0;
        else if (kx[u] < 0 || (uint32_t)kx[u] >= nokey) e |= 1 << 20;  // SWE_KEYS (la_bin)
        else bin = (uint32_t)kx[u];
      }
      atomicAdd(&h[bin], 1u);
    }
    if (FC) {
      int64_t run = INT64_MIN;  // the wave's running max over its chunks
#pragma unroll
      for (int u = 0; u < 4; u++) {
        int64_t v = c[u];
        dpp_scan_steps(lane, [&](auto ctl, bool take) {
          const int64_t y = (int64_t)dpp64<decltype(ctl)::value>((uint64_t)v);
          if (take) v = max(v, y);
        });
        c[u] = max(v, run);
        run = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(c[u] >> 32), 63) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane((int)c[u], 63));
      }
      if (lane == 0) wtot[w] = run;
      __syncthreads();
      int64_t pre = carry;
      for (uint32_t v = 0; v < w; v++) pre = max(pre, wtot[v]);
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int64_t x = g + 64 * u;
        if (x < hi) rloc[x] = max(c[u], pre);
      }
      carry = max(max(carry, max(wtot[0], wtot[1])), max(wtot[2], wtot[3]));
      __syncthreads();  // (wtot is rewritten next round)
    }
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nb; b += 256) cnt[(int64_t)b * nseg + blockIdx.x] = h[b];
  if (FC && threadIdx.x == 0) segmax[blockIdx.x] = carry;
  if (e) atomicOr(err, e);
}
// the clock before each segment: exclusive max-scan of the segment maxima seeded with the carried
// clock (one workgroup; nseg = n / 16384, ~6k at 10^8 events)
static __global__ __launch_bounds__(1024) void k_la_seg_clock(int64_t* __restrict__ segclk, int32_t nseg,
                                                             int64_t clock0) {
  __shared__ int64_t part[1024];
  const int t = threadIdx.x;
  const int per = (nseg + 1023) / 1024;
  const int a = min(nseg, t * per), b = min(nseg, a + per);
  int64_t m = INT64_MIN;
  for (int i = a; i < b; i++) m = max(m, segclk[i]);
  part[t] = m;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {  // inclusive max-scan of the chunk maxima (Hillis-Steele)
    const int64_t o = t >= d ? part[t - d] : INT64_MIN;
    __syncthreads();
    part[t] = max(part[t], o);
    __syncthreads();
  }
  int64_t run = max(clock0, t > 0 ? part[t - 1] : INT64_MIN);
  for (int i = a; i < b; i++) {
    segclk[nseg + i] = run;
    run = max(run, segclk[i]);
  }
}
// FC (the fused clock): rmax holds the segment-local clock (k_la_ms_count<true>); the events it leaves
// below the clock carried into the segment (k_la_seg_clock) are raised to it here -- in place of a
// device-wide max-scan and a clamp
template <bool FC>
static __global__ __launch_bounds__(64) void k_la_ms_scatter(LabsDev D, BatchView B, const int32_t* __restrict__ key,
                                                             int64_t n, uint32_t nokey, int32_t nseg, int bits,
                                                             const uint32_t* __restrict__ off, int* err,
                                                             int64_t* __restrict__ rmax_out) {
  // the keys' cursors.  The fixed 16 KB table also sets the residency: 10 waves a CU measured best
  // (C4 scatter 2.63 ms; 24 waves with only the 4 KB 1000 keys need: 3.29 ms, 6 waves: 2.87, 5: 4.09 --
  // its partial-line writes contend, profiles/r06_scatter_occupancy.txt)
  __shared__ uint32_t cur[LA_MS_BINS];
  const uint32_t nb = nokey + 1u, lane = threadIdx.x;
  const int seg = blockIdx.x;
  for (uint32_t b = lane; b < nb; b += 64) cur[b] = off[(int64_t)b * nseg + seg];
  __syncthreads();
  const uint64_t lt = sw_lanemask_lt();
  LaEv16* out = reinterpret_cast<LaEv16*>(D.s_ev);
  const int64_t base = B.n > 0 ? B.ts[0] : 0;
  int e = 0;
  const int64_t lo = (int64_t)seg * LA_MS_SEG, hi = min(n, lo + LA_MS_SEG);
  // one step of 64 events in arrival order; the next step's columns load before this one is placed.
  // The value column follows from the stream, so the three roles' columns (uniform pointers, one
  // load when they are the same array) are read independently of it and the role picks one.
  const uint32_t* cp[3];
  const uint8_t* np[3];
#pragma unroll
  for (int r = 0; r < 3; r++) {
    cp[r] = D.col[r] >= 0 ? (const uint32_t*)B.cols[D.col[r]] : nullptr;
    np[r] = D.col[r] >= 0 ? B.nulls[D.col[r]] : nullptr;
  }
  const bool onecol = cp[0] == cp[1] && cp[1] == cp[2] && np[0] == np[1] && np[1] == np[2];
  struct Pf {
    int64_t ts, clk;
    int32_t st, k;
    uint32_t v[3];
    uint8_t n[3];
  };
  auto fetch = [&](Pf& f, int64_t g) __attribute__((always_inline)) {
    if (g < hi) {
      f.st = B.stream ? B.stream[g] : 0;
      f.k = B.partitioned ? key[g] : 0;
      f.ts = B.ts[g];
      f.clk = B.rmax[g];  // FC: segment-local (k_la_ms_count<true>), completed in place()
#pragma unroll
      for (int r = 0; r < 3; r++) {
        if (r > 0 && onecol) {
          f.v[r] = f.v[0];
          f.n[r] = f.n[0];
        } else {
          f.v[r] = cp[r] ? cp[r][g] : 0u;
          f.n[r] = cp[r] == nullptr ? 1 : (np[r] ? np[r][g] : 0);
        }
      }
    }
  };
  unsigned long long mxs = 0;  // the push's largest clock step after its first send (k_labs_w's check)
  // the clock before the step's first event
  const int64_t cin = FC ? D.segclk[nseg + seg] : INT64_MIN;  // FC: the clock carried into the segment
  int64_t pclk = FC ? cin : (lo > 0 ? B.rmax[lo - 1] : INT64_MIN);
  auto place = [&](const Pf& f, int64_t g0) __attribute__((always_inline)) {
    const int64_t g = g0 + lane;
    const bool valid = g < hi;
    int64_t clk = f.clk;
    if (FC) {  // rmax[g] = max(the clock carried into the segment, the segment-local clock): rewritten
               // only where the carried clock is larger (a segment's first events, on disordered input)
      clk = max(clk, cin);
      if (valid && clk != f.clk) rmax_out[g] = clk;
    }
    {
      int64_t pc = __shfl_up(clk, 1, 64);
      if (lane == 0) pc = pclk;
      if (valid && g >= 1) mxs = max(mxs, (unsigned long long)(clk - pc));
      pclk = __shfl(clk, 63, 64);
    }
    const int rl = la_pack_role(D, f.st);
    const uint32_t xv = rl == 0 ? f.v[0] : (rl == 1 ? f.v[1] : (rl == 2 ? f.v[2] : 0u));
    const bool nl = rl == 0 ? f.n[0] != 0 : (rl == 1 ? f.n[1] != 0 : (rl == 2 ? f.n[2] != 0 : true));
    uint32_t bin = nokey;
    if (valid && f.st >= 0) {
      if (!B.partitioned) bin = 0;
      else if (f.k < 0 || (uint32_t)f.k >= nokey) bin = nokey;  // (k_la_ms_count raised SWE_KEYS)
      else bin = (uint32_t)f.k;
    }
    const uint64_t peers = sw_match_peers(bin, bits, valid);
    const uint32_t below = (uint32_t)__popcll(peers & lt);
    const bool lead = valid && (peers & lt) == 0;
    const uint32_t ldl = peers ? (uint32_t)__ffsll((unsigned long long)peers) - 1u : 0u;
    uint32_t old = 0;
    if (lead) {
      old = cur[bin];
      cur[bin] = old + (uint32_t)__popcll(peers);
    }
    const uint32_t pos = __shfl(old, (int)ldl, 64) + below;
    if (valid) {
      const int64_t dt = f.ts - base, dc = clk - base;
      if (dt != (int64_t)(int32_t)dt || dc != (int64_t)(int32_t)dc || g >= (1ll << 27)) e |= LA_WIDE;
      LaEv16 x;
      x.ts = (int32_t)dt;
      x.clk = (int32_t)dc;
      x.v = xv;
      x.gs = ((uint32_t)g & 0x7FFFFFFu) | (uint32_t)(rl + 1) << 27 | (la_pack_q(D, rl, xv, nl) ? 1u << 29 : 0u) |
             (nl ? 0x80000000u : 0u);
      out[pos] = x;
    }
  };
  // two register sets, so a step's loads land where the step after next reads them (no copies,
  // whose waits would hold each step for the loads just issued)
  Pf fa{}, fb{};
  fetch(fa, lo + lane);
  for (int64_t g0 = lo; g0 < hi; g0 += 128) {
    fetch(fb, g0 + 64 + lane);
    place(fa, g0);
    if (g0 + 64 >= hi) break;
    fetch(fa, g0 + 128 + lane);
    place(fb, g0 + 64);
  }
  for (int o = 32; o > 0; o >>= 1) mxs = max(mxs, (unsigned long long)__shfl_xor((long long)mxs, o, 64));
  if (lane == 0 && mxs) atomicMax(D.maxstep, mxs);
  if (e) atomicOr(err, e);
}
// each key's run: kbeg = its bin's first position, kcnt = its length (bins 0..nk-1; bin nk: no key)
static __global__ void k_la_ms_bounds(const uint32_t* __restrict__ off, int32_t nseg, uint32_t nk, uint32_t* kbeg,
                                      uint32_t* kcnt) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nk) return;
  const uint32_t a = off[(int64_t)k * nseg], b = off[(int64_t)(k + 1) * nseg];
  kbeg[k] = a;
  kcnt[k] = b - a;
}

// sorted position i <- the packed event perm[i]
static __global__ void k_labs_gather(LabsDev D, const uint32_t* __restrict__ perm, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    D.s_ev[i] = D.p_ev[perm[i]];
}

__device__ __forceinline__ double la_val(uint32_t v, int8_t tag, bool flt) {
  if (tag == T_FLOAT) return (double)__uint_as_float(v);
  const int32_t x = (int32_t)v;
  return flt ? (double)(float)x : (double)x;
}

// The three role values (x, y, z) travel as scalars and are picked with selects: an indexed
// local array would live in scratch memory (measured: k_labs ran 2.4 us per event).
struct LaVals {
  uint32_t v0, v1, v2;
  bool n0, n1, n2;
  int8_t t0, t1, t2;
};
// one operand as a double: every role's value is converted and the kind picks one with selects
// over scalars (a select over the fields of one object became an indexed scratch load)
__device__ __forceinline__ double la_side(int kind, double c, int8_t flt, uint32_t v0, uint32_t v1, uint32_t v2,
                                          int8_t t0, int8_t t1, int8_t t2) {
  const uint32_t v = kind == 1 ? v0 : (kind == 2 ? v1 : v2);
  const int8_t tg = kind == 1 ? t0 : (kind == 2 ? t1 : t2);
  return kind == 0 ? c : la_val(v, tg, flt);
}
__device__ __forceinline__ bool la_term(const LaTermD& t, const LaVals& V) {
  const uint32_t v0 = V.v0, v1 = V.v1, v2 = V.v2;
  const bool n0 = V.n0, n1 = V.n1, n2 = V.n2;
  const double A = la_side(t.ak, t.ac, t.aflt, v0, v1, v2, V.t0, V.t1, V.t2);
  const double B = la_side(t.bk, t.bc, t.bflt, v0, v1, v2, V.t0, V.t1, V.t2);
  const bool nul = (t.ak == 1 && n0) || (t.ak == 2 && n1) || (t.ak == 3 && n2) || (t.bk == 1 && n0) ||
                   (t.bk == 2 && n1) || (t.bk == 3 && n2);
  const int o3 = (A < B ? 1 : 0) | (A == B ? 2 : 0) | (A > B ? 4 : 0);
  return !nul && ((o3 | (o3 == 0 ? 8 : 0)) & t.mask) != 0;  // CompareConditionExpressionExecutor
}

__device__ __forceinline__ bool la_pred(const LaPredD& p, const LaVals& V) {
  if (p.n == 0) return true;
  const bool a = la_term(p.t[0], V);
  if (p.n == 1) return a;
  const bool b = la_term(p.t[1], V);
  return p.combine ? (a || b) : (a && b);
}
__device__ __forceinline__ bool la_pack_q(const LabsDev& D, int role, uint32_t v, bool nl) {
  const LaVals V0{v, v, 0u, nl, nl, true, D.tag[0], D.tag[1], D.tag[2]};
  return (role == 0 && la_pred(D.fx, V0)) || (role == 1 && la_pred(D.fy, V0));
}

// ------------------------------------------------------------------ k_labs: the exact rule
// One thread per key over its events in arrival order, with the state of the reference's
// processors for this shape (tests/labs_exact.py states it and checks it against the oracle for any
// timestamp order):
//   the logical partial (x / y slots);
//   the pairs on the absent state's lists in list order, the last `nae` of them on new-and-every
//     (AbsentStreamPreStateProcessor.addState :80-103 appends there; updateState moves them, stably
//     sorted by ts, StreamPreStateProcessor.java:308-323);
//   the key's Scheduler queue (a FIFO of notify times, Scheduler.java:113-127, 332) and
//     lastScheduledTime.
// A queue entry fires at the first send at or after it was queued whose clock reaches it and that
// sets the clock (TimestampGeneratorImpl.setCurrentTimestamp :105-121: a send below the clock fires
// no timer), behind the entries ahead of it; the timer then runs AbsentStreamPreStateProcessor.process
// (:151-227): new-and-every -> pending, expired pairs dropped, due pairs emitted with ts = the entry,
// lastScheduledTime = clock + T when the clock passed entry + T, and with nothing emitted and
// lastScheduledTime below the entry a re-arm entry + T.  Each key event: the timers its send fires,
// then expireEvents (the partial; the pending list's expired head, every expired new-and-every pair),
// then Z: new-and-every -> pending and each pending pair fz matches is dropped with a queue entry
// ts + T (AbsentStreamPostStateProcessor.process :36-56 -> updateLastArrivalTime :68-78); X / Y: a
// slot fill, and with both slots the pair joins new-and-every with an entry ts + T.
// Two passes: EMIT = false counts each key's records (working rings: wtmp / ftmp), EMIT = true
// writes them at the key's offset (an exclusive scan of the counts) and the state into copy wr.
// The rings grow by capacity tier (E_LIST: the push re-runs at the next one).
__device__ __forceinline__ bool la_expired(int64_t xts, int64_t yts, int64_t t, int64_t W) {
  return W >= 0 && (llabs(xts - t) > W || llabs(yts - t) > W);
}

// the batch index at which a queue entry for time t fires, queued so that it may fire from batch
// index i0 on: the first send in [i0, hi] whose clock reaches t and sets the clock, or hi + 1 (the
// playback clock B.rmax is non-decreasing; a send sets it iff tclk == rmax).  The caller knows the
// clock at hi reached t.
__device__ int64_t la_fire_at(const BatchView& B, int64_t t, int64_t i0, int64_t hi) {
  int64_t a = i0, b = hi;
  while (a < b) {
    const int64_t m = a + ((b - a) >> 1);
    if (B.rmax[m] >= t) b = m;
    else a = m + 1;
  }
  if (a == i0 && (i0 == 0 ? B.clock0 : B.rmax[i0 - 1]) >= t)
    while (a <= hi && B.tclk[a] != B.rmax[a]) a++;  // the clock was already there: the next send that sets it
  return a;
}

// the state k_labs_w may run from (its ordered formulation holds for events that do not go back in
// time): queue sorted, its last entry <= last ts + T and <= lastScheduledTime (no re-arm), pairs in
// ts order at or before the last event, the pending pairs' expiry bounds in list order, the partial's
// slots between the pairs' slots and the last event
__device__ __forceinline__ int la_regular(const LaPend& s, const LaWait* wq, const LaEnt* fq, int msk, int64_t W,
                                          int64_t T) {
  const int64_t Wn = W >= 0 ? W : (1ll << 60);
  for (int i = 1; i < s.ne; i++)
    if (fq[(s.eh + i) & msk].t < fq[(s.eh + i - 1) & msk].t) return 0;
  if (s.ne > 0) {
    const int64_t tmax = fq[(s.eh + s.ne - 1) & msk].t;
    if (s.last == INT64_MIN || tmax > s.last + T || s.lst < tmax) return 0;
  }
  int64_t pdue = INT64_MIN, pd = INT64_MIN, slots = INT64_MIN;
  for (int i = 0; i < s.nw; i++) {
    const LaWait& w = wq[(s.wh + i) & msk];
    if (w.due < pdue || w.due - T > s.last) return 0;
    pdue = w.due;
    const int64_t d = min(w.xts, w.yts) + Wn;
    if (i < s.nw - s.nae && d < pd) return 0;
    pd = max(pd, d);
    slots = max(slots, max(w.xts, w.yts));
  }
  if (s.xseq >= 0 && (s.xts > s.last || s.xts < slots)) return 0;
  if (s.yseq >= 0 && (s.yts > s.last || s.yts < slots)) return 0;
  return 1;
}

// KPB keys per 64-thread block: 64 (a lane per key), or 1 for few keys (a wave per key: the lanes
// of a wave would otherwise run the three streams' branches one after another, and the SIMDs
// beyond 1 / 64 of the keys sit idle)
template <bool EMIT, int KPB>
__global__ __launch_bounds__(64) void k_labs(LabsDev D, BatchView B, MatchOut O, const uint32_t* __restrict__ perm,
                                             const uint32_t* __restrict__ kbeg, const uint32_t* __restrict__ kcnt,
                                             int* err) {
  __shared__ LaEv SB[KPB][LA_SB];
  if (threadIdx.x >= KPB) return;
  const int k = blockIdx.x * KPB + threadIdx.x;
  const uint32_t lane = threadIdx.x;
  const bool live = k < D.nk;
  const int rd = D.cur, wr = D.cur ^ 1;
  const int cap = D.wcap;
  const int msk = cap - 1;
  LaWait* wq = (EMIT ? D.wq[wr] : D.wtmp) + (int64_t)(live ? k : 0) * cap;
  LaEnt* fq = (EMIT ? D.fq[wr] : D.ftmp) + (int64_t)(live ? k : 0) * cap;
  LaPend s{};
  s.xseq = s.yseq = -1;
  s.last = INT64_MIN;
  uint32_t beg = 0, cnt = 0;
  if (live) {
    s = D.pend[rd][k];
    for (int i = 0; i < s.nw; i++) {
      const int r = (s.wh + i) & msk;
      wq[r] = D.wq[rd][(int64_t)k * cap + r];
    }
    for (int i = 0; i < s.ne; i++) {
      const int r = (s.eh + i) & msk;
      LaEnt x = D.fq[rd][(int64_t)k * cap + r];
      x.i0 = 0;  // queued in an earlier push
      fq[r] = x;
    }
    beg = kbeg[k];
    cnt = kcnt[k];
  }
  const int64_t Wn = D.within, Tw = D.wait;
  int e = 0;
  uint32_t nm = 0;
  int64_t mi = 0;
  if (EMIT && live) {
    mi = D.om[k];
    if (k == D.nk - 1) {  // the push's totals
      O.count[0] = (unsigned long long)(mi + D.cm[k]);
      O.count[1] = 2ull * (unsigned long long)(mi + D.cm[k]);
    }
  }
  int64_t gfired = 0;  // batch index of this push's latest firing of the key's queue (a FIFO)
  auto pair_at = [&](int i) -> LaWait& { return wq[(s.wh + i) & msk]; };
  auto push_entry = [&](int64_t t, int64_t i0) {
    if (s.ne >= cap) {
      e |= E_LIST;
      return;
    }
    LaEnt x;
    x.t = t;
    x.i0 = (int32_t)i0;
    x.pad = 0;
    fq[(s.eh + s.ne) & msk] = x;
    s.ne++;
  };
  // updateState: the new-and-every pairs, stably sorted by ts, join the pending list
  auto move_nae = [&]() {
    const int b0 = s.nw - s.nae;
    for (int i = b0 + 1; i < s.nw; i++) {
      const LaWait x = pair_at(i);
      int j = i;
      while (j > b0 && pair_at(j - 1).due > x.due) {
        pair_at(j) = pair_at(j - 1);
        j--;
      }
      pair_at(j) = x;
    }
    s.nae = 0;
  };
  auto emit = [&](const LaWait& w, int64_t et, int64_t g) {
    nm++;
    if (!EMIT) return;
    if (mi >= O.cap || 2 * mi + 2 > O.refcap) {
      e |= E_OUT;
    } else {
      O.key[mi] = B.partitioned ? k : 0;
      O.ts[mi] = et;  // the timer's time (AbsentStreamPreStateProcessor: ev.ts = currentTime)
      O.type[mi] = 0;
      O.pos[mi] = bseq(B, g);
      O.ref_off[mi] = 2 * mi;
      int64_t r = 2 * mi;
      for (int q = 0; q < 3; q++) {
        const bool isx = q == D.sid[0], isy = q == D.sid[1];
        O.slot_len[mi * MAXS + q] = (int16_t)((isx || isy) ? 1 : 0);
        if (isx) O.refs[r++] = w.xseq;
        if (isy) O.refs[r++] = w.yseq;
      }
    }
    mi++;
  };
  // the timer of entry et, fired at batch index g (AbsentStreamPreStateProcessor.process)
  auto process = [&](int64_t et, int64_t g) {
    move_nae();
    int o = 0;
    bool sent = false;
    for (int i = 0; i < s.nw; i++) {
      const LaWait w = pair_at(i);
      if (la_expired(w.xts, w.yts, et, Wn)) continue;
      if (et >= w.due) {
        sent = true;
        emit(w, et, g);
        continue;
      }
      pair_at(o++) = w;
    }
    s.nw = o;
    const int64_t actual = B.rmax[g];
    if (actual > Tw + et) s.lst = actual + Tw;
    if (!sent && s.lst < et) {  // the re-arm
      s.lst = et + Tw;
      push_entry(et + Tw, g);
    }
  };
  // the queue's heads that fire at a send at or before batch index upto (whose clock is clk_upto)
  auto fire = [&](int64_t upto, int64_t clk_upto) {
    while (s.ne > 0) {
      const LaEnt x = fq[s.eh & msk];
      const int64_t i0 = max((int64_t)x.i0, gfired);
      if (i0 > upto || clk_upto < x.t) break;  // (the clock is non-decreasing: not yet reached)
      const int64_t g = la_fire_at(B, x.t, i0, upto);
      if (g > upto) break;
      s.eh = (s.eh + 1) & msk;
      s.ne--;
      gfired = g;
      process(x.t, g);
    }
  };
  auto step = [&](const LaEv& x) {
    fire((int64_t)x.g, x.clk);
    const int64_t t = x.ts;
    s.last = t;
    // expireEvents over every pre of the key (StreamPreStateProcessor.expireEvents :326-361)
    if (Wn >= 0 && ((s.xseq >= 0 && llabs(s.xts - t) > Wn) || (s.yseq >= 0 && llabs(s.yts - t) > Wn))) {
      s.xseq = s.yseq = -1;  // the logical partial expired: `every` re-arms a fresh one
      s.fl = 0;
    }
    if (Wn >= 0) {
      while (s.nw - s.nae > 0 && la_expired(pair_at(0).xts, pair_at(0).yts, t, Wn)) {  // pending: from the head
        s.wh = (s.wh + 1) & msk;
        s.nw--;
      }
      if (s.nae > 0) {  // new-and-every: every expired pair
        const int b0 = s.nw - s.nae;
        int o = b0;
        for (int i = b0; i < s.nw; i++) {
          const LaWait w = pair_at(i);
          if (!la_expired(w.xts, w.yts, t, Wn)) pair_at(o++) = w;
        }
        s.nae = o - b0;
        s.nw = o;
      }
    }
    const int role = x.role;
    if (role < 0) return;
    const bool en = (x.n & 1u) != 0;
    LaVals V{s.xv, s.yv, 0u, (s.fl & 1u) != 0, (s.fl & 2u) != 0, true, D.tag[0], D.tag[1], D.tag[2]};
    if (role == 2) {  // Z: new-and-every -> pending, then each pending pair fz matches is dropped
      move_nae();
      V.v2 = x.v;
      V.n2 = en;
      int o = 0;
      for (int i = 0; i < s.nw; i++) {
        const LaWait w = pair_at(i);
        V.v0 = w.xv;
        V.v1 = w.yv;
        V.n0 = (w.fl & 1u) != 0;
        V.n1 = (w.fl & 2u) != 0;
        if (la_pred(D.fz, V)) {
          s.lst = t + Tw;
          push_entry(t + Tw, (int64_t)x.g + 1);
        } else {
          pair_at(o++) = w;
        }
      }
      s.nw = o;
      return;
    }
    if (role == 0) {
      V.v0 = x.v;
      V.n0 = en;
      if (!la_pred(D.fx, V)) return;
    } else {
      V.v1 = x.v;
      V.n1 = en;
      if (!la_pred(D.fy, V)) return;
    }
    const int64_t seqg = bseq(B, (int64_t)x.g);
    if (role == 0 && s.xseq < 0) {
      s.xseq = seqg;
      s.xts = t;
      s.xv = x.v;
      s.fl = (s.fl & ~1u) | (en ? 1u : 0u);
    } else if (role == 1 && s.yseq < 0) {
      s.yseq = seqg;
      s.yts = t;
      s.yv = x.v;
      s.fl = (s.fl & ~2u) | (en ? 2u : 0u);
    } else {
      return;  // the slot is taken: the partial waits for its partner
    }
    if (s.xseq >= 0 && s.yseq >= 0) {  // the pair completes: new-and-every of the absent state
      if (s.nw >= cap) {
        e |= E_LIST;
      } else {
        LaWait& w = pair_at(s.nw++);
        w.due = t + Tw;
        w.xseq = s.xseq;
        w.xts = s.xts;
        w.yseq = s.yseq;
        w.yts = s.yts;
        w.xv = s.xv;
        w.yv = s.yv;
        w.fl = s.fl;
        w.pad = 0;
        s.nae++;
      }
      s.lst = t + Tw;
      push_entry(t + Tw, (int64_t)x.g + 1);
      s.xseq = s.yseq = -1;  // every: a fresh partial
      s.fl = 0;
    }
  };
  // the key's run (contiguous in key order) is staged in LDS LA_SB events at a time; the step body
  // is not unrolled (copies of it overflowed the instruction cache)
  LaEv* sb = SB[lane];
  for (uint32_t j0 = 0; live && j0 < cnt; j0 += LA_SB) {
#pragma unroll
    for (int q = 0; q < LA_SB; q++) {
      if (j0 + q < cnt) sb[q] = la_ev_at(D, B, (int64_t)beg + j0 + q);
    }
    const uint32_t nq = min((uint32_t)LA_SB, cnt - j0);
#pragma unroll 1
    for (uint32_t q = 0; q < nq; q++) step(sb[q]);
  }
  if (live && B.n > 0) fire(B.n - 1, B.rmax[B.n - 1]);  // the timers the push's last clock reaches
  if (!EMIT) {
    if (live) D.cm[k] = nm;
    return;
  }
  if (live) {
    for (int i = 0; i < s.ne; i++) fq[(s.eh + i) & msk].i0 = 0;
    s.reg = la_regular(s, wq, fq, msk, Wn, Tw);
    D.pend[wr][k] = s;
  }
  if (e) atomicOr(err, e);
}

// ------------------------------------------------------------------ k_labs_w: a wave per key
// The same rule with the key's events taken 64 at a time (one per lane), for filters of x and y
// that read only their own event (LabsState::wave_ok; C4's `S1[price>20]`, `S2[price>20]`):
//   pend    wave-uniform scalars stepped from event to event with ballots: from an empty partial
//           the next qualifying X or Y fills its slot; from a half partial filled at t0 the pair
//           completes at the next qualifying partner unless an event later than t0 + W comes first
//           (that event resets the partial and is then taken from empty) -- one loop trip per
//           fill, completion or reset, not per event;
//   waits   one lane per waiting pair (FIFO in LDS, at most 64): the pair fires at the first event
//           after its completion whose clock reaches the due time (monotone clock: a scan of the
//           64 clocks), and dies at a Z event between completion and firing whose filter holds.
//           Firing follows completion order, so the emitted records keep the FIFO order.
// More than 64 waiting pairs in a key raise LA_SLOW: the engine re-runs the push with k_labs.
constexpr int LA_SLOW = 1 << 28;
constexpr int LA_SEGMISS = 1 << 27;  // a warmed-up segment start differed from the state before it: re-run unsegmented
constexpr int LA_BOUND = 1 << 29;  // a key's records would leave its region (a broken invariant: fail, never write)

__device__ __forceinline__ int64_t la_rl64(int64_t x, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)x >> 32), l);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

__host__ __device__ __forceinline__ int64_t la_region(uint32_t kb, int k) { return (int64_t)((kb + 1u) >> 1) + 65ll * k; }

// fz for one waiting pair: the x / y sides of each term converted once (per block), the z side per Z
struct LaKill {
  double a[2], b[2];
  bool nul[2];
};
__device__ __forceinline__ LaKill la_kill_pre(const LaPredD& p, const LaWait& w, int8_t t0, int8_t t1, int8_t t2) {
  LaKill K{};
  const bool xn = (w.fl & 1u) != 0, yn = (w.fl & 2u) != 0;
#pragma unroll
  for (int i = 0; i < 2; i++) {
    if (i < p.n) {
      const LaTermD& t = p.t[i];
      K.a[i] = la_side(t.ak, t.ac, t.aflt, w.xv, w.yv, 0u, t0, t1, t2);
      K.b[i] = la_side(t.bk, t.bc, t.bflt, w.xv, w.yv, 0u, t0, t1, t2);
      K.nul[i] = (t.ak == 1 && xn) || (t.ak == 2 && yn) || (t.bk == 1 && xn) || (t.bk == 2 && yn);
    }
  }
  return K;
}
__device__ __forceinline__ bool la_kill(const LaPredD& p, const LaKill& K, double zd0, double zd1, bool zn) {
  if (p.n == 0) return true;
  bool r[2] = {false, false};
#pragma unroll
  for (int i = 0; i < 2; i++) {
    if (i < p.n) {
      const LaTermD& t = p.t[i];
      const double A = t.ak == 3 ? (t.aflt ? zd1 : zd0) : K.a[i];
      const double Bv = t.bk == 3 ? (t.bflt ? zd1 : zd0) : K.b[i];
      const bool nul = K.nul[i] || ((t.ak == 3 || t.bk == 3) && zn);
      const int o3 = (A < Bv ? 1 : 0) | (A == Bv ? 2 : 0) | (A > Bv ? 4 : 0);
      r[i] = !nul && ((o3 | (o3 == 0 ? 8 : 0)) & t.mask) != 0;
    }
  }
  return p.n == 1 ? r[0] : (p.combine ? (r[0] || r[1]) : (r[0] && r[1]));
}

// one pass: records into the key's region of D.rec, the key's count into D.cm, the state into
// copy wr; k_labs_out then writes the push's records contiguously.
// The state it leaves is the exact rule's (k_labs; tests/labs_exact.py FastC4 states the formulas
// and checks them against the exact rule, state included): when the key's events do not go back in
// time, no event lags the clock by T or more and the clock never steps by more than T, the
// Scheduler queue stays sorted and every entry the clock reached has fired, so per pair P
// (completed at c, slots' earliest ts m, due = c + T, D = m + W):
//   E_D   = min(due, the first queued entry > max(D, clock(c)) at c): P leaves the pending list --
//           emitted when due <= D, else expired -- at the first key event q > c with clock(q) >= E_D
//           or ts(q) > D (or when the push's last clock reaches E_D);
//   kill  = the first Z event in (c, that q) whose fz holds; it queues an entry ts + T;
//   P is still on new-and-every at the end iff no Z event of the key and no firing of its queue
//   came after c;
// lastScheduledTime = ts + T of the key's last completion or kill; the queue keeps every entry past
// the last clock.  A push or state outside that raises LA_SLOW (k_labs re-runs it exactly).
// The queue lives in registers, entry i in lane i (sorted); the entries a block queues are counted
// per event lane (a completion, or the pairs a Z event kills), all at that event's ts + T.
constexpr int LA_WF = 64;  // queue entries k_labs_w holds (one per lane)
// diagnostic build (SHP_SW_STAMPS): per key, phase cycles 0 load, 1 partial, 2 doomed E_D, 3 leave
// search, 4 settle, 5 queue, 8 Z kills, 9 firings, 13 exact blocks (15: their timer firings); counts
// 6 pairs, 7 events, 10 kill rounds, 11 Z events, 12 events by the exact rule, 14 run by the exact variant
constexpr int LA_NSTAMP = 16;

// Segments (round 5).  With few keys (one wave each cannot fill the CUs) a key's events are cut into
// up to LA_H segments of whole 64-event blocks, one wave each.  The state at a cut depends only on the
// key's recent events (a pair leaves at its due or when its slots pass W, a timer fires once the
// clock reaches it, the partial expires after W), so the wave of segment h > 0 starts from the empty
// state LA_WARM events before its cut and runs them without writing records; at the cut it stores
// the state it reached, the wave of segment h - 1 stores the state it ends with, and k_labs_segcheck
// compares the two field by field.  Any difference raises LA_SEGMISS and the engine re-runs the push
// unsegmented, so the records and the state are always the sequential kernel's.  Only the last
// segment settles the push's end and writes the key's state.
constexpr int LA_H = 4;
constexpr uint32_t LA_MINSEG = 4096;   // events per segment at least
constexpr uint32_t LA_WARM = 4 * 64;   // warm-up events before a cut
constexpr int LA_SEG_MAXKEYS = 4096;   // segments only while keys are this few
struct LaSnap {
  int64_t xseq, xts, yseq, yts, last, lsched, lo;
  uint32_t xv, yv, fl, hxy, nal, nef;
  uint32_t xm, xnae;   // exact mode (round 6): its new-and-every count
  uint64_t qat;        // exact mode: the entries already reached when queued
  LaWait A[64];
  int64_t ed[64];
  int64_t qe[64];
  uint8_t nae[64];
};
__host__ __device__ __forceinline__ int la_nseg(uint32_t cnt, int H) {
  return H <= 1 ? 1 : (int)min((uint32_t)H, max(1u, cnt / LA_MINSEG));
}
__host__ __device__ __forceinline__ uint32_t la_segb(uint32_t cnt, int hk, int i) {  // cut i of hk segments
  return i >= hk ? cnt : (uint32_t)(((uint64_t)cnt * (uint64_t)i / (uint64_t)hk) & ~63ull);
}

// FZ1: fz is one term comparing the Z event's value with a constant or a slot's value (C4's
// `S3[price > e1.price]`): the Z side is converted once per event, the other once per pair, and the
// kill test in the pairs' walk over the Z events is one double compare (la_fz1_side / la_kill1)
__host__ __device__ inline bool la_fz1(const LaPredD& p) {
  return p.n == 1 && ((p.t[0].ak == 3) != (p.t[0].bk == 3));
}
// XB: the exact blocks (round 6) are a second variant of the kernel, so the ordered formulation's
// variant keeps its registers: it marks a (key, segment) whose blocks break the formulation
// (cm = LA_XMARK) and stops there; the XB variant, launched after it, re-runs only the marked ones
// from the committed state, the broken blocks by the exact rule (the records and state of the others
// stand).
constexpr uint32_t LA_XMARK = 0xFFFFFFFFu;
// The exact variant runs only the marked slots, wave-wide; unlimited it takes 143 registers (three
// waves a SIMD).  Built for four (128) it takes C4 at 1 % disorder from 18.5 to 14.5 ms (five: 15.9,
// six: 18.4 -- their spills), while a limit on the ordered variant only costs it (five: 7.8 -> 8.5 ms;
// profiles/r06_wpe_ab.txt)
#ifndef SHP_LABS_XWPE
#define SHP_LABS_XWPE 4
#endif
template <bool FZ1, bool XB>
static __global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(XB ? SHP_LABS_XWPE : 1))) void k_labs_w(LabsDev D, BatchView B, const uint32_t* __restrict__ perm,
                                               const uint32_t* __restrict__ kbeg, const uint32_t* __restrict__ kcnt,
                                               int H, int* err) {
  __shared__ LaWait A[64];      // the pairs on the absent state's lists, list (= completion) order
  __shared__ int32_t Ac[64];    // completing lane in the current block (-1: an earlier block)
  __shared__ int64_t Aed[64];   // E_D of each pair
  __shared__ uint8_t Anae[64];  // on new-and-every (no Z event and no firing since its completion)
  __shared__ int32_t Ec[64];    // per event lane of the block: entries it queued (completion + kills)
  __shared__ int64_t Es[64];    // staging of the queue's new order
  const int S = D.seg;  // slot stride
  const int k = blockIdx.x / S, h = blockIdx.x % S, ks = blockIdx.x;
  if (k >= D.nk) return;
  if (XB && D.cm[ks] != LA_XMARK) return;  // (the ordered variant ran this one through)
  const int lane = (int)threadIdx.x;
  const uint32_t beg = kbeg[k], cnt = kcnt[k];
  const int hk = la_nseg(cnt, H);
  if (h >= hk) {  // (an unused slot: no records)
    if (lane == 0) D.cm[ks] = 0;
    return;
  }
  const uint32_t s_beg = la_segb(cnt, hk, h), s_end = la_segb(cnt, hk, h + 1);
  const uint32_t w_beg = h == 0 ? 0u : (s_beg > D.warm ? s_beg - D.warm : 0u);
  const bool lastseg = h == hk - 1;
  const uint64_t lt = sw_lanemask_lt();
  const int rd = D.cur, wr = rd ^ 1;
  const int cap = D.wcap, msk = cap - 1;
  LaPend s0{};
  if (h == 0) {
    s0 = D.pend[rd][k];
  } else {  // the empty state (k_labs_init's)
    s0.xseq = s0.yseq = -1;
    s0.last = INT64_MIN;
    s0.reg = 1;
  }
  const bool useW = D.within >= 0;
  const int64_t Wn = D.within, Tw = D.wait;
  const int64_t Wb = useW ? Wn : (1ll << 60);  // D = min slot ts + Wb
  int nal = s0.nw;
  int nef = s0.ne;
  const int64_t mstep = (int64_t)*D.maxstep;  // the push's largest clock step after its first send
  {  // capacity and the push's clock steps (else k_labs re-runs the push)
    bool slow = nal > 64 || nef > LA_WF;
    if (!slow && nef > 0 && B.n > 0 && B.rmax[0] - B.clock0 > Tw) slow = true;  // a step at the first send
    if (!slow && mstep > Tw) slow = true;                                       // a step at a later send
    if (slow) {
      if (lane == 0) {
        D.cm[ks] = 0;  // k_labs_out runs before the host sees LA_SLOW
        atomicOr(err, LA_SLOW);
      }
      return;
    }
  }
  int64_t qe = lane < nef ? D.fq[rd][(int64_t)k * cap + ((s0.eh + lane) & msk)].t : INT64_MAX;  // the queue
  // Exact blocks (round 6).  A block the ordered formulation does not cover (a key's ts going back, an
  // event lagging the clock by T) runs the exact rule of k_labs instead, event by event on the whole wave:
  // the pairs stay in A[] in list order (the last xnae on new-and-every), the Scheduler FIFO in qe (entry
  // j in lane j, unsorted) with, per entry, its first batch index Qi0 and whether the clock had already
  // reached it when it was queued (Qat: it fires at the next send that sets the clock).  After each such
  // block the state goes back to the ordered formulation when it is regular there (to_wave), so only
  // the disordered stretches of a key pay for the exact rule.  A firing's send is kept as a window and
  // a clock threshold (the first send from plo on whose clock reaches pthr) and found by k_labs_out, as
  // for the ordered blocks' records; it is searched here only when the clock at it decides
  // lastScheduledTime.  The carried state starts here too and converts when regular.
  int32_t Qi0 = 0;
  bool Qat = lane < nef && qe <= B.clock0;
  LaWait P{};          // exact mode: pair `lane` of the absent state's lists (list order), in registers
  int xnae = s0.nae;
  bool xm = true;      // exact mode (wave-uniform)
  bool xover = false;  // exact mode outgrew 64 pairs or entries: the push re-runs on k_labs
  Ec[lane] = 0;
  if (lane < nal) {
    const LaWait w = D.wq[rd][(int64_t)k * cap + ((s0.wh + lane) & msk)];
    A[lane] = w;
    Ac[lane] = -1;
    P = w;
  }
  __syncthreads();
  LaRec* rec = D.rec + la_region(beg + s_beg, ks);
  const uint32_t rcap = (s_end - s_beg + 1u) / 2u + 64u;  // the region's records (la_region)
  bool emit_on = w_beg == s_beg;  // (warm-up blocks write no records)
  const int8_t t0g = D.tag[0], t1g = D.tag[1], t2g = D.tag[2];
  int e = 0;
  uint32_t nm = 0;
  // the logical partial (wave-uniform)
  bool hx = s0.xseq >= 0, hy = s0.yseq >= 0;
  int64_t xseq = s0.xseq, xts = s0.xts, yseq = s0.yseq, yts = s0.yts;
  uint32_t xv = s0.xv, yv = s0.yv, fl = s0.fl;
  int64_t last = s0.last;
  int64_t lsched = s0.lst;  // lastScheduledTime
  int64_t lo = 0;  // first batch index a timer can fire at (after the key's previous event)
  int64_t lclk = B.clock0;  // the clock at the key's previous event
  // the pairs (one per lane) leave (left: in [flo, fhi]) -- emitted when within W of their due
  // time -- or are killed; the survivors are compacted in order
  auto settle = [&](bool left, bool killed, bool tonae, int64_t flo, int64_t fhi, LaWait w, int64_t ed)
                    __attribute__((always_inline)) {
    const bool ok = emit_on && lane < nal && left && !killed &&
                    (!useW || (llabs(w.xts - w.due) <= Wn && llabs(w.yts - w.due) <= Wn));
    const uint64_t em = __ballot(ok);
    if (nm + (uint32_t)__popcll(em) > rcap) e |= LA_BOUND;
    else if (ok) {
      LaRec r;
      r.due = w.due;
      r.xseq = w.xseq;
      r.yseq = w.yseq;
      r.flo = (uint32_t)flo;
      r.fhi = (uint32_t)fhi;
      r.thr = w.due;
      rec[nm + (uint32_t)__popcll(em & lt)] = r;
    }
    nm += (uint32_t)__popcll(em);
    const bool surv = lane < nal && !left && !killed;
    const uint64_t sm = __ballot(surv);
    __syncthreads();  // every lane holds its pair before the compaction writes
    if (surv) {
      const int d = __popcll(sm & lt);
      A[d] = w;
      Ac[d] = -1;
      Aed[d] = ed;
      Anae[d] = tonae ? 1 : 0;
    }
    nal = __popcll(sm);
    __syncthreads();
  };
#ifdef SHP_SW_STAMPS  // diagnostic build: wave cycles per phase, and counts (trips, pairs, Z events)
  unsigned long long lst[LA_NSTAMP] = {};
  uint64_t lsp = clock64();
#define LA_STAMP(x)               \
  do {                            \
    const uint64_t t_ = clock64(); \
    lst[x] += t_ - lsp;           \
    lsp = t_;                     \
  } while (0)
#define LA_COUNT(x, v) lst[x] += (v)
#else
#define LA_STAMP(x) \
  do {              \
  } while (0)
#define LA_COUNT(x, v) \
  do {                 \
  } while (0)
#endif
  // ---- exact blocks: conversions between the two forms and the exact rule (k_labs) on the wave
  // the exact state -> the ordered formulation's, when regular after the key's event at clock clkl
  // (la_regular's conditions, every entry past the clock, every pair's E_D past it)
  auto to_wave = [&](int64_t clkl) __attribute__((always_inline)) {
    const LaWait w = P;
    const int64_t qp = __shfl_up(qe, 1, 64);
    bool bad = lane >= 1 && lane < nef && qe < qp;   // the queue sorted
    bad |= lane < nef && (qe <= clkl || Qat);          // every entry the clock reached has fired
    const int64_t dp = __shfl_up(w.due, 1, 64);
    bad |= lane >= 1 && lane < nal && w.due < dp;      // the pairs by due, each completed by the last event
    bad |= lane < nal && w.due - Tw > last;
    const int64_t dd = min(w.xts, w.yts) + Wb;
    const int64_t ddp = __shfl_up(dd, 1, 64);
    bad |= lane >= 1 && lane < nal - xnae && dd < ddp; // the pending pairs' expiry bounds in list order
    int64_t sl = lane < nal ? max(w.xts, w.yts) : INT64_MIN;
    for (int o = 32; o > 0; o >>= 1) sl = max(sl, (int64_t)__shfl_xor(sl, o, 64));
    bool ubad = false;
    if (nef > 0) {
      const int64_t tmax = la_rl64(qe, nef - 1);
      ubad = last == INT64_MIN || tmax > last + Tw || lsched < tmax;
    }
    ubad |= hx && (xts > last || xts < sl);
    ubad |= hy && (yts > last || yts < sl);
    int64_t ed = w.due;  // E_D: the first queued entry past D
    for (int i = 0; i < nef; i++) {
      const int64_t t = la_rl64(qe, i);
      if (t > dd) ed = min(ed, t);
    }
    bad |= lane < nal && ed <= clkl;
    if (ubad || __ballot(bad)) return;
    if (lane < nal) {
      A[lane] = w;
      Aed[lane] = ed;
      Anae[lane] = lane >= nal - xnae ? 1 : 0;
      Ac[lane] = -1;
    }
    __syncthreads();
    xm = false;
  };
  // the ordered formulation's state -> the exact rule's (its entries all past the clock)
  auto to_exact = [&]() __attribute__((always_inline)) {
    const uint64_t m = __ballot(lane < nal && Anae[lane]);
    const uint64_t all = nal >= 64 ? ~0ull : ((1ull << nal) - 1ull);
    const uint64_t notq = all & ~m;
    xnae = notq ? nal - 1 - (63 - __builtin_clzll(notq)) : nal;
    Qi0 = (int32_t)lo;
    Qat = false;
    P = lane < nal ? A[lane] : LaWait{};
    xm = true;
  };
  // the pairs in registers move between lanes through A[] (a scratch in exact mode).  The workgroup is
  // one wave, whose LDS operations complete in order: a wave-scope fence between the stores and the
  // loads is the whole synchronisation (as in sl_expand_block)
  auto xcompact = [&](uint64_t keep) __attribute__((always_inline)) {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if ((keep >> lane) & 1ull) A[__popcll(keep & lt)] = P;
    nal = __popcll(keep);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    P = lane < nal ? A[lane] : LaWait{};
  };
  // updateState: the new-and-every pairs, stably sorted by due, join the pending list
  auto xmove_nae = [&]() __attribute__((always_inline)) {
    if (xnae > 1) {
      const int b0 = nal - xnae;
      const bool in = lane >= b0 && lane < nal;
      int r = b0;
      for (int j = b0; j < nal; j++) {
        const int64_t dj = la_rl64(P.due, j);
        if (in && (dj < P.due || (dj == P.due && j < lane))) r++;
      }
      if (__ballot(in && r != (int)lane)) {  // (already in order: nothing moves)
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (in) A[r] = P;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (in) P = A[lane];
      }
    }
    xnae = 0;
  };
  auto xpush = [&](int64_t t, int64_t i0, bool at) __attribute__((always_inline)) {
    if (nef >= LA_WF) {
      xover = true;
      return;
    }
    if (lane == nef) {
      qe = t;
      Qi0 = (int32_t)i0;
      Qat = at;
    }
    nef++;
  };
  auto xpop = [&]() __attribute__((always_inline)) {
    qe = __shfl_down(qe, 1, 64);
    Qi0 = __shfl_down(Qi0, 1, 64);
    Qat = __shfl_down((int)Qat, 1, 64) != 0;
    nef--;
    if (lane >= nef) {
      qe = INT64_MAX;
      Qat = false;
    }
  };
  // the first batch index in [a, b] whose clock reaches thr (64 lanes over the coarse clock, then over
  // the block's clocks)
  auto xresolve = [&](int64_t a, int64_t b, int64_t thr) __attribute__((always_inline)) -> int64_t {
    int64_t jb = a >> 6;
    const int64_t je = b >> 6;
    for (;;) {
      const int64_t j = jb + lane;
      const uint64_t m = __ballot(j <= je && D.rc[j] >= thr);
      if (m) {
        jb += __builtin_ctzll(m);
        break;
      }
      jb += 64;
      if (jb > je) {
        jb = je;
        break;
      }
    }
    const int64_t i = (jb << 6) + lane;
    const uint64_t m = __ballot(i >= a && i <= b && B.rmax[i] >= thr);
    return m ? (jb << 6) + __builtin_ctzll(m) : b;
  };
  // AbsentStreamPreStateProcessor.process for the timer of entry et, at the firing send: a known
  // one (pex: pidx, its clock pclk) or the first send from plo on whose clock reaches pthr (<= upto)
  auto xprocess = [&](int64_t et, bool pex, int64_t pidx, int64_t pclk, int64_t plo, int64_t pthr, int64_t upto)
                      __attribute__((always_inline)) {
    xmove_nae();
    const LaWait w = P;
    const bool in = lane < nal;
    const bool ex = in && la_expired(w.xts, w.yts, et, Wn);
    const bool emt = in && !ex && et >= w.due;
    const uint64_t em = __ballot(emt);
    if (emit_on && em) {
      const uint32_t c = (uint32_t)__popcll(em);
      if (nm + c > rcap) {
        e |= LA_BOUND;
      } else if (emt) {
        LaRec r;
        r.due = et;  // the match's ts: the timer's time
        r.xseq = w.xseq;
        r.yseq = w.yseq;
        r.flo = (uint32_t)(pex ? pidx : plo);
        r.fhi = (uint32_t)(pex ? pidx : upto);
        r.thr = pex ? INT64_MIN : pthr;
        rec[nm + (uint32_t)__popcll(em & lt)] = r;
      }
      nm += c;
    }
    const uint64_t keep = __ballot(in && !ex && !emt);
    if (__popcll(keep) != nal) xcompact(keep);
    if (pex && pclk > Tw + et) lsched = pclk + Tw;
    if (!em && lsched < et) {  // the re-arm
      lsched = et + Tw;
      xpush(et + Tw, pex ? pidx : plo, false);
    }
  };
  // the queue's heads that fire at a send in the window [lo, upto] (the clock at upto: clk_upto), in
  // FIFO order: an entry fires at the first send that sets the clock to or past it, behind the entries
  // ahead of it (Scheduler.sendTimerEvents; k_labs' fire / la_fire_at)
  auto xfire = [&](int64_t upto, int64_t clk_upto) __attribute__((always_inline)) {
    bool hp = false, pex = false;
    int64_t pidx = 0, pclk = 0, plo = 0, pthr = 0;
    while (nef > 0 && !xover) {
      const int64_t t = la_rl64(qe, 0);
      const bool at = __builtin_amdgcn_readlane((int)Qat, 0) != 0;
      bool cex = pex;
      int64_t cidx = pidx, cclk = pclk, clo = plo, cthr = pthr;
      if (at) {  // reached when queued: the next send that sets the clock (or the previous firing's)
        if (!hp) {
          int64_t a = -1;
          for (int64_t c0 = lo; c0 <= upto && a < 0; c0 += 64) {
            const int64_t i = c0 + lane;
            const uint64_t m = __ballot(i <= upto && B.tclk[i] == B.rmax[i]);
            if (m) a = c0 + __builtin_ctzll(m);
          }
          if (a < 0) break;
          cex = true;
          cidx = a;
          cclk = B.rmax[a];
        }
      } else {
        if (!hp) {
          cex = false;
          clo = lo;
          cthr = t;
        } else if (pex) {
          if (pclk < t) {
            cex = false;
            clo = pidx + 1;
            cthr = t;
          }
        } else if (t > pthr) {
          cthr = t;
        }
        if (!cex && clk_upto < cthr) break;
      }
      xpop();
      hp = true;
      pex = cex;
      pidx = cidx;
      pclk = cclk;
      plo = clo;
      pthr = cthr;
      if (!pex && pthr + mstep > t + Tw) {  // the clock at the send may pass t + T: find the send
        pidx = xresolve(plo, upto, pthr);
        pclk = B.rmax[pidx];
        pex = true;
      }
      xprocess(t, pex, pidx, pclk, plo, pthr, upto);
    }
  };
  // one key event q of the block (lane q's registers) by the exact rule (k_labs' step)
  auto xstep = [&](int q, int64_t ts_, int64_t clk_, uint32_t g_, uint32_t v_, int role_, bool en_, bool qf_)
                   __attribute__((always_inline)) {
    const int64_t t = la_rl64(ts_, q), xc = la_rl64(clk_, q);
    const uint32_t xg = (uint32_t)__builtin_amdgcn_readlane((int)g_, q);
    const uint32_t xv_ = (uint32_t)__builtin_amdgcn_readlane((int)v_, q);
    const int xr = __builtin_amdgcn_readlane(role_, q);
    const bool xen = __builtin_amdgcn_readlane((int)en_, q) != 0;
    const bool xqf = __builtin_amdgcn_readlane((int)qf_, q) != 0;
    LA_STAMP(13);
    xfire((int64_t)xg, xc);
    LA_STAMP(15);
    lo = (int64_t)xg + 1;
    lclk = xc;
    last = t;
    if (xover) return;
    // expireEvents: the partial; the pending list's expired head, every expired new-and-every pair
    if (useW && ((hx && llabs(xts - t) > Wn) || (hy && llabs(yts - t) > Wn))) {
      hx = hy = false;
      xseq = yseq = -1;
      fl = 0;
    }
    if (useW && nal > 0) {
      const uint64_t exm = __ballot(lane < nal && la_expired(P.xts, P.yts, t, Wn));
      if (exm) {
        const int np = nal - xnae;
        const uint64_t pm = np >= 64 ? ~0ull : ((1ull << np) - 1ull);
        const uint64_t all = nal >= 64 ? ~0ull : ((1ull << nal) - 1ull);
        const uint64_t live = ~exm & pm;
        const int nh = live ? __builtin_ctzll(live) : np;
        const uint64_t drop = (nh >= 64 ? ~0ull : ((1ull << nh) - 1ull)) | (exm & all & ~pm);
        const uint64_t keep = all & ~drop;
        if (keep != all) {
          const int nk = __popcll(keep & ~pm);
          xcompact(keep);
          xnae = nk;
        }
      }
    }
    if (xr < 0) return;
    if (xr == 2) {  // Z: new-and-every -> pending, then each pending pair fz matches is dropped
      xmove_nae();
      const LaVals V{P.xv, P.yv, xv_, (P.fl & 1u) != 0, (P.fl & 2u) != 0, xen, t0g, t1g, t2g};
      const uint64_t km = __ballot(lane < nal && la_pred(D.fz, V));
      if (km) {
        lsched = t + Tw;
        for (int i = __popcll(km); i > 0; i--) xpush(t + Tw, (int64_t)xg + 1, xc >= t + Tw);
        const uint64_t all = nal >= 64 ? ~0ull : ((1ull << nal) - 1ull);
        xcompact(all & ~km);
      }
      return;
    }
    if (!xqf) return;  // X / Y: its own filter (la_pack_q)
    const int64_t sq = bseq(B, (int64_t)xg);
    const bool en1 = xen;
    if (xr == 0 && !hx) {
      hx = true;
      xseq = sq;
      xts = t;
      xv = xv_;
      fl = (fl & ~1u) | (en1 ? 1u : 0u);
    } else if (xr == 1 && !hy) {
      hy = true;
      yseq = sq;
      yts = t;
      yv = xv_;
      fl = (fl & ~2u) | (en1 ? 2u : 0u);
    } else {
      return;  // the slot is taken: the partial waits for its partner
    }
    if (hx && hy) {  // the pair completes: new-and-every of the absent state, an entry t + T
      if (nal >= 64) {
        xover = true;
        return;
      }
      if (lane == nal) {
        P.due = t + Tw;
        P.xseq = xseq;
        P.xts = xts;
        P.yseq = yseq;
        P.yts = yts;
        P.xv = xv;
        P.yv = yv;
        P.fl = fl;
        P.pad = 0;
      }
      nal++;
      xnae++;
      lsched = t + Tw;
      xpush(t + Tw, (int64_t)xg + 1, xc >= t + Tw);
      hx = hy = false;
      xseq = yseq = -1;
      fl = 0;
    }
  };
  to_wave(B.clock0);  // the carried state: the ordered formulation's when regular
  if (!XB && xm) {  // (the exact variant takes this one)
    if (lane == 0) D.cm[ks] = LA_XMARK;
    return;
  }
  // the key's events 64 at a time; the next block's loads are issued before this one is worked
  int64_t n_ts = 0, n_clk = 0;
  uint32_t n_g = 0, n_v = 0, n_n = 1;
  int32_t n_st = -1;
  auto fetch = [&](uint32_t j0) __attribute__((always_inline)) {
    if (j0 + (uint32_t)lane < s_end) {
      const LaEv x = la_ev_at(D, B, (int64_t)beg + j0 + lane);
      n_ts = x.ts;
      n_clk = x.clk;
      n_g = x.g;
      n_v = x.v;
      n_st = x.role;
      n_n = x.n;
    }
  };
  // the state at a cut, for k_labs_segcheck (between blocks: the pairs are compacted, Ac = -1, Ec = 0)
  auto dump = [&](LaSnap* sp) __attribute__((always_inline)) {
    if (lane == 0) {
      sp->xseq = hx ? xseq : -1;
      sp->yseq = hy ? yseq : -1;
      sp->xts = hx ? xts : 0;
      sp->yts = hy ? yts : 0;
      sp->xv = hx ? xv : 0u;
      sp->yv = hy ? yv : 0u;
      sp->fl = fl;
      sp->hxy = (hx ? 1u : 0u) | (hy ? 2u : 0u);
      sp->last = last;
      sp->lsched = lsched;
      sp->lo = lo;
      sp->nal = (uint32_t)nal;
      sp->nef = (uint32_t)nef;
      sp->xm = xm ? 1u : 0u;
      sp->xnae = xm ? (uint32_t)xnae : 0u;
    }
    const uint64_t qa = __ballot(xm && lane < nef && Qat);
    if (lane == 0) sp->qat = qa;
    if (lane < nal) {
      sp->A[lane] = xm ? P : A[lane];
      sp->ed[lane] = xm ? 0 : Aed[lane];
      sp->nae[lane] = xm ? 0 : Anae[lane];
    }
    if (lane < nef) sp->qe[lane] = qe;
  };
  fetch(w_beg);
  uint32_t adv = 64;  // events this step took (exact stretches hand the rest of a block back early)
  for (uint32_t j0 = w_beg; j0 < s_end; j0 += adv) {
    if (j0 == s_beg && h > 0) {  // the cut: the state the warm-up reached
      if (XB && xm) to_wave(lclk);
      dump(D.snap[0] + ks);
      emit_on = true;
    }
    const uint32_t jend = (h > 0 && j0 < s_beg) ? s_beg : s_end;  // (a step never crosses the cut)
    const int nv0 = (int)min(64u, jend - j0);
    const int64_t ts = n_ts, clk = n_clk;
    const uint32_t g = n_g, v = n_v;
    const int st0 = n_st;
    const bool en = (n_n & 1u) != 0;
    const bool qf = (n_n & 2u) != 0;  // its own filter (la_pack_q)
    uint64_t brk;
    int nv = nv0;
    {  // the ordered formulation: timestamps do not decrease within the key, and no event lags the
       // clock by T or more (an entry queued then could fire at a send far past it); a block that
       // breaks it runs the exact rule from its first break on (the events before it are this step)
      const int64_t tp = __shfl_up(ts, 1, 64);
      const int64_t prev = lane == 0 ? last : tp;
      brk = __ballot((int)lane < nv0 && ((prev != INT64_MIN && ts < prev) || clk - ts >= Tw));
      if (!xm && brk) {
        if constexpr (!XB) {  // the exact variant re-runs this (key, segment)
          if (lane == 0) D.cm[ks] = LA_XMARK;
          return;
        }
        const int F = __builtin_ctzll(brk);
        if (F > 0) nv = F;
        else to_exact();
      }
    }
    adv = (uint32_t)nv;
    if (j0 + nv < s_end) fetch(j0 + nv);
    const bool valid = lane < nv;
    const int role = valid ? st0 : -1;
    if (XB && xm) {
      // the exact rule through the event after the block's last break (or 8 events when the block
      // has none: a carried irregular state), then back to the ordered formulation when the state is
      // regular there -- its next step starts after that event -- else the block's rest exactly
      const int E = brk ? min(64 - __builtin_clzll(brk), nv - 1) : min(7, nv - 1);
      int q = 0;
      LA_STAMP(0);
      int qe_ = E;  // the next event after which the state is checked (then every 4 events)
#pragma unroll 1
      while (q < nv && !xover) {
        for (; q <= qe_ && !xover; q++) xstep(q, ts, clk, g, v, role, en, qf);
        if (xover || q >= nv) break;
        to_wave(lclk);
        if (!xm) break;
        qe_ = min(q + 3, nv - 1);
      }
      if (!xover && q < nv) {  // regular again before the block's end: the next step starts at q
        LA_COUNT(12, q);
        LA_STAMP(13);
        adv = (uint32_t)q;
        fetch(j0 + adv);  // (the prefetch above read the step after this block)
        continue;
      }
      LA_COUNT(12, q);
      LA_STAMP(13);
      if (xover) {
        if (lane == 0) {
          D.cm[ks] = 0;
          atomicOr(err, LA_SLOW);
        }
        return;
      }
      to_wave(lclk);  // (still exact after it: the next block runs the exact rule too)
      continue;
    }
    const int64_t seqg = bseq(B, g);
    const uint64_t QX = __ballot(valid && role == 0 && qf);
    const uint64_t QY = __ballot(valid && role == 1 && qf);
    LA_STAMP(0);
    // 1. the partial.  A half partial carried into the block resolves first (its partner, or the
    //    first event beyond W).  Then, from an empty partial at lane p, the next step depends on
    //    the block alone: the first qualifying event a >= p fills a slot; the first qualifying
    //    partner b > a completes the pair if ts_b - ts_a <= W (no event between them is later
    //    than ts_b), else the first event beyond ts_a + W resets the partial and starts afresh.
    //    Every lane computes that step for p = itself, and the chain from the block's first empty
    //    position is walked with one readlane per step.
    int p0 = 0;
    if (hx || hy) {
      const int64_t tf = hx ? xts : yts;
      const uint64_t Em = useW ? __ballot(valid && ts - tf > Wn) : 0ull;
      const uint64_t Om = hx ? QY : QX;
      const int z = Em ? __builtin_ctzll(Em) : 64, b = Om ? __builtin_ctzll(Om) : 64;
      if (b < z) {  // the partner: the pair completes and waits on the absent state
        if (nal >= 64) {
          if (lane == 0) {
            D.cm[ks] = 0;
            atomicOr(err, LA_SLOW);
          }
          return;
        }
        const uint32_t bn = (uint32_t)__builtin_amdgcn_readlane((int)en, b);
        const int64_t bseqv = la_rl64(seqg, b), bts = la_rl64(ts, b);
        const uint32_t bv = (uint32_t)__builtin_amdgcn_readlane((int)v, b);
        if (hx) {
          yseq = bseqv;
          yts = bts;
          yv = bv;
          fl = (fl & ~2u) | (bn ? 2u : 0u);
        } else {
          xseq = bseqv;
          xts = bts;
          xv = bv;
          fl = (fl & ~1u) | (bn ? 1u : 0u);
        }
        if (lane == 0) {
          LaWait w;
          w.due = bts + Tw;
          w.xseq = xseq;
          w.xts = xts;
          w.yseq = yseq;
          w.yts = yts;
          w.xv = xv;
          w.yv = yv;
          w.fl = fl;
          w.pad = 0;
          A[nal] = w;
          Ac[nal] = b;
          Anae[nal] = 1;
          Aed[nal] = w.due;
          Ec[b] = 1;
        }
        nal++;
        hx = hy = false;
        xseq = yseq = -1;
        fl = 0;
        p0 = b + 1;
      } else if (z < 64) {  // expired (StreamPreStateProcessor.expireEvents): event z starts afresh
        hx = hy = false;
        xseq = yseq = -1;
        fl = 0;
        p0 = z;
      } else {
        p0 = 64;
      }
    }
    // the step from an empty partial at p = this lane
    const uint64_t mq = (QX | QY) & (~0ull << lane);
    const int a = mq ? __builtin_ctzll(mq) : 64;
    const int ac = a < 64 ? a : 0;
    const bool ax = ((QX >> ac) & 1ull) != 0;
    const uint64_t opp = (ax ? QY : QX) & (a < 63 ? (~0ull << (a + 1)) : 0ull);
    const int b = opp ? __builtin_ctzll(opp) : 64;
    const int bc = b < 64 ? b : 0;
    const int64_t tsa = __shfl(ts, ac, 64), tsb = __shfl(ts, bc, 64);
    // kind: 0 nothing fills a slot in [p, nv); 1 pair (a, b), empty at b + 1; 2 no partner within W:
    // a reset at the first event beyond ts_a + W if the block has one (found by a ballot when the
    // chain reaches the step -- few steps a block), else a half partial (a) at the block's end
    int kind, J;
    if (a >= nv) {
      kind = 0;
      J = 64;
    } else if (b < nv && (!useW || tsb - tsa <= Wn)) {
      kind = 1;
      J = b + 1;
    } else {
      kind = 2;
      J = a;
    }
    const int KJ = J | (kind << 8);
    uint64_t PM = 0;  // chain positions whose step completes a pair
    int hk = -1;      // chain position that leaves a half partial
    for (int p = p0; p < nv;) {
      const int kj = __builtin_amdgcn_readlane(KJ, p);
      const int kd = kj >> 8;
      if (kd == 1) {
        PM |= 1ull << p;
        p = kj & 0xFF;
      } else if (kd == 2) {
        const int ap = kj & 0xFF;
        const int64_t tap = la_rl64(ts, ap);
        const uint64_t zb = useW ? __ballot(valid && lane > ap && ts - tap > Wn) : 0ull;
        if (!zb) {
          hk = p;
          break;
        }
        p = __builtin_ctzll(zb);
      } else {
        break;
      }
    }
    if (PM) {  // the completed pairs, in completion order, join the absent state's new-and-every list
      const int npm = __popcll(PM);
      if (nal + npm > 64) {
        if (lane == 0) {
          D.cm[ks] = 0;
          atomicOr(err, LA_SLOW);
        }
        return;
      }
      const int xi = ax ? ac : bc, yi = ax ? bc : ac;
      const int64_t sx = __shfl(seqg, xi, 64), sy = __shfl(seqg, yi, 64);
      const int64_t tx = __shfl(ts, xi, 64), ty = __shfl(ts, yi, 64);
      const uint32_t vx = (uint32_t)__shfl((int)v, xi, 64), vy = (uint32_t)__shfl((int)v, yi, 64);
      const int nx = __shfl((int)en, xi, 64), ny = __shfl((int)en, yi, 64);
      if ((PM >> lane) & 1ull) {
        const int d = nal + __popcll(PM & lt);
        LaWait w;
        w.due = tsb + Tw;
        w.xseq = sx;
        w.xts = tx;
        w.yseq = sy;
        w.yts = ty;
        w.xv = vx;
        w.yv = vy;
        w.fl = (nx ? 1u : 0u) | (ny ? 2u : 0u);
        w.pad = 0;
        A[d] = w;
        Ac[d] = b;
        Anae[d] = 1;
        Aed[d] = w.due;
        Ec[b] = 1;
      }
      nal += npm;
    }
    if (hk >= 0) {  // the slot event a of the chain's last step
      const int ha = __builtin_amdgcn_readlane(a, hk);
      const bool hxs = __builtin_amdgcn_readlane((int)ax, hk) != 0;
      const uint32_t an = (uint32_t)__builtin_amdgcn_readlane((int)en, ha);
      if (hxs) {
        hx = true;
        xseq = la_rl64(seqg, ha);
        xts = la_rl64(ts, ha);
        xv = (uint32_t)__builtin_amdgcn_readlane((int)v, ha);
        fl = (fl & ~1u) | (an ? 1u : 0u);
      } else {
        hy = true;
        yseq = la_rl64(seqg, ha);
        yts = la_rl64(ts, ha);
        yv = (uint32_t)__builtin_amdgcn_readlane((int)v, ha);
        fl = (fl & ~2u) | (an ? 2u : 0u);
      }
    }
    __syncthreads();
    LA_STAMP(1);
    LA_COUNT(6, nal);
    const uint64_t zm = __ballot(valid && role == 2);
    LA_COUNT(11, __popcll(zm));
    // FZ1: the Z side of fz per event (a null Z event kills nothing: left out of the kills' walk)
    const LaTermD& z1 = D.fz.t[0];
    const bool z1a = z1.ak == 3;
    const double zd1 = FZ1 ? la_val(v, t2g, z1a ? z1.aflt : z1.bflt) : 0.0;
    const uint64_t zmk = FZ1 ? zm & __ballot(!en) : zm;  // the Z events that may kill
    const int lastz = zm ? 63 - __builtin_clzll(zm) : -1;  // the block's last Z event (new-and-every -> pending)
    const int64_t clkl = la_rl64(clk, nv - 1);            // the clock at the block's last event
    const uint64_t cmask = __ballot(valid && Ec[lane] != 0);  // lanes that completed a pair
    const int64_t qt = ts + Tw;                            // the time of an entry this event queues
    // 2. the pairs against this block's events
    if (nal > 0) {
      LaWait w{};
      int c = 64;
      int64_t ed = 0;
      if (lane < nal) {
        w = A[lane];
        c = Ac[lane];
        ed = Aed[lane];
      }
      const int64_t dd = min(w.xts, w.yts) + Wb;
      // pairs completed in this block and past their D before their due: their E_D looks at the queue
      const uint64_t doomall = __ballot(lane < nal && w.due > dd);  // past D before their due
      const uint64_t doom = doomall & __ballot(c >= 0);              // ... and completed in this block
      // E_D of pair j (completed at cj): the first entry past max(D, clock(cj)) among the queue and
      // the block's entries queued before cj (em: the event lanes that queued some)
      auto edj = [&](int j, uint64_t em) __attribute__((always_inline)) -> int64_t {
        const int cj = __builtin_amdgcn_readlane(c, j);
        const int64_t thr = max(la_rl64(dd, j), la_rl64(clk, cj));
        int64_t r = la_rl64(w.due, j);
        const uint64_t qm = __ballot(lane < nef && qe > thr);
        if (qm) r = min(r, la_rl64(qe, __builtin_ctzll(qm)));
        const uint64_t bm = em & __ballot(lane < cj && qt > thr);
        if (bm) r = min(r, la_rl64(qt, __builtin_ctzll(bm)));
        return r;
      };
      for (uint64_t m = doom; m; m &= m - 1) {
        const int j = __builtin_ctzll(m);
        const int64_t r = edj(j, cmask);
        if (lane == j) ed = r;
      }
      LA_STAMP(2);
      int f = 64, kq = 64;
      bool killed = false;
      // the leave event: the first event after c whose clock reaches E_D or whose ts passes D (both
      // ascend in the block); the kill: the first Z event before it whose filter holds.  A kill queues
      // an entry that may lower a later doomed pair's E_D: repeat until none changes
      for (int it = 0; it < 65; it++) {
        // (a pair not past D before its due leaves at its due: ts > D implies clock > due there)
        int l2 = c + 1, h2 = nv;  // the answer lies in [l2, h2]; h2 = nv: not in this block
#pragma unroll
        for (int st7 = 0; st7 < 7; st7++) {
          const int mid = (l2 + h2) >> 1;
          const int64_t cm = __shfl(clk, mid < 64 ? mid : 0, 64);
          if (l2 < h2) {
            if (mid < nv && cm >= ed) h2 = mid;
            else l2 = mid + 1;
          }
        }
        f = lane < nal && l2 < nv ? l2 : 64;
        for (uint64_t m = doomall; m; m &= m - 1) {  // a pair past D before its due: or the first event beyond D
          const int j = __builtin_ctzll(m);
          const int cj = __builtin_amdgcn_readlane(c, j);
          const uint64_t xm = __ballot(valid && lane > cj && ts > la_rl64(dd, j));
          const int fx = xm ? __builtin_ctzll(xm) : 64;
          if (lane == j) f = min(f, fx);
        }
        LA_STAMP(3);
        LA_COUNT(10, 1);
        killed = false;
        kq = 64;
        if (FZ1 && zmk) {  // each pair walks its Z events (c, f): one shuffle and one compare a step
          const int oi = z1a ? 0 : 1;  // the pair's side of the term
          const LaKill K = la_kill_pre(D.fz, w, t0g, t1g, t2g);
          const double kv = oi == 0 ? K.b[0] : K.a[0];
          auto nextz = [&](int x) __attribute__((always_inline)) -> int {
            if (x >= 64) return 64;
            const uint64_t r = zmk >> x;
            return r ? x + __builtin_ctzll(r) : 64;
          };
          int q = nextz(c + 1);
          bool act = lane < nal && q < f && !K.nul[0];
          while (__ballot(act)) {
            const double zq = __shfl(zd1, q < 64 ? q : 0, 64);
            if (act) {
              const double A = z1a ? zq : kv, Bv = z1a ? kv : zq;
              const int o3 = (A < Bv ? 1 : 0) | (A == Bv ? 2 : 0) | (A > Bv ? 4 : 0);
              killed = ((o3 | (o3 == 0 ? 8 : 0)) & z1.mask) != 0;
              if (killed) kq = q;
              q = nextz(q + 1);
              act = !killed && q < f;
            }
          }
        } else if (!FZ1 && zm) {
          const LaKill K = la_kill_pre(D.fz, w, t0g, t1g, t2g);
          auto nextz = [&](int x) __attribute__((always_inline)) -> int {
            if (x >= 64) return 64;
            const uint64_t r = zm >> x;
            return r ? x + __builtin_ctzll(r) : 64;
          };
          int q = nextz(c + 1);
          bool act = lane < nal && q < f;
          while (__ballot(act)) {
            const int qs = q < 64 ? q : 0;
            const uint32_t zv = (uint32_t)__shfl((int)v, qs, 64);
            const bool zn = __shfl((int)en, qs, 64) != 0;
            if (act) {
              killed = la_kill(D.fz, K, la_val(zv, t2g, false), la_val(zv, t2g, true), zn);
              if (killed) kq = q;
              q = nextz(q + 1);
              act = !killed && q < f;
            }
          }
        }
        LA_STAMP(8);
        const uint64_t km = __ballot(killed);
        if (!km || !doom) break;
        // the kills' lanes: do they come before a doomed pair's completion?
        int kmin = killed ? kq : 64;
        for (int o = 32; o > 0; o >>= 1) kmin = min(kmin, __shfl_xor(kmin, o, 64));
        uint64_t redo = 0;
        for (uint64_t m = doom; m; m &= m - 1) {
          const int j = __builtin_ctzll(m);
          if (__builtin_amdgcn_readlane(c, j) <= kmin) continue;
          uint64_t kl = 0;  // event lanes with a kill
          for (uint64_t mm = km; mm; mm &= mm - 1) kl |= 1ull << __builtin_amdgcn_readlane(kq, __builtin_ctzll(mm));
          const int64_t r = edj(j, cmask | kl);
          const int64_t cur = la_rl64(ed, j);
          if (r != cur) {
            redo |= 1ull << j;
            if (lane == j) ed = r;
          }
        }
        if (!redo) break;
      }
      LA_STAMP(8);
      // the kills, counted per event lane (each queues an entry at the event's ts + T)
      if (killed) atomicAdd(&Ec[kq], 1);
      __syncthreads();
      const uint64_t emk = __ballot(valid && Ec[lane] != 0);  // event lanes that queued entries
      const bool left = f < 64;
      const int64_t gp = (int64_t)(uint32_t)__shfl(g, f > 0 ? f - 1 : 0, 64);
      const int64_t gf = (int64_t)(uint32_t)__shfl(g, f < 64 ? f : 0, 64);
      // the block's last firing of the queue (before which event lane): of its latest fired entry,
      // an old one (queued before the block) or one the block queued
      int lastf = -1;
      {
        const uint64_t fo = __ballot(lane < nef && qe <= clkl);
        if (fo) {
          const int64_t t = la_rl64(qe, 63 - __builtin_clzll(fo));
          const uint64_t r = __ballot(valid && clk >= t);
          lastf = max(lastf, __builtin_ctzll(r));
        }
        const uint64_t fb = emk & __ballot(valid && qt <= clkl);
        if (fb) {
          const int p = 63 - __builtin_clzll(fb);
          const int64_t t = la_rl64(qt, p);
          const uint64_t r = __ballot(valid && lane > p && clk >= t);
          lastf = max(lastf, __builtin_ctzll(r));
        }
      }
      LA_STAMP(9);
      const bool tonae = lane < nal && Anae[lane] && c >= lastf && c >= lastz;  // no Z / firing after it
      settle(left, killed, tonae, f == 0 ? lo : gp + 1, gf, w, ed);
      LA_STAMP(4);
    }
    LA_STAMP(0);
    // the queue: the entries the block's clock reached have fired; the block's own join in lane
    // (= time) order; lastScheduledTime from the block's last completion or kill
    {
      const int ecl = valid ? Ec[lane] : 0;
      const uint64_t qm = __ballot(ecl != 0);
      if (qm || nef) {
        const uint64_t keep = __ballot(lane < nef && qe > clkl);  // a suffix (sorted)
        const int n0 = __popcll(keep);
        const int drop = nef - n0;
        int64_t x = __shfl(qe, lane + drop < 64 ? lane + drop : 63, 64);
        // the block's entries still queued, expanded (a Z event that kills several pairs queues several)
        const int ec2 = qt > clkl ? ecl : 0;
        int pos = ec2;
        for (int o = 1; o < 64; o <<= 1) {  // inclusive scan of the counts
          const int y = __shfl_up(pos, o, 64);
          if (lane >= o) pos += y;
        }
        const int n1 = __shfl(pos, 63, 64);
        if (n0 + n1 > LA_WF) {
          if (lane == 0) {
            D.cm[ks] = 0;
            atomicOr(err, LA_SLOW);
          }
          return;
        }
        for (int i = pos - ec2; i < pos; i++) Es[n0 + i] = qt;
        __syncthreads();
        if (lane < n0) Es[lane] = x;
        __syncthreads();
        nef = n0 + n1;
        qe = lane < nef ? Es[lane] : INT64_MAX;
        if (qm) lsched = la_rl64(qt, 63 - __builtin_clzll(qm));
        __syncthreads();
      }
      Ec[lane] = 0;
    }
    LA_STAMP(5);
    lo = (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)g, nv - 1) + 1;
    last = la_rl64(ts, nv - 1);
    lclk = clkl;
    __syncthreads();
  }
  auto stamps_out = [&]() {
#ifdef SHP_SW_STAMPS
    LA_COUNT(7, s_end - w_beg);
    LA_COUNT(14, XB ? 1 : 0);
    if (lane == 0 && D.stamps)
      for (int x = 0; x < LA_NSTAMP; x++) D.stamps[(int64_t)ks * LA_NSTAMP + x] = lst[x];
#endif
  };
  if (!lastseg) {  // the state this segment ends with, for the next one's check; no push-end settle
    stamps_out();
    if (XB && xm) to_wave(lclk);
    dump(D.snap[1] + ks + 1);
    if (lane == 0) D.cm[ks] = min(nm, rcap);
    if (e) atomicOr(err, e);
    return;
  }
  // the timers the push's last clock reaches
  const int64_t lastclk = B.n > 0 ? B.rmax[B.n - 1] : B.clock0;
  if (XB && xm) {  // the exact rule's push end (k_labs): the timers the last clock reaches, then its state
    if (B.n > 0) xfire(B.n - 1, lastclk);
    if (xover) {
      if (lane == 0) {
        D.cm[ks] = 0;
        atomicOr(err, LA_SLOW);
      }
      return;
    }
    stamps_out();
    if (nal > cap || nef > cap) {
      e |= E_LIST;
    } else {
      if (lane < nal) D.wq[wr][(int64_t)k * cap + lane] = P;
      if (lane < nef) {
        LaEnt y;
        y.t = qe;
        y.i0 = 0;
        y.pad = 0;
        D.fq[wr][(int64_t)k * cap + lane] = y;
      }
    }
    if (lane == 0) {
      D.cm[ks] = min(nm, rcap);
      LaPend s{};
      s.xseq = hx ? xseq : -1;
      s.yseq = hy ? yseq : -1;
      s.xts = xts;
      s.yts = yts;
      s.xv = xv;
      s.yv = yv;
      s.fl = fl;
      s.nw = nal;
      s.wh = 0;
      s.nae = xnae;
      s.last = last;
      s.lst = lsched;
      s.ne = nef;
      s.eh = 0;
      s.reg = 0;  // (k_labs_w decides from the state itself: to_wave)
      D.pend[wr][k] = s;
    }
    if (e) atomicOr(err, e);
    return;
  }
  const bool flushed = __ballot(lane < nef && qe <= lastclk) != 0;  // a firing after every event of the key
  if (nal > 0) {
    LaWait w{};
    int64_t ed = 0;
    bool nae = false;
    if (lane < nal) {
      w = A[lane];
      ed = Aed[lane];
      nae = Anae[lane] != 0 && !flushed;
    }
    settle(lane < nal && ed <= lastclk, false, nae, lo, B.n - 1, w, ed);
  }
  {  // the queue keeps the entries past the last clock
    const uint64_t keep = __ballot(lane < nef && qe > lastclk);
    const int n0 = __popcll(keep);
    const int drop = nef - n0;
    const int64_t x = __shfl(qe, lane + drop < 64 ? lane + drop : 63, 64);
    nef = n0;
    if (nef <= cap && lane < nef) {
      LaEnt y;
      y.t = x;
      y.i0 = 0;
      y.pad = 0;
      D.fq[wr][(int64_t)k * cap + lane] = y;
    }
  }
  // new-and-every: the trailing pairs with no Z event and no firing since their completion
  int nae = 0;
  {
    const uint64_t m = __ballot(lane < nal && Anae[lane]);
    const uint64_t all = nal >= 64 ? ~0ull : ((1ull << nal) - 1ull);
    const uint64_t notq = all & ~m;
    nae = notq ? nal - 1 - (63 - __builtin_clzll(notq)) : nal;
  }
  stamps_out();
#undef LA_STAMP
#undef LA_COUNT
  if (nal > cap || nef > cap) e |= E_LIST;
  else if (lane < nal) D.wq[wr][(int64_t)k * cap + lane] = A[lane];
  if (lane == 0) {
    D.cm[ks] = min(nm, rcap);
    LaPend s{};
    s.xseq = hx ? xseq : -1;
    s.yseq = hy ? yseq : -1;
    s.xts = xts;
    s.yts = yts;
    s.xv = xv;
    s.yv = yv;
    s.fl = fl;
    s.nw = nal;
    s.wh = 0;
    s.nae = nae;
    s.last = last;
    s.lst = lsched;
    s.ne = nef;
    s.eh = 0;
    s.reg = 1;
    D.pend[wr][k] = s;
  }
  if (e) atomicOr(err, e);
}

// first index in (lo, hi] whose clock reaches thr, given c[lo] < thr (hi when none does), over a
// non-decreasing clock array: a push's clock is close to linear in the index, so an interpolated
// guess probed with both neighbours (three loads at once, one latency) usually ends the search;
// bisection steps between the guesses bound the worst case
__device__ __forceinline__ int64_t la_clock_lb(const int64_t* __restrict__ c, int64_t lo, int64_t hi, int64_t rlo,
                                               int64_t rhi, int64_t thr) {
  bool interp = true;
  while (hi - lo > 1) {
    int64_t m;
    if (interp && rhi > rlo) {
      const double f = (double)(thr - rlo) / (double)(rhi - rlo);
      m = lo + (int64_t)(f * (double)(hi - lo));
      m = m <= lo ? lo + 1 : (m >= hi ? hi - 1 : m);
    } else {
      m = lo + ((hi - lo) >> 1);
    }
    const bool pl = interp && m - 1 > lo, pr = interp && m + 1 < hi;
    interp = !interp;
    const int64_t rm = c[m];
    const int64_t rp = pl ? c[m - 1] : 0, rn = pr ? c[m + 1] : 0;
    if (rm >= thr) {
      hi = m;
      rhi = rm;
      if (pl) {
        if (rp >= thr) {
          hi = m - 1;
          rhi = rp;
        } else {
          lo = m - 1;
          rlo = rp;
        }
      }
    } else {
      lo = m;
      rlo = rm;
      if (pr) {
        if (rn >= thr) {
          hi = m + 1;
          rhi = rn;
        } else {
          lo = m + 1;
          rlo = rn;
        }
      }
    }
  }
  return hi;
}

// k_labs_w's records of each key (its region of D.rec) to the push's output at the key's offset,
// with the fire event found as k_labs_pos does
static __global__ __launch_bounds__(256) void k_labs_out(LabsDev D, BatchView B, MatchOut O, const uint32_t* __restrict__ kbeg,
                                                  const uint32_t* __restrict__ kcnt, int H, int* err) {
  const int S = D.seg;
  const int ks = blockIdx.x * 4 + (int)(threadIdx.x >> 6);  // a slot: key k's segment h
  if (ks >= D.nk * S) return;
  const int k = ks / S, h = ks % S;
  const int lane = (int)(threadIdx.x & 63);
  const int64_t mi = D.om[ks];
  const uint32_t cnt = kcnt[k];
  const int hk = la_nseg(cnt, H);
  const uint32_t s_beg = h < hk ? la_segb(cnt, hk, h) : 0u, s_end = h < hk ? la_segb(cnt, hk, h + 1) : 0u;
  const uint32_t nm = h < hk ? min(D.cm[ks], (s_end - s_beg + 1u) / 2u + 64u) : 0u;
  if (ks == D.nk * S - 1 && lane == 0) {
    O.count[0] = (unsigned long long)(mi + nm);
    O.count[1] = 2ull * (unsigned long long)(mi + nm);
  }
  const LaRec* rec = D.rec + la_region(kbeg[k] + s_beg, ks);
  int e = 0;
  for (uint32_t r = (uint32_t)lane; r < nm; r += 64) {
    const int64_t m = mi + r;
    if (m >= O.cap || 2 * m + 2 > O.refcap) {
      e |= E_OUT;
      break;
    }
    const LaRec x = rec[r];
    int64_t a = x.flo, b = min((int64_t)x.fhi, B.n - 1);
    if (x.thr == INT64_MIN) b = a;  // (an exact block's firing at a known send)
    if (D.rc && a < b) {  // the 64-event block first reaching thr (rc: each block's last clock), then within it
      int64_t ja = a >> 6;
      const int64_t jb = b >> 6;
      if (ja < jb) {
        const int64_t r0 = D.rc[ja];
        if (r0 < x.thr) ja = la_clock_lb(D.rc, ja, jb, r0, D.rc[jb], x.thr);
      }
      a = max(a, ja << 6);
      b = min(b, (ja << 6) + 63);
    }
    if (a < b) {
      const int64_t r0 = B.rmax[a];
      if (r0 < x.thr) a = la_clock_lb(B.rmax, a, b, r0, B.rmax[b], x.thr);
    }
    O.key[m] = B.partitioned ? k : 0;
    O.ts[m] = x.due;
    O.type[m] = 0;
    O.pos[m] = bseq(B, a);
    O.ref_off[m] = 2 * m;
    int64_t q = 2 * m;
#pragma unroll
    for (int s = 0; s < 3; s++) {
      const bool isx = s == D.sid[0], isy = s == D.sid[1];
      O.slot_len[m * MAXS + s] = (int16_t)((isx || isy) ? 1 : 0);
      if (isx) O.refs[q++] = x.xseq;
      if (isy) O.refs[q++] = x.yseq;
    }
  }
  if (e) atomicOr(err, e);
}

// the segment cuts: the warmed-up state of segment h against the state segment h - 1 ended with
static __global__ __launch_bounds__(64) void k_labs_segcheck(LabsDev D, const uint32_t* __restrict__ kcnt, int H,
                                                            int* err) {
  const int S = D.seg;
  const int k = blockIdx.x / S, h = blockIdx.x % S;
  if (k >= D.nk || h == 0 || h >= la_nseg(kcnt[k], H)) return;
  const int lane = (int)threadIdx.x;
  const LaSnap& a = D.snap[0][blockIdx.x];
  const LaSnap& b = D.snap[1][blockIdx.x];
  bool bad = false;
  if (lane == 0)
    bad = a.xseq != b.xseq || a.yseq != b.yseq || a.xts != b.xts || a.yts != b.yts || a.xv != b.xv || a.yv != b.yv ||
          a.fl != b.fl || a.hxy != b.hxy || a.last != b.last || a.lsched != b.lsched || a.lo != b.lo ||
          a.nal != b.nal || a.nef != b.nef || a.xm != b.xm || a.xnae != b.xnae || a.qat != b.qat;
  const uint32_t nal = min(a.nal, 64u), nef = min(a.nef, 64u);
  if ((uint32_t)lane < nal && (uint32_t)lane < b.nal) {
    const LaWait& x = a.A[lane];
    const LaWait& y = b.A[lane];
    bad |= x.due != y.due || x.xseq != y.xseq || x.xts != y.xts || x.yseq != y.yseq || x.yts != y.yts ||
           x.xv != y.xv || x.yv != y.yv || x.fl != y.fl || a.ed[lane] != b.ed[lane] || a.nae[lane] != b.nae[lane];
  }
  if ((uint32_t)lane < nef && (uint32_t)lane < b.nef) bad |= a.qe[lane] != b.qe[lane];
  if (__ballot(bad) && lane == 0) atomicOr(err, LA_SEGMISS);
}

static __global__ void k_labs_coarse(const int64_t* __restrict__ rmax, int64_t n, int64_t* __restrict__ rc) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if ((j << 6) < n) rc[j] = rmax[min((j << 6) + 63, n - 1)];
}

// a key's pairs and queue entries into rings of another capacity (tier change), heads reset to 0
static __global__ void k_labs_migrate(LabsDev Dn, LabsDev Do) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= Do.nk) return;
  const int c = Do.cur;
  LaPend s = Do.pend[c][k];
  for (int i = 0; i < s.nw && i < Dn.wcap; i++)
    Dn.wq[c][k * Dn.wcap + i] = Do.wq[c][k * Do.wcap + ((s.wh + i) & (Do.wcap - 1))];
  for (int i = 0; i < s.ne && i < Dn.wcap; i++)
    Dn.fq[c][k * Dn.wcap + i] = Do.fq[c][k * Do.wcap + ((s.eh + i) & (Do.wcap - 1))];
  s.wh = 0;
  s.eh = 0;
  Dn.pend[c][k] = s;
}

static __global__ void k_labs_init(LabsDev D) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < D.nk) {
    LaPend s{};
    s.xseq = s.yseq = -1;
    s.last = INT64_MIN;
    s.reg = 1;
    D.pend[0][i] = s;
    D.pend[1][i] = s;
  }
}

// the push's largest step of the playback clock after its first send (k_labs_w's formulation needs
// every step <= T: then an entry fires at most T past its time, and lastScheduledTime never moves
// to the clock); the first send's step is checked per key (it matters only where entries are queued)
static __global__ void k_labs_steps(const int64_t* __restrict__ rmax, int64_t n, unsigned long long* out) {
  unsigned long long m = 0;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x + 1; g < n; g += (int64_t)gridDim.x * blockDim.x)
    m = max(m, (unsigned long long)(rmax[g] - rmax[g - 1]));
  for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned long long)__shfl_xor((long long)m, o, 64));
  if ((threadIdx.x & 63) == 0 && m) atomicMax(out, m);
}

struct LabsState {
  LabsDev D{};
  int tier = 0;
  bool wave_ok = false;  // k_labs_w applies: x's and y's filters read only their own event
  bool slow = false;     // this push re-runs on k_labs (k_labs_w raised LA_SLOW)
  bool noseg = false;    // this push re-runs k_labs_w unsegmented (LA_SEGMISS)
  bool steps_done = false;  // this push's largest clock step is in D.maxstep (the multisplit)
  bool sorted = false;   // this push's key-order batch came from sort_events (no pack + gather)
  void* stmp = nullptr;  // sort_events' rocPRIM scratch
  size_t stmp_bytes = 0;

  static bool lower_term(const LaTermS& t, const LabsShape& sh, const DevProg& P, LaTermD& o) {
    static const int32_t masks[6] = {4, 6, 1, 3, 2, 13};  // gt ge lt le eq ne
    o = LaTermD{};
    o.mask = t.ptype == T_STR ? (t.cmp == 4 ? 2 : 13) : masks[t.cmp];
    auto side = [&](const LaOperand& a, int8_t& kind, int8_t& flt, double& c) {
      if (a.kind == 0) {
        FOperand f{};
        f.kind = 0;
        f.tag = a.tag;
        f.imm = a.imm;
        int8_t kk;
        return SweepState::lower_operand(f, t.ptype, T_NULL, kk, c);
      }
      kind = (int8_t)(a.state == sh.sx ? 1 : (a.state == sh.sy ? 2 : 3));
      flt = (int8_t)(P.colTag[a.col] == T_INT && t.ptype == T_FLOAT);
      return P.colTag[a.col] == T_INT || P.colTag[a.col] == T_FLOAT || P.colTag[a.col] == T_STR;
    };
    return side(t.a, o.ak, o.aflt, o.ac) && side(t.b, o.bk, o.bflt, o.bc);
  }
  static bool lower(const LaPredS& p, const LabsShape& sh, const DevProg& P, LaPredD& o) {
    o = LaPredD{};
    o.n = p.n;
    o.combine = p.combine;
    for (int i = 0; i < p.n; i++)
      if (!lower_term(p.t[i], sh, P, o.t[i])) return false;
    return true;
  }
  static bool shape_ok(const DevProg& P, const LabsShape& sh) {
    if (!sh.ok) return false;
    LaPredD a;
    return lower(sh.fx, sh, P, a) && lower(sh.fy, sh, P, a) && lower(sh.fz, sh, P, a);
  }

  template <class T>
  static void al(T*& p, int64_t n) {
    if (hipMalloc((void**)&p, std::max<int64_t>(n, 1) * sizeof(T)) != hipSuccess)
      throw std::runtime_error("hipMalloc failed (logical-absent path)");
  }

  void create(const DevProg& P, const LabsShape& sh, int32_t max_keys, int64_t mcap, int64_t cap, hipStream_t s) {
    if (!lower(sh.fx, sh, P, D.fx) || !lower(sh.fy, sh, P, D.fy) || !lower(sh.fz, sh, P, D.fz))
      throw std::runtime_error("logical-absent: predicate not lowerable");
    const int32_t st[3] = {sh.stx, sh.sty, sh.stz}, col[3] = {sh.colx, sh.coly, sh.colz},
                  sid[3] = {sh.sx, sh.sy, sh.sz};
    for (int i = 0; i < 3; i++) {
      D.st[i] = st[i];
      D.col[i] = col[i];
      D.sid[i] = sid[i];
      D.tag[i] = col[i] >= 0 ? P.colTag[col[i]] : T_NULL;
    }
    D.wait = sh.wait;
    D.within = sh.within;
    D.nk = max_keys;
    D.cur = 0;
    for (int c = 0; c < 2; c++) {
      al(D.pend[c], max_keys);
      al(D.wq[c], (int64_t)max_keys * LA_WCAP);
      al(D.fq[c], (int64_t)max_keys * LA_WCAP);
    }
    al(D.wtmp, (int64_t)max_keys * LA_WCAP);
    al(D.ftmp, (int64_t)max_keys * LA_WCAP);
    al(D.maxstep, 1);
    // segments while the keys are few (a wave per key leaves CUs idle) and k_labs_w can run
    D.seg = max_keys <= LA_SEG_MAXKEYS && !getenv("SHP_LABS_NOSEG") ? LA_H : 1;
    D.warm = LA_WARM;
    if (const char* w = getenv("SHP_LABS_WARM")) D.warm = (uint32_t)(atoi(w) / 64 * 64);  // (a multiple of 64)
    al(D.cm, (int64_t)max_keys * D.seg);
    al(D.om, (int64_t)max_keys * D.seg);
    al(D.p_ev, cap);
    al(D.s_ev, cap);
    D.wcap = LA_CAPS[0];
    tier = 0;
    auto own = [](const LaPredD& p, int kind) {
      for (int i = 0; i < p.n; i++)
        for (int8_t kk : {p.t[i].ak, p.t[i].bk})
          if (kk != 0 && kk != kind) return false;
      return true;
    };
    wave_ok = own(D.fx, 1) && own(D.fy, 2) && !getenv("SHP_NO_LABS_W");
    if (!wave_ok) D.seg = 1;
    if (wave_ok) al(D.rec, la_region((uint32_t)std::min<int64_t>(cap, 0xFFFFFFFFll), max_keys * D.seg) + 1);
    if (wave_ok) al(D.rc, (cap + 63) / 64 + 1);
    if (D.seg > 1) {
      al(D.snap[0], (int64_t)max_keys * D.seg + 1);
      al(D.snap[1], (int64_t)max_keys * D.seg + 1);
    }
#ifdef SHP_SW_STAMPS
    al(D.stamps, (int64_t)max_keys * D.seg * LA_NSTAMP);
    (void)hipMemset(D.stamps, 0, (size_t)max_keys * D.seg * LA_NSTAMP * sizeof(unsigned long long));
#endif
    k_labs_init<<<(unsigned)((max_keys + 255) / 256), 256, 0, s>>>(D);
  }

  template <bool EMIT>
  void launch(unsigned gk, bool few, const BatchView& B, const MatchOut& O, const uint32_t* perm, const uint32_t* kbeg,
              const uint32_t* kcnt, int* err, hipStream_t s) {
    if (few) k_labs<EMIT, 1><<<gk, 64, 0, s>>>(D, B, O, perm, kbeg, kcnt, err);
    else k_labs<EMIT, 64><<<gk, 64, 0, s>>>(D, B, O, perm, kbeg, kcnt, err);
  }

  void run(const BatchView& B, const MatchOut& O, const uint32_t* perm, const uint32_t* kbeg, const uint32_t* kcnt,
           int* err, void* tmp, size_t tmp_bytes, hipStream_t s, KTimer& kt) {
    const bool few = D.nk <= 8192;  // a wave per key while that fills the CUs
    const unsigned gk = few ? (unsigned)D.nk : (unsigned)((D.nk + 63) / 64);
    kt.mark("labs_gather", s);
    if (!sorted) D.ev16 = 0;
    if (B.n > 0 && !sorted) {  // (sort_events already left the batch in key order)
      k_labs_pack<<<2048, 256, 0, s>>>(D, B, B.n);
      k_labs_gather<<<4096, 256, 0, s>>>(D, perm, B.n);
    }
    if (wave_ok && !slow) {  // one pass, then the records to their offsets
      if (!steps_done) {  // (the multisplit found it)
        kt.mark("labs_steps", s);
        (void)hipMemsetAsync(D.maxstep, 0, sizeof(unsigned long long), s);
        if (B.n > 1) k_labs_steps<<<1024, 256, 0, s>>>(B.rmax, B.n, D.maxstep);
      }
      // the coarse clock (each 64-event block's last) for k_labs_w's exact blocks and k_labs_out
      if (D.rc && B.n > 0) k_labs_coarse<<<(unsigned)(((B.n + 63) / 64 + 255) / 256), 256, 0, s>>>(B.rmax, B.n, D.rc);
      kt.mark("labs", s);
      const int H = noseg ? 1 : D.seg;
      const unsigned gs = (unsigned)(D.nk * D.seg);
      if (la_fz1(D.fz)) {
        k_labs_w<true, false><<<gs, 64, 0, s>>>(D, B, perm, kbeg, kcnt, H, err);
        k_labs_w<true, true><<<gs, 64, 0, s>>>(D, B, perm, kbeg, kcnt, H, err);  // (the marked ones only)
      } else {
        k_labs_w<false, false><<<gs, 64, 0, s>>>(D, B, perm, kbeg, kcnt, H, err);
        k_labs_w<false, true><<<gs, 64, 0, s>>>(D, B, perm, kbeg, kcnt, H, err);
      }
      if (H > 1) {
        kt.mark("labs_segcheck", s);
        k_labs_segcheck<<<gs, 64, 0, s>>>(D, kcnt, H, err);
      }
      kt.mark("labs_scan", s);
      size_t tb = tmp_bytes;
      (void)rocprim::exclusive_scan(tmp, tb, D.cm, D.om, 0u, (size_t)gs, rocprim::plus<uint32_t>(), s);
      kt.mark("labs_out", s);
      k_labs_out<<<(gs + 3) / 4, 256, 0, s>>>(D, B, O, kbeg, kcnt, H, err);
      kt.mark(nullptr, s);
      return;
    }
    kt.mark("labs_count", s);
    launch<false>(gk, few, B, O, perm, kbeg, kcnt, err, s);
    kt.mark("labs_scan", s);
    size_t tb = tmp_bytes;
    (void)rocprim::exclusive_scan(tmp, tb, D.cm, D.om, 0u, (size_t)D.nk, rocprim::plus<uint32_t>(), s);
    kt.mark("labs", s);
    launch<true>(gk, few, B, O, perm, kbeg, kcnt, err, s);  // (k_labs writes each record's fire event)
    kt.mark(nullptr, s);
  }

  // the push's events in key order with their sort keys (skey_out, for the key runs): k_labs_pack2,
  // then one stable radix sort of (key, record) pairs
  // (ms: the multisplit's counts / offsets; bounds: kbeg / kcnt were set here, no key_bounds pass)
  uint32_t* ms_cnt = nullptr;
  uint32_t* ms_off = nullptr;
  bool bounds = false;
  // the fused clock (k_la_ms_count / k_la_seg_clock / k_la_ms_scatter<true>): set by the engine for a
  // push that skips the device-wide clock scan (the count pass and the scatter then write rmax_out)
  bool fuse_clock = false;
  int64_t* rmax_out = nullptr;
  bool fuses_clock() const { return ms_cnt != nullptr && D.segclk != nullptr && !getenv("SHP_LABS_SCAN_CLOCK"); }
  bool split_ok(int64_t cap) const {
    return D.nk + 1 <= LA_MS_BINS && cap < (1ll << 27) && !getenv("SHP_LABS_SORT");
  }
  void sort_events(const BatchView& B, const int32_t* key, uint32_t* skey_in, uint32_t* skey_out, int key_bits,
                   int* err, hipStream_t s, KTimer& kt, uint32_t* kbeg = nullptr, uint32_t* kcnt = nullptr) {
    bounds = false;
    steps_done = false;
    if (ms_cnt && kbeg && B.n > 0) {  // the stable multisplit
      const int32_t nseg = (int32_t)((B.n + LA_MS_SEG - 1) / LA_MS_SEG);
      const uint32_t nokey = (uint32_t)D.nk;
      int bits = 0;
      while ((1u << bits) < nokey + 1u) bits++;
      const size_t nc = (size_t)(nokey + 1) * nseg + 1;
      kt.mark("labs_count", s);
      const bool fc = fuse_clock;
      if (fc) k_la_ms_count<true><<<(unsigned)nseg, 256, 0, s>>>(B, key, B.n, nokey, nseg, ms_cnt, err, D.segclk, rmax_out);
      else k_la_ms_count<false><<<(unsigned)nseg, 256, 0, s>>>(B, key, B.n, nokey, nseg, ms_cnt, err, nullptr, nullptr);
      if (fc) k_la_seg_clock<<<1, 1024, 0, s>>>(D.segclk, nseg, B.clock0);
      (void)hipMemsetAsync(ms_cnt + nc - 1, 0, sizeof(uint32_t), s);
      kt.mark("labs_mscan", s);
      size_t tb = stmp_bytes;
      (void)rocprim::exclusive_scan(stmp, tb, ms_cnt, ms_off, 0u, nc, rocprim::plus<uint32_t>(), s);
      kt.mark("labs_split", s);
      (void)hipMemsetAsync(D.maxstep, 0, sizeof(unsigned long long), s);
      steps_done = true;
      if (fc) k_la_ms_scatter<true><<<(unsigned)nseg, 64, 0, s>>>(D, B, key, B.n, nokey, nseg, bits, ms_off, err, rmax_out);
      else k_la_ms_scatter<false><<<(unsigned)nseg, 64, 0, s>>>(D, B, key, B.n, nokey, nseg, bits, ms_off, err, nullptr);
      k_la_ms_bounds<<<(unsigned)((nokey + 255) / 256), 256, 0, s>>>(ms_off, nseg, nokey, kbeg, kcnt);
      kt.mark(nullptr, s);
      sorted = true;
      bounds = true;
      D.ev16 = 1;
      return;
    }
    kt.mark("labs_pack", s);
    if (B.n > 0) k_labs_pack2<<<2048, 256, 0, s>>>(D, B, key, B.n, (uint32_t)D.nk, skey_in, err);
    kt.mark("labs_sort", s);
    size_t tb = stmp_bytes;
    if (B.n > 0)
      (void)rocprim::radix_sort_pairs(stmp, tb, skey_in, skey_out, reinterpret_cast<LaEv16*>(D.p_ev),
                                      reinterpret_cast<LaEv16*>(D.s_ev), (size_t)B.n, 0, key_bits + 1, s);
    kt.mark(nullptr, s);
    sorted = true;
    D.ev16 = 1;
  }
  void sort_scratch(int64_t cap, int key_bits, hipStream_t s) {
    size_t b = 0;
    (void)rocprim::radix_sort_pairs(nullptr, b, (uint32_t*)nullptr, (uint32_t*)nullptr, (LaEv16*)nullptr,
                                    (LaEv16*)nullptr, (size_t)std::max<int64_t>(cap, 1), 0, key_bits + 1, s);
    if (split_ok(cap)) {
      const size_t nc = (size_t)(D.nk + 1) * (size_t)((std::max<int64_t>(cap, 1) + LA_MS_SEG - 1) / LA_MS_SEG) + 1;
      al(ms_cnt, (int64_t)nc);
      al(ms_off, (int64_t)nc);
      al(D.segclk, 2 * ((std::max<int64_t>(cap, 1) + LA_MS_SEG - 1) / LA_MS_SEG));
      size_t b2 = 0;
      (void)rocprim::exclusive_scan(nullptr, b2, ms_cnt, ms_off, 0u, nc, rocprim::plus<uint32_t>(), s);
      b = std::max(b, b2);
    }
    stmp_bytes = std::max<size_t>(b, 16);
    if (hipMalloc(&stmp, stmp_bytes) != hipSuccess) throw std::runtime_error("hipMalloc failed (logical-absent sort)");
  }

  void commit() { D.cur ^= 1; }

  // capacity tier t: new rings of LA_CAPS[t] per key; with migrate the committed waits move over
  // (else the caller overwrites them, e.g. a restore).  False when device memory is short.
  bool set_tier(int t, bool migrate, hipStream_t s) {
    if (t < 0 || t >= LA_TIERS) return false;
    LabsDev Dn = D;
    Dn.wcap = LA_CAPS[t];
    const int64_t n = (int64_t)D.nk * Dn.wcap;
    LaWait* q[3] = {nullptr, nullptr, nullptr};
    LaEnt* f[3] = {nullptr, nullptr, nullptr};
    bool ok = true;
    for (int i = 0; i < 3 && ok; i++)
      ok = hipMalloc((void**)&q[i], (size_t)n * sizeof(LaWait)) == hipSuccess &&
           hipMalloc((void**)&f[i], (size_t)n * sizeof(LaEnt)) == hipSuccess;
    if (!ok) {
      for (int i = 0; i < 3; i++) {
        if (q[i]) (void)hipFree(q[i]);
        if (f[i]) (void)hipFree(f[i]);
      }
      return false;
    }
    Dn.wq[0] = q[0];
    Dn.wq[1] = q[1];
    Dn.wtmp = q[2];
    Dn.fq[0] = f[0];
    Dn.fq[1] = f[1];
    Dn.ftmp = f[2];
    if (migrate) k_labs_migrate<<<(unsigned)((D.nk + 255) / 256), 256, 0, s>>>(Dn, D);
    if (hipStreamSynchronize(s) != hipSuccess) return false;
    for (void* p : {(void*)D.wq[0], (void*)D.wq[1], (void*)D.wtmp, (void*)D.fq[0], (void*)D.fq[1], (void*)D.ftmp})
      if (p) (void)hipFree(p);
    D = Dn;
    tier = t;
    return true;
  }

  void release() {
    for (int c = 0; c < 2; c++) {
      if (D.pend[c]) (void)hipFree(D.pend[c]);
      if (D.wq[c]) (void)hipFree(D.wq[c]);
      if (D.fq[c]) (void)hipFree(D.fq[c]);
    }
    if (D.wtmp) (void)hipFree(D.wtmp);
    if (D.ftmp) (void)hipFree(D.ftmp);
    void* qs[] = {D.cm, D.om, D.p_ev, D.s_ev, D.rec, D.stamps, stmp, D.maxstep, ms_cnt, ms_off, D.snap[0], D.snap[1], D.rc, D.segclk};
    for (void* p : qs)
      if (p) (void)hipFree(p);
    D = LabsDev{};
    stmp = nullptr;
    ms_cnt = ms_off = nullptr;
  }
};

}  // namespace shp
