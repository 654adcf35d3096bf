// CPU debug harness for the lane interpreter (TESTS ONLY, never loaded by the product).
// Compiles siddhi_amd/csrc/nfa_lane.h for the host and drives it exactly like
// k_nfa_lanes does (stable key partition, running clock, one lane per key), so the
// lane logic can be checked against the oracle in a container without a GPU.
#include <algorithm>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "../../siddhi_amd/csrc/compile.h"
#include "../../siddhi_amd/csrc/nfa_lane.h"

using namespace shp;

struct HC {
  ProgramCompiler comp;
  LaneLayout Y;
  std::vector<char> arena;
  int nk;
  int64_t seq = 0, clock = 0, start = 0;
  std::vector<int32_t> key;
  std::vector<int64_t> ts, pos, off, refs;
  std::vector<int8_t> type;
  std::vector<int16_t> slot;
  int64_t m = 0;
  int err = 0;
};

// the lanes of one push at capacity tier T (LaneCaps), as k_nfa_lanes<T> runs them
template <int T>
static int run_lanes(HC* h, const BatchView& B, const MatchOut& O, const std::vector<uint32_t>& kbeg,
                     const std::vector<uint32_t>& kcnt, const std::vector<uint32_t>& perm, int64_t n) {
  const DevProg& P = h->comp.P;
  int err = 0;
  for (int k = 0; k < h->nk; k++) {
    LaneT<0, T> ln(P, h->Y, h->arena.data(), k, k, B, O);
    if (!P.partitioned && !ln.template at<uint8_t>(h->Y.o_kinit, 0)) {
      ln.clock = h->start; ln.emit_pos = h->seq; ln.init_partition();
    }
    int64_t lo = 0;
    for (uint32_t p = kbeg[k]; p < kbeg[k] + kcnt[k] && !ln.err; p++) {
      int64_t g = perm[p];
      ln.maybe_gc(); ln.timers(lo, g); ln.on_event(g); lo = g + 1;
    }
    if (!ln.err) { ln.maybe_gc(); ln.timers(lo, n - 1); }
    ln.flush_ret();
    err |= ln.err;
  }
  return err;
}

extern "C" {

// capacity tier of the arena (before the first push)
int hc_set_tier(void* hp, int tier) {
  HC* h = (HC*)hp;
  if (tier < 0 || tier >= LANE_TIERS) return -1;
  h->Y.build(h->nk, tier);
  h->arena.assign(h->Y.bytes, 0);
  return 0;
}

void* hc_create(const char* json, int64_t start_clock, int max_keys) {
  auto* h = new HC();
  try {
    h->comp.compile(json);
  } catch (std::exception& e) {
    fprintf(stderr, "hc_create: %s\n", e.what());
    delete h;
    return nullptr;
  }
  h->nk = h->comp.P.partitioned ? max_keys : 1;
  h->Y.build(h->nk);
  h->arena.assign(h->Y.bytes, 0);
  h->clock = h->start = start_clock;
  return h;
}

int hc_push(void* hp, int64_t n, const int64_t* ts, const int32_t* key, const int32_t* stream,
            const void* const* cols, const uint8_t* const* nulls, int clock_only) {
  HC* h = (HC*)hp;
  const DevProg& P = h->comp.P;
  std::vector<int64_t> rmax(n);
  int64_t c = h->clock;
  for (int64_t i = 0; i < n; i++) { c = std::max(c, ts[i]); rmax[i] = c; }
  std::vector<uint32_t> perm(n);
  std::iota(perm.begin(), perm.end(), 0);
  auto kof = [&](int64_t i) -> int64_t { return stream[i] < 0 ? (int64_t)h->nk : (P.partitioned ? key[i] : 0); };
  std::stable_sort(perm.begin(), perm.end(), [&](uint32_t a, uint32_t b) { return kof(a) < kof(b); });
  std::vector<uint32_t> kbeg(h->nk + 1, 0), kcnt(h->nk + 1, 0);
  for (int64_t i = 0; i < n; i++) {
    int64_t k = kof(i);
    if (k < h->nk) kcnt[k]++;
  }
  for (int k = 1; k <= h->nk; k++) kbeg[k] = kbeg[k - 1] + kcnt[k - 1];
  BatchView B{};
  B.n = n; B.seq0 = h->seq; B.clock0 = h->clock; B.init_clock = h->start; B.partitioned = P.partitioned;
  B.ts = ts; B.tclk = ts; B.stream = stream; B.rmax = rmax.data();
  for (int i = 0; i < P.ncol; i++) { B.cols[i] = cols[i]; B.nulls[i] = nulls ? nulls[i] : nullptr; }
  int64_t cap = 1 << 20;
  std::vector<int32_t> mk(cap); std::vector<int64_t> mts(cap), mpos(cap), moff(cap), mrefs(cap * 4);
  std::vector<int8_t> mty(cap); std::vector<int16_t> msl(cap * MAXS);
  unsigned long long cnt[2] = {0, 0};
  MatchOut O{cap, cap * 4, cnt, mk.data(), mts.data(), mty.data(), mpos.data(), moff.data(), msl.data(), mrefs.data()};
  int err = 0;
  if (h->Y.tier == 0) err = run_lanes<0>(h, B, O, kbeg, kcnt, perm, n);
  else if (h->Y.tier == 1) err = run_lanes<1>(h, B, O, kbeg, kcnt, perm, n);
  else if (h->Y.tier == 2) err = run_lanes<2>(h, B, O, kbeg, kcnt, perm, n);
  else if (h->Y.tier == 3) err = run_lanes<3>(h, B, O, kbeg, kcnt, perm, n);
  else err = run_lanes<4>(h, B, O, kbeg, kcnt, perm, n);
  if (n) h->clock = rmax[n - 1];
  if (!clock_only) h->seq += n;
  int64_t m = (int64_t)cnt[0];
  std::vector<int64_t> idx(m);
  std::iota(idx.begin(), idx.end(), 0);
  std::stable_sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) {
    if (mpos[a] != mpos[b]) return mpos[a] < mpos[b];
    if (mk[a] != mk[b]) return mk[a] < mk[b];
    return a < b;
  });
  int S = P.nstates;
  for (int64_t j : idx) {
    h->key.push_back(mk[j]); h->ts.push_back(mts[j]); h->pos.push_back(mpos[j]); h->type.push_back(mty[j]);
    int64_t o = moff[j];
    for (int s = 0; s < S; s++) {
      h->slot.push_back(msl[j * MAXS + s]);
      for (int t = 0; t < msl[j * MAXS + s]; t++) h->refs.push_back(mrefs[o++]);
    }
  }
  h->m += m;
  h->err |= err;
  return err;
}

int hc_num_states(void* hp) { return ((HC*)hp)->comp.P.nstates; }
int64_t hc_num_matches(void* hp) { return ((HC*)hp)->m; }
int64_t hc_num_refs(void* hp) { return (int64_t)((HC*)hp)->refs.size(); }
int hc_fast(void* hp) { return ((HC*)hp)->comp.fast.ok; }
int hc_fetch(void* hp, int32_t* key, int64_t* ts, int8_t* type, int64_t* pos, int32_t* slot_len, int64_t* refs) {
  HC* h = (HC*)hp;
  for (int64_t i = 0; i < h->m; i++) { key[i] = h->key[i]; ts[i] = h->ts[i]; type[i] = h->type[i]; pos[i] = h->pos[i]; }
  for (size_t i = 0; i < h->slot.size(); i++) slot_len[i] = h->slot[i];
  for (size_t i = 0; i < h->refs.size(); i++) refs[i] = h->refs[i];
  h->key.clear(); h->ts.clear(); h->type.clear(); h->pos.clear(); h->slot.clear(); h->refs.clear(); h->m = 0;
  return 0;
}
void hc_destroy(void* hp) { delete (HC*)hp; }
}
