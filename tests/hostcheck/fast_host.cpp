// CPU debug harness for the specialised 2-state kernels (TESTS ONLY). Runs the exact
// per-item bodies of siddhi_amd/csrc/fast_core.h in host loops, with buffers sized as
// the engine sizes them, so AddressSanitizer and the oracle can check them without a GPU.
#include <algorithm>
#include <cstring>
#include <numeric>
#include <vector>

#include "../../siddhi_amd/csrc/compile.h"
#include "../../siddhi_amd/csrc/fast_core.h"

using namespace shp;

struct FH {
  ProgramCompiler comp;
  int nk;
  int64_t cap, mcap;
  std::vector<int64_t> c_seq, c_ts, c_val, last_ts, s_ts, s_val;
  std::vector<uint8_t> c_null, s_null, slow, last_cand;
  std::vector<int32_t> c_n, c_match, match;
  std::vector<uint32_t> nclose, moff, first_open;
  FastDev F{};
  int64_t seq = 0;
  std::vector<int32_t> key;
  std::vector<int64_t> ts, pos, refs;
  std::vector<int8_t> type;
  std::vector<int16_t> slot;
  int64_t m = 0;
};

extern "C" {

void* fh_create(const char* json, int max_keys, int64_t max_batch, int64_t max_matches) {
  auto* h = new FH();
  try {
    h->comp.compile(json);
  } catch (std::exception& e) {
    delete h;
    return nullptr;
  }
  if (!h->comp.fast.ok) { delete h; return nullptr; }
  h->nk = h->comp.P.partitioned ? max_keys : 1;
  h->cap = max_batch + 1;
  h->mcap = max_matches;
  int64_t nk = h->nk, cap = h->cap;
  h->c_seq.assign(nk * FCC, 0); h->c_ts.assign(nk * FCC, 0); h->c_val.assign(nk * FCC * 2, 0);
  h->c_null.assign(nk * FCC * 2, 0); h->c_n.assign(nk, 0); h->c_match.assign(nk * FCC, 0);
  h->last_ts.assign(nk, INT64_MIN); h->first_open.assign(nk, 0xffffffffu);
  h->slow.assign(nk, 0); h->last_cand.assign(nk, 0);
  h->s_ts.assign(cap, 0); h->s_val.assign(cap * 2, 0); h->s_null.assign(cap * 2, 0);
  h->match.assign(cap, 0); h->nclose.assign(cap, 0); h->moff.assign(cap + 1, 0);
  FastDev& F = h->F;
  F.within = h->comp.fast.within; F.nk = h->nk; F.nv = h->comp.P.ncol; F.f1 = h->comp.fast.f1; F.f2 = h->comp.fast.f2;
  F.c_seq = h->c_seq.data(); F.c_ts = h->c_ts.data(); F.c_val = h->c_val.data(); F.c_null = h->c_null.data();
  F.c_n = h->c_n.data(); F.c_match = h->c_match.data(); F.last_ts = h->last_ts.data(); F.s_ts = h->s_ts.data();
  F.s_val = h->s_val.data(); F.s_null = h->s_null.data(); F.match = h->match.data(); F.nclose = h->nclose.data();
  F.moff = h->moff.data(); F.first_open = h->first_open.data();
  F.slow = h->slow.data(); F.last_cand = h->last_cand.data(); F.fstream = h->comp.fast.stream;
  return h;
}

int fh_push(void* hp, int64_t n, const int64_t* ts, const int32_t* key, const int32_t* stream,
            const void* const* cols, const uint8_t* const* nulls) {
  FH* h = (FH*)hp;
  const DevProg& P = h->comp.P;
  if (n + 1 > h->cap) return -1;
  std::vector<uint32_t> perm(n), skey(n);
  std::iota(perm.begin(), perm.end(), 0);
  auto kof = [&](int64_t i) -> uint32_t { return stream[i] < 0 ? (uint32_t)h->nk : (P.partitioned ? key[i] : 0); };
  std::stable_sort(perm.begin(), perm.end(), [&](uint32_t a, uint32_t b) { return kof(a) < kof(b); });
  for (int64_t p = 0; p < n; p++) skey[p] = kof(perm[p]);
  std::vector<uint32_t> kbeg(h->nk + 1, 0), kcnt(h->nk + 1, 0);
  for (int64_t i = 0; i < n; i++) if (kof(i) < (uint32_t)h->nk) kcnt[kof(i)]++;
  for (int k = 1; k <= h->nk; k++) kbeg[k] = kbeg[k - 1] + kcnt[k - 1];
  BatchView B{};
  B.n = n; B.seq0 = h->seq; B.ts = ts; B.tclk = ts; B.stream = stream; B.partitioned = P.partitioned;
  for (int i = 0; i < P.ncol; i++) { B.cols[i] = cols[i]; B.nulls[i] = nulls ? nulls[i] : nullptr; }
  int err = 0;
  int fstream = h->comp.fast.stream;
  for (int64_t p = 0; p < n; p++) fast_gather_item(P, B, h->F, perm.data(), skey.data(), p, &err);
  for (int64_t i = 0; i < n; i++) fast_search_item(B, h->F, perm.data(), skey.data(), kbeg.data(), kcnt.data(), i, fstream);
  for (int64_t c = 0; c < (int64_t)h->nk * FCC; c++)
    fast_search_carry_item(B, h->F, perm.data(), kbeg.data(), kcnt.data(), c, fstream);
  for (int k = 0; k < h->nk; k++) fast_seq_item(h->F, B, perm.data(), kbeg.data(), kcnt.data(), k, fstream);
  uint32_t acc = 0;
  for (int64_t p = 0; p < n; p++) { h->moff[p] = acc; acc += h->nclose[p]; }
  int64_t total = acc;
  int64_t mcap = h->mcap, rcap = mcap * P.nstates * 2 + 64;
  if (total > mcap) return -4;
  std::vector<int32_t> mk(mcap); std::vector<int64_t> mts(mcap), mpos(mcap), moff(mcap), mrefs(rcap);
  std::vector<int8_t> mty(mcap); std::vector<int16_t> msl(mcap * MAXS);
  unsigned long long cnt[2] = {(unsigned long long)total, (unsigned long long)(2 * total)};
  MatchOut O{mcap, rcap, cnt, mk.data(), mts.data(), mty.data(), mpos.data(), moff.data(), msl.data(), mrefs.data()};
  for (int64_t q = 0; q < n; q++) fast_emit_item(h->F, B, O, perm.data(), skey.data(), kbeg.data(), q);
  for (int k = 0; k < h->nk; k++) fast_carry_item(h->F, B, perm.data(), kbeg.data(), kcnt.data(), k, &err);
  h->seq += n;
  int S = P.nstates;
  std::vector<int64_t> idx(total);
  std::iota(idx.begin(), idx.end(), 0);
  std::stable_sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) {
    if (mpos[a] != mpos[b]) return mpos[a] < mpos[b];
    if (mk[a] != mk[b]) return mk[a] < mk[b];
    return a < b;
  });
  for (int64_t j : idx) {
    h->key.push_back(mk[j]); h->ts.push_back(mts[j]); h->pos.push_back(mpos[j]); h->type.push_back(mty[j]);
    int64_t o = moff[j];
    for (int s = 0; s < S; s++) {
      h->slot.push_back(msl[j * MAXS + s]);
      for (int t = 0; t < msl[j * MAXS + s]; t++) h->refs.push_back(mrefs[o++]);
    }
  }
  h->m += total;
  return err;
}

int fh_num_states(void* hp) { return ((FH*)hp)->comp.P.nstates; }
int64_t fh_num_matches(void* hp) { return ((FH*)hp)->m; }
int64_t fh_num_refs(void* hp) { return (int64_t)((FH*)hp)->refs.size(); }
int fh_fetch(void* hp, int32_t* key, int64_t* ts, int8_t* type, int64_t* pos, int32_t* slot_len, int64_t* refs) {
  FH* h = (FH*)hp;
  for (int64_t i = 0; i < h->m; i++) { key[i] = h->key[i]; ts[i] = h->ts[i]; type[i] = h->type[i]; pos[i] = h->pos[i]; }
  for (size_t i = 0; i < h->slot.size(); i++) slot_len[i] = h->slot[i];
  for (size_t i = 0; i < h->refs.size(); i++) refs[i] = h->refs[i];
  h->key.clear(); h->ts.clear(); h->type.clear(); h->pos.clear(); h->slot.clear(); h->refs.clear(); h->m = 0;
  return 0;
}
void fh_destroy(void* hp) { delete (FH*)hp; }
}
