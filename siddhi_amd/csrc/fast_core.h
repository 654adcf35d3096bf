// siddhi-hip: the specialised 2-state kernels' per-item bodies (host+device).
//
// For `every e1=S[f1] -> e2=S[f2] within W` the processor chain (SURVEY.md Appendix
// A.7, derived from StreamPreStateProcessor.processAndReturn/expireEvents :326-403 and
// the reversed same-stream order of PatternMultiProcessStreamReceiver :32-39) reduces,
// per key with non-decreasing timestamps, to: every event i with f1(i) opens candidate
// i; candidate i closes at the first later event j of the key with f2(i, j) and
// ts_j - ts_i <= W, else it expires; matches are emitted ordered by j, then i.
// Candidates are independent, so the work is data-parallel over events:
//   gather  key-sorted SoA (ts, predicate columns) + per-key ts monotonicity check
//   search  one item per candidate: forward scan to its closing event
//   seq     keys whose ts decrease: the processor chain replayed exactly, one item per key
//   emit    one item per closing event: backward scan writes (j, i) in order
//   carry   per key: candidates still open at the batch end -> next batch
// These bodies are SHP_HD so tests/hostcheck can run them under AddressSanitizer.
#pragma once
#include <stdint.h>

#include "nfa_lane.h"
#include "prog.h"

namespace shp {

constexpr int FCC = 64;  // carried open candidates per key

SHP_HD inline void at_add_u32(uint32_t* p, uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  atomicAdd(p, v);
#else
  *p += v;
#endif
}
SHP_HD inline void at_min_u32(uint32_t* p, uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  atomicMin(p, v);
#else
  if (v < *p) *p = v;
#endif
}
SHP_HD inline void at_or_i32(int* p, int v) {
#if defined(__HIP_DEVICE_COMPILE__)
  atomicOr(p, v);
#else
  *p |= v;
#endif
}

struct FastDev {
  FPred f1, f2;
  int64_t within;
  int32_t nk;            // keys
  int32_t nv;            // predicate columns (<= 2)
  int32_t fstream;       // the query's stream (program stream index)
  int32_t pad_;
  // carry (per key)
  int64_t* c_seq;        // nk * FCC
  int64_t* c_ts;
  int64_t* c_val;        // nk * FCC * 2  (value bits)
  uint8_t* c_null;       // nk * FCC * 2
  int32_t* c_n;          // nk
  int32_t* c_match;      // nk * FCC : matched sorted position, -1 dead, -2 open
  int64_t* last_ts;      // nk, INT64_MIN when unseen
  uint8_t* slow;         // nk: the key's ts decrease in this batch -> exact replay (fast_seq_item)
  uint8_t* last_cand;    // nk: the key's latest event opened a candidate (the last carried one; it
                         // is on the new-and-every list when the next event arrives)
  // batch scratch
  int64_t* s_ts;         // n (key-sorted)
  int64_t* s_val;        // n * 2
  uint8_t* s_null;       // n * 2
  int32_t* match;        // n : sorted position of closing event, -1 none/dead, -2 open, -3 not a candidate
  uint32_t* nclose;      // n
  uint32_t* moff;        // n (exclusive scan of nclose)
  uint32_t* first_open;  // nk : lowest sorted position of a still-open batch candidate
};

// Candidate / closing-event values live in registers (2 predicate columns each).
struct FVals {
  int64_t v0, v1;
  uint8_t n0, n1;  // null flags
};

SHP_HD inline Val fast_operand(const FOperand& o, const FVals& c, const FVals& e, bool has_e) {
  Val r{T_NULL, 0};
  if (o.kind == 0) {
    r.tag = o.tag;
    r.bits = o.imm;
    return r;
  }
  if (o.state == 1 && !has_e) return r;
  const FVals& x = o.state == 0 ? c : e;
  bool nul = o.pos == 0 ? x.n0 : x.n1;
  if (nul) return r;
  r.tag = o.tag;
  r.bits = o.pos == 0 ? x.v0 : x.v1;
  return r;
}

SHP_HD inline bool fast_term(const FTerm& t, const FVals& c, const FVals& e, bool has_e) {
  Instr in{};
  in.a = (uint8_t)t.cmp;
  in.b = (uint8_t)t.ptype;
  Val r = java_cmp(in, fast_operand(t.a, c, e, has_e), fast_operand(t.b, c, e, has_e));
  return r.bits != 0;
}

// FilterProcessor semantics: null / false drop (CompareConditionExpressionExecutor returns
// false on a null operand; And/Or short-circuit on Boolean.TRUE)
SHP_HD inline bool fast_pred(const FPred& p, const FVals& c, const FVals& e, bool has_e) {
  if (p.n == 0) return true;
  bool a = fast_term(p.t[0], c, e, has_e);
  if (p.n == 1) return a;
  if (p.combine == 0) return a && fast_term(p.t[1], c, e, has_e);
  return a || fast_term(p.t[1], c, e, has_e);
}

SHP_HD inline void fast_load(const DevProg& P, const BatchView& B, int64_t g, int64_t* v, uint8_t* nul) {
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

SHP_HD inline void fast_gather_item(const DevProg& P, const BatchView& B, const FastDev& F, const uint32_t* perm,
                                    const uint32_t* skey, int64_t p, int* err) {
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
    if (t < prev) F.slow[k] = 1;  // the closed form needs non-decreasing ts: replay the key exactly
  }
  (void)err;
}

// forward scan from `from` (sorted position) to `end` for the closing event of a candidate
SHP_HD inline int32_t fast_scan(const FastDev& F, const FVals& c, int64_t ti, int64_t from, int64_t end,
                                int fstream, const BatchView& B, const uint32_t* perm) {
  for (int64_t q = from; q < end; q++) {
    uint32_t g = perm[q];
    if (B.stream[g] != fstream) continue;  // other partition streams never reach this query
    int64_t tq = F.s_ts[q];
    if (tq - ti > F.within) return -1;  // expired (expireEvents before processAndReturn)
    FVals e{F.s_val[2 * q], F.s_val[2 * q + 1], F.s_null[2 * q], F.s_null[2 * q + 1]};
    if (fast_pred(F.f2, c, e, true)) return (int32_t)q;
  }
  return -2;  // still open at the batch end
}

// batch candidate at sorted position i
SHP_HD inline void fast_search_item(const BatchView& B, const FastDev& F, const uint32_t* perm, const uint32_t* skey,
                                    const uint32_t* kbeg, const uint32_t* kcnt, int64_t i, int fstream) {
  uint32_t k = skey[i];
  if (k >= (uint32_t)F.nk || B.stream[perm[i]] != fstream || F.slow[k]) {
    F.match[i] = -3;  // (a slow key's positions are set by fast_seq_item)
    return;
  }
  FVals c{F.s_val[2 * i], F.s_val[2 * i + 1], F.s_null[2 * i], F.s_null[2 * i + 1]};
  if (!fast_pred(F.f1, c, c, false)) {
    F.match[i] = -3;
    return;
  }
  int64_t end = (int64_t)kbeg[k] + kcnt[k];
  int32_t q = fast_scan(F, c, F.s_ts[i], i + 1, end, fstream, B, perm);
  F.match[i] = q;
  if (q >= 0) at_add_u32(&F.nclose[q], 1u);
  if (q == -2) at_min_u32(&F.first_open[k], (uint32_t)i);
}

// carried candidate c = key * FCC + j
SHP_HD inline void fast_search_carry_item(const BatchView& B, const FastDev& F, const uint32_t* perm,
                                          const uint32_t* kbeg, const uint32_t* kcnt, int64_t c, int fstream) {
  int32_t k = (int32_t)(c / FCC);
  int32_t j = (int32_t)(c % FCC);
  if (j >= F.c_n[k] || F.slow[k]) return;
  if (kcnt[k] == 0) {
    F.c_match[c] = -2;
    return;
  }
  FVals cv{F.c_val[2 * c], F.c_val[2 * c + 1], F.c_null[2 * c], F.c_null[2 * c + 1]};
  int64_t b = kbeg[k];
  int32_t q = fast_scan(F, cv, F.c_ts[c], b, b + kcnt[k], fstream, B, perm);
  F.c_match[c] = q;
  if (q >= 0) at_add_u32(&F.nclose[q], 1u);
}

// Exact replay of one key whose timestamps decrease (the closed form above assumes they do not):
// StreamPreStateProcessor.expireEvents (:326-361) expires the pending list from its head while
// |ts - now| > within and stops at the first live partial; the new-and-every list (the candidate
// the key's previous event opened) is expired whole; processAndReturn (:364-403) then tries every
// pending partial in list order with no expiry test.  Writes the same match / c_match / nclose /
// first_open the parallel items write for the other keys.
SHP_HD inline void fast_seq_item(const FastDev& F, const BatchView& B, const uint32_t* perm, const uint32_t* kbeg,
                                 const uint32_t* kcnt, int32_t k, int fstream) {
  if (!F.slow[k]) return;
  const int64_t b = kbeg[k], e = b + kcnt[k];
  const int64_t cb = (int64_t)k * FCC;
  const int cn = F.c_n[k];
  for (int j = 0; j < cn; j++) F.c_match[cb + j] = -2;
  for (int64_t i = b; i < e; i++) F.match[i] = -3;
  // list entries: carried j as -(j + 1), batch positions as themselves
  auto st = [&](int64_t x) -> int32_t& { return x < 0 ? F.c_match[cb + (-x - 1)] : F.match[x]; };
  auto tsx = [&](int64_t x) -> int64_t { return x < 0 ? F.c_ts[cb + (-x - 1)] : F.s_ts[x]; };
  auto valx = [&](int64_t x) -> FVals {
    if (x < 0) {
      const int64_t c = cb + (-x - 1);
      return FVals{F.c_val[2 * c], F.c_val[2 * c + 1], F.c_null[2 * c], F.c_null[2 * c + 1]};
    }
    return FVals{F.s_val[2 * x], F.s_val[2 * x + 1], F.s_null[2 * x], F.s_null[2 * x + 1]};
  };
  auto nexte = [&](int64_t x) -> int64_t { return x < 0 ? (x == -(int64_t)cn ? b : x - 1) : x + 1; };
  const int64_t first = cn > 0 ? -1 : b;
  int64_t prevc = (cn > 0 && F.last_cand[k]) ? -(int64_t)cn : INT64_MIN;
  uint32_t fo = 0xffffffffu;
  for (int64_t q = b; q < e; q++) {
    if (B.stream[perm[q]] != fstream) continue;  // other partition streams never reach the query
    const int64_t tq = F.s_ts[q];
    for (int64_t x = first; x != q; x = nexte(x)) {  // expireEvents: pending list from the head
      if (st(x) != -2) continue;
      if (x == prevc) break;
      const int64_t d = tsx(x) - tq;
      if (d > F.within || d < -F.within) st(x) = -1;
      else break;
    }
    if (prevc != INT64_MIN && st(prevc) == -2) {  // ... and the new-and-every list, whole
      const int64_t d = tsx(prevc) - tq;
      if (d > F.within || d < -F.within) st(prevc) = -1;
    }
    const FVals ev{F.s_val[2 * q], F.s_val[2 * q + 1], F.s_null[2 * q], F.s_null[2 * q + 1]};
    for (int64_t x = first; x != q; x = nexte(x)) {  // processAndReturn, list order
      if (st(x) != -2) continue;
      if (fast_pred(F.f2, valx(x), ev, true)) {
        st(x) = (int32_t)q;
        F.nclose[q] += 1;
      }
    }
    if (fast_pred(F.f1, ev, ev, false)) {
      F.match[q] = -2;
      prevc = q;
    } else {
      prevc = INT64_MIN;
    }
  }
  for (int64_t i = b; i < e; i++)
    if (F.match[i] == -2) {
      fo = (uint32_t)i;
      break;
    }
  F.first_open[k] = fo;
}

SHP_HD inline void fast_emit_item(const FastDev& F, const BatchView& B, const MatchOut& O, const uint32_t* perm,
                                  const uint32_t* skey, const uint32_t* kbeg, int64_t q) {
  uint32_t cnt = F.nclose[q];
  if (!cnt) return;
  uint32_t k = skey[q];
  int64_t base = F.moff[q];
  if (base + cnt > O.cap) return;
  int64_t tq = F.s_ts[q];
  int64_t seqq = bseq(B, perm[q]);
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
  // batch candidates closed by q lie in [kbeg, q) within W of ts_q: collect backwards,
  // place forwards (ascending i)
  uint32_t nb = cnt - w;
  uint32_t placed = 0;
  const bool slow = F.slow[k] != 0;  // no ts order to stop at
  for (int64_t i = q - 1; i >= (int64_t)kbeg[k] && placed < nb; i--) {
    if (!slow && tq - F.s_ts[i] > F.within) break;
    if (F.match[i] == (int32_t)q) {
      put(bseq(B, perm[i]), w + nb - 1 - placed);
      placed++;
    }
  }
}

SHP_HD inline void fast_carry_item(const FastDev& F, const BatchView& B, const uint32_t* perm, const uint32_t* kbeg,
                                   const uint32_t* kcnt, int32_t k, int* err) {
  uint32_t cnt = kcnt[k];
  F.slow[k] = 0;
  if (cnt == 0) return;
  int64_t b = kbeg[k], e = b + cnt;
  F.last_ts[k] = F.s_ts[e - 1];
  for (int64_t i = e - 1; i >= b; i--)  // the key's latest event of this query's stream
    if (B.stream[perm[i]] == F.fstream) {
      F.last_cand[k] = F.match[i] != -3 ? 1 : 0;
      break;
    }
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
      at_or_i32(err, E_LIST);
      break;
    }
    int64_t c = base + w;
    F.c_seq[c] = bseq(B, perm[i]);
    F.c_ts[c] = F.s_ts[i];
    F.c_val[2 * c] = F.s_val[2 * i];
    F.c_val[2 * c + 1] = F.s_val[2 * i + 1];
    F.c_null[2 * c] = F.s_null[2 * i];
    F.c_null[2 * c + 1] = F.s_null[2 * i + 1];
    w++;
  }
  F.c_n[k] = w;
}

}  // namespace shp
