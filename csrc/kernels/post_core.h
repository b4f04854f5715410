// Element functions of the post-match pipeline (host + device), shared by the per-batch kernels of
// lp_post.hip, the bucket-sorted bulk path of post_bulk.hip and the host twins: the same arithmetic
// and ordering rules on every backend (reference semantics: AnalysisService.java:89-156,
// ScoringService.java:84-88).
#pragma once
#include <stdint.h>

#include "lp_api.h"
#include "lp_core.h"

namespace lp {

// unused slots of a fixed-capacity key region: sorts after every real key, never a hit
constexpr uint64_t LP_PAD_KEY = ~0ull;

// segment of local line x: the last segment whose first line is <= x (a document with zero kept
// lines, e.g. "\n\n" under Java split, has lo == hi and is skipped by taking the last match)
LP_HD int seg_of(const int32_t* lo, int nseg, int32_t x) {
  int a = 0, b = nseg;
  while (b - a > 1) {
    const int m = (a + b) >> 1;
    if (lo[m] <= x) a = m; else b = m;
  }
  return a;
}

LP_HD int64_t lower_bound64(const int64_t* a, int64_t n, int64_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (a[m] < v) lo = m + 1; else hi = m;
  }
  return lo;
}

LP_HD int64_t lower_bound_u32(const uint32_t* a, int64_t n, uint32_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (a[m] < v) lo = m + 1; else hi = m;
  }
  return lo;
}

// events a hit produces: one per pattern whose primary regex it is, on lines the segment owns
LP_HD int64_t hit_event_count(const EvTables& E, int64_t key) {
  const int r = (int)(key >> 32);
  const int32_t x = (int32_t)(key & 0xFFFFFFFFll);
  const int64_t c = E.prim_off[r + 1] - E.prim_off[r];
  if (c == 0) return 0;
  const int s = seg_of(E.seg_lo, E.nseg, x);
  return (x >= E.own_lo[s] && x < E.own_hi[s]) ? c : 0;
}

// context window [a, b) of an event (AnalysisService.java:132-156 clipping; [x, x+1) when the
// pattern has no context rules)
LP_HD void event_window(const EvTables& E, int32_t x, int p, int s, int32_t& a, int32_t& b) {
  const int32_t before = E.ctx_before[p], after = E.ctx_after[p];
  if (before < 0) {
    a = x;
    b = x + 1;
    return;
  }
  const int64_t aa = (int64_t)x - before, bb = (int64_t)x + 1 + after;
  a = (int32_t)(aa < E.seg_lo[s] ? E.seg_lo[s] : aa);
  b = (int32_t)(bb > E.seg_hi[s] ? E.seg_hi[s] : bb);
}

// sorted packed keys ((regex << lbits | line) << 1 | pre-verified): the first key of every run is
// the hit; it holds when any copy was pre-verified or the regex's DFA accepts the line
LP_HD bool dedupe_verify_one(const uint64_t* keys, int64_t n, int64_t i, int lbits, const uint8_t* text,
                             const int64_t* ls, const int32_t* ll, const DfaPool& P, int64_t* std_key) {
  if (keys[i] == LP_PAD_KEY) {
    *std_key = 0;
    return false;
  }
  const uint64_t k = keys[i] >> 1;
  if (i > 0 && (keys[i - 1] >> 1) == k) return false;
  bool pre = false;  // pre-verified copies sort last inside a run
  for (int64_t j = i; j < n && (keys[j] >> 1) == k; ++j) pre |= (keys[j] & 1) != 0;
  const int r = (int)(k >> lbits);
  const int64_t x = (int64_t)(k & ((1ull << lbits) - 1));
  *std_key = ((int64_t)r << 32) | x;
  return pre || dfa_run(P, r, text + ls[x], ll[x]);
}

// per event (line << pbits | pattern) key: outputs, context window; returns the event's frequency
// sort key (its frequency key, or nkeys when it has none)
LP_HD uint32_t ev_post_one(const EvTables& E, uint64_t key, int64_t e, int32_t* ev_line, int32_t* ev_pat,
                           int32_t* ev_seg, int32_t& a, int32_t& b) {
  const int32_t x = (int32_t)(key >> E.pbits);
  const int p = (int)(key & ((1ull << E.pbits) - 1));
  const int s = seg_of(E.seg_lo, E.nseg, x);
  ev_line[e] = x;
  ev_pat[e] = p;
  ev_seg[e] = s;
  event_window(E, x, p, s, a, b);
  const int32_t fk = E.freq_key[p];
  return fk >= 0 ? (uint32_t)fk : (uint32_t)E.nkeys;
}

// rank of the event at sorted slot j among earlier events of the same frequency key
LP_HD void rank_one(const uint32_t* fs, const int32_t* idx, int64_t ne, int64_t j, int nkeys, int64_t* ev_rank,
                    int64_t* ev_fkey, int64_t* freq_counts) {
  const uint32_t fk = fs[j];
  const int32_t e = idx[j];
  if ((int)fk >= nkeys) {
    ev_rank[e] = -1;
    ev_fkey[e] = -1;
    return;
  }
  const int64_t start = lower_bound_u32(fs, j, fk);
  ev_rank[e] = j - start;
  ev_fkey[e] = fk;
  if (j + 1 == ne || fs[j + 1] != fk) freq_counts[fk] = j - start + 1;
}

// launchers of lp_post.hip kernels reused by the bulk path
void dedupe_verify_dev(const uint64_t* keys, int64_t n, int lbits, const uint8_t* text, const int64_t* ls,
                       const int32_t* ll, const DfaPool& P, int64_t* stdk, uint8_t* flag, uint64_t stream);
void feat_cov_dev(const int32_t* cov, int64_t L, const uint8_t* text, const int64_t* ls, const int32_t* ll,
                  const DfaPool& P, int ctx_trans, int ctx_acc, uint8_t* feat, uint64_t stream);

// bulk post-match path without device-wide radix sorts (post_bulk.hip); both return the workspace
// bytes they need and run only when ws_bytes suffices. *_ok: the layout limits of the path.
bool hits_bulk_ok(const HitsArgs& A);
size_t hits_bulk_dev(const HitsArgs& A, void* ws, size_t ws_bytes, uint64_t stream);
bool events_bulk_ok(const EventsArgs& A);
size_t events_bulk_dev(const EventsArgs& A, void* ws, size_t ws_bytes, uint64_t stream);

}  // namespace lp
