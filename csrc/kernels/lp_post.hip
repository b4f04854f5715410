// Post-match pipeline: candidates -> hit CSR -> events in reference order -> in-batch frequency
// ranks -> context coverage -> context features. Replaces ~150 small framework ops and ~15 host
// round trips per batch with a handful of gfx950 kernels + rocPRIM device primitives on ONE
// stream and ONE 16-byte host read in the middle (sizes for the event buffers).
//
//   hits_dev    pack (regex, line) + "pre-verified" bit into a (1 + rbits + lbits)-bit key, radix
//               sort (only the bits in use), dedupe + DFA-verify the first key of every run
//               (k_dedupe_verify), select -> sorted unique hits = per-regex line CSR shared by the
//               primary / secondary / sequence roles; CSR offsets + per-hit event counts
//               (primary role x owned line, k_csr_evcount); inclusive scan -> event offsets.
//   events_dev  expand (line << pbits | pattern) keys (k_expand); radix sort = the reference's
//               event order (line, then pattern: AnalysisService.java:89-113); per event segment,
//               frequency key and context window (k_ev_post marks the window's lines covered);
//               stable radix sort by frequency key -> rank among earlier same-key events and
//               per-key counts (k_rank: the in-batch part of the penalty-before-record scan,
//               ScoringService.java:84-88); features only for covered lines (k_feat_cov, ContextAnalysisService.java:
//               46-117 reads the 4 features of window lines only).
//
// The host twins below run the same element functions (the LP_HD helpers of post_core.h) with
// std::sort, so CPU tests exercise the GPU arithmetic and ordering rules.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <numeric>
#include <rocprim/rocprim.hpp>
#include <stdexcept>
#include <string>
#include <vector>

#include "lp_api.h"
#include "lp_core.h"
#include "lp_host.h"
#include "post_core.h"

namespace lp {

#define LP_PCHECK(x)                                                                                            \
  do {                                                                                                          \
    hipError_t e_ = (x);                                                                                        \
    if (e_ != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e_) + " at " #x); \
  } while (0)

static inline hipStream_t pstream(uint64_t s) { return reinterpret_cast<hipStream_t>(s); }
static inline unsigned nblk(int64_t n, int t = 256) { return (unsigned)std::max<int64_t>(1, (n + t - 1) / t); }

int bits_for(int64_t n) {  // bits needed to hold values 0..n-1 (>= 1)
  int b = 1;
  while (b < 62 && (int64_t(1) << b) < n) ++b;
  return b;
}

// ---------------------------------------------------------------------------------------------
// kernels (element functions: post_core.h)

__global__ __launch_bounds__(256) void k_pack(const int64_t* __restrict__ cand, int64_t n, int64_t pre_from, int lbits,
                                              uint64_t* __restrict__ keys) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t k = cand[i];            // -1: a dropped key (failed verify, a relaxation's candidate)
  keys[i] = k < 0 ? LP_PAD_KEY
                  : (((((uint64_t)k >> 32) << lbits) | ((uint64_t)k & 0xFFFFFFFFull)) << 1) | (i >= pre_from ? 1ull : 0ull);
}

// device-count mode: region 1 (to verify) then region 2 (pre-verified), each a fixed capacity
// with its used length in a device counter; unused slots become LP_PAD_KEY (post_core.h), which
// sorts after every real key (bit kbits set; the sort covers one extra bit)
__global__ __launch_bounds__(256) void k_pack_dc(const int64_t* __restrict__ cand, int64_t cap1,
                                                 const int64_t* __restrict__ cand2, int64_t cap2,
                                                 const unsigned long long* __restrict__ dcount, int lbits,
                                                 uint64_t* __restrict__ keys) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cap1 + cap2) return;
  const int64_t n1 = (int64_t)min((unsigned long long)cap1, dcount[0]);
  const int64_t n2 = (int64_t)min((unsigned long long)cap2, dcount[1]);
  uint64_t key = LP_PAD_KEY;
  const bool pre = i >= cap1;
  const int64_t j = pre ? i - cap1 : i;
  if (j < (pre ? n2 : n1)) {
    const int64_t k = pre ? cand2[j] : cand[j];
    if (k >= 0) key = (((((uint64_t)k >> 32) << lbits) | ((uint64_t)k & 0xFFFFFFFFull)) << 1) | (pre ? 1ull : 0ull);
  }
  keys[i] = key;
}


__global__ __launch_bounds__(256) void k_dedupe_verify(const uint64_t* __restrict__ keys, int64_t n, int lbits,
                                                       const uint8_t* __restrict__ text,
                                                       const int64_t* __restrict__ ls, const int32_t* __restrict__ ll,
                                                       DfaPool P, int64_t* __restrict__ std_key,
                                                       uint8_t* __restrict__ flag) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int64_t sk = 0;
  flag[i] = dedupe_verify_one(keys, n, i, lbits, text, ls, ll, P, &sk) ? 1 : 0;
  std_key[i] = sk;
}

__global__ __launch_bounds__(256) void k_csr_evcount(const int64_t* __restrict__ hits,
                                                     const int64_t* __restrict__ counters, int64_t n, int R, EvTables E,
                                                     int64_t* __restrict__ hit_off, int32_t* __restrict__ hit_line,
                                                     int64_t* __restrict__ ev_cnt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nh = counters[0];
  if (i <= R) hit_off[i] = lower_bound64(hits, nh, (int64_t)i << 32);
  if (i < n) {
    if (i < nh) {
      const int64_t k = hits[i];
      hit_line[i] = (int32_t)(k & 0xFFFFFFFFll);
      ev_cnt[i] = hit_event_count(E, k);
    } else {
      ev_cnt[i] = 0;
    }
  }
}

__global__ void k_total(const int64_t* __restrict__ ev_end, int64_t n, int64_t* __restrict__ counters) {
  if (threadIdx.x == 0 && blockIdx.x == 0) counters[1] = n > 0 ? ev_end[n - 1] : 0;
}

__global__ __launch_bounds__(256) void k_expand(const int64_t* __restrict__ hits, int64_t nh,
                                                const int64_t* __restrict__ ev_cnt, const int64_t* __restrict__ ev_end,
                                                EvTables E, uint64_t* __restrict__ evk) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nh) return;
  const int64_t c = ev_cnt[i];
  if (c == 0) return;
  const int64_t k = hits[i];
  const int r = (int)(k >> 32);
  const uint64_t x = (uint64_t)(k & 0xFFFFFFFFll);
  const int64_t base = ev_end[i] - c, p0 = E.prim_off[r];
  for (int64_t j = 0; j < c; ++j) evk[base + j] = (x << E.pbits) | (uint64_t)E.prim_pats[p0 + j];
}


__global__ __launch_bounds__(256) void k_ev_post(const uint64_t* __restrict__ evk, int64_t ne, EvTables E,
                                                 int32_t* __restrict__ ev_line, int32_t* __restrict__ ev_pat,
                                                 int32_t* __restrict__ ev_seg, uint32_t* __restrict__ fsort,
                                                 int32_t* __restrict__ idx, int32_t* __restrict__ cov) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= ne) return;
  int32_t a, b;
  fsort[e] = ev_post_one(E, evk[e], e, ev_line, ev_pat, ev_seg, a, b);
  idx[e] = (int32_t)e;
  // window coverage: mark the window's lines (consumers test cov > 0; equal concurrent stores
  // from overlapping windows are benign) -- no difference array, no scan over all L lines
  for (int32_t x = a; x < b; ++x) cov[x] = 1;
}


__global__ __launch_bounds__(256) void k_rank(const uint32_t* __restrict__ fs, const int32_t* __restrict__ idx,
                                              int64_t ne, int nkeys, int64_t* __restrict__ ev_rank,
                                              int64_t* __restrict__ ev_fkey, int64_t* __restrict__ freq_counts) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < ne) rank_one(fs, idx, ne, j, nkeys, ev_rank, ev_fkey, freq_counts);
}

// Context walk on row-offset tables (k_feat_cov's LDS path). DFA k's states are rows of W_k =
// nc_k + 2 uint16 entries: column 0 = hold (the row's own offset), columns 1..nc_k = the BYTE offset
// (from the table base) of the next state's row, column nc_k + 1 = the state's accept flags. The
// dead and match states (0, 1) hold on every column. One packed word per byte, bm4[c], holds
// 2 * column of byte c for the 4 DFAs in its 4 bytes; a byte outside the walked range uses 0
// (hold). A step is one byte extract + one 3-way add + one ds_read_u16 per DFA: about half the
// VALU work of the state-id walk (mad, address, terminal-state select), which is what bound
// k_feat_cov (profiles/r3_al: 22 us without walks, 110 us with).
struct CtxRows {
  int w2[4];      // 2 * W_k (row bytes)
  int live[4];    // byte offset of state 2's row: offsets >= live[k] are live states
  int one[4];     // byte offset of state 1's row (match found)
};

__device__ __forceinline__ uint32_t ctx_row_ld(const uint8_t* rows, uint32_t off) {
  return *reinterpret_cast<const uint16_t*>(rows + off);
}

__device__ __forceinline__ void ctx_rows_advance(const uint8_t* rows, const uint32_t* bm4, const CtxRows& R,
                                                 const uint8_t* s, int e, uint32_t (&off)[4]) {
  if (e <= 0) return;
  const int sh = (int)((uintptr_t)s & 15);
  const uint4* blk = reinterpret_cast<const uint4*>(s - sh);
  uint4 cur = blk[0];
  for (int t0 = -sh; t0 < e; t0 += 16) {
    const uint4 nxt = blk[1];
    ++blk;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int t = t0 + j;
      const uint32_t w = (j < 4) ? cur.x : (j < 8) ? cur.y : (j < 12) ? cur.z : cur.w;
      const uint32_t c = (w >> (8 * (j & 3))) & 0xFFu;
      const uint32_t b = ((t >= 0) & (t < e)) ? bm4[c] : 0u;
#pragma unroll
      for (int k = 0; k < 4; ++k) off[k] = ctx_row_ld(rows, off[k] + ((b >> (8 * k)) & 0xFFu));
    }
    cur = nxt;
    bool alive = false;
#pragma unroll
    for (int k = 0; k < 4; ++k) alive |= off[k] >= (uint32_t)R.live[k];
    if (!alive) return;
  }
}

// Matcher.find semantics of dfa_find_k / context_feat on the row-offset tables
__device__ __forceinline__ uint8_t ctx_rows_feat(const uint8_t* rows, const uint32_t* bm4, const CtxRows& R,
                                                 const uint8_t* s, int n) {
  uint32_t off[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) off[k] = (uint32_t)R.live[k];       // state 2 = start
  const int ftl = final_term_len(s, n);
  const int ft = ftl ? n - ftl : n;
  ctx_rows_advance(rows, bm4, R, s, ft, off);
  if (ftl) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (off[k] >= (uint32_t)R.live[k] && (ctx_row_ld(rows, off[k] + R.w2[k] - 2) & 2)) off[k] = (uint32_t)R.one[k];
    ctx_rows_advance(rows, bm4, R, s + ft, ftl, off);
  }
  uint32_t res = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bool acc = off[k] == (uint32_t)R.one[k] ||
                     (off[k] >= (uint32_t)R.live[k] && (ctx_row_ld(rows, off[k] + R.w2[k] - 2) & 1));
    res |= (acc ? 1u : 0u) << k;
  }
  const uint8_t f = (res & 1u) ? 1 : ((res & 2u) ? 2 : 0);
  return (uint8_t)(f | (res & 12u));
}

// Context features of covered lines. A block owns `per_block` consecutive lines: it compacts the
// covered ones into an LDS list (uncovered lines get 0) and then runs the 4 DFAs with every lane
// busy -- covered lines come in short runs, so one lane per line would idle most of each wave.
// The 4 context DFAs (~2 KB) are staged in LDS: a DFA walk is a chain of dependent table loads,
// ~64-cycle LDS hits instead of ~500-cycle L2 trips (a 10k-line request ran 136 us -> see profiles).
constexpr int FC_MAX_LINES = 4096;
constexpr int FC_TRANS = 4096;   // uint16 entries (context DFAs need ~900)
constexpr int FC_ACC = 1024;
constexpr int FC_ROWS = FC_TRANS; // uint16 row-offset entries (context DFAs need ~1,100)
__global__ __launch_bounds__(256) void k_feat_cov(const int32_t* __restrict__ cov, int64_t L, int per_block,
                                                  const uint8_t* __restrict__ text, const int64_t* __restrict__ ls,
                                                  const int32_t* __restrict__ ll, DfaPool P, int ctx_trans,
                                                  int ctx_acc, uint8_t* __restrict__ feat) {
  __shared__ uint16_t list[FC_MAX_LINES];         // block-relative line numbers (< FC_MAX_LINES)
  __shared__ int n;
  __shared__ int32_t s_meta[16];
  __shared__ __attribute__((aligned(16))) uint8_t s_bm[4 * 256];
  __shared__ __attribute__((aligned(16))) uint16_t s_trans[FC_TRANS];
  __shared__ uint8_t s_acc[FC_ACC];
  // the row-offset path keeps its tables in the state-id path's arrays (one of the two is used)
  uint16_t* s_rows = s_trans;
  uint32_t* s_bm4 = reinterpret_cast<uint32_t*>(s_bm);
  // row-offset tables (ctx_rows_feat) when they fit: rows of nc_k + 2 entries, columns in a byte
  int nst[4], W[4], rbase[4];
  int rows_total = 0;
  bool fit = true;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int nc = P.meta[4 * k + 1];
    const int t0 = P.meta[4 * k], t1 = k < 3 ? P.meta[4 * k + 4] : ctx_trans;
    nst[k] = nc > 0 ? (t1 - t0) / nc : 0;
    W[k] = nc + 2;
    rbase[k] = rows_total;
    rows_total += nst[k] * W[k];
    fit = fit && nc > 0 && 2 * (nc + 1) <= 255 && nst[k] >= 3 && t0 >= 0 && t1 <= ctx_trans;
  }
  const bool lds = ctx_trans <= FC_TRANS && ctx_acc <= FC_ACC;
  const bool rows_ok = fit && rows_total <= FC_ROWS && 2 * rows_total < 65536;
  CtxRows R;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    R.w2[k] = 2 * W[k];
    R.live[k] = 2 * (rbase[k] + 2 * W[k]);
    R.one[k] = 2 * (rbase[k] + W[k]);
  }
  if (threadIdx.x == 0) n = 0;
  if (rows_ok) {
    for (int i = threadIdx.x; i < rows_total; i += blockDim.x) {
      int k = 0;
#pragma unroll
      for (int q = 1; q < 4; ++q) k += i >= rbase[q] ? 1 : 0;
      const int loc = i - rbase[k], st = loc / W[k], col = loc - st * W[k];
      const int self = 2 * (rbase[k] + st * W[k]);
      int v;
      if (col == 0) v = self;
      else if (col == W[k] - 1) v = P.acc[P.meta[4 * k + 2] + st];
      else if (st < 2) v = self;
      else v = 2 * (rbase[k] + (int)P.trans[P.meta[4 * k] + st * (W[k] - 2) + col - 1] * W[k]);
      s_rows[i] = (uint16_t)v;
    }
    {
      const int c = threadIdx.x;                  // blockDim.x == 256
      uint32_t b = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) b |= (uint32_t)(2 * (P.bytemap[256 * k + c] + 1)) << (8 * k);
      s_bm4[c] = b;
    }
  } else if (lds) {
    if (threadIdx.x < 16) s_meta[threadIdx.x] = P.meta[threadIdx.x];
    lds_fill<uint8_t, 4>(s_bm, P.bytemap, 4 * 256);
    lds_fill<uint16_t, 4>(s_trans, P.trans, ctx_trans);
    lds_fill<uint8_t, 4>(s_acc, P.acc, ctx_acc);
  }
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * per_block;
  for (int k = threadIdx.x; k < per_block; k += blockDim.x) {
    const int64_t x = base + k;
    if (x < L) {                                 // (no coverage array: every line)
      if (!cov || cov[x] > 0) list[atomicAdd(&n, 1)] = (uint16_t)k;
      else feat[x] = 0;
    }
  }
  __syncthreads();
  const int m = n;
  // two call sites, each with a provable address space: the LDS copy compiles to ds_read (a
  // runtime select between LDS and global pointers degrades every table read to a flat load)
  if (rows_ok) {
    const uint8_t* rows = reinterpret_cast<const uint8_t*>(s_rows);
    for (int j = threadIdx.x; j < m; j += blockDim.x) {
      const int64_t x = base + list[j];
      feat[x] = ctx_rows_feat(rows, s_bm4, R, text + ls[x], ll[x]);
    }
  } else if (lds) {
    const DfaPool Q{s_meta, s_bm, s_trans, s_acc};
    for (int j = threadIdx.x; j < m; j += blockDim.x) {
      const int64_t x = base + list[j];
      feat[x] = context_feat(Q, text + ls[x], ll[x]);
    }
  } else {
    for (int j = threadIdx.x; j < m; j += blockDim.x) {
      const int64_t x = base + list[j];
      feat[x] = context_feat(P, text + ls[x], ll[x]);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Small batches (a request of a few thousand lines): the whole hit stage and the whole event stage
// are ONE workgroup each -- LDS bitonic sorts and block scans replace the rocPRIM sort / select /
// scan launches and their temp-storage passes (8 + 9 launches -> 1 + 1). Same results as the bulk
// path: sorted unique hits, events in (line, pattern) order, ranks from a stable sort by key.
constexpr int SB_THREADS = 1024;
constexpr int SB_MAX = 4096;           // keys / events held in LDS
constexpr int SB_MAX_LINES = 16384;    // window-coverage difference array in LDS

// Diagnostic phase clock of the two single-workgroup kernels (set_small_profile): thread 0 stores
// wall_clock64() after each phase into g_sb_prof[slot] (null: off, one scalar load per phase).
// Slots 0-4 k_hits_small, 8-13 k_events_small (5: live keys, 14: events); k_request_tail runs both
// bodies and adds 6 (score), 7 (frequency record), 15 (publish).
__device__ int64_t* g_sb_prof = nullptr;
#define LP_SB_STAMP(slot)                                                    \
  do {                                                                     \
    int64_t* pp_ = g_sb_prof;                                              \
    if (pp_ && threadIdx.x == 0) pp_[slot] = (int64_t)wall_clock64();     \
  } while (0)

__device__ __forceinline__ int sb_pow2(int64_t n) {
  int p = 64;
  while (p < n) p <<= 1;
  return p;
}

// ascending bitonic sort of s[0, n) (n a power of two <= SB_MAX), whole block
__device__ void sb_sort(uint64_t* s, int n) {
  for (int size = 2; size <= n; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < n / 2; t += SB_THREADS) {
        const int lo = 2 * t - (t & (stride - 1)), hi = lo + stride;
        const uint64_t a = s[lo], b = s[hi];
        if ((b < a) == ((lo & size) == 0)) {
          s[lo] = b;
          s[hi] = a;
        }
      }
      __syncthreads();
    }
}

constexpr int SB_RANK_MAX = 512;   // live keys up to which sb_sort_live ranks instead of sorting

// Ascending sort of the n live keys s[0, n) (the slots past n keep their pad keys), whole block.
// Up to SB_RANK_MAX keys by RANKS: key t goes to #{j : s[j] < s[t]} + #{j < t : s[j] == s[t]}
// (duplicates keep distinct slots), G = 2..64 lanes per key count a share of the j's and reduce by
// shuffles -- one pass of independent broadcast LDS reads and two barriers. A request's 90-250 keys
// sorted by the bitonic network took 4.6-6 us in its 28-36 dependent LDS + barrier steps
// (tools/small_phases.py; a register / shuffle network measured the same per step). Larger n:
// the bitonic sort of the padded power of two np.
__device__ void sb_sort_live(uint64_t* s, int n, int np) {
  if (n > SB_RANK_MAX) {
    sb_sort(s, np);
    return;
  }
  int G = 2;
  while (G < 64 && 2 * G * n <= SB_THREADS) G <<= 1;
  const int t = (int)threadIdx.x / G, part = (int)threadIdx.x & (G - 1);
  const uint64_t key = t < n ? s[t] : 0ull;
  int cnt = 0;
  if (t < n) {
    // 8 independent broadcast reads in flight per step (a loop of one read at a time waited on each)
    int j = part;
    for (; j + 7 * G < n; j += 8 * G) {
      uint64_t v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = s[j + u * G];
#pragma unroll
      for (int u = 0; u < 8; ++u) cnt += (v[u] < key || (v[u] == key && j + u * G < t)) ? 1 : 0;
    }
    for (; j < n; j += G) {
      const uint64_t v = s[j];
      cnt += (v < key || (v == key && j < t)) ? 1 : 0;
    }
  }
  for (int d = 1; d < G; d <<= 1) cnt += __shfl_xor(cnt, d, 64);
  __syncthreads();
  if (t < n && part == 0) s[cnt] = key;
  __syncthreads();
}

// exclusive prefix of v over the block (thread order); *total = block sum. Uses scratch[SB_THREADS/64 + 1].
__device__ int64_t sb_excl_scan(int64_t v, int64_t* scratch, int64_t* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int64_t incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const long long u = __shfl_up((long long)incl, d, 64);
    if (lane >= d) incl += u;
  }
  if (lane == 63) scratch[wid] = incl;
  __syncthreads();
  int64_t base = 0, tot = 0;
  for (int w = 0; w < SB_THREADS / 64; ++w) {
    if (w < wid) base += scratch[w];
    tot += scratch[w];
  }
  __syncthreads();
  *total = tot;
  return base + incl - v;
}

// small path, step 1 (all CUs): DFA-verify every prefilter candidate in place (a failed one
// becomes -1). A DFA walk is a chain of dependent table loads; in one workgroup the ~1k walks
// of a request queue behind one CU's memory pipeline, spread over the grid they do not.
__global__ __launch_bounds__(256) void k_cand_verify(HitsArgs A) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n1 = A.dcount ? (int64_t)min((unsigned long long)A.pre_from, A.dcount[0]) : A.pre_from;
  if (i >= n1) return;
  int64_t* cand = const_cast<int64_t*>(A.cand);
  const int64_t k = cand[i];
  if (k < 0) return;                           // dropped (a relaxation's key: k_take_host)
  const int r = (int)(k >> 32);
  if (is_bpg(A.dfa, r)) return;                // bit-parallel Glushkov program: k_bpg_cand
  const int64_t x = k & 0xFFFFFFFFll;
  if (!dfa_run(A.dfa, r, A.text + A.ls[x], A.ll[x])) cand[i] = -1;
}

// small path, step 2 (one workgroup): every remaining candidate is verified; sort, keep the first
// of each (regex, line) run, CSR, event counts and their scan
// the body of k_hits_small on LDS arrays the caller declares (keys / hk: SB_MAX entries, scratch:
// SB_THREADS / 64 + 1); *s_nh / *s_ne (LDS) receive the hit and event counts
__device__ __forceinline__ void hits_small_body(const HitsArgs& A, uint64_t* keys, int64_t* hk, int64_t* scratch,
                                                int* s_live_p, int64_t* s_nh, int64_t* s_ne) {
  int& s_live = *s_live_p;
  const int64_t n = A.n;
  const bool dc = A.dcount != nullptr;
  const int64_t n1 = dc ? (int64_t)min((unsigned long long)A.pre_from, A.dcount[0]) : A.pre_from;
  const int64_t n2 = dc ? (int64_t)min((unsigned long long)(n - A.pre_from), A.dcount[1]) : n - A.pre_from;
  // the live entries of both regions, compacted (most prefilter candidates failed their verify and
  // are -1): the sort covers pow2(live), not pow2(used) or the capacities
  LP_SB_STAMP(0);
  if (threadIdx.x == 0) s_live = 0;
  __syncthreads();
  for (int64_t i = threadIdx.x; i < n1 + n2; i += SB_THREADS) {
    const bool pre = i >= n1;
    const int64_t k = pre ? (dc ? A.cand2[i - n1] : A.cand[A.pre_from + i - n1]) : A.cand[i];
    if (k >= 0)                     // -1: failed k_cand_verify; every other key counts as verified
      keys[atomicAdd(&s_live, 1)] = (((((uint64_t)k >> 32) << A.lbits) | ((uint64_t)k & 0xFFFFFFFFull)) << 1) | 1ull;
  }
  __syncthreads();
  const int live = s_live;
  const int np = sb_pow2(live);
  for (int i = live + threadIdx.x; i < np; i += SB_THREADS) keys[i] = LP_PAD_KEY;
  __syncthreads();
  LP_SB_STAMP(1);
  sb_sort_live(keys, live, np);
  LP_SB_STAMP(2);
  // dedupe + DFA verify, then compaction in sorted order: 4 consecutive keys per thread
  constexpr int PER = SB_MAX / SB_THREADS;
  bool keep[PER];
  int64_t sk[PER];
  int c = 0;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int i = threadIdx.x * PER + q;
    keep[q] = i < np && dedupe_verify_one(keys, np, i, A.lbits, A.text, A.ls, A.ll, A.dfa, &sk[q]);
    c += keep[q];
  }
  int64_t nh = 0;
  int64_t o = sb_excl_scan(c, scratch, &nh);
#pragma unroll
  for (int q = 0; q < PER; ++q)
    if (keep[q]) {
      hk[o] = sk[q];
      A.hits[o] = sk[q];
      ++o;
    }
  __syncthreads();
  LP_SB_STAMP(3);
  // CSR per regex, hit lines, events per hit and their inclusive scan (4 consecutive per thread)
  for (int r = threadIdx.x; r <= A.R; r += SB_THREADS) A.hit_off[r] = lower_bound64(hk, nh, (int64_t)r << 32);
  int64_t ec[PER], e = 0;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int i = threadIdx.x * PER + q;
    ec[q] = 0;
    if (i < nh) {
      A.hit_line[i] = (int32_t)(hk[i] & 0xFFFFFFFFll);
      ec[q] = hit_event_count(A.ev, hk[i]);
      A.ev_cnt[i] = ec[q];
    }
    e += ec[q];
  }
  int64_t ne = 0;
  int64_t run = sb_excl_scan(e, scratch, &ne);
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int i = threadIdx.x * PER + q;
    run += ec[q];
    if (i < nh) A.ev_end[i] = run;
  }
  if (threadIdx.x == 0) {
    A.counters[0] = nh;
    A.counters[1] = ne;
    *s_nh = nh;
    *s_ne = ne;
  }
  LP_SB_STAMP(4);
  if (threadIdx.x == 0 && g_sb_prof) g_sb_prof[5] = live;
}

__global__ __launch_bounds__(SB_THREADS) void k_hits_small(HitsArgs A) {
  __shared__ uint64_t keys[SB_MAX];
  __shared__ int64_t hk[SB_MAX];
  __shared__ int64_t scratch[SB_THREADS / 64 + 1];
  __shared__ int s_live;
  __shared__ int64_t s_nh, s_ne;
  hits_small_body(A, keys, hk, scratch, &s_live, &s_nh, &s_ne);
}



// the body of k_events_small for nh hits and ne events (both within the capacities) on LDS arrays the
// caller declares (keys: SB_MAX, diff: SB_MAX_LINES + 1, scratch: SB_THREADS / 64 + 1)
__device__ __forceinline__ void events_small_body(const EventsArgs& A, int32_t* __restrict__ cov_out, uint64_t* keys,
                                                  int32_t* diff, int64_t* scratch, int64_t nh, int64_t ne) {
  const EvTables& E = A.ev;
  const int64_t L = A.L;
  const int np = sb_pow2(ne);
  LP_SB_STAMP(8);
  for (int i = threadIdx.x; i <= L; i += SB_THREADS) diff[i] = 0;
  for (int k = threadIdx.x; k < E.nkeys; k += SB_THREADS) A.freq_counts[k] = 0;
  for (int i = threadIdx.x; i < np; i += SB_THREADS) keys[i] = LP_PAD_KEY;
  __syncthreads();
  // expand: each hit's events, keyed (line, pattern)
  for (int64_t i = threadIdx.x; i < nh; i += SB_THREADS) {
    const int64_t c = A.ev_cnt[i];
    if (c == 0) continue;
    const int64_t k = A.hits[i];
    const int r = (int)(k >> 32);
    const uint64_t x = (uint64_t)(k & 0xFFFFFFFFll);
    const int64_t b0 = A.ev_end[i] - c, p0 = E.prim_off[r];
    for (int64_t j = 0; j < c; ++j) keys[b0 + j] = (x << E.pbits) | (uint64_t)E.prim_pats[p0 + j];
  }
  __syncthreads();
  LP_SB_STAMP(9);
  sb_sort_live(keys, (int)ne, np);
  LP_SB_STAMP(10);
  // per event: outputs + window coverage; then re-key by (frequency key, event) for the ranks
  for (int e = threadIdx.x; e < ne; e += SB_THREADS) {
    int32_t a, b;
    const uint32_t fs = ev_post_one(E, keys[e], e, A.ev_line, A.ev_pat, A.ev_seg, a, b);
    if (a < b) {
      atomicAdd(diff + a, 1);
      atomicAdd(diff + b, -1);
    }
    keys[e] = ((uint64_t)fs << 32) | (uint32_t)e;
  }
  __syncthreads();
  LP_SB_STAMP(11);
  sb_sort_live(keys, (int)ne, np);
  LP_SB_STAMP(12);
  for (int j = threadIdx.x; j < ne; j += SB_THREADS) {
    const uint32_t fk = (uint32_t)(keys[j] >> 32);
    const int32_t e = (int32_t)(keys[j] & 0xFFFFFFFFull);
    if ((int)fk >= E.nkeys) {
      A.ev_rank[e] = -1;
      A.ev_fkey[e] = -1;
      continue;
    }
    int64_t lo = 0, hi = j;                      // first slot of this key
    while (lo < hi) {
      const int64_t m = (lo + hi) >> 1;
      if ((uint32_t)(keys[m] >> 32) < fk) lo = m + 1; else hi = m;
    }
    A.ev_rank[e] = j - lo;
    A.ev_fkey[e] = fk;
    if (j + 1 == ne || (uint32_t)(keys[j + 1] >> 32) != fk) A.freq_counts[fk] = j - lo + 1;
  }
  // coverage = inclusive scan of diff over [0, L): contiguous runs per thread
  const int64_t per = (L + SB_THREADS - 1) / SB_THREADS;
  const int64_t lo = (int64_t)threadIdx.x * per, hi = lo + per < L ? lo + per : L;
  int64_t s = 0;
  for (int64_t i = lo; i < hi; ++i) s += diff[i];
  int64_t tot = 0;
  int64_t run = sb_excl_scan(s, scratch, &tot);
  for (int64_t i = lo; i < hi; ++i) {
    run += diff[i];
    cov_out[i] = (int32_t)run;
  }
  LP_SB_STAMP(13);
  if (threadIdx.x == 0 && g_sb_prof) g_sb_prof[14] = ne;
}

__global__ __launch_bounds__(SB_THREADS) void k_events_small(EventsArgs A, int32_t* __restrict__ cov_out) {
  __shared__ uint64_t keys[SB_MAX];
  __shared__ int32_t diff[SB_MAX_LINES + 1];
  __shared__ int64_t scratch[SB_THREADS / 64 + 1];
  int64_t ne = A.ne, nh = A.nh;
  if (A.dcounts) {                 // device-count mode: A.ne / A.nh are capacities
    nh = A.dcounts[0];
    ne = A.dcounts[1];
    const bool over = ne > A.ne || nh > A.nh;
    if (A.ne_fit && threadIdx.x == 0) A.ne_fit[0] = over ? 0 : ne;
    if (over) return;                     // over capacity: the host re-runs with read counts
  }
  events_small_body(A, cov_out, keys, diff, scratch, nh, ne);
}

// A request's whole tail in ONE workgroup (the runner's device-count fast path with its own window):
// hit CSR, events, the fp64 score, then the capacity-gated frequency record and the results
// published to pinned host memory -- the work of k_hits_small, k_events_small, k_score and
// k_publish_record, without the three kernel boundaries between them (each a dispatch plus a
// drain of the chip for a kernel that fills one CU). An over-capacity batch publishes its counters
// only (the host re-runs it).
__global__ __launch_bounds__(SB_THREADS) void k_request_tail(HitsArgs HA, EventsArgs EA, int32_t* __restrict__ cov_out,
                                                             ScoreTables T, ScoreParams S, FreqIn F,
                                                             RequestTailOut P) {
  __shared__ uint64_t keys[SB_MAX];
  __shared__ int32_t raw[SB_MAX_LINES + 1];                // the events' diff; the hits' hk before it
  static_assert(sizeof(raw) >= SB_MAX * sizeof(int64_t), "hk fits the diff array");
  __shared__ int64_t scratch[SB_THREADS / 64 + 1];
  __shared__ int s_live;
  __shared__ int64_t s_nh, s_ne;
  hits_small_body(HA, keys, reinterpret_cast<int64_t*>(raw), scratch, &s_live, &s_nh, &s_ne);
  __syncthreads();
  const int64_t nh = s_nh, ne = s_ne;
  const bool over = ne > EA.ne || nh > EA.nh;
  if (!over) {
    events_small_body(EA, cov_out, keys, raw, scratch, nh, ne);
    __syncthreads();
    // the score's factors in different waves: proximity, temporal and context are each a chain of
    // dependent table / hit-list loads, so they run side by side (waves 0-3, 4-7, 8-11) while waves
    // 12-15 load the event's own factors and multiply in score_event's order (bit-identical)
    constexpr int SC_EV = SB_THREADS / 4;                      // events per pass
    double* fx = reinterpret_cast<double*>(keys);              // [3][SC_EV] (the sorts' LDS is free)
    static_assert(sizeof(keys) >= 3 * SC_EV * sizeof(double), "score factors fit keys");
    const int part = (int)threadIdx.x / SC_EV, i = (int)threadIdx.x % SC_EV;   // part: wave-uniform
    for (int64_t b0 = 0; b0 < ne; b0 += SC_EV) {
      const int64_t e = b0 + i;
      double conf = 0.0, sev = 0.0, chrono = 0.0, pen = 0.0;
      if (e < ne) {
        const int32_t x = EA.ev_line[e], p = EA.ev_pat[e], sg = EA.ev_seg[e];
        const int32_t lo = T.seg_lo[sg], hi = T.seg_hi[sg];
        if (part == 0) {
          fx[i] = prox_factor(T, S, x, p, lo, hi);
        } else if (part == 1) {
          fx[SC_EV + i] = temp_factor(T, x, p, lo, hi, T.seg_own_lo[sg]);
        } else if (part == 2) {
          fx[2 * SC_EV + i] = ctx_factor(T, S, x, p, lo, hi);
        } else {
          conf = T.conf[p];
          sev = T.sev[p];
          chrono = chrono_factor(T.seg_g0[sg] + (x - lo), T.seg_n[sg], S);
          pen = pen_factor(S, freq_before(F, e));
        }
      }
      __syncthreads();
      if (part == 3 && e < ne)
        P.score[e] = conf * sev * chrono * fx[i] * fx[SC_EV + i] * fx[2 * SC_EV + i] * (1.0 - pen);
      __syncthreads();
    }
  }
  LP_SB_STAMP(6);
  // the frequency record of the batch's per-key counts (penalty before record: after the score),
  // gated on the matcher capacities as k_publish_record / k_freq_record
  const int64_t* cnt = P.cnt;
  const RecordGate& G = P.gate;
  const bool fits = !over && !(G.cnt && (G.cnt[0] > G.cap[0] || G.cnt[1] > G.cap[1] || G.cnt[2] > G.cap[2] ||
                                         ne > G.cap[3]));
  if (fits) {
    const FreqRing& R = P.ring;
    for (int k = threadIdx.x; k < P.K; k += SB_THREADS) {
      const int64_t c = P.counts[k];
      if (c <= 0) continue;
      const int64_t q = (int64_t)atomicAdd(reinterpret_cast<unsigned long long*>(R.ht + 1), 1ull);
      const int64_t s = q % R.cap;
      R.t[s] = P.now;
      R.key[s] = k;
      R.cnt[s] = (int32_t)c;
      R.tot[k] += c;
      R.seen[k] = 1;
    }
  }
  LP_SB_STAMP(7);
  // counters + compacted results into pinned host memory (k_publish_record's layout)
  if (threadIdx.x < 5) P.cnt_host[threadIdx.x] = threadIdx.x == 3 ? nh : threadIdx.x == 4 ? ne : cnt[threadIdx.x];
  const int64_t E = P.E;
  if (over || ne < 0 || ne > E) return;
  const uint8_t* out = P.out;
  const double* score = reinterpret_cast<const double*>(out);
  const int64_t* counts_e = reinterpret_cast<const int64_t*>(out + 8 * E);
  const int32_t* cols = reinterpret_cast<const int32_t*>(out + 8 * E + 8 * (int64_t)P.K1);
  double* h_score = reinterpret_cast<double*>(P.res_host);
  int64_t* h_counts = reinterpret_cast<int64_t*>(P.res_host + 8 * ne);
  int32_t* h_cols = reinterpret_cast<int32_t*>(P.res_host + 8 * ne + 8 * (int64_t)P.K1);
  const int64_t total = ne + P.K1 + 3 * ne;
  for (int64_t i = threadIdx.x; i < total; i += SB_THREADS) {
    if (i < ne) {
      h_score[i] = score[i];
    } else if (i < ne + P.K1) {
      h_counts[i - ne] = counts_e[i - ne];
    } else {
      const int64_t j = i - ne - P.K1;
      const int64_t c = j / ne, r = j - c * ne;
      h_cols[j] = cols[c * E + r];
    }
  }
  __syncthreads();
  LP_SB_STAMP(15);
}




void set_small_profile(uint64_t dev_ptr) {
  int64_t* p = reinterpret_cast<int64_t*>(dev_ptr);
  LP_PCHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_sb_prof), &p, sizeof(p)));
}

bool hits_small_ok(const HitsArgs& A) { return A.n > 0 && A.n <= SB_MAX; }
bool events_small_ok(const EventsArgs& A) { return A.ne <= SB_MAX && A.L <= SB_MAX_LINES; }
int64_t request_event_cap() { return SB_MAX; }
int64_t request_line_cap() { return SB_MAX_LINES; }

// coarse byte-block -> line index (blk[b] = line containing byte b << 12), one lane per block
__global__ __launch_bounds__(256) void k_blk_index(const int64_t* __restrict__ ls, int64_t L, int64_t nblk,
                                                   int32_t* __restrict__ blk) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblk) return;
  const int64_t i = upper_idx(ls, L, b << LINE_BLK_SHIFT);
  blk[b] = (int32_t)(i < 0 ? 0 : i);
}

// ---------------------------------------------------------------------------------------------
// workspace carving: the same code path sizes (base == nullptr) and carves

struct Carve {
  uint8_t* base;
  size_t used = 0;
  template <class T>
  T* take(size_t n) {
    const size_t off = (used + 255) & ~size_t(255);
    used = off + std::max<size_t>(n, 1) * sizeof(T);
    return base ? reinterpret_cast<T*>(base + off) : nullptr;
  }
  void* take_bytes(size_t n) { return take<uint8_t>(n); }
};

void request_tail_dev(const HitsArgs& HA, const EventsArgs& EA, const ScoreTables& T, const ScoreParams& S,
                      const FreqIn& F, const RequestTailOut& P, void* ws, size_t ws_bytes, uint64_t stream) {
  Carve D{static_cast<uint8_t*>(ws)};
  int32_t* cov_s = EA.cov ? EA.cov : D.take<int32_t>(EA.L);
  if (!EA.cov && (!ws || D.used > ws_bytes)) throw std::runtime_error("request_tail_dev: coverage workspace");
  hipLaunchKernelGGL(k_request_tail, dim3(1), dim3(SB_THREADS), 0, pstream(stream), HA, EA, cov_s, T, S, F, P);
  LP_PCHECK(hipGetLastError());
}

void dedupe_verify_dev(const uint64_t* keys, int64_t n, int lbits, const uint8_t* text, const int64_t* ls,
                       const int32_t* ll, const DfaPool& P, int64_t* stdk, uint8_t* flag, uint64_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_dedupe_verify, dim3(nblk(n)), dim3(256), 0, pstream(stream), keys, n, lbits, text, ls, ll, P,
                     stdk, flag);
  LP_PCHECK(hipGetLastError());
}

void feat_all_dev(int64_t L, const uint8_t* text, const int64_t* ls, const int32_t* ll, const DfaPool& P,
                  int ctx_trans, int ctx_acc, uint8_t* feat, uint64_t stream) {
  feat_cov_dev(nullptr, L, text, ls, ll, P, ctx_trans, ctx_acc, feat, stream);
}

void feat_cov_dev(const int32_t* cov, int64_t L, const uint8_t* text, const int64_t* ls, const int32_t* ll,
                  const DfaPool& P, int ctx_trans, int ctx_acc, uint8_t* feat, uint64_t stream) {
  if (L <= 0 || !feat) return;
  // lines per block: enough blocks to spread a small request over the CUs, 4096 for big ones
  int per = (int)std::min<int64_t>(FC_MAX_LINES, std::max<int64_t>(256, L / 1024));
  per = (per + 255) / 256 * 256;
  hipLaunchKernelGGL(k_feat_cov, dim3(nblk(L, per)), dim3(256), 0, pstream(stream), cov, L, per, text, ls, ll, P,
                     ctx_trans, ctx_acc, feat);
  LP_PCHECK(hipGetLastError());
}

size_t hits_dev(const HitsArgs& A, void* ws, size_t ws_bytes, uint64_t stream) {
  const int64_t n = A.n;
  if (hits_small_ok(A)) {          // a request: verify on the grid, the rest in one workgroup
    if (!A.cand_verified &&
        !cand_verify_all_dev(const_cast<int64_t*>(A.cand), A.pre_from, A.dcount, A.text, A.ls, A.ll, A.dfa, stream)) {
      hipLaunchKernelGGL(k_cand_verify, dim3(nblk(A.pre_from)), dim3(256), 0, pstream(stream), A);
      bpg_cand_dev(const_cast<int64_t*>(A.cand), A.pre_from, A.dcount, A.text, A.ls, A.ll, A.dfa, stream);
    }
    hipLaunchKernelGGL(k_hits_small, dim3(1), dim3(SB_THREADS), 0, pstream(stream), A);
    LP_PCHECK(hipGetLastError());
    return 0;
  }
  if (hits_bulk_ok(A)) return hits_bulk_dev(A, ws, ws_bytes, stream);   // bucket sorts (post_bulk.hip)
  const bool dc = A.dcount != nullptr;
  const int kbits = 2 + A.lbits + A.rbits;    // + the pad bit (dropped keys pad in both modes)
  Carve C{static_cast<uint8_t*>(ws)};
  hipStream_t st = pstream(stream);
  uint64_t* kin = C.take<uint64_t>(n);
  uint64_t* kout = C.take<uint64_t>(n);
  int64_t* stdk = C.take<int64_t>(n);
  uint8_t* flag = C.take<uint8_t>(n);
  size_t t_sort = 0, t_sel = 0, t_scan = 0;
  if (n > 0) {
    LP_PCHECK(rocprim::radix_sort_keys(nullptr, t_sort, kin, kout, (size_t)n, 0, kbits, st));
    LP_PCHECK(rocprim::select(nullptr, t_sel, stdk, flag, A.hits, A.counters, (size_t)n, st));
    LP_PCHECK(rocprim::inclusive_scan(nullptr, t_scan, A.ev_cnt, A.ev_end, (size_t)n, rocprim::plus<int64_t>(), st));
  }
  void* tmp = C.take_bytes(std::max(t_sort, std::max(t_sel, t_scan)));
  if (!ws || C.used > ws_bytes) return C.used;
  if (n == 0) {
    LP_PCHECK(hipMemsetAsync(A.counters, 0, 2 * sizeof(int64_t), st));
    LP_PCHECK(hipMemsetAsync(A.hit_off, 0, (size_t)(A.R + 1) * sizeof(int64_t), st));
    return C.used;
  }
  if (dc)
    hipLaunchKernelGGL(k_pack_dc, dim3(nblk(n)), dim3(256), 0, st, A.cand, A.pre_from, A.cand2, n - A.pre_from,
                       A.dcount, A.lbits, kin);
  else
    hipLaunchKernelGGL(k_pack, dim3(nblk(n)), dim3(256), 0, st, A.cand, n, A.pre_from, A.lbits, kin);
  LP_PCHECK(hipGetLastError());
  size_t tb = t_sort;
  LP_PCHECK(rocprim::radix_sort_keys(tmp, tb, kin, kout, (size_t)n, 0, kbits, st));
  hipLaunchKernelGGL(k_dedupe_verify, dim3(nblk(n)), dim3(256), 0, st, kout, n, A.lbits, A.text, A.ls, A.ll, A.dfa,
                     stdk, flag);
  LP_PCHECK(hipGetLastError());
  bpg_dedupe_dev(kout, n, A.lbits, A.text, A.ls, A.ll, A.dfa, flag, stream);
  tb = t_sel;
  LP_PCHECK(rocprim::select(tmp, tb, stdk, flag, A.hits, A.counters, (size_t)n, st));
  hipLaunchKernelGGL(k_csr_evcount, dim3(nblk(std::max<int64_t>(n, A.R + 1))), dim3(256), 0, st, A.hits, A.counters,
                     n, A.R, A.ev, A.hit_off, A.hit_line, A.ev_cnt);
  LP_PCHECK(hipGetLastError());
  tb = t_scan;
  LP_PCHECK(rocprim::inclusive_scan(tmp, tb, A.ev_cnt, A.ev_end, (size_t)n, rocprim::plus<int64_t>(), st));
  hipLaunchKernelGGL(k_total, dim3(1), dim3(64), 0, st, A.ev_end, n, A.counters);
  LP_PCHECK(hipGetLastError());
  return C.used;
}

size_t events_dev(const EventsArgs& A, void* ws, size_t ws_bytes, uint64_t stream) {
  const int64_t ne = A.ne, L = A.L;
  const EvTables& E = A.ev;
  const int ebits = E.pbits + A.lbits;
  const int fbits = bits_for((int64_t)E.nkeys + 1);
  Carve C{static_cast<uint8_t*>(ws)};
  hipStream_t st = pstream(stream);
  uint64_t* kin = C.take<uint64_t>(ne);
  uint64_t* kout = C.take<uint64_t>(ne);
  uint32_t* fin = C.take<uint32_t>(ne);
  uint32_t* fout = C.take<uint32_t>(ne);
  int32_t* iin = C.take<int32_t>(ne);
  int32_t* iout = C.take<int32_t>(ne);
  if (events_small_ok(A)) {        // a request: one workgroup for expand / sort / ranks / coverage
    Carve D{static_cast<uint8_t*>(ws)};
    int32_t* cov_s = A.cov ? A.cov : D.take<int32_t>(L);
    if (!A.cov && (!ws || D.used > ws_bytes)) return D.used;
    hipLaunchKernelGGL(k_events_small, dim3(1), dim3(SB_THREADS), 0, pstream(stream), A, cov_s);
    LP_PCHECK(hipGetLastError());
    if (L > 0 && A.feat && !A.feat_ready) {
      int per = (int)std::min<int64_t>(FC_MAX_LINES, std::max<int64_t>(256, L / 1024));
      per = (per + 255) / 256 * 256;
      hipLaunchKernelGGL(k_feat_cov, dim3(nblk(L, per)), dim3(256), 0, pstream(stream), cov_s, L, per, A.text, A.ls,
                         A.ll, A.dfa, A.ctx_trans, A.ctx_acc, A.feat);
      LP_PCHECK(hipGetLastError());
    }
    return D.used;
  }
  if (events_bulk_ok(A)) return events_bulk_dev(A, ws, ws_bytes, stream);   // bucket sorts (post_bulk.hip)
  int32_t* cov = A.cov ? A.cov : C.take<int32_t>(L);
  size_t t_sort = 0, t_pairs = 0;
  if (ne > 0) {
    LP_PCHECK(rocprim::radix_sort_keys(nullptr, t_sort, kin, kout, (size_t)ne, 0, ebits, st));
    LP_PCHECK(rocprim::radix_sort_pairs(nullptr, t_pairs, fin, fout, iin, iout, (size_t)ne, 0, fbits, st));
  }
  void* tmp = C.take_bytes(std::max(t_sort, t_pairs));
  if (!ws || C.used > ws_bytes) return C.used;
  if (E.nkeys > 0) LP_PCHECK(hipMemsetAsync(A.freq_counts, 0, (size_t)E.nkeys * sizeof(int64_t), st));
  if (L > 0) LP_PCHECK(hipMemsetAsync(cov, 0, (size_t)L * sizeof(int32_t), st));
  if (ne > 0) {
    hipLaunchKernelGGL(k_expand, dim3(nblk(A.nh)), dim3(256), 0, st, A.hits, A.nh, A.ev_cnt, A.ev_end, E, kin);
    LP_PCHECK(hipGetLastError());
    size_t tb = t_sort;
    LP_PCHECK(rocprim::radix_sort_keys(tmp, tb, kin, kout, (size_t)ne, 0, ebits, st));
    hipLaunchKernelGGL(k_ev_post, dim3(nblk(ne)), dim3(256), 0, st, kout, ne, E, A.ev_line, A.ev_pat, A.ev_seg, fin,
                       iin, cov);
    LP_PCHECK(hipGetLastError());
    tb = t_pairs;
    LP_PCHECK(rocprim::radix_sort_pairs(tmp, tb, fin, fout, iin, iout, (size_t)ne, 0, fbits, st));
    hipLaunchKernelGGL(k_rank, dim3(nblk(ne)), dim3(256), 0, st, fout, iout, ne, E.nkeys, A.ev_rank, A.ev_fkey,
                       A.freq_counts);
    LP_PCHECK(hipGetLastError());
  }
  if (L > 0) {
    if (A.feat) {
      // lines per block: enough blocks to spread a small request over the CUs, 4096 for big ones
      int per = (int)std::min<int64_t>(FC_MAX_LINES, std::max<int64_t>(256, L / 1024));
      per = (per + 255) / 256 * 256;
      hipLaunchKernelGGL(k_feat_cov, dim3(nblk(L, per)), dim3(256), 0, st, cov, L, per, A.text, A.ls, A.ll, A.dfa,
                         A.ctx_trans, A.ctx_acc, A.feat);
      LP_PCHECK(hipGetLastError());
    }
  }
  return C.used;
}

void blk_index_dev(const int64_t* ls, int64_t L, int64_t nblocks, int32_t* blk, uint64_t stream) {
  if (nblocks <= 0) return;
  hipLaunchKernelGGL(k_blk_index, dim3(nblk(nblocks)), dim3(256), 0, pstream(stream), ls, L, nblocks, blk);
  LP_PCHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------------------------
// host twins

void hits_host(const HitsArgs& A) {
  const int64_t n = A.n;
  std::vector<uint64_t> keys(n);
  for (int64_t i = 0; i < n; ++i) {
    const int64_t k = A.cand[i];
    keys[i] = k < 0 ? LP_PAD_KEY
                    : (((((uint64_t)k >> 32) << A.lbits) | ((uint64_t)k & 0xFFFFFFFFull)) << 1) |
                          (i >= A.pre_from ? 1ull : 0ull);
  }
  std::sort(keys.begin(), keys.end());
  std::vector<int64_t> stdk(n);
  std::vector<uint8_t> flag(n);
  host_parallel(n, 4096, [&](int, int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i)
      flag[i] = dedupe_verify_one(keys.data(), n, i, A.lbits, A.text, A.ls, A.ll, A.dfa, &stdk[i]) ? 1 : 0;
  });
  int64_t nh = 0;
  for (int64_t i = 0; i < n; ++i)
    if (flag[i]) A.hits[nh++] = stdk[i];
  A.counters[0] = nh;
  for (int r = 0; r <= A.R; ++r) A.hit_off[r] = lower_bound64(A.hits, nh, (int64_t)r << 32);
  int64_t run = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (i < nh) {
      A.hit_line[i] = (int32_t)(A.hits[i] & 0xFFFFFFFFll);
      A.ev_cnt[i] = hit_event_count(A.ev, A.hits[i]);
    } else {
      A.ev_cnt[i] = 0;
    }
    run += A.ev_cnt[i];
    A.ev_end[i] = run;
  }
  A.counters[1] = run;
}

void events_host(const EventsArgs& A) {
  const int64_t ne = A.ne, L = A.L;
  const EvTables& E = A.ev;
  std::vector<uint64_t> evk(ne);
  for (int64_t i = 0; i < A.nh; ++i) {
    const int64_t c = A.ev_cnt[i];
    if (!c) continue;
    const int64_t k = A.hits[i];
    const int r = (int)(k >> 32);
    const uint64_t x = (uint64_t)(k & 0xFFFFFFFFll);
    const int64_t base = A.ev_end[i] - c, p0 = E.prim_off[r];
    for (int64_t j = 0; j < c; ++j) evk[base + j] = (x << E.pbits) | (uint64_t)E.prim_pats[p0 + j];
  }
  std::sort(evk.begin(), evk.end());
  std::vector<uint32_t> fs(ne);
  std::vector<int32_t> idx(ne);
  std::vector<int32_t> diff(L + 1, 0);
  for (int64_t e = 0; e < ne; ++e) {
    int32_t a, b;
    fs[e] = ev_post_one(E, evk[e], e, A.ev_line, A.ev_pat, A.ev_seg, a, b);
    if (a < b) {
      ++diff[a];
      --diff[b];
    }
  }
  std::iota(idx.begin(), idx.end(), 0);
  std::stable_sort(idx.begin(), idx.end(), [&](int32_t u, int32_t v) { return fs[u] < fs[v]; });
  std::vector<uint32_t> fsorted(ne);
  for (int64_t j = 0; j < ne; ++j) fsorted[j] = fs[idx[j]];
  for (int k = 0; k < E.nkeys; ++k) A.freq_counts[k] = 0;
  for (int64_t j = 0; j < ne; ++j) rank_one(fsorted.data(), idx.data(), ne, j, E.nkeys, A.ev_rank, A.ev_fkey,
                                            A.freq_counts);
  std::vector<int32_t> covv;
  int32_t* cov = A.cov;
  if (!cov) {
    covv.resize(std::max<int64_t>(L, 1));
    cov = covv.data();
  }
  int32_t c = 0;
  for (int64_t x = 0; x < L; ++x) cov[x] = (c += diff[x]);
  if (A.feat)
    host_parallel(L, 4096, [&](int, int64_t a, int64_t b) {
      for (int64_t x = a; x < b; ++x) A.feat[x] = cov[x] > 0 ? context_feat(A.dfa, A.text + A.ls[x], A.ll[x]) : 0;
    });
}

void blk_index_host(const int64_t* ls, int64_t L, int64_t nblocks, int32_t* blk) {
  for (int64_t b = 0; b < nblocks; ++b) {
    const int64_t i = upper_idx(ls, L, b << LINE_BLK_SHIFT);
    blk[b] = (int32_t)(i < 0 ? 0 : i);
  }
}

}  // namespace lp
