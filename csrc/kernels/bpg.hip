// gfx950 kernels of the bit-parallel Glushkov programs (bpg.h, jregex.cpp bpg_program): the regexes
// whose DFA blows up or that need code-point contexts, verified on prefilter candidate lines or
// scanned over every line.
//
// Two walks of the same program:
//   * one lane per line (bpg_find_dev<W>, W <= 8 words): throughput -- the bulk path's first-of-run
//     keys and the literal-free scan of W <= 8 programs;
//   * a GROUP of G lanes per line (bpg_coop_walk<G>, any width up to 32 words = 2,048 positions):
//     latency -- request-path candidates, and every line of programs wider than 8 words.
// The DFA kernels next to them (k_cand_verify, k_dedupe_verify, k_scan) never carry the BPG walk --
// folding it into dfa_run took those kernels from ~40 to 130 VGPRs plus 580 B of scratch per lane.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <stdexcept>
#include <string>

#include "lp_api.h"
#include "lp_core.h"
#include "post_core.h"

namespace lp {

namespace {

constexpr uint64_t kPadKey = ~0ull;   // lp_post.hip LP_PAD_KEY
constexpr int kScanLines = 256;
constexpr int kLdsProgWords = 1024;   // 8 KiB (larger programs read from global memory)
// The candidate kernels stage the library's WHOLE program pool in LDS when it fits: a walk's
// per-character reads (class map, class rows, first / last sets, exceptions) are then LDS hits, not
// a chain of global-memory round trips (k_bpg_coop / k_bpg_dedupe_all are latency-bound on one
// line's walk: a request verifies a handful of candidates, a bulk step a few thousand)
constexpr uint32_t kPoolLdsWords = 8192;   // 64 KiB

inline size_t pool_lds_bytes(const DfaPool& P) {
  return (P.bpg_words && P.bpg_words <= kPoolLdsWords) ? (size_t)P.bpg_words * 8 : 0;
}

// every thread of the block calls this (it synchronises): the pool in LDS, or in global memory
__device__ __forceinline__ const uint64_t* stage_pool(const DfaPool& P, uint64_t* lds, bool staged) {
  if (!staged) return P.bpg;
  for (uint32_t i = threadIdx.x; i < P.bpg_words; i += blockDim.x) lds[i] = P.bpg[i];
  __syncthreads();
  return lds;
}

inline unsigned nblocks(int64_t n, int t = 256) { return (unsigned)std::max<int64_t>(1, (n + t - 1) / t); }

// the staged pool as an LDS pointer: the walks' reads compile to ds_read (a generic pointer that may
// be LDS or global compiles to flat loads, which wait on both the LDS and the vector-memory counters)
typedef const __attribute__((address_space(3))) uint64_t* LdsWords;
__device__ __forceinline__ LdsWords lds_words(const uint64_t* lds) { return (LdsWords)lds; }

// The lean walks of a wave's pending one-word program keys, TWO lanes per key: a line of >= 64 bytes
// (program not nullable) is split at an ASCII character pair near its middle -- the even lane walks
// the first part (only threads that start there, each followed to its end), the odd lane the second
// part from an empty state with the split point's previous kind -- so one lane's chain is about half
// a line (bpg_walk1's prevk0 / inj_end; exact: every thread starts in one part). need / r / x: this
// lane's own key (regex, line); done(src_lane, hit) runs on the even lane of the pair that walked the
// key of lane src_lane. Every lane of the wave calls this (ballots inside).
template <typename F>
__device__ __forceinline__ void bpg_walk1_pairs(bool staged, const uint64_t* pool_lds, const DfaPool& P, bool need,
                                                int r, int64_t x, const uint8_t* __restrict__ text,
                                                const int64_t* __restrict__ ls, const int32_t* __restrict__ ll,
                                                F&& done) {
  const int lane = (int)(threadIdx.x & 63);
  const int pair = lane >> 1, part = lane & 1;
  uint64_t todo = __ballot(need);
  while (todo) {                                 // wave-uniform
    int src = -1;
    uint64_t m = todo;
#pragma unroll 1
    for (int k = 0; k < 32; ++k) {               // pair k takes the k-th lowest pending slot
      const int b = m ? __builtin_ctzll(m) : -1;
      if (k == pair) src = b;
      m &= m ? m - 1 : 0ull;
    }
    todo = m;
    const int sl = src < 0 ? lane : src;
    const int rr = __shfl(r, sl, 64);
    const long long xx = __shfl((long long)x, sl, 64);
    const bool valid = src >= 0;
    const int off = valid ? P.meta[4 * rr] : 0;
    const uint8_t* s = text + (valid ? ls[xx] : 0);
    const int len = valid ? ll[xx] : 0;
    const uint64_t h0 = valid ? (staged ? pool_lds[off] : P.bpg[off]) : 0ull;
    int mid = -1;
    if (valid && len >= 64 && ((h0 >> 32) & 0xFFFFFFu) == 0u) {
      // the split point: the first t in [len/2, len/2 + 16) with s[t-1] and s[t] ASCII (a 32-byte
      // aligned window around it; texts are padded)
      const uint8_t* w = reinterpret_cast<const uint8_t*>((uintptr_t)(s + len / 2 - 1) & ~(uintptr_t)15);
      const uint4 c0 = reinterpret_cast<const uint4*>(w)[0], c1 = reinterpret_cast<const uint4*>(w)[1];
      const int j0 = (int)((s + len / 2) - w);   // window index of t = len / 2 (1..16)
#pragma unroll 1
      for (int q = 0; q < 16 && mid < 0; ++q) {
        const int t = len / 2 + q;
        if (t >= len - 4 || j0 + q >= 32) break;
        if (win_byte(c0, c1, j0 + q - 1) < 0x80 && win_byte(c0, c1, j0 + q) < 0x80) mid = t;
      }
    }
    const bool split = mid > 0;
    const bool v = valid && (part == 0 || split);
    const uint8_t* ws = (part == 1 && split) ? s + mid : s;
    const int wn = part == 0 ? len : (split ? len - mid : 0);
    const int wpk = (part == 1 && split) ? prev_of(ascii_kind(s[mid - 1])) : 0;
    const int wend = (part == 0 && split) ? mid : 0x7FFFFFFF;
    const bool hit = staged ? bpg_walk1(lds_words(pool_lds) + off, ws, wn, v, wpk, wend)
                            : bpg_walk1(P.bpg + off, ws, wn, v, wpk, wend);
    const bool other = __shfl_xor(hit ? 1 : 0, 1, 64) != 0;
    if (valid && part == 0) done(src, hit || other);
  }
}

// WMAX: the library's widest program of <= 8 words -- only walks up to that width are compiled
// into the kernel, so a library of one-word programs (the common case since counted positions)
// runs at a one-word walk's register count (a W = 8 walk's 256 VGPRs allowed one wave per SIMD)
template <int WMAX>
__device__ __forceinline__ bool lane_walk(const uint64_t* prog, const uint8_t* s, int len) {
  const int w = (int)(prog[0] & 0xFF);
  if constexpr (WMAX == 1) return bpg_find_dev<1>(prog, s, len);
  if (w <= 1) return bpg_find_dev<1>(prog, s, len);
  if constexpr (WMAX == 2) return bpg_find_dev<2>(prog, s, len);
  if (w == 2) return bpg_find_dev<2>(prog, s, len);
  if constexpr (WMAX <= 4) {
    if (w == 3) return bpg_find_dev<3>(prog, s, len);
    return bpg_find_dev<4>(prog, s, len);
  } else {
    if (w == 3) return bpg_find_dev<3>(prog, s, len);
    if (w == 4) return bpg_find_dev<4>(prog, s, len);
    if (w <= 6) return bpg_find_dev<6>(prog, s, len);
    return bpg_find_dev<8>(prog, s, len);
  }
}

inline int narrow_wmax(uint32_t widths) {       // WMAX of lane_walk for a bpg_widths mask
  if (widths & 0x1E0u) return 8;                 // 5 .. 8 words
  if (widths & 0x18u) return 4;                  // 3 / 4 words
  if (widths & 0x4u) return 2;
  return 1;
}

// bulk path: sorted packed keys ((regex << lbits | line) << 1 | pre-verified); the first key of
// every run whose regex is a program of <= 8 words and that no engine pre-verified gets its flag
// here (k_dedupe_verify left it 0). Every width in one kernel (registers of the widest walk: fine
// for a few waves). Keys of wider programs are appended to `wlist` (count in `wcnt`, zeroed by the
// caller) for k_bpg_coop_list: a regex's keys are contiguous in the sorted array,
// so walking them where they sit would serialise up to 64 / (64 / G) walks in one wave (a W = 12
// program's keys cost 1.17 ms per bench step that way).
template <int WMAX>
__global__ __launch_bounds__(256) void k_bpg_dedupe_all(const uint64_t* __restrict__ keys, int64_t n, int lbits,
                                                        const uint8_t* __restrict__ text,
                                                        const int64_t* __restrict__ ls,
                                                        const int32_t* __restrict__ ll, DfaPool P,
                                                        uint8_t* __restrict__ flag, uint32_t* __restrict__ wcnt,
                                                        uint32_t* __restrict__ wlist, int64_t* __restrict__ std_key) {
  extern __shared__ uint64_t pool_lds[];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (std_key && i < n) {                       // fused k_dedupe_verify: the DFA keys' walks run beside
    int64_t sk = 0;                             // the BPG walks (one launch: the two tails overlap)
    flag[i] = dedupe_verify_one(keys, n, i, lbits, text, ls, ll, P, &sk) ? 1 : 0;
    std_key[i] = sk;
  }
  bool walk = false;
  int r = 0;
  int64_t x = 0;
  if (i < n) {
    const uint64_t key = keys[i];
    const uint64_t k = key >> 1;
    if (key != kPadKey && !(i > 0 && (keys[i - 1] >> 1) == k)) {
      r = (int)(k >> lbits);
      if (is_bpg(P, r)) {
        const bool is_wide = (int)(P.bpg[P.meta[4 * r]] & 0xFF) > BPG_LANE_MAX_W;
        bool pre = false;
        for (int64_t j = i; j < n && (keys[j] >> 1) == k; ++j) pre |= (keys[j] & 1) != 0;
        if (!pre && !(is_wide && !wcnt)) {   // pre-verified: flag already 1
          if (is_wide) {
            wlist[atomicAdd(wcnt, 1u)] = (uint32_t)i;
          } else {
            walk = true;
            x = (int64_t)(k & ((1ull << lbits) - 1));
          }
        }
      }
    }
  }
  if (!__syncthreads_or(walk)) return;          // block-uniform: most blocks hold no program key
  const bool staged = P.bpg_words != 0;
  const uint64_t* pool = stage_pool(P, pool_lds, staged);
  if constexpr (WMAX == 1) {                    // one-word programs: the lean walk, every lane in
    // (one lane per key: the bulk path's keys are dense, so two lanes per key -- bpg_walk1_pairs --
    // measured slower here: device step 2.81 -> 2.86 ms, config 2 0.51 -> 0.57 ms)
    if (__ballot(walk) == 0) return;
    const int off = walk ? P.meta[4 * r] : 0;
    const uint8_t* s = text + (walk ? ls[x] : 0);
    const int len = walk ? ll[x] : 0;
    const bool hit = staged ? bpg_walk1(lds_words(pool_lds) + off, s, len, walk) : bpg_walk1(P.bpg + off, s, len, walk);
    if (walk) flag[i] = hit ? 1 : 0;
  } else {
    if (walk) flag[i] = lane_walk<WMAX>(pool + P.meta[4 * r], text + ls[x], ll[x]) ? 1 : 0;
  }
}

// Request path for libraries of one-word programs (bpg_widths == 1 << 1, the common case): the lean
// walk (bpg_walk1) over the pool staged in LDS, two lanes per BPG candidate that split a long line
// (bpg_walk1_pairs: a request's candidates are sparse, so the lanes are free and one walk's chain
// halves) -- the cooperative walk cost ~340 ns per byte at one word (profiles/r5_c) -- and, MODE 2,
// the DFA candidates in the grid's upper half (k_bpg_coop's layout).
template <int MODE>
__global__ __launch_bounds__(256) void k_bpg_cand1(int64_t* __restrict__ cand, int64_t cap,
                                                   const unsigned long long* __restrict__ dcount,
                                                   const uint8_t* __restrict__ text, const int64_t* __restrict__ ls,
                                                   const int32_t* __restrict__ ll, DfaPool P) {
  const int64_t n = dcount ? (int64_t)min((unsigned long long)cap, dcount[0]) : cap;
  if (MODE == 2 && blockIdx.x >= (gridDim.x >> 1)) {
    const int64_t jj = (int64_t)(blockIdx.x - (gridDim.x >> 1)) * blockDim.x + threadIdx.x;
    if (jj >= n) return;
    const int64_t k = cand[jj];
    if (k < 0) return;
    const int r = (int)(k >> 32);
    if (is_bpg(P, r)) return;
    const int64_t x = k & 0xFFFFFFFFll;
    if (!dfa_run(P, r, text + ls[x], ll[x])) cand[jj] = -1;
    return;
  }
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int r = 0;
  int64_t x = 0;
  bool need = false;
  if (i < n) {
    const int64_t k = cand[i];
    if (k >= 0) {
      r = (int)(k >> 32);
      x = k & 0xFFFFFFFFll;
      need = is_bpg(P, r);
    }
  }
  extern __shared__ uint64_t pool_lds[];
  if (!__syncthreads_or(need)) return;          // block-uniform (the DFA half returned above)
  const bool staged = P.bpg_words != 0;
  stage_pool(P, pool_lds, staged);
  if (__ballot(need) == 0) return;              // wave-uniform
  const int64_t base = i - (int64_t)(threadIdx.x & 63);
  bpg_walk1_pairs(staged, pool_lds, P, need, r, x, text, ls, ll, [&](int src, bool hit) {
    if (!hit) cand[base + src] = -1;
  });
}

// ---------------------------------------------------------------------------------------------
// Wave-cooperative walk (candidate verification: few lines, so the latency of ONE line's walk
// decides; and programs too wide for one lane's registers).
//
// The one-lane walk is a serial chain of ~40 dependent VALU ops per 64-bit word per character
// (~240 for a 6-word program: 75 us for one 10k-line request's candidates, profiles/r3_h). Here a
// line is walked by a GROUP of G lanes (G = power of two >= 2W), lane j holding 32-bit word j of
// every mask, so a character costs ~20 ops on the chain whatever the width:
//   * shift edges: the carry of word j-1 arrives by DPP row_shr:1 when groups fit in a 16-lane row
//     (G <= 16), else from a ballot of the words' top bits;
//   * spread fields: the multi-word subtraction's borrow chain is a carry-lookahead on two ballots --
//     generate g = df < lo, propagate p = df == lo; the borrow INTO lane i is bit i of
//     (X + G) ^ X ^ G with X = G | P (a 64-bit scalar add resolves every group's chain at once;
//     each group's top lane is masked out of G and P, so no borrow crosses into the next group);
//   * exceptions: the source bit's owner lane votes (ballot), every lane of the group reads it;
//   * class / first / last words for 16 bytes are loaded before the 16 serial updates (they depend
//     on the text only), so no load latency sits on the state chain; UTF-8 continuation bytes keep
//     the state (a select), lead bytes are decoded from the 32-byte window of this block and the next.
// A wave takes 64 candidate slots, compacts the ones that need a BPG walk (ballot) and walks them
// 64 / G at a time.

__device__ __forceinline__ uint64_t coop_chain_mask(int G) {   // every lane but each group's top lane
  uint64_t top = 0;
  for (int b = G - 1; b < 64; b += G) top |= 1ull << b;
  return ~top;
}

template <int G>
__device__ __forceinline__ bool bpg_coop_walk(const uint64_t* __restrict__ P, const uint8_t* __restrict__ s, int n,
                                              bool valid) {
  const int lane = (int)(threadIdx.x & 63);
  const int j = lane & (G - 1);
  const int gb = lane & ~(G - 1);
  const uint64_t gm = (G >= 64 ? ~0ull : ((1ull << G) - 1ull)) << gb;
  const uint64_t chain = coop_chain_mask(G);
  BpgLayout L = bpg_layout(P);
  if (!valid) { L.W = 0; L.E = 0; L.uniform = true; L.nullm = 0; L.nctr = 0; }
  const int W = L.W;
  const int E = L.E;
  const bool uniform = L.uniform;
  const uint32_t nullm = L.nullm;
  const bool wl = valid && j < 2 * W;           // this lane holds a program word
  const uint32_t* p32 = reinterpret_cast<const uint32_t*>(P);
  // uint32 index of word j of the 64-bit mask at uint64 offset o
#define LP_W32(o) (p32[2 * (o) + j])
  // word j of every structural mask; lanes past the program (and invalid groups) hold zeros, so
  // their state stays empty. The last position never has a shift edge (no position above), so no
  // shift carry leaves a group.
  const uint32_t shm = wl ? LP_W32(2) : 0u, selfm = wl ? LP_W32(2 + W) : 0u, src = wl ? LP_W32(2 + 2 * W) : 0u;
  const uint32_t R = wl ? LP_W32(2 + 3 * W) : 0u, lo = wl ? LP_W32(2 + 4 * W) : 0u, hi = wl ? LP_W32(2 + 5 * W) : 0u;
  const int first_o = L.o_first, last_o = L.o_last, cls_o = L.o_cls, exc_o = L.o_exc;
  const uint32_t f0 = wl ? LP_W32(first_o) : 0u, l0 = wl ? LP_W32(last_o) : 0u;
  const int ftl = valid ? final_term_len(s, n) : 0;
  const int ft = ftl ? n - ftl : -1;
  // counted positions: the lane holding the position's word keeps its count (bpg.h). A lane's own
  // counters are compacted to the front (ncl of them, bits cmask of its word): the per-character
  // update runs only while some counted position of the wave is alive or entered -- a dead
  // position's count is never read (it restarts at 1 on entry), so skipping it changes nothing
  const int nctr = L.nctr;
  uint32_t cpos[BPG_CTR_MAX], cbound[BPG_CTR_MAX], cnt[BPG_CTR_MAX];
  int ncl = 0;
  uint32_t cmask = 0;
#pragma unroll
  for (int c = 0; c < BPG_CTR_MAX; ++c) {
    cpos[c] = 0;
    cbound[c] = 0;
    cnt[c] = 0;
  }
#pragma unroll
  for (int c = 0; c < BPG_CTR_MAX; ++c) {
    const uint64_t e = c < nctr ? P[L.o_ctr + c] : 0ull;
    const bool own = c < nctr && j == (int)((e & 0xFFFF) >> 5);
#pragma unroll
    for (int q = 0; q < BPG_CTR_MAX; ++q)
      if (own && q == ncl) {
        cpos[q] = (uint32_t)(e & 31);
        cbound[q] = (uint32_t)(e >> 16);
      }
    cmask |= own ? 1u << (e & 31) : 0u;
    ncl += own ? 1 : 0;
  }
  const bool wctr = __ballot(nctr > 0) != 0;
  // the first BPG_EXC_REG exceptions' headers and this lane's target words, in registers (a load of
  // each per character sat on the state chain)
  uint64_t eh[BPG_EXC_REG];
  uint32_t etw[BPG_EXC_REG];
#pragma unroll
  for (int e = 0; e < BPG_EXC_REG; ++e) {
    eh[e] = e < E ? P[exc_o + e * (W + 1)] : 0ull;
    etw[e] = (e < E && wl) ? LP_W32(exc_o + e * (W + 1) + 1) : 0u;
  }
  // wave-uniform feature switches: the common program (uniform first/last sets, no exception edges,
  // not nullable, line without a final terminator) walks only the shift / self / spread chain
  const bool wnon = __ballot(valid && !uniform) != 0;
  const bool wexc = __ballot(valid && E > 0) != 0;
  const bool wctx = wnon || wexc || __ballot(valid && nullm != 0) != 0;
  const bool wft = __ballot(ftl > 0) != 0;
  const int sh = valid ? (int)((uintptr_t)s & 15) : 0;
  const uint4* blk = reinterpret_cast<const uint4*>(s - sh);
  int T = valid ? n + sh : 0;                    // position of this group's end of line (pos = t + sh)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) T = max(T, __shfl_xor(T, o, 64));
  uint32_t S = 0, acc = 0, Sft = 0;
  int ftctx = 0;
  bool nullhit = false;
  int prevk = 0;                                 // P_BOS
  for (int b0 = 0; b0 <= T; b0 += 16) {          // wave-uniform
    const bool inl = valid && b0 < sh + n;
    const uint4 cur = inl ? blk[b0 >> 4] : make_uint4(0, 0, 0, 0);
    const uint4 nxt = (inl && b0 + 16 < sh + n) ? blk[(b0 >> 4) + 1] : make_uint4(0, 0, 0, 0);
    // text-only operands of the 16 bytes, off the state chain: class words (0 outside [0, n): the
    // state is empty before the line and dies after its end), skip flags of UTF-8 continuation
    // bytes, boundary contexts, first / last words
    uint32_t cw[16], fw[16], lw[16];
    int ctxq[16];
    uint32_t skipm = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int t = b0 + q - sh;
      const bool lv = valid && t >= 0 && t < n;
      int nk = 0, k = 0;
      if (lv) k = bpg_char_win(P, L, cur, nxt, q, t, n, &nk);
      const bool skip = lv && k < 0;
      skipm |= skip ? 1u << q : 0u;
      cw[q] = (wl && lv && !skip) ? LP_W32(cls_o + k * W) : 0u;
      ctxq[q] = prevk * 6 + nk;                  // N_EOS from the end of line on
      if (wctx && !skip) {
        if (wft && t == ft) ftctx = prevk * 6 + 1;
        nullhit |= valid && t >= 0 && t <= n && ((nullm >> ctxq[q]) & 1u);
      }
      if (lv && !skip) prevk = prev_of(nk);
    }
    if (wnon) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        fw[q] = uniform ? f0 : (wl ? LP_W32(first_o + ctxq[q] * W) : 0u);
        lw[q] = uniform ? l0 : (wl ? LP_W32(last_o + ctxq[q] * W) : 0u);
      }
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const bool skip = (skipm >> q) & 1u;
      // accept before this character (the state after the last one is checked at t = n; later
      // positions see the empty state)
      acc |= skip ? 0u : (S & (wnon ? lw[q] : l0));
      if (wft) Sft = (b0 + q - sh == ft) ? S : Sft;
      // shift edges with the carry out of word j-1, self loops
      const uint32_t x = S & shm;
      uint32_t y;
      if (G <= 16) {
        y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(x >> 31), 0x111 /* row_shr:1 */, 0xF, 0xF, true);
      } else {
        const uint64_t cm = __ballot((x >> 31) != 0u);
        y = (uint32_t)(((cm << 1) >> lane) & 1ull);
      }
      uint32_t F = (x << 1) | y | (S & selfm);
      // spread fields: d = df - lo over the group; borrow INTO lane i = bit i of (X + G) ^ X ^ G
      const uint32_t df = (S & src) | hi;
      const uint64_t Gm = __ballot(df < lo) & chain;
      const uint64_t Pm = __ballot(df == lo) & chain;
      const uint64_t X = Gm | Pm;
      const uint64_t Cm = (X + Gm) ^ X ^ Gm;
      const uint32_t d = df - lo - (uint32_t)((Cm >> lane) & 1ull);
      F |= R & ~(d ^ df);
      if (wexc) {                                // exception edges: the source word's lane votes
        const int ctx = ctxq[q];
#pragma unroll
        for (int e = 0; e < BPG_EXC_REG; ++e) {  // headers / target words in registers
          const uint64_t h = eh[e];
          const int p = (int)(h & 0xFFFF);
          const uint64_t M = __ballot(e < E && j == (p >> 5) && ((S >> (p & 31)) & 1u));
          if (e < E && ((M >> (gb + (p >> 5))) & 1ull) && ((((uint32_t)(h >> 16) & 0xFFFFFFu) >> ctx) & 1u))
            F |= etw[e];
        }
        for (int e = BPG_EXC_REG; e < E; ++e) {  // E varies across groups: lanes past their E idle
          const uint64_t h = P[exc_o + e * (W + 1)];
          const uint32_t tw = wl ? LP_W32(exc_o + e * (W + 1) + 1) : 0u;
          const int p = (int)(h & 0xFFFF);
          const uint64_t M = __ballot(j == (p >> 5) && ((S >> (p & 31)) & 1u));
          if (((M >> (gb + (p >> 5))) & 1ull) && ((((uint32_t)(h >> 16) & 0xFFFFFFu) >> ctx) & 1u)) F |= tw;
        }
      }
      F |= wnon ? fw[q] : f0;
      if (wctr && __ballot(((F | S) & cmask) != 0u) != 0) {   // (bpg_ctr_step, one counter at a time)
#pragma unroll
        for (int c = 0; c < BPG_CTR_MAX; ++c) {
          if (__ballot(c < ncl) == 0) break;
          if (c < ncl) {
            const uint32_t b = cpos[c];
            const uint32_t entry = (F >> b) & 1u;
            const uint32_t lt = cnt[c] < cbound[c] ? 1u : 0u;
            F |= (((S >> b) & 1u) & lt) << b;    // stay while the count is below the bound
            const uint32_t k = entry ? 1u : cnt[c] + lt;   // saturates at the bound
            cnt[c] = skip ? cnt[c] : k;
          }
        }
      }
      const uint32_t Sn = F & cw[q];
      S = skip ? S : Sn;
    }
    // a group is finished once it accepted or its line ended; the wave stops when all are
    const uint64_t hitm = __ballot(acc != 0 || nullhit);
    const bool fin = !valid || (hitm & gm) != 0 || b0 + 16 > sh + n;
    if (__ballot(!fin) == 0) break;
  }
  if (wft && ft >= 0) acc |= Sft & (uniform ? l0 : (wl ? LP_W32(last_o + ftctx * W) : 0u));
#undef LP_W32
  return (__ballot(acc != 0 || nullhit) & gm) != 0;
}

// mode 0: cand[i] = -1 for BPG candidates that do not match (request path, k_cand_verify did the
// DFA ones); mode 2: the same, with the DFA candidates verified by the grid's upper half; mode 1:
// flag the first key of every sorted run whose regex is a program of >= wmin words that no engine
// pre-verified (bulk path, k_dedupe_verify left the flag 0)
template <int G, int MODE>
__global__ __launch_bounds__(256) void k_bpg_coop(int64_t* __restrict__ cand, const uint64_t* __restrict__ keys,
                                                  int64_t cap, const unsigned long long* __restrict__ dcount, int lbits,
                                                  const uint8_t* __restrict__ text, const int64_t* __restrict__ ls,
                                                  const int32_t* __restrict__ ll, DfaPool P,
                                                  uint8_t* __restrict__ flag, int wmin) {
  const int lane = (int)(threadIdx.x & 63);
  const int64_t n = (MODE != 1 && dcount) ? (int64_t)min((unsigned long long)cap, dcount[0]) : cap;
  if (MODE == 2 && blockIdx.x >= (gridDim.x >> 1)) {
    // the grid's upper half: DFA candidates, one lane each (k_cand_verify's work), side by side
    // with the BPG walks of the lower half -- one launch, and a request's critical path is the
    // longer of the two instead of their sum
    const int64_t jj = (int64_t)(blockIdx.x - (gridDim.x >> 1)) * blockDim.x + threadIdx.x;
    if (jj >= n) return;
    const int64_t k = cand[jj];
    if (k < 0) return;
    const int r = (int)(k >> 32);
    if (is_bpg(P, r)) return;
    const int64_t x = k & 0xFFFFFFFFll;
    if (!dfa_run(P, r, text + ls[x], ll[x])) cand[jj] = -1;
    return;
  }
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int r = 0;
  int64_t x = 0;
  bool need = false;
  if (i < n) {
    if (MODE != 1) {
      const int64_t k = cand[i];
      if (k >= 0) {
        r = (int)(k >> 32);
        x = k & 0xFFFFFFFFll;
        need = is_bpg(P, r);
      }
    } else {
      const uint64_t key = keys[i];
      const uint64_t k = key >> 1;
      if (key != kPadKey && !(i > 0 && (keys[i - 1] >> 1) == k)) {
        r = (int)(k >> lbits);
        x = (int64_t)(k & ((1ull << lbits) - 1));
        need = is_bpg(P, r) && (int)(P.bpg[P.meta[4 * r]] & 0xFF) >= wmin;
        for (int64_t q = i; need && q < n && (keys[q] >> 1) == k; ++q)
          if (keys[q] & 1) need = false;         // pre-verified: flag already 1
      }
    }
  }
  extern __shared__ uint64_t pool_lds[];
  if (!__syncthreads_or(need)) return;          // block-uniform (the DFA half returned above)
  const uint64_t* pool = stage_pool(P, pool_lds, P.bpg_words != 0);
  uint64_t todo = __ballot(need);                // wave-uniform
  constexpr int NG = 64 / G;
  const int g = lane / G;
  while (todo) {
    // group g takes the g-th lowest pending slot of the wave
    int src = -1;
    uint64_t m = todo;
#pragma unroll
    for (int k = 0; k < NG; ++k) {
      const int b = m ? __builtin_ctzll(m) : -1;
      if (k == g) src = b;
      m &= m ? m - 1 : 0ull;
    }
    todo = m;
    const int sl = src < 0 ? lane : src;
    const int rr = __shfl(r, sl, 64);
    const int64_t xx = __shfl(x, sl, 64);
    const bool valid = src >= 0;
    const uint64_t* prog = pool + (valid ? P.meta[4 * rr] : 0);
    const uint8_t* s = text + (valid ? ls[xx] : 0);
    const int len = valid ? ll[xx] : 0;
    const bool hit = bpg_coop_walk<G>(prog, s, len, valid);
    if (valid && (lane & (G - 1)) == 0) {
      const int64_t slot = (i - lane) + src;
      if (MODE != 1) {
        if (!hit) cand[slot] = -1;
      } else {
        flag[slot] = hit ? 1 : 0;
      }
    }
  }
}

// the listed keys of wide programs (k_bpg_dedupe_all): one group of G lanes per key, the groups
// of a fixed grid striding over the list (the walks' collectives need whole waves: a wave leaves
// the loop together, idle groups walk as invalid)
template <int G>
__global__ __launch_bounds__(256) void k_bpg_coop_list(const uint64_t* __restrict__ keys, int lbits,
                                                       const uint32_t* __restrict__ wcnt,
                                                       const uint32_t* __restrict__ wlist,
                                                       const uint8_t* __restrict__ text,
                                                       const int64_t* __restrict__ ls,
                                                       const int32_t* __restrict__ ll, DfaPool P,
                                                       uint8_t* __restrict__ flag) {
  const uint32_t cnt = *wcnt;
  const int lane = (int)(threadIdx.x & 63);
  const int64_t gid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
  const int64_t ngroups = (int64_t)gridDim.x * blockDim.x / G;
  for (int64_t j = gid;; j += ngroups) {
    const bool valid = j < (int64_t)cnt;
    if (!__ballot(valid)) break;
    int64_t i = 0, x = 0;
    int r = 0;
    if (valid) {
      i = wlist[j];
      const uint64_t k = keys[i] >> 1;
      r = (int)(k >> lbits);
      x = (int64_t)(k & ((1ull << lbits) - 1));
    }
    const uint64_t* prog = P.bpg + (valid ? P.meta[4 * r] : 0);
    const bool hit = bpg_coop_walk<G>(prog, text + (valid ? ls[x] : 0), valid ? ll[x] : 0, valid);
    if (valid && (lane & (G - 1)) == 0) flag[i] = hit ? 1 : 0;
  }
}

int coop_group(uint32_t widths) {                // lanes per line: power of two >= 2 x the widest program
  int w = 0;
  for (int b = 31; b >= 0; --b)
    if (widths & (1u << b)) { w = b; break; }
  if (widths & 0x80000000u) w = 32;              // bit 31 stands for 32 words (bpg_widths)
  int g = 2;
  while (g < 2 * w) g <<= 1;
  return g;
}

template <int MODE>
void launch_coop(int64_t* cand, const uint64_t* keys, int64_t cap, const unsigned long long* dcount, int lbits,
                 const uint8_t* text, const int64_t* ls, const int32_t* ll, const DfaPool& P, uint8_t* flag,
                 hipStream_t st, int wmin) {
  const dim3 grid(nblocks(cap) * (MODE == 2 ? 2 : 1)), block(256);
  const size_t lds = pool_lds_bytes(P);
  DfaPool Q = P;
  if (!lds) Q.bpg_words = 0;                     // the kernels stage the pool iff bpg_words != 0
  if (MODE != 1 && P.bpg_widths == (1u << 1)) {
    if (MODE == 2) hipLaunchKernelGGL((k_bpg_cand1<2>), grid, block, lds, st, cand, cap, dcount, text, ls, ll, Q);
    else hipLaunchKernelGGL((k_bpg_cand1<0>), grid, block, lds, st, cand, cap, dcount, text, ls, ll, Q);
    return;
  }
  switch (coop_group(P.bpg_widths)) {
    case 2: hipLaunchKernelGGL((k_bpg_coop<2, MODE>), grid, block, lds, st, cand, keys, cap, dcount, lbits, text, ls, ll, Q, flag, wmin); break;
    case 4: hipLaunchKernelGGL((k_bpg_coop<4, MODE>), grid, block, lds, st, cand, keys, cap, dcount, lbits, text, ls, ll, Q, flag, wmin); break;
    case 8: hipLaunchKernelGGL((k_bpg_coop<8, MODE>), grid, block, lds, st, cand, keys, cap, dcount, lbits, text, ls, ll, Q, flag, wmin); break;
    case 16: hipLaunchKernelGGL((k_bpg_coop<16, MODE>), grid, block, lds, st, cand, keys, cap, dcount, lbits, text, ls, ll, Q, flag, wmin); break;
    case 32: hipLaunchKernelGGL((k_bpg_coop<32, MODE>), grid, block, lds, st, cand, keys, cap, dcount, lbits, text, ls, ll, Q, flag, wmin); break;
    default: hipLaunchKernelGGL((k_bpg_coop<64, MODE>), grid, block, lds, st, cand, keys, cap, dcount, lbits, text, ls, ll, Q, flag, wmin); break;
  }
}

// literal-free programs of <= 8 words over every line: blockIdx.y = regex slot (block-uniform),
// the program is staged in LDS so class / first / last / exception reads are LDS hits
template <int W>
__global__ __launch_bounds__(kScanLines) void k_bpg_scan(const uint8_t* __restrict__ text,
                                                         const int64_t* __restrict__ ls,
                                                         const int32_t* __restrict__ ll, int64_t L,
                                                         const int32_t* __restrict__ regs, DfaPool P,
                                                         int64_t* out, int64_t cap, unsigned long long* count) {
  __shared__ uint64_t sp[kLdsProgWords];
  const int r = regs[blockIdx.y];
  if (!is_bpg(P, r)) return;                  // block-uniform
  const uint64_t* prog = P.bpg + P.meta[4 * r];
  if ((int)(prog[0] & 0xFF) != W) return;
  const int nw = bpg_words(prog);
  const int64_t line = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool m = false;
  if (nw <= kLdsProgWords) {
    for (int i = threadIdx.x; i < nw; i += blockDim.x) sp[i] = prog[i];
    __syncthreads();
    if constexpr (W == 1) {
      const bool v = line < L;
      m = bpg_walk1(lds_words(sp), text + (v ? ls[line] : 0), v ? ll[line] : 0, v);
    } else if (line < L) {
      m = bpg_find_dev<W>(sp, text + ls[line], ll[line]);
    }
  } else if (line < L) {
    m = bpg_find_dev<W>(prog, text + ls[line], ll[line]);
  }
  if (m) {
    const unsigned long long i = atomicAdd(count, 1ull);
    if ((int64_t)i < cap) out[i] = ((int64_t)r << 32) | line;
  }
}

// literal-free programs wider than 8 words over every line: a group of G lanes per line
template <int G>
__global__ __launch_bounds__(256) void k_bpg_scan_coop(const uint8_t* __restrict__ text,
                                                       const int64_t* __restrict__ ls,
                                                       const int32_t* __restrict__ ll, int64_t L,
                                                       const int32_t* __restrict__ regs, DfaPool P,
                                                       int64_t* out, int64_t cap, unsigned long long* count) {
  const int r = regs[blockIdx.y];
  if (!is_bpg(P, r)) return;                  // block-uniform
  const uint64_t* prog = P.bpg + P.meta[4 * r];
  if ((int)(prog[0] & 0xFF) <= BPG_LANE_MAX_W) return;
  constexpr int NG = 64 / G;
  const int lane = (int)(threadIdx.x & 63);
  const int64_t line = ((int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)) * NG + lane / G;
  const bool valid = line < L;
  const bool hit = bpg_coop_walk<G>(prog, text + (valid ? ls[line] : 0), valid ? ll[line] : 0, valid);
  if (valid && hit && (lane & (G - 1)) == 0) {
    const unsigned long long i = atomicAdd(count, 1ull);
    if ((int64_t)i < cap) out[i] = ((int64_t)r << 32) | line;
  }
}

void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e) + " in " + what);
}

template <typename F>
void for_widths(uint32_t mask, F&& f) {
  if (mask & (1u << 1)) f(std::integral_constant<int, 1>{});
  if (mask & (1u << 2)) f(std::integral_constant<int, 2>{});
  if (mask & (1u << 3)) f(std::integral_constant<int, 3>{});
  if (mask & (1u << 4)) f(std::integral_constant<int, 4>{});
  if (mask & (1u << 6)) f(std::integral_constant<int, 6>{});
  if (mask & (1u << 8)) f(std::integral_constant<int, 8>{});
}

constexpr uint32_t kWideMask = ~0x1FFu;        // bpg_widths bits of programs wider than 8 words

}  // namespace

void bpg_cand_dev(int64_t* cand, int64_t cap, const unsigned long long* dcount, const uint8_t* text, const int64_t* ls,
                  const int32_t* ll, const DfaPool& P, uint64_t stream) {
  if (!P.bpg_widths || cap <= 0) return;
  launch_coop<0>(cand, nullptr, cap, dcount, 0, text, ls, ll, P, nullptr, reinterpret_cast<hipStream_t>(stream), 0);
  check_launch("k_bpg_coop<cand>");
}

namespace {
bool g_cand_split = false;
}  // namespace
void set_cand_verify_split(bool on) { g_cand_split = on; }

bool cand_verify_all_dev(int64_t* cand, int64_t cap, const unsigned long long* dcount, const uint8_t* text,
                         const int64_t* ls, const int32_t* ll, const DfaPool& P, uint64_t stream) {
  if (!P.bpg_widths || cap <= 0 || g_cand_split) return false;   // caller runs k_cand_verify
  launch_coop<2>(cand, nullptr, cap, dcount, 0, text, ls, ll, P, nullptr, reinterpret_cast<hipStream_t>(stream), 0);
  check_launch("k_bpg_coop<cand+dfa>");
  return true;
}

bool bpg_dedupe_dev(const uint64_t* keys, int64_t n, int lbits, const uint8_t* text, const int64_t* ls,
                    const int32_t* ll, const DfaPool& P, uint8_t* flag, uint64_t stream, uint32_t* wcnt,
                    uint32_t* wlist, int64_t* std_key) {
  if (!P.bpg_widths || n <= 0) return false;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const bool any_wide = (P.bpg_widths & kWideMask) != 0;
  // programs of <= 8 words: ONE launch for every width, a lane per key (a step's BPG candidates are
  // few -- hundreds to thousands, a handful of waves -- and each walk is a serial chain, so
  // per-width launches added up their slowest walks where one launch runs them side by side)
  const bool listed = any_wide && wcnt && wlist;
  const bool fused = (P.bpg_widths & 0x1FFu) || listed;
  if (std_key && !fused) {                      // only in-place wide walks: the DFA verify goes first
    dedupe_verify_dev(keys, n, lbits, text, ls, ll, P, std_key, flag, stream);
    std_key = nullptr;
  }
  if (fused) {
    DfaPool Q = P;
    if (!pool_lds_bytes(P)) Q.bpg_words = 0;     // the kernel stages the pool iff bpg_words != 0
#define LP_DEDUPE(WM)                                                                                      \
  hipLaunchKernelGGL(k_bpg_dedupe_all<WM>, dim3(nblocks(n)), dim3(256), pool_lds_bytes(P), st, keys, n, lbits, text, ls, \
                     ll, Q, flag, \
                     listed ? wcnt : nullptr, listed ? wlist : nullptr, std_key)
    switch (narrow_wmax(P.bpg_widths)) {
      case 1: LP_DEDUPE(1); break;
      case 2: LP_DEDUPE(2); break;
      case 4: LP_DEDUPE(4); break;
      default: LP_DEDUPE(8); break;
    }
#undef LP_DEDUPE
    check_launch("k_bpg_dedupe_all");
  }
  if (!any_wide) return true;
  if (listed) {                                 // wider programs: a lane group per listed key
    const int G = coop_group(P.bpg_widths);
    const dim3 grid(256), block(256);
    switch (G) {
      case 16: hipLaunchKernelGGL(k_bpg_coop_list<16>, grid, block, 0, st, keys, lbits, wcnt, wlist, text, ls, ll, P, flag); break;
      case 32: hipLaunchKernelGGL(k_bpg_coop_list<32>, grid, block, 0, st, keys, lbits, wcnt, wlist, text, ls, ll, P, flag); break;
      default: hipLaunchKernelGGL(k_bpg_coop_list<64>, grid, block, 0, st, keys, lbits, wcnt, wlist, text, ls, ll, P, flag); break;
    }
    check_launch("k_bpg_coop_list");
  } else {                                      // no list memory: a lane group per key in place
    launch_coop<1>(nullptr, keys, n, nullptr, lbits, text, ls, ll, P, flag, st, BPG_LANE_MAX_W + 1);
    check_launch("k_bpg_coop<dedupe>");
  }
  return true;
}

void bpg_scan_dev(const uint8_t* text, const int64_t* ls, const int32_t* ll, int64_t L, const int32_t* regs,
                  int nregs, const DfaPool& P, int64_t* out, int64_t cap, unsigned long long* count,
                  uint64_t stream) {
  if (!P.bpg_widths || L <= 0 || nregs <= 0) return;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid(nblocks(L, kScanLines), (unsigned)nregs);
  for_widths(P.bpg_widths, [&](auto w) {
    hipLaunchKernelGGL(k_bpg_scan<decltype(w)::value>, grid, dim3(kScanLines), 0, st, text, ls, ll, L, regs, P, out,
                       cap, count);
    check_launch("k_bpg_scan");
  });
  if (P.bpg_widths & kWideMask) {
    const int G = coop_group(P.bpg_widths);
    const int64_t per_block = 4 * (64 / G);      // 4 waves x lines per wave
    const dim3 g2((unsigned)std::max<int64_t>(1, (L + per_block - 1) / per_block), (unsigned)nregs);
    switch (G) {
      case 32: hipLaunchKernelGGL(k_bpg_scan_coop<32>, g2, dim3(256), 0, st, text, ls, ll, L, regs, P, out, cap, count); break;
      default: hipLaunchKernelGGL(k_bpg_scan_coop<64>, g2, dim3(256), 0, st, text, ls, ll, L, regs, P, out, cap, count); break;
    }
    check_launch("k_bpg_scan_coop");
  }
}

}  // namespace lp
