// gfx950 (MI355X) kernels of the log-analysis pipeline + their host (CPU backend) twins.
//
// Hot loops of the reference and the kernel that replaces each:
//   K1 line split     AnalysisService.java:53              -> k_line_index (line_index.hip)
//   K3 primary match  AnalysisService.java:89-95           -> k_prefilter (literal bloom + Teddy in LDS)
//                                                             + k_pf_verify, DFA verify in lp_post.hip
//   K4/K5 aux match   ScoringService.java:272-347          -> same engine, all aux regexes
//   K6 context feats  ContextAnalysisService.java:27-83    -> k_feat_cov (lp_post.hip)
//   K7-K9 scoring     ScoringService.java:63-151           -> k_score (fp64, one thread / event)
// Wave64 throughout; block sizes are multiples of 64; persistent grid-stride grids sized to the
// 256 CUs so the LDS-resident bloom filter is loaded once per block, not once per tile.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "lp_api.h"
#include "lp_core.h"
#include "lp_host.h"

namespace lp {

#define LP_CHECK(x)                                                                           \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e_) + " at " #x); \
  } while (0)

static inline hipStream_t as_stream(uint64_t s) { return reinterpret_cast<hipStream_t>(s); }

// ---- host twins: the CPU backend (no-GPU serving, availability fallback, tests). Parallel over
// independent items with plain threads (lp_host.h); results are order-insensitive (callers sort).
void set_host_threads(int n) { host_threads() = std::max(1, n); }

// ------------------------------------------------------------------------------------------
// K3a: literal prefilter.  Bloom filter (2 hashes) of every literal's leading 2/3/4-gram lives
// in LDS; each lane scans 16 consecutive positions from one dwordx4 (+1 dword look-ahead),
// ASCII-lower-cased with SWAR, grams extracted with v_alignbyte. Bloom hits (rare) probe the
// global hash table and verify the whole literal; survivors append (regex, line) candidates.
constexpr int PF_THREADS = 512;


struct Appender {
  int64_t* out;
  int64_t cap;
  unsigned long long* count;
  __device__ void operator()(int64_t v) const {
    unsigned long long i = atomicAdd(count, 1ull);
    if ((int64_t)i < cap) out[i] = v;
  }
};

// Block-level candidate staging: LDS atomics per candidate, ONE global atomic per flush.
constexpr int PF_BUF = 1024;
struct LdsAppender {
  int64_t* buf;
  int* cnt;
  int64_t* out;
  int64_t cap;
  unsigned long long* gcount;
  __device__ void operator()(int64_t v) const {
    const int s = atomicAdd(cnt, 1);
    if (s < PF_BUF) {
      buf[s] = v;
    } else {  // overflow inside one iteration: spill straight to global
      unsigned long long i = atomicAdd(gcount, 1ull);
      if ((int64_t)i < cap) out[i] = v;
    }
  }
};

__device__ __forceinline__ void pf_flush(int64_t* buf, int* cnt, unsigned long long* gbase, int c, int64_t* out,
                                         int64_t cap, unsigned long long* gcount) {
  const int m = c < PF_BUF ? c : PF_BUF;
  if (threadIdx.x == 0) *gbase = atomicAdd(gcount, (unsigned long long)m);
  __syncthreads();
  const unsigned long long base = *gbase;
  for (int i = threadIdx.x; i < m; i += blockDim.x)
    if ((int64_t)(base + i) < cap) out[base + i] = buf[i];
  __syncthreads();
  if (threadIdx.x == 0) *cnt = 0;
  __syncthreads();
}

template <int G>
__device__ __forceinline__ uint32_t pf_bloom(const uint32_t* bl, int bits, uint32_t g4) {
  return bloom_test(bl, g4 & gram_mask(G), G, bits) ? 1u : 0u;
}

// Hot loop: only filter tests (tight, fully unrolled, branch-free). Rare path: one non-unrolled loop
// over the hit bitmask stages the hit; verification runs in k_pf_verify, so the probe/verify code
// exists once in the binary (no I-cache blow-up).
//   bloom tier (GM != 0): GM = set of gram lengths present (bit g), a compile-time constant so the
//     16 / S LDS reads of a unit pipeline behind one wait. S in {1, 2, 4}: every bloom literal
//     indexes S adjacent 4-byte windows, so only positions divisible by S are tested -- every
//     occurrence still has exactly one indexed window starting there.
//   short-literal tier (TD): Teddy byte-position masks. One 16-byte LDS read per text byte gives
//     (M0, M1, M2)[byte]; the rolling AND of three consecutive reads is the bucket mask of a 3-byte
//     window. 18 reads per 16-byte unit, ~5 VALU per position, no hashing. (A/B, profiles/r3_p:
//     a 4 KiB bloom of 3-byte windows tested at every position -- 4-byte reads, 4.5x less LDS
//     traffic -- was SLOWER, 824 -> 933 us per 1.33 GB: the hash multiply and bit math per
//     position outweigh the wider reads.)
//   Teddy table layout (profiles/r3_t PMC: the 4 KiB table read with ds_read_b128 at random byte
//     values ran 8.2 bank-conflict cycles per LDS instruction, LDS-bound): 16 copies, entry c of
//     copy j at 16-byte slot c * 16 + j, and lane l reads copy l & 15. A b128 read is serviced in
//     four 16-lane groups over 16 slots of 16 B; the lanes of each group have distinct l & 15, so
//     every group hits 16 distinct slots -- conflict-free for any bytes. 64 KiB of LDS: the TD
//     variant runs 1024-thread blocks, one per CU.
//   NLF: the line index's first pass rides on this read of the text (bulk DP steps): per 16-byte
//     unit the '\n' bits, four lanes' bits form the 64-bit mask word of 64 bytes (lanes 4q..4q+3
//     hold consecutive units), a wave's 64 units are 1 KiB of one 16 KiB tile -> one atomic count
//     per wave and tile; a '\r' right before a '\n' flags the '\n''s tile (CRLF logs). Counts and
//     masks equal line_index.hip k_nl_count's (which then does not run); its CRLF flags are a
//     superset of these (both are only hints for k_nl_lines' exact '\r' masks).
template <bool TD>
constexpr int pf_threads() { return TD ? 1024 : PF_THREADS; }

constexpr int NL_WORDS_PER_TILE = 256;     // line_index.hip: 64-byte mask words per 16 KiB tile

__device__ __forceinline__ uint32_t nl_zero_bytes(uint32_t t) {   // high bit of every 0x00 byte (exact)
  const uint32_t y = (t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
  return ~(y | t | 0x7F7F7F7Fu);
}
__device__ __forceinline__ uint32_t nl_pack4(uint32_t x) {          // bits 7, 15, 23, 31 -> bits 0..3
  const uint32_t y = x >> 7;
  const uint32_t z = (y | (y >> 7)) & 0x00030003u;
  return (z | (z >> 14)) & 0xFu;
}

template <int GM, int S, int PF_UNROLL, bool TD, bool NLF>
__global__ __launch_bounds__(pf_threads<TD>()) void k_prefilter(const uint8_t* __restrict__ text, int64_t nbytes,
                                                          PfTables T, const int64_t* __restrict__ line_start,
                                                          int64_t nlines, int64_t* cand, int64_t cap,
                                                          unsigned long long* count, NlOut NL) {
  // dynamic LDS: [bloom (1<<bits)/8 B, GM only][teddy 16 x 4 KiB, TD only][candidates PF_BUF x 8 B][cnt | pad | gbase]
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int bits = T.bloom_bits;
  const int nwords = GM ? (1 << bits) >> 5 : 0;
  uint32_t* bl = smem;
  uint32_t* td = smem + nwords;
  int64_t* buf = reinterpret_cast<int64_t*>(td + (TD ? 16 * 1024 : 0));
  int* cnt = reinterpret_cast<int*>(buf + PF_BUF);
  unsigned long long* gbase = reinterpret_cast<unsigned long long*>(buf + PF_BUF + 1);
  for (int i = threadIdx.x * 4; i < nwords; i += blockDim.x * 4)
    *reinterpret_cast<uint4*>(bl + i) = *reinterpret_cast<const uint4*>(T.bloom + i);
  if constexpr (TD)
    for (int i = threadIdx.x; i < 16 * 256; i += blockDim.x)   // slot i = entry i >> 4, copy i & 15
      reinterpret_cast<uint4*>(td)[i] = reinterpret_cast<const uint4*>(T.teddy)[i >> 4];
  if (threadIdx.x == 0) *cnt = 0;
  __syncthreads();
  const LdsAppender app{buf, cnt, cand, cap, count};
  const int64_t nunits = (nbytes + 15) >> 4;
  constexpr bool g2 = GM & 4, g3 = GM & 8, g4on = GM & 16;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const uint4* tt = reinterpret_cast<const uint4*>(td) + (threadIdx.x & 15);   // this lane's copy
  // one 16-byte unit: lower-case, test the grams / windows, stage the (rare) hits
  auto scan_unit = [&](int64_t p0, const uint4 v, const uint32_t nx) {
    const uint32_t w[5] = {lower4(v.x), lower4(v.y), lower4(v.z), lower4(v.w), lower4(nx)};
    const int64_t rem = nbytes - p0;
    const uint32_t valid = rem >= 16 ? 0xFFFFu : ((1u << rem) - 1u);
    if constexpr (GM != 0) {
      uint32_t m4 = 0, m3 = 0, m2 = 0;
#pragma unroll
      for (int k = 0; k < 16; k += S) {
        const uint32_t gram = (k & 3) ? __builtin_amdgcn_alignbyte(w[(k >> 2) + 1], w[k >> 2], k & 3) : w[k >> 2];
        if constexpr (g4on) m4 |= pf_bloom<4>(bl, bits, gram) << k;
        if constexpr (g3) m3 |= pf_bloom<3>(bl, bits, gram) << k;
        if constexpr (g2) m2 |= pf_bloom<2>(bl, bits, gram) << k;
      }
      uint64_t hm = ((uint64_t)(m4 & valid) << 32) | ((uint64_t)(m3 & valid) << 16) | (uint64_t)(m2 & valid);
      while (hm) {  // rare: stage the gram hit; literal verification runs in k_pf_verify
        const int b = __ffsll((unsigned long long)hm) - 1;
        hm &= hm - 1;
        app(((p0 + (b & 15)) << 2) | (int64_t)(b >> 4));   // (position, gram length - 2)
      }
    }
    if constexpr (TD) {
      uint32_t r0 = 0, r1 = 0, any = 0;
#pragma unroll
      for (int k = 0; k < 18; ++k) {
        const uint4 e = tt[((w[k >> 2] >> (8 * (k & 3))) & 0xFFu) << 4];
        if (k >= 2) any |= r1 & e.z;           // window starting at k - 2 complete
        r1 = r0 & e.y;
        r0 = e.x;
      }
      if (any) {                               // rare: which positions
        uint32_t hm = 0;
        for (int k = 0; k < 16; ++k) {
          const uint32_t b0 = (w[k >> 2] >> (8 * (k & 3))) & 0xFFu;
          const uint32_t b1 = (w[(k + 1) >> 2] >> (8 * ((k + 1) & 3))) & 0xFFu;
          const uint32_t b2 = (w[(k + 2) >> 2] >> (8 * ((k + 2) & 3))) & 0xFFu;
          if (tt[b0 << 4].x & tt[b1 << 4].y & tt[b2 << 4].z) hm |= 1u << k;
        }
        hm &= valid;
        while (hm) {
          const int b = __ffs(hm) - 1;
          hm &= hm - 1;
          app(((p0 + b) << 2) | 3);            // code 3: short-literal tier
        }
      }
    }
  };
  // PF_UNROLL units per lane per iteration, all loads issued before any is scanned: more bytes in
  // flight per barrier interval (the strided scan is latency-, not VALU-bound)
  for (int64_t ub = (int64_t)blockIdx.x * blockDim.x * PF_UNROLL; ub < nunits; ub += PF_UNROLL * stride) {
    uint4 v[PF_UNROLL];
    uint32_t nx[PF_UNROLL];
#pragma unroll
    for (int j = 0; j < PF_UNROLL; ++j) {
      const int64_t u = ub + threadIdx.x + (int64_t)j * blockDim.x;
      v[j] = {0, 0, 0, 0};
      nx[j] = 0;
      if (u < nunits) {
        v[j] = *reinterpret_cast<const uint4*>(text + (u << 4));
        nx[j] = *reinterpret_cast<const uint32_t*>(text + (u << 4) + 16);
      }
    }
    if constexpr (NLF) {
#pragma unroll
      for (int j = 0; j < PF_UNROLL; ++j) {
        const int64_t u = ub + threadIdx.x + (int64_t)j * blockDim.x;
        const int64_t p0 = u << 4;
        uint32_t m16 = 0;
        if (u < nunits) {
          const uint32_t w4[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
          uint32_t cr16 = 0;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            m16 |= nl_pack4(nl_zero_bytes(w4[q] ^ 0x0A0A0A0Au)) << (4 * q);
            cr16 |= nl_pack4(nl_zero_bytes(w4[q] ^ 0x0D0D0D0Du)) << (4 * q);
          }
          const int64_t rem = nbytes - p0;
          const uint32_t valid = rem >= 16 ? 0xFFFFu : ((1u << rem) - 1u);
          m16 &= valid;
          cr16 &= valid;
          if (cr16) {                          // rare outside CRLF logs
            const uint32_t nl_next = (rem > 16 && (nx[j] & 0xFFu) == 0x0Au) ? 1u : 0u;
            uint32_t pairs = cr16 & ((m16 | (nl_next << 16)) >> 1);
            while (pairs) {
              const int b = __ffs(pairs) - 1;
              pairs &= pairs - 1;
              atomicOr(NL.crf + ((p0 + b + 1) >> 14), 1);
            }
          }
        }
        // every lane shuffles (convergent); lane 4q writes the word of units 4q..4q+3
        const uint32_t m01 = m16 | ((uint32_t)__shfl_down((int)m16, 1, 64) << 16);
        const uint32_t m23 = (uint32_t)__shfl_down((int)m01, 2, 64);
        const int64_t word = u >> 2;
        if ((threadIdx.x & 3) == 0 && word < NL.ntiles * NL_WORDS_PER_TILE)
          NL.nlm[word] = (uint64_t)m01 | ((uint64_t)m23 << 32);
        int c = __popc(m16);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
        if ((threadIdx.x & 63) == 0 && c) atomicAdd(NL.cnt + ((u >> 10)), c);   // lane 0: the wave's first unit
      }
    }
#pragma unroll
    for (int j = 0; j < PF_UNROLL; ++j) {
      const int64_t u = ub + threadIdx.x + (int64_t)j * blockDim.x;
      if (u < nunits) scan_unit(u << 4, v[j], nx[j]);
    }
    __syncthreads();
    const int c = *reinterpret_cast<volatile int*>(cnt);
    if (c >= PF_BUF / 2) pf_flush(buf, cnt, gbase, c, cand, cap, count);
  }
  __syncthreads();
  const int c = *reinterpret_cast<volatile int*>(cnt);
  if (c > 0) pf_flush(buf, cnt, gbase, c, cand, cap, count);
}

// K3a': literal verification of staged gram hits. A 16-lane group takes one gram hit: all lanes
// probe the (small) hash table together, then the bucket's literals are split across the lanes --
// a hit's cost is ~4 dependent memory round trips instead of ~3 per literal in the bucket, which
// decides the latency of small requests (shared grams give buckets of up to ~70 literals).
// LANES per gram hit: 16 for small inputs (latency: a 67-literal bucket is 5 rounds), 4 for large
// ones (throughput: the typical bucket holds ~3 literals, so 16 lanes would idle 13 of them).
template <int PV_LANES>
__global__ __launch_bounds__(256) void k_pf_verify(const int64_t* __restrict__ ghits, int64_t n,
                                                   const unsigned long long* __restrict__ dn,
                                                   const uint8_t* __restrict__ text, int64_t nbytes, PfTables T,
                                                   const int64_t* __restrict__ line_start, int64_t nlines,
                                                   const int32_t* __restrict__ blk_line, int64_t* cand, int64_t cap,
                                                   unsigned long long* count) {
  // candidates staged in LDS, one global atomic per flush (a per-candidate atomic on one counter
  // serialises ~1M appends per step at the L2). With `dn` the hit count is read on the device
  // (capped at the buffer size n) and the grid strides over it: no host round trip in between.
  __shared__ int64_t buf[PF_BUF];
  __shared__ int cnt;
  __shared__ unsigned long long gbase;
  if (threadIdx.x == 0) cnt = 0;
  __syncthreads();
  if (dn) {
    const int64_t d = (int64_t)*dn;
    n = d < n ? d : n;
  }
  const LdsAppender app{buf, &cnt, cand, cap, count};
  constexpr int HITS_PER_BLOCK = 256 / PV_LANES;
  const int sub = threadIdx.x / PV_LANES, lane = threadIdx.x % PV_LANES;
  const int64_t stride = (int64_t)gridDim.x * HITS_PER_BLOCK;
  for (int64_t base = (int64_t)blockIdx.x * HITS_PER_BLOCK; base < n; base += stride) {
    const int64_t i = base + sub;
    if (i < n) {
      const int64_t h = ghits[i];
      const int64_t p = h >> 2;
      const bool td = (h & 3) == 3;
      const int G = td ? 3 : 2 + (int)(h & 3);
      // the 16 text bytes [p - 4, p + 12), lower-cased: window + the fingerprint context of every
      // literal of the bucket (4 bytes before, 4 after the window)
      uint32_t a[4];
      if (p >= 4) {
        load16u(text + p - 4, a);
      } else {
        for (int k = 0; k < 4; ++k) {
          uint32_t v = 0;
          for (int b = 3; b >= 0; --b) {
            const int64_t x = p - 4 + 4 * k + b;
            v = (v << 8) | (x >= 0 ? (uint32_t)text[x] : 0u);
          }
          a[k] = v;
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) a[k] = lower4(a[k]);
      const uint64_t t8 = (uint64_t)a[0] |
                          ((uint64_t)(G == 4 ? a[2] : __builtin_amdgcn_alignbyte(a[2], a[1], G)) << 32);
      int64_t line = -1;
      // one bucket (bloom tier) or the buckets of a Teddy mask: entries [j0, j1) of ents / fps
      auto walk = [&](const int32_t* ents, const uint64_t* fps, int j0, int j1) {
        for (int j = j0 + lane; j < j1; j += PV_LANES) {
          const uint4 f = *reinterpret_cast<const uint4*>(fps + 2 * j);    // {fingerprint, mask}
          const uint64_t fp = (uint64_t)f.x | ((uint64_t)f.y << 32), fm = (uint64_t)f.z | ((uint64_t)f.w << 32);
          if ((t8 ^ fp) & fm) continue;            // a context byte differs: not this literal
          const int32_t e = ents[j];
          if (!pf_lit_at(T, text, nbytes, p, e)) continue;
          const int lit = pf_entry_lit(e);
          if (line < 0) line = locate_line(line_start, nlines, blk_line, p);
          if (line < 0) line = 0;
          for (int r = T.lit_reg_off[lit]; r < T.lit_reg_off[lit + 1]; ++r) app(((int64_t)T.lit_reg[r] << 32) | line);
        }
      };
      if (td) {                                    // short-literal tier: every literal of the buckets
        const uint32_t b1 = p + 1 < nbytes ? (a[1] >> 8) & 0xFF : 0u, b2 = p + 2 < nbytes ? (a[1] >> 16) & 0xFF : 0u;
        uint32_t m = T.teddy[4 * (a[1] & 0xFF)] & T.teddy[4 * b1 + 1] & T.teddy[4 * b2 + 2];
        while (m) {
          const int b = __ffs(m) - 1;
          m &= m - 1;
          walk(T.tb_lits, T.tb_fp, T.tb_off[b], T.tb_off[b + 1]);
        }
      } else {
        int s0, c;
        pf_bucket(T, a[1] & gram_mask(G), G, s0, c);
        walk(T.gram_lits, T.gram_fp, s0, s0 + c);
      }
    }
    __syncthreads();
    const int c = *reinterpret_cast<volatile int*>(&cnt);
    if (c >= PF_BUF / 2) pf_flush(buf, &cnt, &gbase, c, cand, cap, count);
  }
  __syncthreads();
  const int c = *reinterpret_cast<volatile int*>(&cnt);
  if (c > 0) pf_flush(buf, &cnt, &gbase, c, cand, cap, count);
}

// K3c: regexes without a usable literal: every line x every scan regex
__global__ __launch_bounds__(256) void k_scan(const uint8_t* __restrict__ text,
                                              const int64_t* __restrict__ line_start,
                                              const int32_t* __restrict__ line_len, int64_t nlines,
                                              const int32_t* __restrict__ regs, int nregs, DfaPool P,
                                              int64_t* out, int64_t cap, unsigned long long* count) {
  const int64_t line = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (line >= nlines) return;
  const uint8_t* s = text + line_start[line];
  const int n = line_len[line];
  const Appender app{out, cap, count};
  for (int j = 0; j < nregs; ++j) {
    const int r = regs[j];
    if (dfa_run(P, r, s, n)) app(((int64_t)r << 32) | line);
  }
}

// ------------------------------------------------------------------------------------------
// K7-K9: fused score epilogue, one lane per event
// 64 events per workgroup, one wave per factor group: proximity (wave 0), temporal (wave 1) and
// context (wave 2) are each a chain of dependent table / hit-list loads and run side by side; wave 3
// loads the event's own factors and multiplies in score_event's order (bit-identical). A batch of a
// few thousand events is latency-bound (a handful of waves per CU), so the chains' overlap is what
// the kernel's time is made of.
constexpr int kScoreEv = 64;
__global__ __launch_bounds__(4 * kScoreEv) void k_score(const int32_t* __restrict__ ev_line,
                                                        const int32_t* __restrict__ ev_pat,
                                                        const int32_t* __restrict__ ev_seg, FreqIn F,
                                                        int64_t n, ScoreTables T, ScoreParams S,
                                                        double* __restrict__ out, double* __restrict__ factors,
                                                        const int64_t* __restrict__ dn) {
  __shared__ double fx[3][kScoreEv];
  const int part = (int)threadIdx.x / kScoreEv, j = (int)threadIdx.x % kScoreEv;   // part: wave-uniform
  const int64_t i = (int64_t)blockIdx.x * kScoreEv + j;
  const bool on = i < n && !(dn && i >= dn[0]);
  double conf = 0.0, sev = 0.0, chrono = 0.0, pen = 0.0;
  if (on) {
    const int32_t x = ev_line[i], p = ev_pat[i], sg = ev_seg[i];
    const int32_t lo = T.seg_lo[sg], hi = T.seg_hi[sg];
    if (part == 0) {
      fx[0][j] = prox_factor(T, S, x, p, lo, hi);
    } else if (part == 1) {
      fx[1][j] = temp_factor(T, x, p, lo, hi, T.seg_own_lo[sg]);
    } else if (part == 2) {
      fx[2][j] = ctx_factor(T, S, x, p, lo, hi);
    } else {
      conf = T.conf[p];
      sev = T.sev[p];
      chrono = chrono_factor(T.seg_g0[sg] + (x - lo), T.seg_n[sg], S);
      pen = pen_factor(S, freq_before(F, i));
    }
  }
  __syncthreads();
  if (part != 3 || !on) return;
  const double prox = fx[0][j], temp = fx[1][j], ctx = fx[2][j];
  if (factors) {
    double* f = factors + 7 * i;
    f[0] = conf; f[1] = sev; f[2] = chrono; f[3] = prox; f[4] = temp; f[5] = ctx; f[6] = pen;
  }
  out[i] = conf * sev * chrono * prox * temp * ctx * (1.0 - pen);
}


// ------------------------------------------------------------------------------------------
// Cross-shard sequence carry: for every sequence-event slot j = (sequence q,
// event k) run the reference's backward chain (ScoringService.java:252-257, 296-305) from the
// END of this rank's owned lines needing events k..0; out[j] = first event index still unmatched
// when the owned range is exhausted (-1: chain complete). Ranks all-gather these tables and
// compose them right-to-left, which reproduces the unbounded backward search across shards.
__global__ __launch_bounds__(256) void k_seq_chain(const int32_t* __restrict__ slot_seq,
                                                   const int32_t* __restrict__ seq_ev_off,
                                                   const int32_t* __restrict__ seq_ev_reg,
                                                   const int64_t* __restrict__ hit_off,
                                                   const int32_t* __restrict__ hit_line, int32_t own_lo,
                                                   int32_t own_hi, int nslots, int32_t* __restrict__ out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nslots) return;
  ScoreTables T;
  T.hit_off = hit_off;
  T.hit_line = hit_line;
  const int q = slot_seq[j];
  const int e0 = seq_ev_off[q];
  int k = j - e0;
  int32_t cur = own_hi;
  while (k >= 0) {
    const int32_t f = pred_hit(T, seq_ev_reg[e0 + k], own_lo, cur);
    if (f < 0) break;
    cur = f;
    --k;
  }
  out[j] = k;
}

// ==========================================================================================
// launchers (device) and host twins
static int num_blocks(int64_t n, int t) { return (int)std::max<int64_t>(1, (n + t - 1) / t); }

template <int GM, int S, bool TD>
static void launch_pf(int g, size_t lds, bool big, hipStream_t st, const uint8_t* text, int64_t nbytes,
                      const PfTables& T, const int64_t* line_start, int64_t nlines, int64_t* cand, int64_t cap,
                      unsigned long long* count, const NlOut* nl) {
  const NlOut NL = nl ? *nl : NlOut();
#define LP_PF_K(U, F)                                                                                          \
  hipLaunchKernelGGL((k_prefilter<GM, S, U, TD, F>), dim3(g), dim3(pf_threads<TD>()), lds, st, text, nbytes, T, \
                     line_start, nlines, cand, cap, count, NL)
  if (big) {
    if (nl) LP_PF_K(4, true); else LP_PF_K(4, false);
  } else {
    if (nl) LP_PF_K(1, true); else LP_PF_K(1, false);
  }
#undef LP_PF_K
}

template <bool TD>
static void dispatch_pf(int g, bool big, hipStream_t st, const uint8_t* text, int64_t nbytes, const PfTables& T,
                        const int64_t* line_start, int64_t nlines, int64_t* cand, int64_t cap,
                        unsigned long long* count, const NlOut* nl) {
  const int gm = T.gmask & 28;
  const size_t lds = (gm ? (size_t(1) << T.bloom_bits) / 8 : 0) + (TD ? 16 * 4096 : 0) + PF_BUF * 8 + 16;
#define LP_PF(GMV, SV) launch_pf<GMV, SV, TD>(g, lds, big, st, text, nbytes, T, line_start, nlines, cand, cap, count, nl)
  if (gm == 16 && T.stride == 4) { LP_PF(16, 4); return; }
  if (gm == 16 && T.stride == 2) { LP_PF(16, 2); return; }
  switch (gm) {
    case 0: if (TD) LP_PF(0, 1); break;      // short literals only
    case 4: LP_PF(4, 1); break;
    case 8: LP_PF(8, 1); break;
    case 12: LP_PF(12, 1); break;
    case 16: LP_PF(16, 1); break;
    case 20: LP_PF(20, 1); break;
    case 24: LP_PF(24, 1); break;
    default: LP_PF(28, 1); break;
  }
#undef LP_PF
}

void prefilter_dev(const uint8_t* text, int64_t nbytes, const PfTables& T, const int64_t* line_start, int64_t nlines,
                   int64_t* cand, int64_t cap, unsigned long long* count, int grid, uint64_t stream, const NlOut* nl) {
  if (nbytes <= 0 || ((T.gmask & 28) == 0 && !T.teddy_on)) {   // no literals: nothing to prefilter
    if (nl) throw std::runtime_error("prefilter_dev: the fused line-index pass needs a prefilter");
    return;
  }
  const int64_t units = (nbytes + 15) / 16;
  // large texts: 4 units per lane per iteration (bytes in flight); small requests: 1, so every
  // launched lane has work (latency)
  const bool big = nbytes >= (int64_t(32) << 20);
  const int threads = T.teddy_on ? pf_threads<true>() : pf_threads<false>();
  const int g = (int)std::min<int64_t>(grid, num_blocks(units, threads * (big ? 4 : 1)));
  if (T.teddy_on)
    dispatch_pf<true>(g, big, as_stream(stream), text, nbytes, T, line_start, nlines, cand, cap, count, nl);
  else
    dispatch_pf<false>(g, big, as_stream(stream), text, nbytes, T, line_start, nlines, cand, cap, count, nl);
  LP_CHECK(hipGetLastError());
}

static int g_pv_lanes_bulk = 4;
void set_pf_verify_lanes(int n) { g_pv_lanes_bulk = (n == 1 || n == 2 || n == 4 || n == 16) ? n : 4; }

void pf_verify_dev(const int64_t* ghits, int64_t n, const uint8_t* text, int64_t nbytes, const PfTables& T,
                   const int64_t* line_start, int64_t nlines, const int32_t* blk_line, int64_t* cand, int64_t cap,
                   unsigned long long* count, uint64_t stream, const unsigned long long* dn, int max_grid) {
  if (n <= 0) return;
  // with a device-side count the grid is sized for the buffer but capped (grid-stride loop)
  const int lanes = nbytes >= (int64_t(64) << 20) ? g_pv_lanes_bulk : 16;
  const int64_t need = (n + 256 / lanes - 1) / (256 / lanes);   // blocks for one pass over n hits
  const int g = dn ? (int)std::min<int64_t>(need, std::max(1, max_grid)) : (int)std::max<int64_t>(1, need);
#define LP_PV(L)                                                                                                  \
  hipLaunchKernelGGL(k_pf_verify<L>, dim3(g), dim3(256), 0, as_stream(stream), ghits, n, dn, text, nbytes, T, \
                     line_start, nlines, blk_line, cand, cap, count)
  switch (lanes) {
    case 1: LP_PV(1); break;
    case 2: LP_PV(2); break;
    case 4: LP_PV(4); break;
    default: LP_PV(16); break;
  }
#undef LP_PV
  LP_CHECK(hipGetLastError());
}

// pre-verified keys from the host (the backtracker side path, bt_prepass) appended to a matcher's
// verified-hit buffer behind the device engines' hits: one reservation per block
__global__ __launch_bounds__(256) void k_append_keys(int64_t* __restrict__ dst, int64_t cap,
                                                     unsigned long long* __restrict__ count,
                                                     const int64_t* __restrict__ src, int64_t n) {
  __shared__ unsigned long long base;
  const int64_t b0 = (int64_t)blockIdx.x * blockDim.x;
  const int64_t nb = min((int64_t)blockDim.x, n - b0);
  if (threadIdx.x == 0) base = atomicAdd(count, (unsigned long long)nb);
  __syncthreads();
  const int64_t i = b0 + threadIdx.x;
  if (i < n && (int64_t)(base + threadIdx.x) < cap) dst[base + threadIdx.x] = src[i];
}

void append_keys_dev(int64_t* dst, int64_t cap, unsigned long long* count, const int64_t* src, int64_t n,
                     uint64_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_append_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), dst, cap, count, src, n);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e) + " in k_append_keys");
}

void scan_dev(const uint8_t* text, const int64_t* line_start, const int32_t* line_len, int64_t nlines,
              const int32_t* regs, int nregs, const DfaPool& P, int64_t* out, int64_t cap, unsigned long long* count,
              uint64_t stream) {
  if (nlines <= 0 || nregs <= 0) return;
  hipLaunchKernelGGL(k_scan, dim3(num_blocks(nlines, 256)), dim3(256), 0, as_stream(stream), text, line_start,
                     line_len, nlines, regs, nregs, P, out, cap, count);
  LP_CHECK(hipGetLastError());
  bpg_scan_dev(text, line_start, line_len, nlines, regs, nregs, P, out, cap, count, stream);   // DFA blow-ups
}

void score_dev(const int32_t* ev_line, const int32_t* ev_pat, const int32_t* ev_seg, const FreqIn& F, int64_t n,
               const ScoreTables& T, const ScoreParams& S, double* out, double* factors, uint64_t stream,
               const int64_t* dn) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_score, dim3(num_blocks(n, kScoreEv)), dim3(4 * kScoreEv), 0, as_stream(stream), ev_line, ev_pat,
                     ev_seg, F, n, T, S, out, factors, dn);
  LP_CHECK(hipGetLastError());
}

void seq_chain_dev(const int32_t* slot_seq, const int32_t* seq_ev_off, const int32_t* seq_ev_reg,
                   const int64_t* hit_off, const int32_t* hit_line, int32_t own_lo, int32_t own_hi, int nslots,
                   int32_t* out, uint64_t stream) {
  if (nslots <= 0) return;
  hipLaunchKernelGGL(k_seq_chain, dim3(num_blocks(nslots, 256)), dim3(256), 0, as_stream(stream), slot_seq,
                     seq_ev_off, seq_ev_reg, hit_off, hit_line, own_lo, own_hi, nslots, out);
  LP_CHECK(hipGetLastError());
}

// ---------------- host twins (CPU backend) ----------------
void seq_chain_host(const int32_t* slot_seq, const int32_t* seq_ev_off, const int32_t* seq_ev_reg,
                    const int64_t* hit_off, const int32_t* hit_line, int32_t own_lo, int32_t own_hi, int nslots,
                    int32_t* out) {
  ScoreTables T;
  T.hit_off = hit_off;
  T.hit_line = hit_line;
  for (int j = 0; j < nslots; ++j) {
    const int q = slot_seq[j];
    const int e0 = seq_ev_off[q];
    int k = j - e0;
    int32_t cur = own_hi;
    while (k >= 0) {
      const int32_t f = pred_hit(T, seq_ev_reg[e0 + k], own_lo, cur);
      if (f < 0) break;
      cur = f;
      --k;
    }
    out[j] = k;
  }
}
int64_t nl_positions_host(const uint8_t* text, int64_t nbytes, int64_t* nl_pos) {
  int64_t c = 0;
  const uint8_t* p = text;
  const uint8_t* e = text + nbytes;
  while (p < e) {
    const void* q = memchr(p, '\n', e - p);
    if (!q) break;
    const uint8_t* qq = static_cast<const uint8_t*>(q);
    if (nl_pos) nl_pos[c] = qq - text;
    ++c;
    p = qq + 1;
  }
  return c;
}

int64_t prefilter_host(const uint8_t* text, int64_t nbytes, const PfTables& T, const int64_t* line_start,
                       int64_t nlines, int64_t* cand, int64_t cap) {
  std::vector<std::vector<int64_t>> part(std::max(1, host_threads()));
  const int S = std::max(1, T.stride);
  // 4-gram-only bloom, no Teddy tier: the AVX-512 path, threads only for multi-MB texts (request-sized
  // texts ran slower on the pool than on the calling thread)
  const bool vec = prefilter_bloom_simd_ok();
  const bool simd = vec && T.gmask == (1 << 4) && (S == 1 || S == 2 || S == 4);
  host_parallel(nbytes, vec ? (int64_t(4) << 20) : (1 << 18), [&](int t, int64_t a, int64_t b) {
    auto& out = part[t];
    auto app = [&](int64_t v) { out.push_back(v); };
    const uint32_t* bl = T.bloom;
    // lower-cased 4-gram starting at p (bytes past the end read as 0): one unaligned load + SWAR
    auto gram = [&](int64_t p) -> uint32_t {
      if (p + 4 <= nbytes) {
        uint32_t w;
        std::memcpy(&w, text + p, 4);
        return lower4(w);
      }
      uint32_t g4 = 0;
      for (int k = 3; k >= 0; --k) g4 = (g4 << 8) | (uint32_t)(p + k < nbytes ? lower_byte(text[p + k]) : 0);
      return g4;
    };
    // bloom tier: like k_prefilter<GM, S>, only positions divisible by the stride (one candidate
    // per literal occurrence, not one per indexed window)
    auto bloom_at = [&](int64_t p) {
      const uint32_t g4 = gram(p);
      for (int g = 4; g >= 2; --g) {
        if (!(T.gmask & (1 << g))) continue;
        const uint32_t key = g4 & gram_mask(g);
        if (!bloom_test(bl, key, g, T.bloom_bits)) continue;
        pf_probe(T, text, nbytes, p, key, g, line_start, nlines, nullptr, app);
      }
    };
    const int64_t p0 = (a + S - 1) / S * S;
    // the two tiers in separate passes (candidates are unordered: the hit CSR sorts them)
    if (simd) {
      const int64_t v0 = (a + 3) & ~int64_t(3);
      for (int64_t p = p0; p < v0 && p < b; p += S) bloom_at(p);
      const int64_t v1 = prefilter_bloom_simd(text, nbytes, T, line_start, nlines, v0, b, out);
      for (int64_t p = std::max(v1, p0); p < b; p += S) bloom_at(p);
    } else if (T.gmask) {           // the stride's positions only
      for (int64_t p = p0; p < b; p += S) bloom_at(p);
    }
    if (T.teddy_on) {
      const int64_t t1 = vec ? prefilter_teddy_simd(text, nbytes, T, line_start, nlines, a, b, out) : a;
      for (int64_t p = t1; p < b; ++p) {
        const uint32_t m = teddy_mask(T, text, nbytes, p);
        if (m) teddy_probe(T, text, nbytes, p, m, line_start, nlines, nullptr, app);
      }
    }
  });
  int64_t count = 0;
  for (auto& v : part)
    for (int64_t x : v) {
      if (count < cap) cand[count] = x;
      ++count;
    }
  return count;
}

int64_t scan_host(const uint8_t* text, const int64_t* line_start, const int32_t* line_len, int64_t nlines,
                  const int32_t* regs, int nregs, const DfaPool& P, int64_t* out, int64_t cap) {
  if (nregs == 0) return 0;
  std::vector<std::vector<int64_t>> part(std::max(1, host_threads()));
  host_parallel(nlines, 2048, [&](int t, int64_t a, int64_t b) {
    for (int64_t line = a; line < b; ++line)
      for (int j = 0; j < nregs; ++j)
        if (dfa_run(P, regs[j], text + line_start[line], line_len[line]))
          part[t].push_back(((int64_t)regs[j] << 32) | line);
  });
  int64_t c = 0;
  for (auto& v : part)
    for (int64_t x : v) {
      if (c < cap) out[c] = x;
      ++c;
    }
  return c;
}

void score_host(const int32_t* ev_line, const int32_t* ev_pat, const int32_t* ev_seg, const FreqIn& F, int64_t n,
                const ScoreTables& T, const ScoreParams& S, double* out, double* factors) {
  host_parallel(n, 1024, [&](int, int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i)
      out[i] = score_event(T, S, ev_line[i], ev_pat[i], ev_seg[i], freq_before(F, i),
                           factors ? factors + 7 * i : nullptr);
  });
}

}  // namespace lp
