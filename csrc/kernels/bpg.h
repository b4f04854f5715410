// Bit-parallel Glushkov ("BPG") find() for regexes whose DFA exceeds engine.dfa-max-states.
//
// The program (built at library load by log_parser_amd/models/bpg.py, which documents the layout)
// decomposes the Glushkov follow relation into word-parallel parts: shift edges p -> p+1, self
// loops, "spread fields" (a bounded gap X.{0,n}Y is one field: every active source reaches every
// target above it, computed for all fields with ONE multi-word subtraction whose guard bits stop
// each borrow inside its field) and a short exception list (loop-backs, boundary-gated edges).
// Per byte and 64 positions that is ~20 VALU ops with no table walk on the dependency chain except
// the byte's class mask -- against M-squared multiply-accumulates for the same step as a
// state-transition GEMM (nfa_mfma.hip; profiles/r3_* hold the A/B).
//
// Matcher.find() semantics as the DFA walk (jregex.h): boundary context ctx = prev kind x next
// kind is checked before every byte (accept) and gates edges; extra accept check before a final
// line terminator; end of line is next kind N_EOS.
#pragma once
#include <stdint.h>

namespace lp {

constexpr int BPG_MAX_W = 8;          // 512 positions (models/bpg.py MAX_WORDS)
constexpr uint64_t BPG_UNIFORM = 1ull << 31;
constexpr uint64_t BPG_ANCHORED = 1ull << 30;

// next-kind of a byte: 2 word, 3 other, 4 UTF-8 continuation (jregex.h N_W / N_N / N_C)
LP_HD int byte_kind(int c) {
  const bool w = (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '_';
  return w ? 2 : (c >= 0x80 && c <= 0xBF) ? 4 : 3;
}

template <int W>
LP_HD bool bpg_find_w(const uint64_t* __restrict__ P, const uint8_t* __restrict__ s, int n) {
  const uint64_t hdr = P[0];
  const int E = (int)((hdr >> 8) & 0xFFF);
  const int ncls = (int)((hdr >> 20) & 0x3FF);
  const bool uniform = (hdr & BPG_UNIFORM) != 0;
  const bool anchored = (hdr & BPG_ANCHORED) != 0;
  const uint32_t nullm = (uint32_t)(hdr >> 32) & 0x7FFFu;
  const uint64_t* q = P + 1;
  uint64_t shm[W], selfm[W], src[W], R[W], lo[W], hi[W], f0[W], l0[W], S[W];
  const uint64_t* first = q + 6 * W;
  const uint64_t* last = first + 15 * W;
  const uint8_t* bm = reinterpret_cast<const uint8_t*>(last + 15 * W);
  const uint64_t* cls = last + 15 * W + 32;
  const uint64_t* exc = cls + (size_t)ncls * W;
#pragma unroll
  for (int w = 0; w < W; ++w) {
    shm[w] = q[w];
    selfm[w] = q[W + w];
    src[w] = q[2 * W + w];
    R[w] = q[3 * W + w];
    lo[w] = q[4 * W + w];
    hi[w] = q[5 * W + w];
    f0[w] = first[w];
    l0[w] = last[w];
    S[w] = 0;
  }
  const int ftl = final_term_len(s, n);
  const int ft = ftl ? n - ftl : -1;
  int prevk = 0;  // P_BOS
  for (int t = 0;; ++t) {
    const int c = t < n ? (int)s[t] : 0;
    const int nk = t < n ? byte_kind(c) : 0;  // N_EOS at end of line
    // accept before this byte (and before a final line terminator)
    for (int pass = (t == ft) ? 0 : 1; pass < 2; ++pass) {
      const int actx = prevk * 5 + (pass == 0 ? 1 : nk);
      if ((nullm >> actx) & 1u) return true;
      const uint64_t* L = uniform ? nullptr : last + actx * W;
      uint64_t any = 0;
#pragma unroll
      for (int w = 0; w < W; ++w) any |= S[w] & (uniform ? l0[w] : L[w]);
      if (any) return true;
    }
    if (t >= n) return false;
    const int ctx = prevk * 5 + nk;
    uint64_t F[W];
    // shift (with the carry across words) + self loops
    uint64_t carry = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) {
      const uint64_t x = S[w] & shm[w];
      F[w] = (x << 1) | carry | (S[w] & selfm[w]);
      carry = x >> 63;
    }
    // spread fields: d = (S & src | hi) - lo (multi-word borrow); targets above the lowest
    // active source of every field = R & ~(d ^ (S & src | hi))
    uint64_t borrow = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) {
      const uint64_t df = (S[w] & src[w]) | hi[w];
      const uint64_t u = df - lo[w];
      const uint64_t b1 = df < lo[w] ? 1ull : 0ull;
      const uint64_t d = u - borrow;
      const uint64_t b2 = u < borrow ? 1ull : 0ull;
      borrow = b1 | b2;
      F[w] |= R[w] & ~(d ^ df);
    }
    // exceptions: (source, condition, targets)
    for (int e = 0; e < E; ++e) {
      const uint64_t* x = exc + (size_t)e * (W + 1);
      const uint64_t h = x[0];
      const int p = (int)(h & 0xFFFF);
      const uint32_t cond = (uint32_t)(h >> 16) & 0xFFFFu;
      uint64_t sw = 0;
#pragma unroll
      for (int w = 0; w < W; ++w) sw = (w == (p >> 6)) ? S[w] : sw;
      if (((sw >> (p & 63)) & 1ull) && ((cond >> ctx) & 1u)) {
#pragma unroll
        for (int w = 0; w < W; ++w) F[w] |= x[1 + w];
      }
    }
    const uint64_t* C = cls + (size_t)bm[c] * W;
    const uint64_t* Fi = uniform ? nullptr : first + ctx * W;
    uint64_t alive = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) {
      S[w] = (F[w] | (uniform ? f0[w] : Fi[w])) & C[w];
      alive |= S[w];
    }
    if (anchored && !alive) return false;  // first set only at the line start: nothing can match
    prevk = nk == 2 ? 1 : 2;
  }
}

#if defined(__HIP__)
// Device walk of one program (kernels in bpg.hip, one instantiation per width W so each kernel's
// registers are sized for its own W): the line's bytes come from 16-byte ALIGNED vector loads one
// block ahead (a byte load per step would put a memory round trip on the dependency chain), the
// structural masks live in registers, class / first / last / exception rows are read through P --
// a global pointer for candidate verification, an LDS copy for the all-lines scan.
template <int W>
__device__ __forceinline__ bool bpg_find_dev(const uint64_t* __restrict__ P, const uint8_t* __restrict__ s, int n) {
  const uint64_t hdr = P[0];
  const int E = (int)((hdr >> 8) & 0xFFF);
  const int ncls = (int)((hdr >> 20) & 0x3FF);
  const bool uniform = (hdr & BPG_UNIFORM) != 0;
  const bool anchored = (hdr & BPG_ANCHORED) != 0;
  const uint32_t nullm = (uint32_t)(hdr >> 32) & 0x7FFFu;
  const uint64_t* q = P + 1;
  uint64_t shm[W], selfm[W], src[W], R[W], lo[W], hi[W], f0[W], l0[W], S[W];
  const uint64_t* first = q + 6 * W;
  const uint64_t* last = first + 15 * W;
  const uint8_t* bm = reinterpret_cast<const uint8_t*>(last + 15 * W);
  const uint64_t* cls = last + 15 * W + 32;
  const uint64_t* exc = cls + (size_t)ncls * W;
#pragma unroll
  for (int w = 0; w < W; ++w) {
    shm[w] = q[w];
    selfm[w] = q[W + w];
    src[w] = q[2 * W + w];
    R[w] = q[3 * W + w];
    lo[w] = q[4 * W + w];
    hi[w] = q[5 * W + w];
    f0[w] = first[w];
    l0[w] = last[w];
    S[w] = 0;
  }
  const int ftl = final_term_len(s, n);
  const int ft = ftl ? n - ftl : -1;
  int prevk = 0;  // P_BOS
// accept in boundary context ACTX (a macro, not a lambda: a lambda capturing S by reference kept
// the state array in scratch memory)
#define LP_BPG_ACCEPT(ACTX, RES)                                                 \
  do {                                                                           \
    const int a_ = (ACTX);                                                       \
    uint64_t any_ = 0;                                                           \
    if (uniform) {                                                               \
      _Pragma("unroll") for (int w = 0; w < W; ++w) any_ |= S[w] & l0[w];        \
    } else {                                                                     \
      const uint64_t* L_ = last + a_ * W;                                        \
      _Pragma("unroll") for (int w = 0; w < W; ++w) any_ |= S[w] & L_[w];        \
    }                                                                            \
    RES = ((nullm >> a_) & 1u) || any_ != 0;                                     \
  } while (0)
  bool hit = false;
  if (n > 0) {
    const int sh = (int)((uintptr_t)s & 15);
    const uint4* blk = reinterpret_cast<const uint4*>(s - sh);
    uint4 cur = blk[0];
    for (int t0 = -sh; t0 < n; t0 += 16) {
      const uint4 nxt = blk[1];   // (text is padded: the look-ahead stays in bounds)
      ++blk;
      const int j0 = t0 < 0 ? -t0 : 0;
      const int j1 = n - t0 < 16 ? n - t0 : 16;
      // PF bytes at a time: their class rows depend on the text only, not on the state, so all
      // PF rows are loaded before the first state update (one load latency per PF bytes instead
      // of two dependent loads -- byte map, then row -- on every byte's chain)
      constexpr int PF = W <= 4 ? 4 : 2;     // rows in flight (registers: PF x W words)
      for (int jb = j0; jb < j1; jb += PF) {
        uint64_t Cr[PF][W];
        int cb[PF];
#pragma unroll
        for (int q = 0; q < PF; ++q) {
          const int j = jb + q < 15 ? jb + q : 15;
          const uint32_t wv = (j < 4) ? cur.x : (j < 8) ? cur.y : (j < 12) ? cur.z : cur.w;
          cb[q] = (int)((wv >> (8 * (j & 3))) & 0xFFu);
          const uint64_t* row = cls + (size_t)bm[cb[q]] * W;
#pragma unroll
          for (int w = 0; w < W; ++w) Cr[q][w] = row[w];
        }
#pragma unroll
        for (int q = 0; q < PF; ++q) {
          if (jb + q >= j1) break;
          const int t = t0 + jb + q;
          const int c = cb[q];
          const int nk = byte_kind(c);
          if (t == ft) {
            LP_BPG_ACCEPT(prevk * 5 + 1, hit);
            if (hit) return true;
          }
          LP_BPG_ACCEPT(prevk * 5 + nk, hit);
          if (hit) return true;
          const int ctx = prevk * 5 + nk;
          uint64_t F[W];
          uint64_t carry = 0, borrow = 0;
#pragma unroll
          for (int w = 0; w < W; ++w) {
            const uint64_t x = S[w] & shm[w];
            F[w] = (x << 1) | carry | (S[w] & selfm[w]);
            carry = x >> 63;
            const uint64_t df = (S[w] & src[w]) | hi[w];
            const uint64_t u = df - lo[w];
            const uint64_t b1 = df < lo[w] ? 1ull : 0ull;
            const uint64_t d = u - borrow;
            const uint64_t b2 = u < borrow ? 1ull : 0ull;
            borrow = b1 | b2;
            F[w] |= R[w] & ~(d ^ df);
          }
          for (int e = 0; e < E; ++e) {
            const uint64_t* x = exc + (size_t)e * (W + 1);
            const uint64_t h = x[0];
            const int p = (int)(h & 0xFFFF);
            uint64_t sw = 0;
#pragma unroll
            for (int w = 0; w < W; ++w) sw = (w == (p >> 6)) ? S[w] : sw;
            if (((sw >> (p & 63)) & 1ull) && (((uint32_t)(h >> 16) >> ctx) & 1u)) {
#pragma unroll
              for (int w = 0; w < W; ++w) F[w] |= x[1 + w];
            }
          }
          uint64_t alive = 0;
          if (uniform) {
#pragma unroll
            for (int w = 0; w < W; ++w) {
              S[w] = (F[w] | f0[w]) & Cr[q][w];
              alive |= S[w];
            }
          } else {
            const uint64_t* Fi = first + ctx * W;
#pragma unroll
            for (int w = 0; w < W; ++w) {
              S[w] = (F[w] | Fi[w]) & Cr[q][w];
              alive |= S[w];
            }
          }
          if (anchored && !alive) return false;
          prevk = nk == 2 ? 1 : 2;
        }
      }
      cur = nxt;
    }
  }
  LP_BPG_ACCEPT(prevk * 5 + 0, hit);  // end of line (N_EOS)
  return hit;
#undef LP_BPG_ACCEPT
}
#endif

// host twin: find() of one BPG program over s[0, n) (width from the header). On the device the
// programs run in their own kernels (bpg.hip): dfa_run never walks them there.
inline bool bpg_find_host(const uint64_t* P, const uint8_t* s, int n) {
  switch ((int)(P[0] & 0xFF)) {
    case 1: return bpg_find_w<1>(P, s, n);
    case 2: return bpg_find_w<2>(P, s, n);
    case 3: return bpg_find_w<3>(P, s, n);
    case 4: return bpg_find_w<4>(P, s, n);
    case 6: return bpg_find_w<6>(P, s, n);
    default: return bpg_find_w<8>(P, s, n);
  }
}

}  // namespace lp
