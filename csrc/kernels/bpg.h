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

// find() of one BPG program over s[0, n), word count rounded up to an instantiated width (unused
// words carry zero masks). The device version is a real call: the walk is long and the per-W bodies
// are large, so inlining them into every DFA-verify kernel would bloat all of those kernels.
#if defined(__HIP_DEVICE_COMPILE__)
static __device__ __attribute__((noinline)) bool bpg_find(const uint64_t* P, const uint8_t* s, int n)
#else
static inline bool bpg_find(const uint64_t* P, const uint8_t* s, int n)
#endif
{
  switch ((int)(P[0] & 0xFF)) {
    case 1: return bpg_find_w<1>(P, s, n);
    case 2: return bpg_find_w<2>(P, s, n);
    case 3: return bpg_find_w<3>(P, s, n);
    case 4: return bpg_find_w<4>(P, s, n);
    case 5: case 6: return bpg_find_w<6>(P, s, n);
    default: return bpg_find_w<8>(P, s, n);
  }
}

}  // namespace lp
