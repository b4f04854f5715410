// Bit-parallel Glushkov ("BPG") find() for regexes whose DFA exceeds engine.dfa-max-states or that
// need code-point boundary contexts (MULTILINE ^ $, Unicode \b).
//
// The program (built at library load by jregex.cpp bpg_program from the CODE-POINT Glushkov NFA)
// decomposes the follow relation into word-parallel parts: shift edges p -> p+1, self loops,
// "spread fields" (a bounded gap X.{0,n}Y is one field: every active source reaches every target
// above it, computed for all fields with ONE multi-word subtraction whose guard bits stop each
// borrow inside its field) and a short exception list (loop-backs, boundary-gated edges). Per code
// point and 64 positions that is ~20 VALU ops with no table walk on the dependency chain except
// the character's class mask -- against M-squared multiply-accumulates for the same step as a
// state-transition GEMM (nfa_mfma.hip; profiles/r3_* hold the A/B).
//
// The walk steps once per CODE POINT: a UTF-8 lead byte is decoded (with its continuation bytes)
// and mapped to its class through a sorted range table, continuation bytes are skipped, ASCII goes
// through a 128-entry map. So '.', [^x] or \p{L} is ONE position (exact: '.' excludes U+0085 /
// U+2028 / U+2029 as Java's does) and X.{0,1000}Y is ~1000 positions = 16 words.
//
// Matcher.find() semantics (jregex.h): boundary context ctx = prev kind x next kind (24 contexts,
// ctx = prev * 6 + next) is checked before every code point (accept) and gates edges; extra accept
// check before a final line terminator; end of line is next kind N_EOS.
//
// Counted positions: a bounded repeat of one class C{m,n} (n - m >= BPG_CTR_MIN) is m plain positions
// plus ONE counted position p for C{0,n-m} (jregex.cpp Glushkov). p has no self edge in the follow
// relation; the walk keeps a count per counted position -- the characters the YOUNGEST thread in p
// has consumed (a thread that entered later is never worse: every thread in p reads the same
// characters and has the same follow set, and only an upper bound applies) -- and p stays active
// through its own loop only while that count is below the bound; an entry (any edge into p,
// first-set included) restarts the count at 1. So X.{0,20000}Y costs 3 positions + 1 count.
//
// Program layout (uint64 words):
//   [0] W | E << 8 | ncls << 20 | anchored << 30 | uniform << 31 | nullable(24) << 32 | uword << 56
//       | ncounters << 57
//   [1] nranges | total words << 32
//   [2 ..]           shm[W] selfm[W] src[W] R[W] lo[W] hi[W]
//   [2 + 6W ..]      first[24][W]           (per boundary context; uniform -> only [0] is read)
//   [2 + 30W ..]     last[24][W]
//   [2 + 54W ..]     amap: 128 x uint16 (ASCII code point -> class), 32 words
//   [2 + 54W + 32..] cls[ncls][W]
//   then             exc[E][1 + W]          (src | cond << 16, then the target mask)
//   then             ranges[nranges]        (lo | class << 21 | kind << 37; kind 0 N, 1 W, 2 T),
//                                           sorted by lo, first lo = 0x80
//   then             ctr[ncounters]         (position | bound << 16)
#pragma once
#include <stdint.h>

namespace lp {

constexpr int BPG_LANE_MAX_W = 8;      // widest program of the one-lane-per-line walk
constexpr int BPG_CTR_MAX = 4;         // counted positions per program (jregex.h BPG_MAX_CTR)
constexpr int BPG_EXC_REG = 4;         // exception headers the device walks keep in registers
constexpr uint64_t BPG_UNIFORM = 1ull << 31;
constexpr uint64_t BPG_ANCHORED = 1ull << 30;

struct BpgLayout {
  int W, E, ncls, nranges, nctr;
  bool uniform, anchored;
  uint32_t nullm;
  int o_first, o_last, o_amap, o_cls, o_exc, o_rng, o_ctr;
};

LP_HD BpgLayout bpg_layout(const uint64_t* P) {
  const uint64_t h = P[0];
  BpgLayout L;
  L.W = (int)(h & 0xFF);
  L.E = (int)((h >> 8) & 0xFFF);
  L.ncls = (int)((h >> 20) & 0x3FF);
  L.anchored = (h & BPG_ANCHORED) != 0;
  L.uniform = (h & BPG_UNIFORM) != 0;
  L.nullm = (uint32_t)(h >> 32) & 0xFFFFFFu;
  L.nranges = (int)(P[1] & 0xFFFFFFFFu);
  L.o_first = 2 + 6 * L.W;
  L.o_last = 2 + 30 * L.W;
  L.o_amap = 2 + 54 * L.W;
  L.o_cls = L.o_amap + 32;
  L.o_exc = L.o_cls + L.ncls * L.W;
  L.o_rng = L.o_exc + L.E * (L.W + 1);
  L.nctr = (int)((h >> 57) & 7);
  L.o_ctr = L.o_rng + L.nranges;
  return L;
}

// one counted position's step (youngest-thread count, see the top): `Fx` = the edges into p this
// step (first set included) in bit b of word `fw`; `s` = p active before the step; returns the
// updated word and advances `cnt` (entry -> 1, stay -> +1, saturating at the bound)
LP_HD uint64_t bpg_ctr_step(uint64_t fw, int b, bool s, uint32_t bound, uint32_t& cnt) {
  const bool entry = (fw >> b) & 1ull;
  const bool stay = s && cnt < bound;
  cnt = entry ? 1u : (cnt < bound ? cnt + 1u : bound);
  return fw | ((uint64_t)stay << b);
}
LP_HD int bpg_words(const uint64_t* P) { return (int)(P[1] >> 32); }

// byte-level next kind (the MFMA NFA engine's 15 contexts, nfa_mfma.hip): 2 word, 3 other,
// 4 UTF-8 continuation
LP_HD int byte_kind(int c) {
  const bool w = (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '_';
  return w ? 2 : (c >= 0x80 && c <= 0xBF) ? 4 : 3;
}

// code-point next kinds (jregex.h): N_EOS 0, N_FT 1, N_W 2, N_N 3, N_T 5; prev kinds P_W 1, P_N 2, P_T 3
LP_HD int ascii_kind(int c) {
  const bool w = (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '_';
  return w ? 2 : (c == '\r' || c == '\n') ? 5 : 3;
}
LP_HD int prev_of(int nk) { return nk == 2 ? 1 : nk == 5 ? 3 : 2; }

// class and next kind of a non-ASCII code point: binary search of the range table
LP_HD int bpg_cp_class(const uint64_t* __restrict__ rg, int nr, uint32_t cp, int* kind) {
  int lo = 0, hi = nr - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if ((uint32_t)(rg[mid] & 0x1FFFFFu) <= cp) lo = mid; else hi = mid - 1;
  }
  const uint64_t e = rg[lo];
  const int kd = (int)((e >> 37) & 3);
  *kind = kd == 1 ? 2 : kd == 2 ? 5 : 3;
  return (int)((e >> 21) & 0xFFFF);
}

// the UTF-8 code point whose lead byte is c, with its continuation bytes b1..b3 (lenient)
LP_HD uint32_t utf8_cp(int c, int b1, int b2, int b3) {
  if (c >= 0xF0) return ((uint32_t)(c & 7) << 18) | ((uint32_t)(b1 & 0x3F) << 12) | ((uint32_t)(b2 & 0x3F) << 6) | (uint32_t)(b3 & 0x3F);
  if (c >= 0xE0) return ((uint32_t)(c & 15) << 12) | ((uint32_t)(b1 & 0x3F) << 6) | (uint32_t)(b2 & 0x3F);
  return ((uint32_t)(c & 31) << 6) | (uint32_t)(b1 & 0x3F);
}

// per-character operands of byte t of the line: class (-1: a continuation byte, skipped) and kind
LP_HD int bpg_char(const uint64_t* __restrict__ P, const BpgLayout& L, const uint8_t* s, int n, int t, int* kind) {
  const int c = s[t];
  if (c < 0x80) { *kind = ascii_kind(c); return reinterpret_cast<const uint16_t*>(P + L.o_amap)[c]; }
  if (c < 0xC0) { *kind = 3; return -1; }
  const int b1 = t + 1 < n ? s[t + 1] : 0x80, b2 = t + 2 < n ? s[t + 2] : 0x80, b3 = t + 3 < n ? s[t + 3] : 0x80;
  return bpg_cp_class(P + L.o_rng, L.nranges, utf8_cp(c, b1, b2, b3), kind);
}

template <int W>
LP_HD bool bpg_find_w(const uint64_t* __restrict__ P, const uint8_t* __restrict__ s, int n) {
  const BpgLayout L = bpg_layout(P);
  const uint64_t* q = P + 2;
  uint64_t shm[W], selfm[W], src[W], R[W], lo[W], hi[W], S[W];
  const uint64_t* first = P + L.o_first;
  const uint64_t* last = P + L.o_last;
  const uint64_t* cls = P + L.o_cls;
  const uint64_t* exc = P + L.o_exc;
  for (int w = 0; w < W; ++w) {
    shm[w] = q[w];
    selfm[w] = q[W + w];
    src[w] = q[2 * W + w];
    R[w] = q[3 * W + w];
    lo[w] = q[4 * W + w];
    hi[w] = q[5 * W + w];
    S[w] = 0;
  }
  const int ftl = final_term_len(s, n);
  const int ft = ftl ? n - ftl : -1;
  int prevk = 0;  // P_BOS
  uint32_t cnt[BPG_CTR_MAX] = {0, 0, 0, 0};
  for (int t = 0;; ++t) {
    int nk = 0, k = 0;                          // N_EOS at end of line
    if (t < n) {
      k = bpg_char(P, L, s, n, t, &nk);
      if (k < 0) continue;                      // inside a code point
    }
    // accept before this character (and before a final line terminator)
    for (int pass = (t == ft) ? 0 : 1; pass < 2; ++pass) {
      const int actx = prevk * 6 + (pass == 0 ? 1 : nk);
      if ((L.nullm >> actx) & 1u) return true;
      const uint64_t* Lm = last + (L.uniform ? 0 : actx * W);
      uint64_t any = 0;
      for (int w = 0; w < W; ++w) any |= S[w] & Lm[w];
      if (any) return true;
    }
    if (t >= n) return false;
    const int ctx = prevk * 6 + nk;
    uint64_t F[W];
    uint64_t carry = 0, borrow = 0;
    for (int w = 0; w < W; ++w) {
      const uint64_t x = S[w] & shm[w];
      F[w] = (x << 1) | carry | (S[w] & selfm[w]);
      carry = x >> 63;
      // spread fields: d = (S & src | hi) - lo (multi-word borrow); targets above the lowest
      // active source of every field = R & ~(d ^ (S & src | hi))
      const uint64_t df = (S[w] & src[w]) | hi[w];
      const uint64_t u = df - lo[w];
      const uint64_t b1 = df < lo[w] ? 1ull : 0ull;
      const uint64_t d = u - borrow;
      const uint64_t b2 = u < borrow ? 1ull : 0ull;
      borrow = b1 | b2;
      F[w] |= R[w] & ~(d ^ df);
    }
    for (int e = 0; e < L.E; ++e) {               // exceptions: (source, condition, targets)
      const uint64_t* x = exc + (size_t)e * (W + 1);
      const int p = (int)(x[0] & 0xFFFF);
      const uint32_t cond = (uint32_t)(x[0] >> 16) & 0xFFFFFFu;
      if (((S[p >> 6] >> (p & 63)) & 1ull) && ((cond >> ctx) & 1u))
        for (int w = 0; w < W; ++w) F[w] |= x[1 + w];
    }
    const uint64_t* C = cls + (size_t)k * W;
    const uint64_t* Fi = first + (L.uniform ? 0 : ctx * W);
    for (int w = 0; w < W; ++w) F[w] |= Fi[w];
    for (int c = 0; c < L.nctr; ++c) {            // counted positions
      const uint64_t e = P[L.o_ctr + c];
      const int p = (int)(e & 0xFFFF);
      F[p >> 6] = bpg_ctr_step(F[p >> 6], p & 63, (S[p >> 6] >> (p & 63)) & 1ull, (uint32_t)(e >> 16), cnt[c]);
    }
    uint64_t alive = 0;
    for (int w = 0; w < W; ++w) {
      S[w] = F[w] & C[w];
      alive |= S[w];
    }
    if (L.anchored && !alive) return false;  // first set only at the line start: nothing can match
    prevk = prev_of(nk);
  }
}

#if defined(__HIP__)
__device__ __forceinline__ int blk_byte(const uint4& v, int j) {   // byte j (0..15) of a 16-byte block
  const uint32_t w = (j < 4) ? v.x : (j < 8) ? v.y : (j < 12) ? v.z : v.w;
  return (int)((w >> (8 * (j & 3))) & 0xFFu);
}
// byte j (0..31) of the 32-byte window cur:nxt
__device__ __forceinline__ int win_byte(const uint4& cur, const uint4& nxt, int j) {
  return j < 16 ? blk_byte(cur, j) : blk_byte(nxt, j - 16);
}
// class (-1: continuation byte) and next kind of the character whose first byte is window byte j
// (text position t of a line of n bytes)
__device__ __forceinline__ int bpg_char_win(const uint64_t* __restrict__ P, const BpgLayout& L, const uint4& cur,
                                            const uint4& nxt, int j, int t, int n, int* kind) {
  const int c = win_byte(cur, nxt, j);
  if (c < 0x80) { *kind = ascii_kind(c); return reinterpret_cast<const uint16_t*>(P + L.o_amap)[c]; }
  if (c < 0xC0) { *kind = 3; return -1; }
  // non-ASCII (rare in logs): decode from the window, binary-search the range table
  const int b1 = t + 1 < n ? win_byte(cur, nxt, j + 1) : 0x80;
  const int b2 = t + 2 < n ? win_byte(cur, nxt, j + 2) : 0x80;
  const int b3 = t + 3 < n ? win_byte(cur, nxt, j + 3) : 0x80;
  return bpg_cp_class(P + L.o_rng, L.nranges, utf8_cp(c, b1, b2, b3), kind);
}

// Device walk of one program, one lane per line (W <= BPG_LANE_MAX_W; kernels in bpg.hip, one
// instantiation per width so each kernel's registers are sized for its own W): the line's bytes
// come from 16-byte ALIGNED vector loads one block ahead (a byte load per step would put a memory
// round trip on the dependency chain), the structural masks live in registers, class / first /
// last / exception rows are read through P -- a global pointer for candidate verification, an LDS
// copy for the all-lines scan.
template <int W>
__device__ __forceinline__ bool bpg_find_dev(const uint64_t* __restrict__ P, const uint8_t* __restrict__ s, int n) {
  const BpgLayout L = bpg_layout(P);
  const uint64_t* q = P + 2;
  uint64_t shm[W], selfm[W], src[W], R[W], lo[W], hi[W], f0[W], l0[W], S[W];
  const uint64_t* first = P + L.o_first;
  const uint64_t* last = P + L.o_last;
  const uint64_t* cls = P + L.o_cls;
  const uint64_t* exc = P + L.o_exc;
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
  const bool uniform = L.uniform;
  const uint32_t nullm = L.nullm;
  const int ftl = final_term_len(s, n);
  const int ft = ftl ? n - ftl : -1;
  int prevk = 0;  // P_BOS
  const int nctr = L.nctr;
  int cpos[BPG_CTR_MAX];
  uint32_t cbound[BPG_CTR_MAX], cnt[BPG_CTR_MAX];
  uint64_t cmk[W];                     // the counted positions' bits, per word
#pragma unroll
  for (int w = 0; w < W; ++w) cmk[w] = 0;
  // the first BPG_EXC_REG exception headers (source | condition) in registers: a per-character load
  // of each header sat on the state chain (a handful of candidates per request: the kernel's time
  // IS one walk's chain)
  const int E = L.E;
  uint64_t eh[BPG_EXC_REG];
#pragma unroll
  for (int e = 0; e < BPG_EXC_REG; ++e) eh[e] = e < E ? exc[(size_t)e * (W + 1)] : 0ull;
#pragma unroll
  for (int c = 0; c < BPG_CTR_MAX; ++c) {
    const uint64_t e = c < nctr ? P[L.o_ctr + c] : 0ull;
    cpos[c] = (int)(e & 0xFFFF);
    cbound[c] = (uint32_t)(e >> 16);
    cnt[c] = 0;
#pragma unroll
    for (int w = 0; w < W; ++w)
      if (c < nctr && w == (cpos[c] >> 6)) cmk[w] |= 1ull << (cpos[c] & 63);
  }
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
      // PF characters at a time: their class rows depend on the text only, not on the state, so
      // all PF rows are loaded before the first state update (one load latency per PF bytes
      // instead of two dependent loads -- class map, then row -- on every byte's chain)
      constexpr int PF = W <= 4 ? 4 : 2;     // rows in flight (registers: PF x W words)
      // narrow programs also prefetch the context-dependent first / last rows of the PF
      // characters (their contexts follow from the text alone)
      constexpr bool PFX = W <= 2;
      for (int jb = j0; jb < j1; jb += PF) {
        uint64_t Cr[PF][W], Fr[PFX ? PF : 1][W], Lr[PFX ? PF : 1][W];
        int kq[PF], nkq[PF];
        int pk = prevk;
#pragma unroll
        for (int qq = 0; qq < PF; ++qq) {
          const int j = jb + qq < 15 ? jb + qq : 15;
          kq[qq] = bpg_char_win(P, L, cur, nxt, j, t0 + j, n, &nkq[qq]);
          const uint64_t* row = cls + (size_t)(kq[qq] < 0 ? 0 : kq[qq]) * W;
#pragma unroll
          for (int w = 0; w < W; ++w) Cr[qq][w] = row[w];
          if constexpr (PFX) {
            const int cx = pk * 6 + nkq[qq];
            const uint64_t* fr = uniform ? first : first + cx * W;
            const uint64_t* lr = uniform ? last : last + cx * W;
#pragma unroll
            for (int w = 0; w < W; ++w) {
              Fr[qq][w] = fr[w];
              Lr[qq][w] = lr[w];
            }
            if (kq[qq] >= 0 && jb + qq < j1) pk = prev_of(nkq[qq]);
          }
        }
#pragma unroll
        for (int qq = 0; qq < PF; ++qq) {
          if (jb + qq >= j1) break;
          if (kq[qq] < 0) continue;             // continuation byte: inside a code point
          const int t = t0 + jb + qq;
          const int nk = nkq[qq];
          if (t == ft) {
            LP_BPG_ACCEPT(prevk * 6 + 1, hit);
            if (hit) return true;
          }
          if constexpr (PFX) {
            uint64_t any = 0;
#pragma unroll
            for (int w = 0; w < W; ++w) any |= S[w] & Lr[qq][w];
            if (((nullm >> (prevk * 6 + nk)) & 1u) || any) return true;
          } else {
            LP_BPG_ACCEPT(prevk * 6 + nk, hit);
            if (hit) return true;
          }
          const int ctx = prevk * 6 + nk;
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
#pragma unroll
          for (int e = 0; e < BPG_EXC_REG; ++e) {   // exceptions: headers in registers, the
            if (e >= E) break;                     // targets loaded only when one fires (rare)
            const uint64_t h = eh[e];
            const int p = (int)(h & 0xFFFF);
            uint64_t sw = 0;
#pragma unroll
            for (int w = 0; w < W; ++w) sw = (w == (p >> 6)) ? S[w] : sw;
            if (((sw >> (p & 63)) & 1ull) && (((uint32_t)(h >> 16) >> ctx) & 1u)) {
              const uint64_t* x = exc + (size_t)e * (W + 1);
#pragma unroll
              for (int w = 0; w < W; ++w) F[w] |= x[1 + w];
            }
          }
          for (int e = BPG_EXC_REG; e < E; ++e) {
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
          if constexpr (PFX) {
#pragma unroll
            for (int w = 0; w < W; ++w) F[w] |= Fr[qq][w];
          } else if (uniform) {
#pragma unroll
            for (int w = 0; w < W; ++w) F[w] |= f0[w];
          } else {
            const uint64_t* Fi = first + ctx * W;
#pragma unroll
            for (int w = 0; w < W; ++w) F[w] |= Fi[w];
          }
          uint64_t act = 0;                        // a counted position alive or entered: a dead
#pragma unroll                                     // one's count is never read (restarts at entry)
          for (int w = 0; w < W; ++w) act |= (F[w] | S[w]) & cmk[w];
#pragma unroll
          for (int c = 0; c < BPG_CTR_MAX; ++c) {  // counted positions (rare: skipped as a whole)
            if (c >= nctr || !act) break;
            const int pw = cpos[c] >> 6;
            uint64_t fw = 0, sw = 0;
#pragma unroll
            for (int w = 0; w < W; ++w) {
              fw = (w == pw) ? F[w] : fw;
              sw = (w == pw) ? S[w] : sw;
            }
            fw = bpg_ctr_step(fw, cpos[c] & 63, (sw >> (cpos[c] & 63)) & 1ull, cbound[c], cnt[c]);
#pragma unroll
            for (int w = 0; w < W; ++w) F[w] = (w == pw) ? fw : F[w];
          }
          uint64_t alive = 0;
#pragma unroll
          for (int w = 0; w < W; ++w) {
            S[w] = F[w] & Cr[qq][w];
            alive |= S[w];
          }
          if (L.anchored && !alive) return false;
          prevk = prev_of(nk);
        }
      }
      cur = nxt;
    }
  }
  LP_BPG_ACCEPT(prevk * 6 + 0, hit);  // end of line (N_EOS)
  return hit;
#undef LP_BPG_ACCEPT
}

// class of a non-ASCII code point through the range table at P[o] (bpg_cp_class over any pointer)
template <typename PT>
__device__ __forceinline__ int bpg_cp_class_p(PT P, int o, int nr, uint32_t cp, int* kind) {
  int lo = 0, hi = nr - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if ((uint32_t)(P[o + mid] & 0x1FFFFFu) <= cp) lo = mid; else hi = mid - 1;
  }
  const uint64_t e = P[o + lo];
  const int kd = (int)((e >> 37) & 3);
  *kind = kd == 1 ? 2 : kd == 2 ? 5 : 3;
  return (int)((e >> 21) & 0xFFFF);
}

// Lean one-lane walk of a ONE-WORD program (<= 64 positions -- every program of the realistic
// library since counted positions), same find() semantics as bpg_find_dev / bpg_find_w.
// bpg_find_dev<1> above compiles to ~150 instructions per character (every optional feature an
// exec-mask branch, SGPR spills) and a request's candidate walk ran at 340-440 ns per byte
// (tools/bpg_probe.py). Here the common character is the structural chain (~25 VALU ops on 64-bit
// masks) plus operands that depend on the TEXT only -- class row, and the first / last rows of the
// character's boundary context (a uniform program stores all 24 identical rows, so no branch on
// uniformity) -- loaded four characters ahead. The optional features (exception edges, counted
// positions, a final line terminator, multi-byte characters) run behind WAVE-uniform ballots: a
// wave none of whose lanes needs one skips it with a scalar branch. `valid` false: the lane takes
// part in the ballots and walks nothing (P must still point at readable program words).
// PT: pointer to the program's words -- LDS (ds_read) when the pool is staged, else global.
template <typename PT>
__device__ __forceinline__ bool bpg_walk1(PT P, const uint8_t* __restrict__ s, int n, bool valid, int prevk0 = 0,
                                          int inj_end = 0x7FFFFFFF) {
  // (split walks: `prevk0` = previous kind before s[0] -- a walk of a line's second part; `inj_end`:
  // no thread starts at or after that position, and the walk stops once no thread is alive past it
  // -- the first part. The two parts' results OR to the whole line's: every thread starts in one.)
  const uint64_t h = P[0];
  const int E = valid ? (int)((h >> 8) & 0xFFF) : 0;
  const int ncls = (int)((h >> 20) & 0x3FF);
  const uint32_t nullm = valid ? (uint32_t)(h >> 32) & 0xFFFFFFu : 0u;
  const int nranges = (int)(P[1] & 0xFFFFFFFFu);
  const int nctr = valid ? (int)((h >> 57) & 7) : 0;
  if (!valid) n = 0;
  constexpr int oF = 8, oL = 32, oA = 56, oC = 88;          // bpg_layout for W = 1
  const int oE = oC + ncls, oR = oE + 2 * E, oT = oR + nranges;
  const uint64_t shm = P[2], selfm = P[3], src = P[4], R = P[5], lo = P[6], hi = P[7];
  // exception edges / counted positions: the first BPG_EXC_REG / all BPG_CTR_MAX in registers;
  // mexc / mctr = the wave's largest counts (uniform trip counts, per-lane predicates)
  uint64_t eh[BPG_EXC_REG], et[BPG_EXC_REG], ebit[BPG_EXC_REG];
  int mexc = 0, mctr = 0;
#pragma unroll
  for (int e = 0; e < BPG_EXC_REG; ++e) {
    eh[e] = e < E ? P[oE + 2 * e] : 0ull;                  // (0 past E: no source bit, no condition)
    et[e] = e < E ? P[oE + 2 * e + 1] : 0ull;
    ebit[e] = e < E ? 1ull << (eh[e] & 63) : 0ull;
    mexc = __ballot(E > e) ? e + 1 : mexc;
  }
  const bool wexc_more = __ballot(E > BPG_EXC_REG) != 0;
  uint64_t cbit[BPG_CTR_MAX];
  uint32_t cbound[BPG_CTR_MAX], cnt[BPG_CTR_MAX];
#pragma unroll
  for (int c = 0; c < BPG_CTR_MAX; ++c) {
    const uint64_t e = c < nctr ? P[oT + c] : 0ull;
    cbit[c] = c < nctr ? 1ull << (e & 63) : 0ull;          // (no bit past nctr: never enters, stays)
    cbound[c] = (uint32_t)(e >> 16);
    cnt[c] = 0;
    mctr = __ballot(nctr > c) ? c + 1 : mctr;
  }
  const int ftl = n > 0 ? final_term_len(s, n) : 0;
  const int ft = ftl ? n - ftl : -1;
  const bool wft = __ballot(ftl > 0) != 0;
  // simple wave: every lane's program has context-free first / last sets, no nullable context and no
  // exception edge -- its characters need no boundary context (kind, previous kind) at all
  const bool uni = (h & BPG_UNIFORM) != 0;
  const bool wsimple = __ballot(valid && !(uni && nullm == 0u && E == 0)) == 0;
  const uint64_t f0 = P[oF], l0 = P[oL];
  uint64_t S = 0, acc = 0, Sft = 0;
  uint32_t nullhit = 0;
  int ftctx = 0;
  int prevk = prevk0;                                      // P_BOS, or the split point's
  const int sh = (int)((uintptr_t)s & 15);
  const uint4* blk = reinterpret_cast<const uint4*>(s - sh);
  uint4 cur = n > 0 ? blk[0] : make_uint4(0, 0, 0, 0);
  for (int b0 = 0;; b0 += 16) {                            // wave-uniform (the break below)
    const bool live = b0 < sh + n;
    const uint4 nxt = live ? blk[(b0 >> 4) + 1] : make_uint4(0, 0, 0, 0);   // (texts are padded)
    const bool wmb = __ballot(live && ((cur.x | cur.y | cur.z | cur.w) & 0x80808080u) != 0) != 0;
    // text-only operands of the block's 16 characters, all loads in flight before the chain
    uint64_t Cq[16], Fq[16], Lq[16];
    int ctxq[16];
    uint32_t onm = 0;
    int pk = prevk;
    if (wsimple && !wmb) {                                 // ASCII block, context-free programs
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int t = b0 + j - sh;
        const int c = blk_byte(cur, j);
        const bool on = t >= 0 && t < n;
        const int k = (int)((P[oA + (c >> 2)] >> (16 * (c & 3))) & 0xFFFFu);
        ctxq[j] = 0;
        onm |= on ? 1u << j : 0u;
        Cq[j] = on ? P[oC + k] : 0ull;
        Fq[j] = f0;
        Lq[j] = l0;
      }
    } else if (!wmb) {                                     // ASCII block
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int t = b0 + j - sh;
        const int c = blk_byte(cur, j);
        const bool on = t >= 0 && t < n;
        const int k = (int)((P[oA + (c >> 2)] >> (16 * (c & 3))) & 0xFFFFu);
        const int nk = ascii_kind(c);
        const int ctx = pk * 6 + nk;
        ctxq[j] = ctx;
        onm |= on ? 1u << j : 0u;
        Cq[j] = on ? P[oC + k] : 0ull;
        Fq[j] = t < inj_end ? P[oF + ctx] : 0ull;
        Lq[j] = P[oL + ctx];
        if (wft && on && t == ft) ftctx = pk * 6 + 1;
        pk = on ? prev_of(nk) : pk;
      }
    } else {                                               // multi-byte characters in some lane
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int t = b0 + j - sh;
        const int c = blk_byte(cur, j);
        bool on = t >= 0 && t < n;
        int k = 0, nk = 3;
        if (c < 0x80) {
          k = (int)((P[oA + (c >> 2)] >> (16 * (c & 3))) & 0xFFFFu);
          nk = ascii_kind(c);
        } else if (c < 0xC0) {
          on = false;                                      // continuation byte: inside a code point
        } else if (on) {
          const int b1 = t + 1 < n ? win_byte(cur, nxt, j + 1) : 0x80;
          const int b2 = t + 2 < n ? win_byte(cur, nxt, j + 2) : 0x80;
          const int b3 = t + 3 < n ? win_byte(cur, nxt, j + 3) : 0x80;
          k = bpg_cp_class_p(P, oR, nranges, utf8_cp(c, b1, b2, b3), &nk);
        }
        const int ctx = pk * 6 + nk;
        ctxq[j] = ctx;
        onm |= on ? 1u << j : 0u;
        Cq[j] = on ? P[oC + k] : 0ull;
        Fq[j] = t < inj_end ? P[oF + ctx] : 0ull;
        Lq[j] = P[oL + ctx];
        if (wft && on && t == ft) ftctx = pk * 6 + 1;
        pk = on ? prev_of(nk) : pk;
      }
    }
    // the state chain of the 16 characters, specialised by what the wave needs (a scalar branch per
    // block): CTX -- boundary contexts (context-dependent first / last rows, nullable contexts,
    // exception conditions), EXC -- exception edges, CTR -- counted positions
#define LP_W1_CHAIN(CTX, EXC, CTR)                                                                  \
  _Pragma("unroll") for (int j = 0; j < 16; ++j) {                                                \
    const bool on = (onm >> j) & 1u;                                                               \
    const int ctx = ctxq[j];                                                                       \
    const uint64_t keep = on ? 0ull : ~0ull;             /* off the line: S stays (no branch) */    \
    acc |= S & (CTX ? Lq[j] : l0) & ~keep;               /* accept before this character */        \
    if (CTX) nullhit |= on ? (nullm >> ctx) & 1u : 0u;                                             \
    if (wft) Sft = (on && b0 + j - sh == ft) ? S : Sft;                                            \
    uint64_t F = ((S & shm) << 1) | (S & selfm) | (CTX ? Fq[j] : (b0 + j - sh < inj_end ? f0 : 0ull)); \
    const uint64_t df = (S & src) | hi;                                                            \
    F |= R & ~((df - lo) ^ df);                          /* spread fields: one word, no borrow */   \
    if (EXC) {                                                                                     \
      _Pragma("unroll") for (int e = 0; e < BPG_EXC_REG; ++e) {                                    \
        if (e >= mexc) break;                                                                      \
        const uint64_t hh = eh[e];                                                                 \
        const bool fire = ((S & ebit[e]) != 0ull) & (((((uint32_t)(hh >> 16) & 0xFFFFFFu) >> ctx) & 1u) != 0u); \
        F |= fire ? et[e] : 0ull;                                                                  \
      }                                                                                            \
      if (wexc_more)                                                                               \
        for (int e = BPG_EXC_REG; e < E; ++e) {                                                    \
          const uint64_t hh = P[oE + 2 * e];                                                       \
          if (((S >> (hh & 63)) & 1ull) && ((((uint32_t)(hh >> 16) & 0xFFFFFFu) >> ctx) & 1u)) F |= P[oE + 2 * e + 1]; \
        }                                                                                          \
    }                                                                                              \
    if (CTR) {                                           /* bpg_ctr_step; a dead position's count */ \
      _Pragma("unroll") for (int c = 0; c < BPG_CTR_MAX; ++c) { /* is never read: every count   */ \
        if (c >= mctr) break;                            /* advances unconditionally          */ \
        const uint64_t cb = cbit[c];                                                               \
        const bool lt = cnt[c] < cbound[c];                                                        \
        const bool entry = (F & cb) != 0ull;                                                       \
        F |= (lt && (S & cb) != 0ull) ? cb : 0ull;                                                 \
        cnt[c] = on ? (entry ? 1u : cnt[c] + (lt ? 1u : 0u)) : cnt[c];                             \
      }                                                                                            \
    }                                                                                              \
    S = (F & Cq[j]) | (S & keep);                        /* Cq = 0 off the line */                 \
  }
    if (wsimple && !wmb) {
      if (mctr) { LP_W1_CHAIN(false, false, true) } else { LP_W1_CHAIN(false, false, false) }
    } else if (mexc) {
      if (mctr) { LP_W1_CHAIN(true, true, true) } else { LP_W1_CHAIN(true, true, false) }
    } else {
      if (mctr) { LP_W1_CHAIN(true, false, true) } else { LP_W1_CHAIN(true, false, false) }
    }
#undef LP_W1_CHAIN
    prevk = pk;
    cur = nxt;
    const bool fin = !live || acc != 0 || nullhit != 0 || b0 + 16 >= sh + n ||
                     (b0 + 16 - sh >= inj_end && S == 0ull);   // a first part with no thread left
    if (__ballot(!fin) == 0) break;
  }
  if (valid && wsimple) {                                  // (every context row is row 0)
    acc |= (S | Sft) & l0;
  } else if (valid) {
    const int ce = prevk * 6 + 0;                          // end of line (N_EOS)
    acc |= S & P[oL + ce];
    nullhit |= (nullm >> ce) & 1u;
    if (ft >= 0) {
      acc |= Sft & P[oL + ftctx];
      nullhit |= (nullm >> ftctx) & 1u;
    }
  }
  return valid && (acc != 0 || nullhit != 0);
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
    case 8: return bpg_find_w<8>(P, s, n);
    case 12: return bpg_find_w<12>(P, s, n);
    case 16: return bpg_find_w<16>(P, s, n);
    case 24: return bpg_find_w<24>(P, s, n);
    default: return bpg_find_w<32>(P, s, n);
  }
}

}  // namespace lp
