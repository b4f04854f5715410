// NFA simulation as a state-transition GEMM on the gfx950 matrix cores.
//
// A "group" packs up to 8 regexes (Glushkov NFAs, jregex.h) into M = 64 positions. A wave advances
// 16 lines one byte per step; the active-state set of every line is the column of a 64 x 16
// matrix S^T and
//
//   S'^T = ( F^T . S^T  > 0   OR  first[ctx] ) AND cls[byte]         (ctx = boundary context)
//
// with F^T . S^T on v_mfma_f32_16x16x32_bf16 (0/1 operands, integer counts <= 64: exact in
// bf16/f32): 4 output tiles x 2 k-steps = 8 MFMAs per byte per 16 lines per edge class (edges
// gated by a boundary assertion, e.g. "foo\bbar", form up to 2 extra classes whose S^T column is
// zeroed for lines where the gate fails).
//
// Lane-resident states. With the transition matrix as the A operand and the states as B, the
// accumulator of lane (line r, group g) holds out-states {16n + 4g + i} (n, i < 4) of line r --
// and the next step's B operand of that lane needs in-state k-slots {32 s2 + 8 g + j}. Numbering
// the k-slots so that slot 32 s2 + 8 g + 4 h + i IS state 16 (2 s2 + h) + 4 g + i (a permutation
// baked into the A tiles at kernel start), every lane finds its next B operand in its own
// accumulators: no ballots, no LDS round trip, no cross-lane traffic per byte. (The first
// version transposed through 16 ballots + LDS per byte: 1 MFMA per 41 VALU, profiles/r1_v4.)
// Per-lane 16-bit views of the class / first / last masks come from small LDS tables.
//
// Used for (a) the context-feature A/B engine (the 4 ContextAnalysisService regexes = one
// 61-position group, ContextAnalysisService.java:27-34) and (b) regexes whose DFA exceeds
// engine.dfa-max-states. Accept checks follow Matcher.find(): before every byte (context with
// the next byte), before a final line terminator and at end of line (jregex.h N_FT / N_EOS).
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#include "lp_api.h"
#include "lp_core.h"

namespace lp {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// group table layout (uint64 words); see log_parser_amd/models/nfa.py
constexpr int G_CLS = 0, G_FIRST = 256, G_LAST = 271, G_REGMASK = 286, G_F = 294, G_META = 486, G_CMASK = 487,
              G_NULL = 488, G_REGID = 496, G_STRIDE = 512;
constexpr int NFA_WAVES = 4;
constexpr int MAX_NFA_REGS = 8;   // regexes per group (models/nfa.py MAX_REGS)

LP_HD uint32_t nfa_accept(const uint64_t* tab, uint64_t S, int ctx, int nreg) {
  const uint64_t hit = S & tab[G_LAST + ctx];
  uint32_t acc = 0;
  for (int q = 0; q < nreg; ++q)
    if ((hit & tab[G_REGMASK + q]) || ((tab[G_NULL + q] >> ctx) & 1)) acc |= 1u << q;
  return acc;
}

// lane-local 16-bit view of a 64-bit state mask: bit 4n + i <- state 16n + 4g + i
LP_HD uint32_t lane16(uint64_t m, int g) {
  uint32_t r = 0;
#pragma unroll
  for (int n = 0; n < 4; ++n) r |= (uint32_t)((m >> (16 * n + 4 * g)) & 0xF) << (4 * n);
  return r;
}

template <int NCLS>
__global__ __launch_bounds__(64 * NFA_WAVES) void k_nfa_mfma(const uint64_t* __restrict__ groups,
                                                             const int32_t* __restrict__ group_list,
                                                             const int32_t* __restrict__ lines, int64_t nsel,
                                                             const uint8_t* __restrict__ text,
                                                             const int64_t* __restrict__ line_start,
                                                             const int32_t* __restrict__ line_len,
                                                             uint8_t* __restrict__ feat, int64_t* hits, int64_t cap,
                                                             unsigned long long* count) {
  __shared__ uint64_t tab[G_STRIDE];
  __shared__ uint16_t s_cls[4][256];      // lane16(cls[c], g)
  __shared__ uint16_t s_first[4][16], s_last[4][16];
  __shared__ uint32_t s_null[16];         // regexes accepting the empty match in context ctx
  __shared__ uint2 s_nib[16];             // 4 state bits -> 4 bf16 (0 / 1.0)
  const uint64_t* G = groups + (size_t)group_list[blockIdx.y] * G_STRIDE;
  for (int i = threadIdx.x; i < G_STRIDE; i += blockDim.x) tab[i] = G[i];
  __syncthreads();
  const int nreg = (int)((tab[G_META] >> 8) & 0xFF);
  for (int i = threadIdx.x; i < 4 * 256; i += blockDim.x) s_cls[i >> 8][i & 255] = (uint16_t)lane16(tab[G_CLS + (i & 255)], i >> 8);
  for (int i = threadIdx.x; i < 4 * 16; i += blockDim.x) {
    const int g = i >> 4, x = i & 15;
    s_first[g][x] = x < 15 ? (uint16_t)lane16(tab[G_FIRST + x], g) : 0;
    s_last[g][x] = x < 15 ? (uint16_t)lane16(tab[G_LAST + x], g) : 0;
  }
  if (threadIdx.x < 16) {
    uint32_t nb = 0;
    for (int q = 0; q < nreg; ++q)
      if (threadIdx.x < 15 && ((tab[G_NULL + q] >> threadIdx.x) & 1)) nb |= 1u << q;
    s_null[threadIdx.x] = nb;
    const uint32_t x = threadIdx.x;
    s_nib[x] = make_uint2(((x & 1) ? 0x3F80u : 0u) | ((x & 2) ? 0x3F800000u : 0u),
                          ((x & 4) ? 0x3F80u : 0u) | ((x & 8) ? 0x3F800000u : 0u));
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t row0 = ((int64_t)blockIdx.x * NFA_WAVES + wave) * 16;
  if (row0 >= nsel) return;  // wave-uniform
  const int r = lane & 15, grp = lane >> 4;
  const int64_t ri = row0 + r;
  const bool valid = ri < nsel;
  const int32_t line = valid ? (lines ? lines[ri] : (int32_t)ri) : 0;
  const uint8_t* s = text + (valid ? line_start[line] : 0);
  const int len = valid ? line_len[line] : 0;
  const int ftl = valid ? final_term_len(s, len) : 0;
  const int ft = ftl ? len - ftl : -1;
  const uint32_t cm1 = (uint32_t)(tab[G_CMASK] & 0xFFFF), cm2 = (uint32_t)((tab[G_CMASK] >> 16) & 0xFFFF);

  // A tiles (transition matrix, permuted k-slots): A[k][n][s2], lane (r, grp): row = out-state
  // 16n + r, slot j -> in-state 16 (2 s2 + (j >> 2)) + 4 grp + (j & 3)
  bf16x8 Af[NCLS][4][2];
#pragma unroll
  for (int k = 0; k < NCLS; ++k)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        u16x8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int in = 16 * (2 * s2 + (j >> 2)) + 4 * grp + (j & 3);
          v[j] = ((tab[G_F + 64 * k + in] >> (16 * n + r)) & 1) ? 0x3F80 : 0;
        }
        Af[k][n][s2] = __builtin_bit_cast(bf16x8, v);
      }
  uint32_t regm[MAX_NFA_REGS];
#pragma unroll
  for (int q = 0; q < MAX_NFA_REGS; ++q) regm[q] = q < nreg ? lane16(tab[G_REGMASK + q], grp) : 0;

  int T = len;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) T = max(T, __shfl_xor(T, off, 64));

  // this line's bytes: 16-byte aligned blocks, one block ahead (text is padded)
  const int sh = (int)((uintptr_t)s & 15);
  const uint4* blk = reinterpret_cast<const uint4*>(s - sh);
  uint4 cur = blk[0], nxt = blk[1];
  int bi = 0;

  uint32_t S = 0, accst = 0, acc = 0;
  int prevk = 0;  // P_BOS
  bool done = !valid;
  for (int t = 0; t <= T; ++t) {
    const bool live = t < len;
    const int idx = t + sh;
    if (live && (idx >> 4) != bi) {  // only while inside this line: never read past its padding
      cur = nxt;
      ++bi;
      nxt = blk[bi + 1];
    }
    const int q4 = (idx >> 2) & 3;
    const uint32_t w = q4 == 0 ? cur.x : q4 == 1 ? cur.y : q4 == 2 ? cur.z : cur.w;
    const int c = live ? (int)((w >> (8 * (idx & 3))) & 0xFF) : 0;
    const int nk = live ? byte_kind(c) : 0;  // N_EOS at end of line
    if (!done) {
      if (t == ft) {
        accst |= S & s_last[grp][prevk * 5 + 1];
        acc |= s_null[prevk * 5 + 1];
      }
      accst |= S & s_last[grp][prevk * 5 + nk];
      acc |= s_null[prevk * 5 + nk];
      if (t == len) done = true;
    }
    if (t == T) break;
    const int ctx = prevk * 5 + (live ? nk : 3);
    // B operand = this lane's 16 state bits as bf16 (slots 8 s2 .. 8 s2 + 7)
    bf16x8 B[2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const uint2 lo = s_nib[(S >> (8 * s2)) & 15], hi = s_nib[(S >> (8 * s2 + 4)) & 15];
      B[s2] = __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
    }
    f32x4 D[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) D[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < NCLS; ++k) {
      bf16x8 Bk[2] = {B[0], B[1]};
      if (k > 0) {
        const uint32_t m = k == 1 ? cm1 : cm2;
        if (!((m >> ctx) & 1)) {  // gate fails for this line: its edges of class k do not fire
          Bk[0] = __builtin_bit_cast(bf16x8, (u16x8){0, 0, 0, 0, 0, 0, 0, 0});
          Bk[1] = Bk[0];
        }
      }
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) D[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Af[k][n][s2], Bk[s2], D[n], 0, 0, 0);
    }
    uint32_t act = 0;
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) act |= (D[n][i] > 0.5f ? 1u : 0u) << (4 * n + i);
    const uint32_t ns = (act | s_first[grp][ctx]) & s_cls[grp][c];
    if (live) {
      S = ns;
      prevk = nk == 2 ? 1 : 2;
    }
  }
  // states accepted somewhere on the line -> regexes; OR over the 4 lane groups of the line
#pragma unroll
  for (int q = 0; q < MAX_NFA_REGS; ++q)
    if (accst & regm[q]) acc |= 1u << q;
  acc |= __shfl_xor(acc, 16, 64);
  acc |= __shfl_xor(acc, 32, 64);
  if (grp == 0 && valid) {
    if (feat) {   // context features: bit = context regex id (0..3); one group per launch
      uint32_t f = 0;
      for (int q = 0; q < nreg; ++q)
        if ((acc >> q) & 1) f |= 1u << (tab[G_REGID + q] & 7);
      feat[line] |= (uint8_t)f;
    } else {
      for (int q = 0; q < nreg; ++q)
        if ((acc >> q) & 1) {
          unsigned long long i = atomicAdd(count, 1ull);
          if ((int64_t)i < cap) hits[i] = ((int64_t)tab[G_REGID + q] << 32) | line;
        }
    }
  }
}

void nfa_mfma_dev(const uint64_t* groups, const int32_t* group_list, int ngroups, int ncls, const int32_t* lines,
                  int64_t nsel, const uint8_t* text, const int64_t* line_start, const int32_t* line_len,
                  uint8_t* feat, int64_t* hits, int64_t cap, unsigned long long* count, uint64_t stream) {
  if (nsel <= 0 || ngroups <= 0) return;
  dim3 grid((unsigned)((nsel + 16 * NFA_WAVES - 1) / (16 * NFA_WAVES)), (unsigned)ngroups);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  switch (ncls) {
    case 1: hipLaunchKernelGGL(k_nfa_mfma<1>, grid, dim3(64 * NFA_WAVES), 0, st, groups, group_list, lines, nsel, text,
                               line_start, line_len, feat, hits, cap, count); break;
    case 2: hipLaunchKernelGGL(k_nfa_mfma<2>, grid, dim3(64 * NFA_WAVES), 0, st, groups, group_list, lines, nsel, text,
                               line_start, line_len, feat, hits, cap, count); break;
    default: hipLaunchKernelGGL(k_nfa_mfma<3>, grid, dim3(64 * NFA_WAVES), 0, st, groups, group_list, lines, nsel,
                                text, line_start, line_len, feat, hits, cap, count); break;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e) + " in nfa_mfma");
}

// host twin: the same recurrence on 64-bit bitsets
int64_t nfa_host(const uint64_t* groups, const int32_t* group_list, int ngroups, const int32_t* lines, int64_t nsel,
                 const uint8_t* text, const int64_t* line_start, const int32_t* line_len, uint8_t* feat,
                 int64_t* hits, int64_t cap) {
  int64_t cnt = 0;
  for (int gi = 0; gi < ngroups; ++gi) {
    const uint64_t* tab = groups + (size_t)group_list[gi] * G_STRIDE;
    const int ncls = (int)(tab[G_META] & 0xFF), nreg = (int)((tab[G_META] >> 8) & 0xFF);
    const uint32_t cm1 = (uint32_t)(tab[G_CMASK] & 0xFFFF), cm2 = (uint32_t)((tab[G_CMASK] >> 16) & 0xFFFF);
    for (int64_t ri = 0; ri < nsel; ++ri) {
      const int32_t line = lines ? lines[ri] : (int32_t)ri;
      const uint8_t* s = text + line_start[line];
      const int len = line_len[line];
      const int ftl = final_term_len(s, len);
      const int ft = ftl ? len - ftl : -1;
      uint64_t S = 0;
      int prevk = 0;
      uint32_t acc = 0;
      for (int t = 0; t <= len; ++t) {
        const int nk = t < len ? byte_kind(s[t]) : 0;
        if (t == ft) acc |= nfa_accept(tab, S, prevk * 5 + 1, nreg);
        acc |= nfa_accept(tab, S, prevk * 5 + nk, nreg);
        if (t == len) break;
        const int ctx = prevk * 5 + nk;
        uint64_t fol = 0;
        for (uint64_t m = S; m; m &= m - 1) {
          const int p = __builtin_ctzll(m);
          fol |= tab[G_F + p];
          if (ncls > 1 && ((cm1 >> ctx) & 1)) fol |= tab[G_F + 64 + p];
          if (ncls > 2 && ((cm2 >> ctx) & 1)) fol |= tab[G_F + 128 + p];
        }
        S = (fol | tab[G_FIRST + ctx]) & tab[G_CLS + s[t]];
        prevk = nk == 2 ? 1 : 2;
      }
      if (feat) {
        uint32_t f = 0;
        for (int q = 0; q < nreg; ++q)
          if ((acc >> q) & 1) f |= 1u << (tab[G_REGID + q] & 7);
        feat[line] |= (uint8_t)f;
      } else {
        for (int q = 0; q < nreg; ++q)
          if ((acc >> q) & 1) {
            if (cnt < cap) hits[cnt] = ((int64_t)tab[G_REGID + q] << 32) | line;
            ++cnt;
          }
      }
    }
  }
  return cnt;
}

}  // namespace lp
