// NFA simulation as a state-transition GEMM on the gfx950 matrix cores.
//
// A "group" packs up to 8 regexes (Glushkov NFAs, jregex.h) into M = 64 positions. For a tile of
// 16 lines, the active-state matrix S (16 x 64, 0/1) advances one byte per step:
//
//   S' = ( S . F  > 0   OR  first[ctx] ) AND cls[byte]          (ctx = boundary context, jregex.h)
//
// S . F runs on v_mfma_f32_16x16x32_bf16 (0/1 operands and integer counts <= 64 are exact in
// bf16/f32): 2 k-steps x 4 column tiles = 8 MFMAs per byte per 16 lines, per edge class. Edges
// gated by a boundary assertion (e.g. "foo\bbar") form up to 2 extra classes whose A operand is
// zeroed for rows where the gate fails. The f32 accumulator (col = lane&15, row = 4*(lane>>4)+i)
// is turned back into the row-major bit image the next A operand needs with 16 wave ballots:
// ballot(i, n) holds, for every 16-lane group g, row 4g+i's columns 16n..16n+15.
//
// Used for (a) the always-on context-feature stage (the 4 ContextAnalysisService regexes =
// one 61-position group, ContextAnalysisService.java:27-34) and (b) regexes whose DFA exceeds
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

LP_HD int byte_kind(int c) {  // next-kind of a byte: 2 word, 3 other, 4 UTF-8 continuation
  const bool w = (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '_';
  return w ? 2 : (c >= 0x80 && c <= 0xBF) ? 4 : 3;
}

LP_HD uint32_t nfa_accept(const uint64_t* tab, uint64_t S, int ctx, int nreg) {
  const uint64_t hit = S & tab[G_LAST + ctx];
  uint32_t acc = 0;
  for (int q = 0; q < nreg; ++q)
    if ((hit & tab[G_REGMASK + q]) || ((tab[G_NULL + q] >> ctx) & 1)) acc |= 1u << q;
  return acc;
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
  __shared__ uint64_t scratch[NFA_WAVES][16];
  const uint64_t* G = groups + (size_t)group_list[blockIdx.y] * G_STRIDE;
  for (int i = threadIdx.x; i < G_STRIDE; i += blockDim.x) tab[i] = G[i];
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
  const int nreg = (int)((tab[G_META] >> 8) & 0xFF);
  const uint32_t cm1 = (uint32_t)(tab[G_CMASK] & 0xFFFF), cm2 = (uint32_t)((tab[G_CMASK] >> 16) & 0xFFFF);

  // B operands: B[k][col] = F_class[k] bit col;  lane holds k = 32*s2 + 8*grp + j, col = 16n + r
  bf16x8 Bf[NCLS][2][4];
#pragma unroll
  for (int k = 0; k < NCLS; ++k)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        u16x8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int kk = 32 * s2 + 8 * grp + j;
          v[j] = ((tab[G_F + 64 * k + kk] >> (16 * n + r)) & 1) ? 0x3F80 : 0;
        }
        Bf[k][s2][n] = __builtin_bit_cast(bf16x8, v);
      }

  int T = len;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) T = max(T, __shfl_xor(T, off, 64));

  uint64_t S = 0;
  int prevk = 0;  // P_BOS
  uint32_t acc = 0;
  bool done = !valid;
  for (int t = 0; t <= T; ++t) {
    const bool live = t < len;
    const int c = live ? s[t] : 0;
    const int nk = live ? byte_kind(c) : 0;  // N_EOS at end of line
    if (!done) {
      if (t == ft) acc |= nfa_accept(tab, S, prevk * 5 + 1, nreg);
      acc |= nfa_accept(tab, S, prevk * 5 + nk, nreg);
      if (t == len) done = true;
    }
    if (t == T) break;
    const int ctx = prevk * 5 + (live ? nk : 3);
    // A operand (row r, bits 32*s2 + 8*grp .. +8), per edge class gated by the boundary context
    bf16x8 A[2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const uint32_t byte = (uint32_t)(S >> (32 * s2 + 8 * grp)) & 0xFF;
      u16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = ((byte >> j) & 1) ? 0x3F80 : 0;
      A[s2] = __builtin_bit_cast(bf16x8, v);
    }
    f32x4 C[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) C[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < NCLS; ++k) {
      bf16x8 Ak[2] = {A[0], A[1]};
      if (k > 0) {
        const uint32_t m = k == 1 ? cm1 : cm2;
        if (!((m >> ctx) & 1)) {
          Ak[0] = __builtin_bit_cast(bf16x8, (u16x8){0, 0, 0, 0, 0, 0, 0, 0});
          Ak[1] = Ak[0];
        }
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int n = 0; n < 4; ++n) C[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ak[s2], Bf[k][s2][n], C[n], 0, 0, 0);
    }
    // accumulator (row 4*grp+i, col 16n+r) -> bits, via ballots
    const int info = c | (ctx << 8);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int inf = __shfl(info, 4 * grp + i, 64);
      const uint64_t clsm = tab[G_CLS + (inf & 0xFF)];
      const uint64_t fm = tab[G_FIRST + (inf >> 8)];
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int col = 16 * n + r;
        const bool bit = ((C[n][i] > 0.5f) || ((fm >> col) & 1)) && ((clsm >> col) & 1);
        const uint64_t b = __ballot(bit);
        if (lane == 0) scratch[wave][4 * i + n] = b;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int g2 = r >> 2, i2 = r & 3;
    uint64_t ns = 0;
#pragma unroll
    for (int n = 0; n < 4; ++n) ns |= ((scratch[wave][4 * i2 + n] >> (16 * g2)) & 0xFFFFull) << (16 * n);
    __builtin_amdgcn_wave_barrier();
    if (live) {
      S = ns;
      prevk = nk == 2 ? 1 : 2;
    }
  }
  if (grp == 0 && valid) {
    if (feat) {
      feat[line] = (uint8_t)acc;
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
        feat[line] = (uint8_t)acc;
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
