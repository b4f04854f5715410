// gfx950 kernels of the bit-parallel Glushkov programs (bpg.h, models/bpg.py): the regexes whose
// DFA blows up, verified on prefilter candidate lines or scanned over every line.
//
// Candidate verification (few lines: the slowest walk decides) is one kernel for every program width;
// the all-lines scan (every line: occupancy decides) is one instantiation per width W (words of 64
// positions), launched only for the widths a library has. The DFA kernels next to them
// (k_cand_verify, k_dedupe_verify, k_scan) never carry the BPG walk -- folding it into dfa_run took
// those kernels from ~40 to 130 VGPRs plus 580 B of scratch per lane (3 waves / SIMD).
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#include "lp_api.h"
#include "lp_core.h"

namespace lp {

namespace {

constexpr uint64_t kPadKey = ~0ull;   // lp_post.hip LP_PAD_KEY
constexpr int kScanLines = 256;

inline unsigned nblocks(int64_t n, int t = 256) { return (unsigned)std::max<int64_t>(1, (n + t - 1) / t); }

// candidates of the small path, in place (-1 = no match; k_cand_verify did the DFA ones): one
// launch for every width -- a step's BPG candidates are few, the launch and the slowest walk are
// what cost, not the registers of the widest walk
__global__ __launch_bounds__(256) void k_bpg_cand_all(int64_t* __restrict__ cand, int64_t cap,
                                                      const unsigned long long* __restrict__ dcount,
                                                      const uint8_t* __restrict__ text, const int64_t* __restrict__ ls,
                                                      const int32_t* __restrict__ ll, DfaPool P) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = dcount ? (int64_t)min((unsigned long long)cap, dcount[0]) : cap;
  if (i >= n) return;
  const int64_t k = cand[i];
  if (k < 0) return;
  const int r = (int)(k >> 32);
  if (!is_bpg(P, r)) return;
  const uint64_t* prog = P.bpg + P.meta[4 * r];
  const int64_t x = k & 0xFFFFFFFFll;
  const uint8_t* s = text + ls[x];
  const int len = ll[x];
  bool m;
  switch ((int)(prog[0] & 0xFF)) {
    case 1: m = bpg_find_dev<1>(prog, s, len); break;
    case 2: m = bpg_find_dev<2>(prog, s, len); break;
    case 3: m = bpg_find_dev<3>(prog, s, len); break;
    case 4: m = bpg_find_dev<4>(prog, s, len); break;
    case 6: m = bpg_find_dev<6>(prog, s, len); break;
    default: m = bpg_find_dev<8>(prog, s, len); break;
  }
  if (!m) cand[i] = -1;
}

// bulk path: sorted packed keys ((regex << lbits | line) << 1 | pre-verified); the first key of
// every run whose regex is a width-W program and that no engine pre-verified gets its flag here
// (k_dedupe_verify left it 0)
constexpr int kLdsProgWords = 1024;   // 8 KiB (larger programs read from global memory)

__device__ __forceinline__ int prog_words(const uint64_t* prog, int W) {   // header, masks, tables
  const uint64_t h = prog[0];
  return 1 + 36 * W + 32 + (int)((h >> 20) & 0x3FF) * W + (int)((h >> 8) & 0xFFF) * (W + 1);
}

// bulk path, every width in one kernel (registers of the widest walk: fine for a few waves)
__global__ __launch_bounds__(256) void k_bpg_dedupe_all(const uint64_t* __restrict__ keys, int64_t n, int lbits,
                                                        const uint8_t* __restrict__ text,
                                                        const int64_t* __restrict__ ls,
                                                        const int32_t* __restrict__ ll, DfaPool P,
                                                        uint8_t* __restrict__ flag) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t key = keys[i];
  if (key == kPadKey) return;
  const uint64_t k = key >> 1;
  if (i > 0 && (keys[i - 1] >> 1) == k) return;
  const int r = (int)(k >> lbits);
  if (!is_bpg(P, r)) return;
  for (int64_t j = i; j < n && (keys[j] >> 1) == k; ++j)
    if (keys[j] & 1) return;                  // pre-verified: flag already 1
  const uint64_t* prog = P.bpg + P.meta[4 * r];
  const int64_t x = (int64_t)(k & ((1ull << lbits) - 1));
  const uint8_t* s = text + ls[x];
  const int len = ll[x];
  bool m;
  switch ((int)(prog[0] & 0xFF)) {
    case 1: m = bpg_find_dev<1>(prog, s, len); break;
    case 2: m = bpg_find_dev<2>(prog, s, len); break;
    case 3: m = bpg_find_dev<3>(prog, s, len); break;
    case 4: m = bpg_find_dev<4>(prog, s, len); break;
    case 6: m = bpg_find_dev<6>(prog, s, len); break;
    default: m = bpg_find_dev<8>(prog, s, len); break;
  }
  flag[i] = m ? 1 : 0;
}

// literal-free programs over every line: blockIdx.y = regex slot (block-uniform), the program is
// staged in LDS so class / first / last / exception reads are LDS hits
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
  const int nw = prog_words(prog, W);
  const int64_t line = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool m = false;
  if (nw <= kLdsProgWords) {
    for (int i = threadIdx.x; i < nw; i += blockDim.x) sp[i] = prog[i];
    __syncthreads();
    if (line < L) m = bpg_find_dev<W>(sp, text + ls[line], ll[line]);
  } else if (line < L) {
    m = bpg_find_dev<W>(prog, text + ls[line], ll[line]);
  }
  if (m) {
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

}  // namespace

void bpg_cand_dev(int64_t* cand, int64_t cap, const unsigned long long* dcount, const uint8_t* text, const int64_t* ls,
                  const int32_t* ll, const DfaPool& P, uint64_t stream) {
  if (!P.bpg_widths || cap <= 0) return;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_bpg_cand_all, dim3(nblocks(cap)), dim3(256), 0, st, cand, cap, dcount, text, ls, ll, P);
  check_launch("k_bpg_cand_all");
}

void bpg_dedupe_dev(const uint64_t* keys, int64_t n, int lbits, const uint8_t* text, const int64_t* ls,
                    const int32_t* ll, const DfaPool& P, uint8_t* flag, uint64_t stream) {
  if (!P.bpg_widths || n <= 0) return;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // ONE launch for every width: a step's BPG candidates are few (hundreds to thousands, a handful of
  // waves) and each walk is a serial chain of ~150 wave instructions per byte, so per-width launches
  // added up their slowest walks (~100 us each) where one launch runs them side by side
  hipLaunchKernelGGL(k_bpg_dedupe_all, dim3(nblocks(n)), dim3(256), 0, st, keys, n, lbits, text, ls, ll, P, flag);
  check_launch("k_bpg_dedupe_all");
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
}

}  // namespace lp
