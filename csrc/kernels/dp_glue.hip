// Per-step bookkeeping of the line-sharded DP step (log_parser_amd/parallel/dp.py) as two tiny
// kernels instead of ~15 ATen launches (casts, cat, partial sums, where-loops, clamp):
//
//   k_dp_pack   the C1+C3+C4 all-gather payload: [owned lines | frequency counts | chain table |
//               overflow flag] -- the flag is set when one of this rank's fixed-capacity match /
//               event buffers overflowed in a step that read no counts back (the step re-runs)
//   k_dp_carry  from the gathered [world][payload] rows and this rank: global line offset of the
//               first owned line and the segment base (C1), global N, the frequency carry
//               (persistent window totals + counts of lower ranks, C3 -- penalty before record in
//               rank order, ScoringService.java:84-88) and the backward sequence-chain carry
//               composed over the lower ranks (C4, ScoringService.java:296-305); it also seeds
//               the all-reduce buffer's frequency tail with this rank's counts, and ORs every
//               rank's overflow flag into the step's veto (no frequency record, re-run)
// Host twins for the CPU (gloo) path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>
#include <string>

#include "lp_api.h"
#include "lp_core.h"

namespace lp {

// overflow of a deferred-count step: a device counter past its buffer's capacity
LP_HD int64_t dp_overflow(const int64_t* cnt, const int64_t* cap) {
  if (!cnt) return 0;
  return (cnt[0] > cap[0] || cnt[1] > cap[1] || cnt[2] > cap[2] || cnt[4] > cap[3]) ? 1 : 0;
}

LP_HD void dp_pack_one(int64_t i, int64_t own_lines, const int64_t* freq, int nk, const int32_t* chain, int ns,
                       const int64_t* cnt, const int64_t* cap, int64_t* pack) {
  if (i == 0)
    pack[0] = own_lines;
  else if (i <= nk)
    pack[i] = freq[i - 1];
  else if (i <= nk + ns)
    pack[i] = chain[i - 1 - nk];
  else
    pack[i] = dp_overflow(cnt, cap);
}

LP_HD void dp_carry_one(int64_t i, const DpCarryArgs& A) {
  const int64_t row = 1 + A.nk + A.ns + 1;
  if (i == 0) {
    int64_t before = 0, total = 0, veto = 0;
    for (int q = 0; q < A.world; ++q) {
      total += A.g[q * row];
      if (q < A.rank) before += A.g[q * row];
      veto |= A.g[q * row + row - 1];
    }
    A.own_start[0] = A.line_base + before;
    A.g0[0] = A.line_base + before - A.halo_left;
    A.n[0] = A.n_fixed > 0 ? A.n_fixed : (total > 1 ? total : 1);
    if (A.veto) A.veto[0] = veto;
  }
  if (i < A.nk) {
    int64_t c = A.tot ? A.tot[i] : 0;
    for (int q = 0; q < A.rank; ++q) c += A.g[q * row + 1 + i];
    A.carry[i] = c;
    if (A.red_tail) A.red_tail[i] = A.g[A.rank * row + 1 + i];
  }
  if (i < A.nzero) A.zero[i] = 0;
  if (i < A.ns) {
    int64_t k = A.slot_k[i];
    for (int q = A.rank - 1; q >= 0 && k >= 0; --q) k = A.g[q * row + 1 + A.nk + A.slot_e0[i] + k];
    A.seq_carry[i] = k < 0 ? 1 : (A.seq_base ? A.seq_base[A.slot_e0[i] + k] : 0);
    if (A.seq_next) {       // the walk over every rank of the step: the state after it
      int64_t kk = A.slot_k[i];
      for (int q = A.world - 1; q >= 0 && kk >= 0; --q) kk = A.g[q * row + 1 + A.nk + A.slot_e0[i] + kk];
      A.seq_next[i] = kk < 0 ? 1 : (A.seq_base ? A.seq_base[A.slot_e0[i] + kk] : 0);
    }
  }
}

struct DpCaps {
  int64_t v[4];
};

__global__ __launch_bounds__(256) void k_dp_pack(int64_t n, int64_t own_lines, const int64_t* __restrict__ freq, int nk,
                                                 const int32_t* __restrict__ chain, int ns, const int64_t* cnt,
                                                 DpCaps caps, int64_t* __restrict__ pack) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dp_pack_one(i, own_lines, freq, nk, chain, ns, cnt, caps.v, pack);
}

__global__ __launch_bounds__(256) void k_dp_carry(int64_t n, DpCarryArgs A) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dp_carry_one(i, A);
}

static void check(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e) + " in " + what);
}

void dp_pack(int64_t own_lines, const int64_t* freq, int nk, const int32_t* chain, int ns, int64_t* pack,
             uint64_t stream, bool dev, const int64_t* cnt, const int64_t* caps) {
  const int64_t n = 1 + nk + ns + 1;
  DpCaps c{{0, 0, 0, 0}};
  if (cnt)
    for (int q = 0; q < 4; ++q) c.v[q] = caps[q];
  if (dev) {
    hipLaunchKernelGGL(k_dp_pack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), n, own_lines, freq, nk, chain, ns, cnt, c, pack);
    check("k_dp_pack");
    return;
  }
  for (int64_t i = 0; i < n; ++i) dp_pack_one(i, own_lines, freq, nk, chain, ns, cnt, c.v, pack);
}

void dp_carry(const DpCarryArgs& A, uint64_t stream, bool dev) {
  const int64_t n = std::max<int64_t>(std::max<int64_t>(1, A.nzero), std::max<int64_t>(A.nk, A.ns));
  if (dev) {
    hipLaunchKernelGGL(k_dp_carry, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), n, A);
    check("k_dp_carry");
    return;
  }
  for (int64_t i = 0; i < n; ++i) dp_carry_one(i, A);
}

}  // namespace lp
