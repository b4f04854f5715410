// Backtracker regexes fed by the device (non-regular regexes -- backreferences,
// lookaround, atomic groups, possessive quantifiers -- are decided by a host backtracker,
// AnalysisService.java:88-95 find() of every primary on every line).
//
// Such a regex r carries, on the device, the automaton of its REGULAR RELAXATION (jregex.cpp
// Relaxer: a superset language; compiled.py host_dev, meta flag 4): its literals go through the
// literal prefilter and, without literals, its DFA joins a literal-free scan group. Every device
// key (r << 32 | line) is therefore only a CANDIDATE:
//   k_take_host   removes r's keys from the matcher buffers (prefilter candidates and the scan
//                 engines' verified hits) and -- export mode -- writes (key, line start, length) of
//                 each candidate (a prefilter candidate first passes r's relaxed DFA) into pinned
//                 host memory; the last block publishes the count, then the batch sequence number;
//   the host      (a helper thread) checks those lines with the C++ backtracker on the batch's host
//                 bytes and writes the verified keys, then the sequence number, into pinned memory;
//   k_wait_host   ONE workgroup, queued right behind, polls that sequence number (system-scope
//                 loads, a 2 s wall-clock limit every wave reaches) and appends the verified keys to
//                 the verified-hit buffer -- so the rest of the step is queued without a host
//                 round trip, and the GPU waits only if the host is not done by then.
// Drop mode (no export): requests and batches whose backtracker regexes ran on the host side path
// before the device work (Engine.host_hits) only remove the relaxation's keys.
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#include "lp_api.h"
#include "lp_core.h"

namespace lp {

namespace {

constexpr int kTakeThreads = 256;

__device__ __forceinline__ int64_t load_sys(const int64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(kTakeThreads) void k_take_host(int64_t* __restrict__ cand,
                                                            const unsigned long long* __restrict__ n1d, int64_t cap1,
                                                            int64_t* __restrict__ ver,
                                                            const unsigned long long* __restrict__ n2d, int64_t cap2,
                                                            const uint8_t* __restrict__ text,
                                                            const int64_t* __restrict__ ls,
                                                            const int32_t* __restrict__ ll, DfaPool P, HostSideOut O) {
  const int64_t n1 = n1d ? (int64_t)min((unsigned long long)cap1, *n1d) : cap1;
  const int64_t n2 = ver ? (n2d ? (int64_t)min((unsigned long long)cap2, *n2d) : cap2) : 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n1 + n2; i += stride) {
    int64_t* slot = i < n1 ? cand + i : ver + (i - n1);
    const int64_t k = *slot;
    if (k < 0) continue;
    const int r = (int)(k >> 32);
    if (!is_host_dev(P, r)) continue;
    *slot = -1;                                  // never a hit by itself: the host decides
    if (!O.keys) continue;
    const int64_t x = k & 0xFFFFFFFFll;
    // a prefilter candidate first passes the relaxed DFA (a BPG relaxation is exported as is)
    if (i < n1 && !is_bpg(P, r) && !dfa_run(P, r, text + ls[x], ll[x])) continue;
    const unsigned long long j = atomicAdd(O.cnt, 1ull);
    if ((int64_t)j < O.cap) {
      O.keys[j] = k;
      O.starts[j] = ls[x];
      O.lens[j] = ll[x];
      __threadfence_system();                    // host-visible before this block counts as done
    }
  }
  if (!O.keys) return;
  // the last block to finish publishes the count, then the sequence number (the host polls it)
  __syncthreads();
  __shared__ bool last;
  if (threadIdx.x == 0) {
    __threadfence_system();
    last = atomicAdd(O.done_blocks, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (last && threadIdx.x == 0) {
    const unsigned long long n = atomicAdd(O.cnt, 0ull);
    O.host_cnt[0] = (int64_t)n;
    __threadfence_system();
    O.host_seq[0] = O.seq;
    __threadfence_system();
    *O.cnt = 0;                                  // ready for the next batch
    *O.done_blocks = 0;
  }
}

__global__ __launch_bounds__(kTakeThreads) void k_wait_host(int64_t* __restrict__ ver, int64_t cap2,
                                                            unsigned long long* __restrict__ n2d, HostSideIn I) {
  __shared__ int64_t n;
  __shared__ unsigned long long base, pad_from;
  if (threadIdx.x == 0) {
    const long long t0 = wall_clock64();
    bool ok = true;
    while (load_sys(I.host_seq) != I.seq) {
      if (wall_clock64() - t0 > I.timeout_ticks) { ok = false; break; }
      __builtin_amdgcn_s_sleep(8);
    }
    const int64_t hc = ok ? load_sys(I.host_cnt) : -1;
    pad_from = ~0ull;
    if (hc < 0) {            // no answer in time, or the host failed / its export overflowed: the
      I.err[0] = ok ? 2 : 1; // batch overflows (its frequency record is vetoed, the caller re-runs)
      pad_from = atomicAdd(n2d, (unsigned long long)(cap2 + 1));
    }
    n = hc < 0 ? 0 : min(hc, I.cap);
    base = n > 0 ? atomicAdd(n2d, (unsigned long long)n) : 0ull;
  }
  __syncthreads();
  // the overflow signal pushes the count past the capacity, so the hit pipeline (which runs before
  // the host sees the counts) reads the WHOLE buffer: its unwritten tail becomes dropped keys
  // (-1), never uninitialised memory
  for (int64_t i = (int64_t)pad_from + threadIdx.x; pad_from != ~0ull && i < cap2; i += blockDim.x) ver[i] = -1;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x)
    if ((int64_t)(base + i) < cap2) ver[base + i] = I.keys[i];
}

void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e) + " in " + what);
}

}  // namespace

void take_host_dev(int64_t* cand, const unsigned long long* n1d, int64_t cap1, int64_t* ver,
                   const unsigned long long* n2d, int64_t cap2, const uint8_t* text, const int64_t* ls,
                   const int32_t* ll, const DfaPool& P, const HostSideOut& O, uint64_t stream) {
  const int64_t n = cap1 + (ver ? cap2 : 0);
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(1024, (n + kTakeThreads - 1) / kTakeThreads));
  hipLaunchKernelGGL(k_take_host, dim3(blocks), dim3(kTakeThreads), 0, reinterpret_cast<hipStream_t>(stream), cand,
                     n1d, cap1, ver, n2d, cap2, text, ls, ll, P, O);
  check_launch("k_take_host");
}

void wait_host_dev(int64_t* ver, int64_t cap2, unsigned long long* n2d, const HostSideIn& I, uint64_t stream) {
  hipLaunchKernelGGL(k_wait_host, dim3(1), dim3(kTakeThreads), 0, reinterpret_cast<hipStream_t>(stream), ver, cap2, n2d,
                     I);
  check_launch("k_wait_host");
}

}  // namespace lp
