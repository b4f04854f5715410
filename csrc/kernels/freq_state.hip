// Device-resident sliding-window frequency state (reference
// FrequencyTrackingService.java:20-162, penalty before record ScoringService.java:84-88).
//
// The reference keeps a process-global map id -> PatternFrequency(window) that survives across
// requests. Here the state lives in HBM next to the score kernel that reads it:
//   tot[K]   matches of every frequency key still inside the window (= the score kernel's carry)
//   seen[K]  key recorded at least once (the reference's map entry exists)
//   ring     FIFO of (timestamp, key, count) batch records, appended in batch (= arrival) order;
//            ht[0] = head, ht[1] = tail (monotonic 64-bit positions, slot = position % cap)
// Per batch: k_freq_evict drops the records at or before now - window from the head (they are
// a prefix: timestamps are non-decreasing) and subtracts them from tot; the fused score kernel
// reads tot as its carry; k_freq_record appends this batch's non-zero per-key counts and adds
// them to tot. No host round trip; the host only supplies the clock scalar.
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#include "lp_api.h"

namespace lp {

constexpr int FREQ_EVICT_THREADS = 1024;

__global__ __launch_bounds__(FREQ_EVICT_THREADS) void k_freq_evict(FreqRing R, double horizon) {
  for (;;) {
    const int64_t head = R.ht[0], tail = R.ht[1];
    const int64_t i = head + threadIdx.x;
    bool v = false;
    if (i < tail) {
      const int64_t s = i % R.cap;
      v = R.t[s] <= horizon;
      if (v) atomicAdd(reinterpret_cast<unsigned long long*>(R.tot + R.key[s]),
                       (unsigned long long)(-(int64_t)R.cnt[s]));
    }
    const int n = __syncthreads_count(v);    // a prefix of the window: timestamps are ordered
    if (threadIdx.x == 0) R.ht[0] = head + n;
    __syncthreads();
    if (n < FREQ_EVICT_THREADS) return;
  }
}

__global__ __launch_bounds__(256) void k_freq_record(const int64_t* __restrict__ counts, int K, double now,
                                                     FreqRing R, RecordGate G) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  if (G.cnt && (G.cnt[0] > G.cap[0] || G.cnt[1] > G.cap[1] || G.cnt[2] > G.cap[2] || G.cnt[4] > G.cap[3])) return;
  if (G.veto && *G.veto) return;
  const int64_t c = counts[k];
  if (c <= 0) return;
  const int64_t p = (int64_t)atomicAdd(reinterpret_cast<unsigned long long*>(R.ht + 1), 1ull);
  const int64_t s = p % R.cap;                // capacity is guaranteed by the host (grow before)
  R.t[s] = now;
  R.key[s] = k;
  R.cnt[s] = (int32_t)c;
  R.tot[k] += c;                              // one thread per key: no race
  R.seen[k] = 1;
}

void freq_evict(const FreqRing& R, double horizon, uint64_t stream, bool dev) {
  if (dev) {
    hipLaunchKernelGGL(k_freq_evict, dim3(1), dim3(FREQ_EVICT_THREADS), 0, reinterpret_cast<hipStream_t>(stream), R,
                       horizon);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e) + " in freq_evict");
    return;
  }
  int64_t h = R.ht[0];
  while (h < R.ht[1] && R.t[h % R.cap] <= horizon) {
    R.tot[R.key[h % R.cap]] -= R.cnt[h % R.cap];
    ++h;
  }
  R.ht[0] = h;
}

void freq_record(const int64_t* counts, int K, double now, const FreqRing& R, uint64_t stream, bool dev,
                 const RecordGate& gate) {
  if (K <= 0) return;
  if (dev) {
    hipLaunchKernelGGL(k_freq_record, dim3((K + 255) / 256), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                       counts, K, now, R, gate);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e) + " in freq_record");
    return;
  }
  if (gate.veto && *gate.veto) return;
  for (int k = 0; k < K; ++k) {
    const int64_t c = counts[k];
    if (c <= 0) continue;
    const int64_t s = R.ht[1]++ % R.cap;
    R.t[s] = now;
    R.key[s] = k;
    R.cnt[s] = (int32_t)c;
    R.tot[k] += c;
    R.seen[k] = 1;
  }
}

}  // namespace lp
