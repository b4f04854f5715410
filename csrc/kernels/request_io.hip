// Request results straight into pinned host memory (the request runner's device-count mode).
//
// A 10k-line request returns ~100 events (reference: the AnalysisResult of Parse.java:41-61 /
// AnalysisService.java:117-180). In device-count mode the host does not know the event count
// until the batch is done, so the results used to come back as a capacity-sized SDMA copy
// (4096 events, 82 KB: ~7 us plus ~10 us of engine start-up) followed by a blit copy of the
// counters (~2 us plus ~8 us of queue gap). k_publish instead reads the device counters and
// writes the counters and the COMPACTED results (event stride = the real event count) into a
// fine-grained (coherent) pinned host buffer over PCIe: one ~3 us kernel, no copy command.
//
// Host layout written (the host-count layout of RequestRunner::result() with E = ne):
//   counters i64 x 5 (gram hits, candidates, scan hits, hits, events) -> cnt_host
//   [score f64 x ne | freq counts i64 x K1 | line i32 x ne | pattern i32 x ne | seg i32 x ne]
//   -> res_host, only when ne <= E (the device layout's capacity); otherwise only the counters
//   (the runner re-runs the batch in host-count mode).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>
#include <string>

#include "lp_api.h"

namespace lp {

__global__ __launch_bounds__(256) void k_publish(const int64_t* __restrict__ cnt, const uint8_t* __restrict__ out,
                                                 int64_t E, int K1, int64_t* __restrict__ cnt_host,
                                                 uint8_t* __restrict__ res_host) {
  const int64_t ne = cnt[4];
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  if (gid < 5) cnt_host[gid] = cnt[gid];
  if (ne < 0 || ne > E) return;
  const double* score = reinterpret_cast<const double*>(out);
  const int64_t* counts = reinterpret_cast<const int64_t*>(out + 8 * E);
  const int32_t* cols = reinterpret_cast<const int32_t*>(out + 8 * E + 8 * (int64_t)K1);
  double* h_score = reinterpret_cast<double*>(res_host);
  int64_t* h_counts = reinterpret_cast<int64_t*>(res_host + 8 * ne);
  int32_t* h_cols = reinterpret_cast<int32_t*>(res_host + 8 * ne + 8 * (int64_t)K1);
  const int64_t total = ne + K1 + 3 * ne;
  for (int64_t i = gid; i < total; i += stride) {
    if (i < ne) {
      h_score[i] = score[i];
    } else if (i < ne + K1) {
      h_counts[i - ne] = counts[i - ne];
    } else {
      const int64_t j = i - ne - K1;           // column c = j / ne, row r = j % ne
      const int64_t c = j / ne, r = j - c * ne;
      h_cols[j] = cols[c * E + r];
    }
  }
}

// Inputs of a request from pinned host memory straight into the workspace: one kernel whose
// lanes each keep up to 4 16-byte PCIe reads in flight. Replaces the SDMA copy, whose completion
// the compute queue only sees ~9 us later (request trace: copy 32 us + 9.6 us gap before it and
// 8.9 us after it).
// With `evict`, block 0 first drops the frequency window's records at or before `horizon` (the
// request's k_freq_evict, freq_state.hip: it reads nothing the fetch writes) and the fetch runs on
// the other blocks: one launch fewer per request.
__global__ __launch_bounds__(256) void k_fetch(const uint4* __restrict__ src, uint4* __restrict__ dst, int64_t n,
                                               int evict, FreqRing R, double horizon) {
  if (evict && blockIdx.x == 0) {
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
      const int c = __syncthreads_count(v);   // a prefix of the window: timestamps are ordered
      if (threadIdx.x == 0) R.ht[0] = head + c;
      __syncthreads();
      if (c < (int)blockDim.x) return;
    }
  }
  const int64_t stride = (int64_t)(gridDim.x - evict) * blockDim.x;
  int64_t i = (int64_t)(blockIdx.x - evict) * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n; i += stride) dst[i] = src[i];
}

void fetch_dev(const void* host_dev, void* dst, int64_t n16, uint64_t stream, const FreqRing* evict, double horizon) {
  if (n16 <= 0 && !evict) return;
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(2048, (n16 + 255) / 256));
  const int ev = evict ? 1 : 0;
  hipLaunchKernelGGL(k_fetch, dim3(blocks + ev), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     static_cast<const uint4*>(host_dev), static_cast<uint4*>(dst), n16, ev,
                     evict ? *evict : FreqRing{}, horizon);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e) + " in fetch");
}

// k_publish and the frequency record of the batch (k_freq_record, freq_state.hip) in ONE launch:
// both only read the finished results, so blocks [0, rec_blocks) record the per-key counts into
// the device window (gated on the matcher capacities, as k_freq_record) and the rest publish.
__global__ __launch_bounds__(256) void k_publish_record(const int64_t* __restrict__ cnt, const uint8_t* __restrict__ out,
                                                        int64_t E, int K1, int64_t* __restrict__ cnt_host,
                                                        uint8_t* __restrict__ res_host,
                                                        const int64_t* __restrict__ counts, int K, double now,
                                                        FreqRing R, RecordGate G, int rec_blocks) {
  if ((int)blockIdx.x < rec_blocks) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= K) return;
    if (G.cnt && (G.cnt[0] > G.cap[0] || G.cnt[1] > G.cap[1] || G.cnt[2] > G.cap[2] || G.cnt[4] > G.cap[3])) return;
    const int64_t c = counts[k];
    if (c <= 0) return;
    const int64_t p = (int64_t)atomicAdd(reinterpret_cast<unsigned long long*>(R.ht + 1), 1ull);
    const int64_t s = p % R.cap;
    R.t[s] = now;
    R.key[s] = k;
    R.cnt[s] = (int32_t)c;
    R.tot[k] += c;
    R.seen[k] = 1;
    return;
  }
  const int64_t ne = cnt[4];
  const int64_t gid = (int64_t)(blockIdx.x - rec_blocks) * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)(gridDim.x - rec_blocks) * blockDim.x;
  if (gid < 5) cnt_host[gid] = cnt[gid];
  if (ne < 0 || ne > E) return;
  const double* score = reinterpret_cast<const double*>(out);
  const int64_t* counts_e = reinterpret_cast<const int64_t*>(out + 8 * E);
  const int32_t* cols = reinterpret_cast<const int32_t*>(out + 8 * E + 8 * (int64_t)K1);
  double* h_score = reinterpret_cast<double*>(res_host);
  int64_t* h_counts = reinterpret_cast<int64_t*>(res_host + 8 * ne);
  int32_t* h_cols = reinterpret_cast<int32_t*>(res_host + 8 * ne + 8 * (int64_t)K1);
  const int64_t total = ne + K1 + 3 * ne;
  for (int64_t i = gid; i < total; i += stride) {
    if (i < ne) {
      h_score[i] = score[i];
    } else if (i < ne + K1) {
      h_counts[i - ne] = counts_e[i - ne];
    } else {
      const int64_t j = i - ne - K1;
      const int64_t c = j / ne, r = j - c * ne;
      h_cols[j] = cols[c * E + r];
    }
  }
}

void publish_record_dev(const int64_t* cnt, const uint8_t* out, int64_t E, int K1, int64_t* cnt_host,
                        uint8_t* res_host, const int64_t* counts, int K, double now, const FreqRing& R,
                        const RecordGate& G, uint64_t stream) {
  const int64_t total = 4 * E + K1;
  const int pub = (int)std::max<int64_t>(1, std::min<int64_t>(64, (total + 255) / 256));
  const int rec = K > 0 ? (K + 255) / 256 : 0;
  hipLaunchKernelGGL(k_publish_record, dim3(rec + pub), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), cnt, out,
                     E, K1, cnt_host, res_host, counts, K, now, R, G, rec);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e) + " in publish_record");
}

void publish_dev(const int64_t* cnt, const uint8_t* out, int64_t E, int K1, int64_t* cnt_host, uint8_t* res_host,
                 uint64_t stream) {
  const int64_t total = 4 * E + K1;
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(64, (total + 255) / 256));
  hipLaunchKernelGGL(k_publish, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), cnt, out, E, K1,
                     cnt_host, res_host);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e) + " in publish");
}

}  // namespace lp
