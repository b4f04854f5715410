// Dependent-load latency probe (pointer chase, one lane) on the MI355X: how long one link of a
// dependency chain costs at each level (L1/L2/MALL/HBM, TLB reach) -- the quantity that bounds
// small-request latency of DFA walks and hash probes. Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

__global__ void chase(const uint32_t* __restrict__ next, int steps, uint32_t* out, long long* cycles) {
  uint32_t i = 0;
  const long long t0 = clock64();
  for (int s = 0; s < steps; ++s) i = next[i];
  const long long t1 = clock64();
  out[0] = i;
  cycles[0] = t1 - t0;
}

__global__ void chase_lds(const uint32_t* __restrict__ next, int n, int steps, uint32_t* out, long long* cycles) {
  __shared__ uint32_t s_next[8192];
  for (int k = threadIdx.x; k < n; k += blockDim.x) s_next[k] = next[k];
  __syncthreads();
  if (threadIdx.x) return;
  uint32_t i = 0;
  const long long t0 = clock64();
  for (int s = 0; s < steps; ++s) i = s_next[i];
  const long long t1 = clock64();
  out[0] = i;
  cycles[0] = t1 - t0;
}

int main() {
  const size_t maxb = size_t(1) << 30;
  uint32_t* d;
  hipMalloc(&d, maxb);
  uint32_t* out;
  long long* cyc;
  hipMalloc(&out, 4);
  hipMalloc(&cyc, 8);
  std::mt19937 rng(1);
  const int steps = 2000;
  for (size_t ws : {size_t(16) << 10, size_t(256) << 10, size_t(2) << 20, size_t(32) << 20, size_t(256) << 20,
                    size_t(1) << 30}) {
    for (size_t stride : {size_t(64), size_t(4096)}) {
      const size_t n = ws / stride;
      if (n < 16) continue;
      std::vector<uint32_t> perm(n);
      for (size_t k = 0; k < n; ++k) perm[k] = (uint32_t)k;
      std::shuffle(perm.begin() + 1, perm.end(), rng);
      std::vector<uint32_t> next(ws / 4, 0);
      const size_t w = stride / 4;
      for (size_t k = 0; k < n; ++k) next[perm[k] * w] = perm[(k + 1) % n] * (uint32_t)w;
      hipMemcpy(d, next.data(), ws, hipMemcpyHostToDevice);
      hipLaunchKernelGGL(chase, 1, 1, 0, 0, d, steps, out, cyc);  // warm
      hipDeviceSynchronize();
      hipEvent_t a, b;
      hipEventCreate(&a);
      hipEventCreate(&b);
      hipEventRecord(a);
      hipLaunchKernelGGL(chase, 1, 1, 0, 0, d, steps, out, cyc);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      long long c = 0;
      hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      printf("{\"ws_bytes\": %zu, \"stride\": %zu, \"ns_per_load\": %.1f, \"cycles_per_load\": %.1f}\n", ws, stride,
             ms * 1e6 / steps, (double)c / steps);
    }
  }
  // LDS
  {
    const int n = 8192;
    std::vector<uint32_t> perm(n), next(n);
    for (int k = 0; k < n; ++k) perm[k] = k;
    std::shuffle(perm.begin() + 1, perm.end(), rng);
    for (int k = 0; k < n; ++k) next[perm[k]] = perm[(k + 1) % n];
    hipMemcpy(d, next.data(), n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(chase_lds, 1, 256, 0, 0, d, n, steps, out, cyc);
    hipDeviceSynchronize();
    long long c = 0;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("{\"lds\": true, \"cycles_per_load\": %.1f}\n", (double)c / steps);
  }
  // empty-kernel dispatch rate
  {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    for (int k = 0; k < 200; ++k) hipLaunchKernelGGL(chase, 1, 1, 0, 0, d, 0, out, cyc);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    printf("{\"empty_kernel_us\": %.2f}\n", ms * 1e3 / 200);
  }
  return 0;
}
