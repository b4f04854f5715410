// Calibration of one wave's dependent-chain latencies on the GPU (the request path's kernels are
// single-walk latency chains): core clock (s_memtime vs the 100 MHz s_memrealtime), cycles per
// dependent 32-bit VALU op, per dependent 64-bit AND/OR/shift step, per dependent LDS read and per
// dependent global (L2-resident) read.
// Build: hipcc -O3 --offload-arch=gfx950 tools/native/clock_probe.hip -o /tmp/clock_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

struct Out {
  long long cyc, wall;
  uint64_t sink;
};

__global__ void k_valu(Out* o, int iters, uint32_t seed) {
  uint32_t x = seed + threadIdx.x;
  const long long c0 = clock64(), w0 = wall_clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 16; ++j) x = x * 2654435761u + 7u;
  }
  const long long c1 = clock64(), w1 = wall_clock64();
  if (threadIdx.x == 0) { o->cyc = c1 - c0; o->wall = w1 - w0; o->sink = x; }
}

__global__ void k_step64(Out* o, int iters, uint64_t m1, uint64_t m2, uint64_t m3) {
  uint64_t S = m1 ^ threadIdx.x;
  const long long c0 = clock64(), w0 = wall_clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {   // one BPG-like step: shift / self / spread / class
      const uint64_t x = S & m1;
      uint64_t F = (x << 1) | (S & m2);
      const uint64_t df = (S & m3) | m2;
      F |= m1 & ~((df - m3) ^ df);
      S = F & (m3 | 1ull);
    }
  }
  const long long c1 = clock64(), w1 = wall_clock64();
  if (threadIdx.x == 0) { o->cyc = c1 - c0; o->wall = w1 - w0; o->sink = S; }
}

__global__ void k_lds(Out* o, int iters) {
  __shared__ uint32_t t[4096];
  for (int i = threadIdx.x; i < 4096; i += blockDim.x) t[i] = (i * 97 + 13) & 4095;
  __syncthreads();
  uint32_t p = threadIdx.x;
  const long long c0 = clock64(), w0 = wall_clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 16; ++j) p = t[p];
  }
  const long long c1 = clock64(), w1 = wall_clock64();
  if (threadIdx.x == 0) { o->cyc = c1 - c0; o->wall = w1 - w0; o->sink = p; }
}

__global__ void k_glob(Out* o, const uint32_t* __restrict__ t, int iters) {
  uint32_t p = threadIdx.x;
  const long long c0 = clock64(), w0 = wall_clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 16; ++j) p = t[p];
  }
  const long long c1 = clock64(), w1 = wall_clock64();
  if (threadIdx.x == 0) { o->cyc = c1 - c0; o->wall = w1 - w0; o->sink = p; }
}

int main() {
  Out* o;
  hipMalloc(&o, sizeof(Out));
  uint32_t* g;
  hipMalloc(&g, 4096 * 4);
  uint32_t h[4096];
  for (int i = 0; i < 4096; ++i) h[i] = (i * 97 + 13) & 4095;
  hipMemcpy(g, h, sizeof(h), hipMemcpyHostToDevice);
  const int iters = 4096;
  Out r;
  auto report = [&](const char* what, int per_iter) {
    hipMemcpy(&r, o, sizeof(Out), hipMemcpyDeviceToHost);
    const double steps = (double)iters * per_iter;
    const double mhz = r.wall > 0 ? (double)r.cyc / ((double)r.wall / 100.0) : 0;   // wall: 100 MHz
    std::printf("{\"probe\": \"%s\", \"cycles_per_step\": %.1f, \"ns_per_step\": %.2f, \"core_mhz\": %.0f}\n", what,
                r.cyc / steps, r.wall * 10.0 / steps, mhz);
  };
  for (int rep = 0; rep < 2; ++rep) {   // the second pass after the clocks ramped
    hipLaunchKernelGGL(k_valu, dim3(1), dim3(64), 0, 0, o, iters, 1u);
    hipDeviceSynchronize();
    if (rep) report("valu32_dependent", 16 * 2);
    hipLaunchKernelGGL(k_step64, dim3(1), dim3(64), 0, 0, o, iters, 0x5555ull, 0x3333ull, 0x0F0Full);
    hipDeviceSynchronize();
    if (rep) report("bpg_like_step64", 16);
    hipLaunchKernelGGL(k_lds, dim3(1), dim3(64), 0, 0, o, iters);
    hipDeviceSynchronize();
    if (rep) report("lds_dependent_read", 16);
    hipLaunchKernelGGL(k_glob, dim3(1), dim3(64), 0, 0, o, g, iters);
    hipDeviceSynchronize();
    if (rep) report("global_dependent_read", 16);
  }
  return 0;
}
