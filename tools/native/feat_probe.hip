// Phase timing of the context-feature walk (k_feat_cov's inner loop) on real tables: where does a
// ~100-byte 4-DFA walk spend its time on gfx950? Reads tables/lines dumped by tools/feat_probe.py.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <fstream>
#include <vector>

#include "kernels/lp_core.h"

using namespace lp;

template <class T>
static std::vector<T> rd(const char* path) {
  std::ifstream f(path, std::ios::binary | std::ios::ate);
  const size_t n = f.tellg();
  f.seekg(0);
  std::vector<T> v(n / sizeof(T));
  f.read(reinterpret_cast<char*>(v.data()), n);
  return v;
}

template <class T>
static T* up(const std::vector<T>& v, size_t pad = 0) {
  T* d;
  hipMalloc(&d, v.size() * sizeof(T) + pad);
  hipMemset(d, 0, v.size() * sizeof(T) + pad);
  hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
  return d;
}

// mode 0: tables in LDS, 4-way interleaved walk; 1: tables in global; 2: LDS, byte loads only
__global__ __launch_bounds__(256) void probe(const uint8_t* text, const int64_t* ls, const int32_t* ll, int nl,
                                             DfaPool P, int ctx_trans, int ctx_acc, int mode, uint8_t* feat,
                                             long long* dbg) {
  __shared__ int32_t s_meta[16];
  __shared__ __attribute__((aligned(16))) uint8_t s_bm[4 * 256];
  __shared__ uint16_t s_trans[8192];
  __shared__ uint8_t s_acc[1024];
  const long long t0 = clock64();
  if (threadIdx.x < 16) s_meta[threadIdx.x] = P.meta[threadIdx.x];
  for (int i = threadIdx.x; i < 4 * 256; i += blockDim.x) s_bm[i] = P.bytemap[i];
  for (int i = threadIdx.x; i < ctx_trans; i += blockDim.x) s_trans[i] = P.trans[i];
  for (int i = threadIdx.x; i < ctx_acc; i += blockDim.x) s_acc[i] = P.acc[i];
  __syncthreads();
  const long long t1 = clock64();
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  uint8_t f = 0;
  if (x < nl) {
    const uint8_t* s = text + ls[x];
    const int n = ll[x];
    if (mode == 0) {
      const DfaPool Q{s_meta, s_bm, s_trans, s_acc};
      f = context_feat(Q, s, n);
    } else if (mode == 1) {
      f = context_feat(P, s, n);
    } else {
      uint32_t acc = 0;
      for (int t = 0; t < n; ++t) acc += s[t];
      f = (uint8_t)acc;
    }
    feat[x] = f;
  }
  const long long t2 = clock64();
  if (x == 0) {
    dbg[0] = t1 - t0;
    dbg[1] = t2 - t1;
  }
}

int main(int argc, char** argv) {
  const char* dir = argc > 1 ? argv[1] : "/tmp/fp";
  std::string d(dir);
  auto meta = rd<int32_t>((d + "/meta.bin").c_str());
  auto bm = rd<uint8_t>((d + "/bm.bin").c_str());
  auto tr = rd<uint16_t>((d + "/trans.bin").c_str());
  auto ac = rd<uint8_t>((d + "/acc.bin").c_str());
  auto text = rd<uint8_t>((d + "/text.bin").c_str());
  auto ls = rd<int64_t>((d + "/ls.bin").c_str());
  auto ll = rd<int32_t>((d + "/ll.bin").c_str());
  auto ext = rd<int32_t>((d + "/ext.bin").c_str());
  DfaPool P{up(meta), up(bm), up(tr), up(ac)};
  uint8_t* dt = up(text, 128);
  int64_t* dls = up(ls);
  int32_t* dll = up(ll);
  const int nl = (int)ls.size();
  uint8_t* feat;
  hipMalloc(&feat, nl);
  long long* dbg;
  hipMalloc(&dbg, 16);
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEvent_t a, b;
      hipEventCreate(&a);
      hipEventCreate(&b);
      hipEventRecord(a);
      hipLaunchKernelGGL(probe, dim3((nl + 255) / 256), dim3(256), 0, 0, dt, dls, dll, nl, P, ext[0], ext[1], mode,
                         feat, dbg);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      long long h[2];
      hipMemcpy(h, dbg, 16, hipMemcpyDeviceToHost);
      printf("{\"mode\": %d, \"rep\": %d, \"lines\": %d, \"us\": %.1f, \"stage_cycles\": %lld, \"walk_cycles\": %lld}\n",
             mode, rep, nl, ms * 1e3, h[0], h[1]);
    }
  }
  return 0;
}
