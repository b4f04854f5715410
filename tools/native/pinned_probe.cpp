// Host-side cost of writing and reading pinned (hipHostMalloc) memory vs pageable memory on the
// serving box: the IO thread's JSON decode of a 1 MB /parse body into a pinned decode buffer took
// ~90 us against ~45 us into a pageable one (profiles/r6_e). Times, per buffer kind, a 1 MB
// memcpy into the buffer, a read pass over it, and the JSON string decode (lp::decode_json_string)
// into it; medians of 200 reps, on the calling thread's CPU.
//   hipcc -O2 -std=c++17 -Icsrc tools/native/pinned_probe.cpp csrc/io/json_in.cpp -o build/pinned_probe
#include <hip/hip_runtime_api.h>
#include <numa.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "io/json_in.h"

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <class F>
static double median_us(F&& f, int reps = 200) {
  std::vector<double> t;
  for (int i = 0; i < reps; ++i) {
    const double a = now_us();
    f();
    t.push_back(now_us() - a);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main() {
  // a 10k-line JSON string body, a '\n' escape every ~100 bytes (what /parse carries)
  std::string esc;
  for (int i = 0; esc.size() < (1 << 20) - 200; ++i)
    esc += "2024-05-01T12:00:00Z INFO  service-" + std::to_string(i % 97) + " request handled in 12 ms status=200 path=/api/v1/items\\n";
  const size_t n = esc.size(), cap = n + (4 << 20);
  std::vector<char> src(esc.begin(), esc.end());
  const std::string quoted = "\"" + esc + "\"";     // decode_json_string reads the closing quote
  struct Kind {
    const char* name;
    char* p;
  };
  std::vector<Kind> kinds;
  kinds.push_back({"pageable new[]", new char[cap]});
  const unsigned flags[] = {hipHostMallocDefault, hipHostMallocPortable, hipHostMallocNumaUser,
                            hipHostMallocNonCoherent, hipHostMallocWriteCombined};
  const char* names[] = {"hipHostMalloc default", "hipHostMalloc portable", "hipHostMalloc numa-user",
                         "hipHostMalloc non-coherent", "hipHostMalloc write-combined"};
  for (int k = 0; k < 5; ++k) {
    void* q = nullptr;
    if (hipHostMalloc(&q, cap, flags[k]) == hipSuccess) kinds.push_back({names[k], static_cast<char*>(q)});
    else (void)hipGetLastError();
  }
  void* reg = nullptr;                                   // pageable memory registered afterwards
  if (posix_memalign(&reg, 4096, cap) == 0) {
    std::memset(reg, 0, cap);
    if (hipHostRegister(reg, cap, hipHostRegisterDefault) == hipSuccess)
      kinds.push_back({"posix_memalign + hipHostRegister", static_cast<char*>(reg)});
    else (void)hipGetLastError();
  }
  std::printf("{\"bytes\": %zu, \"cpu\": %d, \"node\": %d, \"rows\": [\n", n, sched_getcpu(),
              numa_available() >= 0 ? numa_node_of_cpu(sched_getcpu()) : -1);
  for (size_t k = 0; k < kinds.size(); ++k) {
    char* p = kinds[k].p;
    int node = -1;
    if (numa_available() >= 0) {
      void* pg = p;
      int st = -1;
      if (numa_move_pages(0, 1, &pg, nullptr, &st, 0) == 0) node = st;
    }
    volatile uint64_t sink = 0;
    const double cp = median_us([&] { std::memcpy(p, src.data(), n); });
    const double rd = median_us([&] {
      uint64_t s = 0;
      for (size_t i = 0; i < n; i += 64) s += (uint8_t)p[i];
      sink = sink + s;
    });
    size_t dn = 0;
    const double dec = median_us([&] { dn = lp::decode_json_string(reinterpret_cast<const uint8_t*>(quoted.data()) + 1, n, p); });
    if (dn == 0) std::fprintf(stderr, "decode failed\n");
    std::printf("  {\"kind\": \"%s\", \"node\": %d, \"memcpy_us\": %.1f, \"read_us\": %.1f, \"decode_us\": %.1f}%s\n",
                kinds[k].name, node, cp, rd, dec, k + 1 < kinds.size() ? "," : "");
  }
  std::printf("]}\n");
  return 0;
}
