// Thread pool-free parallel-for used by the host twins (CPU backend): independent items are
// split into contiguous ranges over plain std::threads. Shared by lp_kernels.hip / lp_post.hip.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <thread>
#include <vector>

namespace lp {

inline int& host_threads() {
  static int n = 8;
  return n;
}

template <class F>
inline void host_parallel(int64_t n, int64_t grain, F&& fn) {
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>(host_threads(), n / std::max<int64_t>(grain, 1)));
  if (T <= 1) {
    fn(0, 0, n);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(T);
  for (int t = 0; t < T; ++t) th.emplace_back([&, t] { fn(t, n * t / T, n * (t + 1) / T); });
  for (auto& x : th) x.join();
}

}  // namespace lp
