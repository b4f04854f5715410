// Host-side parallel-for of the native runtime: a persistent worker pool (request packing, JSON
// emission, the CPU backend's host twins). Threads are started once; a parallel region hands out
// work items through an atomic counter and the calling thread takes items too, so a region whose
// workers are slow to wake degrades to the serial loop instead of waiting for them (spawning
// std::threads per call cost 20-50 us -- as much as packing a whole 1 MB request).
// Shared by lp_kernels.hip / lp_post.hip / scan_multi.hip and csrc/io.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <pthread.h>

#include <thread>
#include <vector>

namespace lp {

inline int& host_threads() {
  static int n = 8;
  return n;
}

class HostPool {
 public:
  // one pool per calling thread: the serving pipeline packs batch k+1 while it emits batch k, and
  // a single shared pool ran whichever region came second serially (10k-request burst: 140k ->
  // 111k req/s). Never destroyed: workers may outlive static teardown.
  static HostPool& get() {
    static thread_local HostPool* p = new HostPool();
    return *p;
  }

  // fn(i) for every i in [0, n), on the caller plus up to `width - 1` workers; returns when all
  // items are done. Another region already running (a concurrent caller): runs serially inline.
  void run(int64_t n, int width, const std::function<void(int64_t)>& fn) {
    if (n <= 0) return;
    const int helpers = (int)std::min<int64_t>(std::min(width, nworkers_ + 1), n) - 1;
    std::unique_lock<std::mutex> region(region_, std::try_to_lock);
    if (helpers <= 0 || !region.owns_lock()) {
      for (int64_t i = 0; i < n; ++i) fn(i);
      return;
    }
    int sleeping;
    {
      std::lock_guard<std::mutex> g(m_);
      fn_ = &fn;
      n_ = n;
      next_.store(0, std::memory_order_relaxed);
      done_.store(0, std::memory_order_relaxed);
      want_ = helpers;
      gen_.fetch_add(1, std::memory_order_release);
      sleeping = sleepers_;
    }
    // spinning workers see the new generation by themselves; wake only as many sleepers as the
    // region can use (notify_all woke every worker: a futex storm costing more than the work)
    for (int k = 0; k < std::min(helpers, sleeping); ++k) cv_.notify_one();
    work();
    // wait until every item is done AND every worker that joined has left work(): the region's
    // state is only rewritten while no worker can read it
    while (done_.load(std::memory_order_acquire) < n_ || active_.load(std::memory_order_acquire) > 0)
      std::this_thread::yield();
    std::lock_guard<std::mutex> g(m_);   // late joiners see want_ = 0 and skip this region
    fn_ = nullptr;
    want_ = 0;
  }

 private:
  // a worker polls for the next region this long after its last one before sleeping (requests
  // arrive back to back under load: a futex wake-up costs tens of microseconds on a server part)
  static constexpr auto kSpin = std::chrono::microseconds(200);

  HostPool() {
    const unsigned hw = std::thread::hardware_concurrency();
    nworkers_ = (int)std::max(1u, std::min(hw ? hw : 8u, 16u)) - 1;
    for (int i = 0; i < nworkers_; ++i)
      std::thread([this, i] {
        pthread_setname_np(pthread_self(), "lp-host");
        loop(i);
      }).detach();
  }

  void work() {
    for (;;) {
      const int64_t i = next_.fetch_add(1, std::memory_order_relaxed);
      if (i >= n_) return;
      (*fn_)(i);
      done_.fetch_add(1, std::memory_order_release);
    }
  }

  void loop(int idx) {
    uint64_t seen = 0;
    for (;;) {
      const auto until = std::chrono::steady_clock::now() + kSpin;
      while (gen_.load(std::memory_order_acquire) == seen && std::chrono::steady_clock::now() < until)
        for (int k = 0; k < 64; ++k) pause();
      {
        std::unique_lock<std::mutex> lk(m_);
        if (gen_.load(std::memory_order_relaxed) == seen) {
          ++sleepers_;
          cv_.wait(lk, [&] { return gen_.load(std::memory_order_relaxed) != seen; });
          --sleepers_;
        }
        seen = gen_.load(std::memory_order_relaxed);
        if (idx >= want_ || fn_ == nullptr) continue;   // this region needs fewer helpers / is over
        active_.fetch_add(1, std::memory_order_relaxed);
      }
      work();
      active_.fetch_sub(1, std::memory_order_release);
    }
  }

  static inline void pause() {
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
  }

  int nworkers_ = 0;
  std::mutex region_;                 // one region at a time
  std::mutex m_;
  std::condition_variable cv_;
  std::atomic<uint64_t> gen_{0};
  int sleepers_ = 0;
  int want_ = 0;
  const std::function<void(int64_t)>* fn_ = nullptr;
  int64_t n_ = 0;
  std::atomic<int64_t> next_{0}, done_{0};
  std::atomic<int> active_{0};
};

// fn(t, begin, end) over `T` contiguous ranges of [0, n) (T from host_threads() and `grain`)
template <class F>
inline void host_parallel(int64_t n, int64_t grain, F&& fn) {
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>(host_threads(), n / std::max<int64_t>(grain, 1)));
  if (T <= 1) {
    fn(0, 0, n);
    return;
  }
  HostPool::get().run(T, T, [&](int64_t t) { fn((int)t, n * t / T, n * (t + 1) / T); });
}

}  // namespace lp
