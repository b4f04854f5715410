// Cross-process serving state (runtime/proc_shared.h).
#include "runtime/proc_shared.h"

#include <errno.h>
#include <fcntl.h>
#include <linux/futex.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <new>
#include <stdexcept>
#include <thread>

namespace lp {

namespace {

constexpr uint64_t kMagic = 0x6c7073686172656bull;     // "lpshare" + version

// shared (not PRIVATE) futex ops: the word lives in a mapping of several processes
void futex_wait(std::atomic<uint32_t>* w, uint32_t val, int64_t ns) {
  timespec ts{(time_t)(ns / 1000000000), (long)(ns % 1000000000)};
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAIT, val, &ts, nullptr, 0);
}

void futex_wake_all(std::atomic<uint32_t>* w) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAKE, INT32_MAX, nullptr, nullptr, 0);
}

void* map_segment(const std::string& name, size_t bytes, bool create) {
  const int fd = shm_open(name.c_str(), create ? (O_CREAT | O_EXCL | O_RDWR) : O_RDWR, 0600);
  if (fd < 0) throw std::runtime_error("shm_open(" + name + "): " + std::strerror(errno));
  if (create && ftruncate(fd, (off_t)bytes) != 0) {
    const int e = errno;
    close(fd);
    shm_unlink(name.c_str());
    throw std::runtime_error("ftruncate(" + name + "): " + std::strerror(e));
  }
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) throw std::runtime_error("mmap(" + name + "): " + std::strerror(errno));
  return p;
}

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e) + " in " + what);
}

}  // namespace

// ---- turns ----------------------------------------------------------------------------------
void ProcTurn::wait(int64_t seq) {
  int64_t slept_ns = 0;
  for (;;) {
    const uint32_t w = b_->word.load(std::memory_order_acquire);
    const int64_t nx = b_->next.load(std::memory_order_acquire);
    if (nx >= seq) return;
    futex_wait(&b_->word, w, 50'000'000);        // 50 ms: then look for a dead ticket holder
    slept_ns += 50'000'000;
    if (slept_ns >= 1'000'000'000) {
      slept_ns = 0;
      const int64_t stuck = b_->next.load(std::memory_order_acquire);
      if (stuck < seq && s_->owner_dead(stuck)) {
        std::fprintf(stderr, "[lp] serving process of ticket %lld exited: releasing it\n", (long long)stuck);
        s_->header()->released_dead.fetch_add(1);
        done(stuck);
      }
    }
  }
}

void ProcTurn::done(int64_t seq) {
  s_->lock();
  int64_t nx = b_->next.load(std::memory_order_relaxed);
  if (seq >= nx) {
    if (seq - nx >= PROC_RING) {
      s_->unlock();
      throw std::runtime_error("ProcTurn: more than PROC_RING tickets in flight");
    }
    b_->done[seq % PROC_RING].store(seq + 1, std::memory_order_relaxed);
    bool moved = false;
    while (b_->done[nx % PROC_RING].load(std::memory_order_relaxed) == nx + 1) {
      b_->done[nx % PROC_RING].store(0, std::memory_order_relaxed);
      ++nx;
      moved = true;
    }
    if (moved) {
      b_->next.store(nx, std::memory_order_release);
      b_->word.fetch_add(1, std::memory_order_acq_rel);
    }
    s_->unlock();
    if (moved) futex_wake_all(&b_->word);
    return;
  }
  s_->unlock();
}

// ---- segment --------------------------------------------------------------------------------
ProcShared::ProcShared(const std::string& name, bool create, int nproc)
    : name_(name), host_(this, nullptr), dev_(this, nullptr) {
  void* p = map_segment(name, sizeof(ProcHeader), create);
  h_ = static_cast<ProcHeader*>(p);
  if (create) {
    std::memset(p, 0, sizeof(ProcHeader));         // zero = every atomic at 0 (shm_open already zeroes)
    h_->nproc = nproc;
    pthread_mutexattr_t a;
    pthread_mutexattr_init(&a);
    pthread_mutexattr_setpshared(&a, PTHREAD_PROCESS_SHARED);
    pthread_mutexattr_setrobust(&a, PTHREAD_MUTEX_ROBUST);
    pthread_mutex_init(&h_->mu, &a);
    pthread_mutexattr_destroy(&a);
    h_->magic.store(kMagic, std::memory_order_release);
  } else {
    for (int i = 0; h_->magic.load(std::memory_order_acquire) != kMagic; ++i) {
      if (i > 20000) throw std::runtime_error("shared segment " + name + " never initialised");
      std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
  }
  host_ = ProcTurn(this, &h_->turn[0]);
  dev_ = ProcTurn(this, &h_->turn[1]);
}

ProcShared::~ProcShared() {
  for (auto& m : maps_) munmap(m.first, m.second);
  if (h_) munmap(h_, sizeof(ProcHeader));
}

void ProcShared::lock() {
  const int r = pthread_mutex_lock(&h_->mu);
  if (r == EOWNERDEAD) pthread_mutex_consistent(&h_->mu);     // its holder died mid-advance: the
  else if (r != 0) throw std::runtime_error("ProcShared: mutex lock failed");   // ring state is whole
}

void ProcShared::unlock() { pthread_mutex_unlock(&h_->mu); }

int64_t ProcShared::take() {
  const int64_t s = h_->ticket.fetch_add(1, std::memory_order_acq_rel);
  h_->owner[s % PROC_RING].store((int32_t)getpid(), std::memory_order_release);
  return s;
}

bool ProcShared::owner_dead(int64_t seq) {
  const int32_t pid = h_->owner[seq % PROC_RING].load(std::memory_order_acquire);
  if (pid <= 0) return false;                // not taken yet: nobody to wait for
  return kill(pid, 0) != 0 && errno == ESRCH;
}

void ProcShared::mark_up(int worker, int32_t pid) {
  if (worker < 0 || worker >= PROC_MAX) throw std::out_of_range("worker index");
  h_->up[worker].store(pid, std::memory_order_release);
}

int32_t ProcShared::up(int worker) const {
  if (worker < 0 || worker >= PROC_MAX) throw std::out_of_range("worker index");
  return h_->up[worker].load(std::memory_order_acquire);
}

void* ProcShared::host_block(int64_t gen, int64_t bytes, bool create) {
  void* p = map_segment(name_ + ".w" + std::to_string(gen), (size_t)bytes, create);
  maps_.push_back({p, (size_t)bytes});
  return p;
}

void ProcShared::unlink(const std::string& name, int64_t max_gen) {
  for (int64_t g = 1; g <= max_gen; ++g) shm_unlink((name + ".w" + std::to_string(g)).c_str());
  shm_unlink(name.c_str());
}

// ---- GPU memory over IPC --------------------------------------------------------------------
std::pair<uint64_t, std::string> ipc_alloc(int device, int64_t bytes) {
  int cur = 0;
  check(hipGetDevice(&cur), "get device");
  check(hipSetDevice(device), "set device");
  void* p = nullptr;
  hipIpcMemHandle_t h;
  try {
    check(hipMalloc(&p, (size_t)bytes), "ipc window malloc");
    check(hipMemset(p, 0, (size_t)bytes), "ipc window memset");
    check(hipDeviceSynchronize(), "ipc window sync");
    check(hipIpcGetMemHandle(&h, p), "hipIpcGetMemHandle");
  } catch (...) {
    if (p) (void)hipFree(p);
    (void)hipSetDevice(cur);
    throw;
  }
  (void)hipSetDevice(cur);
  static_assert(sizeof(h) <= 64, "IPC handle fits the segment's slot");
  return {reinterpret_cast<uint64_t>(p), std::string(reinterpret_cast<const char*>(&h), sizeof(h))};
}

uint64_t ipc_open(int device, const std::string& handle) {
  hipIpcMemHandle_t h;
  if (handle.size() < sizeof(h)) throw std::invalid_argument("short IPC handle");
  std::memcpy(&h, handle.data(), sizeof(h));
  int cur = 0;
  check(hipGetDevice(&cur), "get device");
  check(hipSetDevice(device), "set device");
  void* p = nullptr;
  const hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
  (void)hipSetDevice(cur);
  check(e, "hipIpcOpenMemHandle");
  return reinterpret_cast<uint64_t>(p);
}

}  // namespace lp
