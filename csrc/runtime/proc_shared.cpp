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

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <limits>
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
  lock();
  const int64_t s = h_->ticket.fetch_add(1, std::memory_order_acq_rel);
  ProcOwner& o = h_->owner[s % PROC_RING];
  o.seq = s;                                 // (seq, pid) together under the mutex
  o.pid = (int32_t)getpid();
  unlock();
  return s;
}

bool ProcShared::owner_dead(int64_t seq) {
  lock();
  const ProcOwner o = h_->owner[seq % PROC_RING];
  unlock();
  if (o.seq != seq || o.pid <= 0) return false;   // not taken yet (or an older ticket's slot)
  return kill(o.pid, 0) != 0 && errno == ESRCH;
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
  // every published generation, then any block past it: a worker that died inside ensure_room,
  // between creating generation max_gen + 1 and publishing it, left that block behind
  for (int64_t g = 1;; ++g) {
    const int r = shm_unlink((name + ".w" + std::to_string(g)).c_str());
    if (g > max_gen && r != 0) break;
  }
  shm_unlink(name.c_str());
}

void ProcShared::drop_block(int64_t gen) { shm_unlink((name_ + ".w" + std::to_string(gen)).c_str()); }

// ---- the window in host shared memory ------------------------------------------------------
size_t SharedWindow::layout(int64_t cap, int K, size_t off[6]) {
  const size_t isz[6] = {8, 4, 4, 8, 8, 1};
  const size_t n[6] = {(size_t)cap, (size_t)cap, (size_t)cap, 2, (size_t)std::max(K, 1), (size_t)std::max(K, 1)};
  size_t o = 0;
  for (int i = 0; i < 6; ++i) {
    off[i] = o;
    o += (isz[i] * n[i] + 255) & ~size_t(255);
  }
  return o;
}

SharedWindow::SharedWindow(ProcShared* s, int nkeys, double window_s, bool create, int64_t capacity)
    : s_(s), K_(std::max(nkeys, 1)) {
  if (!create) return;
  ProcWindowMeta& m = s_->win();
  m.nkeys = K_;
  m.window_s = window_s;
  m.last_now = -std::numeric_limits<double>::infinity();
  map_gen(1, std::max<int64_t>(capacity, 2 * K_), true);
  m.generation.store(1, std::memory_order_release);     // published last: the block is complete
}

void SharedWindow::map_gen(int64_t gen, int64_t cap, bool create) {
  size_t off[6];
  const size_t bytes = layout(cap, K_, off);
  auto* b = static_cast<uint8_t*>(s_->host_block(gen, (int64_t)bytes, create));
  a_.t = reinterpret_cast<double*>(b + off[0]);
  a_.key = reinterpret_cast<int32_t*>(b + off[1]);
  a_.cnt = reinterpret_cast<int32_t*>(b + off[2]);
  a_.ht = reinterpret_cast<int64_t*>(b + off[3]);
  a_.tot = reinterpret_cast<int64_t*>(b + off[4]);
  a_.seen = b + off[5];
  a_.cap = cap;
  gen_ = gen;
  if (create) {
    s_->win().cap = cap;
    s_->win().block_bytes = (int64_t)bytes;
  }
}

WinArrays SharedWindow::arrays() {
  const int64_t g = s_->win().generation.load(std::memory_order_acquire);
  if (g == 0) throw std::runtime_error("the shared frequency window has not been created yet");
  if (g != gen_) map_gen(g, s_->win().cap, false);
  return a_;
}

void SharedWindow::ensure_room(int64_t k) {
  WinArrays a = arrays();
  const int64_t h = a.ht[0], tl = a.ht[1], n = tl - h;
  if (n + k <= a.cap) return;
  // a new generation: the live records compacted to [0, n), totals and seen flags carried over
  const int64_t cap = std::max<int64_t>(2 * a.cap, n + 2 * k);
  const WinArrays old = a;
  // the next generation is not published yet, so a block of that name can only be left over from
  // a process that died between creating and publishing it (this runs inside the window section:
  // no live process is building it): drop it, or O_EXCL would refuse every later growth
  s_->drop_block(gen_ + 1);
  map_gen(gen_ + 1, cap, true);
  for (int64_t i = 0; i < n; ++i) {
    const int64_t so = (h + i) % old.cap;
    a_.t[i] = old.t[so];
    a_.key[i] = old.key[so];
    a_.cnt[i] = old.cnt[so];
  }
  std::memcpy(a_.tot, old.tot, sizeof(int64_t) * (size_t)K_);
  std::memcpy(a_.seen, old.seen, (size_t)K_);
  a_.ht[0] = 0;
  a_.ht[1] = n;
  s_->win().generation.store(gen_, std::memory_order_release);
}

double SharedWindow::now(double t) {
  ProcWindowMeta& m = s_->win();
  if (t > m.last_now) m.last_now = t;
  return m.last_now;
}

void SharedWindow::evict(double horizon) {
  WinArrays a = arrays();
  int64_t h = a.ht[0];
  while (h < a.ht[1] && a.t[h % a.cap] <= horizon) {
    a.tot[a.key[h % a.cap]] -= a.cnt[h % a.cap];
    ++h;
  }
  a.ht[0] = h;
}

void SharedWindow::record(const int64_t* counts, int K, double t) {
  // a ring record holds an int32 count (the device ring's layout): a larger per-key batch count is
  // split over several records, so eviction subtracts exactly what was added to the total
  constexpr int64_t kMaxRec = std::numeric_limits<int32_t>::max();
  int64_t extra = 0;
  for (int k = 0; k < std::min(K, K_); ++k)
    if (counts[k] > kMaxRec) extra += (counts[k] - 1) / kMaxRec;
  if (extra > 0) ensure_room(K_ + extra);      // (the caller's ensure_room counted one per key)
  WinArrays a = arrays();
  for (int k = 0; k < std::min(K, K_); ++k) {
    int64_t c = counts[k];
    if (c <= 0) continue;
    a.tot[k] += c;
    a.seen[k] = 1;
    while (c > 0) {
      const int32_t part = (int32_t)std::min(c, kMaxRec);
      const int64_t sl = a.ht[1]++ % a.cap;     // room: ensure_room() before
      a.t[sl] = t;
      a.key[sl] = k;
      a.cnt[sl] = part;
      c -= part;
    }
  }
}

int64_t SharedWindow::enter() {
  const int64_t seq = s_->take();
  try {
    s_->host().wait(seq);
    s_->dev().wait(seq);
  } catch (...) {
    leave(seq);
    throw;
  }
  return seq;
}

void SharedWindow::leave(int64_t seq) {
  s_->header()->sections.fetch_add(1, std::memory_order_relaxed);
  s_->host().done(seq);
  s_->dev().done(seq);
}

double SharedWindow::evict_carry(double t, int64_t* carry, int K) {
  const double nw = now(t);
  evict(nw - s_->win().window_s);
  const WinArrays a = arrays();
  std::memcpy(carry, a.tot, sizeof(int64_t) * (size_t)std::min(K, K_));
  return nw;
}

}  // namespace lp
