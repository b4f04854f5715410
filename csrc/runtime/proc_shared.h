// Node-scale serving: the state several serving PROCESSES share (one process per GPU, each with
// its own HTTP listeners, GIL and pipeline), so they keep the reference's single frequency window
// (FrequencyTrackingService.java:25 one map for all request threads, :41-56 record; penalty before
// record in arrival order, ScoringService.java:84-88).
//
// One POSIX shared-memory segment holds
//   * the arrival ticket: every batch takes the next sequence number when it enters its device
//     stage (fetch-add), on whichever process it runs;
//   * two cross-process turns (ProcTurn): `host` orders the window's host bookkeeping (record
//     timestamps, ring tail bound, growth), `dev` orders the window sections on the device
//     (eviction, score with the carry, record) -- the same split as the in-process
//     SharedWindowTurn, and ProcTurn is a Turn, so the native request runner takes it as is;
//   * the window's metadata: where the ring lives (a hipIpcGetMemHandle of GPU memory on the
//     window's home GPU, or a host shared-memory block for CPU engines), its capacity and
//     generation (the ring grows by re-allocation: a process that grows it publishes a new
//     generation, the others re-map at their next window access, which the host turn orders after
//     the growth), the tail / head bounds and the last record timestamp.
// Waits sleep on a futex in the segment; a waiter that sleeps long checks whether the process
// holding the awaited ticket is still alive and releases the ticket of a dead one (availability:
// the other processes keep serving).
#pragma once
#include <pthread.h>

#include <atomic>
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#include "runtime/request.h"

namespace lp {

constexpr int PROC_RING = 4096;     // tickets in flight at once (a few per process)
constexpr int PROC_MAX = 64;

struct ProcTurnBlock {
  std::atomic<int64_t> next;
  std::atomic<uint32_t> word;                 // futex word: bumped whenever `next` advances
  uint32_t pad;
  std::atomic<int64_t> done[PROC_RING];       // seq + 1 once `seq` is done (slot seq % PROC_RING)
};

struct ProcWindowMeta {                       // written inside the host turn only
  std::atomic<int64_t> generation;            // 0 = no window yet
  int64_t cap;
  int64_t tail_bound, head_known;
  double last_now;
  int64_t block_bytes;
  int32_t kind;                               // 0 = host shared memory, 1 = GPU memory (IPC handle)
  int32_t home_device;
  uint8_t handle[64];
};

struct ProcHeader {
  std::atomic<uint64_t> magic;
  int32_t nproc;
  int32_t pad;
  std::atomic<int64_t> ticket;
  pthread_mutex_t mu;                         // robust + process-shared: advancing a turn
  std::atomic<int32_t> owner[PROC_RING];      // pid that took ticket seq (slot seq % PROC_RING)
  std::atomic<int32_t> up[PROC_MAX];          // pid of worker i once it serves (0: not yet)
  std::atomic<int64_t> released_dead;         // tickets released on behalf of dead processes
  ProcWindowMeta win;
  ProcTurnBlock turn[2];                      // 0 = host, 1 = dev
};

class ProcShared;

class ProcTurn : public Turn {
 public:
  ProcTurn(ProcShared* s, ProcTurnBlock* b) : s_(s), b_(b) {}
  void wait(int64_t seq) override;
  void done(int64_t seq) override;
  int64_t next() const { return b_->next.load(std::memory_order_acquire); }

 private:
  ProcShared* s_;
  ProcTurnBlock* b_;
};

class ProcShared {
 public:
  // create: a fresh segment (the launcher; fails if the name exists); else attach to one
  ProcShared(const std::string& name, bool create, int nproc = 0);
  ~ProcShared();
  ProcShared(const ProcShared&) = delete;
  ProcShared& operator=(const ProcShared&) = delete;

  int64_t take();                             // next arrival ticket
  ProcTurn& host() { return host_; }
  ProcTurn& dev() { return dev_; }
  ProcHeader* header() { return h_; }
  ProcWindowMeta& win() { return h_->win; }
  const std::string& name() const { return name_; }
  void mark_up(int worker, int32_t pid);
  int32_t up(int worker) const;
  int nproc() const { return h_->nproc; }
  void lock();
  void unlock();
  bool owner_dead(int64_t seq);               // the ticket's process has exited

  // host shared-memory blocks (CPU windows): `<name>.w<gen>`; returns the mapping (kept until
  // the ProcShared is destroyed)
  void* host_block(int64_t gen, int64_t bytes, bool create);
  static void unlink(const std::string& name, int64_t max_gen);

 private:
  std::string name_;
  ProcHeader* h_ = nullptr;
  ProcTurn host_, dev_;
  std::vector<std::pair<void*, size_t>> maps_;
};

// GPU memory shared across processes (hipIpcGetMemHandle / hipIpcOpenMemHandle)
std::pair<uint64_t, std::string> ipc_alloc(int device, int64_t bytes);     // zeroed; (ptr, handle)
uint64_t ipc_open(int device, const std::string& handle);

}  // namespace lp
