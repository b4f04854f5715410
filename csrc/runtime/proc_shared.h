// Node-scale serving: the state several serving PROCESSES share (one process per GPU, each with
// its own HTTP listeners, GIL and pipeline), so they keep the reference's single frequency window
// (FrequencyTrackingService.java:25 one map for all request threads, :41-56 record; penalty before
// record in arrival order, ScoringService.java:84-88).
//
// One POSIX shared-memory segment holds
//   * the arrival ticket: a batch takes the next sequence number when its MATCHING IS DONE (the
//     native request runner draws it after the batch's events / features / ranks have finished on
//     its GPU), so the cross-process critical section holds no other process's matching;
//   * two cross-process turns (ProcTurn): a ticket's window section runs after every earlier
//     ticket's, on whichever process (`host` and `dev` are both passed by every ticket: the Python
//     paths use the split, the runner takes both at once);
//   * the window itself lives in HOST shared memory (SharedWindow below, one block per generation
//     `<name>.w<gen>`): ring of (timestamp, key, count) records, in-window totals per key, a seen
//     flag per key. Every process -- whatever GPU it drives -- evicts, reads the carry and records
//     on the host inside its section; its score kernel reads the carry from a pinned copy. No IPC
//     of GPU memory, no peer access, and the native runner on every GPU.
// Waits sleep on a futex in the segment. A waiter that sleeps long checks whether the process
// holding the awaited ticket is still alive and releases the ticket of a dead one; the supervisor
// restarts dead workers and the survivors keep serving (serve/procs.py).
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

struct ProcWindowMeta {                       // written inside a window section only
  std::atomic<int64_t> generation;            // 0 = no window yet
  int64_t cap;                                // ring records of the current generation
  int64_t block_bytes;
  int32_t nkeys;                              // frequency keys of the library
  int32_t pad;
  double window_s;                            // scoring.frequency.time-window-hours in seconds
  double last_now;                            // timestamps of the ring never go backwards
};

// ticket owner: written under the segment mutex together (seq first), so a waiter checking for a
// dead holder never sees the pid left behind by ticket seq - PROC_RING
struct ProcOwner {
  int64_t seq;
  int32_t pid;
  int32_t pad;
};

struct ProcHeader {
  std::atomic<uint64_t> magic;
  int32_t nproc;
  int32_t pad;
  std::atomic<int64_t> ticket;
  pthread_mutex_t mu;                         // robust + process-shared: tickets, turn advances
  ProcOwner owner[PROC_RING];                 // slot seq % PROC_RING (under mu)
  std::atomic<int32_t> up[PROC_MAX];          // pid of worker i once it serves (0: not yet)
  std::atomic<int64_t> released_dead;         // tickets released on behalf of dead processes
  std::atomic<int64_t> sections;              // window sections completed (diagnostics)
  std::atomic<int64_t> restarts;              // workers restarted by the supervisor
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

// The window arrays of one generation (the layout frequency.SharedFrequencyState maps too:
// t f64[cap] | key i32[cap] | cnt i32[cap] | ht i64[2] | tot i64[K] | seen u8[K], 256-byte aligned).
struct WinArrays {
  double* t = nullptr;
  int32_t* key = nullptr;
  int32_t* cnt = nullptr;
  int64_t* ht = nullptr;                      // [head, tail): monotonic positions, slot = pos % cap
  int64_t* tot = nullptr;
  uint8_t* seen = nullptr;
  int64_t cap = 0;
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

  // host shared-memory blocks of the window: `<name>.w<gen>`; returns the mapping (kept until
  // the ProcShared is destroyed)
  void* host_block(int64_t gen, int64_t bytes, bool create);
  static void unlink(const std::string& name, int64_t max_gen);
  void drop_block(int64_t gen);   // unlink the host block of generation `gen` (an unpublished orphan)

 private:
  std::string name_;
  ProcHeader* h_ = nullptr;
  ProcTurn host_, dev_;
  std::vector<std::pair<void*, size_t>> maps_;
};

// The node's ONE frequency window in host shared memory (see the top). Every method but
// create / arrays / the ticket calls runs inside a window section (the caller holds the turns).
class SharedWindow : public HostWindow {
 public:
  // create: allocate generation 1 (the first worker, inside a ticket of its own); else attach
  SharedWindow(ProcShared* s, int nkeys, double window_s, bool create, int64_t capacity);
  static size_t layout(int64_t cap, int K, size_t off[6]);
  WinArrays arrays();                         // the current generation (re-mapped after a growth)
  void ensure_room(int64_t k);                // >= k free ring slots (grows to a new generation)
  double now(double t);                       // max(last record time, t): ring times never go back
  void evict(double horizon);                 // drop the records at or before `horizon`
  void record(const int64_t* counts, int K, double now);   // append the non-zero counts
  // HostWindow (the native request runner): ticket + turns, and the window section's host steps
  int64_t enter() override;
  void leave(int64_t seq) override;
  double evict_carry(double now, int64_t* carry, int K) override;
  void record_batch(const int64_t* counts, int K, double now) override { ensure_room(K); record(counts, K, now); }
  ProcShared* shared() { return s_; }
  int nkeys() const { return K_; }

 private:
  ProcShared* s_;
  int K_;
  int64_t gen_ = 0;
  WinArrays a_;
  void map_gen(int64_t gen, int64_t cap, bool create);
};

}  // namespace lp
