// Native request runner: the whole device half of one continuous batch (Engine.device_batch on
// a GPU that owns its frequency state) in one C++ call with the GIL released.
//
// The Python orchestration of the same stages (log_parser_amd/engine.py prepare / finish,
// ops/kernels.py match_and_hits / post_events) spent ~150 us of host time per 10k-line request
// on tuple conversion, ~15 torch allocations and ~20 launches from Python -- more than the
// GPU's ~200 us of kernels, so the GPU idled between them. Here every buffer comes from one
// grow-only device workspace, the tables are converted once, and the stages are launched back to
// back on the caller's stream: H2D of the packed text + line index + segments, frequency
// eviction, matchers (prefilter + verify, scan groups), hit CSR + events (ONE counter read),
// events / context features / ranks, fp64 score, frequency record, ONE results read.
//
// Semantics are those of the Python path it replaces (which stays for the CPU backend, tracing,
// host-fallback regexes, MFMA scan groups and engines sharing a frequency state): same kernels,
// same arguments, same order on the stream.
#pragma once
#include <stdint.h>

#include <condition_variable>
#include <mutex>
#include <set>
#include <vector>

#include "kernels/lp_api.h"

namespace lp {

// Arrival-order gate of ONE shared frequency window used by several runners (engines on several
// GPUs, or several streams of one GPU): batch `seq` runs its window section -- eviction, score with
// the in-window carry, record (ScoringService.java:84-88 penalty before record, in arrival order,
// FrequencyTrackingService.java:25 one map for all workers) -- only after every earlier batch has
// finished its own. Matching runs before the gate, concurrently. done() is idempotent and may
// come out of order (a failed batch releases its slot).
//
// Turn is the interface the runner sees; WindowTurn orders the runners of ONE process,
// ProcTurn (runtime/proc_shared.h) the serving processes of a node over shared memory.
class Turn {
 public:
  virtual ~Turn() = default;
  virtual void wait(int64_t seq) = 0;
  virtual void done(int64_t seq) = 0;
};

class WindowTurn : public Turn {
 public:
  void wait(int64_t seq) override {
    std::unique_lock<std::mutex> g(m_);
    cv_.wait(g, [&] { return next_ >= seq; });
  }
  void done(int64_t seq) override {
    std::lock_guard<std::mutex> g(m_);
    if (seq < next_) return;
    done_.insert(seq);
    while (!done_.empty() && *done_.begin() == next_) {
      done_.erase(done_.begin());
      ++next_;
    }
    cv_.notify_all();
  }
  int64_t next() {
    std::lock_guard<std::mutex> g(m_);
    return next_;
  }

 private:
  std::mutex m_;
  std::condition_variable cv_;
  int64_t next_ = 0;
  std::set<int64_t> done_;
};

// A frequency window the runner does not own and that lives in HOST memory shared with the other
// serving processes of the node (proc_shared.h SharedWindow). The runner draws the batch's
// arrival ticket itself once the batch's matching, events, context features and frequency ranks
// have FINISHED on its GPU (everything that does not read the window), so the section other
// processes wait for is short: enter() -> evict + carry copy on the host -> score kernel (reads the
// pinned carry) -> results to the host -> record_batch() -> leave().
class HostWindow {
 public:
  virtual ~HostWindow() = default;
  virtual int64_t enter() = 0;                                           // ticket + turns -> seq
  virtual void leave(int64_t seq) = 0;
  // in the section: now' = max(last record time, now); evict at now' - window; tot -> carry[K]
  virtual double evict_carry(double now, int64_t* carry, int K) = 0;
  virtual void record_batch(const int64_t* counts, int K, double now) = 0;   // in the section
};

struct RequestStatic {
  PfTables pf;
  DfaPool dfa;
  std::vector<ScanPass> scans;
  std::vector<int> scan_grids;      // persistent grid of each scan pass
  const int32_t* scan_regs = nullptr;
  int n_scan_regs = 0;
  ScoreTables st;                   // per-pattern tables (batch fields filled per run)
  ScoreParams sp;
  EvTables ev;                      // static fields (segments filled per run)
  int R = 0;                        // regexes
  int npat = 0;
  int nkeys = 0;                    // frequency keys
  int nseq = 0;                     // sequence-event slots
  int ctx_trans = 0, ctx_acc = 0;   // context DFA extents (LDS staging)
  int pf_grid = 1;
  int device = 0;
  bool device_counts = true;        // requests: no mid-batch host read (see run())
  bool host_dev = false;            // backtracker regexes with relaxed automata: drop their device keys
                                    // (the host side path decided them: `inj`; side_path.hip)
};

struct RequestCounts {
  int64_t gram = 0, cand = 0, ver = 0, hits = 0, events = 0, lines = 0;
};

class RequestRunner {
 public:
  explicit RequestRunner(const RequestStatic& S);
  ~RequestRunner();
  RequestRunner(const RequestRunner&) = delete;
  RequestRunner& operator=(const RequestRunner&) = delete;

  // host_text: pinned packed bytes [0, nbytes) with room up to the padded length (zero-filled
  // here); host_cap: bytes usable at host_text -- when upload_bytes(nbytes, L, D) fit, the line
  // index, segments and the zero-initialised counters are laid out behind the text exactly as
  // the device workspace is carved and everything goes up in ONE H2D copy (otherwise one copy
  // per array); starts / lens: pinned line index (L lines); seg_*: D documents (host arrays).
  // ring: the device frequency state; evict_before / now: its eviction horizon and record time.
  // Returns the number of events ne; the results stay in result() until the next run:
  // [score f64 x E | freq counts i64 x max(nkeys, 1) | line i32 x E | pattern i32 x E | seg i32 x E]
  // with E = stride() >= ne (the event capacity of a device-count-mode request, else ne).
  // turn / seq: a shared window (WindowTurn above): the eviction moves from the start of the run to
  // the window section, entered through turn->wait(seq) once the matchers are queued and left
  // (turn->done(seq)) when the batch's record has completed -- also on errors.
  // hw: the window is a HostWindow (`ring` unused): the runner takes the ticket itself once the
  // carry-independent stages have finished, and records on the host (see HostWindow).
  int64_t run(uint8_t* host_text, int64_t nbytes, const int64_t* starts, const int32_t* lens, int64_t L,
              const int32_t* seg_lo, const int32_t* seg_hi, const int64_t* seg_g0, const int64_t* seg_n, int D,
              const FreqRing& ring, double evict_before, double now, uint64_t stream, int64_t host_cap = 0,
              Turn* turn = nullptr, int64_t seq = 0, const int64_t* inj = nullptr, int64_t ninj = 0,
              HostWindow* hw = nullptr, int64_t pre_token = 0);
  // Queue the upload of a request's packed TEXT (host_text[0, nbytes), pinned, 16-byte aligned) into
  // the workspace ahead of run(): the caller still builds the line index meanwhile (the text of a
  // /parse body is in its pinned decode buffer as soon as the body is validated). run() with the
  // same host_text / nbytes then uploads only what follows the text. Only when nothing in flight
  // uses the workspace (a lone request; the caller's job) and the workspace already holds the
  // text.
  // Returns a token (> 0) for run(pre_token = ...), 0 when nothing was queued.
  int64_t prefetch_text(uint8_t* host_text, int64_t nbytes, int64_t host_cap, uint64_t stream);
  // the batch's frequency record was enqueued (a failure after it must not record the batch again)
  bool recorded() const { return recorded_; }
  // host bytes the single-copy upload needs (text padded, index, segments, counters, carry)
  int64_t upload_bytes(int64_t nbytes, int64_t L, int D) const;
  const uint8_t* result() const { return res_host_; }
  size_t result_bytes() const { return res_bytes_; }
  const RequestCounts& counts() const { return counts_; }
  int64_t stride() const { return stride_; }

 private:
  uint8_t* dev(size_t bytes);          // carve from the device workspace (grown between runs)
  uint8_t* inj_host_ = nullptr;        // pinned staging of host-verified keys (backtracker side path)
  size_t inj_cap_ = 0;
  RequestStatic S_;
  // matcher capacity rates per line (as ops/kernels.py MatchArena)
  double rate_gram_ = 0.08, rate_cand_ = 0.03, rate_ver_ = 0.01;
  uint8_t* ws_ = nullptr;              // device workspace
  size_t ws_cap_ = 0, ws_used_ = 0, ws_need_ = 0;
  uint8_t* post_ws_ = nullptr;         // rocPRIM / post-pipeline scratch
  size_t post_cap_ = 0;
  uint8_t* up_host_ = nullptr;         // pinned upload staging (segments)
  size_t up_cap_ = 0;
  uint8_t* res_host_ = nullptr;        // pinned results
  size_t res_cap_ = 0, res_bytes_ = 0;
  int64_t* cnt_host_ = nullptr;        // pinned counters (fine-grained: k_publish writes them)
  int64_t* cnt_host_dev_ = nullptr;    // ... and the device's address of them
  uint8_t* res_host_dev_ = nullptr;    // device address of res_host_
  bool publish_ = true;                // device-count mode: results published by k_publish
  bool fetch_ = true;                  // single-copy inputs read by k_fetch from the pinned stage
  bool evict_in_fetch_ = false;        // the window eviction runs inside the k_fetch launch (opt-in)
  uint8_t* fetch_host_ = nullptr;      // last stage buffer seen ...
  uint8_t* fetch_dev_ = nullptr;       // ... and its device address (null: not mapped, SDMA copy)
  int64_t fetch_cap_ = 0;
  uint8_t* pre_host_ = nullptr;        // prefetch_text: the text queued ahead of run() ...
  int64_t pre_n_ = -1;                 // ... its length ...
  uint8_t* pre_ws_ = nullptr;          // ... into this workspace ...
  int64_t pre_token_ = 0, pre_next_ = 0;   // ... under this token (run() must name it)
  bool map_fetch(uint8_t* host_text, int64_t host_cap);   // fetch_dev_ for host_text (k_fetch source)
  RequestCounts counts_;
  int64_t stride_ = 0;
  bool recorded_ = false;
  int64_t* carry_host_ = nullptr;      // host window: the section's carry (pinned, device-visible)
  int64_t* carry_dev_ = nullptr;
  // literal-free scans on a second stream of the device, beside the literal chain and the
  // candidate verification (fork after the inputs, join before the hit pipeline)
  hipStream_t side_ = nullptr;
  hipEvent_t fork_ = nullptr, join_ = nullptr;
  bool side_on_ = true;
};

}  // namespace lp
