// Native HTTP/1.1 front end of the REST service (reference: Quarkus REST on Vert.x, Parse.java).
//
// epoll IO threads (one SO_REUSEPORT listener each) parse requests and decode POST /parse bodies
// natively (json_in.cpp); decoded requests wait in one queue that the Python side drains in
// batches with the GIL released (`next_requests`), then answers with `respond`. The analysis
// engine, batching and every other route stay in Python; the per-request HTTP + JSON work of the
// hot path does not.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "io/json_in.h"

namespace lp {

// Uninitialised, recycled storage for a body's `logs` text decoded by the IO thread (no memset of
// a fresh megabyte per request, as a std::string resize would do). Pinned (page-locked, GPU-mapped)
// for large bodies when the server feeds a GPU engine: the engine then uses the decoded text as its
// staging buffer in place -- with the decoder's newline positions, packing a 1 MB request is the
// line index alone, not a 40 us copy of the text across cores (profiles/r6_e).
struct DecodeBuf {
  char* p = nullptr;
  size_t cap = 0;
  bool pinned = false;
  void (*pfree)(void*) = nullptr;   // pinned: how to free it (the allocator of set_pinned_decode)
  NlPos nl;             // positions of the decoded text's '\n' bytes (recorded by the decoder)
  bool has_nl = false;  //   valid for this text
  DecodeBuf() = default;
  DecodeBuf(const DecodeBuf&) = delete;
  DecodeBuf& operator=(const DecodeBuf&) = delete;
  DecodeBuf(DecodeBuf&& o) noexcept
      : p(o.p), cap(o.cap), pinned(o.pinned), pfree(o.pfree), nl(std::move(o.nl)), has_nl(o.has_nl) {
    o.p = nullptr;
    o.cap = 0;
    o.has_nl = false;
  }
  DecodeBuf& operator=(DecodeBuf&& o) noexcept {
    if (this != &o) {
      release();
      p = o.p;
      cap = o.cap;
      pinned = o.pinned;
      pfree = o.pfree;
      nl = std::move(o.nl);
      has_nl = o.has_nl;
      o.p = nullptr;
      o.cap = 0;
      o.has_nl = false;
    }
    return *this;
  }
  ~DecodeBuf() { release(); }
  void release();
};
struct DecodePool {
  std::mutex m;
  std::vector<DecodeBuf> v;
  std::atomic<int> pinned_live{0};   // pinned buffers in existence (pooled or in flight)
  std::atomic<int> pinned_limit{0};  // 0: never pinned (set_pinned_decode)
  size_t pinned_min = 256 << 10;     // bodies at least this large get a pinned buffer
  void* (*palloc)(size_t) = nullptr; // pinned allocator / deallocator (the bindings pass HIP's):
  void (*pfree)(void*) = nullptr;    //   this file stays free of GPU runtime calls
  DecodeBuf take(size_t need);
  void give(DecodeBuf&& b);
};

struct HttpRequest {
  uint64_t id = 0;          // reply handle
  int kind = 0;             // 0 = decoded POST /parse, 1 = other route (raw method/path/body)
  std::string method, path, body;
  std::string logs;         // decoded UTF-8 log text (callers of the decode_logs mode)
  size_t logs_off = 0;      // kind 0: `body` is the raw request buffer and the JSON `logs`
  size_t logs_len = 0;      //   string's escaped content is body[logs_off, logs_off + logs_len)
  size_t logs_dlen = 0;     //   decoded UTF-8 length (counted while validating)
  DecodeBuf dec;            //   the decoded text (dec.p valid: decoded by the IO thread while validating)
  std::string pod_name;     // kind 0: pod.metadata.name or "" (unknown)
  double t_arrival = 0;     // monotonic seconds, when the body was complete
};

// Receive buffers recycled between requests (a fresh megabyte-sized allocation page-faults).
// Shared: a drained request's buffer may outlive the server (RawLogs in bind.cpp holds it until
// the engine has decoded it into its pinned stage).
struct BufferPool {
  std::mutex m;
  std::vector<std::string> v;
  std::string take();
  void give(std::string&& buf);
};

struct HttpStats {
  std::atomic<uint64_t> accepted{0}, requests{0}, bad_requests{0}, native_400{0};
};

// Where a decoded POST /parse spends its time on the native side (nanosecond sums; the Python
// side -- pack / device / emit -- is added by serve/native_http.py): receive = first byte -> body
// complete, validate = the JSON validation, queue = body complete -> drained by the pump,
// handoff = respond() -> the IO thread picks the response up, send = picked up -> last byte
// written to the socket; prefetch = the logs-string decoding done while bodies were arriving
// (inside `receive`), prefetched = bodies whose final validation resumed a prefetch.
struct HttpStageStats {
  std::atomic<uint64_t> parse{0}, receive_ns{0}, validate_ns{0}, drained{0}, queue_ns{0};
  std::atomic<uint64_t> prefetch_ns{0}, prefetched{0}, pump_prefetch_ns{0};
  std::atomic<uint64_t> responses{0}, handoff_ns{0}, sent{0}, send_ns{0};
};

// Tuning of the front end (config keys server.io-spin-us, server.pump-spin-us, server.tcp-quickack,
// server.rcvbuf-bytes, server.trace-requests; serve/native_http.py passes them)
struct HttpOptions {
  double io_spin_us = 0;        // IO threads poll (no sleep) this long after activity
  double pump_spin_us = 1000;   // next_requests polls this long before sleeping on the queue
  bool quickack = true;         // TCP_QUICKACK re-armed per read
  int rcvbuf = 0;               // SO_RCVBUF of accepted sockets (0 = autotuned)
  bool trace = false;           // per-request receive / validate timings on stderr
  bool conn_trace = false;      // per /parse response: accept / first byte / parsed / handed back / sent times
  bool prefetch = true;         // decode a large /parse body's logs string while it arrives
  // an IO thread decodes a /parse body's logs string itself only while it holds at most this many
  // connections; under a burst the bodies go to the packer undecoded (IO threads then only receive)
  int64_t io_decode_max_conns = 64;
};

// A large /parse body still arriving, registered by its IO thread so that the PUMP thread -- idle,
// spinning in next_requests while it waits for the next request -- decodes the arrived part of its
// logs string (logs_prefetch) on another core while the IO thread keeps receiving (the IO thread
// was the receive's bottleneck: decoding there moved ~40-70 us per MB into the receive, profiles/r6_e).
// Slots are never freed, so a thread reading one never dereferences a dead object; the state word
// decides who may touch the body, the decode buffer and the prefetch state:
//   FREE -> (IO thread registers) -> IDLE <-> PUMP (one prefetch step) ; IDLE -> IO (the IO thread
//   takes it back: body complete, buffer about to grow, connection closing) -> FREE.
struct ArrivalSlot {
  enum { FREE = 0, IDLE = 1, PUMP = 2, IO = 3 };
  std::atomic<int> state{FREE};
  std::atomic<size_t> avail{0};   // body bytes arrived (release-stored by the IO thread)
  std::atomic<size_t> seen{0};    // avail at the pump's last step (~0: nothing more to do)
  const uint8_t* body = nullptr;  // the connection's receive buffer at the body start
  char* dst = nullptr;            // the decode buffer
  size_t cap = 0;
  NlPos* nl = nullptr;
  LogsPrefetch pf;
};

class HttpServer {
 public:
  HttpServer(const std::string& host, int port, int io_threads, int64_t max_body, double idle_timeout_s = 60.0,
             const HttpOptions& opt = HttpOptions());
  ~HttpServer();
  int port() const { return port_; }
  // up to `max_n` pending requests; waits up to `timeout_ms` for the first one
  std::vector<HttpRequest> next_requests(int max_n, int timeout_ms);
  // requests parsed and waiting to be drained
  size_t pending() {
    std::lock_guard<std::mutex> g(qm_);
    return q_.size();
  }
  // queue the response of request `id` (ignored if its connection is gone)
  void respond(uint64_t id, int status, const std::string& content_type, const std::string& body);
  void respond(uint64_t id, int status, const std::string& content_type, const char* body, size_t n);
  // many responses of one status / content type: one outbox lock and one wake-up per IO thread
  void respond_many(const uint64_t* ids, size_t k, int status, const std::string& content_type,
                    const char* const* bodies, const size_t* lens);
  // hand a drained request's raw buffer back (its capacity serves a later request: no page faults
  // of a fresh megabyte-sized allocation per request)
  void recycle(std::string&& buf) { pool_->give(std::move(buf)); }
  const std::shared_ptr<BufferPool>& pool() const { return pool_; }
  const std::shared_ptr<DecodePool>& decode_pool() const { return dpool_; }
  // IO-thread CPU sets by load: an IO thread holding more than `hi` connections moves itself to
  // `wide` (a burst needs every core), back to `narrow` (the cores of the decode helper's L3) below
  // `lo`. Empty sets: no change.
  void set_affinity_sets(const std::vector<int>& narrow, const std::vector<int>& wide, int hi, int lo);
  // up to `limit` pinned decode buffers for bodies >= min_bytes (a GPU engine serves this server)
  void set_pinned_decode(int limit, size_t min_bytes, void* (*alloc)(size_t), void (*release)(void*)) {
    dpool_->pinned_min = min_bytes;
    dpool_->palloc = alloc;
    dpool_->pfree = release;
    dpool_->pinned_limit = alloc && release ? limit : 0;
  }
  void stop();
  HttpStats stats;
  HttpStageStats stages;
  // conn_trace: one record per /parse response sent since the last call -- (IO thread, accept,
  // first byte, request parsed, response handed to the IO thread, response sent), steady-clock
  // seconds (= Python time.perf_counter on Linux)
  std::vector<std::vector<double>> conn_trace();

  struct Conn;
  struct Io;

 private:
  void io_loop(Io* io);
  void handle_readable(Io* io, Conn* c);
  bool parse_one(Io* io, Conn* c);
  void send_now(Io* io, Conn* c, int status, const std::string& ctype, const std::string& body, bool keep);
  void flush(Io* io, Conn* c);
  void set_events(Io* io, Conn* c);
  void close_conn(Io* io, Conn* c);
  std::string take_buffer();
  bool advance_arrivals();                 // pump: one prefetch step per arrival slot with new bytes
  void publish_arrival(Conn* c);           // IO thread: the registered body's arrived length
  ArrivalSlot* acquire_slot(Conn* c);      // IO thread: take the connection's slot back (IO state)

  std::string host_;
  int port_;
  int64_t max_body_;
  double idle_timeout_s_;
  double io_spin_s_ = 0;     // HttpOptions (seconds)
  bool trace_ = false;
  bool conn_trace_ = false;
  bool prefetch_ = true;
  size_t io_decode_max_ = 64;
  double pump_spin_s_ = 0;
  bool quickack_ = true;
  int rcvbuf_ = 0;
  std::atomic<bool> stop_{false};
  std::vector<std::unique_ptr<Io>> ios_;
  std::vector<std::thread> threads_;
  // pending requests (Python side drains)
  std::mutex qm_;
  std::condition_variable qcv_;
  std::deque<HttpRequest> q_;
  std::atomic<size_t> qn_{0};   // q_.size(), for the pump's lock-free spin
  std::atomic<uint64_t> next_id_{1};
  std::shared_ptr<BufferPool> pool_ = std::make_shared<BufferPool>();
  std::shared_ptr<DecodePool> dpool_ = std::make_shared<DecodePool>();
  static constexpr int kSlots = 32;
  ArrivalSlot slots_[kSlots];
  std::atomic<int> arrivals_{0};           // registered slots (the pump wakes up for them)
  std::atomic<uint64_t> arr_gen_{0};       // bumped on every arrival the pump could act on
  std::atomic<bool> pump_waiting_{false};  // the pump sleeps on qcv_ (an arrival then notifies)
  // the decode helper: a thread that only advances the arrival slots (the pump helps while it
  // waits, but it is often still finishing the previous request when the next body starts)
  std::thread helper_;
  std::mutex hm_;
  std::condition_variable hcv_;
  std::atomic<bool> helper_waiting_{false};
  void helper_loop();
  // set_affinity_sets
  std::vector<int> aff_narrow_, aff_wide_;
  std::atomic<int> aff_hi_{0}, aff_lo_{0};
  std::atomic<uint64_t> aff_gen_{0};       // bumped by set_affinity_sets (IO threads re-apply)
};

}  // namespace lp
