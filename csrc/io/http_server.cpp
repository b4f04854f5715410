// Native HTTP/1.1 front end (see http_server.h). Level-triggered epoll, one listener per IO thread
// (SO_REUSEPORT: the kernel spreads connections), keep-alive, `Expect: 100-continue`, one request
// in flight per connection (responses therefore stay in request order without pipelining state).
#include "io/http_server.h"

#include <pthread.h>
#include <cstdio>

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/resource.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

#include "io/json_in.h"

namespace lp {

namespace {
constexpr size_t kMaxHeader = 64 << 10;
constexpr int kMaxIo = 255;
// /parse bodies from this size on have their logs string decoded while they arrive
constexpr int64_t kPrefetchMin = 64 << 10;
// ... while its IO thread holds at most this many connections
constexpr size_t kPrefetchMaxConns = 64;
const char kInvalid[] = "{\"error\":\"Invalid PodFailureData provided\"}";
const char kUnsupported[] = "{\"error\":\"Content-Type must be application/json\"}";

// media type of a Content-Type value (parameters such as charset ignored, case-insensitive) is
// application/json; an absent header is accepted (see log_parser_amd/serve/app.py)
bool is_json_media_type(const std::string& v) {
  size_t e = v.find(';');
  if (e == std::string::npos) e = v.size();
  size_t a = 0;
  while (a < e && (v[a] == ' ' || v[a] == '\t')) ++a;
  while (e > a && (v[e - 1] == ' ' || v[e - 1] == '\t')) --e;
  static const char kJson[] = "application/json";
  if (e - a != sizeof(kJson) - 1) return false;
  for (size_t i = 0; i < e - a; ++i)
    if (tolower((unsigned char)v[a + i]) != kJson[i]) return false;
  return true;
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

const char* reason(int s) {
  switch (s) {
    case 100: return "Continue";
    case 200: return "OK";
    case 400: return "Bad Request";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 411: return "Length Required";
    case 413: return "Payload Too Large";
    case 415: return "Unsupported Media Type";
    case 431: return "Request Header Fields Too Large";
    case 500: return "Internal Server Error";
    case 501: return "Not Implemented";
    case 503: return "Service Unavailable";
    default: return "Status";
  }
}

bool ieq(const char* a, size_t n, const char* lit) {
  const size_t m = strlen(lit);
  if (n != m) return false;
  for (size_t i = 0; i < n; ++i)
    if (tolower((unsigned char)a[i]) != lit[i]) return false;
  return true;
}

std::string trim(const char* a, size_t n) {
  size_t i = 0, j = n;
  while (i < j && (a[i] == ' ' || a[i] == '\t')) ++i;
  while (j > i && (a[j - 1] == ' ' || a[j - 1] == '\t')) --j;
  return std::string(a + i, j - i);
}
// Grow this process's file-descriptor table to its final size now, before the IO threads run. The
// kernel grows the table by doubling as accept() hands out higher fds, and in a multi-threaded
// process every growth waits for an RCU grace period (expand_files -> synchronize_rcu): during a
// burst of thousands of new connections the IO threads sat in accept4 in D state for tens of ms
// at a time (utils/threadsample.py: 43% "accept4/expand_files" + 7% "accept4/__wait_rcu_gp" of the
// IO threads' samples in the slow config-5 runs, none in the fast ones, profiles/r5_b). Raising
// the table to the fd limit once (a descriptor at the highest fd, then closed: the table never shrinks)
// pays that wait once, at start-up.
void reserve_fd_table(int fd) {
  rlimit rl{};
  if (getrlimit(RLIMIT_NOFILE, &rl) != 0 || rl.rlim_cur == RLIM_INFINITY) return;
  const long top = std::min<long>((long)rl.rlim_cur, 1L << 17) - 1;
  if (top < 1024) return;
  // F_DUPFD_CLOEXEC takes the lowest FREE fd >= top: unlike dup2 it never closes a descriptor that
  // is already open there (inherited, or a library's), and the probe fd is close-on-exec meanwhile
  const int d = fcntl(fd, F_DUPFD_CLOEXEC, (int)top);
  if (d >= 0) close(d);
}

// Transfer-Encoding of a request (RFC 9112 §6.1): a comma-separated list of codings, applied in
// order. `identity` entries are no coding; the body is framed by chunked when it is the last
// coding. Any other coding (gzip, deflate, ...) is not decoded here (501).
enum { TE_NONE = 0, TE_CHUNKED = 1, TE_BAD_LAST = 2, TE_UNSUPPORTED = 3 };
int transfer_coding(const std::string& v) {
  int r = TE_NONE;
  size_t a = 0;
  while (a <= v.size()) {
    size_t e = v.find(',', a);
    if (e == std::string::npos) e = v.size();
    size_t i = a, j = e;
    while (i < j && (v[i] == ' ' || v[i] == '\t')) ++i;
    while (j > i && (v[j - 1] == ' ' || v[j - 1] == '\t')) --j;
    const size_t sc = v.find(';', i);   // transfer parameters are not meaningful for these codings
    if (sc != std::string::npos && sc < j) j = sc;
    while (j > i && (v[j - 1] == ' ' || v[j - 1] == '\t')) --j;
    if (j > i && !ieq(v.data() + i, j - i, "identity")) {
      if (!ieq(v.data() + i, j - i, "chunked")) return TE_UNSUPPORTED;
      r = (r == TE_NONE) ? TE_CHUNKED : TE_BAD_LAST;   // chunked applied twice
    }
    a = e + 1;
  }
  return r;
}

int hexval(char ch) {
  if (ch >= '0' && ch <= '9') return ch - '0';
  if (ch >= 'a' && ch <= 'f') return ch - 'a' + 10;
  if (ch >= 'A' && ch <= 'F') return ch - 'A' + 10;
  return -1;
}

enum { CH_MORE = 0, CH_DONE = 1, CH_BAD = -1, CH_BIG = -2 };
}  // namespace

// Incremental, in-place decoder of a chunked request body (RFC 9112 §7.1: size line with optional
// extensions, data, CRLF, ..., a zero-size chunk, trailer fields, empty line). The decoded bytes are
// compacted to [b0, dst) of the connection's receive buffer, directly behind the headers, so a
// complete body leaves the buffer laid out exactly like a Content-Length request (headers, body,
// pipelined bytes) and the rest of parse_one -- validation in place, zero-copy hand-off -- is
// shared. Each call resumes where the last one stopped and drops the framing it consumed, so the
// buffer holds at most one partial size / trailer line of framing and the decoded size, not the
// encoded one, is what `server.max-body-bytes` bounds (413).
struct ChunkDecoder {
  size_t dst = 0, src = 0;   // 0: not started (b0 > 0 always: the headers precede the body)
  uint64_t left = 0;         // bytes of the current chunk's data still to come
  int phase = 0;             // 0 size line, 1 data, 2 CRLF after the data, 3 trailer fields

  void reset() { *this = ChunkDecoder(); }

  int step(std::string& in, size_t b0, int64_t max_body) {
    if (src == 0) dst = src = b0;
    char* p = &in[0];
    const size_t n = in.size();
    int rc = CH_MORE;
    for (;;) {
      if (phase == 1) {
        const size_t k = (size_t)std::min<uint64_t>(left, n - src);
        if (k == 0) break;
        if (dst != src) memmove(p + dst, p + src, k);
        dst += k;
        src += k;
        left -= k;
        if (left == 0) phase = 2;
        continue;
      }
      if (phase == 2) {
        if (n - src < 2) break;
        if (p[src] != '\r' || p[src + 1] != '\n') {
          rc = CH_BAD;
          break;
        }
        src += 2;
        phase = 0;
        continue;
      }
      const char* nl = (const char*)memchr(p + src, '\n', n - src);
      if (!nl) {
        if (n - src > kMaxHeader) rc = CH_BAD;   // an unbounded size / trailer line
        break;
      }
      const size_t e = (size_t)(nl - p);           // index of the '\n'
      if (e == src || p[e - 1] != '\r') {
        rc = CH_BAD;
        break;
      }
      if (phase == 3) {                            // trailer fields: skipped up to the empty line
        const bool empty = e == src + 1;
        src = e + 1;
        if (empty) {
          rc = CH_DONE;
          break;
        }
        continue;
      }
      // phase 0: chunk-size [ BWS ; chunk-ext ] CRLF
      size_t i = src;
      uint64_t v = 0;
      int nd = 0;
      for (int h; i < e - 1 && (h = hexval(p[i])) >= 0; ++i) {
        if (++nd > 15) break;                      // > 2^60: refused below
        v = (v << 4) | (uint64_t)h;
      }
      while (i < e - 1 && (p[i] == ' ' || p[i] == '\t')) ++i;
      if (nd == 0 || nd > 15 || (i < e - 1 && p[i] != ';')) {
        rc = CH_BAD;
        break;
      }
      src = e + 1;
      if (v == 0) {
        phase = 3;
        continue;
      }
      if ((int64_t)(dst - b0) + (int64_t)v > max_body) {
        rc = CH_BIG;
        break;
      }
      left = v;
      phase = 1;
    }
    if (src > dst) {                               // drop the consumed framing
      in.erase(dst, src - dst);
      src = dst;
    }
    return rc;
  }
};

struct HttpServer::Conn {
  int fd = -1;
  uint64_t id = 0;
  std::string in, out;
  size_t out_off = 0;
  bool busy = false;        // a request is with the Python side
  bool keep = true;         // keep-alive of the request in flight
  bool sent_continue = false;
  bool closing = false;     // close once `out` is flushed
  bool want_out = false;
  bool paused = false;      // EPOLLIN off: too much pipelined input while a request is in flight
  bool dead = false;        // closed; freed at the end of the event-loop iteration
  double last = 0;          // last read / write activity (idle-timeout sweep)
  double t_first = 0;       // first byte of the request being received
  double t_resp = 0;        // respond() of the response being written (0: none timed)
  double t_accept = 0, t_parse = 0, t_handoff = 0;   // conn_trace
  int n_recv = 0, n_wake = 0;
  ChunkDecoder chunk;       // Transfer-Encoding: chunked body being received
  LogsPrefetch pf;          // POST /parse body being received: its logs string decoded so far
  DecodeBuf pdec;           //   into this buffer (handed to the request when the body completes)
  int slot = -1;            // arrival slot the pump decodes this body in (-1: none)
  bool early = false;       // parse_one already ran inside the receive loop for this request
  size_t slot_b0 = 0, slot_len = 0;   //   body offset in `in` and Content-Length
};

struct HttpServer::Io {
  int ep = -1, lfd = -1, efd = -1, index = 0;
  int wide = -1;                          // CPU set in force: -1 none set, 0 narrow, 1 wide
  uint64_t aff_gen = 0;
  uint64_t next_conn = 1;
  std::unordered_map<uint64_t, Conn*> conns;
  std::vector<Conn*> graveyard;   // closed this iteration (callers may still hold the pointer)
  double last_sweep = 0;
  std::mutex om;
  struct Out {
    uint64_t conn;
    std::string data;
    bool keep;
    double t_resp;
  };
  std::vector<Out> outbox;
  std::mutex tm;                          // conn_trace records (HttpOptions.conn_trace)
  std::vector<std::vector<double>> trace;
};

HttpServer::HttpServer(const std::string& host, int port, int io_threads, int64_t max_body, double idle_timeout_s,
                       const HttpOptions& opt)
    : host_(host), port_(port), max_body_(max_body), idle_timeout_s_(idle_timeout_s) {
  io_threads = std::max(1, std::min(io_threads, kMaxIo));
  io_spin_s_ = opt.io_spin_us * 1e-6;
  // the pump polls for the next request this long before sleeping on the queue's condition
  // variable (a sleeping pump took ~45 us to wake: /parse "queue" time, tools/parse_tail.py)
  pump_spin_s_ = opt.pump_spin_us * 1e-6;
  // Receive-side TCP: ACK every read at once. With delayed ACKs ~1-2% of 1 MB request bodies
  // stalled ~1.5 ms in the receive (the sender waiting on a window update): /parse p99 2.1 ms ->
  // 0.56 ms (profiles/r2_v12/tail_*.json; server.tcp-quickack=false restores delayed ACKs).
  quickack_ = opt.quickack;
  rcvbuf_ = opt.rcvbuf;
  trace_ = opt.trace;
  conn_trace_ = opt.conn_trace;
  prefetch_ = opt.prefetch;
  io_decode_max_ = opt.io_decode_max_conns < 0 ? SIZE_MAX : (size_t)opt.io_decode_max_conns;
  for (int i = 0; i < io_threads; ++i) {
    auto io = std::make_unique<Io>();
    io->index = i;
    io->lfd = socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    if (io->lfd < 0) throw std::runtime_error("socket() failed");
    int one = 1;
    setsockopt(io->lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    setsockopt(io->lfd, SOL_SOCKET, SO_REUSEPORT, &one, sizeof(one));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port_);
    if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) a.sin_addr.s_addr = htonl(INADDR_ANY);
    if (bind(io->lfd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0)
      throw std::runtime_error(std::string("bind() failed: ") + strerror(errno));
    if (port_ == 0) {  // ephemeral: every further listener binds the port the first one got
      socklen_t len = sizeof(a);
      getsockname(io->lfd, reinterpret_cast<sockaddr*>(&a), &len);
      port_ = ntohs(a.sin_port);
    }
    // (the kernel clamps the backlog to net.core.somaxconn: a 10k-connection burst spread over a
    // few listeners overflowed 1024 per listener while accept was slow)
    if (listen(io->lfd, 65535) != 0) throw std::runtime_error("listen() failed");
    io->ep = epoll_create1(EPOLL_CLOEXEC);
    io->efd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u64 = 0;  // 0 = listener
    epoll_ctl(io->ep, EPOLL_CTL_ADD, io->lfd, &ev);
    ev.data.u64 = 1;  // 1 = wake-up eventfd
    epoll_ctl(io->ep, EPOLL_CTL_ADD, io->efd, &ev);
    ios_.push_back(std::move(io));
  }
  reserve_fd_table(ios_[0]->lfd);
  if (prefetch_)
    helper_ = std::thread([this] {
      pthread_setname_np(pthread_self(), "lp-decode");
      helper_loop();
    });
  for (auto& io : ios_)
    threads_.emplace_back([this, p = io.get(), k = (int)threads_.size()] {
      char nm[16];
      std::snprintf(nm, sizeof nm, "lp-io%d", k);
      pthread_setname_np(pthread_self(), nm);     // (serving diagnostics: utils/threadsample.py)
      io_loop(p);
    });
}

HttpServer::~HttpServer() { stop(); }

void HttpServer::stop() {
  if (stop_.exchange(true)) return;
  for (auto& io : ios_) {
    uint64_t one = 1;
    (void)!write(io->efd, &one, 8);
  }
  for (auto& t : threads_)
    if (t.joinable()) t.join();
  {
    std::lock_guard<std::mutex> g(hm_);
  }
  hcv_.notify_all();
  if (helper_.joinable()) helper_.join();
  for (auto& io : ios_) {
    for (auto& kv : io->conns)
      if (kv.second->slot >= 0) {   // (a pump step in progress finishes first)
        acquire_slot(kv.second)->state.store(ArrivalSlot::FREE, std::memory_order_release);
        arrivals_.fetch_sub(1);
        kv.second->slot = -1;
      }
    for (auto& kv : io->conns) {
      close(kv.second->fd);
      delete kv.second;
    }
    io->conns.clear();
    close(io->lfd);
    close(io->efd);
    close(io->ep);
  }
  qcv_.notify_all();
}

std::vector<HttpRequest> HttpServer::next_requests(int max_n, int timeout_ms) {
  // system_clock deadline: pthread_cond_timedwait (steady-clock waits map to pthread_cond_clockwait,
  // which the ThreadSanitizer runtime of this toolchain does not intercept); a short poll anyway
  const auto deadline = std::chrono::system_clock::now() + std::chrono::milliseconds(std::max(0, timeout_ms));
  std::unique_lock<std::mutex> lk(qm_, std::defer_lock);
  for (;;) {
    // while waiting, decode the arriving bodies registered in the arrival slots
    double until = now_s() + pump_spin_s_;
    while (qn_.load(std::memory_order_acquire) == 0 && !stop_ && now_s() <= until) {
      if (advance_arrivals()) {
        until = now_s() + pump_spin_s_;
        continue;
      }
      for (int i = 0; i < 32; ++i) __builtin_ia32_pause();
    }
    const uint64_t gen = arr_gen_.load(std::memory_order_acquire);
    lk.lock();
    if (!q_.empty() || stop_) break;
    pump_waiting_.store(true, std::memory_order_seq_cst);
    const bool woke = qcv_.wait_until(lk, deadline, [&] {
      return !q_.empty() || stop_ || arr_gen_.load(std::memory_order_acquire) != gen;
    });
    pump_waiting_.store(false, std::memory_order_relaxed);
    if (!woke || !q_.empty() || stop_) break;
    lk.unlock();                                 // new arrivals only: decode them, then wait again
  }
  std::vector<HttpRequest> r;
  const double t = now_s();
  uint64_t qns = 0;
  while (!q_.empty() && (int)r.size() < max_n) {
    r.push_back(std::move(q_.front()));
    q_.pop_front();
    qn_.store(q_.size(), std::memory_order_release);
    qns += (uint64_t)std::max(0.0, (t - r.back().t_arrival) * 1e9);
  }
  if (!r.empty()) {
    stages.drained += r.size();
    stages.queue_ns += qns;
  }
  return r;
}

static std::string head(int status, const std::string& ctype, size_t n, bool keep) {
  std::string h = "HTTP/1.1 " + std::to_string(status) + " " + reason(status) + "\r\nContent-Type: " + ctype +
                  "\r\nContent-Length: " + std::to_string(n) + "\r\n";
  if (!keep) h += "Connection: close\r\n";
  h += "\r\n";
  return h;
}

void HttpServer::respond(uint64_t id, int status, const std::string& content_type, const std::string& body) {
  respond(id, status, content_type, body.data(), body.size());
}

void HttpServer::respond(uint64_t id, int status, const std::string& content_type, const char* body, size_t n) {
  const int ioi = (int)(id & 0xFF);
  if (ioi >= (int)ios_.size()) return;
  Io* io = ios_[ioi].get();
  const bool keep = (id >> 63) == 0;
  std::string data = head(status, content_type, n, keep);
  data.append(body, n);   // header + body in one buffer: one send() for a small response
  {
    std::lock_guard<std::mutex> lk(io->om);
    io->outbox.push_back(Io::Out{(id & ~(uint64_t(1) << 63)) >> 8, std::move(data), keep, now_s()});
  }
  uint64_t one = 1;
  (void)!write(io->efd, &one, 8);
}

void HttpServer::respond_many(const uint64_t* ids, size_t k, int status, const std::string& content_type,
                              const char* const* bodies, const size_t* lens) {
  std::vector<std::vector<Io::Out>> per(ios_.size());
  const double t = now_s();
  for (size_t i = 0; i < k; ++i) {
    const uint64_t id = ids[i];
    const int ioi = (int)(id & 0xFF);
    if (ioi >= (int)ios_.size()) continue;
    const bool keep = (id >> 63) == 0;
    std::string data = head(status, content_type, lens[i], keep);
    data.append(bodies[i], lens[i]);
    per[ioi].push_back(Io::Out{(id & ~(uint64_t(1) << 63)) >> 8, std::move(data), keep, t});
  }
  for (size_t q = 0; q < per.size(); ++q) {
    if (per[q].empty()) continue;
    Io* io = ios_[q].get();
    {
      std::lock_guard<std::mutex> lk(io->om);
      for (auto& o : per[q]) io->outbox.push_back(std::move(o));
    }
    uint64_t one = 1;
    (void)!write(io->efd, &one, 8);
  }
}

std::string BufferPool::take() {
  std::lock_guard<std::mutex> g(m);
  if (v.empty()) return std::string();
  std::string b = std::move(v.back());
  v.pop_back();
  return b;
}

void BufferPool::give(std::string&& buf) {
  if (buf.capacity() < (64u << 10) || buf.capacity() > (size_t(256) << 20)) return;
  buf.clear();
  std::lock_guard<std::mutex> g(m);
  if (v.size() < 64) v.push_back(std::move(buf));
}

std::string HttpServer::take_buffer() { return pool_->take(); }

void DecodeBuf::release() {
  if (!p) return;
  if (pinned)
    pfree(p);
  else
    delete[] p;
  p = nullptr;
  cap = 0;
}

DecodeBuf DecodePool::take(size_t need) {
  const bool want_pinned = pinned_limit.load() > 0 && need >= pinned_min;
  {
    std::lock_guard<std::mutex> g(m);
    // a pooled buffer that fits: pinned first when wanted (the engine stages in place)
    int best = -1;
    for (int i = (int)v.size() - 1; i >= 0; --i) {
      if (v[i].cap < need) continue;
      if (best < 0 || (v[i].pinned == want_pinned && v[best].pinned != want_pinned)) best = i;
    }
    if (best >= 0 && (v[best].pinned || !want_pinned || pinned_live.load() >= pinned_limit.load())) {
      DecodeBuf b = std::move(v[best]);
      v.erase(v.begin() + best);
      b.has_nl = false;
      return b;
    }
  }
  DecodeBuf b;
  if (want_pinned && pinned_live.fetch_add(1) < pinned_limit.load()) {
    // room for the engine's staging layout behind the text: padding, the line index (~12 bytes a
    // line), segments and counters (request.cpp single-copy upload)
    const size_t cap = (need + need / 4 + (96 << 10) + 4095) & ~size_t(4095);
    if (void* q = palloc(cap)) {
      b.p = static_cast<char*>(q);
      b.cap = cap;
      b.pinned = true;
      b.pfree = pfree;
      return b;
    }
    pinned_limit = 0;                      // no pinned memory here: pageable from now on
  }
  if (want_pinned) pinned_live.fetch_sub(1);
  b.cap = std::max<size_t>(need + need / 8, 64 << 10);
  b.p = new char[b.cap];
  return b;
}

void DecodePool::give(DecodeBuf&& b) {
  if (!b.p) return;
  if (b.cap <= (size_t(256) << 20)) {
    std::lock_guard<std::mutex> g(m);
    if (v.size() < 64) {
      v.push_back(std::move(b));
      return;
    }
  }
  if (b.pinned) pinned_live.fetch_sub(1);
  b.release();
}

void HttpServer::send_now(Io* io, Conn* c, int status, const std::string& ctype, const std::string& body,
                          bool keep) {
  c->out += head(status, ctype, body.size(), keep);
  c->out += body;
  if (!keep) c->closing = true;
  flush(io, c);
}

void HttpServer::flush(Io* io, Conn* c) {
  if (c->dead) return;
  while (c->out_off < c->out.size()) {
    const ssize_t k = ::send(c->fd, c->out.data() + c->out_off, c->out.size() - c->out_off, MSG_NOSIGNAL);
    if (k > 0) {
      c->out_off += (size_t)k;
      continue;
    }
    if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
    if (k < 0 && errno == EINTR) continue;
    close_conn(io, c);
    return;
  }
  if (c->out_off >= c->out.size()) {
    c->out.clear();
    c->out_off = 0;
    if (c->t_resp > 0) {
      const double ts = now_s();
      stages.sent++;
      stages.send_ns += (uint64_t)std::max(0.0, (ts - c->t_resp) * 1e9);
      c->t_resp = 0;
      if (conn_trace_ && c->t_parse > 0) {
        std::lock_guard<std::mutex> lk(io->tm);
        io->trace.push_back({(double)io->index, c->t_accept, c->t_first, c->t_parse, c->t_handoff, ts});
        c->t_parse = 0;
      }
    }
    if (c->closing) {
      close_conn(io, c);
      return;
    }
  }
  const bool want = !c->out.empty();
  if (want != c->want_out) {
    c->want_out = want;
    set_events(io, c);
  }
}

void HttpServer::set_events(Io* io, Conn* c) {
  epoll_event ev{};
  ev.events = EPOLLRDHUP | (c->paused ? 0 : EPOLLIN) | (c->want_out ? EPOLLOUT : 0);
  ev.data.u64 = c->id;
  epoll_ctl(io->ep, EPOLL_CTL_MOD, c->fd, &ev);
}

void HttpServer::close_conn(Io* io, Conn* c) {
  if (c->dead) return;
  if (c->slot >= 0) {                            // the body's buffers die with the connection
    acquire_slot(c)->state.store(ArrivalSlot::FREE, std::memory_order_release);
    arrivals_.fetch_sub(1);
    c->slot = -1;
  }
  if (c->pdec.p) dpool_->give(std::move(c->pdec));   // (a pinned one keeps the pool's count right)
  c->dead = true;
  epoll_ctl(io->ep, EPOLL_CTL_DEL, c->fd, nullptr);
  close(c->fd);
  io->conns.erase(c->id);
  io->graveyard.push_back(c);
}

void HttpServer::set_affinity_sets(const std::vector<int>& narrow, const std::vector<int>& wide, int hi, int lo) {
  {
    std::lock_guard<std::mutex> g(qm_);          // (read by the IO threads under the same lock)
    aff_narrow_ = narrow;
    aff_wide_ = wide;
  }
  aff_hi_ = hi;
  aff_lo_ = lo;
  aff_gen_.fetch_add(1);
}

static void apply_cpus(const std::vector<int>& cpus) {
  if (cpus.empty()) return;
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int c : cpus)
    if (c >= 0 && c < CPU_SETSIZE) CPU_SET(c, &set);
  (void)pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
}

void HttpServer::helper_loop() {
  while (!stop_) {
    // spin while registered bodies make progress (a step per 32-64 KiB of arrival); sleep after
    // 2 ms without work (no body, or a stalled client) until the next arrival is published
    double last = now_s();
    uint64_t gen = arr_gen_.load(std::memory_order_acquire);
    while (!stop_ && now_s() - last < 2e-3) {
      gen = arr_gen_.load(std::memory_order_acquire);
      if (advance_arrivals()) {
        last = now_s();
        continue;
      }
      for (int i = 0; i < 32; ++i) __builtin_ia32_pause();
    }
    std::unique_lock<std::mutex> lk(hm_);
    helper_waiting_.store(true, std::memory_order_seq_cst);
    // (system_clock deadline: see next_requests)
    hcv_.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(100),
                    [&] { return stop_.load() || arr_gen_.load(std::memory_order_acquire) != gen; });
    helper_waiting_.store(false, std::memory_order_relaxed);
  }
}

void HttpServer::publish_arrival(Conn* c) {
  ArrivalSlot& sl = slots_[c->slot];
  const size_t got = c->in.size() > c->slot_b0 ? std::min(c->in.size() - c->slot_b0, c->slot_len) : 0;
  if (got < sl.avail.load(std::memory_order_relaxed) + (32 << 10) && got < c->slot_len) return;   // (batched)
  sl.avail.store(got, std::memory_order_release);
  arr_gen_.fetch_add(1, std::memory_order_release);
  if (helper_waiting_.load(std::memory_order_seq_cst)) {
    { std::lock_guard<std::mutex> g(hm_); }
    hcv_.notify_one();
  }
  if (pump_waiting_.load(std::memory_order_seq_cst)) {
    { std::lock_guard<std::mutex> g(qm_); }      // (no lost wake-up against the pump's predicate)
    qcv_.notify_one();
  }
}

bool HttpServer::advance_arrivals() {
  if (arrivals_.load(std::memory_order_acquire) == 0) return false;
  bool worked = false;
  for (ArrivalSlot& sl : slots_) {
    if (sl.state.load(std::memory_order_relaxed) != ArrivalSlot::IDLE) continue;
    // a step per >= 32 KiB of new bytes (the body's tail is the IO thread's, at completion)
    if (sl.avail.load(std::memory_order_acquire) < sl.seen.load(std::memory_order_relaxed) + (32 << 10)) continue;
    int e = ArrivalSlot::IDLE;
    if (!sl.state.compare_exchange_strong(e, ArrivalSlot::PUMP, std::memory_order_acquire)) continue;
    // at most 64 KiB of new bytes per step: the IO thread that completes the body waits for the
    // step in progress (a step over everything that had arrived cost it ~60 us: the pump decodes
    // slower than a loopback body arrives), then decodes the remainder itself
    const size_t av = std::min(sl.avail.load(std::memory_order_acquire),
                               sl.seen.load(std::memory_order_relaxed) + (64 << 10));
    const double t0 = now_s();
    logs_prefetch(sl.body, av, sl.pf, sl.dst, sl.cap, sl.nl);
    stages.pump_prefetch_ns += (uint64_t)std::max(0.0, (now_s() - t0) * 1e9);
    sl.seen.store(sl.pf.state < 0 || sl.pf.state == 2 ? ~size_t(0) >> 1 : av, std::memory_order_relaxed);
    sl.state.store(ArrivalSlot::IDLE, std::memory_order_release);
    worked = true;
  }
  return worked;
}

ArrivalSlot* HttpServer::acquire_slot(Conn* c) {
  ArrivalSlot& sl = slots_[c->slot];
  for (;;) {                                     // a pump step is short (<= a few 10 us)
    int e = ArrivalSlot::IDLE;
    if (sl.state.compare_exchange_weak(e, ArrivalSlot::IO, std::memory_order_acquire)) return &sl;
    __builtin_ia32_pause();
  }
}

// Parses one complete request from c->in; false when more bytes are needed or the connection
// was closed.
bool HttpServer::parse_one(Io* io, Conn* c) {
  const size_t he = c->in.find("\r\n\r\n");
  if (he == std::string::npos) {
    if (c->in.size() > kMaxHeader) send_now(io, c, 431, "application/json", "{\"error\":\"headers too large\"}", false);
    return false;
  }
  const char* s = c->in.data();
  const size_t le = c->in.find("\r\n");
  // request line
  const char* sp1 = (const char*)memchr(s, ' ', le);
  const char* sp2 = sp1 ? (const char*)memchr(sp1 + 1, ' ', le - (sp1 + 1 - s)) : nullptr;
  if (!sp1 || !sp2) {
    send_now(io, c, 400, "application/json", "{\"error\":\"malformed request line\"}", false);
    return false;
  }
  std::string method(s, sp1 - s), path(sp1 + 1, sp2 - sp1 - 1), version(sp2 + 1, s + le - sp2 - 1);
  bool keep = version != "HTTP/1.0";
  int64_t clen = 0;
  bool has_len = false, expect = false, json_ctype = true, has_te = false;
  std::string te_list;
  size_t p = le + 2;
  while (p < he) {
    const size_t e = c->in.find("\r\n", p);
    const char* l = s + p;
    const size_t n = e - p;
    const char* colon = (const char*)memchr(l, ':', n);
    if (colon) {
      const size_t kn = colon - l;
      const std::string v = trim(colon + 1, n - kn - 1);
      if (ieq(l, kn, "content-length")) {
        has_len = true;
        clen = 0;
        for (char ch : v) {
          if (ch < '0' || ch > '9' || clen > (int64_t(1) << 50)) {
            clen = -1;
            break;
          }
          clen = clen * 10 + (ch - '0');
        }
      } else if (ieq(l, kn, "connection")) {
        std::string lv;
        for (char ch : v) lv.push_back((char)tolower((unsigned char)ch));
        if (lv.find("close") != std::string::npos) keep = false;
        if (lv.find("keep-alive") != std::string::npos) keep = true;
      } else if (ieq(l, kn, "transfer-encoding")) {
        if (has_te) te_list += ',';    // several header lines form one list (RFC 9110 §5.3)
        te_list += v;
        has_te = true;
      } else if (ieq(l, kn, "expect")) {
        expect = true;
      } else if (ieq(l, kn, "content-type")) {
        json_ctype = is_json_media_type(v);
      }
    }
    p = e + 2;
  }
  const int te = has_te ? transfer_coding(te_list) : TE_NONE;
  if (te == TE_UNSUPPORTED) {
    c->chunk.reset();
    send_now(io, c, 501, "application/json", "{\"error\":\"unsupported Transfer-Encoding\"}", false);
    return false;
  }
  if (te == TE_BAD_LAST) {   // RFC 9112 §6.3: a request whose final coding is not chunked is a 400
    c->chunk.reset();
    send_now(io, c, 400, "application/json", "{\"error\":\"chunked must be the final transfer coding\"}", false);
    return false;
  }
  if (te == TE_CHUNKED) {    // framing by chunks: Content-Length, if any, is ignored (RFC 9112 §6.3)
    const int rc = c->chunk.step(c->in, he + 4, max_body_);
    if (rc == CH_BAD) {
      c->chunk.reset();
      send_now(io, c, 400, "application/json", "{\"error\":\"malformed chunked body\"}", false);
      return false;
    }
    if (rc == CH_BIG) {
      c->chunk.reset();
      send_now(io, c, 413, "application/json", "{\"error\":\"request body too large\"}", false);
      return false;
    }
    if (rc == CH_MORE) {
      if (expect && !c->sent_continue) {
        c->out += "HTTP/1.1 100 Continue\r\n\r\n";
        c->sent_continue = true;
        flush(io, c);
      }
      return false;
    }
    clen = (int64_t)(c->chunk.dst - (he + 4));   // the buffer is now headers + body + pipelined bytes
    c->chunk.reset();
  }
  if (clen < 0) {
    send_now(io, c, 400, "application/json", "{\"error\":\"bad Content-Length\"}", false);
    return false;
  }
  if (clen > max_body_) {
    send_now(io, c, 413, "application/json", "{\"error\":\"request body too large\"}", false);
    return false;
  }
  const size_t total = he + 4 + (size_t)clen;
  const size_t q = path.find('?');
  const std::string route = q == std::string::npos ? path : path.substr(0, q);
  const size_t b0 = he + 4;
  if (c->in.size() < total) {
    if (c->in.capacity() < total) c->in.reserve(total);   // one allocation, not log2(n) regrowths
    if (expect && !c->sent_continue) {
      c->out += "HTTP/1.1 100 Continue\r\n\r\n";
      c->sent_continue = true;
      flush(io, c);
    }
    // a large /parse body: decode the part of its logs string that has arrived now, while this
    // thread would otherwise wait for the rest (the validation then ends with the last read)
    if (c->slot >= 0) {
      publish_arrival(c);
    } else if (prefetch_ && te == TE_NONE && clen >= kPrefetchMin && method == "POST" && route == "/parse" &&
               json_ctype && c->pf.state >= 0 && c->in.size() > b0 && io->conns.size() <= kPrefetchMaxConns) {
      // (a burst of connections: every IO thread is busy and decodes its own bodies at completion,
      // side by side; one helper core decoding them all would serialise them)
      if (!c->pdec.p) c->pdec = dpool_->take((size_t)clen + 64);
      // hand the body to the pump thread (arrival slot): it decodes while this thread receives.
      // The receive buffer must not move while registered -- room for some pipelined bytes too
      if (c->in.capacity() < total + (64 << 10)) c->in.reserve(total + (64 << 10));
      int k = -1;
      for (int i = 0; i < kSlots && k < 0; ++i) {
        int e = ArrivalSlot::FREE;
        if (slots_[i].state.compare_exchange_strong(e, ArrivalSlot::IO, std::memory_order_acquire)) k = i;
      }
      if (k >= 0) {
        ArrivalSlot& sl = slots_[k];
        sl.body = reinterpret_cast<const uint8_t*>(c->in.data()) + b0;
        sl.dst = c->pdec.p;
        sl.cap = c->pdec.cap;
        sl.nl = &c->pdec.nl;
        sl.pf = c->pf;
        sl.avail.store(0, std::memory_order_relaxed);   // (the slot's previous body's length)
        sl.seen.store(0, std::memory_order_relaxed);
        c->slot = k;
        c->slot_b0 = b0;
        c->slot_len = (size_t)clen;
        arrivals_.fetch_add(1);
        sl.state.store(ArrivalSlot::IDLE, std::memory_order_release);
        publish_arrival(c);
      } else {                                   // every slot taken: decode here between reads
        const double t0 = now_s();
        logs_prefetch(reinterpret_cast<const uint8_t*>(c->in.data()) + b0, c->in.size() - b0, c->pf, c->pdec.p,
                      c->pdec.cap, &c->pdec.nl);
        stages.prefetch_ns += (uint64_t)std::max(0.0, (now_s() - t0) * 1e9);
      }
    }
    return false;
  }
  c->sent_continue = false;
  stats.requests++;
  if (c->slot >= 0) {                            // the pump's part of the decoding is done
    ArrivalSlot* sl = acquire_slot(c);
    c->pf = sl->pf;
    sl->state.store(ArrivalSlot::FREE, std::memory_order_release);
    arrivals_.fetch_sub(1);
    c->slot = -1;
  }
  c->early = false;
  // the body's prefetch state (only for this request: reset whatever the outcome)
  LogsPrefetch pf = c->pf;
  DecodeBuf pdec = std::move(c->pdec);
  c->pf.reset();
  struct GiveBack {   // a prefetch buffer the request did not take goes back to the pool
    DecodePool* pool;
    DecodeBuf& b;
    ~GiveBack() {
      if (b.p) pool->give(std::move(b));
    }
  } give_back{dpool_.get(), pdec};
  auto consume = [&] { c->in.erase(0, total); };
  if (method == "GET" && route == "/health") {
    consume();
    send_now(io, c, 200, "application/json", "{\"status\":\"UP\"}", keep);
    return !c->closing && !c->dead;
  }
  HttpRequest r;
  r.t_arrival = now_s();
  if (method == "POST" && route == "/parse" && !json_ctype) {
    // @Consumes(MediaType.APPLICATION_JSON) (Parse.java:42): another media type is a 415
    consume();
    send_now(io, c, 415, "application/json", kUnsupported, keep);
    return !c->closing && !c->dead;
  }
  if (method == "POST" && route == "/parse") {
    // validated in place; the logs string is decoded later, once, straight into the Python bytes
    // object the engine packs from (bind.cpp next_requests)
    PodRequest pr;
    const double tv = r.t_arrival;
    c->t_parse = tv;
    // bodies of >= 4 KiB: the logs text is decoded by this thread in the validating pass, while the
    // bytes are in its cache -- the engine's packer then copies plain text instead of unescaping
    // bytes received on another core (server-side pack of a 1 MB body: 107 us, profiles/r6_c).
    // Not under a burst of connections (server.io-decode-max-conns): the IO threads are then the
    // front's bottleneck and the packer unescapes the batch's bodies instead.
    DecodeBuf dec;
    int st;
    if (clen >= (4 << 10) && (pdec.p || io->conns.size() <= io_decode_max_)) {
      const bool resume = pdec.p && pf.state >= 1;
      dec = pdec.p ? std::move(pdec) : dpool_->take((size_t)clen + 64);
      st = parse_pod_request_into(reinterpret_cast<const uint8_t*>(c->in.data()) + b0, (size_t)clen, pr,
                                  dec.p, dec.cap, resume ? &pf : nullptr, &dec.nl);
      dec.has_nl = st == JIN_OK && pr.logs_kind == 1 && pr.logs_decoded;
      if (resume) stages.prefetched++;
    } else {
      st = parse_pod_request(reinterpret_cast<const uint8_t*>(c->in.data()) + b0, (size_t)clen, pr, false);
    }
    if (st != JIN_OK || pr.logs_kind != 1 || !pr.logs_decoded) dpool_->give(std::move(dec));
    const double tz = now_s();
    stages.parse++;
    stages.receive_ns += (uint64_t)std::max(0.0, (tv - c->t_first) * 1e9);
    stages.validate_ns += (uint64_t)std::max(0.0, (tz - tv) * 1e9);
    if (trace_)
      fprintf(stderr, "lp-http-trace bytes %zu receive_us %.1f recvs %d wakeups %d validate_us %.1f prefetched %zu\n",
              total, (tv - c->t_first) * 1e6, c->n_recv, c->n_wake, (tz - tv) * 1e6,
              pf.state >= 1 ? pf.src - pf.s0 : (size_t)0);
    if (st == JIN_OK && (!pr.pod_nonnull || pr.logs_kind != 1)) {
      stats.native_400++;
      consume();
      if (!pr.pod_nonnull)
        send_now(io, c, 400, "application/json", kInvalid, keep);
      else
        send_now(io, c, 400, "application/json", "{\"error\":\"PodFailureData.logs must be a string\"}", keep);
      return !c->closing && !c->dead;
    }
    if (st == JIN_INVALID || st == JIN_NOT_OBJECT || clen == 0) {
      stats.native_400++;
      consume();
      send_now(io, c, 400, "application/json", kInvalid, keep);
      return !c->closing && !c->dead;
    }
    if (st == JIN_OK) {
      r.kind = 0;
      r.pod_name = pr.has_name ? pr.pod_name : std::string();
      r.logs_off = b0 + pr.logs_off;
      r.logs_len = pr.logs_len;
      r.logs_dlen = pr.logs_dlen;
      if (dec.p) r.dec = std::move(dec);
      if (c->in.size() == total) {   // the usual case: hand the whole buffer over, no copy
        r.body.swap(c->in);
        c->in = take_buffer();
      } else {                       // pipelined bytes follow: copy this request out
        r.body.assign(c->in, 0, total);
        consume();
      }
    } else {
      r.kind = 1;  // JIN_FALLBACK: the Python route decodes it with json.loads
    }
  } else {
    r.kind = 1;
  }
  if (r.kind == 1) {
    r.body = c->in.substr(b0, (size_t)clen);
    consume();
  }
  r.method = std::move(method);
  r.path = std::move(path);
  r.id = (c->id << 8) | (uint64_t)io->index | (keep ? 0 : (uint64_t(1) << 63));
  c->busy = true;
  c->keep = keep;
  {
    std::lock_guard<std::mutex> lk(qm_);
    q_.push_back(std::move(r));
    qn_.store(q_.size(), std::memory_order_release);
  }
  qcv_.notify_one();
  return false;
}

void HttpServer::handle_readable(Io* io, Conn* c) {
  if (c->dead) return;
  char buf[65536];
  c->n_wake++;
  for (;;) {
    const ssize_t k = ::recv(c->fd, buf, sizeof(buf), 0);
    if (k > 0 && quickack_) {      // the kernel leaves quick-ack mode on its own: re-arm per read
      int one = 1;
      setsockopt(c->fd, IPPROTO_TCP, TCP_QUICKACK, &one, sizeof(one));
    }
    if (k > 0) {
      c->last = now_s();
      if (c->in.empty()) {
        c->t_first = c->last;
        c->n_recv = 0;
        c->n_wake = 1;
      }
      c->n_recv++;
      if (c->slot >= 0 && c->in.size() + (size_t)k > c->in.capacity()) {
        // the buffer moves: take the body back from the pump for the append
        ArrivalSlot* sl = acquire_slot(c);
        c->in.append(buf, (size_t)k);
        sl->body = reinterpret_cast<const uint8_t*>(c->in.data()) + c->slot_b0;
        sl->state.store(ArrivalSlot::IDLE, std::memory_order_release);
      } else {
        c->in.append(buf, (size_t)k);
      }
      if (c->slot >= 0) {
        publish_arrival(c);
      } else if (!c->early && !c->busy && !c->closing && c->in.size() >= (64u << 10) && prefetch_ &&
                 io->conns.size() <= kPrefetchMaxConns) {
        // a large body is streaming in faster than this loop drains the socket: parse its headers
        // now (once), so its arrival slot is registered while the rest is still coming
        c->early = true;
        if (parse_one(io, c) || c->dead) {
          c->early = false;                      // (a complete request was dispatched here)
          if (c->dead) return;
        }
      }
      if ((int64_t)c->in.size() > max_body_ + (int64_t)kMaxHeader + 4) {
        if (c->busy) {  // stop reading until the in-flight request is answered
          c->paused = true;
          set_events(io, c);
        }
        break;  // not busy: parse_one answers 413
      }
      continue;
    }
    if (k == 0) {  // peer closed
      close_conn(io, c);
      return;
    }
    if (errno == EINTR) continue;
    if (errno == EAGAIN || errno == EWOULDBLOCK) break;
    close_conn(io, c);
    return;
  }
  while (!c->dead && !c->busy && !c->closing) {
    if (!parse_one(io, c)) break;
  }
}

void HttpServer::io_loop(Io* io) {
  epoll_event evs[256];
  double active = 0;
  while (!stop_) {
    const bool spin = io_spin_s_ > 0 && now_s() - active < io_spin_s_;
    const int n = epoll_wait(io->ep, evs, 256, spin ? 0 : 200);
    if (n > 0) active = now_s();
    for (int i = 0; i < n; ++i) {
      const uint64_t tag = evs[i].data.u64;
      if (tag == 0) {  // accept
        for (;;) {
          const int fd = accept4(io->lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
          if (fd < 0) break;
          int one = 1;
          setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
          if (rcvbuf_ > 0) setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &rcvbuf_, sizeof(rcvbuf_));
          if (quickack_) setsockopt(fd, IPPROTO_TCP, TCP_QUICKACK, &one, sizeof(one));
          Conn* c = new Conn();
          c->fd = fd;
          c->last = now_s();
          c->t_accept = c->last;
          c->id = (io->next_conn++) + 1;  // ids 0 / 1 are the listener / eventfd tags
          io->conns[c->id] = c;
          epoll_event ev{};
          ev.events = EPOLLIN | EPOLLRDHUP;
          ev.data.u64 = c->id;
          epoll_ctl(io->ep, EPOLL_CTL_ADD, fd, &ev);
          stats.accepted++;
        }
        continue;
      }
      if (tag == 1) {  // responses from Python
        uint64_t cnt;
        (void)!read(io->efd, &cnt, 8);
        std::vector<Io::Out> out;
        {
          std::lock_guard<std::mutex> lk(io->om);
          out.swap(io->outbox);
        }
        for (auto& o : out) {
          auto it = io->conns.find(o.conn);
          if (it == io->conns.end()) continue;  // client went away
          Conn* c = it->second;
          c->busy = false;
          if (c->paused) {
            c->paused = false;
            set_events(io, c);
          }
          const double tp = now_s();
          c->t_handoff = tp;
          stages.responses++;
          stages.handoff_ns += (uint64_t)std::max(0.0, (tp - o.t_resp) * 1e9);
          if (c->out.empty()) c->t_resp = tp;
          c->out += o.data;
          c->last = now_s();
          if (!o.keep) c->closing = true;
          flush(io, c);
          // next request already buffered on this keep-alive connection
          while (!c->dead && !c->busy && !c->closing) {
            if (!parse_one(io, c)) break;
          }
        }
        continue;
      }
      auto it = io->conns.find(tag);
      if (it == io->conns.end()) continue;
      Conn* c = it->second;
      if (evs[i].events & EPOLLOUT) {
        flush(io, c);
        if (c->dead) continue;
      }
      if (evs[i].events & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR)) {
        if (c->busy) {
          // a request is in flight: keep reading (pipelined bytes wait in `in`), detect hang-up
          if (evs[i].events & (EPOLLHUP | EPOLLERR)) {
            close_conn(io, c);
            continue;
          }
        }
        handle_readable(io, c);
      }
    }
    // CPU set by load (set_affinity_sets): wide under a burst of connections, narrow again when few
    const uint64_t ag = aff_gen_.load(std::memory_order_relaxed);
    if (ag != 0) {
      const size_t nc = io->conns.size();
      int want = io->wide;
      if (ag != io->aff_gen) want = -1;          // (new sets: re-apply)
      if (want != 1 && (int64_t)nc > aff_hi_.load(std::memory_order_relaxed)) want = 1;
      else if (want != 0 && (int64_t)nc < aff_lo_.load(std::memory_order_relaxed)) want = 0;
      else if (want < 0) want = 0;
      if (want != io->wide) {
        std::vector<int> cpus;
        {
          std::lock_guard<std::mutex> g(qm_);
          cpus = want == 1 ? aff_wide_ : aff_narrow_;
        }
        apply_cpus(cpus);
        io->wide = want;
      }
      io->aff_gen = ag;
    }
    // idle sweep (slow / stalled clients): a connection without a request in flight and without
    // traffic for idle_timeout_s is closed
    const double t = now_s();
    if (t - io->last_sweep > 1.0) {
      io->last_sweep = t;
      std::vector<Conn*> idle;
      for (auto& kv : io->conns)
        if (!kv.second->busy && t - kv.second->last > idle_timeout_s_) idle.push_back(kv.second);
      for (Conn* c : idle) close_conn(io, c);
    }
    for (Conn* c : io->graveyard) delete c;
    io->graveyard.clear();
  }
  for (Conn* c : io->graveyard) delete c;
  io->graveyard.clear();
}

}  // namespace lp

namespace lp {
std::vector<std::vector<double>> HttpServer::conn_trace() {
  std::vector<std::vector<double>> out;
  for (auto& io : ios_) {
    std::lock_guard<std::mutex> lk(io->tm);
    out.insert(out.end(), io->trace.begin(), io->trace.end());
    io->trace.clear();
  }
  return out;
}
}  // namespace lp
