// Native HTTP/1.1 load generator for BASELINE config 5 ("10k concurrent /parse requests, mixed
// sizes"): N keep-alive connections to the server, all established first, then ONE request per
// connection fired at once -- N requests in flight together -- with per-request latency from the
// first byte sent to the last byte of the response. A Python client would add its own scheduling
// delay to every one of 10k latencies; an epoll loop in C++ adds microseconds.
//
// Requests are pre-serialised HTTP messages (the caller builds them); connection c sends message
// idx[c]. Responses are parsed just enough to find their end (Content-Length, no chunking: the
// server always sends a length).
#include "io/loadgen.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstring>
#include <condition_variable>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>

namespace lp {
namespace {
// a one-shot barrier (std::barrier is C++20; the build is C++17)
struct OnceBarrier {
  explicit OnceBarrier(int n) : left(n) {}
  void arrive_and_wait() {
    std::unique_lock<std::mutex> lk(m);
    if (--left == 0) { cv.notify_all(); return; }
    cv.wait(lk, [&] { return left == 0; });
  }
  std::mutex m;
  std::condition_variable cv;
  int left;
};

double mono() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

struct Conn {
  int fd = -1;
  const std::string* msg = nullptr;
  size_t sent = 0;
  std::string in;
  size_t need = 0;          // total response bytes once the header is complete (0 = unknown)
  double t0 = 0, t1 = 0;
  int status = 0;
  bool connected = false, done = false;
};

// parse "HTTP/1.1 200 ...\r\n...Content-Length: n\r\n\r\n": returns header+body size or 0
size_t response_size(const std::string& s, int* status) {
  const size_t e = s.find("\r\n\r\n");
  if (e == std::string::npos) return 0;
  if (s.size() >= 12) *status = std::atoi(s.c_str() + 9);
  size_t len = 0;
  size_t p = 0;
  while (p < e) {
    size_t q = s.find("\r\n", p);
    if (q == std::string::npos || q > e) q = e;
    if (q - p > 15 && strncasecmp(s.c_str() + p, "content-length:", 15) == 0) len = std::strtoull(s.c_str() + p + 15, nullptr, 10);
    p = q + 2;
  }
  return e + 4 + len;
}

}  // namespace

namespace {

// one client thread: connections [lo, hi) on its own epoll set -- connect, wait for the common
// start, send, collect the responses
struct Group {
  std::vector<Conn>* conns;
  size_t lo, hi;
  const sockaddr_in* addr;
  const std::vector<std::string>* msgs;
  const std::vector<int32_t>* idx;
  double deadline;
  LoadResult* R;
  std::string error;
};

void run_group(Group& G, OnceBarrier& ready) {
  std::vector<Conn>& conns = *G.conns;
  const int ep = epoll_create1(EPOLL_CLOEXEC);
  std::vector<epoll_event> evs(1024);
  try {
    if (ep < 0) throw std::runtime_error("epoll_create1 failed");
    // 1) connections, in waves of at most 128 pending connects per thread (finite listen backlogs)
    size_t next = G.lo, pending = 0, up = 0;
    const size_t n = G.hi - G.lo;
    while (up < n) {
      while (next < G.hi && pending < 128) {
        Conn& c = conns[next];
        c.fd = socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
        if (c.fd < 0) throw std::runtime_error("socket() failed: " + std::string(strerror(errno)) + " (fd limit?)");
        int one = 1;
        setsockopt(c.fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
        const int r = connect(c.fd, reinterpret_cast<const sockaddr*>(G.addr), sizeof *G.addr);
        if (r != 0 && errno != EINPROGRESS) throw std::runtime_error("connect() failed: " + std::string(strerror(errno)));
        epoll_event ev{};
        ev.events = EPOLLOUT;
        ev.data.u64 = next;
        epoll_ctl(ep, EPOLL_CTL_ADD, c.fd, &ev);
        ++next;
        ++pending;
      }
      const int k = epoll_wait(ep, evs.data(), (int)evs.size(), 100);
      for (int i = 0; i < k; ++i) {
        Conn& c = conns[evs[i].data.u64];
        if (c.connected) continue;
        int err = 0;
        socklen_t sl = sizeof err;
        getsockopt(c.fd, SOL_SOCKET, SO_ERROR, &err, &sl);
        if (err) throw std::runtime_error("connect failed: " + std::string(strerror(err)));
        c.connected = true;
        epoll_event ev{};
        ev.events = EPOLLIN;          // quiet until the burst
        ev.data.u64 = evs[i].data.u64;
        epoll_ctl(ep, EPOLL_CTL_MOD, c.fd, &ev);
        --pending;
        ++up;
      }
      if (mono() > G.deadline) throw std::runtime_error("load generator: connecting timed out");
    }
  } catch (const std::exception& e) {
    G.error = e.what();
  }
  ready.arrive_and_wait();            // every thread connected (or failed): the burst starts
  if (!G.error.empty()) {
    if (ep >= 0) close(ep);
    return;
  }
  // 2) the burst: every connection of this thread sends its request now
  for (size_t i = G.lo; i < G.hi; ++i) {
    Conn& c = conns[i];
    c.msg = &G.msgs->at((size_t)(*G.idx)[i]);
    c.t0 = mono();
    const ssize_t w = send(c.fd, c.msg->data(), c.msg->size(), MSG_NOSIGNAL);
    if (w > 0) c.sent = (size_t)w;
    if (c.sent < c.msg->size()) {
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLOUT;
      ev.data.u64 = i;
      epoll_ctl(ep, EPOLL_CTL_MOD, c.fd, &ev);
    }
  }
  // 3) responses
  size_t finished = 0;
  const size_t n = G.hi - G.lo;
  std::vector<char> buf(1 << 16);
  while (finished < n) {
    if (mono() > G.deadline) break;
    const int k = epoll_wait(ep, evs.data(), (int)evs.size(), 100);
    for (int i = 0; i < k; ++i) {
      const size_t ci = evs[i].data.u64;
      Conn& c = conns[ci];
      if (c.done) continue;
      if ((evs[i].events & EPOLLOUT) && c.sent < c.msg->size()) {
        const ssize_t w = send(c.fd, c.msg->data() + c.sent, c.msg->size() - c.sent, MSG_NOSIGNAL);
        if (w > 0) c.sent += (size_t)w;
        if (c.sent == c.msg->size()) {
          epoll_event ev{};
          ev.events = EPOLLIN;
          ev.data.u64 = ci;
          epoll_ctl(ep, EPOLL_CTL_MOD, c.fd, &ev);
        }
      }
      if (evs[i].events & (EPOLLIN | EPOLLHUP | EPOLLERR)) {
        for (;;) {
          const ssize_t r = recv(c.fd, buf.data(), buf.size(), 0);
          if (r > 0) {
            c.in.append(buf.data(), (size_t)r);
            continue;
          }
          if (r == 0 || (errno != EAGAIN && errno != EWOULDBLOCK)) {   // closed / error: incomplete
            c.done = true;
            ++finished;
          }
          break;
        }
        if (!c.done) {
          if (!c.need) c.need = response_size(c.in, &c.status);
          if (c.need && c.in.size() >= c.need) {
            c.t1 = mono();
            c.done = true;
            G.R->latency[ci] = c.t1 - c.t0;
            G.R->status[ci] = c.status;
            ++finished;
          }
        }
      }
    }
  }
  close(ep);
}

}  // namespace

LoadResult http_burst(const std::string& host, int port, const std::vector<std::string>& msgs,
                      const std::vector<int32_t>& idx, double timeout_s, int nthreads) {
  const size_t n = idx.size();
  LoadResult R;
  R.latency.assign(n, -1.0);
  R.status.assign(n, 0);
  if (n == 0) return R;
  std::vector<Conn> conns(n);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) throw std::runtime_error("bad host " + host);
  const int T = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::max(nthreads, 1), n));
  std::vector<Group> groups(T);
  const double deadline = mono() + timeout_s;
  OnceBarrier ready(T + 1);
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) {
    groups[t] = Group{&conns, n * t / T, n * (t + 1) / T, &a, &msgs, &idx, deadline, &R, {}};
    th.emplace_back(run_group, std::ref(groups[t]), std::ref(ready));
  }
  ready.arrive_and_wait();
  R.t_start = mono();
  for (auto& x : th) x.join();
  R.t_end = 0;
  for (auto& c : conns) R.t_end = std::max(R.t_end, c.t1);
  if (R.t_end == 0) R.t_end = mono();
  for (auto& c : conns)
    if (c.fd >= 0) close(c.fd);
  for (auto& g : groups)
    if (!g.error.empty()) throw std::runtime_error(g.error);
  R.completed = (int64_t)std::count_if(R.latency.begin(), R.latency.end(), [](double x) { return x >= 0; });
  return R;
}

}  // namespace lp
