// Host-side self test for the sanitizer builds: ASan+UBSan and TSan binaries built by
// tools/sanitize_host.sh / tests/test_sanitizers.py from the pure-C++ sources (no HIP, no Python).
//
//  * fuzzes the Java-regex compiler (parser, Glushkov builder, subset construction) with random
//    token strings, and checks the prefilter soundness invariant on random subjects: a line the
//    DFA matches contains at least one of the regex's required literals (ASCII-lowercased);
//  * runs the parallel request-batch packer/splitter (csrc/io/docs.cpp) with 1 and 8 threads on
//    random documents and requires identical results (TSan watches the worker threads);
//  * fuzzes the /parse body decoder (csrc/io/json_in.cpp, untrusted network input) with random
//    byte mutations of valid requests: every input must return one of the 4 statuses without an
//    out-of-bounds access, and the unmutated requests must decode their `logs` exactly;
//  * runs the native HTTP front end (csrc/io/http_server.cpp) with 2 IO threads, a responder
//    thread playing the Python side and 8 client threads on keep-alive connections (TSan watches
//    the queue / outbox / eventfd hand-offs, ASan the connection lifetime).
#include <cstdio>
#include <chrono>
#include <cstring>
#include <functional>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "io/docs.h"
#include "io/json_in.h"
#include "io/http_server.h"

#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>
#include <atomic>
#include <thread>
#include "regex/jregex.h"

using namespace lp;

static int failures = 0;
#define CHECK(c, ...)                         \
  do {                                        \
    if (!(c)) {                               \
      std::fprintf(stderr, "FAIL: " __VA_ARGS__); \
      std::fprintf(stderr, "\n");             \
      ++failures;                             \
    }                                         \
  } while (0)

static std::string lower(const std::string& s) {
  std::string o = s;
  for (auto& c : o)
    if (c >= 'A' && c <= 'Z') c = (char)(c + 32);
  return o;
}

static void fuzz_regex(int iters, uint32_t seed) {
  static const char* toks[] = {"a", "b", "c", "ab", "Error", "x", ".", "*", "+", "?", "|", "(", ")", "(?:", "[",
                               "]", "[a-c]", "[^x]", "\\d", "\\w", "\\s", "\\b", "\\B", "^", "$", "{2}", "{1,3}",
                               "\\.", "(?i)", "é", "\\Q.*\\E", "[[a]&&[b]]", "\\p{L}", "-", "0", "9", " "};
  const int ntok = sizeof(toks) / sizeof(toks[0]);
  std::mt19937 rng(seed);
  int dfa = 0, invalid = 0;
  for (int it = 0; it < iters; ++it) {
    std::string p;
    const int n = 1 + rng() % 10;
    for (int i = 0; i < n; ++i) p += toks[rng() % ntok];
    Compiled c = compile(p, 256, 512);
    if (c.kind == Kind::INVALID) { ++invalid; continue; }
    if (c.kind != Kind::DFA) continue;
    ++dfa;
    for (int s = 0; s < 40; ++s) {
      std::string subj;
      const int m = rng() % 24;
      for (int i = 0; i < m; ++i) subj += "abcxE rRo.9_\n"[rng() % 13];
      if (rng() % 3 == 0) subj += "Error";
      const bool hit = dfa_find(c.dfa, reinterpret_cast<const uint8_t*>(subj.data()), (int64_t)subj.size());
      if (hit && c.has_literals) {
        const std::string ls = lower(subj);
        bool any = false;
        for (auto& lit : c.literals) any |= ls.find(lit) != std::string::npos;
        CHECK(any, "regex %s matched '%s' without any required literal", p.c_str(), subj.c_str());
      }
    }
  }
  std::printf("regex fuzz: %d patterns, %d DFA, %d invalid\n", iters, dfa, invalid);
}

static void docs_threads(uint32_t seed) {
  std::mt19937 rng(seed);
  std::vector<std::string> docs;
  for (int d = 0; d < 3000; ++d) {
    std::string s;
    const int parts = rng() % 40;
    for (int i = 0; i < parts; ++i) {
      s += std::string(rng() % 12, "ab\r x"[rng() % 5]);
      s += (rng() % 4) ? "\n" : "\r\n";
    }
    if (d % 97 == 0) s += std::string(400000, 'z');
    docs.push_back(s);
  }
  std::vector<const char*> src;
  std::vector<int64_t> off(1, 0);
  for (auto& s : docs) { src.push_back(s.data()); off.push_back(off.back() + (int64_t)s.size()); }
  std::vector<uint8_t> b1(off.back() + 1), b8(off.back() + 1);
  DocBatchIndex i1, i8;
  pack_split_docs(src.data(), off.data(), (int64_t)docs.size(), b1.data(), 1, i1);
  pack_split_docs(src.data(), off.data(), (int64_t)docs.size(), b8.data(), 8, i8, 1 << 16);  // force 8 threads
  CHECK(b1 == b8, "packed bytes differ between 1 and 8 threads");
  auto same = [](const auto& x, const auto& y) {
    return x.size() == y.size() && (x.size() == 0 || memcmp(x.data(), y.data(), x.size() * sizeof(x[0])) == 0);
  };
  CHECK(same(i1.line_start, i8.line_start) && same(i1.line_len, i8.line_len) && same(i1.doc_line_off, i8.doc_line_off),
        "line index differs between 1 and 8 threads");
  std::printf("docs: %zu docs, %zu lines\n", docs.size(), i8.line_start.size());
}

static void fuzz_json_in(int iters, uint32_t seed) {
  std::mt19937 rng(seed);
  const std::string base[] = {
      "{\"pod\":{\"metadata\":{\"name\":\"p-1\"}},\"logs\":\"line 1\\nERROR x\\u00e9\\\"q\\\"\\r\\n\"}",
      "{\"logs\":\"a\",\"pod\":{\"spec\":[1,2.5e3,true,null,{\"k\":[]}]},\"events\":[]}",
      " { \"pod\" : { } , \"logs\" : \"\" } "};
  const std::string want[] = {"line 1\nERROR x\xc3\xa9\"q\"\r\n", "a", ""};
  for (int b = 0; b < 3; ++b) {
    PodRequest r;
    const int st = parse_pod_request(reinterpret_cast<const uint8_t*>(base[b].data()), base[b].size(), r);
    CHECK(st == JIN_OK && r.pod_nonnull && r.logs_kind == 1 && r.logs == want[b], "json_in base %d", b);
  }
  static const char bytes[] = "{}[]\",:\\un0123456789.eE+-tfalsrn \t\n\x01\xc3\xa9\xff\xed";
  for (int it = 0; it < iters; ++it) {
    std::string s = base[rng() % 3];
    const int muts = 1 + rng() % 4;
    for (int m = 0; m < muts && !s.empty(); ++m) {
      const size_t at = rng() % s.size();
      switch (rng() % 3) {
        case 0: s[at] = bytes[rng() % (sizeof(bytes) - 1)]; break;
        case 1: s.erase(at, 1 + rng() % 3); break;
        default: s.insert(at, 1, bytes[rng() % (sizeof(bytes) - 1)]); break;
      }
    }
    // exact-size heap copy so ASan flags any read past the end
    std::vector<uint8_t> buf(s.begin(), s.end());
    PodRequest r;
    const int st = parse_pod_request(buf.data(), buf.size(), r);
    CHECK(st >= JIN_OK && st <= JIN_FALLBACK, "json_in status %d", st);
  }
}

// logs_prefetch over exact-size prefix copies (ASan flags a read past the arrived bytes), then the
// resumed final parse: same status and bytes as the one-pass parse
static void fuzz_prefetch(int iters, uint32_t seed) {
  std::mt19937 rng(seed);
  static const char* atoms[] = {"abc ", "\\n", "\\\\", "\\\"", "\\u00e9", "\\u20AC", "\xc3\xa9", "\xf0\x9f\x98\x80",
                                "xxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxx", "\\t", "\x01", "\\q"};
  int resumed = 0;
  for (int it = 0; it < iters; ++it) {
    std::string logs;
    const int na = (int)(rng() % 400);
    const size_t nat = sizeof(atoms) / sizeof(atoms[0]) - (rng() % 8 ? 2 : 0);   // 1 in 8: invalid atoms too
    for (int a = 0; a < na; ++a) logs += atoms[rng() % nat];
    std::string body = "{\"pod\":{\"metadata\":{\"name\":\"p\"}},\"logs\":\"" + logs + "\"}";
    if (rng() % 10 == 0) body.back() = ']';
    const size_t n = body.size();
    std::unique_ptr<char[]> d1(new char[n + 64]), d2(new char[n + 64]);
    PodRequest r1, r2;
    const int s1 = parse_pod_request_into(reinterpret_cast<const uint8_t*>(body.data()), n, r1, d1.get(), n + 64);
    LogsPrefetch pf;
    size_t at = 0;
    while (at < n) {
      at = std::min(n, at + 1 + (size_t)(rng() % (rng() % 4 ? 97 : 4000)));
      std::vector<uint8_t> pre(body.begin(), body.begin() + (ptrdiff_t)at);
      logs_prefetch(pre.data(), pre.size(), pf, d2.get(), n + 64);
    }
    const int s2 = parse_pod_request_into(reinterpret_cast<const uint8_t*>(body.data()), n, r2, d2.get(), n + 64, &pf);
    CHECK(s1 == s2 && r1.logs_kind == r2.logs_kind, "prefetch status %d vs %d", s2, s1);
    if (s1 == JIN_OK && r1.logs_kind == 1) {
      CHECK(r1.logs_dlen == r2.logs_dlen && memcmp(d1.get(), d2.get(), r1.logs_dlen) == 0, "prefetch bytes differ");
      resumed += pf.state >= 1;
    }
  }
  CHECK(resumed > iters / 2, "prefetch resumed only %d of %d", resumed, iters);
  std::printf("prefetch: %d bodies, %d resumed\n", iters, resumed);
}

// large /parse bodies written in small pieces with pauses: the IO thread prefetches between reads
static void http_prefetch_selftest(int rounds) {
  HttpServer srv("127.0.0.1", 0, 2, 8 << 20);
  std::atomic<bool> done{false};
  std::thread responder([&] {
    while (!done)
      for (auto& r : srv.next_requests(16, 20)) {
        const size_t n = r.kind == 0 && r.dec.p ? r.logs_dlen : (size_t)-1;
        const uint64_t h = n == (size_t)-1 ? 0 : std::hash<std::string>()(std::string(r.dec.p, n));
        srv.respond(r.id, 200, "application/json", "{\"n\":" + std::to_string(n) + ",\"h\":" + std::to_string(h) + "}");
      }
  });
  const int fd = socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)srv.port());
  inet_pton(AF_INET, "127.0.0.1", &a.sin_addr);
  int ok = 0;
  if (connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) == 0) {
    for (int i = 0; i < rounds; ++i) {
      std::string logs, raw;
      for (int k = 0; k < 3000 + 500 * i; ++k) {
        logs += "ERROR line " + std::to_string(k) + " \xc3\xa9\"q\"\n";
        raw += "ERROR line " + std::to_string(k) + " \xc3\xa9\\\"q\\\"\\n";
      }
      const std::string body = "{\"pod\":{},\"logs\":\"" + raw + "\"}";
      const std::string req = "POST /parse HTTP/1.1\r\nContent-Length: " + std::to_string(body.size()) + "\r\n\r\n" + body;
      size_t off = 0;
      while (off < req.size()) {
        const size_t k = std::min(req.size() - off, (size_t)(1000 + 7919 * (off % 13)));
        if (send(fd, req.data() + off, k, 0) != (ssize_t)k) break;
        off += k;
        if (off % 5 == 0) std::this_thread::sleep_for(std::chrono::microseconds(200));
      }
      std::string resp;
      char b[4096];
      while (resp.find("\r\n\r\n") == std::string::npos || resp.back() != '}') {
        const ssize_t k = recv(fd, b, sizeof(b), 0);
        if (k <= 0) break;
        resp.append(b, (size_t)k);
      }
      const std::string want = "{\"n\":" + std::to_string(logs.size()) + ",\"h\":" + std::to_string(std::hash<std::string>()(logs)) + "}";
      ok += resp.rfind(want) != std::string::npos;
    }
    close(fd);
  }
  done = true;
  responder.join();
  const uint64_t pre = srv.stages.prefetched.load(), pump_ns = srv.stages.pump_prefetch_ns.load();
  srv.stop();
  CHECK(ok == rounds, "http prefetch: %d of %d responses", ok, rounds);
  CHECK(pre > 0, "http prefetch: no body was prefetched");
  CHECK(pump_ns > 0, "http prefetch: the responder (pump) thread decoded nothing while bodies arrived");
  std::printf("http prefetch: %d large bodies, %llu prefetched\n", ok, (unsigned long long)pre);
}

// burst mode (server.io-decode-max-conns exceeded; here the limit is 0 and the arrival-time decode
// off): large bodies reach the consumer undecoded -- no decode buffer -- and the raw logs span
// decodes to the same text
static void http_undecoded_selftest(int rounds) {
  HttpOptions o;
  o.prefetch = false;
  o.io_decode_max_conns = 0;
  HttpServer srv("127.0.0.1", 0, 2, 8 << 20, 60.0, o);
  std::atomic<bool> done{false};
  std::atomic<int> with_dec{0};
  std::thread responder([&] {
    while (!done)
      for (auto& r : srv.next_requests(16, 20)) {
        size_t n = (size_t)-1;
        uint64_t h = 0;
        if (r.kind == 0) {
          if (r.dec.p) ++with_dec;
          std::string logs(r.logs_len + 64, '\0');
          n = decode_json_string(reinterpret_cast<const uint8_t*>(r.body.data()) + r.logs_off, r.logs_len, &logs[0]);
          h = std::hash<std::string>()(std::string(logs.data(), n));
          srv.recycle(std::move(r.body));
        }
        srv.respond(r.id, 200, "application/json", "{\"n\":" + std::to_string(n) + ",\"h\":" + std::to_string(h) + "}");
      }
  });
  const int fd = socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)srv.port());
  inet_pton(AF_INET, "127.0.0.1", &a.sin_addr);
  int ok = 0;
  if (connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) == 0) {
    for (int i = 0; i < rounds; ++i) {
      std::string logs, raw;
      for (int k = 0; k < 500 + 700 * i; ++k) {
        logs += "WARN line " + std::to_string(k) + " \xc3\xa9\t\"q\"\n";
        raw += "WARN line " + std::to_string(k) + " \xc3\xa9\\t\\\"q\\\"\\n";
      }
      const std::string body = "{\"pod\":{},\"logs\":\"" + raw + "\"}";
      const std::string req = "POST /parse HTTP/1.1\r\nContent-Length: " + std::to_string(body.size()) + "\r\n\r\n" + body;
      if (send(fd, req.data(), req.size(), 0) != (ssize_t)req.size()) break;
      std::string resp;
      char b[4096];
      while (resp.find("\r\n\r\n") == std::string::npos || resp.back() != '}') {
        const ssize_t k = recv(fd, b, sizeof(b), 0);
        if (k <= 0) break;
        resp.append(b, (size_t)k);
      }
      const std::string want = "{\"n\":" + std::to_string(logs.size()) + ",\"h\":" + std::to_string(std::hash<std::string>()(logs)) + "}";
      ok += resp.rfind(want) != std::string::npos;
    }
    close(fd);
  }
  done = true;
  responder.join();
  const uint64_t pre = srv.stages.prefetched.load();
  srv.stop();
  CHECK(ok == rounds, "http undecoded: %d of %d responses", ok, rounds);
  CHECK(with_dec.load() == 0, "http undecoded: %d bodies were decoded by the IO thread", with_dec.load());
  CHECK(pre == 0, "http undecoded: a body was prefetched");
  std::printf("http undecoded (burst mode): %d bodies\n", ok);
}

static void http_selftest(int rounds) {
  HttpServer srv("127.0.0.1", 0, 2, 1 << 20);
  std::atomic<bool> done{false};
  std::atomic<int> served{0};
  std::thread responder([&] {
    while (!done) {
      for (auto& r : srv.next_requests(64, 20)) {
        size_t n = 0;
        if (r.kind == 0) {   // the bindings' path: unescape the raw span, recycle the buffer
          std::string logs(r.logs_len + 64, '\0');
          n = decode_json_string(reinterpret_cast<const uint8_t*>(r.body.data()) + r.logs_off, r.logs_len, &logs[0]);
          srv.recycle(std::move(r.body));
        }
        const std::string body = r.kind == 0 ? "{\"n\":" + std::to_string(n) + "}" : "{}";
        srv.respond(r.id, 200, "application/json", body);
        ++served;
      }
    }
  });
  std::atomic<int> ok{0};
  std::vector<std::thread> clients;
  for (int t = 0; t < 8; ++t)
    clients.emplace_back([&, t] {
      const int fd = socket(AF_INET, SOCK_STREAM, 0);
      sockaddr_in a{};
      a.sin_family = AF_INET;
      a.sin_port = htons((uint16_t)srv.port());
      inet_pton(AF_INET, "127.0.0.1", &a.sin_addr);
      if (connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) return;
      for (int i = 0; i < rounds; ++i) {
        const std::string logs(100 + 37 * ((t + i) % 11), 'x');
        const std::string body = "{\"pod\":{},\"logs\":\"" + logs + "\"}";
        const std::string req = (i % 5 == 4) ? std::string("GET /health HTTP/1.1\r\n\r\n")
                                             : "POST /parse HTTP/1.1\r\nContent-Length: " +
                                                   std::to_string(body.size()) + "\r\n\r\n" + body;
        if (send(fd, req.data(), req.size(), 0) != (ssize_t)req.size()) break;
        std::string resp;
        char b[4096];
        while (resp.find("\r\n\r\n") == std::string::npos || resp.back() != '}') {
          const ssize_t k = recv(fd, b, sizeof(b), 0);
          if (k <= 0) break;
          resp.append(b, (size_t)k);
        }
        const std::string want = (i % 5 == 4) ? "{\"status\":\"UP\"}" : "{\"n\":" + std::to_string(logs.size()) + "}";
        if (resp.rfind(want) != std::string::npos) ++ok;
      }
      close(fd);
    });
  for (auto& c : clients) c.join();
  done = true;
  responder.join();
  srv.stop();
  CHECK(ok == 8 * rounds, "http: %d of %d responses", ok.load(), 8 * rounds);
  std::printf("http: %d requests over 8 keep-alive connections\n", ok.load());
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 3000;
  fuzz_regex(iters, 12345);
  docs_threads(777);
  fuzz_json_in(iters * 10, 4242);
  fuzz_prefetch(iters / 3 + 50, 99);
  http_selftest(iters / 20 + 10);
  http_prefetch_selftest(12);
  http_undecoded_selftest(8);
  const uint8_t t[] = {'a', 0xE2, 0x80, 0xA8};
  CHECK(final_terminator_len(t, 4) == 3, "U+2028 final terminator");
  std::printf("%s (%d failures)\n", failures ? "FAILED" : "OK", failures);
  return failures ? 1 : 0;
}
