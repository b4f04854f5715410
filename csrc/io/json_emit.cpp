#include "json_emit.h"

#if defined(__SSE2__)
#include <emmintrin.h>
#endif

#if defined(__x86_64__)
#include <immintrin.h>
#endif
#include <algorithm>
#include <atomic>
#include <charconv>
#include <random>
#include <stdexcept>
#include <thread>
#include <string>
#include <vector>

#include "kernels/lp_host.h"

namespace py = pybind11;

namespace lp {
namespace {

// bytes that need a JSON escape: '"', '\\' and control characters
struct EscTable {
  bool esc[256];
  constexpr EscTable() : esc() {
    for (int c = 0; c < 256; ++c) esc[c] = c < 0x20 || c == '"' || c == '\\';
  }
};
constexpr EscTable kEsc;

#if defined(__x86_64__)
// first byte of s[j, n) that needs an escape (n if none), 64 bytes per step (AVX-512BW): a log line's
// ~100 clean bytes take two compares instead of six 16-byte steps
__attribute__((target("avx512f,avx512bw,bmi,bmi2"))) int64_t clean_run_512(const uint8_t* s, int64_t j, int64_t n) {
  const __m512i q = _mm512_set1_epi8('"'), bs = _mm512_set1_epi8('\\'), sp = _mm512_set1_epi8(0x20);
  while (j + 64 <= n) {
    const __m512i v = _mm512_loadu_si512(reinterpret_cast<const void*>(s + j));
    const uint64_t m = _mm512_cmpeq_epi8_mask(v, q) | _mm512_cmpeq_epi8_mask(v, bs) | _mm512_cmplt_epu8_mask(v, sp);
    if (m) return j + (int64_t)__builtin_ctzll(m);
    j += 64;
  }
  if (j < n) {                                   // masked tail load: no byte past n is read
    const __mmask64 k = _bzhi_u64(~0ull, (unsigned)(n - j));
    const __m512i v = _mm512_maskz_loadu_epi8(k, reinterpret_cast<const void*>(s + j));
    const uint64_t m = (_mm512_cmpeq_epi8_mask(v, q) | _mm512_cmpeq_epi8_mask(v, bs) | _mm512_cmplt_epu8_mask(v, sp)) & k;
    return m ? j + (int64_t)__builtin_ctzll(m) : n;
  }
  return n;
}
bool have_avx512bw() {
  static const bool ok = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
                         __builtin_cpu_supports("bmi") && __builtin_cpu_supports("bmi2");
  return ok;
}
#endif

void put_str(std::string& o, const uint8_t* s, int64_t n) {
  static const char* hex = "0123456789abcdef";
  o.push_back('"');
  int64_t i = 0;
#if defined(__x86_64__)
  const bool wide = have_avx512bw();
#endif
  while (i < n) {
    int64_t j = i;
#if defined(__x86_64__)
    if (wide) j = clean_run_512(s, j, n);
#endif
#if defined(__SSE2__)
    // 16 bytes per step: '"', '\\' and control bytes (<= 0x1F: saturating c - 0x1F == 0) end a run
    {
      const __m128i q = _mm_set1_epi8('"'), bs = _mm_set1_epi8('\\'), lim = _mm_set1_epi8(0x1F);
      while (j + 16 <= n) {
        const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + j));
        const __m128i m = _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(v, q), _mm_cmpeq_epi8(v, bs)),
                                       _mm_cmpeq_epi8(_mm_subs_epu8(v, lim), _mm_setzero_si128()));
        const int bits = _mm_movemask_epi8(m);
        if (bits) {
          j += __builtin_ctz((unsigned)bits);
          break;
        }
        j += 16;
      }
    }
#endif
    while (j < n && !kEsc.esc[s[j]]) ++j;       // copy clean runs in one append
    if (j > i) o.append(reinterpret_cast<const char*>(s + i), (size_t)(j - i));
    if (j >= n) break;
    const uint8_t c = s[j];
    switch (c) {
      case '"': o.append("\\\""); break;
      case '\\': o.append("\\\\"); break;
      case '\n': o.append("\\n"); break;
      case '\r': o.append("\\r"); break;
      case '\t': o.append("\\t"); break;
      case '\b': o.append("\\b"); break;
      case '\f': o.append("\\f"); break;
      default:
        o.append("\\u00");
        o.push_back(hex[c >> 4]);
        o.push_back(hex[c & 15]);
    }
    i = j + 1;
  }
  o.push_back('"');
}

void put_double(std::string& o, double v) {
  char b[64];
  auto r = std::to_chars(b, b + sizeof(b), v);
  o.append(b, r.ptr);
}

void put_int(std::string& o, int64_t v) {
  char b[32];
  auto r = std::to_chars(b, b + sizeof(b), v);
  o.append(b, r.ptr);
}

// events [a, z) of a document whose lines are [doc_lo, doc_hi) of the line index, without the
// enclosing brackets; a comma precedes every event but the document's first (index e_first)
void emit_event_range(std::string& o, const uint8_t* b, const int64_t* LS, const int32_t* LL, int64_t doc_lo,
                      int64_t doc_hi, const int32_t* EL, const int32_t* EP, const double* ES, int64_t a, int64_t z,
                      int64_t e_first, const PatternTable& T) {
  auto line = [&](int64_t j) { put_str(o, b + LS[j], LL[j]); };
  for (int64_t e = a; e < z; ++e) {
    if (e > e_first) o.push_back(',');
    const int64_t x = EL[e];
    const int32_t p = EP[e];
    o.append("{\"lineNumber\":");
    put_int(o, x - doc_lo + 1);
    o.append(",\"matchedPattern\":");
    o.append(T.json[p]);
    o.append(",\"context\":{\"matchedLine\":");
    line(x);
    const int32_t bf = T.before[p], af = T.after[p];
    if (bf < 0) {
      o.append(",\"linesBefore\":null,\"linesAfter\":null}");
    } else {
      o.append(",\"linesBefore\":[");
      const int64_t lo = x - bf < doc_lo ? doc_lo : x - bf;
      for (int64_t j = lo; j < x; ++j) { if (j > lo) o.push_back(','); line(j); }
      o.append("],\"linesAfter\":[");
      const int64_t hi = x + 1 + af > doc_hi ? doc_hi : x + 1 + af;
      for (int64_t j = x + 1; j < hi; ++j) { if (j > x + 1) o.push_back(','); line(j); }
      o.append("]}");
    }
    o.append(",\"score\":");
    put_double(o, ES[e]);
    o.push_back('}');
  }
}

// events [e0, e1) of one document whose lines are [doc_lo, doc_hi) of the line index
void emit_events(std::string& o, const uint8_t* b, const int64_t* LS, const int32_t* LL, int64_t doc_lo,
                 int64_t doc_hi, const int32_t* EL, const int32_t* EP, const double* ES, int64_t e0, int64_t e1,
                 const PatternTable& T) {
  o.push_back('[');
  emit_event_range(o, b, LS, LL, doc_lo, doc_hi, EL, EP, ES, e0, e1, e0, T);
  o.push_back(']');
}

// per-call UUID seed: one entropy read per process (std::random_device per call opened the
// entropy source on every request), then a splitmix64 sequence
uint64_t uuid_seed() {
  static const uint64_t base = [] {
    std::random_device rd;
    return ((uint64_t)rd() << 32) ^ rd();
  }();
  static std::atomic<uint64_t> ctr{0};
  uint64_t z = base + 0x9E3779B97F4A7C15ull * (ctr.fetch_add(1, std::memory_order_relaxed) + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// RFC 4122 version-4 UUID (UUID.randomUUID, AnalysisService.java:117)
void put_uuid4(std::string& o, std::mt19937_64& rng) {
  static const char* hex = "0123456789abcdef";
  uint64_t a = rng(), b = rng();
  a = (a & 0xFFFFFFFFFFFF0FFFull) | 0x0000000000004000ull;   // version 4
  b = (b & 0x3FFFFFFFFFFFFFFFull) | 0x8000000000000000ull;   // variant 10
  char u[36];
  int k = 0;
  for (int i = 0; i < 32; ++i) {
    if (i == 8 || i == 12 || i == 16 || i == 20) u[k++] = '-';
    const uint64_t w = i < 16 ? a : b;
    u[k++] = hex[(w >> (60 - 4 * (i & 15))) & 15];
  }
  o.append(u, 36);
}

// summary of events [e0, e1) (AnalysisService.java:188-215): count, severity histogram in
// first-occurrence order, highest = max rank among known severities, else the first event's
void put_summary(std::string& o, const int32_t* EP, int64_t e0, int64_t e1, const PatternTable& T) {
  o.append("\"summary\":{\"significantEvents\":");
  put_int(o, e1 - e0);
  if (e1 == e0) {
    o.append(",\"highestSeverity\":\"NONE\",\"severityDistribution\":{}}");
    return;
  }
  std::vector<std::pair<const std::string*, int64_t>> dist;   // distinct severities, in order
  std::vector<int32_t> rank;
  for (int64_t e = e0; e < e1; ++e) {
    const std::string* s = &T.sev_json[EP[e]];
    bool found = false;
    for (auto& kv : dist)
      if (*kv.first == *s) { ++kv.second; found = true; break; }
    if (!found) {
      dist.emplace_back(s, 1);
      rank.push_back(T.sev_rank[EP[e]]);
    }
  }
  size_t best = 0;
  int32_t br = -1;
  for (size_t i = 0; i < dist.size(); ++i)
    if (rank[i] > br) { br = rank[i]; best = i; }
  o.append(",\"highestSeverity\":");
  o.append(br >= 0 ? *dist[best].first : T.sev_json[EP[e0]]);
  o.append(",\"severityDistribution\":{");
  for (size_t i = 0; i < dist.size(); ++i) {
    if (i) o.push_back(',');
    o.append(*dist[i].first);
    o.push_back(':');
    put_int(o, dist[i].second);
  }
  o.append("}}");
}

template <class F>
void parallel_docs(const int64_t* eo, int64_t D, int nthreads, F&& run) {
  // documents are independent: ranges of ~equal document counts on the host pool
  const int64_t E = eo[D];
  const int T_ = (int)std::max<int64_t>(1, std::min<int64_t>({(int64_t)nthreads, D, 1 + (E + D) / 2048}));
  if (T_ == 1) {
    run(0, D);
    return;
  }
  HostPool::get().run(T_, T_, [&](int64_t t) { run(D * t / T_, D * (t + 1) / T_); });
}

// events [e0, e1) of one document, emitted in `chunks` pieces on the host pool and joined (a
// single large request is one document: its ~1 KB-per-event context text is the emitter's work)
void emit_events_parallel(std::string& o, const uint8_t* b, const int64_t* LS, const int32_t* LL, int64_t doc_lo,
                          int64_t doc_hi, const int32_t* EL, const int32_t* EP, const double* ES, int64_t e0,
                          int64_t e1, const PatternTable& T, int nthreads) {
  const int64_t n = e1 - e0;
  // >= 2048 events per helper: below that the caller's cache-hot serial loop wins (see docs.cpp)
  const int chunks = (int)std::max<int64_t>(1, std::min<int64_t>(nthreads, n / 2048));
  if (chunks <= 1) {
    emit_events(o, b, LS, LL, doc_lo, doc_hi, EL, EP, ES, e0, e1, T);
    return;
  }
  std::vector<std::string> part(chunks);
  HostPool::get().run(chunks, chunks, [&](int64_t c) {
    const int64_t a = e0 + n * c / chunks, z = e0 + n * (c + 1) / chunks;
    std::string& s = part[c];
    s.reserve((size_t)(z - a) * 1536);
    emit_event_range(s, b, LS, LL, doc_lo, doc_hi, EL, EP, ES, a, z, e0, T);
  });
  size_t tot = 2;
  for (auto& s : part) tot += s.size();
  o.reserve(o.size() + tot);
  o.push_back('[');
  for (auto& s : part) o.append(s);
  o.push_back(']');
}

}  // namespace

void PatternTable::set_severity(py::list sev, py::array_t<int32_t> rank) {
  sev_json.clear();
  sev_rank.clear();
  auto R = rank.unchecked<1>();
  py::ssize_t i = 0;
  for (auto h : sev) {
    const std::string s = h.cast<std::string>();
    std::string j;
    put_str(j, reinterpret_cast<const uint8_t*>(s.data()), (int64_t)s.size());
    sev_json.push_back(j);
    sev_rank.push_back(R(i++));
  }
}

py::list emit_batch_results_py(const PatternTable& T, uint64_t buf, py::array_t<int64_t> line_start,
                               py::array_t<int32_t> line_len, py::array_t<int64_t> doc_line_off,
                               py::array_t<int32_t> ev_line, py::array_t<int32_t> ev_pat,
                               py::array_t<double> ev_score, py::array_t<int64_t> ev_doc_off,
                               int64_t processing_ms, const std::string& meta_tail, int nthreads) {
  const int64_t D = doc_line_off.shape(0) - 1;
  if ((int64_t)T.sev_json.size() < (int64_t)T.json.size()) throw std::runtime_error("PatternTable: severities not set");
  // per calling thread, recycled: a fresh ~130 KB response buffer per request was an mmap'd
  // allocation whose pages faulted in on first write (and unmapped after the bytes copy)
  static thread_local std::vector<std::string> tl_outs;
  if ((int64_t)tl_outs.size() < D) tl_outs.resize((size_t)D);
  std::vector<std::string>& outs = tl_outs;
  for (int64_t d = 0; d < D; ++d) outs[d].clear();
  {
    py::gil_scoped_release nogil;
    const int64_t* dl = doc_line_off.data();
    const int64_t* eo = ev_doc_off.data();
    const uint64_t seed = uuid_seed();
    const bool one = D == 1;            // one document: parallel over its events instead
    parallel_docs(eo, D, nthreads, [&](int64_t a, int64_t z) {
      std::mt19937_64 rng(seed ^ (0x9E3779B97F4A7C15ull * (uint64_t)(a + 1)));
      for (int64_t d = a; d < z; ++d) {
        std::string& o = outs[d];
        o.reserve(256 + (size_t)(eo[d + 1] - eo[d]) * 1536);
        o.append("{\"analysisId\":\"");
        put_uuid4(o, rng);
        o.append("\",\"metadata\":{\"processingTimeMs\":");
        put_int(o, processing_ms);
        o.append(",\"totalLines\":");
        put_int(o, dl[d + 1] - dl[d]);
        o.append(meta_tail);
        o.append("},\"events\":");
        emit_events_parallel(o, reinterpret_cast<const uint8_t*>(buf), line_start.data(), line_len.data(), dl[d],
                             dl[d + 1], ev_line.data(), ev_pat.data(), ev_score.data(), eo[d], eo[d + 1], T,
                             one ? nthreads : 1);
        o.push_back(',');
        put_summary(o, ev_pat.data(), eo[d], eo[d + 1], T);
        o.push_back('}');
      }
    });
  }
  py::list r;
  for (int64_t d = 0; d < D; ++d) r.append(py::bytes(outs[d]));
  // keep what a request-sized response needs; give back what a burst batch grew
  size_t held = 0;
  for (auto& o : outs) held += o.capacity();
  if (held > (size_t(64) << 20) || outs.size() > 4096) {
    std::vector<std::string>().swap(outs);
  }
  return r;
}

PatternTable::PatternTable(py::list pattern_json, py::array_t<int32_t> ctx_before, py::array_t<int32_t> ctx_after) {
  json.reserve(pattern_json.size());
  for (auto h : pattern_json) json.push_back(h.cast<std::string>());
  auto B = ctx_before.unchecked<1>();
  auto A = ctx_after.unchecked<1>();
  for (py::ssize_t i = 0; i < B.shape(0); ++i) { before.push_back(B(i)); after.push_back(A(i)); }
}

py::bytes emit_events_json_py(const PatternTable& T, uint64_t buf, py::array_t<int64_t> line_start,
                              py::array_t<int32_t> line_len, int64_t doc_lo, int64_t doc_hi,
                              py::array_t<int32_t> ev_line, py::array_t<int32_t> ev_pat,
                              py::array_t<double> ev_score) {
  const int64_t n = ev_line.shape(0);
  std::string o;
  o.reserve((size_t)n * 512 + 16);
  {
    py::gil_scoped_release nogil;
    emit_events(o, reinterpret_cast<const uint8_t*>(buf), line_start.data(), line_len.data(), doc_lo, doc_hi,
                ev_line.data(), ev_pat.data(), ev_score.data(), 0, n, T);
  }
  return py::bytes(o);
}

py::list emit_batch_json_py(const PatternTable& T, uint64_t buf, py::array_t<int64_t> line_start,
                            py::array_t<int32_t> line_len, py::array_t<int64_t> doc_line_off,
                            py::array_t<int32_t> ev_line, py::array_t<int32_t> ev_pat,
                            py::array_t<double> ev_score, py::array_t<int64_t> ev_doc_off, int nthreads) {
  const int64_t D = doc_line_off.shape(0) - 1;
  std::vector<std::string> outs(D);
  {
    py::gil_scoped_release nogil;
    const int64_t* dl = doc_line_off.data();
    const int64_t* eo = ev_doc_off.data();
    auto run = [&](int64_t a, int64_t z) {
      for (int64_t d = a; d < z; ++d)
        emit_events(outs[d], reinterpret_cast<const uint8_t*>(buf), line_start.data(), line_len.data(), dl[d],
                    dl[d + 1], ev_line.data(), ev_pat.data(), ev_score.data(), eo[d], eo[d + 1], T);
    };
    // documents are independent: split them into ranges of ~equal event counts
    const int64_t E = eo[D];
    const int T_ = (int)std::max<int64_t>(1, std::min<int64_t>({(int64_t)nthreads, D, 1 + E / 2048}));
    if (T_ == 1) {
      run(0, D);
    } else {
      std::vector<int64_t> cut(T_ + 1, D);
      cut[0] = 0;
      for (int t = 1; t < T_; ++t)
        cut[t] = std::max(cut[t - 1], (int64_t)(std::upper_bound(eo, eo + D + 1, E / T_ * t) - eo - 1));
      std::vector<std::thread> th;
      for (int t = 0; t < T_; ++t)
        if (cut[t + 1] > cut[t]) th.emplace_back(run, cut[t], cut[t + 1]);
      for (auto& x : th) x.join();
    }
  }
  py::list r;
  for (auto& s : outs) r.append(py::bytes(s));
  return r;
}

}  // namespace lp
