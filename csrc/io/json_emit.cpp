#include "json_emit.h"

#include <algorithm>
#include <charconv>
#include <random>
#include <stdexcept>
#include <thread>
#include <string>
#include <vector>

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

void put_str(std::string& o, const uint8_t* s, int64_t n) {
  static const char* hex = "0123456789abcdef";
  o.push_back('"');
  int64_t i = 0;
  while (i < n) {
    int64_t j = i;
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

// events [e0, e1) of one document whose lines are [doc_lo, doc_hi) of the line index
void emit_events(std::string& o, const uint8_t* b, const int64_t* LS, const int32_t* LL, int64_t doc_lo,
                 int64_t doc_hi, const int32_t* EL, const int32_t* EP, const double* ES, int64_t e0, int64_t e1,
                 const PatternTable& T) {
  auto line = [&](int64_t j) { put_str(o, b + LS[j], LL[j]); };
  o.push_back('[');
  for (int64_t e = e0; e < e1; ++e) {
    if (e > e0) o.push_back(',');
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
      const int64_t a = x - bf < doc_lo ? doc_lo : x - bf;
      for (int64_t j = a; j < x; ++j) { if (j > a) o.push_back(','); line(j); }
      o.append("],\"linesAfter\":[");
      const int64_t z = x + 1 + af > doc_hi ? doc_hi : x + 1 + af;
      for (int64_t j = x + 1; j < z; ++j) { if (j > x + 1) o.push_back(','); line(j); }
      o.append("]}");
    }
    o.append(",\"score\":");
    put_double(o, ES[e]);
    o.push_back('}');
  }
  o.push_back(']');
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
  // documents are independent: split them into ranges of ~equal event counts
  const int64_t E = eo[D];
  const int T_ = (int)std::max<int64_t>(1, std::min<int64_t>({(int64_t)nthreads, D, 1 + (E + D) / 2048}));
  if (T_ == 1) {
    run(0, D);
    return;
  }
  std::vector<int64_t> cut(T_ + 1, D);
  cut[0] = 0;
  for (int t = 1; t < T_; ++t) cut[t] = std::max(cut[t - 1], D * t / T_);
  std::vector<std::thread> th;
  for (int t = 0; t < T_; ++t)
    if (cut[t + 1] > cut[t]) th.emplace_back(run, cut[t], cut[t + 1]);
  for (auto& x : th) x.join();
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
  std::vector<std::string> outs(D);
  {
    py::gil_scoped_release nogil;
    const int64_t* dl = doc_line_off.data();
    const int64_t* eo = ev_doc_off.data();
    std::random_device rd;
    const uint64_t seed = ((uint64_t)rd() << 32) ^ rd();
    parallel_docs(eo, D, nthreads, [&](int64_t a, int64_t z) {
      std::mt19937_64 rng(seed ^ (0x9E3779B97F4A7C15ull * (uint64_t)(a + 1)));
      for (int64_t d = a; d < z; ++d) {
        std::string& o = outs[d];
        o.reserve(256 + (size_t)(eo[d + 1] - eo[d]) * 512);
        o.append("{\"analysisId\":\"");
        put_uuid4(o, rng);
        o.append("\",\"metadata\":{\"processingTimeMs\":");
        put_int(o, processing_ms);
        o.append(",\"totalLines\":");
        put_int(o, dl[d + 1] - dl[d]);
        o.append(meta_tail);
        o.append("},\"events\":");
        emit_events(o, reinterpret_cast<const uint8_t*>(buf), line_start.data(), line_len.data(), dl[d], dl[d + 1],
                    ev_line.data(), ev_pat.data(), ev_score.data(), eo[d], eo[d + 1], T);
        o.push_back(',');
        put_summary(o, ev_pat.data(), eo[d], eo[d + 1], T);
        o.push_back('}');
      }
    });
  }
  py::list r;
  for (auto& s : outs) r.append(py::bytes(s));
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
