#include "json_emit.h"

#include <algorithm>
#include <charconv>
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

}  // namespace

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
