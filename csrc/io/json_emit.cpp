#include "json_emit.h"

#include <charconv>
#include <string>
#include <vector>

namespace py = pybind11;

namespace lp {
namespace {

void put_str(std::string& o, const uint8_t* s, int64_t n) {
  static const char* hex = "0123456789abcdef";
  o.push_back('"');
  for (int64_t i = 0; i < n; ++i) {
    const uint8_t c = s[i];
    switch (c) {
      case '"': o.append("\\\""); break;
      case '\\': o.append("\\\\"); break;
      case '\n': o.append("\\n"); break;
      case '\r': o.append("\\r"); break;
      case '\t': o.append("\\t"); break;
      case '\b': o.append("\\b"); break;
      case '\f': o.append("\\f"); break;
      default:
        if (c < 0x20) {
          o.append("\\u00");
          o.push_back(hex[c >> 4]);
          o.push_back(hex[c & 15]);
        } else {
          o.push_back((char)c);
        }
    }
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

}  // namespace

py::bytes emit_events_json_py(uint64_t buf, py::array_t<int64_t> line_start, py::array_t<int32_t> line_len,
                              int64_t doc_lo, int64_t doc_hi, py::array_t<int32_t> ev_line,
                              py::array_t<int32_t> ev_pat, py::array_t<double> ev_score, py::list pattern_json,
                              py::array_t<int32_t> ctx_before, py::array_t<int32_t> ctx_after) {
  const uint8_t* b = reinterpret_cast<const uint8_t*>(buf);
  auto LS = line_start.unchecked<1>();
  auto LL = line_len.unchecked<1>();
  auto EL = ev_line.unchecked<1>();
  auto EP = ev_pat.unchecked<1>();
  auto ES = ev_score.unchecked<1>();
  auto CB = ctx_before.unchecked<1>();
  auto CA = ctx_after.unchecked<1>();
  std::vector<std::string> pj;
  pj.reserve(pattern_json.size());
  for (auto h : pattern_json) pj.push_back(h.cast<std::string>());
  const int64_t n = EL.shape(0);
  std::string o;
  o.reserve((size_t)n * 512 + 16);
  {
    py::gil_scoped_release nogil;
    auto line = [&](int64_t j) { put_str(o, b + LS(j), LL(j)); };
    o.push_back('[');
    for (int64_t e = 0; e < n; ++e) {
      if (e) o.push_back(',');
      const int64_t x = EL(e);
      const int32_t p = EP(e);
      o.append("{\"lineNumber\":");
      put_int(o, x - doc_lo + 1);
      o.append(",\"matchedPattern\":");
      o.append(pj[p]);
      o.append(",\"context\":{\"matchedLine\":");
      line(x);
      const int32_t bf = CB(p), af = CA(p);
      if (bf < 0) {
        o.append(",\"linesBefore\":null,\"linesAfter\":null}");
      } else {
        o.append(",\"linesBefore\":[");
        int64_t a = x - bf < doc_lo ? doc_lo : x - bf;
        for (int64_t j = a; j < x; ++j) { if (j > a) o.push_back(','); line(j); }
        o.append("],\"linesAfter\":[");
        int64_t z = x + 1 + af > doc_hi ? doc_hi : x + 1 + af;
        for (int64_t j = x + 1; j < z; ++j) { if (j > x + 1) o.push_back(','); line(j); }
        o.append("]}");
      }
      o.append(",\"score\":");
      put_double(o, ES(e));
      o.push_back('}');
    }
    o.push_back(']');
  }
  return py::bytes(o);
}

}  // namespace lp
