// Native JSON emitter for AnalysisResult.events (reference: Jackson serialization of
// MatchedEvent/EventContext, AnalysisService.java:100-107,132-156). Context lines are gathered
// straight from the request byte buffer via the line index, so a large result never
// materialises per-line Python strings. The pattern echo (matchedPattern, snake_case JSON) is
// serialised once per library into a PatternTable and spliced per event.
#pragma once
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <string>
#include <vector>

namespace lp {

struct PatternTable {
  std::vector<std::string> json;
  std::vector<int32_t> before, after;   // context rules, -1 = null rules
  std::vector<std::string> sev_json;    // upper-cased severity as a JSON string
  std::vector<int32_t> sev_rank;        // index in [INFO, LOW, MEDIUM, HIGH, CRITICAL], -1 unknown
  PatternTable(pybind11::list pattern_json, pybind11::array_t<int32_t> ctx_before,
               pybind11::array_t<int32_t> ctx_after);
  void set_severity(pybind11::list sev, pybind11::array_t<int32_t> rank);
};

pybind11::bytes emit_events_json_py(const PatternTable& T, uint64_t buf, pybind11::array_t<int64_t> line_start,
                                    pybind11::array_t<int32_t> line_len, int64_t doc_lo, int64_t doc_hi,
                                    pybind11::array_t<int32_t> ev_line, pybind11::array_t<int32_t> ev_pat,
                                    pybind11::array_t<double> ev_score);

// one call per request batch: returns the events array JSON of every document
pybind11::list emit_batch_json_py(const PatternTable& T, uint64_t buf, pybind11::array_t<int64_t> line_start,
                                  pybind11::array_t<int32_t> line_len, pybind11::array_t<int64_t> doc_line_off,
                                  pybind11::array_t<int32_t> ev_line, pybind11::array_t<int32_t> ev_pat,
                                  pybind11::array_t<double> ev_score, pybind11::array_t<int64_t> ev_doc_off,
                                  int nthreads);
// one call per request batch: the complete AnalysisResult JSON of every document
// (AnalysisService.java:115-121 + buildMetadata :166-180 + buildSummary :188-215); `meta_tail`
// = ',"analyzedAt":"...","patternsUsed":[...]' (+ optional extra fields), shared by the batch
pybind11::list emit_batch_results_py(const PatternTable& T, uint64_t buf, pybind11::array_t<int64_t> line_start,
                                     pybind11::array_t<int32_t> line_len, pybind11::array_t<int64_t> doc_line_off,
                                     pybind11::array_t<int32_t> ev_line, pybind11::array_t<int32_t> ev_pat,
                                     pybind11::array_t<double> ev_score, pybind11::array_t<int64_t> ev_doc_off,
                                     int64_t processing_ms, const std::string& meta_tail, int nthreads);
}  // namespace lp
