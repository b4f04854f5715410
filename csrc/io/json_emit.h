// Native JSON emitter for AnalysisResult.events (reference: Jackson serialization of
// MatchedEvent/EventContext, AnalysisService.java:100-107,132-156). Context lines are gathered
// straight from the request byte buffer via the line index, so a large result never
// materialises per-line Python strings.
#pragma once
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

namespace lp {
pybind11::bytes emit_events_json_py(uint64_t buf, pybind11::array_t<int64_t> line_start,
                                    pybind11::array_t<int32_t> line_len, int64_t doc_lo, int64_t doc_hi,
                                    pybind11::array_t<int32_t> ev_line, pybind11::array_t<int32_t> ev_pat,
                                    pybind11::array_t<double> ev_score, pybind11::list pattern_json,
                                    pybind11::array_t<int32_t> ctx_before, pybind11::array_t<int32_t> ctx_after);
}
