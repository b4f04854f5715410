// Request-batch staging for continuous batching: pack many request bodies into one (pinned)
// staging buffer and build the per-document Java String.split("\\r?\\n") line index, in parallel
// across documents. One host copy per byte (the reference-equivalent of reading the request).
#pragma once
#include <cstdint>
#include <vector>

namespace lp {

struct DocBatchIndex {
  std::vector<int64_t> line_start;   // absolute offsets into the packed buffer
  std::vector<int32_t> line_len;     // '\r' before '\n' excluded
  std::vector<int64_t> doc_line_off; // D+1
};

// src[d], len[d]: document bytes; dst receives them back to back at doc_off (D+1, prefix sums).
// nthreads <= 1 runs inline.
void pack_split_docs(const char* const* src, const int64_t* doc_off, int64_t D, uint8_t* dst, int nthreads,
                     DocBatchIndex& out);

}  // namespace lp
