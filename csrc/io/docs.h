// Request-batch staging for continuous batching: pack many request bodies into one (pinned)
// staging buffer and build the per-document Java String.split("\\r?\\n") line index, in parallel
// across documents. One host copy per byte (the reference-equivalent of reading the request).
#pragma once
#include <cstddef>
#include <cstdint>
#include <memory>
#include <vector>

namespace lp {

// Uninitialised, releasable array: the line index is written once and handed to numpy without a
// zero-fill or a copy (1.9M lines = 23 MB per 2k-request batch).
template <class T>
struct RawBuf {
  std::unique_ptr<T[]> p;
  size_t n = 0;
  void alloc(size_t k) {
    p.reset(new T[k > 0 ? k : 1]);
    n = k;
  }
  T* data() { return p.get(); }
  const T* data() const { return p.get(); }
  size_t size() const { return n; }
  bool empty() const { return n == 0; }
  T& operator[](size_t i) { return p[i]; }
  const T& operator[](size_t i) const { return p[i]; }
  T* release() {
    n = 0;
    return p.release();
  }
};

struct DocBatchIndex {
  RawBuf<int64_t> line_start;   // absolute offsets into the packed buffer
  RawBuf<int32_t> line_len;     // '\r' before '\n' excluded
  RawBuf<int64_t> doc_line_off; // D+1
  // caller-provided destination (e.g. pinned memory the device copies from directly): used when
  // the line count fits `ext_cap`; line_start / line_len then stay empty and `external` is set
  int64_t* ext_start = nullptr;
  int32_t* ext_len = nullptr;
  int64_t ext_cap = 0;
  bool external = false;
};

// src[d], len[d]: document bytes; dst receives them back to back at doc_off (D+1, prefix sums).
// nthreads <= 1 runs inline. nlpos[d] (optional, non-null per document): the positions of document
// d's '\n' bytes, nlcnt[d] of them, already known (the HTTP front end's decoder recorded them) --
// that document is copied without a newline scan.
// dst[0, n) = src[0, n) through the cache (AVX-512 stores; glibc's memcpy streams megabyte copies
// past it, and the packed text is read again right after)
void copy_cached(uint8_t* dst, const uint8_t* src, int64_t n);

void pack_split_docs(const char* const* src, const int64_t* doc_off, int64_t D, uint8_t* dst, int nthreads,
                     DocBatchIndex& out, int64_t min_bytes_per_thread = int64_t(4) << 20,
                     const int64_t* const* nlpos = nullptr, const int64_t* nlcnt = nullptr);

}  // namespace lp
