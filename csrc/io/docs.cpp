#include "io/docs.h"

#include <algorithm>
#include <cstring>
#include <thread>

namespace lp {

// Java logs.split("\\r?\\n") of b[s0, s1): trailing empty strings removed, a document without
// any '\n' is one line (possibly empty). emit(start, len) for the first `limit` kept lines;
// returns the number of kept lines.
template <class F>
static int64_t split_doc(const uint8_t* b, int64_t s0, int64_t s1, int64_t limit, F&& emit) {
  int64_t start = s0, n = 0, kept = 0;
  bool any = false;
  for (;;) {
    const void* q = memchr(b + start, '\n', (size_t)(s1 - start));
    if (!q) break;
    any = true;
    const int64_t nl = static_cast<const uint8_t*>(q) - b;
    int64_t end = nl;
    if (end > start && b[end - 1] == '\r') --end;
    if (n < limit) emit(start, end - start);
    ++n;
    if (end > start) kept = n;
    start = nl + 1;
  }
  if (n < limit) emit(start, s1 - start);
  ++n;
  if (s1 > start || !any) kept = n;
  return kept;
}

template <class F>
static void parallel_docs(const int64_t* doc_off, int64_t D, int nthreads, F&& fn) {
  const int64_t total = doc_off[D];
  int T = std::max(1, std::min<int>(nthreads, (int)std::min<int64_t>(D, 1 + total / (1 << 20))));
  if (T == 1) {
    fn(0, D);
    return;
  }
  // contiguous document ranges of ~equal bytes
  std::vector<int64_t> cut(T + 1, D);
  cut[0] = 0;
  for (int t = 1; t < T; ++t) {
    const int64_t target = total / T * t;
    cut[t] = std::max(cut[t - 1], (int64_t)(std::upper_bound(doc_off, doc_off + D + 1, target) - doc_off - 1));
  }
  std::vector<std::thread> th;
  th.reserve(T);
  for (int t = 0; t < T; ++t)
    if (cut[t + 1] > cut[t]) th.emplace_back([&, t] { fn(cut[t], cut[t + 1]); });
  for (auto& x : th) x.join();
}

void pack_split_docs(const char* const* src, const int64_t* doc_off, int64_t D, uint8_t* dst, int nthreads,
                     DocBatchIndex& out) {
  std::vector<int64_t> cnt(D);
  parallel_docs(doc_off, D, nthreads, [&](int64_t a, int64_t b) {
    for (int64_t d = a; d < b; ++d) {
      const int64_t s0 = doc_off[d], s1 = doc_off[d + 1];
      if (s1 > s0) memcpy(dst + s0, src[d], (size_t)(s1 - s0));
      cnt[d] = split_doc(dst, s0, s1, 0, [](int64_t, int64_t) {});
    }
  });
  out.doc_line_off.assign(D + 1, 0);
  for (int64_t d = 0; d < D; ++d) out.doc_line_off[d + 1] = out.doc_line_off[d] + cnt[d];
  out.line_start.resize(out.doc_line_off[D]);
  out.line_len.resize(out.doc_line_off[D]);
  parallel_docs(doc_off, D, nthreads, [&](int64_t a, int64_t b) {
    for (int64_t d = a; d < b; ++d) {
      int64_t o = out.doc_line_off[d];
      split_doc(dst, doc_off[d], doc_off[d + 1], cnt[d], [&](int64_t s, int64_t l) {
        out.line_start[o] = s;
        out.line_len[o] = (int32_t)l;
        ++o;
      });
    }
  });
}

}  // namespace lp
