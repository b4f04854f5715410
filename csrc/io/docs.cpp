#include "io/docs.h"

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <thread>

#include "kernels/lp_host.h"

#if defined(__SSE2__)
#include <emmintrin.h>
#endif
#if defined(__x86_64__)
#include <immintrin.h>
#endif

namespace lp {

// Newline positions of one unit: grow-only, uninitialised storage (a zero-filled vector costs a
// memset of its capacity per request).
struct NlBuf {
  std::unique_ptr<int64_t[]> p;
  int64_t n = 0, cap = 0;
  void reserve(int64_t c) {
    if (c <= cap) return;
    std::unique_ptr<int64_t[]> q(new int64_t[(size_t)c]);
    if (n) std::memcpy(q.get(), p.get(), (size_t)n * sizeof(int64_t));
    p = std::move(q);
    cap = c;
  }
  void push_back(int64_t v) {
    if (n == cap) reserve(std::max<int64_t>(64, 2 * cap));
    p[n++] = v;
  }
  int64_t size() const { return n; }
  bool empty() const { return n == 0; }
  int64_t back() const { return p[n - 1]; }
  int64_t operator[](int64_t i) const { return p[i]; }
};

#if defined(__x86_64__)
// AVX-512 VBMI2: 64 bytes per step, copied with one load / store; the newline offsets of the block
// are compressed out of an iota vector (vpcompressb) and the first 8 widened to absolute int64
// positions and stored unconditionally -- no branch per newline (the bit loop mispredicted on
// every ~100-byte line). Blocks with more than 8 newlines take a short scalar loop. Returns the
// bytes consumed (a multiple of 64, stops early when `nl` lacks 64 + 8 free slots).
// NT: dst is 64-byte aligned and the stores stream past the cache (the destination is the
// pinned staging buffer the GPU's DMA reads next, never this core: no read-for-ownership of the
// destination lines).
template <int MODE>   // 0: stores, 1: streaming stores, 2: no stores (src == dst)
__attribute__((target("avx512f,avx512bw,avx512vbmi,avx512vbmi2,bmi,bmi2,popcnt")))
static int64_t copy_scan_nl_512(const uint8_t* src, uint8_t* dst, int64_t n, int64_t base, NlBuf& nl) {
  alignas(64) static const uint8_t kIota[64] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15,
                                                16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31,
                                                32, 33, 34, 35, 36, 37, 38, 39, 40, 41, 42, 43, 44, 45, 46, 47,
                                                48, 49, 50, 51, 52, 53, 54, 55, 56, 57, 58, 59, 60, 61, 62, 63};
  const __m512i iota = _mm512_load_si512(reinterpret_cast<const void*>(kIota));
  const __m512i NL = _mm512_set1_epi8('\n');
  int64_t i = 0, k = nl.n;
  int64_t* out = nl.p.get();
  const int64_t room = nl.cap - 72;
  for (; i + 64 <= n && k <= room; i += 64) {
    const __m512i v = _mm512_loadu_si512(reinterpret_cast<const void*>(src + i));
    if constexpr (MODE == 1)
      _mm512_stream_si512(reinterpret_cast<__m512i*>(dst + i), v);
    else if constexpr (MODE == 0)
      _mm512_storeu_si512(reinterpret_cast<void*>(dst + i), v);
    const uint64_t m = _mm512_cmpeq_epi8_mask(v, NL);
    const __m512i offs = _mm512_maskz_compress_epi8(m, iota);
    const __m512i pos = _mm512_add_epi64(_mm512_cvtepu8_epi64(_mm512_castsi512_si128(offs)), _mm512_set1_epi64(base + i));
    _mm512_storeu_si512(reinterpret_cast<void*>(out + k), pos);
    const int c = (int)_mm_popcnt_u64(m);
    if (c > 8) {   // rare: short lines
      uint64_t r = m;
      for (int j = 0; j < 8; ++j) r &= r - 1;
      int64_t q = k + 8;
      while (r) {
        out[q++] = base + i + __builtin_ctzll(r);
        r &= r - 1;
      }
    }
    k += c;
  }
  if constexpr (MODE == 1) _mm_sfence();
  nl.n = k;
  return i;
}

// plain copy through the cache (regular 64-byte stores): glibc's memcpy switches to non-temporal
// stores for megabyte copies, and the stage is read right after (the line pass, the emitter's
// context lines) -- a 1 MB request packed with memcpy took 79-97 us against 44-66 us for the
// copy + scan below (profiles/r6_e)
__attribute__((target("avx512f")))
static void copy_cached_512(uint8_t* dst, const uint8_t* src, int64_t n) {
  int64_t i = 0;
  for (; i + 256 <= n; i += 256) {
    const __m512i a = _mm512_loadu_si512(reinterpret_cast<const void*>(src + i));
    const __m512i b = _mm512_loadu_si512(reinterpret_cast<const void*>(src + i + 64));
    const __m512i c = _mm512_loadu_si512(reinterpret_cast<const void*>(src + i + 128));
    const __m512i d = _mm512_loadu_si512(reinterpret_cast<const void*>(src + i + 192));
    _mm512_storeu_si512(reinterpret_cast<void*>(dst + i), a);
    _mm512_storeu_si512(reinterpret_cast<void*>(dst + i + 64), b);
    _mm512_storeu_si512(reinterpret_cast<void*>(dst + i + 128), c);
    _mm512_storeu_si512(reinterpret_cast<void*>(dst + i + 192), d);
  }
  for (; i + 64 <= n; i += 64)
    _mm512_storeu_si512(reinterpret_cast<void*>(dst + i), _mm512_loadu_si512(reinterpret_cast<const void*>(src + i)));
  if (i < n) std::memcpy(dst + i, src + i, (size_t)(n - i));
}

// streaming (non-temporal) stores of the pack are off: a 10k-line request measured 0.299-0.302 ms
// with them vs 0.282 ms without -- the '\r' checks of the line pass and the JSON emitter's context
// lines then read the stage from DRAM instead of the cache
static bool pack_nt_enabled() { return false; }

static bool have_avx512_vbmi2() {
  static const bool ok = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
                         __builtin_cpu_supports("avx512vbmi") && __builtin_cpu_supports("avx512vbmi2") &&
                         __builtin_cpu_supports("bmi2") && __builtin_cpu_supports("popcnt");
  return ok;
}
#endif

// Copy src[0, n) to dst and record the absolute position (base + i) of every '\n', in ONE pass
// over the bytes: 64-byte blocks are loaded once, stored, and compared into a bit mask whose set
// bits are the newlines (a memchr call per ~100-byte log line costs more than the bytes
// themselves: 1.9M calls per 2k-request batch).
static void copy_scan_nl(const uint8_t* src, uint8_t* dst, int64_t n, int64_t base, NlBuf& nl) {
  int64_t i = 0;
#if defined(__x86_64__)
  if (have_avx512_vbmi2()) {
    // src == dst: the bytes were decoded into the stage already (RawLogs): scan only
    const int mode = src == dst ? 2 : (((uintptr_t)dst & 63) == 0 && pack_nt_enabled()) ? 1 : 0;
    while (i + 64 <= n) {
      nl.reserve(nl.n + std::max<int64_t>(1024, (n - i) / 32) + 72);
      i += mode == 2 ? copy_scan_nl_512<2>(src + i, dst + i, n - i, base + i, nl)
           : mode == 1 ? copy_scan_nl_512<1>(src + i, dst + i, n - i, base + i, nl)
                       : copy_scan_nl_512<0>(src + i, dst + i, n - i, base + i, nl);
    }
  }
#endif
#if defined(__SSE2__)
  const __m128i NL = _mm_set1_epi8('\n');
  for (; i + 64 <= n; i += 64) {
    const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i));
    const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 16));
    const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 32));
    const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 48));
    _mm_storeu_si128(reinterpret_cast<__m128i*>(dst + i), a);
    _mm_storeu_si128(reinterpret_cast<__m128i*>(dst + i + 16), b);
    _mm_storeu_si128(reinterpret_cast<__m128i*>(dst + i + 32), c);
    _mm_storeu_si128(reinterpret_cast<__m128i*>(dst + i + 48), d);
    uint64_t m = (uint64_t)(uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(a, NL)) |
                 ((uint64_t)(uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(b, NL)) << 16) |
                 ((uint64_t)(uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(c, NL)) << 32) |
                 ((uint64_t)(uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(d, NL)) << 48);
    while (m) {
      nl.push_back(base + i + __builtin_ctzll(m));
      m &= m - 1;
    }
  }
#endif
  for (; i < n; ++i) {
    dst[i] = src[i];
    if (src[i] == '\n') nl.push_back(base + i);
  }
}

// Work unit: one document, or a ~128 KiB slice of a large one (so a single big request also
// copies and splits on several threads).
struct Unit {
  int64_t doc, a, b;           // bytes [a, b) of document `doc` (absolute packed offsets)
  NlBuf nl;                    // '\n' positions inside [a, b)
  int64_t first_nl = 0;        // index of nl[0] among the document's newlines
  int64_t prev = 0;            // position of the newline before this unit (doc start - 1 if none)
};

template <class F>
static void parallel_units(std::vector<Unit>& U, int64_t total, int nthreads, int64_t per_thread, F&& fn) {
  const int64_t n = (int64_t)U.size();
  // >= per_thread bytes per helper (4 MB default): a request's bytes sit in the caller's cache,
  // and on a many-chiplet host, moving them to helpers on other CCDs costs more than the copy
  // (measured on the MI355X box's EPYC: 1 MB pack 46 us on one thread, 93-111 us on the pool)
  const int T = std::max(1, std::min<int>(nthreads, (int)std::min<int64_t>(n, 1 + total / std::max<int64_t>(1, per_thread))));
  if (T == 1) {
    for (int64_t u = 0; u < n; ++u) fn(U[u]);
    return;
  }
  HostPool::get().run(n, T, [&](int64_t u) { fn(U[u]); });
}

void copy_cached(uint8_t* dst, const uint8_t* src, int64_t n) {
#if defined(__x86_64__)
  if (__builtin_cpu_supports("avx512f")) {
    copy_cached_512(dst, src, n);
    return;
  }
#endif
  std::memcpy(dst, src, (size_t)n);
}

void pack_split_docs(const char* const* src, const int64_t* doc_off, int64_t D, uint8_t* dst, int nthreads,
                     DocBatchIndex& out, int64_t min_bytes_per_thread, const int64_t* const* nlpos,
                     const int64_t* nlcnt) {
  constexpr int64_t SLICE = 128 << 10;
  std::vector<Unit> U;
  U.reserve(D);
  for (int64_t d = 0; d < D; ++d) {
    const int64_t s0 = doc_off[d], s1 = doc_off[d + 1];
    const bool known = nlpos && nlpos[d];
    const int64_t k = nthreads > 1 && !known ? std::max<int64_t>(1, (s1 - s0) / SLICE) : 1;
    for (int64_t i = 0; i < k; ++i) U.push_back(Unit{d, s0 + (s1 - s0) * i / k, s0 + (s1 - s0) * (i + 1) / k, {}});
  }
  const int64_t total = doc_off[D];
  // phase 1: copy + newline positions, one pass over the bytes (known positions: a plain copy)
  parallel_units(U, total, nthreads, min_bytes_per_thread, [&](Unit& u) {
    const int64_t s0 = doc_off[u.doc];
    if (nlpos && nlpos[u.doc]) {
      const int64_t c = nlcnt[u.doc];
      if (src[u.doc] != reinterpret_cast<const char*>(dst + u.a))
        copy_cached(dst + u.a, reinterpret_cast<const uint8_t*>(src[u.doc]), u.b - u.a);
      u.nl.reserve(c + 1);
      const int64_t* q = nlpos[u.doc];
      for (int64_t j = 0; j < c; ++j) u.nl.p[j] = q[j] + u.a;
      u.nl.n = c;
      return;
    }
    u.nl.reserve((u.b - u.a) / 64 + 4);
    copy_scan_nl(reinterpret_cast<const uint8_t*>(src[u.doc]) + (u.a - s0), dst + u.a, u.b - u.a, u.a, u.nl);
  });
  // per document: newline numbering, kept lines (Java split: trailing empty strings dropped; a
  // document without any '\n' is one line, possibly empty)
  auto line_end = [&](int64_t nlpos, int64_t start) {   // '\r' before '\n' excluded
    return (nlpos > start && dst[nlpos - 1] == '\r') ? nlpos - 1 : nlpos;
  };
  out.doc_line_off.alloc(D + 1);
  out.doc_line_off[0] = 0;
  std::vector<int64_t> kept(D, 0);
  for (size_t i = 0; i < U.size();) {
    const int64_t d = U[i].doc, s0 = doc_off[d], s1 = doc_off[d + 1];
    size_t j = i;
    int64_t nnl = 0, prev = s0 - 1;
    for (; j < U.size() && U[j].doc == d; ++j) {
      U[j].first_nl = nnl;
      U[j].prev = prev;
      nnl += (int64_t)U[j].nl.size();
      if (!U[j].nl.empty()) prev = U[j].nl.back();
    }
    int64_t k = 0;
    if (nnl == 0) {
      k = 1;
    } else if (s1 > prev + 1) {
      k = nnl + 1;                       // last line (after the last '\n') is non-empty
    } else {                             // walk back over the newlines to the last non-empty line
      for (size_t v = j; v-- > i && k == 0;) {
        const auto& nl = U[v].nl;
        for (int64_t w = (int64_t)nl.size() - 1; w >= 0; --w) {
          const int64_t start = w > 0 ? nl[w - 1] + 1 : U[v].prev + 1;
          if (line_end(nl[w], start) > start) {
            k = U[v].first_nl + w + 1;
            break;
          }
        }
      }
    }
    kept[d] = k;
    i = j;
  }
  for (int64_t d = 0; d < D; ++d) out.doc_line_off[d + 1] = out.doc_line_off[d] + kept[d];
  const int64_t L = out.doc_line_off[D];
  int64_t* ls = out.ext_start;
  int32_t* ll = out.ext_len;
  out.external = ls && ll && L <= out.ext_cap;
  if (!out.external) {
    out.line_start.alloc(L);
    out.line_len.alloc(L);
    ls = out.line_start.data();
    ll = out.line_len.data();
  }
  // phase 2: line starts / lengths, each unit writes its own newlines' lines
  parallel_units(U, total, nthreads, min_bytes_per_thread, [&](Unit& u) {
    const int64_t k = kept[u.doc], base = out.doc_line_off[u.doc];
    int64_t start = u.prev + 1;
    for (size_t w = 0; w < u.nl.size(); ++w) {
      const int64_t g = u.first_nl + (int64_t)w;
      if (g >= k) return;
      ls[base + g] = start;
      ll[base + g] = (int32_t)(line_end(u.nl[w], start) - start);
      start = u.nl[w] + 1;
    }
    // the line after the document's last newline belongs to the document's last unit
    const bool last_unit = u.b == doc_off[u.doc + 1];
    const int64_t g = u.first_nl + (int64_t)u.nl.size();
    if (last_unit && g < k) {
      ls[base + g] = start;
      ll[base + g] = (int32_t)(u.b - start);
    }
  });
}

}  // namespace lp
