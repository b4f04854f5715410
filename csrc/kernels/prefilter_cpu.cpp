// CPU backend of the literal prefilter's bloom tier (the host twin of k_prefilter<16, S>), AVX-512.
//
// The CPU backend serves BASELINE config 1 (CPU-only POST /parse) and is the availability fallback.
// Its scalar twin spent ~7 ns per tested position (a 1 MB request: 262k stride-4 positions, 1.8 ms
// on one core; more on the host pool, whose wake-ups cost more than the work). Here 16 positions
// per step: one 64-byte load holds the 16 4-grams at p, p + 4, ..., p + 60 (stride 4; strides 2 and 1
// add the loads at p + 2 / p + 1, p + 3), lower-cased with byte masks, hashed with vpmulld, the
// bloom words fetched with one gather and the 3-bit word masks built with variable shifts. Only
// positions whose bloom bits are all set (~0.2% of them on log text) go to the scalar probe.
#include <immintrin.h>

#include <cstring>

#include "kernels/lp_api.h"
#include "kernels/lp_core.h"

namespace lp {

bool prefilter_bloom_simd_ok() {
  static const bool ok = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw");
  return ok;
}

// positions p in [a, b) with p % S == 0, p + 64 + 3 < nbytes handled here; returns the first
// position NOT handled (the caller's scalar loop finishes the range)
__attribute__((target("avx512f,avx512bw"))) int64_t prefilter_bloom_simd(
    const uint8_t* text, int64_t nbytes, const PfTables& T, const int64_t* line_start, int64_t nlines, int64_t a,
    int64_t b, std::vector<int64_t>& out) {
  const int S = T.stride == 2 ? 2 : T.stride == 4 ? 4 : 1;
  auto app = [&](int64_t v) { out.push_back(v); };
  const __m512i cA = _mm512_set1_epi8('A' - 1), cZ = _mm512_set1_epi8('Z' + 1), c20 = _mm512_set1_epi8(0x20);
  const __m512i seed = _mm512_set1_epi32((int)(4u * 0x9E3779B9u)), mul = _mm512_set1_epi32((int)0x85EBCA6Bu);
  const __m512i k31 = _mm512_set1_epi32(31), one = _mm512_set1_epi32(1);
  const __m128i wsh = _mm_cvtsi32_si128(32 - (T.bloom_bits - 5));
  const uint32_t* bl = T.bloom;
  int64_t p = (a + 3) & ~int64_t(3);                   // 4-aligned start: every stride divides it
  // the loads read [p, p + 64 + 3): stay clear of the text end (bytes past it must read as 0)
  for (; p + 64 + 4 <= b && p + 64 + 4 <= nbytes; p += 64) {
    for (int o = 0; o < 4; o += S) {
      __m512i v = _mm512_loadu_si512(reinterpret_cast<const void*>(text + p + o));
      // ASCII lower-casing: 'A' <= c <= 'Z' (unsigned compares leave bytes >= 0x80 alone)
      const __mmask64 up = _mm512_cmpgt_epu8_mask(v, cA) & _mm512_cmplt_epu8_mask(v, cZ);
      v = _mm512_mask_add_epi8(v, up, v, c20);
      const __m512i h = _mm512_mullo_epi32(_mm512_xor_si512(v, seed), mul);          // bloom_hash(key, 4)
      const __m512i widx = _mm512_srl_epi32(h, wsh);
      const __m512i q = _mm512_xor_si512(h, _mm512_srli_epi32(h, 15));              // bloom_bits_of
      const __m512i m = _mm512_or_si512(
          _mm512_or_si512(_mm512_sllv_epi32(one, _mm512_and_si512(q, k31)),
                          _mm512_sllv_epi32(one, _mm512_and_si512(_mm512_srli_epi32(q, 5), k31))),
          _mm512_sllv_epi32(one, _mm512_and_si512(_mm512_srli_epi32(q, 10), k31)));
      const __m512i w = _mm512_i32gather_epi32(widx, reinterpret_cast<const void*>(bl), 4);
      __mmask16 hit = _mm512_cmpeq_epi32_mask(_mm512_and_si512(w, m), m);
      if (__builtin_expect(hit != 0, 0)) {
        alignas(64) uint32_t g[16];
        _mm512_store_si512(reinterpret_cast<void*>(g), v);
        while (hit) {
          const int k = __builtin_ctz(hit);
          hit &= hit - 1;
          const int64_t pos = p + o + 4 * k;
          if (pos >= a) pf_probe(T, text, nbytes, pos, g[k], 4, line_start, nlines, nullptr, app);
        }
      }
    }
  }
  return p;
}

// Short-literal (Teddy) tier, every position p in [a, b): the bucket mask of the 3-byte window is
// teddy[4 c0] & teddy[4 c1 + 1] & teddy[4 c2 + 2] (lower-cased bytes); 16 positions per step with
// three gathers, the scalar probe only where the mask is non-zero. Returns the first position not
// handled (the window must stay clear of the text end: bytes past it read as 0).
__attribute__((target("avx512f,avx512bw"))) int64_t prefilter_teddy_simd(
    const uint8_t* text, int64_t nbytes, const PfTables& T, const int64_t* line_start, int64_t nlines, int64_t a,
    int64_t b, std::vector<int64_t>& out) {
  auto app = [&](int64_t v) { out.push_back(v); };
  const __m512i cA = _mm512_set1_epi32('A'), cZ = _mm512_set1_epi32('Z'), c20 = _mm512_set1_epi32(0x20);
  const __m512i j1 = _mm512_set1_epi32(1), j2 = _mm512_set1_epi32(2);
  const void* tb = reinterpret_cast<const void*>(T.teddy);
#define LP_TEDDY_LANES(q, out)                                                                       \
  do {                                                                                               \
    __m512i v_ = _mm512_cvtepu8_epi32(_mm_loadu_si128(reinterpret_cast<const __m128i*>(q)));        \
    const __mmask16 up_ = _mm512_cmpge_epu32_mask(v_, cA) & _mm512_cmple_epu32_mask(v_, cZ);        \
    out = _mm512_slli_epi32(_mm512_mask_add_epi32(v_, up_, v_, c20), 2);                            \
  } while (0)
  int64_t p = a;
  for (; p + 16 + 2 <= b && p + 16 + 2 <= nbytes; p += 16) {
    __m512i i0, i1, i2;                 // 16 lower-cased bytes as dwords, x4 (table index)
    LP_TEDDY_LANES(text + p, i0);
    LP_TEDDY_LANES(text + p + 1, i1);
    LP_TEDDY_LANES(text + p + 2, i2);
    const __m512i m0 = _mm512_i32gather_epi32(i0, tb, 4);
    const __m512i m1 = _mm512_i32gather_epi32(_mm512_add_epi32(i1, j1), tb, 4);
    const __m512i m2 = _mm512_i32gather_epi32(_mm512_add_epi32(i2, j2), tb, 4);
    const __m512i m = _mm512_and_si512(_mm512_and_si512(m0, m1), m2);
    __mmask16 hit = _mm512_test_epi32_mask(m, m);
    if (hit) {
      alignas(64) uint32_t mk[16];
      _mm512_store_si512(reinterpret_cast<void*>(mk), m);
      while (hit) {
        const int k = __builtin_ctz(hit);
        hit &= hit - 1;
        teddy_probe(T, text, nbytes, p + k, mk[k], line_start, nlines, nullptr, app);
      }
    }
  }
  return p;
}
#undef LP_TEDDY_LANES

}  // namespace lp
