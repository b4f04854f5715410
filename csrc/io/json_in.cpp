// Native request decoder for POST /parse bodies (PodFailureData, reference Parse.java:41-61).
//
// The service only needs three things from the body: whether `pod` is present and non-null, the
// pod name for the request log (pod.metadata.name), and the `logs` string. Python's json.loads
// builds the whole object tree and a str for a ~1 MB log (0.9 ms per 10k-line request, more
// than the GPU analysis itself); this single pass validates the JSON grammar, skips everything
// else and unescapes `logs` straight to UTF-8 bytes, which the batch packer consumes as-is.
//
// Anything unusual returns FALLBACK so the caller uses json.loads and keeps its exact acceptance
// rules: non-UTF-8 encodings / BOM, invalid UTF-8, NaN/Infinity literals, \u escapes of
// surrogates, nesting deeper than 512. Duplicate keys: the last one wins (as in json.loads).
#include "io/json_in.h"

#include <cstring>

#if defined(__SSE2__)
#include <emmintrin.h>
#endif
#if defined(__x86_64__)
#include <immintrin.h>
#endif

namespace lp {
namespace {

struct Cur {
  const uint8_t* p;
  const uint8_t* e;
  int depth = 0;
  bool fallback = false;
  bool closed = false;   // str_loop consumed the closing quote (span mode: the string ended in the span)
  NlPos* nl = nullptr;   // str_loop records the decoded '\n' positions (relative to w0)
  const char* w0 = nullptr;
};

// one decoded '\n' at w (scalar escapes)
inline void nl_push(Cur& c, const char* w) {
  if (!c.nl) return;
  if (c.nl->n + 1 > c.nl->cap) c.nl->reserve(c.nl->n + 4096);
  c.nl->p[c.nl->n++] = (int64_t)(w - c.w0);
}

inline void ws(Cur& c) {
  while (c.p < c.e && (*c.p == ' ' || *c.p == '\t' || *c.p == '\n' || *c.p == '\r')) ++c.p;
}

inline int hexv(uint8_t h) {
  if (h >= '0' && h <= '9') return h - '0';
  if (h >= 'a' && h <= 'f') return h - 'a' + 10;
  if (h >= 'A' && h <= 'F') return h - 'A' + 10;
  return -1;
}

// length of a valid UTF-8 sequence starting at p (>= 0x80 lead byte), 0 if invalid
inline int utf8_len(const uint8_t* p, const uint8_t* e) {
  const uint8_t b = p[0];
  auto cont = [&](int i) { return p + i < e && (p[i] & 0xC0) == 0x80; };
  if (b >= 0xC2 && b <= 0xDF) return cont(1) ? 2 : 0;
  if (b >= 0xE0 && b <= 0xEF) {
    if (!cont(1) || !cont(2)) return 0;
    if (b == 0xE0 && p[1] < 0xA0) return 0;   // overlong
    if (b == 0xED && p[1] >= 0xA0) return 0;  // encoded surrogate
    return 3;
  }
  if (b >= 0xF0 && b <= 0xF4) {
    if (!cont(1) || !cont(2) || !cont(3)) return 0;
    if (b == 0xF0 && p[1] < 0x90) return 0;
    if (b == 0xF4 && p[1] >= 0x90) return 0;
    return 4;
  }
  return 0;
}

#if defined(__x86_64__)
// AVX-512 VBMI2 block decoder (Zen 4/5 and Ice Lake+ servers): one 64-byte block of a JSON
// string per call, branch-free. Escape-initiating backslashes are found from backslash-run
// parity (carries of run_start + backslashes mark each run and the byte after it), escaped bytes
// are translated through a 128-entry vpermi2b table and the initiating backslashes are dropped with
// vpcompressb. A log line costs no branch per escape (one "\n" every ~100 bytes made the scalar
// loop mispredict-bound: 265 us per MB on a Zen 5 core). Returns false -- nothing consumed -- for
// any block the scalar path must handle: the closing quote, control or non-ASCII bytes, \u or
// invalid escapes, a backslash in the last byte (a run that may continue into the next block).
// Needs 64 readable bytes at p and 64 writable bytes at w.
// With Store = false the block is only validated (skip mode of a string nobody reads).
template <bool Store>
__attribute__((target("avx512f,avx512bw,avx512vbmi,avx512vbmi2,bmi,bmi2,popcnt")))
bool block64(const uint8_t*& p, char*& w, size_t* kept = nullptr, NlPos* nl = nullptr, const char* w0 = nullptr) {
  const __m512i v = _mm512_loadu_si512(reinterpret_cast<const void*>(p));
  const uint64_t B = _mm512_cmpeq_epi8_mask(v, _mm512_set1_epi8('\\'));
  const uint64_t Q = _mm512_cmpeq_epi8_mask(v, _mm512_set1_epi8('"'));
  const uint64_t CH = _mm512_cmplt_epu8_mask(v, _mm512_set1_epi8(0x20)) | _mm512_movepi8_mask(v);
  constexpr uint64_t EVEN = 0x5555555555555555ull, ODD = ~EVEN;
  const uint64_t starts = B & ~(B << 1);                  // first backslash of each run
  // adding a run's start bit carries through the run: the run's bits clear and the byte after
  // it sets. Inside a run every second backslash is escaped; the byte after the run is escaped
  // iff the run is odd -- for a run starting at an even position, both are the odd positions.
  const uint64_t sum_e = B + (starts & EVEN), sum_o = B + (starts & ODD);
  const uint64_t run_e = (B & ~sum_e) | (sum_e & ~B);     // even-start runs + the byte after
  const uint64_t run_o = (B & ~sum_o) | (sum_o & ~B);     // odd-start runs + the byte after
  const uint64_t escaped = (run_e & ODD) | (run_o & EVEN);
  const uint64_t initiators = B & ~escaped;
  // escape letter -> decoded byte (0 = not a simple escape: \u or invalid)
  alignas(64) static const uint8_t kEsc[128] = {
      0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
      0, 0, '"', 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, '/',  0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
      0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, '\\', 0, 0, 0,
      0, 0, '\b', 0, 0, 0, '\f', 0, 0, 0, 0, 0, 0, 0, '\n', 0,  0, 0, '\r', 0, '\t', 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  const __m512i t0 = _mm512_load_si512(reinterpret_cast<const void*>(kEsc));
  const __m512i t1 = _mm512_load_si512(reinterpret_cast<const void*>(kEsc + 64));
  const __m512i tr = _mm512_permutex2var_epi8(t0, v, t1);                 // low 7 bits index
  const uint64_t bad_esc = escaped & _mm512_cmpeq_epi8_mask(tr, _mm512_setzero_si512());
  if ((Q & ~escaped) | CH | bad_esc | (B >> 63)) return false;
  if (kept) *kept += (size_t)_mm_popcnt_u64(~initiators);
  if (Store) {
    const __m512i o = _mm512_mask_blend_epi8(escaped, v, tr);
    const uint64_t keep = ~initiators;
    const __m512i out = _mm512_maskz_compress_epi8(keep, o);
    _mm512_storeu_si512(reinterpret_cast<void*>(w), out);
    const int nk = (int)_mm_popcnt_u64(keep);
    if (nl) {   // the block's decoded newlines: offsets compressed out of an iota, 8 stored per step
      const uint64_t valid = nk >= 64 ? ~0ull : ((1ull << nk) - 1);
      uint64_t m = _mm512_cmpeq_epi8_mask(out, _mm512_set1_epi8('\n')) & valid;
      if (m) {
        alignas(64) static const uint8_t kIota[64] = {
            0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21,
            22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 36, 37, 38, 39, 40, 41, 42, 43,
            44, 45, 46, 47, 48, 49, 50, 51, 52, 53, 54, 55, 56, 57, 58, 59, 60, 61, 62, 63};
        if (nl->n + 72 > nl->cap) nl->reserve(nl->n + 4096);
        const __m512i offs = _mm512_maskz_compress_epi8(m, _mm512_load_si512(reinterpret_cast<const void*>(kIota)));
        const int64_t base = (int64_t)(w - w0);
        _mm512_storeu_si512(reinterpret_cast<void*>(nl->p.get() + nl->n),
                            _mm512_add_epi64(_mm512_cvtepu8_epi64(_mm512_castsi512_si128(offs)), _mm512_set1_epi64(base)));
        const int c = (int)_mm_popcnt_u64(m);
        if (c > 8) {
          for (int j = 0; j < 8; ++j) m &= m - 1;
          size_t q = nl->n + 8;
          while (m) {
            nl->p[q++] = base + __builtin_ctzll(m);
            m &= m - 1;
          }
        }
        nl->n += (size_t)c;
      }
    }
    w += nk;
  }
  p += 64;
  return true;
}

bool have_block64() {
  static const bool ok = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
                         __builtin_cpu_supports("avx512vbmi") && __builtin_cpu_supports("avx512vbmi2") &&
                         __builtin_cpu_supports("bmi2") && __builtin_cpu_supports("popcnt");
  return ok;
}
#endif

// Decodes the string at c.p (opening quote) into `w`, which has room for (c.e - c.p) + 64 bytes
// (decoded JSON is never longer than its encoding). Copy-then-check: every 16-byte block is
// stored unconditionally and the write cursor advances only past the plain bytes, so a run of
// ordinary text costs one load, one store and one compare per 16 bytes, and an escape (a log has
// one "\n" every ~100 bytes) only a few scalar steps -- no per-run append. Returns the end of the
// decoded bytes, or nullptr on error (c.fallback set when json.loads must decide).
template <bool Span>
char* str_loop(Cur& c, char* w) {
#if defined(__x86_64__)
  const bool wide = have_block64();
#endif
  for (;;) {
#if defined(__x86_64__)
    if (wide)
      while (c.e - c.p >= 64 && block64<true>(c.p, w, nullptr, c.nl, c.w0)) {
      }
#endif
#if defined(__SSE2__)
    {
      const __m128i q = _mm_set1_epi8('"'), bs = _mm_set1_epi8('\\'), sp = _mm_set1_epi8(0x20);
      while (c.e - c.p >= 16) {
        const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(c.p));
        _mm_storeu_si128(reinterpret_cast<__m128i*>(w), v);
        const __m128i m = _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(v, q), _mm_cmpeq_epi8(v, bs)), _mm_cmplt_epi8(v, sp));
        const int bits = _mm_movemask_epi8(m);
        if (bits) {
          const int k = __builtin_ctz((unsigned)bits);
          c.p += k;
          w += k;
          break;
        }
        c.p += 16;
        w += 16;
      }
    }
#endif
    while (c.p < c.e && *c.p != '"' && *c.p != '\\' && *c.p >= 0x20 && *c.p < 0x80) *w++ = (char)*c.p++;
    if (c.p >= c.e) return Span ? w : nullptr;
    const uint8_t b = *c.p;
    if (b == '"') {
      ++c.p;
      c.closed = true;
      return w;
    }
    if (b < 0x20) return nullptr;  // json.loads(strict=True) rejects raw control characters
    if (b >= 0x80) {
      const int k = utf8_len(c.p, c.e);
      if (!k) {
        c.fallback = true;
        return nullptr;
      }
      for (int i = 0; i < k; ++i) *w++ = (char)c.p[i];
      c.p += k;
      continue;
    }
    if (c.p + 1 >= c.e) return nullptr;
    const uint8_t x = c.p[1];
    c.p += 2;
    switch (x) {
      case '"': *w++ = '"'; break;
      case '\\': *w++ = '\\'; break;
      case '/': *w++ = '/'; break;
      case 'b': *w++ = '\b'; break;
      case 'f': *w++ = '\f'; break;
      case 'n': nl_push(c, w); *w++ = '\n'; break;
      case 'r': *w++ = '\r'; break;
      case 't': *w++ = '\t'; break;
      case 'u': {
        if (c.p + 4 > c.e) return nullptr;
        int v = 0;
        for (int i = 0; i < 4; ++i) {
          const int h = hexv(c.p[i]);
          if (h < 0) return nullptr;
          v = (v << 4) | h;
        }
        c.p += 4;
        if (v >= 0xD800 && v <= 0xDFFF) {
          c.fallback = true;
          return nullptr;
        }
        if (v < 0x80) {
          if (v == '\n') nl_push(c, w);
          *w++ = (char)v;
        } else if (v < 0x800) {
          *w++ = (char)(0xC0 | (v >> 6));
          *w++ = (char)(0x80 | (v & 0x3F));
        } else {
          *w++ = (char)(0xE0 | (v >> 12));
          *w++ = (char)(0x80 | ((v >> 6) & 0x3F));
          *w++ = (char)(0x80 | (v & 0x3F));
        }
        break;
      }
      default:
        return nullptr;
    }
  }
}

char* str_into(Cur& c, char* w) {
  if (c.p >= c.e || *c.p != '"') return nullptr;
  ++c.p;
  return str_loop<false>(c, w);
}

// the content bytes [c.p, c.e) of a string (no quotes), cut where no escape / UTF-8 sequence
// straddles c.e: decoded to w (block stores may run past the returned end)
char* str_into_span(Cur& c, char* w) { return str_loop<true>(c, w); }

// string at c.p (opening quote); appends the decoded UTF-8 to `out` when non-null; adds the
// decoded length to *dlen when non-null (skip mode: the batch packer decodes later, in parallel,
// straight to the offsets these lengths give)
bool str(Cur& c, std::string* out, size_t* dlen = nullptr) {
  if (c.p >= c.e || *c.p != '"') return false;
  ++c.p;
  size_t dn = 0;
  struct Flush {
    size_t* d;
    size_t& n;
    ~Flush() { if (d) *d += n; }
  } flush{dlen, dn};
#if defined(__x86_64__)
  const bool wide = out == nullptr && have_block64();
  char* none = nullptr;
#endif
  for (;;) {
#if defined(__x86_64__)
    if (wide)
      while (c.e - c.p >= 64 && block64<false>(c.p, none, &dn)) {
      }
#endif
    const uint8_t* run = c.p;
#if defined(__SSE2__)
    // 16 bytes per step: '"', '\\', control bytes and bytes >= 0x80 (signed < 0x20) end the run
    {
      const __m128i q = _mm_set1_epi8('"'), bs = _mm_set1_epi8('\\'), sp = _mm_set1_epi8(0x20);
      while (c.e - c.p >= 16) {
        const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(c.p));
        const __m128i m = _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(v, q), _mm_cmpeq_epi8(v, bs)), _mm_cmplt_epi8(v, sp));
        const int bits = _mm_movemask_epi8(m);
        if (bits) {
          c.p += __builtin_ctz((unsigned)bits);
          break;
        }
        c.p += 16;
      }
    }
#endif
    while (c.p < c.e && *c.p != '"' && *c.p != '\\' && *c.p >= 0x20 && *c.p < 0x80) ++c.p;
    dn += (size_t)(c.p - run);
    if (out && c.p > run) out->append(reinterpret_cast<const char*>(run), c.p - run);
    if (c.p >= c.e) return false;
    const uint8_t b = *c.p;
    if (b == '"') {
      ++c.p;
      return true;
    }
    if (b < 0x20) return false;  // json.loads(strict=True) rejects raw control characters
    if (b >= 0x80) {
      const int k = utf8_len(c.p, c.e);
      if (!k) {
        c.fallback = true;  // let json.loads produce its own error for bad UTF-8
        return false;
      }
      if (out) out->append(reinterpret_cast<const char*>(c.p), k);
      dn += (size_t)k;
      c.p += k;
      continue;
    }
    // escape
    if (c.p + 1 >= c.e) return false;
    const uint8_t x = c.p[1];
    c.p += 2;
    char ch;
    switch (x) {
      case '"': ch = '"'; break;
      case '\\': ch = '\\'; break;
      case '/': ch = '/'; break;
      case 'b': ch = '\b'; break;
      case 'f': ch = '\f'; break;
      case 'n': ch = '\n'; break;
      case 'r': ch = '\r'; break;
      case 't': ch = '\t'; break;
      case 'u': {
        if (c.p + 4 > c.e) return false;
        int v = 0;
        for (int i = 0; i < 4; ++i) {
          const int h = hexv(c.p[i]);
          if (h < 0) return false;
          v = (v << 4) | h;
        }
        c.p += 4;
        if (v >= 0xD800 && v <= 0xDFFF) {  // surrogate pairs / lone surrogates: json.loads rules
          c.fallback = true;
          return false;
        }
        dn += v < 0x80 ? 1 : v < 0x800 ? 2 : 3;
        if (out) {
          if (v < 0x80) {
            out->push_back((char)v);
          } else if (v < 0x800) {
            out->push_back((char)(0xC0 | (v >> 6)));
            out->push_back((char)(0x80 | (v & 0x3F)));
          } else {
            out->push_back((char)(0xE0 | (v >> 12)));
            out->push_back((char)(0x80 | ((v >> 6) & 0x3F)));
            out->push_back((char)(0x80 | (v & 0x3F)));
          }
        }
        continue;
      }
      default:
        return false;
    }
    ++dn;
    if (out) out->push_back(ch);
  }
}

bool number(Cur& c) {
  const uint8_t* s = c.p;
  if (c.p < c.e && *c.p == '-') ++c.p;
  if (c.p < c.e && (*c.p == 'I' || *c.p == 'N')) {  // -Infinity: json.loads extension
    c.fallback = true;
    return false;
  }
  if (c.p >= c.e) return false;
  if (*c.p == '0') {
    ++c.p;
  } else if (*c.p >= '1' && *c.p <= '9') {
    while (c.p < c.e && *c.p >= '0' && *c.p <= '9') ++c.p;
  } else {
    return false;
  }
  if (c.p < c.e && *c.p == '.') {
    ++c.p;
    const uint8_t* d = c.p;
    while (c.p < c.e && *c.p >= '0' && *c.p <= '9') ++c.p;
    if (c.p == d) return false;
  }
  if (c.p < c.e && (*c.p == 'e' || *c.p == 'E')) {
    ++c.p;
    if (c.p < c.e && (*c.p == '+' || *c.p == '-')) ++c.p;
    const uint8_t* d = c.p;
    while (c.p < c.e && *c.p >= '0' && *c.p <= '9') ++c.p;
    if (c.p == d) return false;
  }
  return c.p > s;
}

bool lit(Cur& c, const char* w) {
  const size_t n = strlen(w);
  if ((size_t)(c.e - c.p) < n || memcmp(c.p, w, n) != 0) return false;
  c.p += n;
  return true;
}

bool value(Cur& c);

// object members; `on_member(key, cursor)` parses the value itself and returns false on error
template <class F>
bool object(Cur& c, F&& on_member) {
  if (++c.depth > 512) {
    c.fallback = true;
    return false;
  }
  ++c.p;  // '{'
  ws(c);
  if (c.p < c.e && *c.p == '}') {
    ++c.p;
    --c.depth;
    return true;
  }
  std::string key;
  for (;;) {
    ws(c);
    key.clear();
    if (!str(c, &key)) return false;
    ws(c);
    if (c.p >= c.e || *c.p != ':') return false;
    ++c.p;
    ws(c);
    if (!on_member(key, c)) return false;
    ws(c);
    if (c.p >= c.e) return false;
    if (*c.p == ',') {
      ++c.p;
      continue;
    }
    if (*c.p == '}') {
      ++c.p;
      --c.depth;
      return true;
    }
    return false;
  }
}

bool value(Cur& c) {
  if (c.p >= c.e) return false;
  switch (*c.p) {
    case '"': return str(c, nullptr);
    case '{': return object(c, [](const std::string&, Cur& cc) { return value(cc); });
    case '[': {
      if (++c.depth > 512) {
        c.fallback = true;
        return false;
      }
      ++c.p;
      ws(c);
      if (c.p < c.e && *c.p == ']') {
        ++c.p;
        --c.depth;
        return true;
      }
      for (;;) {
        ws(c);
        if (!value(c)) return false;
        ws(c);
        if (c.p >= c.e) return false;
        if (*c.p == ',') {
          ++c.p;
          continue;
        }
        if (*c.p == ']') {
          ++c.p;
          --c.depth;
          return true;
        }
        return false;
      }
    }
    case 't': return lit(c, "true");
    case 'f': return lit(c, "false");
    case 'n': return lit(c, "null");
    case 'N':
    case 'I': c.fallback = true; return false;  // NaN / Infinity: json.loads extensions
    default: return number(c);
  }
}

}  // namespace

size_t decode_json_string(const uint8_t* p, size_t n, char* w) {
  Cur c{p - 1, p + n + 1};   // the opening quote .. one past the closing quote
  char* e = str_into(c, w);
  return e ? (size_t)(e - w) : 0;
}

size_t decode_json_string_exact(const uint8_t* p, size_t n, char* w) {
  // the block decoders store whole 16 / 64-byte blocks past their write cursor, so they run on a
  // prefix only: its unconditional stores stay inside this string's output while >= 64 decoded
  // bytes follow -- 384 encoded bytes are >= 64 decoded ones even if all are 6-byte \u escapes
  constexpr size_t kTail = 384;
  const uint8_t* const end = p + n;
  char* const w0 = w;
  const uint8_t* q = p;
  if (n > kTail + 64) {
    // the prefix ends at a position no escape straddles: walk back over a backslash run
    const uint8_t* cut = end - kTail;
    const uint8_t* b = cut;
    while (b > p && b[-1] == '\\') --b;
    if (((cut - b) & 1) != 0) --cut;                     // odd run: cut sits on an escaped byte
    while (cut > p && (*cut & 0xC0) == 0x80) --cut;      // not inside a UTF-8 sequence
    // a \uXXXX escape: its 4 hex digits must not be split either
    for (int k = 1; k <= 4 && cut - k >= p; ++k) {
      if (cut[-k] == 'u' && cut - k - 1 >= p && cut[-k - 1] == '\\') {
        const uint8_t* bb = cut - k - 1;
        size_t run = 0;
        while (bb - run > p && bb[-1 - (ptrdiff_t)run] == '\\') ++run;
        if ((run & 1) == 0) { cut -= k + 1; break; }   // an initiating backslash
      }
    }
    // decode [p, cut) with the block decoders
    Cur c{p, cut};
    char* e = str_into_span(c, w);
    if (!e) return 0;
    w = e;
    q = c.p;
  }
  // exact scalar tail: no store past the decoded end
  while (q < end) {
    const uint8_t b = *q;
    if (b != '\\') {
      *w++ = (char)b;
      ++q;
      continue;
    }
    const uint8_t x = q[1];
    q += 2;
    switch (x) {
      case '"': *w++ = '"'; break;
      case '\\': *w++ = '\\'; break;
      case '/': *w++ = '/'; break;
      case 'b': *w++ = '\b'; break;
      case 'f': *w++ = '\f'; break;
      case 'n': *w++ = '\n'; break;
      case 'r': *w++ = '\r'; break;
      case 't': *w++ = '\t'; break;
      case 'u': {
        int v = 0;
        for (int i = 0; i < 4; ++i) v = (v << 4) | hexv(q[i]);
        q += 4;
        if (v < 0x80) {
          *w++ = (char)v;
        } else if (v < 0x800) {
          *w++ = (char)(0xC0 | (v >> 6));
          *w++ = (char)(0x80 | (v & 0x3F));
        } else {
          *w++ = (char)(0xE0 | (v >> 12));
          *w++ = (char)(0x80 | ((v >> 6) & 0x3F));
          *w++ = (char)(0x80 | (v & 0x3F));
        }
        break;
      }
      default: return 0;
    }
  }
  return (size_t)(w - w0);
}

namespace {
int parse_pod_impl(const uint8_t* body, size_t n, PodRequest& out, bool decode_logs, char* dst, size_t cap,
                   const LogsPrefetch* pf, NlPos* nl);

// Body offset of the opening quote of the top-level `logs` string, found by the validating parser
// over the prefix [body, body + avail); 0 when the prefix does not reach it (truncated before it,
// invalid so far, or `logs` not a string). The parser is the one parse_pod_impl runs, so on the
// same bytes it reaches the same member at the same offset.
size_t locate_logs(const uint8_t* body, size_t avail) {
  if (avail >= 2 && (body[0] == 0 || body[1] == 0)) return 0;
  if (avail >= 3 && body[0] == 0xEF && body[1] == 0xBB && body[2] == 0xBF) return 0;
  Cur c{body, body + avail};
  ws(c);
  if (c.p >= c.e || *c.p != '{') return 0;
  size_t at = 0;
  object(c, [&](const std::string& key, Cur& cc) {
    if (key == "logs" && cc.p < cc.e && *cc.p == '"') {
      at = (size_t)(cc.p - body);
      return false;   // stop: the rest of the body has not arrived
    }
    return value(cc);
  });
  return at;
}

// [lo, cut) of a string's content still arriving, moved back so that no escape sequence, \u
// escape or UTF-8 sequence straddles `cut` (the byte at `cut` must be readable)
const uint8_t* safe_cut(const uint8_t* lo, const uint8_t* cut) {
  const uint8_t* b = cut;
  while (b > lo && b[-1] == '\\') --b;
  if (((cut - b) & 1) != 0) --cut;                       // odd run: the byte at cut is escaped
  while (cut > lo && (*cut & 0xC0) == 0x80) --cut;       // inside a UTF-8 sequence
  for (int k = 1; k <= 4 && cut - k > lo; ++k) {         // inside the 4 hex digits of a \u escape
    if (cut[-k] == 'u' && cut[-k - 1] == '\\') {
      const uint8_t* bb = cut - k - 1;
      size_t run = 0;
      while (bb - run > lo && bb[-1 - (ptrdiff_t)run] == '\\') ++run;
      if ((run & 1) == 0) {
        cut -= k + 1;
        break;
      }
    }
  }
  return cut;
}
}  // namespace

void logs_prefetch(const uint8_t* body, size_t avail, LogsPrefetch& st, char* dst, size_t cap, NlPos* nl) {
  if (st.state < 0 || st.state == 2 || !dst) return;
  if (st.state == 0) {
    // locate the member at geometrically growing prefixes (the locating parses cost at most twice
    // the prefix); a body whose `logs` member is not within its first 256 KiB is not prefetched
    if (st.tries > 0 && avail < 2 * st.tried_at) return;
    if (st.tried_at > (256u << 10)) {
      st.state = -1;
      return;
    }
    ++st.tries;
    st.tried_at = avail;
    const size_t at = locate_logs(body, avail);
    if (at == 0) return;
    st.state = 1;
    st.s0 = at;
    st.src = at + 1;
    st.dlen = 0;
    if (nl) nl->n = 0;
  }
  // decode [src, cut): 8 bytes stay behind the arrival front so the cut test reads arrived bytes
  if (avail < st.src + 64 + 8) return;
  const uint8_t* lo = body + st.s0 + 1;
  const uint8_t* cut = safe_cut(lo, body + avail - 8);
  if (cut <= body + st.src) return;
  if ((size_t)(cut - lo) + 64 > cap) {
    st.state = -1;
    return;
  }
  Cur c{body + st.src, cut};
  c.nl = nl;
  c.w0 = dst;
  char* w = str_into_span(c, dst + st.dlen);
  if (!w) {        // invalid or json.loads territory: the final parse decides (and answers)
    st.state = -1;
    return;
  }
  st.dlen = (size_t)(w - dst);
  st.src = (size_t)(c.p - body);
  if (c.closed) st.state = 2;
}

int parse_pod_request(const uint8_t* body, size_t n, PodRequest& out, bool decode_logs) {
  return parse_pod_impl(body, n, out, decode_logs, nullptr, 0, nullptr, nullptr);
}

int parse_pod_request_into(const uint8_t* body, size_t n, PodRequest& out, char* dst, size_t cap,
                           const LogsPrefetch* pf, NlPos* nl) {
  return parse_pod_impl(body, n, out, false, dst, cap, pf && pf->state >= 1 ? pf : nullptr, nl);
}

namespace {
int parse_pod_impl(const uint8_t* body, size_t n, PodRequest& out, bool decode_logs, char* dst, size_t cap,
                   const LogsPrefetch* pf, NlPos* nl) {
  out = PodRequest{};
  if (n >= 2 && (body[0] == 0 || body[1] == 0)) return JIN_FALLBACK;      // UTF-16/32
  if (n >= 3 && body[0] == 0xEF && body[1] == 0xBB && body[2] == 0xBF) return JIN_FALLBACK;  // BOM
  Cur c{body, body + n};
  ws(c);
  if (c.p >= c.e) return JIN_INVALID;
  bool ok;
  if (*c.p != '{') {
    ok = value(c);                       // valid JSON that is not an object -> invalid request
    ws(c);
    if (c.fallback) return JIN_FALLBACK;
    return (ok && c.p == c.e) ? JIN_NOT_OBJECT : JIN_INVALID;
  }
  ok = object(c, [&](const std::string& key, Cur& cc) {
    if (key == "logs") {
      if (cc.p < cc.e && *cc.p == '"' && dst && (size_t)(cc.e - cc.p) + 64 <= cap) {
        // validated and decoded in one pass into the caller's buffer (a later duplicate key
        // overwrites it: the last one wins, as in json.loads). A prefix decoded while the body
        // arrived (logs_prefetch, same member: same offset) resumes at its end.
        const uint8_t* s0 = cc.p;
        char* end;
        cc.w0 = dst;
        cc.nl = nl;
        if (pf && (size_t)(s0 - body) == pf->s0 && pf->src <= n) {
          cc.p = body + pf->src;
          end = pf->state == 2 ? dst + pf->dlen : str_loop<false>(cc, dst + pf->dlen);
        } else {
          if (nl) nl->n = 0;
          end = str_into(cc, dst);
        }
        cc.nl = nullptr;
        if (!end) {
          out.logs_decoded = false;
          return false;
        }
        out.logs.clear();
        out.logs_kind = 1;
        out.logs_decoded = true;
        out.logs_dlen = (size_t)(end - dst);
        out.logs_off = (size_t)(s0 + 1 - body);
        out.logs_len = (size_t)(cc.p - s0 - 2);
        return true;
      }
      out.logs_decoded = false;
      if (cc.p < cc.e && *cc.p == '"' && !decode_logs) {
        out.logs.clear();
        out.logs_kind = 1;
        const uint8_t* s0 = cc.p;
        out.logs_dlen = 0;
        if (!str(cc, nullptr, &out.logs_dlen)) return false;
        out.logs_off = (size_t)(s0 + 1 - body);
        out.logs_len = (size_t)(cc.p - s0 - 2);
        return true;
      }
      if (cc.p < cc.e && *cc.p == '"') {
        // one allocation for the (large) log text, decoded in place, then trimmed
        out.logs.resize((size_t)(cc.e - cc.p) + 64);
        out.logs_kind = 1;
        char* end = str_into(cc, &out.logs[0]);
        if (!end) {
          out.logs.clear();
          return false;
        }
        out.logs.resize((size_t)(end - out.logs.data()));
        return true;
      }
      out.logs.clear();
      out.logs_kind = (cc.p < cc.e && *cc.p == 'n') ? 0 : 2;
      return value(cc);
    }
    if (key == "pod") {
      out.has_name = false;
      out.pod_name.clear();
      if (cc.p < cc.e && *cc.p == 'n') {
        out.pod_nonnull = false;
        return lit(cc, "null");
      }
      out.pod_nonnull = true;
      if (cc.p < cc.e && *cc.p == '{') {
        return object(cc, [&](const std::string& k2, Cur& c2) {
          if (k2 == "metadata" && c2.p < c2.e && *c2.p == '{') {
            out.has_name = false;
            out.pod_name.clear();
            return object(c2, [&](const std::string& k3, Cur& c3) {
              if (k3 == "name" && c3.p < c3.e && *c3.p == '"') {
                out.pod_name.clear();
                out.has_name = true;
                return str(c3, &out.pod_name);
              }
              if (k3 == "name") {
                out.has_name = false;
                out.pod_name.clear();
              }
              return value(c3);
            });
          }
          if (k2 == "metadata") {
            out.has_name = false;
            out.pod_name.clear();
          }
          return value(c2);
        });
      }
      return value(cc);
    }
    return value(cc);
  });
  if (c.fallback) return JIN_FALLBACK;
  if (!ok) return JIN_INVALID;
  ws(c);
  if (c.p != c.e) return JIN_INVALID;
  return JIN_OK;
}
}  // namespace

}  // namespace lp
