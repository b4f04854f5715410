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

namespace lp {
namespace {

struct Cur {
  const uint8_t* p;
  const uint8_t* e;
  int depth = 0;
  bool fallback = false;
};

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

// string at c.p (opening quote); appends the decoded UTF-8 to `out` when non-null
bool str(Cur& c, std::string* out) {
  if (c.p >= c.e || *c.p != '"') return false;
  ++c.p;
  for (;;) {
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

int parse_pod_request(const uint8_t* body, size_t n, PodRequest& out) {
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
      if (cc.p < cc.e && *cc.p == '"') {
        out.logs.clear();
        out.logs.reserve((size_t)(cc.e - cc.p));   // one allocation for the (large) log text
        out.logs_kind = 1;
        return str(cc, &out.logs);
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

}  // namespace lp
