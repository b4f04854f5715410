// Native decoder of POST /parse request bodies (see json_in.cpp).
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <memory>
#include <string>

namespace lp {

enum { JIN_OK = 0, JIN_INVALID = 1, JIN_NOT_OBJECT = 2, JIN_FALLBACK = 3 };

struct PodRequest {
  bool pod_nonnull = false;   // `pod` present and not null (Parse.java:45)
  bool has_name = false;      // pod.metadata.name is a string
  std::string pod_name;
  int logs_kind = 0;          // 0 absent / null, 1 string, 2 other type
  std::string logs;           // UTF-8, escapes decoded (decode_logs mode)
  size_t logs_off = 0;        // logs_kind 1: the raw JSON string's content (between the quotes)
  size_t logs_len = 0;        //   as an offset / length into the body
  size_t logs_dlen = 0;       //   and its decoded UTF-8 length
  bool logs_decoded = false;  // parse_pod_request_into: the text is decoded in the caller's buffer
};

// Validates the whole body. With decode_logs the `logs` string is unescaped into out.logs;
// without it only its raw span is recorded (decode later with decode_json_string, e.g. straight
// into a Python bytes object -- the HTTP front end's one-copy path).
int parse_pod_request(const uint8_t* body, size_t n, PodRequest& out, bool decode_logs = true);

// Positions (offsets into the decoded text) of the '\n' bytes the decoder writes -- in a JSON string
// every newline is an escape (\n or \u000a: raw control bytes are invalid), so the decoder sees each
// one anyway and the batch packer need not scan the text again (pack_split_docs `nlpos`).
// Grow-only, uninitialised storage; the block decoder stores 8 positions unconditionally per block.
struct NlPos {
  std::unique_ptr<int64_t[]> p;
  size_t n = 0, cap = 0;
  void reserve(size_t c) {
    if (c <= cap) return;
    const size_t k = c < 2 * cap ? 2 * cap : c;
    std::unique_ptr<int64_t[]> q(new int64_t[k]);
    if (n) std::memcpy(q.get(), p.get(), n * sizeof(int64_t));
    p = std::move(q);
    cap = k;
  }
};

// Decoding of the top-level `logs` string while a body is still arriving (the HTTP front end's IO
// thread between reads: the 1 MB string's validation and unescaping overlap the receive instead of
// following its last byte). The prefix [s0 + 1, src) of the string is decoded to dst[0, dlen);
// `src` is always a token boundary, so the final parse resumes there and produces exactly the
// bytes and verdict of a one-pass parse. Nothing here decides a request: an invalid or unusual
// prefix only turns the prefetch off (state -1), and the final parse answers.
struct LogsPrefetch {
  int state = 0;        // 0 locating the member, 1 decoding, 2 closing quote consumed, -1 off
  int tries = 0;        // locate attempts (at prefixes of doubling length)
  size_t tried_at = 0;  // bytes available at the last attempt
  size_t s0 = 0;        // body offset of the string's opening quote
  size_t src = 0;       // body offset decoded up to (state 2: one past the closing quote)
  size_t dlen = 0;      // decoded bytes in dst
  void reset() { *this = LogsPrefetch(); }
};

// Advances `st` over the first `avail` arrived bytes of a body. `dst` / `cap` as for
// parse_pod_request_into (the same buffer must be passed there with `st`).
// `nl` (optional): the decoded newlines' positions (kept in step with dlen; reset when the decoding
// restarts).
void logs_prefetch(const uint8_t* body, size_t avail, LogsPrefetch& st, char* dst, size_t cap, NlPos* nl = nullptr);

// Validates the whole body like parse_pod_request and decodes the `logs` string into `dst` in the
// same pass (the HTTP front end's IO thread, while the bytes are in its cache): logs_decoded is set
// and logs_dlen is the decoded length. `dst` needs room for the escaped length + 64 bytes (block
// stores run past the decoded end); a string that does not fit is only validated (skip mode).
// With `pf` (a logs_prefetch state over a prefix of this body, into this dst) the string's
// decoding resumes where the prefetch stopped.
// `nl` (optional): the positions of the '\n' bytes in dst[0, logs_dlen) (with `pf`: the prefetch's
// sink, continued).
int parse_pod_request_into(const uint8_t* body, size_t n, PodRequest& out, char* dst, size_t cap,
                           const LogsPrefetch* pf = nullptr, NlPos* nl = nullptr);

// Unescapes the content of a JSON string that parse_pod_request validated (`n` raw bytes between
// the quotes) into `w`, which must have room for n + 64 bytes; returns the decoded length.
size_t decode_json_string(const uint8_t* p, size_t n, char* w);
// the same, writing nothing past the decoded end (documents decoded side by side by several
// threads into one buffer); returns the decoded length, 0 on an invalid escape
size_t decode_json_string_exact(const uint8_t* p, size_t n, char* w);

}  // namespace lp
