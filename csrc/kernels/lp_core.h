// Shared host/device building blocks of the log-analysis pipeline.
//
// Every routine here is compiled twice from the same source: into gfx950 kernels (HIP) and into
// the host (CPU) backend used by CPU-only tests and as the availability fallback. Keeping one
// source guarantees the CPU tests exercise the exact arithmetic the GPU runs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define LP_HD __host__ __device__ __forceinline__

namespace lp {

// Block-wide global -> LDS staging of a table with U loads in flight per lane: all of a lane's
// loads are issued before its first LDS store, so staging costs ~one memory round trip per U
// elements per lane instead of one per element (a loop of load -> ds_write pairs waits on every
// load: ~10 serial L2/HBM trips per lane for a 42 KB scan blob in a 256-thread block).
// The loads are unconditional (index clamped to n - 1) so `v` stays in registers: a guarded
// load left the array partially defined and the compiler put it in scratch memory.
template <typename T, int U = 8>
__device__ __forceinline__ void lds_fill(T* dst, const T* __restrict__ src, int n) {
  for (int b = threadIdx.x; b < n; b += U * (int)blockDim.x) {
    T v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int i = b + j * (int)blockDim.x;
      v[j] = src[i < n ? i : n - 1];
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int i = b + j * (int)blockDim.x;
      if (i < n) dst[i] = v[j];
    }
  }
}

// --------------------------------------------------------------------------------------------
// DFA pool (all regexes of a library, concatenated).  meta[r*4 + {0,1,2,3}] =
//   {trans offset (uint16 units), nclasses, accflags offset, flags(bit0 anchored)}
struct DfaPool {
  const int32_t* meta;
  const uint8_t* bytemap;   // [R][256]
  const uint16_t* trans;
  const uint8_t* acc;
  const uint64_t* bpg = nullptr;   // bit-parallel Glushkov programs (meta flag bit1, offset in meta[0])
  uint32_t bpg_widths = 0;         // bit W set: some program has W words (which bpg.hip kernels to launch)
  uint32_t bpg_words = 0;          // length of the program pool (uint64 words): staged in LDS when it fits
};

LP_HD int final_term_len(const uint8_t* s, int n) {
  if (n >= 1 && s[n - 1] == '\r') return 1;
  if (n >= 2 && s[n - 2] == 0xC2 && s[n - 1] == 0x85) return 2;
  if (n >= 3 && s[n - 3] == 0xE2 && s[n - 2] == 0x80 && (s[n - 1] == 0xA8 || s[n - 1] == 0xA9)) return 3;
  return 0;
}
}  // namespace lp

#include "bpg.h"

namespace lp {

// One DFA of the pool: transition rows (nc classes per state), byte -> class map, accept flags
// (bit0: accepting at end of line, bit1: accepting before a final line terminator). States 0
// (dead) and 1 (match found) are terminal.
struct DfaRef {
  const uint16_t* T;
  const uint8_t* bm;
  const uint8_t* A;
  int nc;
};
LP_HD DfaRef dfa_ref(const DfaPool& P, int r) {
  const int32_t* m = P.meta + 4 * r;
  return DfaRef{P.trans + m[0], P.bytemap + 256 * r, P.acc + m[2], m[1]};
}

#if defined(__HIP_DEVICE_COMPILE__)
// Advance K DFAs together over bytes s[0, e). Device form of the walk: bytes come from 16-byte
// ALIGNED vector loads one block ahead (a 1-byte load per step would put a memory round trip on
// the dependency chain); every step is branch-free (terminal states absorb via a select) and the
// K chains are independent, so a step costs ~6 instructions per DFA and the table reads of the K
// walks overlap. The earlier byte-at-a-time walk with per-step early exits compiled to ~500
// instructions per step (~1900 cycles, tools/feat_probe). Callers' buffers are padded (text:
// TEXT_PAD) so the look-ahead load stays in bounds.
template <int K>
__device__ __forceinline__ void dfa_advance(const DfaRef (&D)[K], const uint8_t* s, int e, int (&st)[K]) {
  if (e <= 0) return;
  const int sh = (int)((uintptr_t)s & 15);
  const uint4* blk = reinterpret_cast<const uint4*>(s - sh);
  uint4 cur = blk[0];
  for (int t0 = -sh; t0 < e; t0 += 16) {
    const uint4 nxt = blk[1];
    ++blk;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int t = t0 + j;
      const bool on = (t >= 0) & (t < e);
      const uint32_t w = (j < 4) ? cur.x : (j < 8) ? cur.y : (j < 12) ? cur.z : cur.w;
      const int c = (int)((w >> (8 * (j & 3))) & 0xFFu);
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int nx = D[k].T[st[k] * D[k].nc + D[k].bm[c]];
        st[k] = (on && st[k] >= 2) ? nx : st[k];
      }
    }
    cur = nxt;
    bool alive = false;
#pragma unroll
    for (int k = 0; k < K; ++k) alive |= st[k] >= 2;
    if (!alive) return;
  }
}

// find() over one line for K DFAs: res bit k = DFA k matches (java.util.regex Matcher.find
// semantics, see jregex.h): accept before a final line terminator, then at end of line.
template <int K>
__device__ __forceinline__ uint32_t dfa_find_k(const DfaRef (&D)[K], const uint8_t* s, int n) {
  int st[K];
#pragma unroll
  for (int k = 0; k < K; ++k) st[k] = 2;
  const int ftl = final_term_len(s, n);
  const int ft = ftl ? n - ftl : n;
  dfa_advance<K>(D, s, ft, st);
  if (ftl) {
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (st[k] >= 2 && (D[k].A[st[k]] & 2)) st[k] = 1;
    dfa_advance<K>(D, s + ft, ftl, st);
  }
  uint32_t res = 0;
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (st[k] == 1 || (st[k] >= 2 && (D[k].A[st[k]] & 1))) res |= 1u << k;
  return res;
}
#endif

// find() of regex r over one line (java.util.regex Matcher.find semantics, see jregex.h)
// regex r is a bit-parallel Glushkov program (DFA blow-up), not a DFA of the pool
LP_HD bool is_bpg(const DfaPool& P, int r) { return (P.meta[4 * r + 3] & 2) != 0; }
// regex r is a backtracker regex whose automaton is its regular RELAXATION: its device keys are
// candidates for the host backtracker, never hits (side_path.hip)
LP_HD bool is_host_dev(const DfaPool& P, int r) { return (P.meta[4 * r + 3] & 4) != 0; }

LP_HD bool dfa_run(const DfaPool& P, int r, const uint8_t* s, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (is_bpg(P, r)) return false;      // verified by the bpg.hip kernels launched next to this one
  const DfaRef D[1] = {dfa_ref(P, r)};
  return dfa_find_k<1>(D, s, n) != 0;
#else
  if (is_bpg(P, r)) return bpg_find_host(P.bpg + P.meta[4 * r], s, n);
  const DfaRef D = dfa_ref(P, r);
  int ft = n - final_term_len(s, n);
  if (ft == n) ft = -1;
  int st = 2;
  for (int t = 0; t < n; ++t) {
    if (t == ft && (D.A[st] & 2)) return true;
    st = D.T[st * D.nc + D.bm[s[t]]];
    if (st < 2) return st == 1;
  }
  return (D.A[st] & 1) != 0;
#endif
}

// Context features of one line (ContextAnalysisService.java:62-83); DFAs 0..3 of the pool are the
// four internal regexes: bit0 ERROR, bit1 WARN (only when not ERROR: the reference's else-if),
// bit2 stack-trace line, bit3 exception/error class name. On the device the 4 walks advance
// together over one byte stream (4 independent dependency chains per step instead of 4 passes).
LP_HD uint8_t context_feat(const DfaPool& P, const uint8_t* s, int len) {
#if defined(__HIP_DEVICE_COMPILE__)
  const DfaRef D[4] = {dfa_ref(P, 0), dfa_ref(P, 1), dfa_ref(P, 2), dfa_ref(P, 3)};
  const uint32_t res = dfa_find_k<4>(D, s, len);
  const uint8_t f = (res & 1u) ? 1 : ((res & 2u) ? 2 : 0);
  return (uint8_t)(f | (res & 12u));
#else
  // host: the 4 walks advance together too (4 independent table-load chains per byte for the
  // out-of-order core instead of 4 passes); same Matcher.find semantics as dfa_find_k
  const DfaRef D[4] = {dfa_ref(P, 0), dfa_ref(P, 1), dfa_ref(P, 2), dfa_ref(P, 3)};
  int st[4] = {2, 2, 2, 2};
  auto advance = [&](const uint8_t* q, int e) {
    for (int t = 0; t < e; ++t) {
      const int c = q[t];
      bool alive = false;
      for (int k = 0; k < 4; ++k) {
        if (st[k] >= 2) st[k] = D[k].T[st[k] * D[k].nc + D[k].bm[c]];
        alive |= st[k] >= 2;
      }
      if (!alive) return;
    }
  };
  const int ftl = final_term_len(s, len);
  const int ft = len - ftl;
  advance(s, ft);
  if (ftl) {
    for (int k = 0; k < 4; ++k)
      if (st[k] >= 2 && (D[k].A[st[k]] & 2)) st[k] = 1;
    advance(s + ft, ftl);
  }
  uint32_t res = 0;
  for (int k = 0; k < 4; ++k)
    if (st[k] == 1 || (st[k] >= 2 && (D[k].A[st[k]] & 1))) res |= 1u << k;
  const uint8_t f = (res & 1u) ? 1 : ((res & 2u) ? 2 : 0);
  return (uint8_t)(f | (res & 12u));
#endif
}

// --------------------------------------------------------------------------------------------
// literal prefilter tables
struct PfTables {
  const uint32_t* bloom;    // 1<<bloom_bits bits
  int bloom_bits;
  const uint64_t* ht_key;   // open addressing, EMPTY = ~0
  const int32_t* ht_val;    // start into gram_lits
  const int32_t* ht_cnt;
  uint32_t ht_mask;
  const int32_t* gram_lits;
  const int32_t* lit_off;   // [nlit+1] into lit_bytes
  const uint8_t* lit_bytes; // ASCII-lowercased
  const int32_t* lit_reg_off;
  const int32_t* lit_reg;
  int gmask;                // bit g set when grams of length g (2..4) exist (bloom tier)
  int stride;               // S in {1, 2, 4}: every bloom literal indexes S adjacent windows -> test
                            // positions divisible by S (literals of >= S + 3 bytes)
  // short-literal (Teddy) tier: teddy[4c + j] = buckets whose 3-byte window has byte c at offset j
  const uint32_t* teddy;    // [256 * 4]
  const int32_t* tb_off;    // [33] bucket CSR into tb_lits
  const int32_t* tb_lits;   // literal id | window offset << 22 (as gram_lits)
  int teddy_on;
  // per bucket entry (gram_lits / tb_lits order): {fingerprint, mask} of the literal's bytes in the 4
  // text positions before and the 4 after the indexed window (models/compiled.py _fingerprint)
  const uint64_t* gram_fp = nullptr;
  const uint64_t* tb_fp = nullptr;
};

// gram_lits entry: literal id | (offset of the indexed window inside the literal << 22)
constexpr int LIT_OFF_SHIFT = 22;
LP_HD int pf_entry_lit(int32_t e) { return e & ((1 << LIT_OFF_SHIFT) - 1); }
LP_HD int pf_entry_off(int32_t e) { return (int)((uint32_t)e >> LIT_OFF_SHIFT); }

LP_HD uint32_t gram_mask(int g) { return g >= 4 ? 0xFFFFFFFFu : ((1u << (8 * g)) - 1u); }
// Blocked bloom filter: one 32-bit word per key holds both probe bits, so a membership test is
// ONE LDS read (the unblocked 2-hash form measured 4.8 bank-conflict cycles per LDS instruction).
// ONE 32-bit multiply per test (v_mul_lo_u32 is quarter rate on CDNA; the previous form used
// two): the word index is the top bits of the product, the two bit positions come from the
// product xor-shifted so its high bits reach the low ones (measured false-positive rate on a
// 1k-pattern library: 2163 vs 2324 passes per 2.1M tests).
LP_HD uint32_t bloom_hash(uint32_t key, int g) { return (key ^ (uint32_t)g * 0x9E3779B9u) * 0x85EBCA6Bu; }
LP_HD uint32_t bloom_word(uint32_t key, int g, int bits) {   // word index among 2^(bits-5) words
  return bloom_hash(key, g) >> (32 - (bits - 5));
}
LP_HD uint32_t bloom_bits_of(uint32_t p) {                     // three bit positions inside the word
  // k = 3: a false positive needs 3 set bits of one word (~20x rarer than k = 2 at our load); it
  // matters because one frequent text gram (a timestamp fragment) colliding costs a hit per line
  const uint32_t q = p ^ (p >> 15);
  return (1u << (q & 31)) | (1u << ((q >> 5) & 31)) | (1u << ((q >> 10) & 31));
}
LP_HD uint32_t bloom_bits2(uint32_t key, int g) { return bloom_bits_of(bloom_hash(key, g)); }
LP_HD bool bloom_test(const uint32_t* bl, uint32_t key, int g, int bits) {
  const uint32_t p = bloom_hash(key, g);
  const uint32_t m = bloom_bits_of(p);
  return (bl[p >> (32 - (bits - 5))] & m) == m;
}
LP_HD uint32_t ht_hash(uint32_t key, int g) {
  uint32_t h = key * 0x9E3779B1u ^ ((uint32_t)g * 0x7FEB352Du);
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  return h;
}
LP_HD int lower_byte(int c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }
// SWAR ASCII lower-casing of 4 packed bytes (bytes >= 0x80 untouched)
LP_HD uint32_t lower4(uint32_t x) {
  uint32_t hi = 0x80808080u;
  uint32_t ge_A = ((x | hi) - 0x41414141u) & hi;   // byte >= 'A' (for < 0x80)
  uint32_t ge_Z1 = ((x | hi) - 0x5B5B5B5Bu) & hi;  // byte >= 'Z'+1
  uint32_t up = ge_A & ~ge_Z1 & ~x & hi;
  return x | (up >> 2);
}

// largest index i in [0,n) with a[i] <= v  (a sorted ascending); -1 if none
LP_HD int64_t upper_idx(const int64_t* a, int64_t n, int64_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (a[mid] <= v) lo = mid + 1; else hi = mid;
  }
  return lo - 1;
}
// first index in [lo,hi) with a[i] >= v
LP_HD int64_t lower_bound32(const int32_t* a, int64_t lo, int64_t hi, int32_t v) {
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// Line containing byte `pos`. With a coarse index blk[b] = line containing byte b << 12 (built
// once per request) the search covers one 4 KiB block's lines instead of all L lines.
constexpr int LINE_BLK_SHIFT = 12;
LP_HD int64_t locate_line(const int64_t* ls, int64_t n, const int32_t* blk, int64_t pos) {
  if (!blk) return upper_idx(ls, n, pos);
  const int64_t b = pos >> LINE_BLK_SHIFT;
  int64_t lo = blk[b], hi = (int64_t)blk[b + 1] + 1;
  if (hi > n) hi = n;
  if (lo > n - 1) lo = n - 1;                    // bytes of trimmed trailing empty lines
  while (lo + 1 < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (ls[mid] <= pos) lo = mid; else hi = mid;
  }
  return lo;
}

#if defined(__HIP__)
// 16 bytes starting at p (any alignment) from two aligned vector loads + byte funnel shifts
__device__ __forceinline__ void load16u(const uint8_t* p, uint32_t out[4]) {
  const int sh = (int)((uintptr_t)p & 15);
  const uint4* b = reinterpret_cast<const uint4*>(p - sh);
  const uint4 x = b[0], y = b[1];
  uint32_t a0 = x.x, a1 = x.y, a2 = x.z, a3 = x.w, a4 = y.x, a5 = y.y, a6 = y.z, a7 = y.w;
  const int q = sh >> 2, r = sh & 3;
  if (q & 2) { a0 = a2; a1 = a3; a2 = a4; a3 = a5; a4 = a6; a5 = a7; }
  if (q & 1) { a0 = a1; a1 = a2; a2 = a3; a3 = a4; a4 = a5; }
  out[0] = __builtin_amdgcn_alignbyte(a1, a0, r);
  out[1] = __builtin_amdgcn_alignbyte(a2, a1, r);
  out[2] = __builtin_amdgcn_alignbyte(a3, a2, r);
  out[3] = __builtin_amdgcn_alignbyte(a4, a3, r);
}
// ASCII-case-insensitive compare of text against a lower-cased literal, 16 bytes per round trip
// (a byte-at-a-time loop with early exit is one dependent memory round trip per byte)
__device__ __forceinline__ bool lit_match16(const uint8_t* t, const uint8_t* lit, int len) {
  for (int q = 0; q < len; q += 16) {
    uint32_t a[4], b[4];
    load16u(t + q, a);
    load16u(lit + q, b);
    const int rem = len - q;
    uint32_t diff = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = rem - 4 * i;
      const uint32_t m = k >= 4 ? 0xFFFFFFFFu : (k <= 0 ? 0u : ((1u << (8 * k)) - 1u));
      diff |= (lower4(a[i]) ^ b[i]) & m;
    }
    if (diff) return false;
  }
  return true;
}
#endif

// Hash-table bucket of a gram hit: literals gram_lits[s .. s+c) share that gram (c = 0: none).
LP_HD void pf_bucket(const PfTables& T, uint32_t gram, int g, int& s, int& c) {
  const uint64_t key = (uint64_t)gram | ((uint64_t)g << 32);
  uint32_t h = ht_hash(gram, g) & T.ht_mask;
  s = 0;
  c = 0;
  for (;;) {
    const uint64_t kk = T.ht_key[h];
    if (kk == ~0ull) return;
    if (kk == key) break;
    h = (h + 1) & T.ht_mask;
  }
  s = T.ht_val[h];
  c = T.ht_cnt[h];
}

// Does the literal of gram entry `e` occur with its indexed window at text position p (ASCII
// case-insensitive)?
LP_HD bool pf_lit_at(const PfTables& T, const uint8_t* text, int64_t nbytes, int64_t p, int32_t e) {
  const int lit = pf_entry_lit(e);
  const int lo = T.lit_off[lit], len = T.lit_off[lit + 1] - lo;
  const int64_t st = p - pf_entry_off(e);
  if (st < 0 || st + len > nbytes) return false;
#if defined(__HIP_DEVICE_COMPILE__)
  return lit_match16(text + st, T.lit_bytes + lo, len);
#else
  for (int q = 0; q < len; ++q)
    if (lower_byte(text[st + q]) != T.lit_bytes[lo + q]) return false;
  return true;
#endif
}

// Probe one gram hit at text position p; appends (regex<<32 | line) candidates. A literal never
// contains '\n', so every literal of the bucket that matches lies on the line of p.
template <typename AppendFn>
LP_HD void pf_probe(const PfTables& T, const uint8_t* text, int64_t nbytes, int64_t p, uint32_t gram, int g,
                    const int64_t* line_start, int64_t nlines, const int32_t* blk_line, AppendFn&& append) {
  int s, c;
  pf_bucket(T, gram, g, s, c);
  int64_t line = -1;
  for (int j = 0; j < c; ++j) {
    const int32_t e = T.gram_lits[s + j];
    if (!pf_lit_at(T, text, nbytes, p, e)) continue;
    const int lit = pf_entry_lit(e);
    if (line < 0) line = locate_line(line_start, nlines, blk_line, p);
    if (line < 0) line = 0;
    for (int r = T.lit_reg_off[lit]; r < T.lit_reg_off[lit + 1]; ++r)
      append(((int64_t)T.lit_reg[r] << 32) | line);
  }
}

// Short-literal tier: bucket mask of the 3-byte window at text position p (bytes past nbytes are
// the zero padding, and byte 0 is in no window: no match there).
LP_HD uint32_t teddy_mask(const PfTables& T, const uint8_t* text, int64_t nbytes, int64_t p) {
  const int b0 = lower_byte(text[p]);
  const int b1 = p + 1 < nbytes ? lower_byte(text[p + 1]) : 0;
  const int b2 = p + 2 < nbytes ? lower_byte(text[p + 2]) : 0;
  return T.teddy[4 * b0] & T.teddy[4 * b1 + 1] & T.teddy[4 * b2 + 2];
}

// Probe one short-literal candidate position (host twin / small inputs): verify every literal of
// every bucket in the mask, append (regex << 32 | line).
template <typename AppendFn>
LP_HD void teddy_probe(const PfTables& T, const uint8_t* text, int64_t nbytes, int64_t p, uint32_t m,
                       const int64_t* line_start, int64_t nlines, const int32_t* blk_line, AppendFn&& append) {
  int64_t line = -1;
  while (m) {
    const int b = __builtin_ctz(m);
    m &= m - 1;
    for (int j = T.tb_off[b]; j < T.tb_off[b + 1]; ++j) {
      const int32_t e = T.tb_lits[j];
      if (!pf_lit_at(T, text, nbytes, p, e)) continue;
      const int lit = pf_entry_lit(e);
      if (line < 0) line = locate_line(line_start, nlines, blk_line, p);
      if (line < 0) line = 0;
      for (int r = T.lit_reg_off[lit]; r < T.lit_reg_off[lit + 1]; ++r)
        append(((int64_t)T.lit_reg[r] << 32) | line);
    }
  }
}

// --------------------------------------------------------------------------------------------
// scoring (fp64, Java double semantics, left-to-right product: ScoringService.java:102-109)
struct ScoreParams {
  double decay;          // scoring.proximity.decay-constant
  double early, maxearly, penalty;   // chronological
  double max_ctx;        // scoring.context.max-context-factor
  double fthr, fmaxp, fwin;          // frequency
};

struct ScoreTables {
  // per pattern
  const double* conf; const double* sev;
  const int32_t* ctx_before; const int32_t* ctx_after;   // -1: rules null
  const int32_t* sec_off; const int32_t* sec_reg; const int32_t* sec_w; const double* sec_weight;
  const int32_t* seq_off; const double* seq_bonus; const int32_t* seq_ev_off; const int32_t* seq_ev_reg;
  const uint8_t* seq_carry;   // per sequence event slot: chain satisfiable in earlier shards
  // per regex hit lists (CSR, lines ascending)
  const int64_t* hit_off; const int32_t* hit_line;
  const uint8_t* feat;        // per local line: 1 ERR, 2 WARN, 4 STACK, 8 EXC
  // per segment (document / shard)
  const int32_t* seg_lo; const int32_t* seg_hi; const int32_t* seg_own_lo;
  const int64_t* seg_g0; const int64_t* seg_n;
};

// Frequency input of the score: penalty count of event i = carry[key] (matches recorded before
// this batch/shard, persistent + earlier ranks) + rank among earlier same-key events of the batch;
// -1 = pattern without id (no penalty). FrequencyTrackingService.java:64-93, ScoringService.java:84-88.
struct FreqIn {
  const int64_t* rank;
  const int64_t* fkey;
  const int64_t* carry;
};
LP_HD int64_t freq_before(const FreqIn& F, int64_t i) {
  const int64_t k = F.fkey[i];
  return k >= 0 ? F.carry[k] + F.rank[i] : -1;
}

LP_HD double chrono_factor(int64_t gi, int64_t n, const ScoreParams& S) {
  const double pos = (double)gi / (double)n;
  if (pos <= S.early) return 1.5 + (S.early - pos) * ((S.maxearly - 1.5) / S.early);
  if (pos <= S.penalty) return 1.0 + (S.penalty - pos) * (0.5 / (S.penalty - S.early));
  return 0.5 + (1.0 - pos);
}

// any hit of regex r within local [a,b)
LP_HD bool any_hit(const ScoreTables& T, int r, int32_t a, int32_t b) {
  if (r < 0 || a >= b) return false;
  const int64_t lo = T.hit_off[r], hi = T.hit_off[r + 1];
  const int64_t i = lower_bound32(T.hit_line, lo, hi, a);
  return i < hi && T.hit_line[i] < b;
}

// nearest hit distance of regex r to x within [a,b), x excluded; -1 if none
LP_HD int32_t nearest_hit(const ScoreTables& T, int r, int32_t x, int32_t a, int32_t b) {
  if (r < 0 || a >= b) return -1;
  const int64_t lo = T.hit_off[r], hi = T.hit_off[r + 1];
  int64_t i = lower_bound32(T.hit_line, lo, hi, x);
  int32_t best = -1;
  int64_t j = i;
  if (j < hi && T.hit_line[j] == x) ++j;
  if (j < hi && T.hit_line[j] < b) best = T.hit_line[j] - x;
  if (i - 1 >= lo) {
    const int32_t y = T.hit_line[i - 1];
    if (y >= a && (best < 0 || x - y < best)) best = x - y;
  }
  return best;
}

// largest hit of regex r in [a, c); -1 if none
LP_HD int32_t pred_hit(const ScoreTables& T, int r, int32_t a, int32_t c) {
  if (r < 0 || a >= c) return -1;
  const int64_t lo = T.hit_off[r], hi = T.hit_off[r + 1];
  const int64_t i = lower_bound32(T.hit_line, lo, hi, c);
  if (i - 1 >= lo && T.hit_line[i - 1] >= a) return T.hit_line[i - 1];
  return -1;
}

// The factors of one event's score, each a function of its own: the request tail runs them in
// different waves (one chain of dependent loads each) and multiplies them as score_event does.
// proximity (ScoringService.java:161-190,315-347)
LP_HD double prox_factor(const ScoreTables& T, const ScoreParams& S, int32_t x, int32_t p, int32_t lo, int32_t hi) {
  double prox = 1.0;
  const int32_t a0 = T.sec_off[p], a1 = T.sec_off[p + 1];
  if (a1 > a0) {
    double tot = 0.0;
    for (int32_t k = a0; k < a1; ++k) {
      const int32_t w = T.sec_w[k];
      const int64_t aa = (int64_t)x - w, bb = (int64_t)x + w + 1;
      const int32_t a = (int32_t)(aa < lo ? lo : aa), b = (int32_t)(bb > hi ? hi : bb);
      const int32_t d = nearest_hit(T, T.sec_reg[k], x, a, b);
      if (d >= 0) tot += T.sec_weight[k] * exp(-(double)d / S.decay);
    }
    prox = 1.0 + tot;
  }
  return prox;
}

// temporal (ScoringService.java:199-305)
LP_HD double temp_factor(const ScoreTables& T, int32_t x, int32_t p, int32_t lo, int32_t hi, int32_t own_lo) {
  double temp = 1.0;
  const int32_t q0 = T.seq_off[p], q1 = T.seq_off[p + 1];
  if (q1 > q0) {
    double tot = 0.0;
    for (int32_t q = q0; q < q1; ++q) {
      const int32_t e0 = T.seq_ev_off[q], e1 = T.seq_ev_off[q + 1];
      const int n = e1 - e0;
      if (n <= 0) continue;
      const int32_t a = x - 5 < lo ? lo : x - 5, b = x + 6 > hi ? hi : x + 6;
      if (!any_hit(T, T.seq_ev_reg[e1 - 1], a, b)) continue;
      bool ok = true;
      int32_t cur = x;
      for (int k = n - 2; k >= 0; --k) {
        const int32_t f = pred_hit(T, T.seq_ev_reg[e0 + k], own_lo, cur);
        if (f < 0) { ok = T.seq_carry[e0 + k] != 0; break; }
        cur = f;
      }
      if (ok) tot += T.seq_bonus[q];
    }
    temp = 1.0 + tot;
  }
  return temp;
}

// context (ContextAnalysisService.java:46-117)
LP_HD double ctx_factor(const ScoreTables& T, const ScoreParams& S, int32_t x, int32_t p, int32_t lo, int32_t hi) {
  int32_t a = x, b = x + 1;
  const int32_t before = T.ctx_before[p], after = T.ctx_after[p];
  if (before >= 0) {
    a = x - before < lo ? lo : x - before;
    b = x + 1 + after > hi ? hi : x + 1 + after;
  }
  double sc = 0.0;
  int err = 0, stack = 0;
  // the window's feature bytes 8 at a time, all loads in flight before the (in-order) sums
  for (int32_t j0 = a; j0 < b; j0 += 8) {
    uint8_t fv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) fv[u] = j0 + u < b ? T.feat[j0 + u] : 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint8_t f = fv[u];
      if (f & 1) { ++err; sc += 0.4; }
      else if (f & 2) { sc += 0.2; }
      if (f & 4) { ++stack; sc += 0.1; }
      if (f & 8) { sc += 0.3; }
    }
  }
  if (stack > 0) { const double sb = stack * 0.1; sc += sb < 0.5 ? sb : 0.5; }
  const int total = b - a;
  if (total > 10 && (double)(stack + err) > total * 0.7) sc *= 0.8;
  double ctx = 1.0 + sc;
  if (ctx > S.max_ctx) ctx = S.max_ctx;
  return ctx;
}

// frequency penalty (FrequencyTrackingService.java:64-93), penalty before record
LP_HD double pen_factor(const ScoreParams& S, int64_t freq_before) {
  double pen = 0.0;
  if (freq_before >= 0) {
    const double rate = (double)freq_before / S.fwin;
    if (rate > S.fthr) { const double v = (rate - S.fthr) / S.fthr; pen = v < S.fmaxp ? v : S.fmaxp; }
  }
  return pen;
}

LP_HD double score_event(const ScoreTables& T, const ScoreParams& S, int32_t x, int32_t p, int32_t s,
                         int64_t freq_before, double* factors /* optional [7] */) {
  const int32_t lo = T.seg_lo[s], hi = T.seg_hi[s], own_lo = T.seg_own_lo[s];
  const int64_t gi = T.seg_g0[s] + (x - lo);
  const double conf = T.conf[p];
  const double sev = T.sev[p];
  const double chrono = chrono_factor(gi, T.seg_n[s], S);
  const double prox = prox_factor(T, S, x, p, lo, hi);
  const double temp = temp_factor(T, x, p, lo, hi, own_lo);
  const double ctx = ctx_factor(T, S, x, p, lo, hi);
  const double pen = pen_factor(S, freq_before);
  if (factors) {
    factors[0] = conf; factors[1] = sev; factors[2] = chrono; factors[3] = prox;
    factors[4] = temp; factors[5] = ctx; factors[6] = pen;
  }
  return conf * sev * chrono * prox * temp * ctx * (1.0 - pen);
}

}  // namespace lp
