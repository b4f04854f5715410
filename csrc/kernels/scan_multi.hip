// Literal-free regexes over every line: multi-regex DFAs walked together, tables in LDS.
//
// The reference runs every primary regex over every line (AnalysisService.java:89-95). Regexes
// with a usable literal factor are reached through the literal prefilter; the rest (e.g.
// "\b[A-Z]{3,}_\d{4}\b", IP:port shapes, "^\s+at ..." frames) must scan the whole text. They are
// compiled at library load into *scan groups*: up to 64 regexes determinised together into one
// multi-regex DFA (jregex.h MultiDfa), so one table walk per byte answers all members. A *pass*
// holds up to 4 groups walked together.
//
// Two copies of every group's automaton (models/compiled.py _scan_blob):
//   * LDS (hot loop): bm4 at byte 0 -- bm4[c] holds 2 x (column of byte c in group g) in byte
//     g, entries 256..511 are 0 (hold) -- then uint16 transition rows whose entries are the LDS
//     BYTE offset of the next state's row, so the next address is row + bm4 byte: one v_add. Row
//     stride is odd (nc + 2 or nc + 3 entries) so rows start on spread-out banks. Column 0 is
//     "hold" (next = self), column 1 is '\n' (next = start state), column 2 + k = byte class k.
//     States are numbered so that every state from which ANY regex can accept
//     (on some next byte, at end of line or before a final terminator) comes last: "a match may
//     have happened" is just max(row offset) >= thr[g] -- one v_max per byte, no mask traffic.
//   * global (rare path): exact rows of next state ids and, indexed alike, uint64 accept masks
//     (the regexes accepting BEFORE the byte; the '\n' column carries the end-of-line accepts),
//     the per-state [EOL, before-final-terminator] masks and the regex ids.
//
// Work split: one lane walks a RUN of SCAN_RUN consecutive lines as ONE byte stream (the '\n'
// between lines is the restart column), so a wave's time is the max of 64 run lengths, not of 64
// line lengths. No byte of the hot loop is masked: the walk starts at the aligned block holding
// the run's first byte and lets the preceding '\n' restart the automaton (garbage prefix), and it
// ends by walking the last line's separator, whose '\n' column yields that line's end-of-line
// accepts (bytes after it are garbage). Only "\r\n"-separated runs take a variant whose bytemap
// has 512 entries: the separator's '\r' indexes entry 256 + c = hold. Per byte: one LDS read of
// bm4, then per group one v_add + one ds_read_u16 + one v_max: G independent dependency chains
// per lane. A 16-byte block whose states crossed a threshold is walked again exactly (global
// tables, out-of-run bytes skipped, separator '\r' held) from the saved states, attributing
// accept masks to lines; garbage bytes can only cause such a re-walk, never a hit. Runs with a
// line whose content ends in a line terminator ('$' must also be tried before it, Matcher.find),
// an unusual separator or a document boundary take the exact per-line walk.
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "lp_api.h"
#include "lp_core.h"
#include "lp_host.h"

namespace lp {

// Bulk texts: 1024-thread blocks (LDS is per block: more waves per staged byte), runs of 4 lines.
// Small texts (a request): 256-thread blocks and one line per lane, so the few thousand lines
// spread over many CUs and each lane's dependent chain is one line, not four.
constexpr int SCAN_THREADS = 1024;
constexpr int SCAN_THREADS_SMALL = 256;
constexpr int SCAN_RUN = 4;
constexpr int SCAN_BM_COPIES = 32;                         // lane-replicated bytemap (bulk variant)
// 256 entries per copy (the CRLF variant's hold entries 256..511 are all 0: a select instead of a
// read): 32 KiB after the blob, so a pass blob up to 48 KiB leaves room for 2 blocks per CU
constexpr int SCAN_BM_REP_BYTES = 256 * SCAN_BM_COPIES * 4;

// LDS loads from a 32-bit LDS address. The blob sits at LDS address 0 (the kernel's only LDS is
// the dynamic blob; checked at entry), so a row offset + a bytemap byte IS the address: one
// v_add_u32_sdwa (byte select folded in) per group per byte, no base add.
typedef __attribute__((address_space(3))) const uint16_t lds_u16_t;
typedef __attribute__((address_space(3))) const uint32_t lds_u32_t;
__device__ __forceinline__ uint32_t lds_ld16(uint32_t a) { return *(lds_u16_t*)(uintptr_t)a; }
__device__ __forceinline__ uint32_t lds_ld32(uint32_t a) { return *(lds_u32_t*)(uintptr_t)a; }

__device__ __forceinline__ uint32_t nz_bytes(uint32_t t) {   // high bit of every zero byte of t
  const uint32_t y = (t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
  return ~(y | t | 0x7F7F7F7Fu);
}

// exact automaton (global tables): state id of an LDS row index, one step, masks
LP_HD uint32_t scan_state_of(const ScanPass& S, int g, uint32_t row_byte) {
  return (row_byte - (uint32_t)S.row_base[g]) / (2u * (uint32_t)S.stride[g]);
}
LP_HD uint32_t scan_step(const ScanPass& S, int g, uint32_t st, uint32_t col) {
  return S.blob[S.gt_off[g] + st * (uint32_t)S.ncol[g] + col];
}
// 64-bit accept masks (bit r: member r of the group) stored as (lo, hi) word pairs
LP_HD uint64_t scan_mask(const ScanPass& S, int g, uint32_t st, uint32_t col) {
  const uint32_t* p = S.blob + S.gm_off[g] + 2 * (st * (uint32_t)S.ncol[g] + col);
  return (uint64_t)p[0] | ((uint64_t)p[1] << 32);
}
LP_HD uint64_t scan_fin(const ScanPass& S, int g, uint32_t st, int ft) {
  const uint32_t* p = S.blob + S.fin_off[g] + 4 * st + 2 * ft;
  return (uint64_t)p[0] | ((uint64_t)p[1] << 32);
}

template <typename Emit>
LP_HD void scan_emit(const ScanPass& S, int g, uint64_t m, int64_t line, Emit&& emit) {
  while (m) {
    const int r = __builtin_ctzll(m);
    m &= m - 1;
    emit(((int64_t)S.blob[S.rid_off + 64 * g + r] << 32) | line);
  }
}

// exact walk of ONE line on the global tables (Matcher.find: accept before a final line
// terminator, at end of line, or before any byte). Shared by the host twin and the device.
template <typename Emit>
LP_HD void scan_line_exact(const ScanPass& S, const uint32_t* bm, const uint8_t* s, int n, int64_t line, Emit&& emit) {
  const int ft = n - final_term_len(s, n);
  for (int g = 0; g < S.ngroups; ++g) {
    uint32_t st = S.init_state[g];
    uint64_t acc = 0;
    for (int t = 0; t < n; ++t) {
      if (t == ft) acc |= scan_fin(S, g, st, 1);
      const uint32_t col = ((bm[s[t]] >> (8 * g)) & 0xFFu) >> 1;
      acc |= scan_mask(S, g, st, col);
      st = scan_step(S, g, st, col);
    }
    acc |= scan_fin(S, g, st, 0);
    scan_emit(S, g, acc, line, emit);
  }
}

struct GlobalEmit {
  int64_t* out;
  int64_t cap;
  unsigned long long* count;
  __device__ void operator()(int64_t v) const {
    const unsigned long long i = atomicAdd(count, 1ull);
    if ((int64_t)i < cap) out[i] = v;
  }
};

// content of line [st, st + n) ends in a line terminator ('\r', U+0085, U+2028, U+2029): two
// aligned dword loads instead of up to three dependent byte loads
__device__ __forceinline__ bool ends_in_terminator(const uint8_t* text, int64_t st, int n) {
  if (n <= 0) return false;
  const int64_t e = st + n;                       // one past the last content byte
  const int64_t a = (e - 1) & ~(int64_t)3;
  const uint32_t hi = *reinterpret_cast<const uint32_t*>(text + a);
  const uint32_t lo = a >= 4 ? *reinterpret_cast<const uint32_t*>(text + a - 4) : 0u;
  const int sh = (int)(e - a);                    // 1..4 bytes of `hi` belong to the content
  const uint64_t v = ((uint64_t)hi << 32 | lo) >> (8 * sh);
  const uint32_t t3 = (uint32_t)(v >> 8) & 0xFFFFFFu;   // bytes -3, -2, -1 in bits 0..7, 8..15, 16..23
  const uint32_t b1 = t3 >> 16, b2 = (t3 >> 8) & 0xFFu, b3 = t3 & 0xFFu;
  return b1 == 0x0Du || (n >= 2 && b2 == 0xC2u && b1 == 0x85u) ||
         (n >= 3 && b3 == 0xE2u && b2 == 0x80u && (b1 == 0xA8u || b1 == 0xA9u));
}

// bit 8b+7 set where byte b of w is '\r' and the byte after it (nx = the following word) '\n'
__device__ __forceinline__ uint32_t crlf_bits(uint32_t w, uint32_t nx) {
  return nz_bytes(w ^ 0x0D0D0D0Du) & nz_bytes(__builtin_amdgcn_alignbyte(nx, w, 1) ^ 0x0A0A0A0Au);
}

// exact re-walk of one 16-byte block [p0, p0 + 16) of a run (rare path): bytes outside
// [p_lo, p_end) are skipped, a separator '\r' is held, '\n' ends line l
template <typename Emit>
__device__ void scan_block_exact(const ScanPass& S, const uint32_t* bm, const uint32_t (&w)[5], int64_t p0,
                                 int64_t p_lo, int64_t p_end, int64_t x0, int64_t x1,
                                 const int64_t* line_start, int g, uint32_t st, Emit&& emit) {
  int64_t l = x0;
  const int64_t first = p0 > p_lo ? p0 : p_lo;
  while (l + 1 < x1 && line_start[l + 1] <= first) ++l;
  if (p0 <= p_lo) st = S.init_state[g];
  uint64_t lacc = 0;
  for (int j = 0; j < 16; ++j) {
    const int64_t pos = p0 + j;
    if (pos < p_lo || pos >= p_end) continue;
    const uint32_t c = (w[j >> 2] >> (8 * (j & 3))) & 0xFFu;
    const uint32_t nx = (w[(j + 1) >> 2] >> (8 * ((j + 1) & 3))) & 0xFFu;
    const uint32_t col = (c == 0x0Du && nx == 0x0Au) ? 0u : ((bm[c] >> (8 * g)) & 0xFFu) >> 1;
    lacc |= scan_mask(S, g, st, col);
    st = scan_step(S, g, st, col);
    if (col == 1u) {
      scan_emit(S, g, lacc, l, emit);
      lacc = 0;
      ++l;
    }
  }
  scan_emit(S, g, lacc, l < x1 ? l : x1 - 1, emit);
}

// exact re-walk of one 16-byte block through the LDS rows (the same transitions as the hot
// walk) with each transition's accept mask from the global u64 mask table laid out like the rows:
// the 16 mask loads depend only on the LDS chain, so they are all in flight together (the
// exact-table walk above is a chain of 16 dependent global loads). xr = group g's row at p0;
// positions outside [p_lo, p_end) are walked but not attributed, as in the hot walk.
template <bool CRLF, typename Emit>
__device__ __forceinline__ void scan_block_masks(const ScanPass& S, const uint32_t (&w)[5], uint32_t hold, int64_t p0,
                                                 int64_t p_lo, int64_t p_end, int64_t x0, int64_t x1,
                                                 const int64_t* __restrict__ line_start, int g, uint32_t xr,
                                                 Emit&& emit) {
  const uint64_t* __restrict__ am = reinterpret_cast<const uint64_t*>(S.blob + S.am_off);   // am_off even
  // in-range positions of the block; a run holds <= SCAN_RUN lines, so an in-range byte belongs
  // to line l0 + k, k = in-range '\n's before it (0..3): per-line masks accumulate branch-free
  const int lo = p_lo > p0 ? (int)(p_lo - p0) : 0;
  const int hi = p_end - p0 < 16 ? (int)(p_end - p0) : 16;
  const uint32_t inr = hi > lo ? (((1u << hi) - 1u) & ~((1u << lo) - 1u)) : 0u;
  uint64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
  uint32_t k = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    uint32_t c = (w[j >> 2] >> (8 * (j & 3))) & 0xFFu;
    if constexpr (CRLF) c |= ((hold >> j) & 1u) << 8;
    const uint32_t b = (lds_ld32(c * 4) >> (8 * g)) & 0xFFu;
    const uint64_t m = ((inr >> j) & 1u) ? am[(xr + b) >> 1] : 0ull;
    a0 |= k == 0 ? m : 0ull;
    a1 |= k == 1 ? m : 0ull;
    a2 |= k == 2 ? m : 0ull;
    a3 |= k == 3 ? m : 0ull;
    k += (b == 2u && ((inr >> j) & 1u)) ? 1u : 0u;     // column 1 = '\n': the line ends here
    xr = lds_ld16(xr + b);
  }
  int64_t l = x0;
  const int64_t first = p0 > p_lo ? p0 : p_lo;
  while (l + 1 < x1 && line_start[l + 1] <= first) ++l;
  const uint64_t acc[4] = {a0, a1, a2, a3};
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (acc[q]) scan_emit(S, g, acc[q], l + q < x1 ? l + q : x1 - 1, emit);
}

// Deferred rare path (bulk variant): a hot block is not re-walked inline -- the re-walk's 16 mask
// loads in flight and its accumulators cost ~50 of the walk's ~107 VGPRs -- but appended as a
// record (block, run bounds, lines, group, the group's row at the block) to a list that
// k_scan_rare walks afterwards, with the same LDS rows and mask table.
struct RareList {
  int64_t* rec;                   // RARE_WORDS int64 per record
  int64_t cap;
  unsigned long long* cnt;        // device: records appended (reset by k_scan_rare's last block)
  unsigned int* done;             // device: k_scan_rare blocks finished
  int64_t* need;                  // pinned host: the record count of an overflowing launch
};
constexpr int RARE_WORDS = 5;

__device__ __forceinline__ void rare_push(const RareList& R, int64_t p0, int64_t p_lo, int64_t p_end, int64_t x0,
                                          int64_t x1, int g, bool crlf, uint32_t xr) {
  const unsigned long long i = atomicAdd(R.cnt, 1ull);
  if ((int64_t)i >= R.cap) return;             // (k_scan_rare reports the overflow)
  int64_t* q = R.rec + RARE_WORDS * (int64_t)i;
  q[0] = p0;
  q[1] = p_lo;
  q[2] = p_end;
  q[3] = x0 | ((x1 - x0) << 56);
  q[4] = (int64_t)g | ((int64_t)crlf << 2) | ((int64_t)xr << 8);
}

// the hot walk of one run over [a0, p_end) in 16-byte blocks; CRLF: separator '\r' -> hold.
// REP: the bytemap read goes to this lane's copy of the lane-replicated bytemap at LDS byte bm_rep
// (entry c < 256 at bm_rep + c * 128; the CRLF hold entries are 0 without a read); otherwise to the
// blob's bm4 at LDS byte 0. DEFER: hot blocks go to
// the rare list instead of the inline re-walk.
template <int G, bool CRLF, bool REP, bool DEFER, typename Emit>
__device__ __forceinline__ void scan_run_fast(const uint32_t* sm, const ScanPass& S, const uint8_t* text, int64_t p_lo,
                                              int64_t p_end, int64_t x0, int64_t x1,
                                              const int64_t* __restrict__ line_start, uint32_t bm_rep, Emit&& emit,
                                              const RareList& rare) {
  uint32_t xr[G];
#pragma unroll
  for (int g = 0; g < G; ++g) xr[g] = (uint32_t)S.init_row[g];
  const int64_t a0 = p_lo & ~(int64_t)15;
  const uint4* blk = reinterpret_cast<const uint4*>(text + a0);
  // the text two blocks ahead: a block's 16 dependent LDS steps (~2k cycles) did not cover an HBM
  // round trip under load, so one block of look-ahead left the walk waiting on its next load
  // (texts are padded by TEXT_PAD >= 48 bytes past the last line: the look-ahead stays in bounds)
  uint4 cur = blk[0], nxt = blk[1];
  for (int64_t p0 = a0; p0 < p_end; p0 += 16) {
    const uint4 nx2 = blk[2];
    ++blk;
    const uint32_t w[5] = {cur.x, cur.y, cur.z, cur.w, nxt.x};
    uint32_t hold = 0;                    // CRLF: byte j of the block is a separator '\r'
    if constexpr (CRLF) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t b = crlf_bits(w[q], w[q + 1]);
        hold |= (((b >> 7) & 1u) | ((b >> 14) & 2u) | ((b >> 21) & 4u) | ((b >> 28) & 8u)) << (4 * q);
      }
    }
    uint32_t xs[G], mx[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      xs[g] = xr[g];
      mx[g] = 0;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      uint32_t c = (w[j >> 2] >> (8 * (j & 3))) & 0xFFu;
      if constexpr (CRLF) c |= ((hold >> j) & 1u) << 8;        // entry 256 + c: hold
      uint32_t b;
      if constexpr (REP) {
        b = lds_ld32(bm_rep + ((c & 0xFFu) << 7));
        if constexpr (CRLF) b = (c >> 8) ? 0u : b;               // entry 256 + c: hold (column 0)
      } else {
        b = lds_ld32(c * 4);
      }
#pragma unroll
      for (int g = 0; g < G; ++g) {
        mx[g] = max(mx[g], xr[g]);
        xr[g] = lds_ld16(xr[g] + ((b >> (8 * g)) & 0xFFu));
      }
    }
    // rare: a state that can accept was visited -- exact re-walk of this block, only for the
    // groups that visited one (a group below its threshold cannot accept anywhere in the block;
    // each re-walk is a chain of 16 dependent global loads, ~8 us, on a request's critical path)
    uint32_t hotm = 0;
#pragma unroll
    for (int g = 0; g < G; ++g) hotm |= (mx[g] >= (uint32_t)S.thr[g] ? 1u : 0u) << g;
    while (hotm) {      // one inlined re-walk, runtime group (an unrolled copy per group cost VGPRs)
      const int g = __builtin_ctz(hotm);
      hotm &= hotm - 1;
      uint32_t xg = xs[0];
#pragma unroll
      for (int q = 1; q < G; ++q)
        if (g == q) xg = xs[q];
      if constexpr (DEFER) rare_push(rare, p0, p_lo, p_end, x0, x1, g, CRLF, xg);
      else scan_block_masks<CRLF>(S, w, hold, p0, p_lo, p_end, x0, x1, line_start, g, xg, emit);
    }
    cur = nxt;
    nxt = nx2;
  }
}

template <int G, int THREADS, bool DEFER>
__global__ __launch_bounds__(THREADS) void k_scan_multi(const uint8_t* __restrict__ text, int64_t nbytes,
                                                        const int64_t* __restrict__ line_start,
                                                        const int32_t* __restrict__ line_len, int64_t nlines,
                                                        ScanPass S, int64_t* __restrict__ out, int64_t cap,
                                                        unsigned long long* __restrict__ count, int run_len,
                                                        RareList rare) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
  lds_fill<uint4>(reinterpret_cast<uint4*>(sm), reinterpret_cast<const uint4*>(S.blob), S.lds_words >> 2);  // multiple of 4
  // bulk variant: a lane-replicated copy of bm4 after the blob (SCAN_BM_COPIES copies: entry c of
  // copy j at word c * 32 + j, lane l reads copy l & 31). A ds_read_b32 is serviced in two 32-lane
  // groups with bank = word mod 32, so the byte-map read of every byte is conflict-free whatever
  // the bytes (profiles/r3_t: 1.5 bank-conflict cycles per LDS instruction over the whole walk)
  constexpr bool REP = THREADS == SCAN_THREADS;
  uint32_t bm_rep = 0;
  if constexpr (REP) {
    uint32_t* rep = sm + S.lds_words;
    for (int i = threadIdx.x; i < 256 * SCAN_BM_COPIES; i += THREADS) rep[i] = S.blob[i / SCAN_BM_COPIES];
    bm_rep = (uint32_t)S.lds_words * 4 + (threadIdx.x & (SCAN_BM_COPIES - 1)) * 4;
  }
  __syncthreads();
  const GlobalEmit emit{out, cap, count};
  // the fast walk addresses LDS absolutely (blob at address 0); otherwise every run walks exactly
  const bool at_zero = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)sm == 0u;
  const int64_t nruns = (nlines + run_len - 1) / run_len;
  const int64_t stride = (int64_t)gridDim.x * THREADS;
  // a run's stream-walk preconditions: "\n" / "\r\n" separators (after every line of the run, the
  // last one included), the run starts right after a '\n', no content ends in a terminator
  struct Run {
    int64_t x0, x1, p_lo, p_end;
    bool fast, crlf;
  };
  auto prep = [&](int64_t run) {
    Run R;
    R.x0 = run * run_len;
    R.x1 = R.x0 + run_len < nlines ? R.x0 + run_len : nlines;
    R.fast = at_zero;
    R.crlf = false;
    if (run_len == SCAN_RUN && R.x0 + SCAN_RUN < nlines) {
      // a full run that is not the text's end (all but the last run): the 5 starts and 4 lengths,
      // then the 8 terminator words and the byte before the run, each batch loaded in one round
      // trip (the loop below waits for every line's loads in turn)
      int64_t s5[SCAN_RUN + 1];
      int n4[SCAN_RUN];
#pragma unroll
      for (int i = 0; i <= SCAN_RUN; ++i) s5[i] = line_start[R.x0 + i];
#pragma unroll
      for (int i = 0; i < SCAN_RUN; ++i) n4[i] = line_len[R.x0 + i];
      bool term = false;
      int64_t sep = 1;
#pragma unroll
      for (int i = 0; i < SCAN_RUN; ++i) {
        term |= ends_in_terminator(text, s5[i], n4[i]);
        sep = s5[i + 1] - s5[i] - n4[i];
        if (sep == 2) R.crlf = true;
        else if (sep != 1) R.fast = false;
      }
      if (term) R.fast = false;
      R.p_lo = s5[0];
      R.p_end = s5[SCAN_RUN - 1] + n4[SCAN_RUN - 1] + sep;
      if (R.p_lo > 0 && text[R.p_lo - 1] != '\n') R.fast = false;
      return R;
    }
    int64_t st_next = line_start[R.x0];
    R.p_lo = st_next;
    R.p_end = 0;
    for (int64_t x = R.x0; x < R.x1; ++x) {
      const int64_t st = st_next;
      const int n = line_len[x];
      if (ends_in_terminator(text, st, n)) R.fast = false;
      int64_t sep;
      if (x + 1 < nlines) {
        st_next = line_start[x + 1];
        sep = st_next - st - n;
      } else {                                   // the text's last line: is there a newline after it?
        const int64_t e = st + n;
        sep = (e < nbytes && text[e] == '\n') ? 1 : (e + 1 < nbytes && text[e] == '\r' && text[e + 1] == '\n') ? 2 : 0;
      }
      if (sep == 2) R.crlf = true;
      else if (sep != 1) R.fast = false;
      R.p_end = st + n + sep;                    // after the last line's separator
    }
    if (R.p_lo > 0 && text[R.p_lo - 1] != '\n') R.fast = false;   // e.g. a document boundary in a batch
    return R;
  };
  auto walk_one = [&](const Run& R) {
    if (!R.fast) {     // rare: exact per-line walks
      for (int64_t x = R.x0; x < R.x1; ++x) scan_line_exact(S, sm, text + line_start[x], line_len[x], x, emit);
    } else if (R.crlf) {
      scan_run_fast<G, true, REP, DEFER>(sm, S, text, R.p_lo, R.p_end, R.x0, R.x1, line_start, bm_rep, emit, rare);
    } else {
      scan_run_fast<G, false, REP, DEFER>(sm, S, text, R.p_lo, R.p_end, R.x0, R.x1, line_start, bm_rep, emit, rare);
    }
  };
  for (int64_t run = (int64_t)blockIdx.x * THREADS + threadIdx.x; run < nruns; run += stride) walk_one(prep(run));
}

// the deferred re-walks: every record is one hot 16-byte block of one group, walked exactly on the
// pass's LDS rows (staged at LDS address 0 as in k_scan_multi) with the global mask table; a fixed
// grid strides over the device count; the last block resets the list and reports an overflow
// (the scan's hit count is pushed past its capacity, so the batch re-runs -- see scan_multi_dev)
__global__ __launch_bounds__(256) void k_scan_rare(const uint8_t* __restrict__ text,
                                                   const int64_t* __restrict__ line_start, ScanPass S,
                                                   int64_t* __restrict__ out, int64_t cap,
                                                   unsigned long long* __restrict__ count, RareList rare) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sm[];   // the only LDS: the blob at address 0
  lds_fill<uint4>(reinterpret_cast<uint4*>(sm), reinterpret_cast<const uint4*>(S.blob), S.lds_words >> 2);
  __syncthreads();
  const GlobalEmit emit{out, cap, count};
  const bool at_zero = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)sm == 0u;
  const int64_t n = (int64_t)*rare.cnt;
  const int64_t m = n < rare.cap ? n : rare.cap;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t* q = rare.rec + RARE_WORDS * i;
    const int64_t p0 = q[0], p_lo = q[1], p_end = q[2], xw = q[3], gw = q[4];
    const int64_t x0 = xw & ((1ll << 56) - 1), x1 = x0 + (xw >> 56);
    const int g = (int)(gw & 3);
    const bool crlf = (gw >> 2) & 1;
    const uint32_t xr = (uint32_t)(gw >> 8);
    const uint4 cur = *reinterpret_cast<const uint4*>(text + p0);
    const uint32_t w[5] = {cur.x, cur.y, cur.z, cur.w, *reinterpret_cast<const uint32_t*>(text + p0 + 16)};
    if (!at_zero) {                              // (never expected) the exact global-table walk
      scan_block_exact(S, S.blob + S.bm_off, w, p0, p_lo, p_end, x0, x1, line_start, g, scan_state_of(S, g, xr), emit);
    } else if (crlf) {
      uint32_t hold = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t b = crlf_bits(w[k], w[k + 1]);
        hold |= (((b >> 7) & 1u) | ((b >> 14) & 2u) | ((b >> 21) & 4u) | ((b >> 28) & 8u)) << (4 * k);
      }
      scan_block_masks<true>(S, w, hold, p0, p_lo, p_end, x0, x1, line_start, g, xr, emit);
    } else {
      scan_block_masks<false>(S, w, 0u, p0, p_lo, p_end, x0, x1, line_start, g, xr, emit);
    }
  }
  __syncthreads();
  volatile uint32_t* last = sm + S.lds_words;    // (words behind the blob: no static LDS)
  volatile unsigned long long* pad = reinterpret_cast<volatile unsigned long long*>(sm + S.lds_words + 2);
  if (threadIdx.x == 0) {
    __threadfence();
    *last = atomicAdd(rare.done, 1u) == gridDim.x - 1 ? 1u : 0u;
    *pad = ~0ull;
  }
  __syncthreads();
  if (!*last) return;
  if (threadIdx.x == 0) {
    if (n > rare.cap) {
      rare.need[0] = n;                          // grown before the re-run
      __threadfence_system();
      *pad = atomicAdd(count, (unsigned long long)(cap + 1));
    }
    *rare.cnt = 0;
    *rare.done = 0;
  }
  __syncthreads();
  // the overflow signal pushes the count past the capacity: the hit pipeline then reads the whole
  // buffer, so its unwritten tail becomes dropped keys (-1), never uninitialised memory
  const unsigned long long p0 = *pad;
  for (int64_t i = (int64_t)p0 + threadIdx.x; p0 != ~0ull && i < cap; i += blockDim.x) out[i] = -1;
}

namespace {
bool g_defer_rare = true;
}  // namespace
bool scan_defer_rare() { return g_defer_rare; }
void set_scan_defer_rare(bool on) { g_defer_rare = on; }

namespace {

// one grow-only rare list per (device, stream); `need` (pinned) carries an overflow's size back
struct RareBuf {
  int64_t* rec = nullptr;
  int64_t cap = 0;
  unsigned long long* cnt = nullptr;
  int64_t* need = nullptr;
};
std::mutex g_rare_mu;
std::map<std::pair<int, uint64_t>, RareBuf> g_rare;

RareList rare_list(int64_t want, uint64_t stream) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_rare_mu);
  RareBuf& b = g_rare[{dev, stream}];
  if (b.need && *b.need > want) want = *b.need;
  if (!b.cnt) {
    if (hipMalloc(reinterpret_cast<void**>(&b.cnt), 16) != hipSuccess ||
        hipMemset(b.cnt, 0, 16) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&b.need), 8, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
      throw std::runtime_error("scan_multi: rare list allocation failed");
    *b.need = 0;
  }
  if (want > b.cap) {              // the stream is idle here: the previous launch's batch has ended
    if (b.rec) (void)hipFree(b.rec);
    b.rec = nullptr;
    const int64_t cap = want + want / 4;
    if (hipMalloc(reinterpret_cast<void**>(&b.rec), (size_t)cap * RARE_WORDS * 8) != hipSuccess)
      throw std::runtime_error("scan_multi: rare list allocation failed");
    b.cap = cap;
    *b.need = 0;
  }
  int64_t* need_dev = nullptr;
  (void)hipHostGetDevicePointer(reinterpret_cast<void**>(&need_dev), b.need, 0);
  return RareList{b.rec, b.cap, b.cnt, reinterpret_cast<unsigned int*>(b.cnt + 1), need_dev};
}

}  // namespace

void scan_multi_dev(const uint8_t* text, int64_t nbytes, const int64_t* line_start, const int32_t* line_len, int64_t nlines,
                    const ScanPass& S, int64_t* out, int64_t cap, unsigned long long* count, int grid,
                    uint64_t stream) {
  if (nlines <= 0 || S.ngroups <= 0) return;
  if (S.ngroups > 4 || (S.lds_words & 3) || S.lds_words * 4 + SCAN_BM_REP_BYTES > (160 << 10))
    throw std::runtime_error("scan_multi: bad pass descriptor");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // small texts: one line per lane in 256-thread blocks (the grid is sized for 1024-thread blocks)
  const bool small = nlines <= (int64_t)grid * SCAN_THREADS_SMALL;
  const size_t lds = (size_t)S.lds_words * 4 + (small ? 0 : SCAN_BM_REP_BYTES);
  // bulk texts of fewer than ~4 lines per lane of the grid (a 1M-line document on 512 blocks of
  // 1024 lanes) walk shorter runs, so every lane of the grid has a run and each lane's dependent
  // chain is shorter; a 12.5M-line shard keeps 4-line runs
  const int64_t lanes = (int64_t)grid * SCAN_THREADS;
  const int run_len = small ? 1 : nlines < 2 * lanes ? 1 : nlines < 4 * lanes ? 2 : SCAN_RUN;
  const int threads = small ? SCAN_THREADS_SMALL : SCAN_THREADS;
  const int64_t runs = (nlines + run_len - 1) / run_len;
  const int64_t need = (runs + threads - 1) / threads;
  const int g = (int)std::max<int64_t>(1, std::min<int64_t>(small ? 4 * (int64_t)grid : grid, need));
  // bulk texts defer the rare re-walks to k_scan_rare (engine.scan-defer-rare, default on)
  const bool defer = !small && scan_defer_rare();
  const RareList rare = defer ? rare_list(std::max<int64_t>(65536, runs), stream) : RareList{};
#define LP_SCAN(GV)                                                                                        \
  if (small)                                                                                               \
    hipLaunchKernelGGL((k_scan_multi<GV, SCAN_THREADS_SMALL, false>), dim3(g), dim3(SCAN_THREADS_SMALL), lds, st, \
                       text, nbytes, line_start, line_len, nlines, S, out, cap, count, run_len, rare);     \
  else if (defer)                                                                                          \
    hipLaunchKernelGGL((k_scan_multi<GV, SCAN_THREADS, true>), dim3(g), dim3(SCAN_THREADS), lds, st, text, \
                       nbytes, line_start, line_len, nlines, S, out, cap, count, run_len, rare);           \
  else                                                                                                     \
    hipLaunchKernelGGL((k_scan_multi<GV, SCAN_THREADS, false>), dim3(g), dim3(SCAN_THREADS), lds, st, text, \
                       nbytes, line_start, line_len, nlines, S, out, cap, count, run_len, rare)
  switch (S.ngroups) {
    case 1: LP_SCAN(1); break;
    case 2: LP_SCAN(2); break;
    case 3: LP_SCAN(3); break;
    default: LP_SCAN(4); break;
  }
#undef LP_SCAN
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e) + " in scan_multi");
  if (defer) {
    hipLaunchKernelGGL(k_scan_rare, dim3(256), dim3(256), (size_t)S.lds_words * 4 + 32, st, text, line_start, S, out,
                       cap, count, rare);
    e = hipGetLastError();
    if (e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e) + " in scan_rare");
  }
}

// host twin: the exact per-line walk over the same blob
int64_t scan_multi_host(const uint8_t* text, const int64_t* line_start, const int32_t* line_len, int64_t nlines,
                        const ScanPass& S, int64_t* out, int64_t cap) {
  const uint32_t* bm = S.blob + S.bm_off;
  std::vector<std::vector<int64_t>> part(std::max(1, host_threads()));
  host_parallel(nlines, 2048, [&](int th, int64_t a, int64_t b) {
    auto emit = [&](int64_t v) { part[th].push_back(v); };
    for (int64_t x = a; x < b; ++x) scan_line_exact(S, bm, text + line_start[x], line_len[x], x, emit);
  });
  int64_t c = 0;
  for (auto& v : part)
    for (int64_t k : v) {
      if (c < cap) out[c] = k;
      ++c;
    }
  return c;
}

}  // namespace lp
