// K1 line index (reference: Java logs.split("\\r?\\n"), AnalysisService.java:53): line starts and
// lengths straight from the bytes, ONE read of the text (+ its 1/8-size newline bitmask) and ONE
// host read.
//
//   k_nl_count   per 16 KiB tile: number of '\n' + a 1-bit-per-byte '\n' mask + a '\r' flag
//   k_tile_scan  exclusive scan of the tile counts (~80k counts, one workgroup)
//   k_nl_lines   4 tiles per workgroup, from the mask (text only in '\r'-flagged tiles): every '\n' at p with global index g writes starts[g+1] = p + 1
//                and, when the previous '\n' is in the same tile, lens[g] = (p minus a '\r' right
//                before it) - start; staged in LDS, stored coalesced. The tile's FIRST line end is
//                recorded (fix_g, fix_end) for
//   k_line_fix   which completes it once every start is written, plus the total (info[0]), the
//                final line (to nbytes) and info[1] = last '\n' position (or -1);
//   k_line_trim  Java's trailing-empty trimming -> info[2] = lines kept.
// k_nl_lines also writes the coarse 4 KiB block -> line index the literal verify uses (one wave
// per block: the line of its first byte is the number of '\n' before it).
// Bulk DP steps fold pass 1 into the literal prefilter's read of the text (lp_kernels.hip
// k_prefilter<..., NLF>): the same counts, masks and flags, one pass over the text fewer.
// A single-pass decoupled look-back variant (tile ticket + 256 predecessor states per round
// trip) was measured at ~1.08 ms per 1.33 GB vs ~0.55 ms for these two passes: the INCLUSIVE
// frontier, not HBM, sets its pace (docs/PERFORMANCE.md).
#include <hip/hip_runtime.h>

#include <cstring>
#include <stdexcept>
#include <string>

#include "lp_api.h"

namespace lp {

constexpr int LI_BYTES_PER_THREAD = 64;
__device__ __forceinline__ uint32_t li_zero_bytes(uint32_t t) {
  const uint32_t y = (t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;   // high bit of every 0x00 byte of t
  return ~(y | t | 0x7F7F7F7Fu);
}

constexpr int LI_THREADS = 256;
constexpr int LI_TILE = LI_THREADS * LI_BYTES_PER_THREAD;
constexpr int LI_STAGE = LI_THREADS * 8;       // staged lines per tile (~150 per 16 KiB of log text)

// '\n' / '\r' byte masks of this lane's 64 bytes (bytes past nbytes are not text)
__device__ __forceinline__ int li_masks(const uint8_t* __restrict__ text, int64_t nbytes, int64_t base,
                                        uint32_t (&m)[16], uint32_t (&cr)[16]) {
  int c = 0;
  if (base < nbytes) {
    const uint4* p = reinterpret_cast<const uint4*>(text + base);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint4 v = p[k];
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        m[4 * k + q] = li_zero_bytes(w[q] ^ 0x0A0A0A0Au);
        cr[4 * k + q] = li_zero_bytes(w[q] ^ 0x0D0D0D0Du);
      }
    }
    if (base + LI_BYTES_PER_THREAD > nbytes) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int64_t valid = nbytes - (base + 4 * k);
        const uint32_t keep = valid >= 4 ? 0xFFFFFFFFu : valid <= 0 ? 0u : ((1u << (8 * valid)) - 1u);
        m[k] &= keep;
      }
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) c += __popc(m[k]);
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k) m[k] = cr[k] = 0;
  }
  return c;
}

// bits 7, 15, 23, 31 of x -> bits 0..3
__device__ __forceinline__ uint32_t li_pack4(uint32_t x) {
  const uint32_t y = x >> 7;                      // bits 0, 8, 16, 24
  const uint32_t z = (y | (y >> 7)) & 0x00030003u; // bits 0, 1, 16, 17
  return (z | (z >> 14)) & 0xFu;
}

// Pass 1: per 16 KiB tile the '\n' count, and per lane (64 bytes) a 64-bit '\n' bitmask -- the
// second pass reads these 2 KiB per tile instead of the tile's 16 KiB of text. A tile holding a
// "\r\n" (a '\r' right before one of its '\n', possibly the previous tile's last byte) is flagged:
// only those tiles (CRLF logs) are read again as text to strip the '\r'. The flag is conservative
// (any '\r' in the tile or right before it): k_nl_lines derives the exact '\r\n' positions.
//
// Loads are coalesced: a wave's k-th 16-byte load covers 1 KiB of its 4 KiB contiguously (lane l
// at k*1024 + 16*l), and the 16-bit masks are transposed through LDS into the per-lane 64-byte
// layout k_nl_lines reads (a lane-strided 64-byte layout touched 64 cache lines per load
// instruction and re-fetched them from L2 four times).
__global__ __launch_bounds__(LI_THREADS) void k_nl_count(const uint8_t* __restrict__ text, int64_t nbytes,
                                                         int32_t* __restrict__ cnt, uint64_t* __restrict__ nlm,
                                                         int32_t* __restrict__ crf) {
  __shared__ __attribute__((aligned(16))) uint16_t s_m[LI_THREADS * 4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t wbase = (int64_t)blockIdx.x * LI_TILE + (int64_t)wid * (64 * LI_BYTES_PER_THREAD);
  int crnl = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t p = wbase + k * 1024 + 16 * lane;
    uint32_t m16 = 0;
    if (p < nbytes) {
      const uint4 v = *reinterpret_cast<const uint4*>(text + p);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        m16 |= li_pack4(li_zero_bytes(w[q] ^ 0x0A0A0A0Au)) << (4 * q);
        crnl |= (int)li_zero_bytes(w[q] ^ 0x0D0D0D0Du);
      }
      const int64_t valid = nbytes - p;
      if (valid < 16) m16 &= (1u << valid) - 1u;
    }
    s_m[wid * 256 + k * 64 + lane] = (uint16_t)m16;
  }
  if (threadIdx.x == 0 && blockIdx.x > 0 && text[(int64_t)blockIdx.x * LI_TILE - 1] == '\r') crnl = 1;
  __syncthreads();
  // lane l's 64 bytes are the 16-byte pieces 4l .. 4l+3 of its wave, stored in that order
  const uint64_t m64 = *reinterpret_cast<const uint64_t*>(&s_m[wid * 256 + 4 * lane]);
  nlm[(int64_t)blockIdx.x * LI_THREADS + threadIdx.x] = m64;
  int c = __popcll(m64);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  const bool anycr = __ballot(crnl != 0) != 0;
  __shared__ int ws[LI_THREADS / 64];
  __shared__ int wcr[LI_THREADS / 64];
  if ((threadIdx.x & 63) == 0) {
    ws[threadIdx.x >> 6] = c;
    wcr[threadIdx.x >> 6] = anycr ? 1 : 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0, f = 0;
    for (int w = 0; w < LI_THREADS / 64; ++w) {
      t += ws[w];
      f |= wcr[w];
    }
    cnt[blockIdx.x] = t;
    crf[blockIdx.x] = f;
  }
}

// One tile of pass 2. m64 / excl / cf were loaded up front (see k_nl_lines); the caller
// separates consecutive tiles of a block with a barrier (the LDS stage is reused).
__device__ __forceinline__ void li_lines_tile(const uint8_t* __restrict__ text, int64_t nbytes, int64_t tile,
                                              uint64_t m64, int64_t excl, int cf, int* s_wcnt,
                                              int32_t* s_start, int32_t* s_end, int64_t* __restrict__ starts,
                                              int32_t* __restrict__ lens, int64_t cap,
                                              int64_t* __restrict__ fix_g, int64_t* __restrict__ fix_end,
                                              int32_t* __restrict__ blk, int64_t nblk) {
  constexpr int NW = LI_THREADS / 64;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t tbase = tile * LI_TILE;
  const int64_t base = tbase + (int64_t)threadIdx.x * LI_BYTES_PER_THREAD;
  // '\r' before a '\n' (bit b: byte b - 1 is '\r') only in flagged tiles, which are read as text again
  uint64_t crb = 0;
  if (cf && base < nbytes) {
    uint32_t m[16], cr[16];
    li_masks(text, nbytes, base, m, cr);
    uint64_t c64 = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) c64 |= (uint64_t)li_pack4(cr[k]) << (4 * k);
    crb = (c64 << 1) | ((base > 0 && text[base - 1] == '\r') ? 1ull : 0ull);
  }
  const int c = __popcll(m64);
  int incl = c;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int t = __shfl_up(incl, d, 64);
    if (lane >= d) incl += t;
  }
  if (lane == 63) s_wcnt[wid] = incl;
  __syncthreads();
  int woff = 0, tot = 0;
  for (int w = 0; w < NW; ++w) {
    if (w < wid) woff += s_wcnt[w];
    tot += s_wcnt[w];
  }
  // coarse index for line lookups (lp_core.h locate_line): a wave covers one 4 KiB block, and the
  // line holding its first byte is the number of '\n' before it
  if (blk && lane == 0 && tile * NW + wid < nblk) blk[tile * NW + wid] = (int32_t)(excl + woff);
  const bool staged = tot <= LI_STAGE;            // block-uniform
  // pass A: every '\n' -> (start of the next line, end of its own line)
  int o = woff + (incl - c);                      // tile-local index of this lane's first '\n'
  for (uint64_t mm = m64; mm; mm &= mm - 1) {
    const int b = __ffsll((unsigned long long)mm) - 1;
    const int64_t pos = base + b;
    if (staged) {
      s_start[o] = (int32_t)(pos + 1 - tbase);
      s_end[o] = (int32_t)(pos - (int64_t)((crb >> b) & 1ull) - tbase);
    } else if (excl + o + 1 < cap) {
      starts[excl + o + 1] = pos + 1;
    }
    ++o;
  }
  __syncthreads();
  if (staged) {
    for (int i = threadIdx.x; i < tot; i += LI_THREADS) {
      const int64_t g = excl + i;
      if (g + 1 < cap) starts[g + 1] = tbase + s_start[i];
      if (i == 0) {
        fix_g[tile] = g;
        fix_end[tile] = tbase + s_end[0];
      } else if (g < cap) {
        lens[g] = s_end[i] - s_start[i - 1];
      }
    }
  } else {
    // pass B (a tile with more lines than the stage): lengths from the starts just stored
    o = woff + (incl - c);
    for (uint64_t mm = m64; mm; mm &= mm - 1) {
      const int b = __ffsll((unsigned long long)mm) - 1;
      const int64_t end = base + b - (int64_t)((crb >> b) & 1ull);
      const int64_t g = excl + o;
      if (o == 0) {
        fix_g[tile] = g;
        fix_end[tile] = end;
      } else if (g < cap) {
        lens[g] = (int32_t)(end - starts[g]);
      }
      ++o;
    }
  }
  if (tot == 0 && threadIdx.x == 0) fix_g[tile] = -1;
  if (tile == 0 && threadIdx.x == 0 && cap > 0) starts[0] = 0;
}

// Pass 2 over LI_LINES_TPB consecutive tiles per workgroup: every tile's mask word, offset and
// CRLF flag are loaded before the first tile is walked, so a workgroup keeps LI_LINES_TPB loads in
// flight instead of one (one tile per workgroup was latency-bound: ~3 us per 2 KiB of masks).
constexpr int LI_LINES_TPB = 4;
__global__ __launch_bounds__(LI_THREADS) void k_nl_lines(const uint8_t* __restrict__ text, int64_t nbytes,
                                                         int64_t ntiles, const uint64_t* __restrict__ nlm,
                                                         const int32_t* __restrict__ crf,
                                                         const int64_t* __restrict__ off,
                                                         int64_t* __restrict__ starts, int32_t* __restrict__ lens,
                                                         int64_t cap, int64_t* __restrict__ fix_g,
                                                         int64_t* __restrict__ fix_end, int32_t* __restrict__ blk,
                                                         int64_t nblk) {
  __shared__ int s_wcnt[LI_THREADS / 64];
  __shared__ int32_t s_start[LI_STAGE];          // tile-relative: start of the next line (= '\n' + 1)
  __shared__ int32_t s_end[LI_STAGE];            // tile-relative end of the line ('\n' minus a '\r')
  const int64_t t0 = (int64_t)blockIdx.x * LI_LINES_TPB;
  uint64_t m[LI_LINES_TPB];
  int64_t ex[LI_LINES_TPB];
  int cf[LI_LINES_TPB];
#pragma unroll
  for (int j = 0; j < LI_LINES_TPB; ++j) {
    const bool in = t0 + j < ntiles;
    m[j] = in ? nlm[(t0 + j) * LI_THREADS + threadIdx.x] : 0ull;
    ex[j] = in ? off[t0 + j] : 0;
    cf[j] = in ? crf[t0 + j] : 0;
  }
#pragma unroll
  for (int j = 0; j < LI_LINES_TPB; ++j) {
    if (t0 + j >= ntiles) break;                  // block-uniform
    if (j) __syncthreads();                       // the previous tile's stage has been stored
    li_lines_tile(text, nbytes, t0 + j, m[j], ex[j], cf[j], s_wcnt, s_start, s_end, starts, lens, cap, fix_g,
                  fix_end, blk, nblk);
  }
}

// Completes what needs every tile's starts: the first line end of each tile, the final line and
// info[1]. Thread t < ntiles: tile t; thread ntiles: the final line.
__global__ __launch_bounds__(256) void k_line_fix(int64_t ntiles, int64_t nbytes, const int64_t* __restrict__ fix_g,
                                                  const int64_t* __restrict__ fix_end,
                                                  const int64_t* __restrict__ off, const int32_t* __restrict__ cnt,
                                                  const int64_t* __restrict__ starts, int32_t* __restrict__ lens,
                                                  int64_t cap, int64_t* __restrict__ info, int32_t* __restrict__ blk,
                                                  int64_t nblk) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < ntiles) {
    const int64_t g = fix_g[t];
    if (g >= 0 && g < cap) lens[g] = (int32_t)(fix_end[t] - (g == 0 ? 0 : starts[g]));
  } else if (t == ntiles) {
    const int64_t total = off[ntiles - 1] + cnt[ntiles - 1];
    info[0] = total;
    if (blk)                                      // coarse-index entries past the last tile
      for (int64_t b = ntiles * (LI_THREADS / 64); b < nblk; ++b) blk[b] = (int32_t)total;
    const int64_t st = total == 0 ? 0 : (total < cap ? starts[total] : -1);
    info[1] = total == 0 ? -1 : (total < cap ? st - 1 : -1);
    if (total < cap) lens[total] = (int32_t)(nbytes - st);
  }
}

// Java String.split drops trailing empty strings -- except that input without any '\n' is one
// line even when empty. One workgroup walks back from the end 256 lines at a time (trailing empty
// lines are rare: one iteration in practice). info[2] = lines kept.
__global__ __launch_bounds__(256) void k_line_trim(const int32_t* __restrict__ lens, int64_t cap,
                                                   int64_t* __restrict__ info) {
  __shared__ int64_t wmax[4];
  const int64_t nl = info[0];
  if (nl == 0) {
    if (threadIdx.x == 0) info[2] = 1;
    return;
  }
  const int64_t n = nl + 1 < cap ? nl + 1 : cap;
  for (int64_t hi = n; hi > 0; hi -= 256) {
    const int64_t i = hi - 1 - threadIdx.x;
    int64_t best = (i >= 0 && lens[i] > 0) ? i : -1;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const long long o = __shfl_xor((long long)best, off, 64);
      best = best > o ? best : o;
    }
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = best;
    __syncthreads();
    const int64_t b = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
    if (b >= 0) {
      if (threadIdx.x == 0) info[2] = b + 1;
      return;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) info[2] = 0;
}

// exclusive prefix of the per-tile '\n' counts (~80k tiles for a 1.3 GB shard) in ONE workgroup,
// in coalesced chunks of 16,384 counts: each thread loads 16 consecutive counts (the next chunk's are
// loaded before this chunk is scanned), scans them, the 1,024 thread sums are scanned through the
// waves' shuffles + LDS, and each thread writes its 16 offsets as 8 16-byte stores. ~10 us against
// rocPRIM's look-back scan (an init kernel + the scan, 81 us per step, profiles/r4_c).
constexpr int LS_THREADS = 1024;
constexpr int LS_PER = 16;
__global__ __launch_bounds__(LS_THREADS) void k_tile_scan(const int32_t* __restrict__ cnt, int64_t nt,
                                                          int64_t* __restrict__ off) {
  __shared__ int64_t wsum[2][LS_THREADS / 64];
  constexpr int64_t CH = (int64_t)LS_THREADS * LS_PER;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int2* c2 = reinterpret_cast<const int2*>(cnt);        // cnt is 8-byte aligned (int64 workspace)
  auto load = [&](int64_t base, int32_t (&v)[LS_PER]) {
    const int64_t i0 = base + (int64_t)threadIdx.x * LS_PER;
    if (i0 + LS_PER <= nt) {
#pragma unroll
      for (int k = 0; k < LS_PER / 2; ++k) {
        const int2 x = c2[(i0 >> 1) + k];
        v[2 * k] = x.x;
        v[2 * k + 1] = x.y;
      }
    } else {
#pragma unroll
      for (int k = 0; k < LS_PER; ++k) v[k] = i0 + k < nt ? cnt[i0 + k] : 0;
    }
  };
  int32_t cur[LS_PER], nxt[LS_PER];
  load(0, cur);
  int64_t carry = 0;
  for (int64_t base = 0, it = 0; base < nt; base += CH, ++it) {
    if (base + CH < nt) load(base + CH, nxt);
    int64_t s = 0;
#pragma unroll
    for (int k = 0; k < LS_PER; ++k) s += cur[k];
    int64_t inc = s;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int64_t o = __shfl_up(inc, d, 64);
      if (lane >= d) inc += o;
    }
    int64_t* ws = wsum[it & 1];                               // alternate: no second barrier per chunk
    if (lane == 63) ws[wv] = inc;
    __syncthreads();
    int64_t wbase = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < LS_THREADS / 64; ++w) {
      const int64_t x = ws[w];
      wbase += w < wv ? x : 0;
      tot += x;
    }
    int64_t run = carry + wbase + inc - s;
    const int64_t i0 = base + (int64_t)threadIdx.x * LS_PER;
    int64_t o[LS_PER];
#pragma unroll
    for (int k = 0; k < LS_PER; ++k) {
      o[k] = run;
      run += cur[k];
    }
    if (i0 + LS_PER <= nt && ((uintptr_t)off & 15) == 0) {
      longlong2* o2 = reinterpret_cast<longlong2*>(off + i0);
#pragma unroll
      for (int k = 0; k < LS_PER / 2; ++k) o2[k] = make_longlong2(o[2 * k], o[2 * k + 1]);
    } else {
#pragma unroll
      for (int k = 0; k < LS_PER; ++k)
        if (i0 + k < nt) off[i0 + k] = o[k];
    }
    carry += tot;
#pragma unroll
    for (int k = 0; k < LS_PER; ++k) cur[k] = nxt[k];
  }
}

int64_t line_index_tiles(int64_t nbytes) { return (nbytes + LI_TILE - 1) / LI_TILE; }

NlOut line_index_pass1_views(const LineIndexWs& W, int64_t nbytes, uint64_t stream) {
  const int64_t nt = line_index_tiles(nbytes);
  if (nt <= 0 || nt > W.ntiles_cap) throw std::runtime_error("line_index: empty text or workspace too small");
  NlOut o;
  o.cnt = reinterpret_cast<int32_t*>(W.buf + 3 * W.ntiles_cap);
  o.crf = o.cnt + W.ntiles_cap;
  o.nlm = reinterpret_cast<uint64_t*>(W.buf + 4 * W.ntiles_cap);
  o.ntiles = nt;
  // counts + flags are accumulated with atomics by the fused pass: zero [cnt, crf + nt) at once
  const hipError_t e = hipMemsetAsync(o.cnt, 0, (size_t)(W.ntiles_cap + nt) * sizeof(int32_t),
                                      reinterpret_cast<hipStream_t>(stream));
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e) + " in line_index");
  return o;
}

void line_index_dev(const uint8_t* text, int64_t nbytes, const LineIndexWs& W, int64_t* starts, int32_t* lens,
                    int64_t cap, int64_t* info, bool trim, int32_t* blk, int64_t nblk, uint64_t stream, bool counted) {
  const int64_t nt = line_index_tiles(nbytes);
  if (nt <= 0 || nt > W.ntiles_cap) throw std::runtime_error("line_index: empty text or workspace too small");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int64_t* off = W.buf;
  int64_t* fix_g = W.buf + W.ntiles_cap;
  int64_t* fix_end = W.buf + 2 * W.ntiles_cap;
  int32_t* cnt = reinterpret_cast<int32_t*>(W.buf + 3 * W.ntiles_cap);
  int32_t* crf = cnt + W.ntiles_cap;               // the int64 slot region holds 2 x ntiles_cap int32
  uint64_t* nlm = reinterpret_cast<uint64_t*>(W.buf + 4 * W.ntiles_cap);   // LI_THREADS words per tile
  if (!counted) hipLaunchKernelGGL(k_nl_count, dim3((unsigned)nt), dim3(LI_THREADS), 0, st, text, nbytes, cnt, nlm, crf);
  hipLaunchKernelGGL(k_tile_scan, dim3(1), dim3(LS_THREADS), 0, st, cnt, nt, off);
  hipLaunchKernelGGL(k_nl_lines, dim3((unsigned)((nt + LI_LINES_TPB - 1) / LI_LINES_TPB)), dim3(LI_THREADS), 0, st,
                     text, nbytes, (int64_t)nt, nlm, crf, off, starts, lens, cap,
                     fix_g, fix_end, blk, nblk);
  hipLaunchKernelGGL(k_line_fix, dim3((unsigned)((nt + 1 + 255) / 256)), dim3(256), 0, st, nt, nbytes, fix_g, fix_end,
                     off, cnt, starts, lens, cap, info, blk, nblk);
  if (trim) hipLaunchKernelGGL(k_line_trim, dim3(1), dim3(256), 0, st, lens, cap, info);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e) + " in line_index");
}

}  // namespace lp
