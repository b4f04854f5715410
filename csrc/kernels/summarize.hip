// Summary + top-k of scored events (reference buildSummary,
// AnalysisService.java:188-215 -- event count, severity histogram, highest severity -- plus the
// north star's top-k event reduction), and the streaming mode's final re-score.
//
//   k_summ_level  one block per 4096-item chunk (1024 when k <= 256): the chunk is bitonic-sorted in LDS by
//                 (score desc, global line asc, pattern asc) -- a total, deterministic order, so
//                 every rank / run agrees on ties -- and its first k rows are written out. Level
//                 0 reads events (and adds them to the pattern / severity histograms with one
//                 global atomic each); later levels read the previous level's rows, so a few
//                 launches reduce any event count to the global top k.
//   k_rescore     streaming: the reference's left-to-right product with the chronological
//                 factor of the true global N (ScoringService.java:102-151), one lane per event,
//                 from the factors the score kernel kept (chrono_factor is the same LP_HD code).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <stdexcept>
#include <string>
#include <vector>

#include "lp_api.h"
#include "lp_core.h"

namespace lp {

constexpr int SUMM_THREADS = 1024;
constexpr int SUMM_CHUNK = 4096;
// k <= 256 (the usual top-100): 1024-row chunks in 256-thread blocks. A 44.5k-event step then runs
// its first level on 44 CUs instead of 11, with 55 barrier stages of 1024 keys instead of 78 of 4096
// (the 4096-row level took 68 + 48 us per step for two levels, profiles/r3_w)
constexpr int SUMM_THREADS_S = 256;
constexpr int SUMM_CHUNK_S = 1024;
constexpr int SUMM_LDS_SEV = 256;             // severity histogram in LDS up to this many names

struct Row {
  double score;
  int64_t line;
  int32_t pat;
};

LP_HD bool row_before(const Row& a, const Row& b) {      // a sorts before b
  if (a.score != b.score) return a.score > b.score;
  if (a.line != b.line) return a.line < b.line;
  return a.pat < b.pat;
}

LP_HD Row empty_row() { return Row{-INFINITY, -1, -1}; }

// A row as one 128-bit key whose ASCENDING unsigned order is the row order: hi = the score's
// order-preserving bit pattern, inverted (higher score first), lo = line << 24 | pattern.
struct Key {
  uint64_t hi, lo;
};

__device__ __forceinline__ Key row_key(const Row& r) {
  uint64_t b;
  __builtin_memcpy(&b, &r.score, 8);
  const uint64_t ord = (b >> 63) ? ~b : (b | 0x8000000000000000ull);
  return Key{~ord, r.line < 0 ? ~0ull : ((uint64_t)r.line << 24) | (uint64_t)(uint32_t)r.pat};
}

__device__ __forceinline__ Row key_row(const Key& k) {
  const uint64_t ord = ~k.hi;
  const uint64_t b = (ord >> 63) ? (ord & 0x7FFFFFFFFFFFFFFFull) : ~ord;
  Row r;
  __builtin_memcpy(&r.score, &b, 8);
  if (k.lo == ~0ull) {
    r.line = -1;
    r.pat = -1;
  } else {
    r.line = (int64_t)(k.lo >> 24);
    r.pat = (int32_t)(k.lo & 0xFFFFFFull);
  }
  return r;
}

__device__ __forceinline__ bool key_less(const Key& a, const Key& b) {
  return a.hi != b.hi ? a.hi < b.hi : a.lo < b.lo;
}

// One CHUNK-row chunk per THREADS-thread block: load (+ histograms, + packed event records), bitonic
// sort of 128-bit keys in LDS (one compare-exchange per thread per stage pair), write the first k.
template <int CHUNK, int THREADS>
__global__ __launch_bounds__(THREADS) void k_summ_level(SummIn in, int64_t n, int k, int nsev,
                                                        double* __restrict__ rows_out,
                                                        unsigned long long* __restrict__ pat_hist,
                                                        unsigned long long* __restrict__ sev_hist) {
  __shared__ Key s_key[CHUNK];
  __shared__ unsigned int s_sev[SUMM_LDS_SEV];
  const bool lds_sev = sev_hist && nsev <= SUMM_LDS_SEV;
  if (lds_sev)
    for (int j = threadIdx.x; j < nsev; j += THREADS) s_sev[j] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * CHUNK;
  const int64_t add = in.line_add ? *in.line_add : 0;
  if (in.dn && !in.rows) n = min(n, *in.dn);      // capacity n, device count *dn
  for (int j = threadIdx.x; j < CHUNK; j += THREADS) {
    const int64_t i = base + j;
    Row r = empty_row();
    if (i < n) {
      if (in.rows) {
        r = Row{in.rows[3 * i], (int64_t)in.rows[3 * i + 1], (int32_t)in.rows[3 * i + 2]};
      } else {
        r.score = in.score[i];
        r.line = (in.line64 ? in.line64[i] : (int64_t)in.line32[i]) + add;
        r.pat = in.pat[i];
        if (pat_hist) atomicAdd(pat_hist + r.pat, 1ull);
        if (sev_hist) {
          const int sv = in.sev_of_pat[r.pat];
          if (lds_sev)
            atomicAdd(s_sev + sv, 1u);
          else
            atomicAdd(sev_hist + sv, 1ull);
        }
        if (in.ev_out) {                      // every event record, packed for one D2H copy
          reinterpret_cast<int64_t*>(in.ev_out)[i] = r.line;
          reinterpret_cast<double*>(in.ev_out)[n + i] = r.score;
          reinterpret_cast<int32_t*>(in.ev_out)[4 * n + i] = r.pat;
        }
      }
    }
    s_key[j] = row_key(r);
  }
  __syncthreads();
  if (lds_sev)
    for (int j = threadIdx.x; j < nsev; j += THREADS)
      if (s_sev[j]) atomicAdd(sev_hist + j, (unsigned long long)s_sev[j]);
  // bitonic sort, ascending key order = row order
  for (int size = 2; size <= CHUNK; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
#pragma unroll
      for (int q = 0; q < CHUNK / 2 / THREADS; ++q) {
        const int t = threadIdx.x + q * THREADS;
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const Key a = s_key[lo], b = s_key[hi];
        if (key_less(b, a) == up) {
          s_key[lo] = b;
          s_key[hi] = a;
        }
      }
      __syncthreads();
    }
  }
  double* o = rows_out + (int64_t)blockIdx.x * k * 3;
  for (int j = threadIdx.x; j < k; j += THREADS) {
    const Row r = key_row(s_key[j]);
    o[3 * j] = r.score;
    o[3 * j + 1] = (double)r.line;
    o[3 * j + 2] = (double)r.pat;
  }
}

// ---------------------------------------------------------------------------------------------
// Event top-k by threshold selection (k <= SEL_K_MAX, event input): the levels above sort every
// 1024-event chunk completely to keep 100 rows of it (3 launches, ~64 us for a 45k-event step).
// Here only the rows that can be in the top k are sorted:
//   k_sel_hist     one lane per event: histogram of the key's top SEL_BITS bits (the key order is
//                  the row order, so a lower bin holds only better rows) + the level-0 duties
//                  (pattern / severity histograms, packed event records);
//   k_sel_pick     one block: the first bin b* at which the cumulative count reaches k;
//   k_sel_collect  the keys of bins <= b* (every row of the top k is among them);
//   k_sel_final    one block: bitonic sort of the collected keys in LDS, first k rows out (keys
//                  stream through LDS against the running k-th best, should a tie-heavy bin
//                  collect more than fits).
constexpr int SEL_BITS = 16;
constexpr int SEL_BINS = 1 << SEL_BITS;
constexpr int SEL_K_MAX = 256;
constexpr int SEL_CH = 2048;
constexpr int SEL_FINAL_THREADS = 1024;

__device__ __forceinline__ uint32_t sel_bin(const Key& k) { return (uint32_t)(k.hi >> (64 - SEL_BITS)); }

__device__ __forceinline__ Row event_row(const SummIn& in, int64_t i, int64_t add) {
  return Row{in.score[i], (in.line64 ? in.line64[i] : (int64_t)in.line32[i]) + add, in.pat[i]};
}

__global__ __launch_bounds__(256) void k_sel_hist(SummIn in, int64_t n, int nsev, unsigned int* __restrict__ bins,
                                                  unsigned long long* __restrict__ pat_hist,
                                                  unsigned long long* __restrict__ sev_hist) {
  __shared__ unsigned int s_sev[SUMM_LDS_SEV];
  const bool lds_sev = sev_hist && nsev <= SUMM_LDS_SEV;
  if (lds_sev)
    for (int j = threadIdx.x; j < nsev; j += blockDim.x) s_sev[j] = 0;
  __syncthreads();
  if (in.dn) n = min(n, *in.dn);
  const int64_t add = in.line_add ? *in.line_add : 0;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const Row r = event_row(in, i, add);
    atomicAdd(bins + sel_bin(row_key(r)), 1u);
    if (pat_hist) atomicAdd(pat_hist + r.pat, 1ull);
    if (sev_hist) {
      const int sv = in.sev_of_pat[r.pat];
      if (lds_sev)
        atomicAdd(s_sev + sv, 1u);
      else
        atomicAdd(sev_hist + sv, 1ull);
    }
    if (in.ev_out) {
      reinterpret_cast<int64_t*>(in.ev_out)[i] = r.line;
      reinterpret_cast<double*>(in.ev_out)[n + i] = r.score;
      reinterpret_cast<int32_t*>(in.ev_out)[4 * n + i] = r.pat;
    }
  }
  __syncthreads();
  if (lds_sev)
    for (int j = threadIdx.x; j < nsev; j += blockDim.x)
      if (s_sev[j]) atomicAdd(sev_hist + j, (unsigned long long)s_sev[j]);
}

// sel[0] = b* (the last bin to collect)
__global__ __launch_bounds__(1024) void k_sel_pick(unsigned int* __restrict__ bins, int k, unsigned int* __restrict__ sel) {
  constexpr int PER = SEL_BINS / 1024;
  __shared__ unsigned int s_sum[1024];
  unsigned int loc[PER];
  unsigned int t = 0;
  const int b0 = threadIdx.x * PER;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    loc[j] = bins[b0 + j];
    t += loc[j];
  }
  s_sum[threadIdx.x] = t;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {           // inclusive scan of the per-thread sums
    const unsigned int v = threadIdx.x >= o ? s_sum[threadIdx.x - o] : 0u;
    __syncthreads();
    s_sum[threadIdx.x] += v;
    __syncthreads();
  }
  const unsigned int before = threadIdx.x ? s_sum[threadIdx.x - 1] : 0u;
  if (threadIdx.x == 1023 && s_sum[1023] < (unsigned int)k) sel[0] = SEL_BINS - 1;   // fewer than k rows
  if (before < (unsigned int)k && s_sum[threadIdx.x] >= (unsigned int)k) {
    unsigned int c = before;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      c += loc[j];
      if (c >= (unsigned int)k) {
        sel[0] = (unsigned int)(b0 + j);
        break;
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_sel_collect(SummIn in, int64_t n, const unsigned int* __restrict__ sel,
                                                     Key* __restrict__ buf, unsigned int* __restrict__ cnt) {
  if (in.dn) n = min(n, *in.dn);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Key kk = row_key(event_row(in, i, in.line_add ? *in.line_add : 0));
  if (sel_bin(kk) <= sel[0]) buf[atomicAdd(cnt, 1u)] = kk;   // (buf holds n keys)
}

__device__ __forceinline__ void bitonic_lds(Key* s, int np) {
  for (int size = 2; size <= np; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < np / 2; t += blockDim.x) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const Key a = s[lo], b = s[hi];
        if (key_less(b, a) == up) {
          s[lo] = b;
          s[hi] = a;
        }
      }
      __syncthreads();
    }
  }
}

__global__ __launch_bounds__(SEL_FINAL_THREADS) void k_sel_final(const Key* __restrict__ buf,
                                                                 const unsigned int* __restrict__ cnt_p, int k,
                                                                 double* __restrict__ rows_out) {
  // the collected keys stream through LDS in batches of one key per thread: a key enters only if it
  // beats the current k-th best (T); when the next batch might not fit, the LDS keys are sorted and
  // cut to the best k. A normal step sorts once; a bin full of tied scores costs one pass over it.
  __shared__ Key s[SEL_CH];
  __shared__ int s_m;
  const int64_t cnt = *cnt_p;
  const Key empty = row_key(empty_row());
  Key T = empty;                                  // rows sort before `empty`: any real key enters
  bool have_t = false;
  if (threadIdx.x == 0) s_m = 0;
  __syncthreads();
  for (int64_t off = 0;;) {
    for (;;) {
      const int cur = s_m;                        // every thread reads it before any thread adds
      __syncthreads();
      if (off >= cnt || cur + (int)blockDim.x > SEL_CH) break;
      const int64_t j = off + threadIdx.x;
      if (j < cnt) {
        const Key key = buf[j];
        if (!have_t || key_less(key, T)) s[atomicAdd(&s_m, 1)] = key;
      }
      off += blockDim.x;
      __syncthreads();
    }
    const int m = s_m;
    int np = 2;
    while (np < m) np <<= 1;
    for (int j = m + threadIdx.x; j < np; j += blockDim.x) s[j] = empty;
    __syncthreads();
    bitonic_lds(s, np);
    const int kept = m < k ? m : k;
    if (off >= cnt) {
      for (int j = threadIdx.x; j < k; j += blockDim.x) {
        const Row r = j < kept ? key_row(s[j]) : empty_row();
        rows_out[3 * j] = r.score;
        rows_out[3 * j + 1] = (double)r.line;
        rows_out[3 * j + 2] = (double)r.pat;
      }
      return;
    }
    if (kept == k) {                              // the k-th best so far: later keys must beat it
      T = s[k - 1];
      have_t = true;
    }
    __syncthreads();
    if (threadIdx.x == 0) s_m = kept;
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void k_rescore(const int64_t* __restrict__ gl, const double* __restrict__ fac,
                                                 int64_t n, int64_t N, ScoreParams S, double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double* f = fac + 7 * i;
  out[i] = f[0] * f[1] * chrono_factor(gl[i], N, S) * f[3] * f[4] * f[5] * (1.0 - f[6]);
}

namespace {
// off by default: on the bench step's 45k events the selection path measured 63.5 (k_sel_hist: its
// global bin atomics collide -- equal scores share a bin) + 13.5 + 5 + 8.6 us against ~63 us for
// the three chunk-sort levels (profiles/r5_c/bench_kernels.txt vs profiles/r4_e)
bool g_summ_select = false;
}  // namespace
bool summ_select() { return g_summ_select; }
void set_summ_select(bool on) { g_summ_select = on; }

static void check(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e) + " in " + what);
}

size_t summarize_dev(const SummIn& in, int64_t n, int k, int nsev, double* top_rows, unsigned long long* pat_hist,
                     unsigned long long* sev_hist, void* ws, size_t ws_bytes, uint64_t stream) {
  if (k < 1 || k > SUMM_CHUNK / 2) throw std::runtime_error("summarize: 1 <= k <= 1024");
  if (!in.rows && k <= SEL_K_MAX && summ_select()) {
    // workspace: [bins u32 x SEL_BINS | sel u32 x 4 | count u32 x 4 | keys 16 B x n]
    const size_t need = (size_t)SEL_BINS * 4 + 32 + (size_t)std::max<int64_t>(n, 1) * sizeof(Key);
    if (!ws || ws_bytes < need) return need;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    unsigned int* bins = static_cast<unsigned int*>(ws);
    unsigned int* sel = bins + SEL_BINS;
    unsigned int* cnt = sel + 4;
    Key* keys = reinterpret_cast<Key*>(static_cast<uint8_t*>(ws) + (size_t)SEL_BINS * 4 + 32);
    // (the workspace is the engine's shared scratch: other stages reuse it between calls)
    if (hipMemsetAsync(ws, 0, (size_t)SEL_BINS * 4 + 32, st) != hipSuccess) throw std::runtime_error("summarize: memset");
    const unsigned nb = (unsigned)std::max<int64_t>(1, (n + 255) / 256);
    hipLaunchKernelGGL(k_sel_hist, dim3(nb), dim3(256), 0, st, in, n, nsev, bins, pat_hist, sev_hist);
    check("k_sel_hist");
    hipLaunchKernelGGL(k_sel_pick, dim3(1), dim3(1024), 0, st, bins, k, sel);
    check("k_sel_pick");
    hipLaunchKernelGGL(k_sel_collect, dim3(nb), dim3(256), 0, st, in, n, sel, keys, cnt);
    check("k_sel_collect");
    hipLaunchKernelGGL(k_sel_final, dim3(1), dim3(SEL_FINAL_THREADS), 0, st, keys, cnt, k, top_rows);
    check("k_sel_final");
    return need;
  }
  const bool small = k <= SUMM_CHUNK_S / 4;
  const int64_t chunk = small ? SUMM_CHUNK_S : SUMM_CHUNK;
  // workspace: two ping-pong row buffers sized for level 0
  const int64_t nb0 = std::max<int64_t>(1, (n + chunk - 1) / chunk);
  const size_t rows_bytes = (size_t)nb0 * k * 3 * sizeof(double);
  const size_t need = 2 * rows_bytes;
  if (!ws || ws_bytes < need) return need;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  double* buf[2] = {static_cast<double*>(ws), reinterpret_cast<double*>(static_cast<uint8_t*>(ws) + rows_bytes)};
  int64_t m = n, nb = nb0;
  SummIn cur = in;
  int which = 0;
  for (int level = 0;; ++level) {
    double* dst = nb == 1 ? top_rows : buf[which];
    if (small)
      hipLaunchKernelGGL((k_summ_level<SUMM_CHUNK_S, SUMM_THREADS_S>), dim3((unsigned)nb), dim3(SUMM_THREADS_S), 0, st,
                         cur, m, k, nsev, dst, level == 0 ? pat_hist : nullptr, level == 0 ? sev_hist : nullptr);
    else
      hipLaunchKernelGGL((k_summ_level<SUMM_CHUNK, SUMM_THREADS>), dim3((unsigned)nb), dim3(SUMM_THREADS), 0, st, cur,
                         m, k, nsev, dst, level == 0 ? pat_hist : nullptr, level == 0 ? sev_hist : nullptr);
    check("k_summ_level");
    if (nb == 1) break;
    SummIn nx{};
    nx.rows = dst;
    cur = nx;
    m = nb * (int64_t)k;
    nb = (m + chunk - 1) / chunk;
    which ^= 1;
  }
  return need;
}

void summarize_host(const SummIn& in, int64_t n, int k, double* top_rows, int64_t* pat_hist, int64_t* sev_hist) {
  const int64_t add = in.line_add ? *in.line_add : 0;
  std::vector<Row> rows(n);
  if (in.dn && !in.rows) n = std::min<int64_t>(n, *in.dn);
  rows.resize(n);
  for (int64_t i = 0; i < n; ++i) {
    if (in.rows) {
      rows[i] = Row{in.rows[3 * i], (int64_t)in.rows[3 * i + 1], (int32_t)in.rows[3 * i + 2]};
      continue;
    }
    rows[i] = Row{in.score[i], (in.line64 ? in.line64[i] : (int64_t)in.line32[i]) + add, in.pat[i]};
    if (in.ev_out) {
      reinterpret_cast<int64_t*>(in.ev_out)[i] = rows[i].line;
      reinterpret_cast<double*>(in.ev_out)[n + i] = rows[i].score;
      reinterpret_cast<int32_t*>(in.ev_out)[4 * n + i] = rows[i].pat;
    }
    if (pat_hist) ++pat_hist[in.pat[i]];
    if (sev_hist) ++sev_hist[in.sev_of_pat[in.pat[i]]];
  }
  const int64_t kk = std::min<int64_t>(k, n);
  std::partial_sort(rows.begin(), rows.begin() + kk, rows.end(), row_before);
  for (int j = 0; j < k; ++j) {
    const Row r = j < kk ? rows[j] : empty_row();
    top_rows[3 * j] = r.score;
    top_rows[3 * j + 1] = (double)r.line;
    top_rows[3 * j + 2] = (double)r.pat;
  }
}

void rescore_dev(const int64_t* gl, const double* fac, int64_t n, int64_t N, const ScoreParams& S, double* out,
                 uint64_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_rescore, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     gl, fac, n, N, S, out);
  check("k_rescore");
}

void rescore_host(const int64_t* gl, const double* fac, int64_t n, int64_t N, const ScoreParams& S, double* out) {
  for (int64_t i = 0; i < n; ++i) {
    const double* f = fac + 7 * i;
    out[i] = f[0] * f[1] * chrono_factor(gl[i], N, S) * f[3] * f[4] * f[5] * (1.0 - f[6]);
  }
}

}  // namespace lp
