// Bulk post-match pipeline without device-wide radix sorts.
//
// lp_post.hip's bulk path sorted every (regex, line) candidate key and every (line, pattern) event
// key with rocPRIM device sorts: ~36 launches per step, most of them ~5 us of launch-latency-bound
// merge / onesweep passes over a few hundred thousand keys (profiles/r3_s timeline). The orders
// needed are bucket orders, so this path builds them with counting sorts whose buckets are small:
//
//   hits    bucket = regex (R buckets; a step's ~200k candidates spread over ~3k regexes):
//           count -> scan -> scatter -> per-regex workgroup sorts its lines in LDS -> the same
//           sorted packed keys the radix sort produced, so the DFA / BPG first-of-run verify kernels
//           run unchanged -> per-regex kept counts -> scan -> per-regex emit of the hit CSR, event
//           counts and their running sums (the reference's per-regex line order of a hit list).
//   events  bucket = block of 2^s lines (<= 4097 buckets): count -> scan -> scatter of each hit's
//           (line << pbits | pattern) keys -> per-bucket LDS sort = the reference's event order
//           (line, then pattern: AnalysisService.java:89-113) + segment, window coverage, frequency
//           key; then bucket = frequency key: count -> scan -> scatter of event indices -> per-key
//           sort = the rank of each event among earlier events of its key (penalty before record,
//           ScoringService.java:84-88) and the per-key counts.
//
// Count and scatter kernels aggregate in LDS first (one global atomic per block and bucket), so a
// hot bucket (one regex or pattern matching most lines) costs no same-address atomic storm. A
// bucket larger than the LDS tile is sorted in tiles and merged bottom-up in global memory by its
// workgroup (each element binary-searches its partner run: stable, no extra launch) -- correct for
// any skew, fast for the common one. 10 + 9 launches per step instead of 29 + 22.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "post_core.h"

namespace lp {

namespace {

#define PB_CHECK(x)                                                                                             \
  do {                                                                                                          \
    hipError_t e_ = (x);                                                                                        \
    if (e_ != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e_) + " at " #x); \
  } while (0)

constexpr int PB_T = 256;             // per-bucket workgroups
constexpr int PB_AT = 1024;           // aggregated count / scatter / scan workgroups
constexpr int PB_IPT = 8;             // items per thread per scatter round
constexpr int PB_LDS_BINS = 16384;    // buckets aggregated in LDS (scatter: count + base = 128 KiB)
constexpr int PB_HIT_CAP = 4096;      // lines (uint32) of one regex sorted in LDS in one piece
constexpr int PB_EV_CAP = 2048;       // event keys (uint64) of one line block
constexpr int PB_KEY_CAP = 4096;      // event indices (uint32) of one frequency key sub-bucket
constexpr int PB_TARGET = 1024;       // expected items per sub-bucket of a split primary bucket
constexpr int PB_EV_TARGET = 256;     // expected events per line block
constexpr int PB_PAD_SPAN = PB_T * 16; // pad-tail entries per filler workgroup

inline hipStream_t pb_stream(uint64_t s) { return reinterpret_cast<hipStream_t>(s); }
inline unsigned pb_blocks(int64_t n, int64_t per) { return (unsigned)std::max<int64_t>(1, (n + per - 1) / per); }
// aggregated kernels: enough blocks to spread the items, few enough that the per-block LDS flush
// (one pass over the buckets) stays small
inline unsigned pb_agg_grid(int64_t n) { return (unsigned)std::min<int64_t>(256, pb_blocks(n, (int64_t)PB_AT * PB_IPT)); }

// exclusive prefix of v over the block (thread order); *total = block sum. scratch: blockDim/64 entries
__device__ int64_t pb_excl_scan(int64_t v, int64_t* scratch, int64_t* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  int64_t incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const long long u = __shfl_up((long long)incl, d, 64);
    if (lane >= d) incl += u;
  }
  if (lane == 63) scratch[wid] = incl;
  __syncthreads();
  int64_t base = 0, tot = 0;
  for (int w = 0; w < nw; ++w) {
    if (w < wid) base += scratch[w];
    tot += scratch[w];
  }
  __syncthreads();
  *total = tot;
  return base + incl - v;
}

// ascending bitonic sort of s[0, np) in LDS, np a power of two, whole block
template <typename T>
__device__ void pb_bitonic(T* s, int np) {
  for (int size = 2; size <= np; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < np / 2; t += blockDim.x) {
        const int lo = 2 * t - (t & (stride - 1)), hi = lo + stride;
        const T a = s[lo], b = s[hi];
        if ((b < a) == ((lo & size) == 0)) {
          s[lo] = b;
          s[hi] = a;
        }
      }
      __syncthreads();
    }
}

// d[0, m) -> lds[0, np) padded with the all-ones value (sorts last), sorted; m <= CAP
template <typename T>
__device__ void pb_sort_lds(const T* d, int m, T* lds) {
  int np = 2;
  while (np < m) np <<= 1;
  for (int i = threadIdx.x; i < np; i += blockDim.x) lds[i] = i < m ? d[i] : (T)~(T)0;
  __syncthreads();
  pb_bitonic(lds, np);
}

// d[0, m) ascending in place, any m: LDS tiles of CAP, then bottom-up merges between d and tmp.
// Merge pass: an element of run A lands at its index + (# of B strictly below it), an element of
// B at its index + (# of A at or below it) -- stable, every element independent. Global writes of
// one pass are visible to the whole workgroup after the barrier (one CU, write-through L1).
template <typename T, int CAP>
__device__ void pb_sort_global(T* d, T* tmp, int64_t m, T* lds) {
  for (int64_t a = 0; a < m; a += CAP) {
    const int cm = (int)(m - a < CAP ? m - a : CAP);
    pb_sort_lds(d + a, cm, lds);
    for (int i = threadIdx.x; i < cm; i += blockDim.x) d[a + i] = lds[i];
    __syncthreads();
  }
  T* src = d;
  T* dst = tmp;
  for (int64_t w = CAP; w < m; w <<= 1) {
    for (int64_t i = threadIdx.x; i < m; i += blockDim.x) {
      const int64_t p = i / (2 * w) * (2 * w);
      const int64_t mid = p + w < m ? p + w : m, end = p + 2 * w < m ? p + 2 * w : m;
      const T v = src[i];
      int64_t pos;
      if (i < mid) {
        int64_t lo = mid, hi = end;
        while (lo < hi) {
          const int64_t q = (lo + hi) >> 1;
          if (src[q] < v) lo = q + 1; else hi = q;
        }
        pos = i + (lo - mid);
      } else {
        int64_t lo = p, hi = mid;
        while (lo < hi) {
          const int64_t q = (lo + hi) >> 1;
          if (src[q] <= v) lo = q + 1; else hi = q;
        }
        pos = (i - mid) + lo;
      }
      dst[pos] = v;
    }
    __syncthreads();
    T* t = src;
    src = dst;
    dst = t;
  }
  if (src != d) {
    for (int64_t i = threadIdx.x; i < m; i += blockDim.x) d[i] = src[i];
    __syncthreads();
  }
}

// Bucket counts: item(i, bucket, weight) for i in [0, n); aggregated in LDS when the buckets fit.
template <typename Item>
__device__ void pb_count(Item&& item, int64_t n, int nb, uint32_t* gcnt, uint32_t* lcnt) {
  const bool lds = nb <= PB_LDS_BINS;
  if (lds) {
    for (int b = threadIdx.x; b < nb; b += blockDim.x) lcnt[b] = 0;
    __syncthreads();
  }
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    uint32_t b, w;
    if (item(i, b, w) && w) {
      if (lds) atomicAdd(&lcnt[b], w);
      else atomicAdd(&gcnt[b], w);
    }
  }
  if (lds) {
    __syncthreads();
    for (int b = threadIdx.x; b < nb; b += blockDim.x)
      if (lcnt[b]) atomicAdd(&gcnt[b], lcnt[b]);
  }
}

// Bucket scatter: item(i, bucket, weight, payload) reserves `weight` consecutive slots of its
// bucket; put(payload, bucket, first slot within the bucket). Rounds of blockDim * PB_IPT items:
// LDS ranks, one global reservation per (block, bucket), then the writes.
template <typename Item, typename Put>
__device__ void pb_scatter(Item&& item, Put&& put, int64_t n, int nb, uint32_t* gfill, uint32_t* lcnt,
                           uint32_t* lbase) {
  const bool lds = nb <= PB_LDS_BINS;
  if (lds) {
    for (int b = threadIdx.x; b < nb; b += blockDim.x) lcnt[b] = 0;
    __syncthreads();
  }
  const int64_t per_round = (int64_t)blockDim.x * PB_IPT;
  for (int64_t base = (int64_t)blockIdx.x * per_round; base < n; base += (int64_t)gridDim.x * per_round) {
    uint32_t bin[PB_IPT], loc[PB_IPT];
    uint64_t pay[PB_IPT];
    bool ok[PB_IPT];
#pragma unroll
    for (int q = 0; q < PB_IPT; ++q) {
      const int64_t i = base + (int64_t)q * blockDim.x + threadIdx.x;
      uint32_t w = 0;
      ok[q] = i < n && item(i, bin[q], w, pay[q]) && w > 0;
      if (ok[q]) loc[q] = lds ? atomicAdd(&lcnt[bin[q]], w) : atomicAdd(&gfill[bin[q]], w);
    }
    if (lds) {
      __syncthreads();
      for (int b = threadIdx.x; b < nb; b += blockDim.x) {
        const uint32_t c = lcnt[b];
        if (c) {
          lbase[b] = atomicAdd(&gfill[b], c);
          lcnt[b] = 0;
        }
      }
      __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < PB_IPT; ++q)
      if (ok[q]) put(pay[q], bin[q], (lds ? lbase[bin[q]] : 0u) + loc[q]);
  }
}

// exclusive scan of in[0, nb) into off[0, nb] (off[nb] = total), one block; then optionally
// copies the counts out (int64) and zeroes `in` (reused as the scatter's fill counters)
template <typename TI>
__global__ __launch_bounds__(PB_AT) void k_pb_scan(TI* in, int64_t nb, int64_t* off, int64_t* copy_out, int zero_in) {
  __shared__ int64_t scratch[PB_AT / 64];
  const int64_t per = (nb + blockDim.x - 1) / blockDim.x;
  const int64_t a = threadIdx.x * per, b = a + per < nb ? a + per : nb;
  int64_t s = 0;
  for (int64_t i = a; i < b; ++i) s += (int64_t)in[i];
  int64_t tot = 0;
  int64_t run = pb_excl_scan(s, scratch, &tot);
  for (int64_t i = a; i < b; ++i) {
    off[i] = run;
    const int64_t c = (int64_t)in[i];
    run += c;
    if (copy_out) copy_out[i] = c;
    if (zero_in) in[i] = 0;
  }
  if (threadIdx.x == 0) off[nb] = tot;
}

// Two-level buckets (hits by regex, event ranks by frequency key): a primary bucket p with more
// than PB_TARGET items is split by its coordinate (line / event index) into sub-buckets of 2^s_p
// coordinates, s_p the largest width whose expected load stays <= PB_TARGET. Sub-buckets of p are
// contiguous and in coordinate order, so the per-sub-bucket LDS sorts still yield p's items in
// order, and a bucket of one hot regex or key is sorted by hundreds of workgroups, not one.
// plan: shift[p], first sub-bucket base[p] (base[np] = total), owner sub_prim[b]; optionally the
// primary counts copied out as int64
__global__ __launch_bounds__(PB_AT) void k_pb_plan(const uint32_t* __restrict__ cnt, int np, int cbits, int64_t range,
                                                  const int64_t* __restrict__ drange, uint8_t* __restrict__ shift,
                                                  uint32_t* __restrict__ base, int32_t* __restrict__ sub_prim,
                                                  int64_t* __restrict__ copy_out) {
  __shared__ int64_t scratch[PB_AT / 64];
  if (drange) range = *drange < range ? *drange : range;     // device count, capped at the capacity
  const int64_t per = (np + blockDim.x - 1) / blockDim.x;
  const int64_t a = threadIdx.x * per, e = a + per < np ? a + per : np;
  auto plan = [&](uint32_t c, int& s) -> int64_t {
    s = cbits;
    if (c == 0) return 0;
    if (c > (uint32_t)PB_TARGET) {
      s = 0;
      while (s < cbits && (double)c * (double)(int64_t(1) << (s + 1)) <= (double)PB_TARGET * (double)range) ++s;
    }
    return ((range - 1) >> s) + 1;
  };
  int64_t tot_mine = 0;
  for (int64_t p = a; p < e; ++p) {
    int s;
    tot_mine += plan(cnt[p], s);
  }
  int64_t tot = 0;
  int64_t run = pb_excl_scan(tot_mine, scratch, &tot);
  for (int64_t p = a; p < e; ++p) {
    int s;
    const uint32_t c = cnt[p];
    const int64_t ns = plan(c, s);
    shift[p] = (uint8_t)s;
    base[p] = (uint32_t)run;
    for (int64_t j = 0; j < ns; ++j) sub_prim[run + j] = (int32_t)p;
    run += ns;
    if (copy_out) copy_out[p] = c;
  }
  if (threadIdx.x == 0) base[np] = (uint32_t)tot;
}

// ---- hits

struct HbIn {            // candidate entries in the HitsArgs layout
  const int64_t* cand;
  const int64_t* cand2;
  int64_t n, pre_from, n1, n2;   // n1 / n2: used lengths of the two regions (device-count mode)
  bool dc;
  uint32_t R, lmask;             // a key outside [0, R) x [0, 2^lbits) is never bucketed
};

__device__ __forceinline__ HbIn hb_in(const HitsArgs& A) {
  HbIn S{A.cand, A.cand2, A.n, A.pre_from, A.pre_from, A.n - A.pre_from, A.dcount != nullptr,
         (uint32_t)A.R, A.lbits >= 32 ? ~0u : ((1u << A.lbits) - 1u)};
  if (S.dc) {
    S.n1 = (int64_t)min((unsigned long long)S.n1, A.dcount[0]);
    S.n2 = (int64_t)min((unsigned long long)S.n2, A.dcount[1]);
  }
  return S;
}

// entry i -> (regex, line << 1 | pre-verified); false for an unused slot or a failed candidate
__device__ __forceinline__ bool hb_get(const HbIn& S, int64_t i, uint32_t& r, uint32_t& v) {
  int64_t k;
  bool pre;
  if (S.dc) {
    if (i < S.pre_from) {
      if (i >= S.n1) return false;
      k = S.cand[i];
      pre = false;
    } else {
      const int64_t j = i - S.pre_from;
      if (j >= S.n2) return false;
      k = S.cand2[j];
      pre = true;
    }
  } else {
    k = S.cand[i];
    pre = i >= S.pre_from;
  }
  if (k < 0) return false;
  r = (uint32_t)(k >> 32);
  const uint32_t x = (uint32_t)(k & 0xFFFFFFFFll);
  if (r >= S.R || (x & ~S.lmask)) return false;   // (defensive: a key no matcher can produce)
  v = (x << 1) | (pre ? 1u : 0u);
  return true;
}

struct HbPlan {
  const uint8_t* shift;     // [R]
  const uint32_t* base;     // [R + 1]
};

__device__ __forceinline__ uint32_t hb_sub(const HbPlan& Q, uint32_t r, uint32_t v) {
  return Q.base[r] + ((v >> 1) >> Q.shift[r]);
}

__global__ __launch_bounds__(PB_AT) void k_hb_count(HitsArgs A, uint32_t* cnt) {
  extern __shared__ uint32_t pb_lds[];
  const HbIn S = hb_in(A);
  pb_count([&](int64_t i, uint32_t& b, uint32_t& w) {
    uint32_t v;
    w = 1;
    return hb_get(S, i, b, v);
  }, S.n, A.R, cnt, pb_lds);
}

__global__ __launch_bounds__(PB_AT) void k_hb_count2(HitsArgs A, HbPlan Q, int bcap, uint32_t* sub_cnt) {
  extern __shared__ uint32_t pb_lds[];
  const HbIn S = hb_in(A);
  pb_count([&](int64_t i, uint32_t& b, uint32_t& w) {
    uint32_t r, v;
    w = 1;
    if (!hb_get(S, i, r, v)) return false;
    b = hb_sub(Q, r, v);
    return true;
  }, S.n, bcap, sub_cnt, pb_lds);
}

__global__ __launch_bounds__(PB_AT) void k_hb_scatter(HitsArgs A, HbPlan Q, int bcap, const int64_t* __restrict__ sub_off,
                                                     uint32_t* fill, uint32_t* __restrict__ vals) {
  extern __shared__ uint32_t pb_lds[];
  const HbIn S = hb_in(A);
  pb_scatter([&](int64_t i, uint32_t& b, uint32_t& w, uint64_t& pay) {
    uint32_t r, v;
    w = 1;
    if (!hb_get(S, i, r, v)) return false;
    b = hb_sub(Q, r, v);
    pay = v;
    return true;
  }, [&](uint64_t pay, uint32_t b, uint32_t o) { vals[sub_off[b] + o] = (uint32_t)pay; },
     S.n, bcap, fill, pb_lds, pb_lds + bcap);
}

// one workgroup per sub-bucket: its lines sorted -> packed keys ((regex << lbits | line) << 1 |
// pre) as the radix sort wrote them; workgroups past bcap fill the pad tail [total, n) with
// LP_PAD_KEY
__global__ __launch_bounds__(PB_T) void k_hb_sort(const int64_t* __restrict__ sub_off, const int32_t* __restrict__ sub_reg,
                                                  const uint32_t* __restrict__ base, int R, int bcap, uint32_t* vals,
                                                  uint32_t* tmp, int lbits, int64_t n, uint64_t* __restrict__ kout) {
  __shared__ uint32_t lds[PB_HIT_CAP];
  const int b = blockIdx.x;
  const int nbk = (int)base[R];
  if (b >= bcap) {
    const int64_t total = sub_off[nbk];
    const int64_t a = (int64_t)(b - bcap) * PB_PAD_SPAN, e = a + PB_PAD_SPAN < n ? a + PB_PAD_SPAN : n;
    for (int64_t j = (a > total ? a : total) + threadIdx.x; j < e; j += blockDim.x) kout[j] = LP_PAD_KEY;
    return;
  }
  if (b >= nbk) return;
  const int64_t o = sub_off[b], m = sub_off[b + 1] - o;
  if (m == 0) return;
  const uint64_t rb = (uint64_t)sub_reg[b] << lbits;
  const uint32_t* src = lds;
  if (m <= PB_HIT_CAP) {
    pb_sort_lds(vals + o, (int)m, lds);
  } else {
    pb_sort_global<uint32_t, PB_HIT_CAP>(vals + o, tmp + o, m, lds);
    src = vals + o;
  }
  for (int64_t j = threadIdx.x; j < m; j += blockDim.x) {
    const uint32_t v = src[j];
    kout[o + j] = ((rb | (v >> 1)) << 1) | (v & 1u);
  }
}

// one workgroup per sub-bucket: verified first-of-run keys and the events they produce
__global__ __launch_bounds__(PB_T) void k_hb_kept(const int64_t* __restrict__ sub_off, const int32_t* __restrict__ sub_reg,
                                                  const uint32_t* __restrict__ base, int R, const uint8_t* __restrict__ flag,
                                                  const int64_t* __restrict__ stdk, EvTables E, uint32_t* kept,
                                                  int64_t* evs) {
  __shared__ int64_t scratch[PB_T / 64];
  const int b = blockIdx.x;
  if (b >= (int)base[R]) return;
  const int64_t o = sub_off[b], m = sub_off[b + 1] - o;
  const int r = sub_reg[b];
  const bool evr = E.prim_off[r + 1] > E.prim_off[r];     // regex with primary roles
  int64_t c = 0, e = 0;
  for (int64_t j = threadIdx.x; j < m; j += blockDim.x)
    if (flag[o + j]) {
      ++c;
      if (evr) e += hit_event_count(E, stdk[o + j]);
    }
  int64_t tc = 0, te = 0;
  pb_excl_scan(c, scratch, &tc);
  pb_excl_scan(e, scratch, &te);
  if (threadIdx.x == 0) {
    kept[b] = (uint32_t)tc;
    evs[b] = te;
  }
}

// offsets of every sub-bucket's kept hits and events; hit_off[r] = offset of r's first sub-bucket
__global__ __launch_bounds__(PB_AT) void k_hb_offsets(const uint32_t* kept, const int64_t* evs,
                                                     const uint32_t* __restrict__ base, int R, int64_t* kept_off,
                                                     int64_t* ev_off, int64_t* hit_off, int64_t* counters) {
  __shared__ int64_t scratch[PB_AT / 64];
  const int64_t nbk = base[R];
  const int64_t per = (nbk + blockDim.x - 1) / blockDim.x;
  const int64_t a = threadIdx.x * per, e = a + per < nbk ? a + per : nbk;
  int64_t sk = 0, se = 0;
  for (int64_t i = a; i < e; ++i) {
    sk += kept[i];
    se += evs[i];
  }
  int64_t tk = 0, te = 0;
  int64_t rk = pb_excl_scan(sk, scratch, &tk);
  int64_t re = pb_excl_scan(se, scratch, &te);
  for (int64_t i = a; i < e; ++i) {
    kept_off[i] = rk;
    ev_off[i] = re;
    rk += kept[i];
    re += evs[i];
  }
  if (threadIdx.x == 0) {
    kept_off[nbk] = tk;
    counters[0] = tk;
    counters[1] = te;
  }
  __syncthreads();
  for (int r = threadIdx.x; r <= R; r += blockDim.x) hit_off[r] = r < R ? kept_off[base[r]] : tk;
}

// one workgroup per sub-bucket: its kept keys in order -> hits / hit lines / events per hit /
// running event ends (inclusive)
__global__ __launch_bounds__(PB_T) void k_hb_emit(const int64_t* __restrict__ sub_off, const int32_t* __restrict__ sub_reg,
                                                  const uint32_t* __restrict__ base, int R,
                                                  const uint8_t* __restrict__ flag, const int64_t* __restrict__ stdk,
                                                  EvTables E, const int64_t* __restrict__ kept_off,
                                                  const int64_t* __restrict__ ev_off, int64_t* __restrict__ hits,
                                                  int32_t* __restrict__ hit_line, int64_t* __restrict__ ev_cnt,
                                                  int64_t* __restrict__ ev_end) {
  __shared__ int64_t scratch[PB_T / 64];
  const int b = blockIdx.x;
  if (b >= (int)base[R]) return;
  const int64_t o = sub_off[b], m = sub_off[b + 1] - o;
  if (m == 0) return;
  const int r = sub_reg[b];
  const bool evr = E.prim_off[r + 1] > E.prim_off[r];
  int64_t out = kept_off[b], ev_run = ev_off[b];
  for (int64_t t = 0; t < m; t += blockDim.x) {
    const int64_t j = t + threadIdx.x;
    const bool f = j < m && flag[o + j];
    int64_t k = 0, ec = 0;
    if (f) {
      k = stdk[o + j];
      ec = evr ? hit_event_count(E, k) : 0;
    }
    // one scan of (kept << 40 | events): a tile holds <= 256 kept keys and < 2^40 events
    int64_t tot = 0;
    const int64_t pre = pb_excl_scan(((f ? (int64_t)1 : 0) << 40) | ec, scratch, &tot);
    if (f) {
      const int64_t q = out + (pre >> 40);
      hits[q] = k;
      hit_line[q] = (int32_t)(k & 0xFFFFFFFFll);
      ev_cnt[q] = ec;
      ev_end[q] = ev_run + (pre & ((1ll << 40) - 1)) + ec;
    }
    out += tot >> 40;
    ev_run += tot & ((1ll << 40) - 1);
  }
}

// ---- events

struct EbIn {
  const int64_t* hits;
  const int64_t* ev_cnt;
  int64_t nh;                 // hits (device-count mode: capacity)
  int shift;
  const int64_t* dcnt;        // device-count mode: [hits, events]; else null
  int64_t ne_cap;             // device-count mode: event capacity
};

// device-count mode: false when the events overflowed their capacity (every kernel then leaves its
// outputs unset; the caller re-runs); n = the hits to read
__device__ __forceinline__ bool eb_live(const EbIn& S, int64_t& n) {
  n = S.nh;
  if (!S.dcnt) return true;
  if (S.dcnt[1] > S.ne_cap) return false;
  n = S.dcnt[0] < n ? S.dcnt[0] : n;
  return true;
}

// device-count mode: the events to read (0 after an overflow)
__device__ __forceinline__ int64_t eb_events(const int64_t* dcnt, int64_t ne) {
  if (!dcnt) return ne;
  return dcnt[1] > ne ? 0 : dcnt[1];
}

__global__ __launch_bounds__(PB_AT) void k_eb_count(EbIn S, int nb, uint32_t* cnt, int64_t* ne_fit) {
  extern __shared__ uint32_t pb_lds[];
  if (ne_fit && blockIdx.x == 0 && threadIdx.x == 0) ne_fit[0] = eb_events(S.dcnt, S.ne_cap);
  int64_t nh;
  if (!eb_live(S, nh)) return;
  pb_count([&](int64_t i, uint32_t& b, uint32_t& w) {
    w = (uint32_t)S.ev_cnt[i];
    b = (uint32_t)(S.hits[i] & 0xFFFFFFFFll) >> S.shift;
    return true;
  }, nh, nb, cnt, pb_lds);
}

__global__ __launch_bounds__(PB_AT) void k_eb_scatter(EbIn S, int nb, EvTables E, const int64_t* __restrict__ bin_off,
                                                     uint32_t* fill, uint64_t* __restrict__ ekeys) {
  extern __shared__ uint32_t pb_lds[];
  int64_t nh;
  if (!eb_live(S, nh)) return;
  pb_scatter([&](int64_t i, uint32_t& b, uint32_t& w, uint64_t& pay) {
    w = (uint32_t)S.ev_cnt[i];
    b = (uint32_t)(S.hits[i] & 0xFFFFFFFFll) >> S.shift;
    pay = (uint64_t)i;
    return true;
  }, [&](uint64_t i, uint32_t b, uint32_t o) {
    const int64_t k = S.hits[i];
    const int r = (int)(k >> 32);
    const uint64_t x = (uint64_t)(k & 0xFFFFFFFFll);
    const int64_t c = S.ev_cnt[i], p0 = E.prim_off[r], q = bin_off[b] + o;
    for (int64_t j = 0; j < c; ++j) ekeys[q + j] = (x << E.pbits) | (uint64_t)E.prim_pats[p0 + j];
  }, nh, nb, fill, pb_lds, pb_lds + nb);
}

// one workgroup per line block: events in (line, pattern) order + their outputs, window coverage
// and frequency sort key (events without a key get rank / key -1 here)
__global__ __launch_bounds__(PB_T) void k_eb_sort(const int64_t* __restrict__ bin_off, uint64_t* ekeys, uint64_t* etmp,
                                                  EvTables E, int32_t* __restrict__ ev_line, int32_t* __restrict__ ev_pat,
                                                  int32_t* __restrict__ ev_seg, uint32_t* __restrict__ fsort,
                                                  int64_t* __restrict__ ev_rank, int64_t* __restrict__ ev_fkey,
                                                  int32_t* __restrict__ cov, const int64_t* dcnt, int64_t ne_cap) {
  __shared__ uint64_t lds[PB_EV_CAP];
  if (dcnt && dcnt[1] > ne_cap) return;
  const int b = blockIdx.x;
  const int64_t o = bin_off[b], m = bin_off[b + 1] - o;
  if (m == 0) return;
  const uint64_t* src = lds;
  if (m <= PB_EV_CAP) {
    pb_sort_lds(ekeys + o, (int)m, lds);
  } else {
    pb_sort_global<uint64_t, PB_EV_CAP>(ekeys + o, etmp + o, m, lds);
    src = ekeys + o;
  }
  for (int64_t j = threadIdx.x; j < m; j += blockDim.x) {
    const int64_t e = o + j;
    int32_t a, w;
    const uint32_t fs = ev_post_one(E, src[j], e, ev_line, ev_pat, ev_seg, a, w);
    fsort[e] = fs;
    if ((int)fs >= E.nkeys) {
      ev_rank[e] = -1;
      ev_fkey[e] = -1;
    }
    // window coverage: consumers test cov > 0; equal concurrent stores from overlapping windows
    for (int32_t x = a; x < w; ++x) cov[x] = 1;
  }
}

struct KbPlan {
  const uint8_t* shift;     // [nk]
  const uint32_t* base;     // [nk + 1]
};

__global__ __launch_bounds__(PB_AT) void k_kb_count(const uint32_t* __restrict__ fsort, int64_t ne, int nk, uint32_t* cnt,
                                                   const int64_t* dcnt) {
  extern __shared__ uint32_t pb_lds[];
  ne = eb_events(dcnt, ne);
  pb_count([&](int64_t e, uint32_t& b, uint32_t& w) {
    b = fsort[e];
    w = 1;
    return (int)b < nk;
  }, ne, nk, cnt, pb_lds);
}

__global__ __launch_bounds__(PB_AT) void k_kb_count2(const uint32_t* __restrict__ fsort, int64_t ne, int nk, KbPlan Q,
                                                    int bcap, uint32_t* sub_cnt, const int64_t* dcnt) {
  extern __shared__ uint32_t pb_lds[];
  ne = eb_events(dcnt, ne);
  pb_count([&](int64_t e, uint32_t& b, uint32_t& w) {
    const uint32_t k = fsort[e];
    w = 1;
    if ((int)k >= nk) return false;
    b = Q.base[k] + (uint32_t)(e >> Q.shift[k]);
    return true;
  }, ne, bcap, sub_cnt, pb_lds);
}

__global__ __launch_bounds__(PB_AT) void k_kb_scatter(const uint32_t* __restrict__ fsort, int64_t ne, int nk, KbPlan Q,
                                                     int bcap, const int64_t* __restrict__ sub_off, uint32_t* fill,
                                                     uint32_t* __restrict__ kidx, const int64_t* dcnt) {
  extern __shared__ uint32_t pb_lds[];
  ne = eb_events(dcnt, ne);
  pb_scatter([&](int64_t e, uint32_t& b, uint32_t& w, uint64_t& pay) {
    const uint32_t k = fsort[e];
    w = 1;
    if ((int)k >= nk) return false;
    b = Q.base[k] + (uint32_t)(e >> Q.shift[k]);
    pay = (uint64_t)e;
    return true;
  }, [&](uint64_t e, uint32_t b, uint32_t o) { kidx[sub_off[b] + o] = (uint32_t)e; },
     ne, bcap, fill, pb_lds, pb_lds + bcap);
}

// one workgroup per key sub-bucket (<= 2^shift event indices, so it always fits LDS when the plan
// split it): its events in event order -> rank among earlier same-key events = slot - key start
__global__ __launch_bounds__(PB_T) void k_kb_rank(const int64_t* __restrict__ sub_off, const int32_t* __restrict__ sub_key,
                                                  const uint32_t* __restrict__ base, int nk, uint32_t* kidx,
                                                  uint32_t* ktmp, int64_t* __restrict__ ev_rank,
                                                  int64_t* __restrict__ ev_fkey) {
  __shared__ uint32_t lds[PB_KEY_CAP];
  const int b = blockIdx.x;
  if (b >= (int)base[nk]) return;
  const int64_t o = sub_off[b], m = sub_off[b + 1] - o;
  if (m == 0) return;
  const int k = sub_key[b];
  const int64_t r0 = o - sub_off[base[k]];
  const uint32_t* src = lds;
  if (m <= PB_KEY_CAP) {
    pb_sort_lds(kidx + o, (int)m, lds);
  } else {
    pb_sort_global<uint32_t, PB_KEY_CAP>(kidx + o, ktmp + o, m, lds);
    src = kidx + o;
  }
  for (int64_t j = threadIdx.x; j < m; j += blockDim.x) {
    const uint32_t e = src[j];
    ev_rank[e] = r0 + j;
    ev_fkey[e] = k;
  }
}

struct Carve {
  uint8_t* base;
  size_t used = 0;
  template <class T>
  T* take(size_t n) {
    const size_t off = (used + 255) & ~size_t(255);
    used = off + std::max<size_t>(n, 1) * sizeof(T);
    return base ? reinterpret_cast<T*>(base + off) : nullptr;
  }
};

size_t agg_lds(int nb, bool scatter) {
  return nb <= PB_LDS_BINS ? (size_t)(scatter ? 2 * nb : nb) * sizeof(uint32_t) : 0;
}

// sub-bucket capacity of a two-level plan: <= 1 per non-empty primary + 2 per PB_TARGET items
int64_t plan_cap(int64_t np, int64_t items) { return np + 2 * (items / PB_TARGET) + 2; }

}  // namespace

bool hits_bulk_ok(const HitsArgs& A) { return A.lbits <= 30 && A.R > 0; }


constexpr int64_t kFuseDedupeKeys = int64_t(1) << 16;
size_t hits_bulk_dev(const HitsArgs& A, void* ws, size_t ws_bytes, uint64_t stream) {
  const int64_t n = A.n;
  const int R = A.R;
  const int64_t L = int64_t(1) << A.lbits;          // line coordinate range (a power of two >= L)
  const int bcap = (int)plan_cap(R, n);
  Carve C{static_cast<uint8_t*>(ws)};
  // [regex counts | sub-bucket counts]: one memset
  uint32_t* cnt = C.take<uint32_t>(R);
  uint32_t* sub_cnt = C.take<uint32_t>(bcap);
  uint32_t* wide_cnt = C.take<uint32_t>(1);        // BPG wide-program list: count (zeroed), entries in tmp
  const size_t zero_end = C.used;
  uint8_t* shift = C.take<uint8_t>(R);
  uint32_t* base = C.take<uint32_t>(R + 1);
  int32_t* sub_reg = C.take<int32_t>(bcap);
  int64_t* sub_off = C.take<int64_t>(bcap + 1);
  uint32_t* vals = C.take<uint32_t>(n);
  uint32_t* tmp = C.take<uint32_t>(n);
  uint64_t* kout = C.take<uint64_t>(n);
  int64_t* stdk = C.take<int64_t>(n);
  uint8_t* flag = C.take<uint8_t>(n);
  uint32_t* kept = C.take<uint32_t>(bcap);
  int64_t* evs = C.take<int64_t>(bcap);
  int64_t* kept_off = C.take<int64_t>(bcap + 1);
  int64_t* ev_off = C.take<int64_t>(bcap + 1);
  if (!ws || C.used > ws_bytes) return C.used;
  hipStream_t st = pb_stream(stream);
  if (n == 0) {
    PB_CHECK(hipMemsetAsync(A.counters, 0, 2 * sizeof(int64_t), st));
    PB_CHECK(hipMemsetAsync(A.hit_off, 0, (size_t)(R + 1) * sizeof(int64_t), st));
    return C.used;
  }
  // whole 256-byte granules (the next carve starts on one): a tail that is not a multiple of 16
  // bytes makes the runtime split the fill into two kernels
  PB_CHECK(hipMemsetAsync(cnt, 0, (zero_end + 255) & ~size_t(255), st));
  const unsigned g = pb_agg_grid(n);
  const HbPlan Q{shift, base};
  hipLaunchKernelGGL(k_hb_count, dim3(g), dim3(PB_AT), agg_lds(R, false), st, A, cnt);
  PB_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_pb_plan, dim3(1), dim3(PB_AT), 0, st, cnt, R, A.lbits, L, nullptr, shift, base, sub_reg,
                     nullptr);
  PB_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_hb_count2, dim3(g), dim3(PB_AT), agg_lds(bcap, false), st, A, Q, bcap, sub_cnt);
  PB_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_pb_scan<uint32_t>, dim3(1), dim3(PB_AT), 0, st, sub_cnt, (int64_t)bcap, sub_off, nullptr, 1);
  PB_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_hb_scatter, dim3(g), dim3(PB_AT), agg_lds(bcap, true), st, A, Q, bcap, sub_off, sub_cnt, vals);
  PB_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_hb_sort, dim3((unsigned)bcap + pb_blocks(n, PB_PAD_SPAN)), dim3(PB_T), 0, st, sub_off, sub_reg,
                     base, R, bcap, vals, tmp, A.lbits, n, kout);
  PB_CHECK(hipGetLastError());
  // BPG programs: one lane per first-of-run key over the sorted keys (a regex's keys are contiguous,
  // so its waves are dense). A workgroup per sub-bucket (lanes looping over its candidates) measured
  // 138 us against this kernel's 118 us: the walks are latency-bound, lanes should not loop.
  // Up to kFuseDedupeKeys keys the DFA keys' dedupe-verify runs in the same launch (std_key): both
  // kernels are then tails of a few long walks, which overlap instead of adding up (config 2, 23k
  // keys: 26 + 49 -> 63 us, resident 0.519 -> 0.493 ms). With many keys the DFA walks need the
  // occupancy the BPG walk's 140 VGPRs take away (bench, ~180k keys: 48 + 62 -> 121 us): two launches.
  // (tmp: free after k_hb_sort)
  if (n > kFuseDedupeKeys) {
    dedupe_verify_dev(kout, n, A.lbits, A.text, A.ls, A.ll, A.dfa, stdk, flag, stream);
    bpg_dedupe_dev(kout, n, A.lbits, A.text, A.ls, A.ll, A.dfa, flag, stream, wide_cnt, tmp);
  } else if (!bpg_dedupe_dev(kout, n, A.lbits, A.text, A.ls, A.ll, A.dfa, flag, stream, wide_cnt, tmp, stdk)) {
    dedupe_verify_dev(kout, n, A.lbits, A.text, A.ls, A.ll, A.dfa, stdk, flag, stream);
  }
  hipLaunchKernelGGL(k_hb_kept, dim3((unsigned)bcap), dim3(PB_T), 0, st, sub_off, sub_reg, base, R, flag, stdk, A.ev,
                     kept, evs);
  PB_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_hb_offsets, dim3(1), dim3(PB_AT), 0, st, kept, evs, base, R, kept_off, ev_off, A.hit_off,
                     A.counters);
  PB_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_hb_emit, dim3((unsigned)bcap), dim3(PB_T), 0, st, sub_off, sub_reg, base, R, flag, stdk, A.ev,
                     kept_off, ev_off, A.hits, A.hit_line, A.ev_cnt, A.ev_end);
  PB_CHECK(hipGetLastError());
  return C.used;
}

bool events_bulk_ok(const EventsArgs& A) { return A.lbits <= 31; }

size_t events_bulk_dev(const EventsArgs& A, void* ws, size_t ws_bytes, uint64_t stream) {
  const int64_t ne = A.ne, L = A.L, nh = A.nh;
  const EvTables& E = A.ev;
  const int nk = E.nkeys;
  // line blocks of ~PB_EV_TARGET events each
  const int shift = std::max(0, A.lbits - bits_for(std::max<int64_t>(1, ne / PB_EV_TARGET)));
  const int nb = (int)((L >> shift) + 1);
  const int ebits = bits_for(std::max<int64_t>(ne, 1));
  const int kcap = (int)plan_cap(nk, ne);
  Carve C{static_cast<uint8_t*>(ws)};
  // [coverage | line-block counts | key counts | key sub-bucket counts]: one memset zeroes all
  int32_t* cov = A.cov ? A.cov : C.take<int32_t>(L);
  uint32_t* bin_cnt = C.take<uint32_t>(nb);
  uint32_t* key_cnt = C.take<uint32_t>(nk);
  uint32_t* ksub_cnt = C.take<uint32_t>(kcap);
  const size_t zero_end = C.used;
  int64_t* bin_off = C.take<int64_t>(nb + 1);
  uint8_t* kshift = C.take<uint8_t>(nk);
  uint32_t* kbase = C.take<uint32_t>(nk + 1);
  int32_t* sub_key = C.take<int32_t>(kcap);
  int64_t* ksub_off = C.take<int64_t>(kcap + 1);
  uint64_t* ekeys = C.take<uint64_t>(ne);
  uint64_t* etmp = C.take<uint64_t>(ne);
  uint32_t* fsort = C.take<uint32_t>(ne);
  uint32_t* kidx = C.take<uint32_t>(ne);
  uint32_t* ktmp = C.take<uint32_t>(ne);
  if (!ws || C.used > ws_bytes) return C.used;
  hipStream_t st = pb_stream(stream);
  uint8_t* zero_from = A.cov ? reinterpret_cast<uint8_t*>(bin_cnt) : reinterpret_cast<uint8_t*>(cov);
  PB_CHECK(hipMemsetAsync(zero_from, 0, static_cast<uint8_t*>(ws) + ((zero_end + 255) & ~size_t(255)) - zero_from, st));
  if (A.cov && L > 0) PB_CHECK(hipMemsetAsync(A.cov, 0, (size_t)L * sizeof(int32_t), st));
  // device-count mode (A.dcounts = [hits, events] on the device): nh / ne are capacities
  const int64_t* dc = A.dcounts;
  if (ne > 0) {
    const EbIn S{A.hits, A.ev_cnt, nh, shift, dc, ne};
    const unsigned g = pb_agg_grid(nh);
    hipLaunchKernelGGL(k_eb_count, dim3(g), dim3(PB_AT), agg_lds(nb, false), st, S, nb, bin_cnt, A.ne_fit);
    PB_CHECK(hipGetLastError());
    hipLaunchKernelGGL(k_pb_scan<uint32_t>, dim3(1), dim3(PB_AT), 0, st, bin_cnt, (int64_t)nb, bin_off, nullptr, 1);
    PB_CHECK(hipGetLastError());
    hipLaunchKernelGGL(k_eb_scatter, dim3(g), dim3(PB_AT), agg_lds(nb, true), st, S, nb, E, bin_off, bin_cnt, ekeys);
    PB_CHECK(hipGetLastError());
    hipLaunchKernelGGL(k_eb_sort, dim3((unsigned)nb), dim3(PB_T), 0, st, bin_off, ekeys, etmp, E, A.ev_line, A.ev_pat,
                       A.ev_seg, fsort, A.ev_rank, A.ev_fkey, cov, dc, ne);
    PB_CHECK(hipGetLastError());
    if (nk > 0) {
      const unsigned gk = pb_agg_grid(ne);
      const KbPlan Q{kshift, kbase};
      hipLaunchKernelGGL(k_kb_count, dim3(gk), dim3(PB_AT), agg_lds(nk, false), st, fsort, ne, nk, key_cnt, dc);
      PB_CHECK(hipGetLastError());
      hipLaunchKernelGGL(k_pb_plan, dim3(1), dim3(PB_AT), 0, st, key_cnt, nk, ebits, ne, dc ? dc + 1 : nullptr, kshift,
                         kbase, sub_key, A.freq_counts);
      PB_CHECK(hipGetLastError());
      hipLaunchKernelGGL(k_kb_count2, dim3(gk), dim3(PB_AT), agg_lds(kcap, false), st, fsort, ne, nk, Q, kcap, ksub_cnt,
                         dc);
      PB_CHECK(hipGetLastError());
      hipLaunchKernelGGL(k_pb_scan<uint32_t>, dim3(1), dim3(PB_AT), 0, st, ksub_cnt, (int64_t)kcap, ksub_off, nullptr, 1);
      PB_CHECK(hipGetLastError());
      hipLaunchKernelGGL(k_kb_scatter, dim3(gk), dim3(PB_AT), agg_lds(kcap, true), st, fsort, ne, nk, Q, kcap, ksub_off,
                         ksub_cnt, kidx, dc);
      PB_CHECK(hipGetLastError());
      hipLaunchKernelGGL(k_kb_rank, dim3((unsigned)kcap), dim3(PB_T), 0, st, ksub_off, sub_key, kbase, nk, kidx, ktmp,
                         A.ev_rank, A.ev_fkey);
      PB_CHECK(hipGetLastError());
    }
  } else {
    if (nk > 0) PB_CHECK(hipMemsetAsync(A.freq_counts, 0, (size_t)nk * sizeof(int64_t), st));
    if (A.ne_fit) PB_CHECK(hipMemsetAsync(A.ne_fit, 0, sizeof(int64_t), st));
  }
  if (A.feat && !A.feat_ready) feat_cov_dev(cov, L, A.text, A.ls, A.ll, A.dfa, A.ctx_trans, A.ctx_acc, A.feat, stream);
  return C.used;
}

}  // namespace lp
