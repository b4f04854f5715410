// Native request runner (see request.h).
#include "runtime/request.h"

#include <cstdio>

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <type_traits>

namespace lp {

namespace {

constexpr int64_t kNlTile = 16384;   // ops/kernels.py NL_TILE / TEXT_PAD
constexpr int64_t kTextPad = 64;
constexpr int kBlkShift = 12;        // LINE_BLK_SHIFT
constexpr size_t kFetchMaxBytes = size_t(4) << 20;   // k_fetch up to this upload size

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error in request runner (") + what + "): " + hipGetErrorString(e));
}

int64_t padded_len(int64_t n) { return ((std::max<int64_t>(n, 1) + kNlTile - 1) / kNlTile) * kNlTile + kTextPad; }

size_t up256(size_t n) { return (n + 255) & ~size_t(255); }

// pinned host memory kernels write into (k_publish): fine-grained, so the GPU's stores go to
// host memory and are visible once the stream has synchronised
constexpr unsigned kCoherentHost = hipHostMallocMapped | hipHostMallocCoherent;

// a device or pinned buffer that only grows (between runs, when nothing in flight uses it)
template <bool Pinned>
void grow(uint8_t*& p, size_t& cap, size_t need, unsigned host_flags = hipHostMallocDefault) {
  if (need <= cap) return;
  const size_t n = std::max(need + need / 4, size_t(1) << 20);
  if (p) check(Pinned ? hipHostFree(p) : hipFree(p), "free");
  p = nullptr;
  cap = 0;
  check(Pinned ? hipHostMalloc(reinterpret_cast<void**>(&p), n, host_flags)
               : hipMalloc(reinterpret_cast<void**>(&p), n), "alloc");
  cap = n;
}

template <typename T>
T* device_view(T* host) {
  void* d = nullptr;
  check(hipHostGetDevicePointer(&d, host, 0), "host device pointer");
  return static_cast<T*>(d);
}

}  // namespace

RequestRunner::RequestRunner(const RequestStatic& S) : S_(S) {
  check(hipSetDevice(S_.device), "set device");
  check(hipHostMalloc(reinterpret_cast<void**>(&cnt_host_), 8 * sizeof(int64_t), kCoherentHost), "pinned counters");
  cnt_host_dev_ = device_view(cnt_host_);
  // k_fetch reads the inputs from pinned memory (no SDMA copy) and k_publish writes the results
  // there (no copy back); the window eviction stays its own launch (inside k_fetch it showed an
  // unexplained engine p99 of 1.97 ms)
  publish_ = true;
  fetch_ = true;
  evict_in_fetch_ = false;
  side_on_ = true;   // (literal-free scans + context features beside the literal chain, r5_c)
  if (side_on_) {
    check(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking), "side stream");
    check(hipEventCreateWithFlags(&fork_, hipEventDisableTiming), "fork event");
    check(hipEventCreateWithFlags(&join_, hipEventDisableTiming), "join event");
  }
}

RequestRunner::~RequestRunner() {
  if (fork_) (void)hipEventDestroy(fork_);
  if (join_) (void)hipEventDestroy(join_);
  if (side_) (void)hipStreamDestroy(side_);
  if (carry_host_) (void)hipHostFree(carry_host_);
  if (ws_) (void)hipFree(ws_);
  if (post_ws_) (void)hipFree(post_ws_);
  if (up_host_) (void)hipHostFree(up_host_);
  if (inj_host_) (void)hipHostFree(inj_host_);
  if (res_host_) (void)hipHostFree(res_host_);
  if (cnt_host_) (void)hipHostFree(cnt_host_);
}

uint8_t* RequestRunner::dev(size_t bytes) {
  uint8_t* p = ws_ ? ws_ + ws_used_ : nullptr;
  ws_used_ += up256(bytes);
  return p;
}

int64_t RequestRunner::upload_bytes(int64_t nbytes, int64_t L, int D) const {
  const size_t seg_bytes = up256(4 * (size_t)D) * 2 + up256(8 * (size_t)D) * 2;
  const size_t L1 = (size_t)std::max<int64_t>(L, 1);
  const size_t n = up256((size_t)padded_len(nbytes)) + up256(8 * L1) + up256(4 * L1) + up256(seg_bytes) +
                   up256(8 * sizeof(int64_t)) + (size_t)std::max(S_.nseq, 1);
  return (int64_t)((n + 15) & ~size_t(15));
}

bool RequestRunner::map_fetch(uint8_t* host_text, int64_t host_cap) {
  if (host_text != fetch_host_ || host_cap != fetch_cap_) {
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, host_text, 0) != hipSuccess) {
      (void)hipGetLastError();
      d = nullptr;
    }
    fetch_host_ = host_text;
    fetch_cap_ = host_cap;
    fetch_dev_ = static_cast<uint8_t*>(d);
  }
  return fetch_dev_ != nullptr;
}

int64_t RequestRunner::prefetch_text(uint8_t* host_text, int64_t nbytes, int64_t host_cap, uint64_t stream) {
  pre_host_ = nullptr;
  pre_n_ = -1;
  pre_token_ = 0;
  const int64_t tsize = padded_len(nbytes);
  if (!fetch_ || !ws_ || (size_t)tsize > ws_cap_ || host_cap < tsize || (size_t)tsize > kFetchMaxBytes ||
      ((uintptr_t)host_text & 15) != 0)
    return 0;
  check(hipSetDevice(S_.device), "set device");
  if (!map_fetch(host_text, host_cap)) return 0;
  std::memset(host_text + nbytes, 0, (size_t)(tsize - nbytes));       // vector loads past the end
  fetch_dev(fetch_dev_, ws_, tsize / 16, stream, nullptr, 0.0);       // the text is the carve's first region
  pre_host_ = host_text;
  pre_n_ = nbytes;
  pre_ws_ = ws_;
  pre_token_ = ++pre_next_;
  return pre_token_;
}

int64_t RequestRunner::run(uint8_t* host_text, int64_t nbytes, const int64_t* starts, const int32_t* lens, int64_t L,
                           const int32_t* seg_lo, const int32_t* seg_hi, const int64_t* seg_g0, const int64_t* seg_n,
                           int D, const FreqRing& ring, double evict_before, double now, uint64_t stream,
                           int64_t host_cap, Turn* turn, int64_t seq, const int64_t* inj, int64_t ninj,
                           HostWindow* hw, int64_t pre_token) {
  if (hw && turn) throw std::invalid_argument("request runner: a host window or a turn, not both");
  // a shared window: released on every exit, also when a HIP call throws
  struct Release {
    Turn* t;
    int64_t s;
    ~Release() { if (t) t->done(s); }
  } release{turn, seq};
  recorded_ = false;
  check(hipSetDevice(S_.device), "set device");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t tsize = padded_len(nbytes);
  std::memset(host_text + nbytes, 0, (size_t)(tsize - nbytes));       // vector loads past the end
  const int64_t nblk = (std::max<int64_t>(nbytes, 1) >> kBlkShift) + 2;
  const int lbits = bits_for(std::max<int64_t>(L, 1)), rbits = bits_for(std::max(S_.R, 1));
  const int K1 = std::max(S_.nkeys, 1);
  const int64_t ecap_small = request_event_cap();

  // Inputs. Single-copy layout (when host_cap allows): the line index, the segments, zeroed
  // matcher counters and a zeroed sequence carry sit behind the padded text at the offsets the
  // workspace carve below gives them, so ONE H2D moves them all (each extra copy of a request
  // cost ~8 us of DMA setup plus ~8 us of queue gap, and the counter memset another fill).
  const int64_t L1 = std::max<int64_t>(L, 1);
  const size_t seg_bytes = up256(4 * (size_t)D) * 2 + up256(8 * (size_t)D) * 2;
  const size_t nseq1 = (size_t)std::max(S_.nseq, 1);
  const size_t o_ls = up256((size_t)tsize), o_ll = o_ls + up256(8 * (size_t)L1), o_seg = o_ll + up256(4 * (size_t)L1);
  const size_t o_cnt = o_seg + up256(seg_bytes), o_seq = o_cnt + up256(8 * sizeof(int64_t));
  const size_t up_total = (o_seq + nseq1 + 15) & ~size_t(15);     // whole 16-byte words
  const bool one_copy = host_cap >= (int64_t)up_total;
  // ... read by a kernel from the pinned buffer itself when the runtime maps it for the device
  const uint8_t* text_dev_src = nullptr;
  // (request-sized uploads only: a multi-MB batch moves faster on the SDMA engine, ~50 vs ~37 GB/s)
  if (one_copy && fetch_ && up_total <= kFetchMaxBytes && ((uintptr_t)host_text & 15) == 0) {
    map_fetch(host_text, host_cap);
    text_dev_src = fetch_dev_;
  }
  // the text already on its way (prefetch_text, same buffer and length): upload what follows it
  bool text_up = pre_token > 0 && pre_token == pre_token_ && pre_host_ == host_text && pre_n_ == nbytes;
  pre_host_ = nullptr;
  pre_n_ = -1;
  pre_token_ = 0;
  uint8_t* segh;
  if (one_copy) {
    if (L > 0) {
      std::memcpy(host_text + o_ls, starts, 8 * (size_t)L);
      std::memcpy(host_text + o_ll, lens, 4 * (size_t)L);
    }
    std::memset(host_text + o_cnt, 0, 8 * sizeof(int64_t));
    std::memset(host_text + o_seq, 0, nseq1);
    segh = host_text + o_seg;
  } else {
    grow<true>(up_host_, up_cap_, seg_bytes);
    segh = up_host_;
  }
  std::memcpy(segh, seg_lo, 4 * (size_t)D);
  std::memcpy(segh + up256(4 * (size_t)D), seg_hi, 4 * (size_t)D);
  std::memcpy(segh + 2 * up256(4 * (size_t)D), seg_g0, 8 * (size_t)D);
  std::memcpy(segh + 2 * up256(4 * (size_t)D) + up256(8 * (size_t)D), seg_n, 8 * (size_t)D);

  // window eviction first (FrequencyState.carry): the totals it leaves are this batch's carry --
  // inside the k_fetch launch when the inputs go up that way, else its own kernel
  const bool evict_in_fetch = turn == nullptr && hw == nullptr && text_dev_src != nullptr && evict_in_fetch_;
  if (!evict_in_fetch && turn == nullptr && hw == nullptr) freq_evict(ring, evict_before, stream, true);
  // shared window: wait for the earlier batches' records, then evict (this batch's carry)
  bool in_window = turn == nullptr;
  auto enter_window = [&]() {
    if (in_window) return;
    turn->wait(seq);
    freq_evict(ring, evict_before, stream, true);
    in_window = true;
  };

  // host window (several serving processes): the arrival ticket is drawn once everything that does
  // not read the window has FINISHED on the GPU; the section = host eviction + carry copy, the score
  // kernel on the pinned carry, the results to the host, the host record. Left on every exit.
  int64_t hw_seq = -1;
  double hw_now = now;
  struct Leave {
    HostWindow* w;
    int64_t* s;
    ~Leave() {             // (a destructor must not throw: a failing turn advance is reported)
      if (!w || *s < 0) return;
      try {
        w->leave(*s);
      } catch (const std::exception& e) {
        std::fprintf(stderr, "[lp] leaving the shared window section failed: %s\n", e.what());
      }
    }
  } leave_guard{hw, &hw_seq};
  const int K1w = std::max(S_.nkeys, 1);
  if (hw && !carry_host_) {
    check(hipHostMalloc(reinterpret_cast<void**>(&carry_host_), 8 * (size_t)K1w, kCoherentHost), "pinned carry");
    carry_dev_ = device_view(carry_host_);
  }
  auto hw_enter = [&]() {
    check(hipStreamSynchronize(st), "matching before the window section");
    hw_seq = hw->enter();
    hw_now = hw->evict_carry(now, carry_host_, K1w);
  };
  auto hw_leave = [&]() {
    if (hw_seq >= 0) {
      const int64_t q = hw_seq;
      hw_seq = -1;
      hw->leave(q);
    }
  };

  RequestCounts c;
  c.lines = L;
  int64_t ne = 0, nh = 0, stride = 0;
  uint8_t* text = nullptr;
  int32_t* blk = nullptr;
  int64_t *ls = nullptr, *hits = nullptr, *hit_off = nullptr, *ev_cnt = nullptr, *ev_end = nullptr, *cnt = nullptr;
  int64_t *gh = nullptr, *cand = nullptr, *ver = nullptr, *inj_dev = nullptr;
  int32_t *ll = nullptr, *hit_line = nullptr, *dlo = nullptr, *dhi = nullptr;
  int64_t *dg0 = nullptr, *dn = nullptr;
  // event-stage buffers (results layout: [score f64 x E | counts i64 x K1 | line | pattern | seg i32 x E])
  uint8_t *out = nullptr, *feat = nullptr, *seq_carry = nullptr;
  int64_t *ev_rank = nullptr, *ev_fkey = nullptr;
  EvTables ev = S_.ev;
  bool done = false;   // events + score already ran (device-count mode)
  bool feat_ready = false;   // every line's features computed on the side stream (this attempt)
  auto carve_events = [&](int64_t E) {
    out = dev(20 * (size_t)E + 8 * (size_t)K1);
    ev_rank = reinterpret_cast<int64_t*>(dev(8 * (size_t)std::max<int64_t>(E, 1)));
    ev_fkey = reinterpret_cast<int64_t*>(dev(8 * (size_t)std::max<int64_t>(E, 1)));
    feat = dev((size_t)std::max<int64_t>(L, 1));
  };
  // events, context features, frequency ranks into the results buffer, then (with_score) the fused
  // fp64 score; `dcnt` = device [nh, ne] (device-count mode, E = capacity) or null (E = ne read back)
  auto run_score = [&](int64_t E, const int64_t* dcnt, const int64_t* tot) {
    if (E <= 0) return;
    double* score = reinterpret_cast<double*>(out);
    int32_t* ev_line = reinterpret_cast<int32_t*>(out + 8 * (size_t)E + 8 * (size_t)K1);
    ScoreTables T = S_.st;
    T.seq_carry = seq_carry;
    T.hit_off = hit_off; T.hit_line = hit_line; T.feat = feat;
    T.seg_lo = dlo; T.seg_hi = dhi; T.seg_own_lo = dlo; T.seg_g0 = dg0; T.seg_n = dn;
    const FreqIn F{ev_rank, ev_fkey, tot};
    score_dev(ev_line, ev_line + E, ev_line + 2 * E, F, E, T, S_.sp, score, nullptr, stream, dcnt ? dcnt + 1 : nullptr);
  };
  auto run_events = [&](int64_t E, int64_t nh_cap, const int64_t* dcnt, bool with_score) {
    double* score = reinterpret_cast<double*>(out);
    int64_t* freq_counts = reinterpret_cast<int64_t*>(out + 8 * (size_t)E);
    int32_t* ev_line = reinterpret_cast<int32_t*>(out + 8 * (size_t)E + 8 * (size_t)K1);
    int32_t* ev_pat = ev_line + E;
    int32_t* ev_seg = ev_pat + E;
    if (S_.nkeys == 0) check(hipMemsetAsync(freq_counts, 0, 8, st), "counts");
    if (L == 0) check(hipMemsetAsync(feat, 0, 1, st), "feat");
    if (!one_copy) check(hipMemsetAsync(seq_carry, 0, nseq1, st), "seq carry");
    EventsArgs A;
    A.ctx_trans = S_.ctx_trans; A.ctx_acc = S_.ctx_acc;
    A.hits = (nh_cap || dcnt) ? hits : nullptr; A.nh = nh_cap; A.ev_cnt = ev_cnt; A.ev_end = ev_end; A.ne = E; A.L = L;
    A.lbits = lbits; A.ev = ev; A.text = text; A.ls = ls; A.ll = ll; A.dfa = S_.dfa;
    A.ev_line = ev_line; A.ev_pat = ev_pat; A.ev_seg = ev_seg; A.ev_rank = ev_rank; A.ev_fkey = ev_fkey;
    A.freq_counts = freq_counts; A.feat = feat; A.cov = nullptr; A.dcounts = dcnt;
    A.feat_ready = feat_ready;
    const size_t need = events_dev(A, post_ws_, post_cap_, stream);
    if (need > post_cap_) {
      if (dcnt) throw std::runtime_error("request runner: event workspace not pre-sized");
      grow<false>(post_ws_, post_cap_, need);   // the stream is idle since the counter read
      events_dev(A, post_ws_, post_cap_, stream);
    }
    (void)score; (void)ev_pat; (void)ev_seg;
    if (with_score) run_score(E, dcnt, ring.tot);
    return freq_counts;
  };

  for (int attempt = 0;; ++attempt) {
    const int64_t cap_g = (int64_t)((double)L * rate_gram_ * 1.25) + 512;
    const int64_t cap_c = (int64_t)((double)L * rate_cand_ * 1.25) + 512;
    const int64_t cap_v = (int64_t)((double)L * rate_ver_ * 1.25) + 512 + ninj;
    const int64_t n = cap_c + cap_v;
    // device-count mode: a request on the single-workgroup paths runs matching, CSR, events,
    // score and the (gated) frequency record without the mid-batch host read
    const bool fast = S_.device_counts && attempt == 0 && n <= ecap_small && L <= request_line_cap();
    for (int pass = 0; pass < 2; ++pass) {   // measure, then carve from a workspace large enough
      ws_used_ = 0;
      // carve order == the single-copy host layout (o_ls .. o_seq above)
      text = dev((size_t)tsize);
      ls = reinterpret_cast<int64_t*>(dev(8 * (size_t)L1));
      ll = reinterpret_cast<int32_t*>(dev(4 * (size_t)L1));
      uint8_t* segs = dev(seg_bytes);
      dlo = reinterpret_cast<int32_t*>(segs);
      dhi = reinterpret_cast<int32_t*>(segs + up256(4 * (size_t)D));
      dg0 = reinterpret_cast<int64_t*>(segs + 2 * up256(4 * (size_t)D));
      dn = reinterpret_cast<int64_t*>(segs + 2 * up256(4 * (size_t)D) + up256(8 * (size_t)D));
      cnt = reinterpret_cast<int64_t*>(dev(8 * sizeof(int64_t)));
      seq_carry = dev(nseq1);
      if (ws_ && (size_t)(seq_carry - text) != o_seq) throw std::runtime_error("request runner: upload layout mismatch");
      blk = reinterpret_cast<int32_t*>(dev(4 * (size_t)nblk));
      gh = reinterpret_cast<int64_t*>(dev(8 * (size_t)cap_g));
      cand = reinterpret_cast<int64_t*>(dev(8 * (size_t)cap_c));
      ver = reinterpret_cast<int64_t*>(dev(8 * (size_t)cap_v));
      hits = reinterpret_cast<int64_t*>(dev(8 * (size_t)n));
      hit_line = reinterpret_cast<int32_t*>(dev(4 * (size_t)n));
      hit_off = reinterpret_cast<int64_t*>(dev(8 * (size_t)(S_.R + 1)));
      ev_cnt = reinterpret_cast<int64_t*>(dev(8 * (size_t)n));
      ev_end = reinterpret_cast<int64_t*>(dev(8 * (size_t)n));
      inj_dev = ninj > 0 ? reinterpret_cast<int64_t*>(dev(8 * (size_t)ninj)) : nullptr;
      if (fast) carve_events(ecap_small);
      if (pass == 0 && ws_used_ > ws_cap_) {   // nothing in flight uses the workspace here
        check(hipStreamSynchronize(st), "sync before growth");
        grow<false>(ws_, ws_cap_, ws_used_);
      }
    }
    if (fast && post_cap_ < 4 * (size_t)std::max<int64_t>(L, 1) + 4096) {   // events' coverage array
      check(hipStreamSynchronize(st), "sync before growth");
      grow<false>(post_ws_, post_cap_, 4 * (size_t)std::max<int64_t>(L, 1) + 4096);
    }
    // inputs: packed text, line index, segments (all pinned -> async)
    if (text_up && (ws_ != pre_ws_ || text != ws_)) text_up = false;   // (the workspace moved: all again)
    if (one_copy && text_dev_src && text_up && attempt == 0) {
      const size_t o_rest = o_ls;                // 256-aligned: the index, segments, counters, carry
      fetch_dev(text_dev_src + o_rest, text + o_rest, (int64_t)((up_total - o_rest) / 16), stream,
                evict_in_fetch ? &ring : nullptr, evict_before);
    } else if (one_copy && text_dev_src) {   // (a re-run's eviction is a no-op: the window's head moved)
      fetch_dev(text_dev_src, text, (int64_t)(up_total / 16), stream, attempt == 0 && evict_in_fetch ? &ring : nullptr,
                evict_before);
    } else if (one_copy) {
      check(hipMemcpyAsync(text, host_text, up_total, hipMemcpyHostToDevice, st), "inputs H2D");
    } else {
      check(hipMemcpyAsync(text, host_text, (size_t)tsize, hipMemcpyHostToDevice, st), "text H2D");
      if (L > 0) {
        check(hipMemcpyAsync(ls, starts, 8 * (size_t)L, hipMemcpyHostToDevice, st), "starts H2D");
        check(hipMemcpyAsync(ll, lens, 4 * (size_t)L, hipMemcpyHostToDevice, st), "lens H2D");
      }
      check(hipMemcpyAsync(dlo, up_host_, seg_bytes, hipMemcpyHostToDevice, st), "segments H2D");
      check(hipMemsetAsync(cnt, 0, 8 * sizeof(int64_t), st), "counters");
    }
    ev.seg_lo = dlo;
    ev.seg_hi = dhi;
    ev.own_lo = dlo;
    ev.own_hi = dhi;
    ev.nseg = D;
    unsigned long long* c0 = reinterpret_cast<unsigned long long*>(cnt);

    // matchers: literal-free scan groups and single-DFA scans (on the side stream when there is
    // one: they overlap the literal chain and the candidate verification), then the literal
    // prefilter chain
    // fast (request-sized) batches also compute every line's context features there, so the event
    // stage needs no feature pass (k_feat_cov over the covered lines sat on the critical path)
    const bool side = side_on_ && (!S_.scans.empty() || S_.n_scan_regs || (fast && L > 0));
    const bool feat_side = side && fast && L > 0;
    const uint64_t sst = side ? reinterpret_cast<uint64_t>(side_) : stream;
    if (side) {
      check(hipEventRecord(fork_, st), "fork");
      check(hipStreamWaitEvent(side_, fork_, 0), "fork wait");
    }
    for (size_t i = 0; i < S_.scans.size(); ++i)
      scan_multi_dev(text, nbytes, ls, ll, L, S_.scans[i], ver, cap_v, c0 + 2, S_.scan_grids[i], sst);
    if (S_.n_scan_regs)
      scan_dev(text, ls, ll, L, S_.scan_regs, S_.n_scan_regs, S_.dfa, ver, cap_v, c0 + 2, sst);
    if (feat_side) feat_all_dev(L, text, ls, ll, S_.dfa, S_.ctx_trans, S_.ctx_acc, feat, sst);
    if (side) check(hipEventRecord(join_, side_), "join");
    blk_index_dev(ls, L, nblk, blk, stream);
    prefilter_dev(text, nbytes, S_.pf, ls, L, gh, cap_g, c0, S_.pf_grid, stream);
    pf_verify_dev(gh, cap_g, text, nbytes, S_.pf, ls, L, blk, cand, cap_c, c0 + 1, stream, c0,
                  (int)std::max<int64_t>(16, std::min<int64_t>(8192, nbytes >> 13)));
    // the prefilter candidates' verification does not read the scans' buffer: it runs before the join
    bool verified = false;
    if (side && fast && n <= request_event_cap())
      verified = cand_verify_all_dev(cand, cap_c, reinterpret_cast<unsigned long long*>(c0 + 1), text, ls, ll, S_.dfa,
                                     stream);
    if (side) check(hipStreamWaitEvent(st, join_, 0), "join wait");
    feat_ready = feat_side;

    if (S_.host_dev)   // the relaxed automata's keys: candidates only, decided by the host side path
      take_host_dev(cand, c0 + 1, cap_c, ver, c0 + 2, cap_v, text, ls, ll, S_.dfa, HostSideOut{}, stream);
    // the backtracker regexes' host-verified hits (Engine.host_hits), pre-verified: appended AFTER
    // the relaxed keys are dropped (the drop clears every key of a device-fed regex)
    if (ninj > 0) {
      if (attempt == 0) {
        grow<true>(inj_host_, inj_cap_, 8 * (size_t)ninj);
        std::memcpy(inj_host_, inj, 8 * (size_t)ninj);
      }
      check(hipMemcpyAsync(inj_dev, inj_host_, 8 * (size_t)ninj, hipMemcpyHostToDevice, st), "host hits H2D");
      append_keys_dev(ver, cap_v, c0 + 2, inj_dev, ninj, stream);
    }
    // hit CSR + event counts: the pipeline reads the matchers' device counters itself
    HitsArgs A;
    A.cand = cand; A.n = n; A.pre_from = cap_c;
    A.cand2 = ver; A.dcount = c0 + 1;
    A.lbits = lbits; A.rbits = rbits; A.R = S_.R;
    A.text = text; A.ls = ls; A.ll = ll; A.dfa = S_.dfa; A.ev = ev;
    A.hits = hits; A.hit_line = hit_line; A.hit_off = hit_off; A.ev_cnt = ev_cnt; A.ev_end = ev_end;
    A.counters = cnt + 3;
    A.cand_verified = verified;
    // the request's whole tail (hits, events, score, record, publish) as ONE single-workgroup kernel:
    // the device-count fast path with its own window, the candidates verified and every line's
    // features computed before the join
    const bool tail = fast && !hw && publish_ && verified && feat_ready && L > 0;
    if (tail) {
      enter_window();
      const int64_t E = ecap_small;
      double* score = reinterpret_cast<double*>(out);
      int64_t* freq_counts = reinterpret_cast<int64_t*>(out + 8 * (size_t)E);
      int32_t* ev_line = reinterpret_cast<int32_t*>(out + 8 * (size_t)E + 8 * (size_t)K1);
      if (S_.nkeys == 0) check(hipMemsetAsync(freq_counts, 0, 8, st), "counts");
      if (!one_copy) check(hipMemsetAsync(seq_carry, 0, nseq1, st), "seq carry");
      EventsArgs EA;
      EA.ctx_trans = S_.ctx_trans; EA.ctx_acc = S_.ctx_acc;
      EA.hits = hits; EA.nh = n; EA.ev_cnt = ev_cnt; EA.ev_end = ev_end; EA.ne = E; EA.L = L;
      EA.lbits = lbits; EA.ev = ev; EA.text = text; EA.ls = ls; EA.ll = ll; EA.dfa = S_.dfa;
      EA.ev_line = ev_line; EA.ev_pat = ev_line + E; EA.ev_seg = ev_line + 2 * E; EA.ev_rank = ev_rank;
      EA.ev_fkey = ev_fkey; EA.freq_counts = freq_counts; EA.feat = feat; EA.cov = nullptr; EA.dcounts = cnt + 3;
      EA.feat_ready = true;
      ScoreTables T = S_.st;
      T.seq_carry = seq_carry;
      T.hit_off = hit_off; T.hit_line = hit_line; T.feat = feat;
      T.seg_lo = dlo; T.seg_hi = dhi; T.seg_own_lo = dlo; T.seg_g0 = dg0; T.seg_n = dn;
      const FreqIn F{ev_rank, ev_fkey, ring.tot};
      const size_t res = 20 * (size_t)E + 8 * (size_t)K1;
      if (res > res_cap_) {
        grow<true>(res_host_, res_cap_, res, kCoherentHost);
        res_host_dev_ = device_view(res_host_);
      }
      RequestTailOut P;
      P.score = score; P.out = out; P.E = E; P.K1 = (int)K1; P.cnt = cnt;
      P.cnt_host = cnt_host_dev_; P.res_host = res_host_dev_;
      P.counts = freq_counts; P.K = S_.nkeys; P.now = now; P.ring = ring;
      P.gate.cnt = cnt;
      P.gate.cap[0] = cap_g; P.gate.cap[1] = cap_c; P.gate.cap[2] = cap_v; P.gate.cap[3] = E;
      request_tail_dev(A, EA, T, S_.sp, F, P, post_ws_, post_cap_, stream);
      recorded_ = true;            // (gated on the device: an overflowing attempt records nothing)
    } else {
    size_t need = hits_dev(A, post_ws_, post_cap_, stream);
    if (need > post_cap_) {       // post_ws_ is not used by anything in flight yet
      if (fast) throw std::runtime_error("request runner: hit workspace on the small path");
      check(hipStreamSynchronize(st), "sync before growth");
      grow<false>(post_ws_, post_cap_, need);
      hits_dev(A, post_ws_, post_cap_, stream);
    }
    }
    if (tail) {
    } else if (fast && hw) {
      run_events(ecap_small, n, cnt + 3, false);
      hw_enter();
      run_score(ecap_small, cnt + 3, carry_dev_);
      const size_t res = 20 * (size_t)ecap_small + 8 * (size_t)K1;
      if (res > res_cap_) {
        grow<true>(res_host_, res_cap_, res, kCoherentHost);
        res_host_dev_ = device_view(res_host_);
      }
      publish_dev(cnt, out, ecap_small, (int)K1, cnt_host_dev_, res_host_dev_, stream);   // recorded on the host
    } else if (fast) {
      enter_window();
      int64_t* fc = run_events(ecap_small, n, cnt + 3, true);
      RecordGate G;
      G.cnt = cnt;
      G.cap[0] = cap_g; G.cap[1] = cap_c; G.cap[2] = cap_v; G.cap[3] = ecap_small;
      if (S_.nkeys > 0 && !publish_) freq_record(fc, S_.nkeys, now, ring, stream, true, G);
      recorded_ = true;            // (gated on the device: an overflowing attempt records nothing)
      const size_t res = 20 * (size_t)ecap_small + 8 * (size_t)K1;
      if (res > res_cap_) {
        grow<true>(res_host_, res_cap_, res, kCoherentHost);
        res_host_dev_ = device_view(res_host_);
      }
      if (publish_) {      // frequency record + counters + compacted results in host memory: one kernel
        publish_record_dev(cnt, out, ecap_small, (int)K1, cnt_host_dev_, res_host_dev_, fc, S_.nkeys, now, ring, G,
                           stream);
      } else {
        check(hipMemcpyAsync(res_host_, out, res, hipMemcpyDeviceToHost, st), "results D2H");
        res_bytes_ = res;
      }
    }
    if (!(fast && (publish_ || hw)) && !tail)
      check(hipMemcpyAsync(cnt_host_, cnt, 5 * sizeof(int64_t), hipMemcpyDeviceToHost, st), "counters D2H");
    check(hipStreamSynchronize(st), "counters");   // fast: the only host read; else the mid-batch one
    c.gram = cnt_host_[0]; c.cand = cnt_host_[1]; c.ver = cnt_host_[2];
    nh = cnt_host_[3]; ne = cnt_host_[4];
    c.hits = nh; c.events = ne;
    const bool ok = c.gram <= cap_g && c.cand <= cap_c && c.ver <= cap_v;
    // MatchArena.learn: overflow -> the exact rates; otherwise decay toward what batches need
    auto learn = [&](double& rate, int64_t v) {
      const double r = (double)v / (double)std::max<int64_t>(L, 1);
      rate = std::max(std::max(r, ok ? rate * 0.5 : rate), 1e-4);
    };
    learn(rate_gram_, c.gram);
    learn(rate_cand_, c.cand);
    learn(rate_ver_, c.ver);
    if (fast) recorded_ = false;             // the gate held: nothing was recorded on this attempt
    if (ok && fast && ne <= ecap_small) {    // recorded through the gate; results already read
      if (hw) {                              // the host record of the section (compacted results)
        if (S_.nkeys > 0) hw->record_batch(reinterpret_cast<const int64_t*>(res_host_ + 8 * (size_t)ne), S_.nkeys, hw_now);
        hw_leave();
      }
      recorded_ = true;
      done = true;
      stride = (publish_ || hw) ? ne : ecap_small;
      if (publish_ || hw) res_bytes_ = 20 * (size_t)ne + 8 * (size_t)K1;
      break;
    }
    hw_leave();                              // an overflowing attempt records nothing: next ticket
    if (ok && !fast) break;
    if (attempt > 8) throw std::runtime_error("request runner: matcher capacities did not converge");
  }

  if (!done) {
    // host-count mode: event buffers sized by the counts just read
    const size_t res = 20 * (size_t)ne + 8 * (size_t)K1;
    const size_t ws2 = up256(res) + 2 * up256(8 * (size_t)std::max<int64_t>(ne, 1)) +
                       up256((size_t)std::max<int64_t>(L, 1)) + up256((size_t)std::max(S_.nseq, 1));
    const size_t base = ws_used_;
    if (base + ws2 > ws_cap_) {
      // the workspace must grow while the inputs / CSR it holds are still needed: move them. The
      // stream is idle (counter read above), so copy the used prefix into the new allocation.
      uint8_t* old = ws_;
      uint8_t* nw = nullptr;
      const size_t ncap = std::max((base + ws2) * 5 / 4, size_t(1) << 20);
      check(hipMalloc(reinterpret_cast<void**>(&nw), ncap), "alloc");
      check(hipMemcpyAsync(nw, old, base, hipMemcpyDeviceToDevice, st), "workspace move");
      check(hipStreamSynchronize(st), "workspace move");
      check(hipFree(old), "free");
      const ptrdiff_t d = nw - old;
      auto mv = [&](auto*& q) { q = reinterpret_cast<std::remove_reference_t<decltype(q)>>(reinterpret_cast<uint8_t*>(q) + d); };
      mv(text); mv(ls); mv(ll); mv(dlo); mv(dhi); mv(dg0); mv(dn); mv(hits); mv(hit_line); mv(hit_off); mv(ev_cnt); mv(ev_end); mv(seq_carry);
      ev.seg_lo = dlo; ev.seg_hi = dhi; ev.own_lo = dlo; ev.own_hi = dhi;
      ws_ = nw;
      ws_cap_ = ncap;
    }
    ws_used_ = base;
    carve_events(ne);
    int64_t* fc;
    if (hw) {
      fc = run_events(ne, nh, nullptr, false);
      hw_enter();
      run_score(ne, nullptr, carry_dev_);
    } else {
      enter_window();
      fc = run_events(ne, nh, nullptr, true);
      // this batch's per-key counts enter the window (after its own scoring: penalty before record)
      if (S_.nkeys > 0) freq_record(fc, S_.nkeys, now, ring, stream, true);
      recorded_ = true;
    }
    if (res > res_cap_) {
      grow<true>(res_host_, res_cap_, res, kCoherentHost);
      res_host_dev_ = device_view(res_host_);
    }
    check(hipMemcpyAsync(res_host_, out, res, hipMemcpyDeviceToHost, st), "results D2H");
    check(hipStreamSynchronize(st), "results");
    if (hw) {
      if (S_.nkeys > 0) hw->record_batch(reinterpret_cast<const int64_t*>(res_host_ + 8 * (size_t)ne), S_.nkeys, hw_now);
      hw_leave();
      recorded_ = true;
    }
    (void)fc;
    res_bytes_ = res;
    stride = ne;
  }
  stride_ = stride;
  counts_ = c;
  return ne;
}

}  // namespace lp
