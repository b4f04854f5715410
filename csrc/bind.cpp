// Python bindings (pybind11) for the native parts of log_parser_amd:
//   * the Java-regex compiler (csrc/regex)
//   * gfx950 kernel launchers and their host twins (csrc/kernels)
//   * host line splitter for request batches and the JSON result emitter (csrc/io)
// Tensors cross the boundary as raw pointers (torch .data_ptr()) plus the HIP stream handle, so
// the module does not depend on libtorch headers and compiles in seconds.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>

#include "io/docs.h"
#include "io/json_in.h"
#include "io/loadgen.h"
#include "io/http_server.h"
#include "io/json_emit.h"
#include "kernels/lp_api.h"
#include "kernels/lp_host.h"
#include "regex/jregex.h"
#include "runtime/proc_shared.h"
#include "runtime/request.h"

namespace py = pybind11;
using namespace lp;

template <typename T>
static T* P(uint64_t v) { return reinterpret_cast<T*>(v); }

static PfTables pf_from(const py::tuple& t) {
  PfTables T;
  T.bloom = P<const uint32_t>(t[0].cast<uint64_t>());
  T.bloom_bits = t[1].cast<int>();
  T.ht_key = P<const uint64_t>(t[2].cast<uint64_t>());
  T.ht_val = P<const int32_t>(t[3].cast<uint64_t>());
  T.ht_cnt = P<const int32_t>(t[4].cast<uint64_t>());
  T.ht_mask = t[5].cast<uint32_t>();
  T.gram_lits = P<const int32_t>(t[6].cast<uint64_t>());
  T.lit_off = P<const int32_t>(t[7].cast<uint64_t>());
  T.lit_bytes = P<const uint8_t>(t[8].cast<uint64_t>());
  T.lit_reg_off = P<const int32_t>(t[9].cast<uint64_t>());
  T.lit_reg = P<const int32_t>(t[10].cast<uint64_t>());
  T.gmask = t[11].cast<int>();
  T.stride = t[12].cast<int>();
  T.teddy = P<const uint32_t>(t[13].cast<uint64_t>());
  T.tb_off = P<const int32_t>(t[14].cast<uint64_t>());
  T.tb_lits = P<const int32_t>(t[15].cast<uint64_t>());
  T.teddy_on = t[16].cast<int>();
  if (t.size() > 18) {
    T.gram_fp = P<const uint64_t>(t[17].cast<uint64_t>());
    T.tb_fp = P<const uint64_t>(t[18].cast<uint64_t>());
  }
  return T;
}

static DfaPool dfa_from(const py::tuple& t) {
  DfaPool D;
  D.meta = P<const int32_t>(t[0].cast<uint64_t>());
  D.bytemap = P<const uint8_t>(t[1].cast<uint64_t>());
  D.trans = P<const uint16_t>(t[2].cast<uint64_t>());
  D.acc = P<const uint8_t>(t[3].cast<uint64_t>());
  D.bpg = t.size() > 4 ? P<const uint64_t>(t[4].cast<uint64_t>()) : nullptr;
  D.bpg_widths = t.size() > 5 ? t[5].cast<uint32_t>() : 0u;
  D.bpg_words = t.size() > 6 ? t[6].cast<uint32_t>() : 0u;
  return D;
}

static ScoreTables st_from(const py::tuple& t) {
  ScoreTables T;
  int i = 0;
  auto nx = [&]() { return t[i++].cast<uint64_t>(); };
  T.conf = P<const double>(nx()); T.sev = P<const double>(nx());
  T.ctx_before = P<const int32_t>(nx()); T.ctx_after = P<const int32_t>(nx());
  T.sec_off = P<const int32_t>(nx()); T.sec_reg = P<const int32_t>(nx()); T.sec_w = P<const int32_t>(nx());
  T.sec_weight = P<const double>(nx());
  T.seq_off = P<const int32_t>(nx()); T.seq_bonus = P<const double>(nx()); T.seq_ev_off = P<const int32_t>(nx());
  T.seq_ev_reg = P<const int32_t>(nx()); T.seq_carry = P<const uint8_t>(nx());
  T.hit_off = P<const int64_t>(nx()); T.hit_line = P<const int32_t>(nx()); T.feat = P<const uint8_t>(nx());
  T.seg_lo = P<const int32_t>(nx()); T.seg_hi = P<const int32_t>(nx()); T.seg_own_lo = P<const int32_t>(nx());
  T.seg_g0 = P<const int64_t>(nx()); T.seg_n = P<const int64_t>(nx());
  return T;
}

static ScoreParams sp_from(const py::tuple& t) {
  ScoreParams S;
  S.decay = t[0].cast<double>(); S.early = t[1].cast<double>(); S.maxearly = t[2].cast<double>();
  S.penalty = t[3].cast<double>(); S.max_ctx = t[4].cast<double>(); S.fthr = t[5].cast<double>();
  S.fmaxp = t[6].cast<double>(); S.fwin = t[7].cast<double>();
  return S;
}

// (prim_off, prim_pats, freq_key, ctx_before, ctx_after, seg_lo, seg_hi, own_lo, own_hi, nseg, nkeys, pbits)
static EvTables ev_from(const py::tuple& t) {
  EvTables E;
  E.prim_off = P<const int64_t>(t[0].cast<uint64_t>());
  E.prim_pats = P<const int32_t>(t[1].cast<uint64_t>());
  E.freq_key = P<const int32_t>(t[2].cast<uint64_t>());
  E.ctx_before = P<const int32_t>(t[3].cast<uint64_t>());
  E.ctx_after = P<const int32_t>(t[4].cast<uint64_t>());
  E.seg_lo = P<const int32_t>(t[5].cast<uint64_t>());
  E.seg_hi = P<const int32_t>(t[6].cast<uint64_t>());
  E.own_lo = P<const int32_t>(t[7].cast<uint64_t>());
  E.own_hi = P<const int32_t>(t[8].cast<uint64_t>());
  E.nseg = t[9].cast<int>();
  E.nkeys = t[10].cast<int>();
  E.pbits = t[11].cast<int>();
  return E;
}

// (blob ptr, lds_words, ngroups, row_base, stride, thr, init_row, init_state, ncol, gt_off, fin_off
//  [each a 4-tuple], bm_off, rid_off, am_off, gm_off [4-tuple])
static ScanPass scan_pass_from(const py::tuple& t) {
  ScanPass S;
  S.blob = P<const uint32_t>(t[0].cast<uint64_t>());
  S.lds_words = t[1].cast<int>();
  S.ngroups = t[2].cast<int>();
  auto q = [&](int i, int g) { return t[i].cast<py::tuple>()[g].cast<int64_t>(); };
  for (int g = 0; g < 4; ++g) {
    S.row_base[g] = (int)q(3, g);
    S.stride[g] = (int)q(4, g);
    S.thr[g] = (int)q(5, g);
    S.init_row[g] = (int)q(6, g);
    S.init_state[g] = (uint32_t)q(7, g);
    S.ncol[g] = (int)q(8, g);
    S.gt_off[g] = (int)q(9, g);
    S.fin_off[g] = (int)q(10, g);
  }
  S.bm_off = t[11].cast<int>();
  S.rid_off = t[12].cast<int>();
  S.am_off = t[13].cast<int>();
  for (int g = 0; g < 4; ++g) S.gm_off[g] = (int)q(14, g);
  return S;
}

// (t, key, cnt, cap, ht, tot, seen)
static FreqRing ring_from(const py::tuple& t) {
  FreqRing R;
  R.t = P<double>(t[0].cast<uint64_t>());
  R.key = P<int32_t>(t[1].cast<uint64_t>());
  R.cnt = P<int32_t>(t[2].cast<uint64_t>());
  R.cap = t[3].cast<int64_t>();
  R.ht = P<int64_t>(t[4].cast<uint64_t>());
  R.tot = P<int64_t>(t[5].cast<uint64_t>());
  R.seen = P<uint8_t>(t[6].cast<uint64_t>());
  return R;
}

// Java-semantics backtracking matchers of a library's non-automaton regexes (host fallback)
struct BtSet {
  std::vector<std::unique_ptr<BtRegex>> rx;
  std::vector<std::string> err;
  std::atomic<int64_t> exhausted{0};
  explicit BtSet(const std::vector<std::string>& pats) {
    for (auto& p : pats) {
      try {
        rx.emplace_back(new BtRegex(p));
        err.emplace_back();
      } catch (const std::exception& e) {
        rx.emplace_back(nullptr);
        err.emplace_back(e.what());
      }
    }
  }
  bool find(int i, const uint8_t* s, int64_t n) {
    if (i < 0 || i >= (int)rx.size() || !rx[i]) return false;
    bool ex = false;
    const bool m = rx[i]->find(s, n, int64_t(1) << 27, &ex);
    if (ex) exhausted++;
    return m;
  }
};

// The host half of the device-fed backtracker regexes (side_path.hip) as a native thread: no
// Python and no GIL between an export and the answer. A job has up to two export regions, each
// published by its own k_take_host (count, then the job's sequence number): A = the prefilter's
// candidates, exported as soon as the literal chain is done -- the host verifies them while the
// GPU is still in the literal-free scan -- and B = the scan engines' keys of relaxed regexes,
// exported after the scan. The worker polls each region's sequence word in pinned memory, checks
// the candidate lines with the backtracker on the batch's host bytes, and publishes (verified keys
// of both regions, their count or -1, then the sequence) for k_wait_host. Layouts (int64 words):
// region = keys | starts | lens | count | seq (cap entries each); inb = keys | count | seq.
class SideWorker {
 public:
  SideWorker(BtSet& bt, std::vector<int32_t> local) : bt_(bt), local_(std::move(local)) {
    th_ = std::thread([this] { loop(); });
  }
  ~SideWorker() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  // outB = 0: one region
  void submit(int64_t seq, uint64_t text, int64_t cap, uint64_t outA, uint64_t outB, uint64_t inb) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      q_.push_back(Job{seq, reinterpret_cast<const uint8_t*>(text), cap, {reinterpret_cast<int64_t*>(outA),
                       reinterpret_cast<int64_t*>(outB)}, reinterpret_cast<int64_t*>(inb)});
    }
    cv_.notify_one();
  }
  int64_t need() const { return need_.load(); }
  void clear_need() { need_.store(0); }
  std::string take_error() {
    std::lock_guard<std::mutex> lk(mu_);
    std::string e;
    e.swap(error_);
    return e;
  }
  int64_t done() const { return done_.load(); }

 private:
  struct Job {
    int64_t seq;
    const uint8_t* text;
    int64_t cap;
    int64_t* out[2];
    int64_t* inb;
  };
  static int64_t load_acq(const int64_t* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
  void fail(const std::string& why) {
    std::lock_guard<std::mutex> lk(mu_);
    if (error_.empty()) error_ = why;
  }
  // verify region `out` (n <= cap keys) into inb[base..]; returns the verified count
  int64_t verify(const Job& j, const int64_t* out, int64_t n, int64_t base) {
    const int64_t c = j.cap;
    const int64_t* K = out;
    const int64_t* S = out + c;
    const int64_t* L = out + 2 * c;
    const int64_t ng = (int64_t)local_.size();
    std::vector<uint8_t> ok(n, 0);
    host_parallel(n, 16, [&](int, int64_t a, int64_t e) {
      for (int64_t i = a; i < e; ++i) {
        const int64_t g = K[i] >> 32;
        if (g < 0 || g >= ng || local_[g] < 0) continue;
        ok[i] = bt_.find(local_[g], j.text + S[i], L[i]) ? 1 : 0;
      }
    });
    int64_t r = 0;
    for (int64_t i = 0; i < n; ++i)
      if (ok[i]) {
        if (base + r < c) j.inb[base + r] = K[i];
        ++r;
      }
    return r;
  }
  // the job's next region to verify: whichever published export comes first (the scan engines'
  // region B is exported as soon as the scans end, often before the literal chain's region A);
  // -1 when none arrives within 5 s
  int next_region(const Job& j, bool (&seen)[2]) {
    // spin (pause) for the first 50 ms: the exports come ~1-2 ms into a step, and a sleeping
    // poll wakes up to ~60 us late (timer slack) -- each late wake-up sat on the GPU's k_wait_host
    const int64_t c = j.cap;
    const auto t0 = std::chrono::steady_clock::now();
    for (int it = 0;; ++it) {
      for (int q = 0; q < 2; ++q)
        if (!seen[q] && j.out[q] && load_acq(j.out[q] + 3 * c + 1) == j.seq) return q;
      const auto dt = std::chrono::steady_clock::now() - t0;
      if (dt < std::chrono::milliseconds(50)) {
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
        continue;
      }
      if (dt > std::chrono::seconds(5)) return -1;
      std::this_thread::sleep_for(std::chrono::microseconds(10));
    }
  }
  void run(const Job& j) {
    const int64_t c = j.cap;
    int64_t res = 0;
    bool seen[2] = {j.out[0] == nullptr, j.out[1] == nullptr};
    for (int k = 0; k < 2 && res >= 0; ++k) {
      if (seen[0] && seen[1]) break;
      const int q = next_region(j, seen);
      if (q < 0) {
        fail("side path: no export for batch " + std::to_string(j.seq) + " within 5 s");
        res = -1;
        break;
      }
      seen[q] = true;
      const int64_t* out = j.out[q];
      const int64_t n = load_acq(out + 3 * c);
      if (n > c) {                           // re-run with a larger buffer (the batch overflows)
        need_.store(std::max(need_.load(), n));
        res = -1;
        break;
      }
      res += verify(j, out, n, res);
      if (res > c) {
        need_.store(std::max(need_.load(), res));
        res = -1;
      }
    }
    __atomic_store_n(j.inb + c, res, __ATOMIC_RELEASE);
    __atomic_store_n(j.inb + c + 1, j.seq, __ATOMIC_RELEASE);   // published last
    done_++;
  }
  void loop() {
    for (;;) {
      Job j;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        j = q_.front();
        q_.pop_front();
      }
      try {
        run(j);
      } catch (const std::exception& e) {
        fail(e.what());
        __atomic_store_n(j.inb + j.cap, (int64_t)-1, __ATOMIC_RELEASE);
        __atomic_store_n(j.inb + j.cap + 1, j.seq, __ATOMIC_RELEASE);
        done_++;
      }
    }
  }
  BtSet& bt_;
  std::vector<int32_t> local_;
  std::thread th_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Job> q_;
  bool stop_ = false;
  std::atomic<int64_t> need_{0}, done_{0};
  std::string error_;
};

// Java String.split("\\r?\\n") line index of ONE document (trim: drop trailing empty lines, as
// split(regex) does; the device line index of a batch / shard uses the same rule)
static void host_line_index(const uint8_t* t, int64_t n, bool trim, std::vector<int64_t>& ls, std::vector<int32_t>& ll) {
  const int T = std::max(1, std::min<int>(host_threads(), (int)(n >> 22) + 1));
  std::vector<std::vector<int64_t>> nl(T);
  host_parallel(n, int64_t(1) << 22, [&](int th, int64_t a, int64_t e) {
    for (const uint8_t* p = t + a; p < t + e;) {
      const void* q = std::memchr(p, '\n', (size_t)(t + e - p));
      if (!q) break;
      nl[th].push_back(static_cast<const uint8_t*>(q) - t);
      p = static_cast<const uint8_t*>(q) + 1;
    }
  });
  std::vector<int64_t> pos;
  for (auto& v : nl) pos.insert(pos.end(), v.begin(), v.end());
  std::sort(pos.begin(), pos.end());
  ls.clear();
  ll.clear();
  int64_t st = 0;
  for (int64_t q : pos) {
    const int64_t e = (q > st && t[q - 1] == '\r') ? q - 1 : q;
    ls.push_back(st);
    ll.push_back((int32_t)(e - st));
    st = q + 1;
  }
  if (st < n || pos.empty()) { ls.push_back(st); ll.push_back((int32_t)(n - st)); }
  if (trim)
    while (ls.size() > (pos.empty() ? 1u : 0u) && ll.back() == 0) { ls.pop_back(); ll.pop_back(); }
}

// Host side path of the backtracker regexes (non-regular: backreferences, lookaround, atomic
// groups, possessive quantifiers), run BEFORE the device pipeline so their hits join it as
// pre-verified keys (append_keys_dev) and no host round trip sits in the middle of a batch:
// lines holding one of a regex's required literals (ASCII case-insensitive, as the device
// prefilter) -- or every line for a literal-free one -- are checked with BtRegex, in parallel.
static py::array_t<int64_t> bt_prepass(BtSet& b, uint64_t text, int64_t nbytes, uint64_t lsp, uint64_t llp, int64_t nlines,
                                       bool trim, const std::vector<int>& locals, const std::vector<int64_t>& globals,
                                       const std::vector<std::vector<std::string>>& lits) {
  const uint8_t* t = P<const uint8_t>(text);
  std::vector<int64_t> ls_own;
  std::vector<int32_t> ll_own;
  const int64_t* ls = P<const int64_t>(lsp);
  const int32_t* ll = P<const int32_t>(llp);
  std::vector<int64_t> keys;
  {
    py::gil_scoped_release nogil;
    if (!ls) {
      host_line_index(t, nbytes, trim, ls_own, ll_own);
      ls = ls_own.data();
      ll = ll_own.data();
      nlines = (int64_t)ls_own.size();
    }
    uint8_t low[256];
    for (int c = 0; c < 256; ++c) low[c] = (uint8_t)((c >= 'A' && c <= 'Z') ? c + 32 : c);
    // candidate (regex slot, line) pairs
    std::vector<std::vector<std::pair<int, int64_t>>> part(std::max(1, host_threads()));
    std::vector<int> scan_all;
    for (size_t k = 0; k < locals.size(); ++k) {
      if (lits[k].empty()) { scan_all.push_back((int)k); continue; }
      for (const std::string& lit : lits[k]) {
        const int64_t m = (int64_t)lit.size();
        if (m == 0 || m > nbytes) continue;
        const uint8_t* L = reinterpret_cast<const uint8_t*>(lit.data());
        host_parallel(nbytes - m + 1, int64_t(1) << 20, [&](int th, int64_t a, int64_t e) {
          for (int64_t i = a; i < e; ++i) {
            if (low[t[i]] != L[0]) continue;
            int64_t j = 1;
            while (j < m && low[t[i + j]] == L[j]) ++j;
            if (j < m) continue;
            const int64_t x = std::upper_bound(ls, ls + nlines, i) - ls - 1;
            if (x >= 0 && i + m <= ls[x] + ll[x]) part[th].push_back({(int)k, x});
          }
        });
      }
    }
    std::vector<std::pair<int, int64_t>> cand;
    for (auto& v : part) cand.insert(cand.end(), v.begin(), v.end());
    std::sort(cand.begin(), cand.end());
    cand.erase(std::unique(cand.begin(), cand.end()), cand.end());
    std::vector<uint8_t> ok(cand.size(), 0);
    host_parallel((int64_t)cand.size(), 64, [&](int, int64_t a, int64_t e) {
      for (int64_t i = a; i < e; ++i) {
        const int64_t x = cand[i].second;
        ok[i] = b.find(locals[cand[i].first], t + ls[x], ll[x]) ? 1 : 0;
      }
    });
    for (size_t i = 0; i < cand.size(); ++i)
      if (ok[i]) keys.push_back((globals[cand[i].first] << 32) | cand[i].second);
    if (!scan_all.empty()) {
      std::vector<std::vector<int64_t>> sk(std::max(1, host_threads()));
      host_parallel(nlines, 256, [&](int th, int64_t a, int64_t e) {
        for (int64_t x = a; x < e; ++x)
          for (int k : scan_all)
            if (b.find(locals[k], t + ls[x], ll[x])) sk[th].push_back((globals[k] << 32) | x);
      });
      for (auto& v : sk) keys.insert(keys.end(), v.begin(), v.end());
    }
  }
  py::array_t<int64_t> r((py::ssize_t)keys.size());
  if (!keys.empty()) std::memcpy(r.mutable_data(), keys.data(), keys.size() * 8);
  return r;
}

static py::bytes vbytes(const void* p, size_t n) { return py::bytes(static_cast<const char*>(p), n); }

// byte-level NFA conditions for the MFMA group builder (models/nfa.py, nfa_mfma.hip), which use
// the 15 byte-level contexts prev * 5 + next (prev < 3, next < 5) of the jregex 24-context masks
static uint32_t legacy_cond(uint32_t c) {
  uint32_t o = 0;
  for (int p = 0; p < 3; ++p)
    for (int n = 0; n < 5; ++n)
      if ((c >> ctx_index(p, n)) & 1u) o |= 1u << (p * 5 + n);
  return o;
}

static py::dict compile_regex(const std::string& pat, int max_states, int max_positions) {
  Compiled c = compile(pat, max_states, max_positions);
  py::dict d;
  d["kind"] = (int)c.kind;
  d["error"] = c.error;
  py::list lits;
  for (auto& s : c.literals) lits.append(py::bytes(s));
  d["literals"] = lits;
  d["has_literals"] = c.has_literals;
  d["bt_ok"] = c.bt_ok;
  d["cp_only"] = c.cp_only;
  d["uword"] = c.uword;
  d["bpg"] = vbytes(c.bpg.data(), c.bpg.size() * 8);
  if (c.kind == Kind::DFA) {
    d["nstates"] = c.dfa.nstates;
    d["nclasses"] = c.dfa.nclasses;
    d["bytemap"] = vbytes(c.dfa.bytemap.data(), c.dfa.bytemap.size());
    d["trans"] = vbytes(c.dfa.trans.data(), c.dfa.trans.size() * 2);
    d["acc"] = vbytes(c.dfa.accflags.data(), c.dfa.accflags.size());
    d["anchored"] = c.dfa.anchored;
  }
  d["npos"] = c.byte_nfa ? c.nfa.npos : 0;   // byte-level NFA (0 also: none -- code-point contexts, too large)
  if ((c.kind == Kind::DFA || c.kind == Kind::NFA) && c.byte_nfa) {
    std::string cls;
    for (auto& b : c.nfa.cls) cls.append(reinterpret_cast<const char*>(b.w), 32);
    d["nfa_cls"] = py::bytes(cls);
    py::list first, last, follow;
    for (auto& e : c.nfa.first) first.append(py::make_tuple(e.to, legacy_cond(e.cond)));
    for (auto& e : c.nfa.last) last.append(py::make_tuple(e.to, legacy_cond(e.cond)));
    for (auto& v : c.nfa.follow) {
      py::list l;
      for (auto& e : v) l.append(py::make_tuple(e.to, legacy_cond(e.cond)));
      follow.append(l);
    }
    d["nfa_first"] = first;
    d["nfa_last"] = last;
    d["nfa_follow"] = follow;
    d["nfa_nullable"] = legacy_cond(c.nfa.nullable);
  }
  return d;
}

static bool dfa_find_py(const std::string& pat, const std::string& line, int max_states) {
  Compiled c = compile(pat, max_states, 4096);
  if (c.kind != Kind::DFA) throw std::runtime_error("not a DFA regex: " + c.error);
  return dfa_find(c.dfa, reinterpret_cast<const uint8_t*>(line.data()), (int64_t)line.size());
}

// Split each document of a concatenated buffer with Java String.split("\\r?\\n") semantics.
// Returns (line_start int64[L], line_len int32[L], doc_line_off int64[D+1]).
static py::tuple split_docs(uint64_t buf, py::array_t<int64_t> doc_off) {
  const uint8_t* b = P<const uint8_t>(buf);
  auto off = doc_off.unchecked<1>();
  const int64_t D = off.shape(0) - 1;
  std::vector<int64_t> st;
  std::vector<int32_t> ln;
  std::vector<int64_t> dl(D + 1, 0);
  for (int64_t d = 0; d < D; ++d) {
    const int64_t s0 = off(d), s1 = off(d + 1);
    const size_t first = st.size();
    int64_t start = s0;
    bool any = false;
    for (;;) {
      const void* q = memchr(b + start, '\n', (size_t)(s1 - start));
      if (!q) break;
      any = true;
      int64_t nl = static_cast<const uint8_t*>(q) - b;
      int64_t end = nl;
      if (end > start && b[end - 1] == '\r') --end;
      st.push_back(start);
      ln.push_back((int32_t)(end - start));
      start = nl + 1;
    }
    st.push_back(start);
    ln.push_back((int32_t)(s1 - start));
    if (any) {
      while (st.size() > first && ln.back() == 0) { st.pop_back(); ln.pop_back(); }
    }
    dl[d + 1] = (int64_t)st.size();
  }
  py::array_t<int64_t> a(st.size());
  py::array_t<int32_t> l(ln.size());
  py::array_t<int64_t> o(dl.size());
  if (!st.empty()) { memcpy(a.mutable_data(), st.data(), st.size() * 8); memcpy(l.mutable_data(), ln.data(), ln.size() * 4); }
  memcpy(o.mutable_data(), dl.data(), dl.size() * 8);
  return py::make_tuple(a, l, o);
}

// A drained POST /parse whose `logs` string is still JSON-escaped inside its receive buffer
// (HttpServer.next_requests(raw=True)). pack_split_docs unescapes it straight into the engine's
// pinned stage -- one pass over the bytes instead of unescape-to-bytes + copy-to-stage -- and the
// buffer goes back to the server's pool when the object dies.
struct RawLogs {
  std::string body;
  size_t off = 0, len = 0;
  size_t dlen = 0;            // decoded length (0: unknown, decode serially)
  std::shared_ptr<BufferPool> pool;
  DecodeBuf dec;              // dec.p: already decoded by the IO thread (dlen bytes): plain text
  std::shared_ptr<DecodePool> dpool;
  RawLogs() = default;
  RawLogs(const RawLogs&) = delete;
  RawLogs& operator=(const RawLogs&) = delete;
  ~RawLogs() {
    if (pool) pool->give(std::move(body));
    if (dpool && dec.p) dpool->give(std::move(dec));
  }
  const uint8_t* data() const { return reinterpret_cast<const uint8_t*>(body.data()) + off; }
  bool decoded() const { return dec.p != nullptr; }
};

static py::bytes raw_logs_decode(const RawLogs& r) {
  if (r.decoded()) return py::bytes(r.dec.p, r.dlen);
  PyObject* b = PyBytes_FromStringAndSize(nullptr, (Py_ssize_t)(r.len + 64));
  if (!b) throw py::error_already_set();
  size_t n;
  {
    py::gil_scoped_release nogil;
    n = decode_json_string(r.data(), r.len, PyBytes_AS_STRING(b));
  }
  if (_PyBytes_Resize(&b, (Py_ssize_t)n) != 0) throw py::error_already_set();
  return py::reinterpret_steal<py::bytes>(b);
}

// Pack request bodies (str via their cached UTF-8 buffer -- no copy for ASCII -- or bytes) into
// dst and split them. Returns None if a str is not UTF-8 encodable (lone surrogates: the caller
// falls back to str.encode(surrogatepass)), the needed byte count (int) if it exceeds cap, or
// (line_start, line_len, doc_line_off, doc_off); with an index buffer `idx` (int64[idx_cap] starts
// then int32[idx_cap] lengths) that holds every line: (L, None, doc_line_off, doc_off).
static py::object pack_split_docs_py(py::list docs, uint64_t dst, int64_t cap, int nthreads, uint64_t idx,
                                     int64_t idx_cap) {
  const int64_t D = (int64_t)docs.size();
  std::vector<const char*> src(D);
  std::vector<int64_t> off(D + 1, 0);
  bool raw = D > 0;
  for (int64_t i = 0; i < D && raw; ++i) raw = py::isinstance<RawLogs>(docs[i]);
  // every body decoded by the IO threads already: plain text sources, packed like bytes (one
  // copy + newline scan pass into the stage, no unescape on this thread)
  bool predecoded = raw;
  for (int64_t i = 0; i < D && predecoded; ++i) predecoded = docs[i].cast<const RawLogs&>().decoded();
  // ... whose decoder recorded the newline positions: no newline scan either
  std::vector<const int64_t*> nlp;
  std::vector<int64_t> nlc;
  if (predecoded) {
    nlp.assign(D, nullptr);
    nlc.assign(D, 0);
    for (int64_t i = 0; i < D; ++i) {
      const RawLogs& r = docs[i].cast<const RawLogs&>();
      src[i] = r.dec.p;
      off[i + 1] = off[i] + (int64_t)r.dlen;
      if (r.dec.has_nl) {
        nlp[i] = r.dec.nl.p ? r.dec.nl.p.get() : reinterpret_cast<const int64_t*>(&nlc[i]);   // (non-null: none)
        nlc[i] = (int64_t)r.dec.nl.n;
      }
    }
    raw = false;
  }
  if (raw) {
    // escaped length bounds the decoded one; the decoder may write 64 bytes past its output
    std::vector<const RawLogs*> rl(D);
    int64_t bound = 64;
    bool known = true;                 // decoded lengths counted by the front end's validation
    for (int64_t i = 0; i < D; ++i) {
      rl[i] = &docs[i].cast<const RawLogs&>();
      bound += (int64_t)rl[i]->len;
      known = known && (rl[i]->dlen > 0 || rl[i]->len == 0);
    }
    if (bound > cap) return py::int_(bound);
    {
      py::gil_scoped_release nogil;
      uint8_t* d = P<uint8_t>(dst);
      if (known) {
        // every document's output offset is known: decode them side by side (exact-bounds
        // decoder: no store past a document's end) -- one thread decoded a 1 GB burst serially
        for (int64_t i = 0; i < D; ++i) off[i + 1] = off[i] + (int64_t)rl[i]->dlen;
        std::atomic<bool> bad{false};
        HostPool::get().run(D, std::max(1, nthreads), [&](int64_t i) {
          if (rl[i]->decoded()) {             // (a mix: this one was decoded by the IO thread)
            std::memcpy(d + off[i], rl[i]->dec.p, rl[i]->dlen);
            return;
          }
          const size_t k = rl[i]->len ? decode_json_string_exact(rl[i]->data(), rl[i]->len,
                                                                 reinterpret_cast<char*>(d + off[i]))
                                      : 0;
          if (k != rl[i]->dlen) bad = true;
        });
        if (bad) known = false;          // (never: the same grammar counted them) -- redo serially
      }
      if (!known) {
        for (int64_t i = 0; i < D; ++i) {
          if (rl[i]->decoded()) {
            std::memcpy(d + off[i], rl[i]->dec.p, rl[i]->dlen);
            off[i + 1] = off[i] + (int64_t)rl[i]->dlen;
            continue;
          }
          off[i + 1] = off[i] + (int64_t)decode_json_string(rl[i]->data(), rl[i]->len, reinterpret_cast<char*>(d + off[i]));
        }
      }
      for (int64_t i = 0; i < D; ++i) src[i] = reinterpret_cast<const char*>(d + off[i]);   // split in place
    }
  }
  for (int64_t i = 0; i < D && !raw && !predecoded; ++i) {
    PyObject* o = docs[i].ptr();
    Py_ssize_t n = 0;
    const char* p = nullptr;
    if (PyUnicode_Check(o)) {
      p = PyUnicode_AsUTF8AndSize(o, &n);
      if (!p) {
        PyErr_Clear();
        return py::none();
      }
    } else if (PyBytes_Check(o)) {
      char* q = nullptr;
      PyBytes_AsStringAndSize(o, &q, &n);
      p = q;
    } else {
      throw std::invalid_argument("pack_split_docs: str or bytes expected");
    }
    src[i] = p;
    off[i + 1] = off[i] + (int64_t)n;
  }
  if (off[D] > cap) return py::int_(off[D]);
  DocBatchIndex ix;
  if (idx && idx_cap > 0) {          // line_start int64[idx_cap] then line_len int32[idx_cap]
    ix.ext_start = P<int64_t>(idx);
    ix.ext_len = reinterpret_cast<int32_t*>(P<int64_t>(idx) + idx_cap);
    ix.ext_cap = idx_cap;
  }
  {
    py::gil_scoped_release nogil;   // `docs` keeps every buffer alive
    pack_split_docs(src.data(), off.data(), D, P<uint8_t>(dst), nthreads, ix, int64_t(4) << 20,
                    nlp.empty() ? nullptr : nlp.data(), nlc.empty() ? nullptr : nlc.data());
  }
  // hand the native buffers to numpy (capsule owns them): no copy of the line index
  auto own = [](auto& buf) {
    using T = std::remove_reference_t<decltype(buf[0])>;
    const size_t n = buf.size();
    T* ptr = buf.release();
    py::capsule cap(ptr, [](void* q) { delete[] static_cast<T*>(q); });
    return py::array_t<T>({(py::ssize_t)n}, {(py::ssize_t)sizeof(T)}, ptr, cap);
  };
  const int64_t L = ix.doc_line_off[D];
  py::array_t<int64_t> o = own(ix.doc_line_off);
  py::array_t<int64_t> d(off.size());
  memcpy(d.mutable_data(), off.data(), off.size() * 8);
  if (ix.external) return py::make_tuple(py::int_(L), py::none(), o, d);   // index is in `idx`
  py::array_t<int64_t> a = own(ix.line_start);
  py::array_t<int32_t> l = own(ix.line_len);
  return py::make_tuple(a, l, o, d);
}

// POST /parse body -> (status, pod_nonnull, pod_name | None, logs_kind, logs bytes | None);
// status: 0 ok, 1 invalid JSON, 2 JSON but not an object, 3 fall back to json.loads
static py::tuple parse_pod_request_py(py::bytes body, bool two_pass, bool into) {
  char* p = nullptr;
  Py_ssize_t n = 0;
  PyBytes_AsStringAndSize(body.ptr(), &p, &n);
  PodRequest r;
  int st;
  {
    py::gil_scoped_release nogil;
    if (into) {     // what the HTTP front end's IO thread does: validate + decode into its buffer
      std::unique_ptr<char[]> dst(new char[(size_t)n + 64]);
      st = parse_pod_request_into(reinterpret_cast<const uint8_t*>(p), (size_t)n, r, dst.get(), (size_t)n + 64);
      if (st == JIN_OK && r.logs_kind == 1) {
        if (!r.logs_decoded) throw std::runtime_error("parse_pod_request_into: logs string not decoded");
        r.logs.assign(dst.get(), r.logs_dlen);
      }
    } else {
    // two_pass: what the HTTP front end did before -- validate, then unescape the recorded span
    st = parse_pod_request(reinterpret_cast<const uint8_t*>(p), (size_t)n, r, !two_pass);
    }
    if (!into && two_pass && st == JIN_OK && r.logs_kind == 1) {
      r.logs.resize(r.logs_len + 64);
      r.logs.resize(decode_json_string(reinterpret_cast<const uint8_t*>(p) + r.logs_off, r.logs_len, &r.logs[0]));
    }
  }
  py::object name = r.has_name ? py::object(py::str(r.pod_name)) : py::object(py::none());
  py::object logs = r.logs_kind == 1 ? py::object(py::bytes(r.logs)) : py::object(py::none());
  return py::make_tuple(st, r.pod_nonnull, name, r.logs_kind, logs);
}

// The front end's arrival path on one body: logs_prefetch after each prefix length in `cuts`
// (as the IO thread runs it between reads), then the final parse resuming the prefetch.
// -> (status, pod_nonnull, pod_name | None, logs_kind, logs bytes | None, prefetch state, prefetched
// escaped bytes, the decoder's '\n' positions) -- equal to parse_pod_request(body, into=True) in the
// first five fields
static py::tuple parse_pod_request_stream_py(py::bytes body, std::vector<size_t> cuts) {
  char* p = nullptr;
  Py_ssize_t n = 0;
  PyBytes_AsStringAndSize(body.ptr(), &p, &n);
  PodRequest r;
  LogsPrefetch pf;
  NlPos nl;
  int st;
  {
    py::gil_scoped_release nogil;
    // each prefix is its own allocation: nothing past the arrived bytes is readable
    std::unique_ptr<char[]> dst(new char[(size_t)n + 64]);
    for (size_t c : cuts) {
      c = std::min(c, (size_t)n);
      std::unique_ptr<uint8_t[]> pre(new uint8_t[std::max<size_t>(c, 1)]);
      std::memcpy(pre.get(), p, c);
      logs_prefetch(pre.get(), c, pf, dst.get(), (size_t)n + 64, &nl);
    }
    st = parse_pod_request_into(reinterpret_cast<const uint8_t*>(p), (size_t)n, r, dst.get(), (size_t)n + 64, &pf,
                                &nl);
    if (st == JIN_OK && r.logs_kind == 1) {
      if (!r.logs_decoded) throw std::runtime_error("parse_pod_request_into: logs string not decoded");
      r.logs.assign(dst.get(), r.logs_dlen);
    }
  }
  py::object name = r.has_name ? py::object(py::str(r.pod_name)) : py::object(py::none());
  py::object logs = r.logs_kind == 1 ? py::object(py::bytes(r.logs)) : py::object(py::none());
  std::vector<int64_t> nlv(nl.p.get(), nl.p.get() + (st == JIN_OK && r.logs_kind == 1 ? nl.n : 0));
  return py::make_tuple(st, r.pod_nonnull, name, r.logs_kind, logs, pf.state,
                        pf.state >= 1 ? pf.src - pf.s0 : (size_t)0, nlv);
}

// ---- DLPack (v0.8 ABI, unversioned "dltensor" capsule) ---------------------------------------
namespace dl {
struct Device { int32_t device_type; int32_t device_id; };
struct DataType { uint8_t code; uint8_t bits; uint16_t lanes; };
struct Tensor { void* data; Device device; int32_t ndim; DataType dtype; int64_t* shape; int64_t* strides;
                uint64_t byte_offset; };
struct Managed { Tensor t; void* ctx; void (*deleter)(Managed*); };
constexpr int32_t kCPU = 1, kROCM = 10;
struct Holder { Managed m; int64_t shape[1]; };
void free_managed(Managed* m) { delete reinterpret_cast<Holder*>(m); }
}  // namespace dl

// device < 0: host memory. The memory itself is not owned (the shared window keeps it mapped).
static py::capsule dlpack_capsule(uint64_t ptr, int64_t numel, const std::string& dtype, int device) {
  auto* h = new dl::Holder();
  dl::DataType t{};
  if (dtype == "float64") t = {2, 64, 1};
  else if (dtype == "int64") t = {0, 64, 1};
  else if (dtype == "int32") t = {0, 32, 1};
  else if (dtype == "uint8") t = {1, 8, 1};
  else { delete h; throw std::invalid_argument("dlpack: unsupported dtype " + dtype); }
  h->shape[0] = numel;
  h->m.t = dl::Tensor{reinterpret_cast<void*>(ptr), {device < 0 ? dl::kCPU : dl::kROCM, device < 0 ? 0 : device},
                      1, t, h->shape, nullptr, 0};
  h->m.ctx = nullptr;
  h->m.deleter = dl::free_managed;
  return py::capsule(&h->m, "dltensor", [](PyObject* cap) {
    // consumed capsules are renamed "used_dltensor": the consumer then owns the deleter call
    if (PyCapsule_IsValid(cap, "dltensor")) {
      auto* m = static_cast<dl::Managed*>(PyCapsule_GetPointer(cap, "dltensor"));
      if (m && m->deleter) m->deleter(m);
    }
  });
}

PYBIND11_MODULE(_lpnative, m) {
  m.doc() = "log_parser_amd native core: Java-regex compiler, gfx950 kernels, host twins, JSON emitter";
  m.def("compile_multi", [](const std::vector<std::string>& pats, int max_states) -> py::object {
    MultiDfa d;
    try {
      d = compile_multi(pats, max_states);
    } catch (const Unsupported&) {
      return py::none();
    }
    py::dict r;
    r["nstates"] = d.nstates;
    r["nclasses"] = d.nclasses;
    r["nregs"] = d.nregs;
    r["bytemap"] = vbytes(d.bytemap.data(), d.bytemap.size());
    r["trans"] = vbytes(d.trans.data(), d.trans.size() * 4);
    r["acc"] = vbytes(d.acc.data(), d.acc.size() * 8);     // uint64 masks
    r["fin"] = vbytes(d.fin.data(), d.fin.size() * 8);
    return r;
  }, py::arg("patterns"), py::arg("max_states") = 4096);
  m.def("multi_find", [](const std::vector<std::string>& pats, const std::string& line) -> py::object {
    MultiDfa d;
    try {
      d = compile_multi(pats, 1 << 16);
    } catch (const Unsupported&) {
      return py::object(py::int_(-1));
    }
    return py::object(py::int_(multi_find(d, reinterpret_cast<const uint8_t*>(line.data()), (int64_t)line.size())));
  });
  py::class_<SideWorker>(m, "SideWorker")
      .def(py::init<BtSet&, std::vector<int32_t>>(), py::keep_alive<1, 2>(), py::arg("bt"), py::arg("local"))
      .def("submit", &SideWorker::submit, py::arg("seq"), py::arg("text"), py::arg("cap"), py::arg("out_a"),
           py::arg("out_b"), py::arg("inb"))
      .def_property_readonly("need", &SideWorker::need)
      .def("clear_need", &SideWorker::clear_need)
      .def("take_error", &SideWorker::take_error)
      .def_property_readonly("done", &SideWorker::done);
  py::class_<BtSet>(m, "BtSet")
      .def(py::init<const std::vector<std::string>&>())
      .def("ok", [](const BtSet& b, int i) { return i >= 0 && i < (int)b.rx.size() && b.rx[i] != nullptr; })
      .def("error", [](const BtSet& b, int i) { return b.err.at(i); })
      .def_property_readonly("exhausted", [](const BtSet& b) { return (int64_t)b.exhausted.load(); })
      .def("find", [](BtSet& b, int i, const std::string& line) {
        return b.find(i, reinterpret_cast<const uint8_t*>(line.data()), (int64_t)line.size());
      })
      // candidates (global regex << 32 | line) with each candidate line's [start, start + len)
      // in `text` -> the ones whose regex finds a match there; local[g] = index of global regex g
      // in this set (-1: not ours, dropped)
      .def("verify", [](BtSet& b, uint64_t text, uint64_t keys, uint64_t starts, uint64_t lens, int64_t nkeys,
                        uint64_t local, int64_t nglobal, uint64_t out) -> int64_t {
        const uint8_t* t = P<const uint8_t>(text);
        const int64_t* K = P<const int64_t>(keys);
        const int64_t* S = P<const int64_t>(starts);
        const int64_t* L = P<const int64_t>(lens);
        const int32_t* loc = P<const int32_t>(local);
        std::vector<uint8_t> ok(nkeys, 0);
        {
          py::gil_scoped_release nogil;
          host_parallel(nkeys, 64, [&](int, int64_t a, int64_t e) {
            for (int64_t i = a; i < e; ++i) {
              const int64_t g = K[i] >> 32;
              if (g < 0 || g >= nglobal || loc[g] < 0) continue;
              ok[i] = b.find(loc[g], t + S[i], L[i]) ? 1 : 0;
            }
          });
        }
        int64_t c = 0;
        int64_t* o = P<int64_t>(out);
        for (int64_t i = 0; i < nkeys; ++i)
          if (ok[i]) o[c++] = K[i];
        return c;
      })
      .def("prepass", &bt_prepass, py::arg("text"), py::arg("nbytes"), py::arg("ls"), py::arg("ll"),
           py::arg("nlines"), py::arg("trim"), py::arg("locals"), py::arg("globals"), py::arg("literals"))
      // every line x every listed regex (fallback regexes without a usable literal)
      .def("scan", [](BtSet& b, uint64_t text, uint64_t ls, uint64_t ll, int64_t nlines, std::vector<int> locals,
                      std::vector<int64_t> globals) -> py::array_t<int64_t> {
        const uint8_t* t = P<const uint8_t>(text);
        const int64_t* L = P<const int64_t>(ls);
        const int32_t* N_ = P<const int32_t>(ll);
        std::vector<std::vector<int64_t>> part(std::max(1, host_threads()));
        {
          py::gil_scoped_release nogil;
          host_parallel(nlines, 256, [&](int th, int64_t a, int64_t e) {
            for (int64_t x = a; x < e; ++x)
              for (size_t k = 0; k < locals.size(); ++k)
                if (b.find(locals[k], t + L[x], N_[x])) part[th].push_back((globals[k] << 32) | x);
          });
        }
        size_t n = 0;
        for (auto& v : part) n += v.size();
        py::array_t<int64_t> r(n);
        int64_t* o = r.mutable_data();
        for (auto& v : part) for (int64_t k : v) *o++ = k;
        return r;
      });
  m.def("compile_regex", &compile_regex, py::arg("pattern"), py::arg("max_states") = 2048, py::arg("max_positions") = 4096);
  m.def("dfa_find", &dfa_find_py, py::arg("pattern"), py::arg("line"), py::arg("max_states") = 4096);
  // host twin of the BPG walk (bpg.h bpg_find_w) over one line, for tests
  m.def("bpg_find", [](py::bytes prog, const std::string& line) {
    const std::string p = prog;
    std::vector<uint64_t> w(p.size() / 8);
    std::memcpy(w.data(), p.data(), w.size() * 8);
    return bpg_find_host(w.data(), reinterpret_cast<const uint8_t*>(line.data()), (int)line.size());
  });
  m.def("unicode_set", [](const std::string& key) {
    py::list out;
    for (auto& r : unicode_set(key).r) out.append(py::make_tuple(r.first, r.second));
    return out;
  });
  m.def("split_docs", &split_docs);
  m.def("set_host_threads", &set_host_threads);
  m.def("set_pf_verify_lanes", &set_pf_verify_lanes);
  m.def("set_scan_defer_rare", &set_scan_defer_rare);
  m.def("set_cand_verify_split", &set_cand_verify_split);
  m.def("set_summ_select", &set_summ_select);
  m.def("set_small_profile", &set_small_profile);
  m.def("pack_split_docs", &pack_split_docs_py, py::arg("docs"), py::arg("dst"), py::arg("cap"),
        py::arg("nthreads") = 8, py::arg("idx") = 0, py::arg("idx_cap") = 0);
  m.def("parse_pod_request", &parse_pod_request_py, py::arg("body"), py::arg("two_pass") = false,
        py::arg("into") = false);
  m.def("parse_pod_request_stream", &parse_pod_request_stream_py, py::arg("body"), py::arg("cuts"));
  // the front end's skip-mode view of a body: (status, logs offset, escaped length, decoded length)
  m.def("pod_logs_span", [](const py::bytes& body) {
    std::string b = body;
    PodRequest pr;
    const int st = parse_pod_request(reinterpret_cast<const uint8_t*>(b.data()), b.size(), pr, false);
    return py::make_tuple(st, pr.logs_off, pr.logs_len, pr.logs_dlen);
  });
  // the packer's exact-bounds decoder of a string's escaped content (tests)
  m.def("decode_json_exact", [](const py::bytes& content) {
    std::string c = content;
    std::string out(c.size() + 128, '\xAB');
    const size_t k = decode_json_string_exact(reinterpret_cast<const uint8_t*>(c.data()), c.size(), &out[0]);
    bool intact = true;                  // nothing stored past the decoded end
    for (size_t i = k; i < out.size(); ++i) intact = intact && out[i] == '\xAB';
    return py::make_tuple(py::bytes(out.data(), k), intact);
  });

  // ---- device launchers
  m.def("line_index_tiles", &line_index_tiles);
  m.def("line_index_dev", [](uint64_t text, int64_t n, uint64_t ws, int64_t ntiles_cap, uint64_t starts, uint64_t lens,
                             int64_t cap, uint64_t info, bool trim, uint64_t blk, int64_t nblk, uint64_t s, bool counted) {
    line_index_dev(P<const uint8_t>(text), n, LineIndexWs{P<int64_t>(ws), ntiles_cap, size_t(1) << 20}, P<int64_t>(starts),
                   P<int32_t>(lens), cap, P<int64_t>(info), trim, P<int32_t>(blk), nblk, s, counted); },
        py::arg("text"), py::arg("n"), py::arg("ws"), py::arg("ntiles_cap"), py::arg("starts"), py::arg("lens"),
        py::arg("cap"), py::arg("info"), py::arg("trim"), py::arg("blk"), py::arg("nblk"), py::arg("s"),
        py::arg("counted") = false);
  // nlp (optional): (nlm, cnt, crf, ntiles) of line_index_pass1 -- the fused line-index pass 1
  m.def("prefilter_dev", [](uint64_t text, int64_t n, py::tuple pf, uint64_t ls, int64_t nl, uint64_t cand, int64_t cap,
                            uint64_t count, int grid, uint64_t s, py::object nlp) {
    NlOut o;
    const bool fused = !nlp.is_none();
    if (fused) {
      py::tuple t = nlp.cast<py::tuple>();
      o.nlm = P<uint64_t>(t[0].cast<uint64_t>());
      o.cnt = P<int32_t>(t[1].cast<uint64_t>());
      o.crf = P<int32_t>(t[2].cast<uint64_t>());
      o.ntiles = t[3].cast<int64_t>();
    }
    prefilter_dev(P<const uint8_t>(text), n, pf_from(pf), P<const int64_t>(ls), nl, P<int64_t>(cand), cap,
                  P<unsigned long long>(count), grid, s, fused ? &o : nullptr); },
        py::arg("text"), py::arg("n"), py::arg("pf"), py::arg("ls"), py::arg("nl"), py::arg("cand"), py::arg("cap"),
        py::arg("count"), py::arg("grid"), py::arg("s"), py::arg("nlp") = py::none());
  // zeroes and returns the line index's pass-1 outputs (nlm, cnt, crf, ntiles) for a fused prefilter
  m.def("line_index_pass1", [](uint64_t ws, int64_t ntiles_cap, int64_t n, uint64_t s) {
    const NlOut o = line_index_pass1_views(LineIndexWs{P<int64_t>(ws), ntiles_cap, size_t(1) << 20}, n, s);
    return py::make_tuple(reinterpret_cast<uint64_t>(o.nlm), reinterpret_cast<uint64_t>(o.cnt),
                          reinterpret_cast<uint64_t>(o.crf), o.ntiles);
  });
  m.def("pf_verify_dev", [](uint64_t gh, int64_t n, uint64_t text, int64_t nb, py::tuple pf, uint64_t ls, int64_t nl,
                            uint64_t blk, uint64_t cand, int64_t cap, uint64_t count, uint64_t s, uint64_t dn,
                            int max_grid) {
    pf_verify_dev(P<const int64_t>(gh), n, P<const uint8_t>(text), nb, pf_from(pf), P<const int64_t>(ls), nl,
                  P<const int32_t>(blk), P<int64_t>(cand), cap, P<unsigned long long>(count), s,
                  P<const unsigned long long>(dn), max_grid); }, py::arg("gh"), py::arg("n"), py::arg("text"),
        py::arg("nb"), py::arg("pf"), py::arg("ls"), py::arg("nl"), py::arg("blk"), py::arg("cand"), py::arg("cap"),
        py::arg("count"), py::arg("s"), py::arg("dn") = 0, py::arg("max_grid") = 8192);
  m.def("append_keys", [](uint64_t dst, int64_t cap, uint64_t count, uint64_t src, int64_t n, uint64_t s) {
    append_keys_dev(P<int64_t>(dst), cap, P<unsigned long long>(count), P<const int64_t>(src), n, s); });
  // backtracker regexes fed by their relaxed automata (side_path.hip). out: None = drop mode, else
  // (keys, starts, lens, cap, cnt, done_blocks, host_cnt, host_seq, seq) device-visible addresses
  m.def("take_host", [](uint64_t cand, uint64_t n1d, int64_t cap1, uint64_t ver, uint64_t n2d, int64_t cap2,
                        uint64_t text, uint64_t ls, uint64_t ll, py::tuple dfa, py::object out, uint64_t s) {
    HostSideOut O;
    if (!out.is_none()) {
      py::tuple t = out.cast<py::tuple>();
      O.keys = P<int64_t>(t[0].cast<uint64_t>()); O.starts = P<int64_t>(t[1].cast<uint64_t>());
      O.lens = P<int64_t>(t[2].cast<uint64_t>()); O.cap = t[3].cast<int64_t>();
      O.cnt = P<unsigned long long>(t[4].cast<uint64_t>()); O.done_blocks = P<unsigned int>(t[5].cast<uint64_t>());
      O.host_cnt = P<int64_t>(t[6].cast<uint64_t>()); O.host_seq = P<int64_t>(t[7].cast<uint64_t>());
      O.seq = t[8].cast<int64_t>();
    }
    take_host_dev(P<int64_t>(cand), P<const unsigned long long>(n1d), cap1, P<int64_t>(ver),
                  P<const unsigned long long>(n2d), cap2, P<const uint8_t>(text), P<const int64_t>(ls),
                  P<const int32_t>(ll), dfa_from(dfa), O, s); });
  // in = (keys, host_cnt, host_seq, cap, seq, err) device-visible addresses of pinned host memory
  m.def("wait_host", [](uint64_t ver, int64_t cap2, uint64_t n2d, py::tuple in, uint64_t s, double timeout_s) {
    HostSideIn I;
    I.keys = P<const int64_t>(in[0].cast<uint64_t>()); I.host_cnt = P<const int64_t>(in[1].cast<uint64_t>());
    I.host_seq = P<const int64_t>(in[2].cast<uint64_t>()); I.cap = in[3].cast<int64_t>(); I.seq = in[4].cast<int64_t>();
    I.err = P<int64_t>(in[5].cast<uint64_t>());
    I.timeout_ticks = (long long)(timeout_s * 1e8);
    wait_host_dev(P<int64_t>(ver), cap2, P<unsigned long long>(n2d), I, s); }, py::arg("ver"), py::arg("cap2"),
    py::arg("n2d"), py::arg("in"), py::arg("stream"), py::arg("timeout_s") = 2.0);
  // pinned host memory the GPU reads and writes coherently (fine-grained): (host address, device
  // address); freed with host_free_coherent
  m.def("host_alloc_coherent", [](int64_t bytes) {
    void* h = nullptr;
    if (hipHostMalloc(&h, (size_t)std::max<int64_t>(bytes, 8), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
      throw std::runtime_error("hipHostMalloc (coherent) failed");
    std::memset(h, 0, (size_t)std::max<int64_t>(bytes, 8));
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
      (void)hipHostFree(h);
      throw std::runtime_error("hipHostGetDevicePointer failed");
    }
    return py::make_tuple(reinterpret_cast<uint64_t>(h), reinterpret_cast<uint64_t>(d));
  });
  m.def("host_free_coherent", [](uint64_t h) { (void)hipHostFree(reinterpret_cast<void*>(h)); });
  m.def("scan_dev", [](uint64_t text, uint64_t ls, uint64_t ll, int64_t nl, uint64_t regs, int nregs, py::tuple dfa,
                       uint64_t out, int64_t cap, uint64_t count, uint64_t s) {
    scan_dev(P<const uint8_t>(text), P<const int64_t>(ls), P<const int32_t>(ll), nl, P<const int32_t>(regs), nregs,
             dfa_from(dfa), P<int64_t>(out), cap, P<unsigned long long>(count), s); });
  // BPG candidate walks (bpg.hip) on their own, for kernel tests / A/B: in-place candidate verify
  // (cand = (regex << 32 | line), -1 = rejected) and first-of-run flags over sorted packed keys
  m.def("bpg_cand_dev", [](uint64_t cand, int64_t cap, uint64_t text, uint64_t ls, uint64_t ll, py::tuple dfa,
                           uint64_t s) {
    bpg_cand_dev(P<int64_t>(cand), cap, nullptr, P<const uint8_t>(text), P<const int64_t>(ls), P<const int32_t>(ll),
                 dfa_from(dfa), s); });
  m.def("bpg_dedupe_dev", [](uint64_t keys, int64_t n, int lbits, uint64_t text, uint64_t ls, uint64_t ll,
                             py::tuple dfa, uint64_t flag, uint64_t s, uint64_t wcnt, uint64_t wlist) {
    bpg_dedupe_dev(P<const uint64_t>(keys), n, lbits, P<const uint8_t>(text), P<const int64_t>(ls),
                   P<const int32_t>(ll), dfa_from(dfa), P<uint8_t>(flag), s, P<uint32_t>(wcnt), P<uint32_t>(wlist)); },
        py::arg("keys"), py::arg("n"), py::arg("lbits"), py::arg("text"), py::arg("ls"), py::arg("ll"), py::arg("dfa"),
        py::arg("flag"), py::arg("stream"), py::arg("wcnt") = 0, py::arg("wlist") = 0);
  // ev_rank / ev_fkey / carry: frequency count before each event = carry[fkey] + rank (fused)
  // dn (optional): device event count, n is then a capacity
  m.def("score_dev", [](uint64_t el, uint64_t ep, uint64_t es, uint64_t rank, uint64_t fkey, uint64_t carry, int64_t n,
                        py::tuple st, py::tuple sp, uint64_t out, uint64_t fac, uint64_t s, uint64_t dn) {
    const FreqIn F{P<const int64_t>(rank), P<const int64_t>(fkey), P<const int64_t>(carry)};
    score_dev(P<const int32_t>(el), P<const int32_t>(ep), P<const int32_t>(es), F, n, st_from(st),
              sp_from(sp), P<double>(out), P<double>(fac), s, P<const int64_t>(dn)); },
        py::arg("el"), py::arg("ep"), py::arg("es"), py::arg("rank"), py::arg("fkey"), py::arg("carry"), py::arg("n"),
        py::arg("st"), py::arg("sp"), py::arg("out"), py::arg("fac"), py::arg("s"), py::arg("dn") = 0);

  // ---- host twins
  m.def("nl_positions_host", [](uint64_t text, int64_t n, uint64_t pos) { return nl_positions_host(P<const uint8_t>(text), n, P<int64_t>(pos)); });
  m.def("prefilter_host", [](uint64_t text, int64_t n, py::tuple pf, uint64_t ls, int64_t nl, uint64_t cand, int64_t cap) {
    return prefilter_host(P<const uint8_t>(text), n, pf_from(pf), P<const int64_t>(ls), nl, P<int64_t>(cand), cap); });
  m.def("scan_host", [](uint64_t text, uint64_t ls, uint64_t ll, int64_t nl, uint64_t regs, int nregs, py::tuple dfa,
                        uint64_t out, int64_t cap) {
    return scan_host(P<const uint8_t>(text), P<const int64_t>(ls), P<const int32_t>(ll), nl, P<const int32_t>(regs),
                     nregs, dfa_from(dfa), P<int64_t>(out), cap); });
  m.def("scan_multi", [](uint64_t text, int64_t nbytes, uint64_t ls, uint64_t ll, int64_t nl, py::tuple pass,
                         uint64_t out, int64_t cap, uint64_t cnt, int grid, uint64_t s, bool dev) -> int64_t {
    const ScanPass S = scan_pass_from(pass);
    if (dev) {
      scan_multi_dev(P<const uint8_t>(text), nbytes, P<const int64_t>(ls), P<const int32_t>(ll), nl, S, P<int64_t>(out), cap,
                     P<unsigned long long>(cnt), grid, s);
      return 0;
    }
    py::gil_scoped_release nogil;
    return scan_multi_host(P<const uint8_t>(text), P<const int64_t>(ls), P<const int32_t>(ll), nl, S, P<int64_t>(out),
                           cap);
  });
  m.def("freq_evict", [](py::tuple ring, double horizon, uint64_t s, bool dev) {
    freq_evict(ring_from(ring), horizon, s, dev);
  });
  // ---- summary + top-k (summarize.hip). in = (score, pat, line32, line64, line_add, sev_of_pat, rows
  // [, packed events out])
  m.def("summarize", [](py::tuple in, int64_t n, int k, int nsev, uint64_t top, uint64_t pat_hist, uint64_t sev_hist,
                        uint64_t ws, uint64_t ws_bytes, uint64_t s, bool dev) -> uint64_t {
    const SummIn I{P<const double>(in[0].cast<uint64_t>()), P<const int32_t>(in[1].cast<uint64_t>()),
                   P<const int32_t>(in[2].cast<uint64_t>()), P<const int64_t>(in[3].cast<uint64_t>()),
                   P<const int64_t>(in[4].cast<uint64_t>()), P<const int32_t>(in[5].cast<uint64_t>()),
                   P<const double>(in[6].cast<uint64_t>()),
                   in.size() > 7 ? P<void>(in[7].cast<uint64_t>()) : nullptr,
                   in.size() > 8 ? P<const int64_t>(in[8].cast<uint64_t>()) : nullptr};
    if (dev)
      return summarize_dev(I, n, k, nsev, P<double>(top), P<unsigned long long>(pat_hist), P<unsigned long long>(sev_hist),
                           P<void>(ws), ws_bytes, s);
    summarize_host(I, n, k, P<double>(top), P<int64_t>(pat_hist), P<int64_t>(sev_hist));
    return 0;
  });
  m.def("rescore", [](uint64_t gl, uint64_t fac, int64_t n, int64_t Nn, py::tuple sp, uint64_t out, uint64_t s,
                      bool dev) {
    if (dev)
      rescore_dev(P<const int64_t>(gl), P<const double>(fac), n, Nn, sp_from(sp), P<double>(out), s);
    else
      rescore_host(P<const int64_t>(gl), P<const double>(fac), n, Nn, sp_from(sp), P<double>(out));
  });
  // ---- DP step bookkeeping (dp_glue.hip)
  // cnt (optional, device [5] match / event counters) + caps [4]: the payload's overflow flag
  m.def("dp_pack", [](int64_t own_lines, uint64_t freq, int nk, uint64_t chain, int ns, uint64_t pack, uint64_t s,
                      bool dev, uint64_t cnt, std::vector<int64_t> caps) {
    if (cnt && caps.size() != 4) throw std::invalid_argument("dp_pack: 4 capacities");
    dp_pack(own_lines, P<const int64_t>(freq), nk, P<const int32_t>(chain), ns, P<int64_t>(pack), s, dev,
            P<const int64_t>(cnt), cnt ? caps.data() : nullptr); },
        py::arg("own_lines"), py::arg("freq"), py::arg("nk"), py::arg("chain"), py::arg("ns"), py::arg("pack"),
        py::arg("s"), py::arg("dev"), py::arg("cnt") = 0, py::arg("caps") = std::vector<int64_t>());
  // a = (g, world, rank, nk, ns, halo_left, tot, slot_e0, slot_k, own_start, g0, n, carry, seq_carry, red_tail)
  m.def("dp_carry", [](py::tuple a, uint64_t s, bool dev) {
    auto u = [&](int i) { return a[i].cast<uint64_t>(); };
    DpCarryArgs A{P<const int64_t>(u(0)), a[1].cast<int>(), a[2].cast<int>(), a[3].cast<int>(), a[4].cast<int>(),
                  a[5].cast<int64_t>(), P<const int64_t>(u(6)), P<const int64_t>(u(7)), P<const int64_t>(u(8)),
                  P<int64_t>(u(9)), P<int64_t>(u(10)), P<int64_t>(u(11)), P<int64_t>(u(12)), P<uint8_t>(u(13)),
                  P<int64_t>(u(14))};
    if (a.size() > 15) A.veto = P<int64_t>(u(15));
    if (a.size() > 17) {
      A.zero = P<int64_t>(u(16));
      A.nzero = a[17].cast<int64_t>();
    }
    if (a.size() > 21) {
      A.seq_base = P<const uint8_t>(u(18));
      A.line_base = a[19].cast<int64_t>();
      A.n_fixed = a[20].cast<int64_t>();
      A.seq_next = P<uint8_t>(u(21));
    }
    dp_carry(A, s, dev);
  });
  // veto (optional, device int64): no record when *veto != 0 (a DP step that re-runs)
  // gate_cnt / gate_caps (device counters [gram, cand, ver, hits, events] + the 4 capacities of
  // gram, cand, ver, events): nothing is recorded when a count exceeds its capacity (a deferred step
  // that re-runs), decided on the device so the record can be queued before the host's count read
  m.def("freq_record", [](uint64_t counts, int K, double now, py::tuple ring, uint64_t s, bool dev, uint64_t veto,
                          uint64_t gate_cnt, py::tuple gate_caps) {
    RecordGate G;
    G.veto = P<const int64_t>(veto);
    G.cnt = P<const int64_t>(gate_cnt);
    for (size_t i = 0; i < 4 && i < gate_caps.size(); ++i) G.cap[i] = gate_caps[i].cast<int64_t>();
    freq_record(P<const int64_t>(counts), K, now, ring_from(ring), s, dev, G);
  }, py::arg("counts"), py::arg("K"), py::arg("now"), py::arg("ring"), py::arg("s"), py::arg("dev"), py::arg("veto") = 0,
     py::arg("gate_cnt") = 0, py::arg("gate_caps") = py::tuple());
  m.def("score_host", [](uint64_t el, uint64_t ep, uint64_t es, uint64_t rank, uint64_t fkey, uint64_t carry,
                         int64_t n, py::tuple st, py::tuple sp, uint64_t out, uint64_t fac) {
    const FreqIn F{P<const int64_t>(rank), P<const int64_t>(fkey), P<const int64_t>(carry)};
    score_host(P<const int32_t>(el), P<const int32_t>(ep), P<const int32_t>(es), F, n, st_from(st),
               sp_from(sp), P<double>(out), P<double>(fac)); });

  // ---- post-match pipeline (lp_post.hip); device calls return the workspace bytes they need and
  // only run when ws_bytes suffices
  m.def("bits_for", &bits_for);

  // ---- native request runner (csrc/runtime/request.cpp): the device half of a batch in one call
  py::class_<RequestRunner>(m, "RequestRunner")
      .def(py::init([](py::tuple pf, py::tuple dfa, py::list scans, py::list grids, uint64_t scan_regs, int n_scan_regs,
                       py::tuple st12, py::tuple sp, py::tuple ev5, int R, int npat, int nkeys, int nseq, int ctx_trans,
                       int ctx_acc, int pf_grid, int device, bool device_counts, bool host_dev) {
             RequestStatic S;
             S.device_counts = device_counts;
             S.host_dev = host_dev;
             S.pf = pf_from(pf);
             S.dfa = dfa_from(dfa);
             for (auto h : scans) S.scans.push_back(scan_pass_from(h.cast<py::tuple>()));
             for (auto h : grids) S.scan_grids.push_back(h.cast<int>());
             if (S.scans.size() != S.scan_grids.size()) throw std::invalid_argument("RequestRunner: one grid per scan pass");
             S.scan_regs = P<const int32_t>(scan_regs);
             S.n_scan_regs = n_scan_regs;
             int i = 0;
             auto nx = [&]() { return st12[i++].cast<uint64_t>(); };
             ScoreTables& T = S.st;
             T.conf = P<const double>(nx()); T.sev = P<const double>(nx());
             T.ctx_before = P<const int32_t>(nx()); T.ctx_after = P<const int32_t>(nx());
             T.sec_off = P<const int32_t>(nx()); T.sec_reg = P<const int32_t>(nx()); T.sec_w = P<const int32_t>(nx());
             T.sec_weight = P<const double>(nx());
             T.seq_off = P<const int32_t>(nx()); T.seq_bonus = P<const double>(nx());
             T.seq_ev_off = P<const int32_t>(nx()); T.seq_ev_reg = P<const int32_t>(nx());
             S.sp = sp_from(sp);
             EvTables& E = S.ev;
             E.prim_off = P<const int64_t>(ev5[0].cast<uint64_t>());
             E.prim_pats = P<const int32_t>(ev5[1].cast<uint64_t>());
             E.freq_key = P<const int32_t>(ev5[2].cast<uint64_t>());
             E.ctx_before = P<const int32_t>(ev5[3].cast<uint64_t>());
             E.ctx_after = P<const int32_t>(ev5[4].cast<uint64_t>());
             E.nkeys = nkeys;
             E.pbits = bits_for(std::max(npat, 1));
             S.R = R; S.npat = npat; S.nkeys = nkeys; S.nseq = nseq;
             S.ctx_trans = ctx_trans; S.ctx_acc = ctx_acc; S.pf_grid = pf_grid; S.device = device;
             return new RequestRunner(S);
           }), py::arg("pf"), py::arg("dfa"), py::arg("scans"), py::arg("grids"), py::arg("scan_regs"),
           py::arg("n_scan_regs"), py::arg("st12"), py::arg("sp"), py::arg("ev5"), py::arg("R"), py::arg("npat"),
           py::arg("nkeys"), py::arg("nseq"), py::arg("ctx_trans"), py::arg("ctx_acc"), py::arg("pf_grid"),
           py::arg("device"), py::arg("device_counts") = true, py::arg("host_dev") = false)
      .def("run", [](RequestRunner& r, uint64_t text, int64_t nbytes, uint64_t starts, uint64_t lens, int64_t L,
                     py::array_t<int32_t, py::array::c_style | py::array::forcecast> lo,
                     py::array_t<int32_t, py::array::c_style | py::array::forcecast> hi,
                     py::array_t<int64_t, py::array::c_style | py::array::forcecast> g0,
                     py::array_t<int64_t, py::array::c_style | py::array::forcecast> n, py::tuple ring,
                     double evict_before, double now, uint64_t stream, int64_t host_cap, Turn* turn, int64_t seq,
                     py::array_t<int64_t, py::array::c_style | py::array::forcecast> inj, SharedWindow* hw,
                     int64_t pre_token) {
        const FreqRing R = hw ? FreqRing{} : ring_from(ring);
        const int D = (int)lo.shape(0);
        int64_t ne;
        {
          py::gil_scoped_release nogil;
          ne = r.run(P<uint8_t>(text), nbytes, P<const int64_t>(starts), P<const int32_t>(lens), L, lo.data(), hi.data(),
                     g0.data(), n.data(), D, R, evict_before, now, stream, host_cap, turn, seq,
                     inj.size() ? inj.data() : nullptr, (int64_t)inj.size(), hw, pre_token);
        }
        py::array_t<uint8_t> out((py::ssize_t)r.result_bytes());
        std::memcpy(out.mutable_data(), r.result(), r.result_bytes());
        const RequestCounts& c = r.counts();
        py::dict d;
        d["lines"] = c.lines; d["gram_hits"] = c.gram; d["prefilter_candidates"] = c.cand; d["scan_hits"] = c.ver;
        d["hits"] = c.hits; d["events"] = c.events;
        return py::make_tuple(ne, out, d, r.stride());
      }, py::arg("text"), py::arg("nbytes"), py::arg("starts"), py::arg("lens"), py::arg("L"), py::arg("lo"),
         py::arg("hi"), py::arg("g0"), py::arg("n"), py::arg("ring"), py::arg("evict_before"), py::arg("now"),
         py::arg("stream"), py::arg("host_cap") = 0, py::arg("turn") = nullptr, py::arg("seq") = 0,
         py::arg("inj") = py::array_t<int64_t>(0), py::arg("hw") = nullptr, py::arg("pre_token") = 0)
      .def_property_readonly("recorded", &RequestRunner::recorded)
      .def("prefetch_text", [](RequestRunner& r, uint64_t text, int64_t nbytes, int64_t host_cap, uint64_t stream) {
        py::gil_scoped_release nogil;
        return r.prefetch_text(P<uint8_t>(text), nbytes, host_cap, stream);   // token for run(pre_token=)
      }, py::arg("text"), py::arg("nbytes"), py::arg("host_cap"), py::arg("stream"))
      .def("upload_bytes", &RequestRunner::upload_bytes);

  // arrival-order gate of a window shared by several runners (csrc/runtime/request.h)
  py::class_<Turn>(m, "Turn")
      .def("wait", [](Turn& t, int64_t seq) { py::gil_scoped_release nogil; t.wait(seq); })
      .def("done", [](Turn& t, int64_t seq) { py::gil_scoped_release nogil; t.done(seq); });
  py::class_<WindowTurn, Turn>(m, "WindowTurn")
      .def(py::init<>())
      .def_property_readonly("next", &WindowTurn::next);
  // the serving processes of a node (csrc/runtime/proc_shared.h): arrival ticket, cross-process
  // turns, the shared window's metadata
  py::class_<ProcTurn, Turn>(m, "ProcTurn").def_property_readonly("next", &ProcTurn::next);
  py::class_<ProcShared>(m, "ProcShared")
      .def(py::init<const std::string&, bool, int>(), py::arg("name"), py::arg("create"), py::arg("nproc") = 0)
      .def("take", &ProcShared::take)
      .def_property_readonly("host", &ProcShared::host, py::return_value_policy::reference_internal)
      .def_property_readonly("dev", &ProcShared::dev, py::return_value_policy::reference_internal)
      .def_property_readonly("name", &ProcShared::name)
      .def_property_readonly("nproc", &ProcShared::nproc)
      .def_property_readonly("ticket", [](ProcShared& s) { return s.header()->ticket.load(); })
      .def_property_readonly("released_dead", [](ProcShared& s) { return s.header()->released_dead.load(); })
      .def_property_readonly("sections", [](ProcShared& s) { return s.header()->sections.load(); })
      .def_property("restarts", [](ProcShared& s) { return s.header()->restarts.load(); },
                    [](ProcShared& s, int64_t v) { s.header()->restarts.store(v); })
      .def("mark_up", &ProcShared::mark_up)
      .def("up", &ProcShared::up)
      .def_property_readonly("generation", [](ProcShared& s) { return s.win().generation.load(std::memory_order_acquire); })
      .def_property_readonly("cap", [](ProcShared& s) { return s.win().cap; })
      .def_property_readonly("nkeys", [](ProcShared& s) { return s.win().nkeys; })
      .def_property_readonly("window_s", [](ProcShared& s) { return s.win().window_s; })
      .def_property_readonly("last_now", [](ProcShared& s) { return s.win().last_now; })
      .def_static("unlink", &ProcShared::unlink);
  // the node's shared frequency window in host shared memory (proc_shared.h): created by the
  // first worker, attached by the others; every call but arrays() inside a window section
  py::class_<SharedWindow>(m, "SharedWindow")
      .def(py::init([](py::object shared, int nkeys, double window_s, bool create, int64_t capacity) {
             return new SharedWindow(&shared.cast<ProcShared&>(), nkeys, window_s, create, capacity);
           }), py::arg("shared"), py::arg("nkeys"), py::arg("window_s"), py::arg("create"),
           py::arg("capacity") = int64_t(1) << 20, py::keep_alive<1, 2>())
      .def("arrays", [](SharedWindow& w) {       // (t, key, cnt, ht, tot, seen) addresses + capacity
        const WinArrays a = w.arrays();
        return py::make_tuple(reinterpret_cast<uint64_t>(a.t), reinterpret_cast<uint64_t>(a.key),
                              reinterpret_cast<uint64_t>(a.cnt), reinterpret_cast<uint64_t>(a.ht),
                              reinterpret_cast<uint64_t>(a.tot), reinterpret_cast<uint64_t>(a.seen), a.cap);
      })
      .def("ensure_room", &SharedWindow::ensure_room)
      .def("now", &SharedWindow::now)
      .def("evict", &SharedWindow::evict)
      .def("record", [](SharedWindow& w, uint64_t counts, int K, double now) {
        w.ensure_room(K);
        w.record(P<const int64_t>(counts), K, now);
      })
      .def("enter", [](SharedWindow& w) { py::gil_scoped_release nogil; return w.enter(); })
      .def("leave", [](SharedWindow& w, int64_t seq) { py::gil_scoped_release nogil; w.leave(seq); })
      .def_property_readonly("nkeys", &SharedWindow::nkeys);
  // a DLPack view (torch.from_dlpack) of raw memory: the shared window's arrays
  m.def("dlpack", [](uint64_t ptr, int64_t numel, const std::string& dtype, int device) {
    return dlpack_capsule(ptr, numel, dtype, device);
  }, py::arg("ptr"), py::arg("numel"), py::arg("dtype"), py::arg("device"));
  // page-lock existing host memory for DMA (a stream source already in RAM: its chunks are copied
  // to the GPU straight from it, no staging copy); false when the runtime refuses
  m.def("host_register", [](uint64_t ptr, int64_t n) {
    if (hipHostRegister(reinterpret_cast<void*>(ptr), (size_t)n, hipHostRegisterDefault) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    return true;
  });
  m.def("host_unregister", [](uint64_t ptr) { return hipHostUnregister(reinterpret_cast<void*>(ptr)) == hipSuccess; });
  // one host -> device copy on a HIP stream, HostToDevice kind (the copy-engine probe compares it
  // with torch's copy_; tools/copy_engine_probe.py)
  m.def("copy_h2d", [](uint64_t dst, uint64_t src, int64_t n, uint64_t stream) {
    if (hipMemcpyAsync(reinterpret_cast<void*>(dst), reinterpret_cast<const void*>(src), (size_t)n,
                       hipMemcpyHostToDevice, reinterpret_cast<hipStream_t>(stream)) != hipSuccess)
      throw std::runtime_error(std::string("copy_h2d: ") + hipGetErrorString(hipGetLastError()));
  });
  // peer access for kernels on `device` reading / writing memory of `peer` (a shared window)
  m.def("enable_peer_access", [](int device, int peer) {
    if (device == peer) return true;
    int can = 0;
    if (hipDeviceCanAccessPeer(&can, device, peer) != hipSuccess || !can) return false;
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(device);
    hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
    (void)hipSetDevice(cur);
    if (e == hipErrorPeerAccessAlreadyEnabled) { (void)hipGetLastError(); return true; }
    return e == hipSuccess;
  });

  // ---- native load generator (csrc/io/loadgen.cpp): config 5 over real connections
  m.def("http_burst", [](const std::string& host, int port, py::list msgs, py::array_t<int32_t> idx, double timeout_s,
                         int nthreads) {
    std::vector<std::string> M;
    for (auto h : msgs) M.push_back(h.cast<std::string>());
    std::vector<int32_t> I(idx.data(), idx.data() + idx.size());
    LoadResult R;
    {
      py::gil_scoped_release nogil;
      R = http_burst(host, port, M, I, timeout_s, nthreads);
    }
    py::array_t<double> lat(R.latency.size());
    std::memcpy(lat.mutable_data(), R.latency.data(), R.latency.size() * sizeof(double));
    py::array_t<int32_t> st(R.status.size());
    std::memcpy(st.mutable_data(), R.status.data(), R.status.size() * sizeof(int32_t));
    return py::make_tuple(lat, st, R.t_end - R.t_start, R.completed);
  }, py::arg("host"), py::arg("port"), py::arg("msgs"), py::arg("idx"), py::arg("timeout_s") = 120.0,
     py::arg("nthreads") = 8);

  // ---- native HTTP/1.1 front end (csrc/io/http_server.cpp)
  py::class_<RawLogs>(m, "RawLogs")
      .def("__len__", [](const RawLogs& r) { return r.len; })
      .def("decode", &raw_logs_decode, "the unescaped UTF-8 log text")
      .def_property_readonly("escaped_len", [](const RawLogs& r) { return r.len; })
      .def_property_readonly("decoded_len", [](const RawLogs& r) { return r.dlen; })
      // decoded by the IO thread into a pinned buffer: (address, capacity) -- the engine stages this
      // request in place; (0, 0) otherwise
      .def_property_readonly("pinned_text", [](const RawLogs& r) {
        const bool pin = r.decoded() && r.dec.pinned;
        return py::make_tuple(pin ? reinterpret_cast<uint64_t>(r.dec.p) : uint64_t(0),
                              pin ? (uint64_t)r.dec.cap : uint64_t(0));
      });

  py::class_<HttpServer>(m, "HttpServer")
      .def(py::init([](const std::string& host, int port, int io_threads, int64_t max_body, double idle,
                       double io_spin_us, double pump_spin_us, bool quickack, int rcvbuf, bool trace,
                       bool conn_trace, bool prefetch, int64_t io_decode_max_conns) {
             HttpOptions o;
             o.prefetch = prefetch;
             o.io_decode_max_conns = io_decode_max_conns;
             o.io_spin_us = io_spin_us; o.pump_spin_us = pump_spin_us; o.quickack = quickack; o.rcvbuf = rcvbuf;
             o.trace = trace;
             o.conn_trace = conn_trace;
             return new HttpServer(host, port, io_threads, max_body, idle, o);
           }), py::arg("host"), py::arg("port"), py::arg("io_threads") = 2, py::arg("max_body") = int64_t(1) << 30,
           py::arg("idle_timeout_s") = 60.0, py::arg("io_spin_us") = 0.0, py::arg("pump_spin_us") = 1000.0,
           py::arg("quickack") = true, py::arg("rcvbuf") = 0, py::arg("trace") = false, py::arg("conn_trace") = false,
           py::arg("prefetch") = true, py::arg("io_decode_max_conns") = int64_t(64))
      .def("conn_trace", [](HttpServer& s) {
        std::vector<std::vector<double>> v;
        {
          py::gil_scoped_release nogil;
          v = s.conn_trace();
        }
        py::array_t<double> a({(py::ssize_t)v.size(), (py::ssize_t)6});
        for (size_t i = 0; i < v.size(); ++i) std::memcpy(a.mutable_data(i, 0), v[i].data(), 6 * sizeof(double));
        return a;
      })
      .def_property_readonly("port", &HttpServer::port)
      .def("set_pinned_decode", [](HttpServer& s, int limit, size_t min_bytes) {
             s.set_pinned_decode(limit, min_bytes,
                                 [](size_t n) -> void* {
                                   void* q = nullptr;
                                   if (hipHostMalloc(&q, n, hipHostMallocDefault) != hipSuccess) {
                                     (void)hipGetLastError();
                                     return nullptr;
                                   }
                                   return q;
                                 },
                                 [](void* q) { (void)hipHostFree(q); });
           }, py::arg("limit"), py::arg("min_bytes") = size_t(256) << 10)
      .def("set_affinity_sets", &HttpServer::set_affinity_sets, py::arg("narrow"), py::arg("wide"), py::arg("hi"),
           py::arg("lo"))
      .def("pending", &HttpServer::pending)
      .def("next_requests", [](HttpServer& s, int max_n, int timeout_ms, bool raw) {
        std::vector<HttpRequest> v;
        {
          py::gil_scoped_release nogil;
          v = s.next_requests(max_n, timeout_ms);
        }
        if (raw) {          // decoded later, straight into the engine's stage (RawLogs)
          py::list out;
          for (auto& r : v) {
            if (r.kind == 0) {
              auto* rl = new RawLogs();
              rl->off = r.logs_off;
              rl->len = r.logs_len;
              rl->dlen = r.logs_dlen;
              rl->body = std::move(r.body);
              rl->pool = s.pool();
              if (r.dec.p) {
                rl->dec = std::move(r.dec);
                rl->dpool = s.decode_pool();
                rl->pool->give(std::move(rl->body));   // the escaped body is not needed any more
                rl->pool = nullptr;
              }
              out.append(py::make_tuple(r.id, 0, py::cast(rl, py::return_value_policy::take_ownership), r.pod_name,
                                        r.t_arrival));
            } else {
              out.append(py::make_tuple(r.id, 1, r.method, r.path, py::bytes(r.body), r.t_arrival));
            }
          }
          return out;
        }
        // decoded POST /parse: one bytes object per request sized for the escaped text, filled by
        // the unescaper with the GIL released (the only copy of the log between the socket
        // buffer and the engine's pinned stage), then trimmed
        std::vector<PyObject*> bufs(v.size(), nullptr);
        for (size_t i = 0; i < v.size(); ++i)
          if (v[i].kind == 0) {
            bufs[i] = PyBytes_FromStringAndSize(nullptr, (Py_ssize_t)(v[i].logs_len + 64));
            if (!bufs[i]) {
              for (PyObject* b : bufs) Py_XDECREF(b);
              throw py::error_already_set();
            }
          }
        std::vector<size_t> lens(v.size(), 0);
        {
          py::gil_scoped_release nogil;
          for (size_t i = 0; i < v.size(); ++i)
            if (v[i].kind == 0) {
              if (v[i].dec.p) {
                std::memcpy(PyBytes_AS_STRING(bufs[i]), v[i].dec.p, v[i].logs_dlen);
                lens[i] = v[i].logs_dlen;
                s.decode_pool()->give(std::move(v[i].dec));
              } else {
                lens[i] = decode_json_string(reinterpret_cast<const uint8_t*>(v[i].body.data()) + v[i].logs_off,
                                             v[i].logs_len, PyBytes_AS_STRING(bufs[i]));
              }
              s.recycle(std::move(v[i].body));
            }
        }
        py::list out;
        for (size_t i = 0; i < v.size(); ++i) {
          auto& r = v[i];
          if (r.kind == 0) {
            PyObject* b = bufs[i];
            if (_PyBytes_Resize(&b, (Py_ssize_t)lens[i]) != 0) {
              for (size_t j = i + 1; j < v.size(); ++j) Py_XDECREF(bufs[j]);
              throw py::error_already_set();
            }
            out.append(py::make_tuple(r.id, 0, py::reinterpret_steal<py::bytes>(b), r.pod_name, r.t_arrival));
          } else {
            out.append(py::make_tuple(r.id, 1, r.method, r.path, py::bytes(r.body), r.t_arrival));
          }
        }
        return out;
      }, py::arg("max_n") = 4096, py::arg("timeout_ms") = 100, py::arg("raw") = false)
      .def("respond", [](HttpServer& s, uint64_t id, int status, const std::string& ctype, py::bytes body) {
        char* p = nullptr;
        Py_ssize_t n = 0;
        PyBytes_AsStringAndSize(body.ptr(), &p, &n);
        py::gil_scoped_release nogil;   // `body` (immutable) stays referenced for the call
        s.respond(id, status, ctype, p, (size_t)n);
      })
      // one status / content type for a whole batch of responses: one call, GIL released
      .def("respond_many", [](HttpServer& s, std::vector<uint64_t> ids, int status, const std::string& ctype,
                              py::list bodies) {
        const size_t k = std::min(ids.size(), (size_t)py::len(bodies));
        std::vector<const char*> ptrs(k);
        std::vector<size_t> lens(k);
        for (size_t i = 0; i < k; ++i) {
          char* p = nullptr;
          Py_ssize_t n = 0;
          PyBytes_AsStringAndSize(bodies[i].ptr(), &p, &n);
          ptrs[i] = p;
          lens[i] = (size_t)n;
        }
        py::gil_scoped_release nogil;   // the list keeps every (immutable) body referenced
        s.respond_many(ids.data(), k, status, ctype, ptrs.data(), lens.data());
      })
      .def("stats", [](HttpServer& s) {
        py::dict d;
        d["accepted"] = s.stats.accepted.load();
        d["requests"] = s.stats.requests.load();
        d["native_400"] = s.stats.native_400.load();
        return d;
      })
      .def("stage_stats", [](HttpServer& s) {
        const HttpStageStats& g = s.stages;
        py::dict d;
        d["parse"] = g.parse.load(); d["receive_s"] = g.receive_ns.load() * 1e-9;
        d["validate_s"] = g.validate_ns.load() * 1e-9; d["drained"] = g.drained.load();
        d["queue_s"] = g.queue_ns.load() * 1e-9; d["responses"] = g.responses.load();
        d["handoff_s"] = g.handoff_ns.load() * 1e-9; d["sent"] = g.sent.load(); d["send_s"] = g.send_ns.load() * 1e-9;
        d["prefetch_s"] = g.prefetch_ns.load() * 1e-9; d["prefetched"] = g.prefetched.load();
        d["pump_prefetch_s"] = g.pump_prefetch_ns.load() * 1e-9;
        return d;
      })
      .def("stop", [](HttpServer& s) {
        py::gil_scoped_release nogil;
        s.stop();
      });
  m.def("post_hits", [](uint64_t cand, int64_t n, int64_t pre_from, int lbits, int rbits, int R, uint64_t text,
                        uint64_t ls, uint64_t ll, py::tuple dfa, py::tuple ev, uint64_t hits, uint64_t hit_line,
                        uint64_t hit_off, uint64_t ev_cnt, uint64_t ev_end, uint64_t counters, uint64_t ws,
                        size_t ws_bytes, uint64_t s, bool dev, uint64_t cand2, uint64_t dcount) -> size_t {
    HitsArgs A;
    A.cand = P<const int64_t>(cand); A.n = n; A.pre_from = pre_from; A.lbits = lbits; A.rbits = rbits; A.R = R;
    A.cand2 = P<const int64_t>(cand2); A.dcount = P<const unsigned long long>(dcount);
    if (A.dcount && !dev) throw std::runtime_error("post_hits: device counters need the device path");
    A.text = P<const uint8_t>(text); A.ls = P<const int64_t>(ls); A.ll = P<const int32_t>(ll);
    A.dfa = dfa_from(dfa); A.ev = ev_from(ev);
    A.hits = P<int64_t>(hits); A.hit_line = P<int32_t>(hit_line); A.hit_off = P<int64_t>(hit_off);
    A.ev_cnt = P<int64_t>(ev_cnt); A.ev_end = P<int64_t>(ev_end); A.counters = P<int64_t>(counters);
    if (dev) return hits_dev(A, P<void>(ws), ws_bytes, s);
    py::gil_scoped_release nogil;
    hits_host(A);
    return 0;
  });
  m.def("post_events", [](uint64_t hits, int64_t nh, uint64_t ev_cnt, uint64_t ev_end, int64_t ne, int64_t L, int lbits,
                          py::tuple ev, uint64_t text, uint64_t ls, uint64_t ll, py::tuple dfa, uint64_t ev_line,
                          uint64_t ev_pat, uint64_t ev_seg, uint64_t ev_rank, uint64_t ev_fkey, uint64_t freq_counts,
                          uint64_t feat, uint64_t cov, int ctx_trans, int ctx_acc, uint64_t ws, size_t ws_bytes,
                          uint64_t s, bool dev, uint64_t dcounts, uint64_t ne_fit) -> size_t {
    EventsArgs A;
    A.dcounts = P<const int64_t>(dcounts);
    A.ne_fit = P<int64_t>(ne_fit);
    if (A.dcounts && !dev) throw std::runtime_error("post_events: device counters need the device path");
    A.ctx_trans = ctx_trans; A.ctx_acc = ctx_acc;
    A.hits = P<const int64_t>(hits); A.nh = nh; A.ev_cnt = P<const int64_t>(ev_cnt);
    A.ev_end = P<const int64_t>(ev_end); A.ne = ne; A.L = L; A.lbits = lbits; A.ev = ev_from(ev);
    A.text = P<const uint8_t>(text); A.ls = P<const int64_t>(ls); A.ll = P<const int32_t>(ll); A.dfa = dfa_from(dfa);
    A.ev_line = P<int32_t>(ev_line); A.ev_pat = P<int32_t>(ev_pat); A.ev_seg = P<int32_t>(ev_seg);
    A.ev_rank = P<int64_t>(ev_rank); A.ev_fkey = P<int64_t>(ev_fkey); A.freq_counts = P<int64_t>(freq_counts);
    A.feat = P<uint8_t>(feat); A.cov = P<int32_t>(cov);
    if (dev) return events_dev(A, P<void>(ws), ws_bytes, s);
    py::gil_scoped_release nogil;
    events_host(A);
    return 0;
  });
  m.def("blk_index", [](uint64_t ls, int64_t L, int64_t nblocks, uint64_t blk, uint64_t s, bool dev) {
    if (dev) blk_index_dev(P<const int64_t>(ls), L, nblocks, P<int32_t>(blk), s);
    else blk_index_host(P<const int64_t>(ls), L, nblocks, P<int32_t>(blk));
  });

  m.def("seq_chain", [](uint64_t slot_seq, uint64_t off, uint64_t reg, uint64_t hoff, uint64_t hline, int32_t lo,
                        int32_t hi, int n, uint64_t out, uint64_t s, bool dev) {
    if (dev)
      seq_chain_dev(P<const int32_t>(slot_seq), P<const int32_t>(off), P<const int32_t>(reg), P<const int64_t>(hoff),
                    P<const int32_t>(hline), lo, hi, n, P<int32_t>(out), s);
    else
      seq_chain_host(P<const int32_t>(slot_seq), P<const int32_t>(off), P<const int32_t>(reg), P<const int64_t>(hoff),
                     P<const int32_t>(hline), lo, hi, n, P<int32_t>(out));
  });

  m.def("nfa", [](uint64_t groups, uint64_t glist, int ng, int ncls, uint64_t lines, int64_t nsel, uint64_t text,
                  uint64_t ls, uint64_t ll, uint64_t feat, uint64_t hits, int64_t cap, uint64_t count, uint64_t s,
                  bool dev) -> int64_t {
    if (dev) {
      nfa_mfma_dev(P<const uint64_t>(groups), P<const int32_t>(glist), ng, ncls, P<const int32_t>(lines), nsel,
                   P<const uint8_t>(text), P<const int64_t>(ls), P<const int32_t>(ll), P<uint8_t>(feat),
                   P<int64_t>(hits), cap, P<unsigned long long>(count), s);
      return -1;
    }
    return nfa_host(P<const uint64_t>(groups), P<const int32_t>(glist), ng, P<const int32_t>(lines), nsel,
                    P<const uint8_t>(text), P<const int64_t>(ls), P<const int32_t>(ll), P<uint8_t>(feat),
                    P<int64_t>(hits), cap);
  });

  // ---- JSON result emitter
  py::class_<PatternTable>(m, "PatternTable")
      .def(py::init<py::list, py::array_t<int32_t>, py::array_t<int32_t>>())
      .def("set_severity", &PatternTable::set_severity);
  m.def("emit_batch_results", &emit_batch_results_py, py::arg("table"), py::arg("buf"), py::arg("line_start"),
        py::arg("line_len"), py::arg("doc_line_off"), py::arg("ev_line"), py::arg("ev_pat"), py::arg("ev_score"),
        py::arg("ev_doc_off"), py::arg("processing_ms"), py::arg("meta_tail"), py::arg("nthreads") = 1);
  m.def("emit_events_json", &emit_events_json_py);
  m.def("emit_batch_json", &emit_batch_json_py, py::arg("table"), py::arg("buf"), py::arg("line_start"),
        py::arg("line_len"), py::arg("doc_line_off"), py::arg("ev_line"), py::arg("ev_pat"), py::arg("ev_score"),
        py::arg("ev_doc_off"), py::arg("nthreads") = 1);
}
