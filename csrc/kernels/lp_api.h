// Launch / host entry points of lp_kernels.hip (bound to Python in csrc/bind.cpp).
#pragma once
#include <stdint.h>

#include <vector>

#include "lp_core.h"

namespace lp {

// worker threads of the host twins (CPU backend)
void set_host_threads(int n);
// lanes per gram hit of the bulk literal verify (k_pf_verify; A/B knob, default 4)
void set_pf_verify_lanes(int n);
// bulk scan walk: hot blocks re-walked by a second kernel (k_scan_rare) instead of inline (A/B knob)
bool scan_defer_rare();
void set_scan_defer_rare(bool on);
// request path: BPG and DFA candidates verified in ONE launch (k_bpg_coop mode 2, default) or in
// two (k_cand_verify, then the BPG walk) -- the diagnostic split shows each half's time
void set_cand_verify_split(bool on);
// event top-k by threshold selection (summarize.hip k_sel_*, default) or the chunk-sort levels
bool summ_select();
void set_summ_select(bool on);
// diagnostic: phase clocks of k_hits_small / k_events_small into a device int64[16] (0: off)
void set_small_profile(uint64_t dev_ptr);
// line-index pass 1 folded into the bulk prefilter (line_index.hip k_nl_count's outputs): per 16 KiB
// tile the '\n' count and the "\r\n" flag (both zeroed by the caller), per 64 bytes a '\n' bitmask
struct NlOut {
  uint64_t* nlm = nullptr;   // [ntiles * 256]
  int32_t* cnt = nullptr;    // [ntiles]
  int32_t* crf = nullptr;    // [ntiles]
  int64_t ntiles = 0;
};
void prefilter_dev(const uint8_t* text, int64_t nbytes, const PfTables& T, const int64_t* line_start, int64_t nlines,
                   int64_t* cand, int64_t cap, unsigned long long* count, int grid, uint64_t stream,
                   const NlOut* nl = nullptr);
void pf_verify_dev(const int64_t* ghits, int64_t n, const uint8_t* text, int64_t nbytes, const PfTables& T,
                   const int64_t* line_start, int64_t nlines, const int32_t* blk_line, int64_t* cand, int64_t cap,
                   unsigned long long* count, uint64_t stream, const unsigned long long* dn = nullptr,
                   int max_grid = 8192);
// bit-parallel Glushkov programs (bpg.hip): candidate verify (small path, in place), first-of-run
// verify of sorted keys (bulk path, flags), all-lines scan of literal-free programs
void bpg_cand_dev(int64_t* cand, int64_t cap, const unsigned long long* dcount, const uint8_t* text, const int64_t* ls,
                  const int32_t* ll, const DfaPool& P, uint64_t stream);
// request path: DFA candidates (grid's upper half) and BPG candidates (lower half, cooperative walk)
// verified in place by ONE launch; false (nothing launched) when the library has no BPG programs
bool cand_verify_all_dev(int64_t* cand, int64_t cap, const unsigned long long* dcount, const uint8_t* text,
                         const int64_t* ls, const int32_t* ll, const DfaPool& P, uint64_t stream);
// wcnt / wlist (optional): a counter zeroed in stream order before the call and n uint32 of scratch --
// keys of programs wider than 8 words are listed there and walked one lane group per key
// std_key (optional): the DFA dedupe-verify of every key (k_dedupe_verify's flag / std_key) runs in
// the same launch; returns false when nothing was launched (no BPG program) -- the caller then runs
// the DFA dedupe-verify itself
bool bpg_dedupe_dev(const uint64_t* keys, int64_t n, int lbits, const uint8_t* text, const int64_t* ls,
                    const int32_t* ll, const DfaPool& P, uint8_t* flag, uint64_t stream, uint32_t* wcnt = nullptr,
                    uint32_t* wlist = nullptr, int64_t* std_key = nullptr);
void bpg_scan_dev(const uint8_t* text, const int64_t* ls, const int32_t* ll, int64_t L, const int32_t* regs,
                  int nregs, const DfaPool& P, int64_t* out, int64_t cap, unsigned long long* count,
                  uint64_t stream);
// backtracker regexes fed by their relaxed automata (side_path.hip): export of the candidates to
// pinned host memory (keys / starts / lens / host_cnt / host_seq are device-visible pointers of
// pinned host memory; cnt / done_blocks device words, zero between uses). keys == null: drop mode.
struct HostSideOut {
  int64_t* keys = nullptr;
  int64_t* starts = nullptr;
  int64_t* lens = nullptr;
  int64_t cap = 0;
  unsigned long long* cnt = nullptr;
  unsigned int* done_blocks = nullptr;
  int64_t* host_cnt = nullptr;
  int64_t* host_seq = nullptr;
  int64_t seq = 0;
};
// ... and the host's verified keys (pinned, device-visible), published with host_seq == seq
struct HostSideIn {
  const int64_t* keys = nullptr;
  const int64_t* host_cnt = nullptr;
  const int64_t* host_seq = nullptr;
  int64_t cap = 0;
  int64_t seq = 0;
  long long timeout_ticks = 200000000;   // wall_clock64 ticks (100 MHz): 2 s
  int64_t* err = nullptr;                // set to 1 when the host did not answer in time
};
void take_host_dev(int64_t* cand, const unsigned long long* n1d, int64_t cap1, int64_t* ver,
                   const unsigned long long* n2d, int64_t cap2, const uint8_t* text, const int64_t* ls,
                   const int32_t* ll, const DfaPool& P, const HostSideOut& O, uint64_t stream);
void wait_host_dev(int64_t* ver, int64_t cap2, unsigned long long* n2d, const HostSideIn& I, uint64_t stream);

// host-verified keys appended to a verified-hit buffer at its device counter (k_append_keys)
void append_keys_dev(int64_t* dst, int64_t cap, unsigned long long* count, const int64_t* src, int64_t n,
                     uint64_t stream);
void scan_dev(const uint8_t* text, const int64_t* line_start, const int32_t* line_len, int64_t nlines,
              const int32_t* regs, int nregs, const DfaPool& P, int64_t* out, int64_t cap, unsigned long long* count,
              uint64_t stream);
void score_dev(const int32_t* ev_line, const int32_t* ev_pat, const int32_t* ev_seg, const FreqIn& F, int64_t n,
               const ScoreTables& T, const ScoreParams& S, double* out, double* factors, uint64_t stream,
               const int64_t* dn = nullptr);   // dn: device event count (n = capacity)

void seq_chain_dev(const int32_t* slot_seq, const int32_t* seq_ev_off, const int32_t* seq_ev_reg,
                   const int64_t* hit_off, const int32_t* hit_line, int32_t own_lo, int32_t own_hi, int nslots,
                   int32_t* out, uint64_t stream);
void seq_chain_host(const int32_t* slot_seq, const int32_t* seq_ev_off, const int32_t* seq_ev_reg,
                    const int64_t* hit_off, const int32_t* hit_line, int32_t own_lo, int32_t own_hi, int nslots,
                    int32_t* out);
int64_t nl_positions_host(const uint8_t* text, int64_t nbytes, int64_t* nl_pos);
// AVX-512 bloom tier of the host twin (prefilter_cpu.cpp): 4-gram-only bloom, no Teddy tier;
// handles positions from the 4-aligned point at or after `a` in 64-byte steps, returns where it stopped
bool prefilter_bloom_simd_ok();
int64_t prefilter_bloom_simd(const uint8_t* text, int64_t nbytes, const PfTables& T, const int64_t* line_start,
                             int64_t nlines, int64_t a, int64_t b, std::vector<int64_t>& out);
int64_t prefilter_teddy_simd(const uint8_t* text, int64_t nbytes, const PfTables& T, const int64_t* line_start,
                             int64_t nlines, int64_t a, int64_t b, std::vector<int64_t>& out);
int64_t prefilter_host(const uint8_t* text, int64_t nbytes, const PfTables& T, const int64_t* line_start,
                       int64_t nlines, int64_t* cand, int64_t cap);
int64_t scan_host(const uint8_t* text, const int64_t* line_start, const int32_t* line_len, int64_t nlines,
                  const int32_t* regs, int nregs, const DfaPool& P, int64_t* out, int64_t cap);
void score_host(const int32_t* ev_line, const int32_t* ev_pat, const int32_t* ev_seg, const FreqIn& F, int64_t n,
                const ScoreTables& T, const ScoreParams& S, double* out, double* factors);

}  // namespace lp

namespace lp {
void nfa_mfma_dev(const uint64_t* groups, const int32_t* group_list, int ngroups, int ncls, const int32_t* lines,
                  int64_t nsel, const uint8_t* text, const int64_t* line_start, const int32_t* line_len,
                  uint8_t* feat, int64_t* hits, int64_t cap, unsigned long long* count, uint64_t stream);
int64_t nfa_host(const uint64_t* groups, const int32_t* group_list, int ngroups, const int32_t* lines, int64_t nsel,
                 const uint8_t* text, const int64_t* line_start, const int32_t* line_len, uint8_t* feat,
                 int64_t* hits, int64_t cap);
}  // namespace lp

// ---- literal-free scan (scan_multi.hip): up to 4 multi-regex DFA groups per pass, tables in LDS
namespace lp {
struct ScanPass {
  const uint32_t* blob;   // device (or host) copy of the whole blob; layout in scan_multi.hip
  int lds_words;          // leading words staged in LDS: u16 rows + bm4 (multiple of 4)
  int ngroups;            // 1..4
  int row_base[4];        // u16 index of group g's first row
  int stride[4];          // row stride (u16 entries, odd)
  int thr[4];             // first row index of a state from which a regex can accept
  int init_row[4];        // row index of the start state
  uint32_t init_state[4]; // start state id (exact tables)
  int ncol[4];            // columns: hold, '\n', byte classes
  int gt_off[4];          // word offset of group g's exact [state][ncol] next-state table
  int gm_off[4];          // word offset of group g's [state][ncol] accept masks (same indexing)
  int fin_off[4];         // word offset of group g's [state][EOL, FT] accept masks
  int bm_off;             // word offset of bm4
  int rid_off;            // word offset of the regex ids (64 per group)
  int am_off;             // word offset (even) of the u64 accept masks laid out like the LDS rows
};
void scan_multi_dev(const uint8_t* text, int64_t nbytes, const int64_t* line_start, const int32_t* line_len, int64_t nlines,
                    const ScanPass& S, int64_t* out, int64_t cap, unsigned long long* count, int grid,
                    uint64_t stream);
int64_t scan_multi_host(const uint8_t* text, const int64_t* line_start, const int32_t* line_len, int64_t nlines,
                        const ScanPass& S, int64_t* out, int64_t cap);
}  // namespace lp

// ---- device-resident frequency state (freq_state.hip)
namespace lp {
struct FreqRing {
  double* t;          // [cap] batch timestamps (seconds)
  int32_t* key;       // [cap] frequency key
  int32_t* cnt;       // [cap] matches of the key in that batch
  int64_t cap;
  int64_t* ht;        // [2] head, tail positions (monotonic)
  int64_t* tot;       // [K] in-window matches per key
  uint8_t* seen;      // [K]
};
void freq_evict(const FreqRing& R, double horizon, uint64_t stream, bool dev);
// gate (device, optional): record only when cnt[0..2] <= cap[0..2] and cnt[4] <= cap[3] -- the
// request runner's matcher / event capacities held, so the counts are this batch's real ones
struct RecordGate {
  const int64_t* cnt = nullptr;
  int64_t cap[4] = {0, 0, 0, 0};
  const int64_t* veto = nullptr;   // (device) record only when *veto == 0: a DP step's overflow veto
};
void freq_record(const int64_t* counts, int K, double now, const FreqRing& R, uint64_t stream, bool dev,
                 const RecordGate& gate = RecordGate());
}  // namespace lp

// ---- line index (line_index.hip)
namespace lp {
struct LineIndexWs {
  int64_t* buf;                // [4 * ntiles_cap] tile offsets, first line ends (line, end), counts;
  int64_t ntiles_cap;          // then tmp_bytes of scan scratch
  size_t tmp_bytes;
};
int64_t line_index_tiles(int64_t nbytes);
// starts/lens [cap]; info[0] = '\n' count, info[1] = last '\n' (or -1), info[2] = lines after
// Java's trailing-empty trimming (trim only). Lines = info[0] + 1 before trimming.
// blk (optional) [nblk]: line holding byte b << 12 (the coarse index of lp_core.h locate_line)
void line_index_dev(const uint8_t* text, int64_t nbytes, const LineIndexWs& W, int64_t* starts, int32_t* lens,
                    int64_t cap, int64_t* info, bool trim, int32_t* blk, int64_t nblk, uint64_t stream,
                    bool counted = false);
// the workspace views pass 1 writes (counted = true: a fused prefilter already wrote them); zeroes
// the counts and flags on `stream`
NlOut line_index_pass1_views(const LineIndexWs& W, int64_t nbytes, uint64_t stream);
}  // namespace lp

// ---- DP step bookkeeping (dp_glue.hip)
namespace lp {
struct DpCarryArgs {
  const int64_t* g;          // [world][1 + nk + ns] gathered payloads
  int world, rank, nk, ns;
  int64_t halo_left;
  const int64_t* tot;        // [nk] persistent window totals (may be null)
  const int64_t* slot_e0;    // [ns] first slot of each sequence-event slot's sequence
  const int64_t* slot_k;     // [ns] event index of the slot
  // outputs
  int64_t* own_start; int64_t* g0; int64_t* n;   // [1] each
  int64_t* carry;            // [nk]
  uint8_t* seq_carry;        // [ns]
  int64_t* red_tail;         // [nk] this rank's counts into the all-reduce buffer (may be null)
  int64_t* veto = nullptr;   // [1] OR of every rank's overflow flag (may be null)
  int64_t* zero = nullptr;   // [nzero] zeroed (this rank's histogram slots of the all-gather buffer)
  int64_t nzero = 0;
  // a stream of DP steps (parallel/stream.py ShardedStreamAnalyzer): the carries of the earlier
  // steps -- sequence-chain state before this step, global index of its first line, an open N
  // (chronological factor rescored at the end) -- and the state after the step (every rank composed)
  const uint8_t* seq_base = nullptr;   // [ns] or null (= nothing matched before the step)
  int64_t line_base = 0;
  int64_t n_fixed = 0;                 // > 0: N written as this instead of the step's line count
  uint8_t* seq_next = nullptr;         // [ns] or null
};
// payload [1 + nk + ns + 1]; cnt (device [5] match / event counters, may be null) and caps (host
// [4]: gram, candidate, verified, event capacities) set the trailing overflow flag
void dp_pack(int64_t own_lines, const int64_t* freq, int nk, const int32_t* chain, int ns, int64_t* pack,
             uint64_t stream, bool dev, const int64_t* cnt = nullptr, const int64_t* caps = nullptr);
void dp_carry(const DpCarryArgs& A, uint64_t stream, bool dev);
}  // namespace lp

// ---- summary + top-k, streaming re-score (summarize.hip)
namespace lp {
struct SummIn {
  // events (level 0): score[i], pattern pat[i], global line = (line64 ? line64 : line32)[i] + *line_add
  const double* score;
  const int32_t* pat;
  const int32_t* line32;
  const int64_t* line64;
  const int64_t* line_add;   // device (host twin: host) scalar, may be null
  const int32_t* sev_of_pat; // [P] severity index 0..4
  // or rows [n][3] = (score, line, pattern) as float64 (merging top-k lists)
  const double* rows;
  // optional (events): every event packed as [global line int64 x n][score f64 x n][pattern i32 x n]
  void* ev_out = nullptr;
  // optional (events): device event count; n is then a capacity and the level-0 pass reads
  // min(n, *dn) events (ev_out packed at stride min(n, *dn))
  const int64_t* dn = nullptr;
};
// writes the k best rows (score desc, line asc, pattern asc; missing rows = (-inf, -1, -1)) and,
// from events, adds the pattern / severity histograms. Device: returns workspace bytes, runs only
// when ws_bytes suffices.
size_t summarize_dev(const SummIn& in, int64_t n, int k, int nsev, double* top_rows, unsigned long long* pat_hist,
                     unsigned long long* sev_hist, void* ws, size_t ws_bytes, uint64_t stream);
void summarize_host(const SummIn& in, int64_t n, int k, double* top_rows, int64_t* pat_hist, int64_t* sev_hist);
void rescore_dev(const int64_t* gl, const double* fac, int64_t n, int64_t N, const ScoreParams& S, double* out,
                 uint64_t stream);
void rescore_host(const int64_t* gl, const double* fac, int64_t n, int64_t N, const ScoreParams& S, double* out);
}  // namespace lp

// ---- post-match pipeline (lp_post.hip): hit CSR, events, frequency ranks, context features
namespace lp {
struct EvTables {
  const int64_t* prim_off;   // [R+1] patterns whose primary regex is r: prim_pats[prim_off[r]..]
  const int32_t* prim_pats;
  const int32_t* freq_key;   // [P] frequency key, -1 = pattern without id
  const int32_t* ctx_before; // [P] -1 = no context rules
  const int32_t* ctx_after;
  const int32_t* seg_lo; const int32_t* seg_hi; const int32_t* own_lo; const int32_t* own_hi;
  int nseg;
  int nkeys;
  int pbits;                 // bits of a pattern index
};

struct HitsArgs {
  const int64_t* cand;       // (regex << 32 | line): [0, pre_from) to DFA-verify, [pre_from, n) pre-verified
  int64_t n, pre_from;
  // device-count mode (dcount != null): cand[0, pre_from) and cand2[0, n - pre_from) are two
  // fixed-capacity regions whose used lengths are the device counters dcount[0] / dcount[1]
  // (the matchers' append counters: no host read between matching and the hit CSR)
  const int64_t* cand2 = nullptr;
  const unsigned long long* dcount = nullptr;
  int lbits, rbits, R;
  const uint8_t* text; const int64_t* ls; const int32_t* ll;
  DfaPool dfa;
  EvTables ev;
  // outputs (capacity n; hit_off R+1)
  int64_t* hits; int32_t* hit_line; int64_t* hit_off; int64_t* ev_cnt; int64_t* ev_end;
  int64_t* counters;         // [0] unique verified hits, [1] events
  bool cand_verified = false;  // small path: the caller ran cand_verify_all_dev already
};

struct EventsArgs {
  const int64_t* hits; int64_t nh;
  const int64_t* ev_cnt; const int64_t* ev_end;
  int64_t ne, L;
  int lbits;
  EvTables ev;
  const uint8_t* text; const int64_t* ls; const int32_t* ll;
  DfaPool dfa;
  int ctx_trans, ctx_acc;    // table extents of the 4 context DFAs (pool entries 0..3), for LDS staging
  // device-count mode (request path): [nh, ne] on the device; nh / ne above are then capacities
  // and a batch over them leaves the outputs unset (the caller re-runs with host counts)
  const int64_t* dcounts = nullptr;
  // device-count mode, bulk path (optional): receives the event count when the events fit ne, else
  // 0 -- the count every later kernel of the batch reads (event fields past it are unset)
  int64_t* ne_fit = nullptr;
  // outputs
  int32_t* ev_line; int32_t* ev_pat; int32_t* ev_seg; int64_t* ev_rank; int64_t* ev_fkey;
  int64_t* freq_counts;      // [nkeys]
  uint8_t* feat;             // [L] context features (nullptr: coverage only)
  int32_t* cov;              // [L] optional: window coverage out
  bool feat_ready = false;   // feat already holds every line's features (feat_all_dev): skip them
};

int bits_for(int64_t n);
// device versions return the workspace bytes they need; they only run when ws_bytes suffices
size_t hits_dev(const HitsArgs& A, void* ws, size_t ws_bytes, uint64_t stream);
// context features of EVERY line (k_feat_cov without a coverage filter): the request runner computes
// them on its side stream while the matchers run, so the event stage needs no feature pass
void feat_all_dev(int64_t L, const uint8_t* text, const int64_t* ls, const int32_t* ll, const DfaPool& P,
                  int ctx_trans, int ctx_acc, uint8_t* feat, uint64_t stream);
size_t events_dev(const EventsArgs& A, void* ws, size_t ws_bytes, uint64_t stream);

// A request's tail in one workgroup (lp_post.hip k_request_tail): hits_dev's and events_dev's small
// paths (device-count mode, features computed already), score_dev and publish_record_dev in one
// launch. The results layout is publish_record_dev's.
struct RequestTailOut {
  double* score;             // = (double*)out: the score column of the results buffer
  const uint8_t* out;        // results [score f64 x E | counts i64 x K1 | line | pattern | seg i32 x E]
  int64_t E;                 // the results' event capacity
  int K1;                    // max(nkeys, 1)
  const int64_t* cnt;        // device counters [gram, cand, ver, hits, events]
  int64_t* cnt_host;         // device views of the pinned host counters / results
  uint8_t* res_host;
  const int64_t* counts;     // the batch's per-key counts (results buffer) for the record
  int K;                     // frequency keys
  double now;
  FreqRing ring;
  RecordGate gate;
};
void request_tail_dev(const HitsArgs& HA, const EventsArgs& EA, const ScoreTables& T, const ScoreParams& S,
                      const FreqIn& F, const RequestTailOut& P, void* ws, size_t ws_bytes, uint64_t stream);
// capacities of the single-workgroup request path (events, lines): a batch within them can run
// the event stage in device-count mode
int64_t request_event_cap();
int64_t request_line_cap();
// device-count-mode results -> pinned host memory (request_io.hip): the 5 matcher/event counters
// and the results compacted to stride ne (cnt[4]) when ne <= E; both pointers device-visible
// n16 16-byte words from device-visible pinned host memory (host_dev) into device memory
// (evict: block 0 also runs the frequency window's eviction at `horizon`, as k_freq_evict)
void fetch_dev(const void* host_dev, void* dst, int64_t n16, uint64_t stream, const FreqRing* evict = nullptr,
               double horizon = 0.0);
void publish_dev(const int64_t* cnt, const uint8_t* out, int64_t E, int K1, int64_t* cnt_host, uint8_t* res_host,
                 uint64_t stream);
// publish_dev + the batch's gated frequency record (k_freq_record) in one launch
void publish_record_dev(const int64_t* cnt, const uint8_t* out, int64_t E, int K1, int64_t* cnt_host,
                        uint8_t* res_host, const int64_t* counts, int K, double now, const FreqRing& R,
                        const RecordGate& G, uint64_t stream);
void blk_index_dev(const int64_t* ls, int64_t L, int64_t nblocks, int32_t* blk, uint64_t stream);
void hits_host(const HitsArgs& A);
void events_host(const EventsArgs& A);
void blk_index_host(const int64_t* ls, int64_t L, int64_t nblocks, int32_t* blk);
}  // namespace lp
