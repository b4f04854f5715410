// java.util.regex (Java 21 defaults) -> automata for the MI355X log engine.
//
// Pipeline (host C++, run once per distinct regex at library load -- the reference recompiles
// every regex on every request, AnalysisService.java:55-86):
//   parse (Java syntax) -> AST over CODE POINTS: every character / class / property is one exact
//          code-point set (sorted disjoint ranges), flags resolved at parse time (CASE_INSENSITIVE
//          with or without UNICODE_CASE, UNICODE_CHARACTER_CLASS, DOTALL, UNIX_LINES, MULTILINE,
//          COMMENTS), Unicode properties from generated tables (unicode_tables.inc)
//   AST -> required-literal factor set (prefilter keys)
//   AST -> byte AST (code-point sets lowered to UTF-8 byte sequences) -> Glushkov NFA over bytes
//          -> byte DFA (subset construction; absorbing DEAD=0 / ACCEPT=1; end-of-line flags)
//   AST -> Glushkov NFA over code points (one position per character / class) -> bit-parallel
//          Glushkov program (bpg_program) for regexes whose DFA blows up or that need code-point
//          boundary contexts (MULTILINE ^ $, Unicode \b)
//
// Only boolean find() is ever used by the reference (AnalysisService.java:95,
// ScoringService.java:281,300,330), so language membership of ".*R.*" is all that matters and
// an automaton is exact for the regular subset. Non-regular / language-changing constructs
// (backrefs, lookaround, possessive, atomic groups) raise Unsupported -> the host backtracker.
#pragma once
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace lp {

struct SyntaxError : std::runtime_error { using std::runtime_error::runtime_error; };
struct Unsupported : std::runtime_error { using std::runtime_error::runtime_error; };

// Boundary contexts: prev in {BOS=0, W=1, N=2, T=3} x next in {EOS=0, FT=1, W=2, N=3, C=4, T=5},
// ctx index = prev * 6 + next (24 contexts). FT = "before the final line terminator".
//   W / N: word / other character (ASCII word characters; Unicode WORD under (?U) \b)
//   T: a line terminator character (\r U+0085 U+2028 U+2029) -- code-point level only, the
//      MULTILINE anchors test it
//   C: the next byte is a UTF-8 continuation byte (a boundary inside one code point) -- byte level
//      only; no assertion holds there, so assertions are only evaluated between whole characters
enum : int { P_BOS = 0, P_W = 1, P_N = 2, P_T = 3 };
enum : int { N_EOS = 0, N_FT = 1, N_W = 2, N_N = 3, N_C = 4, N_T = 5 };
constexpr int NCTX = 24;
constexpr uint32_t CTX_ALL = (1u << NCTX) - 1;
constexpr uint32_t CTX_NOT_BOS = CTX_ALL & ~0x3Fu;      // prev != BOS
inline int ctx_index(int prev, int next) { return prev * 6 + next; }

struct ByteSet {
  uint64_t w[4] = {0, 0, 0, 0};
  void set(int b) { w[b >> 6] |= 1ull << (b & 63); }
  bool test(int b) const { return (w[b >> 6] >> (b & 63)) & 1; }
  void set_range(int lo, int hi) { for (int b = lo; b <= hi; ++b) set(b); }
  ByteSet operator|(const ByteSet& o) const { ByteSet r; for (int i = 0; i < 4; ++i) r.w[i] = w[i] | o.w[i]; return r; }
  bool operator==(const ByteSet& o) const { return w[0]==o.w[0]&&w[1]==o.w[1]&&w[2]==o.w[2]&&w[3]==o.w[3]; }
  bool empty() const { return !(w[0] | w[1] | w[2] | w[3]); }
  int count() const { return __builtin_popcountll(w[0]) + __builtin_popcountll(w[1]) + __builtin_popcountll(w[2]) + __builtin_popcountll(w[3]); }
};

// Exact set of Unicode code points: sorted, disjoint, non-adjacent [lo, hi] ranges.
struct CpSet {
  std::vector<std::pair<uint32_t, uint32_t>> r;
  static constexpr uint32_t MAX = 0x10FFFF;
  void add(uint32_t c) { add_range(c, c); }
  void add_range(uint32_t lo, uint32_t hi);
  void unite(const CpSet& o);
  void intersect(const CpSet& o);
  void negate();
  bool contains(uint32_t c) const;
  bool covers(uint32_t lo, uint32_t hi) const;       // [lo, hi] entirely inside
  bool touches(uint32_t lo, uint32_t hi) const;      // [lo, hi] intersects
  bool empty() const { return r.empty(); }
  uint64_t count() const;
  bool operator==(const CpSet& o) const { return r == o.r; }
};

enum class Kind : int { DFA = 0, NFA = 1, FALLBACK = 2, INVALID = 3 };

struct Edge { int to; uint32_t cond; };

struct Nfa {
  int npos = 0;
  std::vector<ByteSet> cls;                 // byte level: per position byte class
  std::vector<CpSet> ccls;                  // code-point level: per position code-point class
  std::vector<std::vector<Edge>> follow;    // per position
  std::vector<Edge> first;                  // (pos, cond)
  std::vector<Edge> last;                   // (pos, cond)
  uint32_t nullable = 0;                    // contexts in which the empty string matches
  // code-point NFAs built with counters: ctr[p] = B > 0 makes p a COUNTED position -- the optional
  // part C{0,B} of a bounded repeat of one character class, one position instead of B. Its self
  // loop is NOT in follow[p]; it is taken while the youngest thread in p has consumed < B
  // characters (bpg.h: the walk keeps one count per counted position). Empty: no counters.
  std::vector<int> ctr;
};

struct Dfa {
  int nstates = 0;                          // incl. DEAD(0) ACCEPT(1) INIT(2)
  int nclasses = 0;
  std::vector<uint8_t> bytemap;             // 256 -> class
  std::vector<uint16_t> trans;              // nstates * nclasses
  std::vector<uint8_t> accflags;            // per state: bit0 accept at EOS, bit1 accept before FT
  bool anchored = false;                    // no restart after BOS -> DEAD reachable
};

struct Compiled {
  Kind kind = Kind::INVALID;
  bool wordb = false;                       // uses \b / \B (prev-character wordness matters)
  bool uword = false;                       // \b / \B with Unicode WORD semantics ((?U))
  bool cp_only = false;                     // needs code-point contexts: no byte automaton (DFA / MFMA)
  std::string error;                        // reason for NFA / FALLBACK / INVALID
  std::vector<std::string> literals;        // OR-set of required factors (ASCII-lowercased bytes)
  bool has_literals = false;
  bool bt_ok = false;                       // the native backtracker (BtRegex) runs it
  bool byte_nfa = false;                    // nfa holds the byte-level Glushkov NFA (DFA / MFMA engines)
  Nfa nfa;
  Dfa dfa;
  std::vector<uint64_t> bpg;                // kind NFA: bit-parallel Glushkov program (empty: none)
};

// max_positions bounds the byte-level NFA; the code-point NFA of a BPG program has <= BPG_MAX_POS.
Compiled compile(const std::string& pattern, int max_dfa_states, int max_positions);

// Multi-regex DFA ("scan group"): the Glushkov NFAs of up to 32 regexes determinised TOGETHER, so
// one table walk per byte answers find() for all of them (Aho-Corasick / RE2::Set style). Used
// for regexes without a usable literal factor, which must be run over every line. Unlike the
// single-regex DFA there is no absorbing ACCEPT state: a transition reports the regexes that
// accept BEFORE its byte and the walk goes on for the others.
//   trans[s * nclasses + cls] = next state (< 65536), acc[same] = accept mask of that transition
//   fin[2 s] = regexes accepting at end of line, fin[2 s + 1] = before a final line terminator
// State 0 = DEAD (every member anchored and failed), state 1 = start of line.
constexpr int MULTI_MAX_REGS = 64;
struct MultiDfa {
  int nstates = 0, nclasses = 0, nregs = 0;
  std::vector<uint8_t> bytemap;
  std::vector<uint32_t> trans;
  std::vector<uint64_t> acc;   // bit r: member r (64-bit masks: up to 64 members per walk)
  std::vector<uint64_t> fin;
};
// throws Unsupported (state limit, > MULTI_MAX_REGS, a member without a byte automaton)
MultiDfa compile_multi(const std::vector<std::string>& patterns, int max_states);
// bit r set <=> patterns[r] finds a match in s[0..n) (host walk; the device kernel is k_scan_multi)
uint64_t multi_find(const MultiDfa& d, const uint8_t* s, int64_t n);

// Host-side exact match of one line with a compiled DFA (CPU backend + tests).
bool dfa_find(const Dfa& d, const uint8_t* s, int64_t n);
// Length in bytes of a final line terminator (\r, U+0085, U+2028, U+2029) ending s[0..n), or 0.
int final_terminator_len(const uint8_t* s, int64_t n);

// ---- bit-parallel Glushkov programs over code points (layout: csrc/kernels/bpg.h) ----------
constexpr int BPG_MAX_POS = 2048;         // 32 words of 64 positions
constexpr int BPG_MAX_EXC = 256;
constexpr int BPG_MAX_CLS = 1023;
// bounded repeats C{m,n} of ONE character class with n - m >= BPG_CTR_MIN become m plain positions
// plus one counted position (Nfa::ctr): X.{0,20000}Y is 3 positions, not 20,002. A program holds
// at most BPG_MAX_CTR counters (more: the repeats are expanded, the pre-counter behaviour).
constexpr int BPG_CTR_MIN = 16;
constexpr int BPG_MAX_CTR = 4;
// code-point NFA -> program; throws Unsupported when it does not fit
std::vector<uint64_t> bpg_program(const Nfa& cnfa, bool uword);

// Java-semantics backtracking matcher (boolean Matcher.find()) for the regexes no automaton can
// express: backreferences, lookahead / lookbehind, atomic groups, possessive quantifiers. The same
// parser builds the AST, lowered to UTF-8 bytes (ASCII or Unicode \b, CI flags), which is compiled
// to a small backtracking program run in Java's priority order (greedy/reluctant, left
// alternative first) -- so atomic / possessive constructs keep exactly the matches Java keeps.
// Host-only; the device prefilter narrows it to candidate lines.
class BtRegex {
 public:
  explicit BtRegex(const std::string& pattern);    // throws SyntaxError / Unsupported
  // steps: optional out-count of VM steps; a find exceeding `budget` steps returns false
  bool find(const uint8_t* s, int64_t n, int64_t budget = int64_t(1) << 27, bool* exhausted = nullptr) const;
  struct Impl;
 private:
  std::shared_ptr<const Impl> p_;
};

// Unicode tables (unicode_tables.inc) for tests / tools: the named set (jregex key, e.g.
// "gc:Lu", "sc:LATIN", "blk:BASICLATIN"); empty when unknown.
CpSet unicode_set(const std::string& key);

}  // namespace lp
