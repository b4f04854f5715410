// java.util.regex (Java 21 defaults) -> byte-level automata for the MI355X log engine.
//
// Pipeline (host C++, run once per distinct regex at library load — the reference recompiles
// every regex on every request, AnalysisService.java:55-86):
//   parse (Java syntax subset) -> AST
//   AST -> required-literal factor set (prefilter keys)
//   AST -> Glushkov position NFA whose edges carry *boundary-context* conditions
//          (^ $ \b \B \A \z \Z as zero-width assertions)
//   NFA -> byte DFA (subset construction, previous-byte wordness folded into the state,
//          absorbing DEAD=0 / ACCEPT=1 states, per-state accept flags for end-of-line).
//
// Only boolean find() is ever used by the reference (AnalysisService.java:95,
// ScoringService.java:281,300,330), so language membership of ".*R.*" is all that matters and
// an automaton is exact for the regular subset. Non-regular / language-changing constructs
// (backrefs, lookaround, possessive, atomic groups) raise Unsupported -> host fallback.
#pragma once
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace lp {

struct SyntaxError : std::runtime_error { using std::runtime_error::runtime_error; };
struct Unsupported : std::runtime_error { using std::runtime_error::runtime_error; };

// Boundary contexts: prev in {BOS=0, W=1, N=2} x next in {EOS=0, FT=1, W=2, N=3, C=4}
// ctx index = prev*5 + next (15 contexts). FT = "before the final line terminator".
enum : int { P_BOS = 0, P_W = 1, P_N = 2 };
// N_C: the next byte is a UTF-8 continuation byte (a boundary inside one code point); no
// assertion holds there, so assertions are only ever evaluated between whole characters.
enum : int { N_EOS = 0, N_FT = 1, N_W = 2, N_N = 3, N_C = 4 };
constexpr uint16_t CTX_ALL = 0x7FFF;                    // 15 contexts
constexpr uint16_t CTX_NOT_BOS = 0x7FE0;                // prev != BOS
inline int ctx_index(int prev, int next) { return prev * 5 + next; }

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

enum class Kind : int { DFA = 0, NFA = 1, FALLBACK = 2, INVALID = 3 };

struct Edge { int to; uint16_t cond; };

struct Nfa {
  int npos = 0;
  std::vector<ByteSet> cls;                 // per position byte class
  std::vector<std::vector<Edge>> follow;    // per position
  std::vector<Edge> first;                  // (pos, cond)
  std::vector<Edge> last;                   // (pos, cond)
  uint16_t nullable = 0;                    // contexts in which the empty string matches
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
  bool wordb = false;                       // uses \b / \B (prev-byte wordness matters)
  std::string error;                        // reason for FALLBACK / INVALID
  std::vector<std::string> literals;        // OR-set of required factors (ASCII-lowercased bytes)
  bool has_literals = false;
  bool bt_ok = false;                       // the native backtracker (BtRegex) runs it
  Nfa nfa;
  Dfa dfa;
};

Compiled compile(const std::string& pattern, int max_dfa_states, int max_positions);

// Multi-regex DFA ("scan group"): the Glushkov NFAs of up to 16 regexes determinised TOGETHER, so
// one table walk per byte answers find() for all of them (Aho-Corasick / RE2::Set style). Used
// for regexes without a usable literal factor, which must be run over every line. Unlike the
// single-regex DFA there is no absorbing ACCEPT state: a transition reports the regexes that
// accept BEFORE its byte and the walk goes on for the others.
//   trans[s * nclasses + cls] = next state (bits 0..15) | accept mask (bits 16..31)
//   fin[2 s] = regexes accepting at end of line, fin[2 s + 1] = before a final line terminator
// State 0 = DEAD (every member anchored and failed), state 1 = start of line.
constexpr int MULTI_MAX_REGS = 16;
struct MultiDfa {
  int nstates = 0, nclasses = 0, nregs = 0;
  std::vector<uint8_t> bytemap;
  std::vector<uint32_t> trans;
  std::vector<uint32_t> fin;
};
// throws Unsupported (state limit, > MULTI_MAX_REGS, a member that is not an automaton regex)
MultiDfa compile_multi(const std::vector<std::string>& patterns, int max_states);
// bit r set <=> patterns[r] finds a match in s[0..n) (host walk; the device kernel is k_scan_multi)
uint32_t multi_find(const MultiDfa& d, const uint8_t* s, int64_t n);

// Host-side exact match of one line with a compiled DFA (CPU backend + tests).
bool dfa_find(const Dfa& d, const uint8_t* s, int64_t n);
// Length in bytes of a final line terminator (\r, U+0085, U+2028, U+2029) ending s[0..n), or 0.
int final_terminator_len(const uint8_t* s, int64_t n);

// Java-semantics backtracking matcher (boolean Matcher.find()) for the regexes no automaton can
// express: backreferences, lookahead / lookbehind, atomic groups, possessive quantifiers,
// MULTILINE anchors. The same parser builds the AST (byte-level UTF-8 lowering, ASCII \b \w,
// CI flag), which is compiled to a small backtracking program run in Java's priority order
// (greedy/reluctant, left alternative first) -- so atomic / possessive constructs keep exactly
// the matches Java keeps. Host-only; the device prefilter narrows it to candidate lines.
class BtRegex {
 public:
  explicit BtRegex(const std::string& pattern);    // throws SyntaxError / Unsupported
  // steps: optional out-count of VM steps; a find exceeding `budget` steps returns false
  bool find(const uint8_t* s, int64_t n, int64_t budget = int64_t(1) << 27, bool* exhausted = nullptr) const;
  struct Impl;
 private:
  std::shared_ptr<const Impl> p_;
};

}  // namespace lp
