// Java-regex -> literal factors + Glushkov NFAs (code-point and byte level) + byte DFA +
// backtracking VM.  See jregex.h for the design.
#include "jregex.h"

#include <algorithm>
#include <cctype>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <unordered_map>

#include "unicode_tables.inc"

namespace lp {

// ------------------------------------------------------------------------------------------
// code-point sets
void CpSet::add_range(uint32_t lo, uint32_t hi) {
  if (hi > MAX) hi = MAX;
  if (lo > hi) return;
  // first range that ends at or after lo - 1 (touching ranges merge)
  size_t i = std::lower_bound(r.begin(), r.end(), lo,
                              [](const std::pair<uint32_t, uint32_t>& p, uint32_t v) {
                                return (uint64_t)p.second + 1 < v;
                              }) - r.begin();
  size_t j = i;
  uint32_t nlo = lo, nhi = hi;
  while (j < r.size() && (uint64_t)r[j].first <= (uint64_t)hi + 1) {
    nlo = std::min(nlo, r[j].first);
    nhi = std::max(nhi, r[j].second);
    ++j;
  }
  r.erase(r.begin() + i, r.begin() + j);
  r.insert(r.begin() + i, {nlo, nhi});
}

void CpSet::unite(const CpSet& o) {
  if (r.empty()) { r = o.r; return; }
  for (auto& p : o.r) add_range(p.first, p.second);
}

void CpSet::intersect(const CpSet& o) {
  std::vector<std::pair<uint32_t, uint32_t>> out;
  size_t i = 0, j = 0;
  while (i < r.size() && j < o.r.size()) {
    const uint32_t lo = std::max(r[i].first, o.r[j].first), hi = std::min(r[i].second, o.r[j].second);
    if (lo <= hi) out.push_back({lo, hi});
    if (r[i].second < o.r[j].second) ++i; else ++j;
  }
  r.swap(out);
}

void CpSet::negate() {
  std::vector<std::pair<uint32_t, uint32_t>> out;
  uint32_t next = 0;
  for (auto& p : r) {
    if (p.first > next) out.push_back({next, p.first - 1});
    next = p.second + 1;
  }
  if (next <= MAX) out.push_back({next, MAX});
  r.swap(out);
}

bool CpSet::contains(uint32_t c) const { return covers(c, c); }

bool CpSet::covers(uint32_t lo, uint32_t hi) const {
  auto it = std::upper_bound(r.begin(), r.end(), lo,
                             [](uint32_t v, const std::pair<uint32_t, uint32_t>& p) { return v < p.first; });
  if (it == r.begin()) return false;
  --it;
  return it->first <= lo && hi <= it->second;
}

bool CpSet::touches(uint32_t lo, uint32_t hi) const {
  auto it = std::lower_bound(r.begin(), r.end(), lo,
                             [](const std::pair<uint32_t, uint32_t>& p, uint32_t v) { return p.second < v; });
  return it != r.end() && it->first <= hi;
}

uint64_t CpSet::count() const {
  uint64_t n = 0;
  for (auto& p : r) n += (uint64_t)p.second - p.first + 1;
  return n;
}

// ------------------------------------------------------------------------------------------
// Unicode tables (generated: tools/gen_unicode_tables.py)
namespace {

const uni::SetRef* uni_find(const std::string& key) {
  const uni::SetRef* b = uni::kSets;
  const uni::SetRef* e = uni::kSets + sizeof(uni::kSets) / sizeof(uni::kSets[0]);
  const uni::SetRef* it = std::lower_bound(b, e, key, [](const uni::SetRef& s, const std::string& k) {
    return std::strcmp(s.key, k.c_str()) < 0;
  });
  return (it != e && key == it->key) ? it : nullptr;
}

bool uni_get(const std::string& key, CpSet& out) {
  const uni::SetRef* s = uni_find(key);
  if (!s) return false;
  out.r.clear();
  out.r.reserve(s->n);
  for (uint32_t k = 0; k < s->n; ++k) out.r.push_back({uni::kRanges[2 * (s->off + k)], uni::kRanges[2 * (s->off + k) + 1]});
  return true;
}

struct CaseMaps {
  std::unordered_map<uint32_t, uint32_t> up, lo;
  std::vector<std::pair<uint32_t, uint32_t>> pairs;      // (c, up(c)) and (c, lo(c))
  std::unordered_map<uint32_t, std::vector<uint32_t>> adj;  // case graph (both directions)
  CaseMaps() {
    for (size_t i = 0; i < sizeof(uni::kUpper) / sizeof(uint32_t); i += 2) {
      up[uni::kUpper[i]] = uni::kUpper[i + 1];
      pairs.push_back({uni::kUpper[i], uni::kUpper[i + 1]});
    }
    for (size_t i = 0; i < sizeof(uni::kLower) / sizeof(uint32_t); i += 2) {
      lo[uni::kLower[i]] = uni::kLower[i + 1];
      pairs.push_back({uni::kLower[i], uni::kLower[i + 1]});
    }
    for (auto& p : pairs) { adj[p.first].push_back(p.second); adj[p.second].push_back(p.first); }
  }
  uint32_t U(uint32_t c) const { auto it = up.find(c); return it == up.end() ? c : it->second; }
  uint32_t L(uint32_t c) const { auto it = lo.find(c); return it == lo.end() ? c : it->second; }
};

const CaseMaps& case_maps() {
  static const CaseMaps m;
  return m;
}

const CpSet& unicode_word() {
  static const CpSet w = [] { CpSet s; uni_get("u:word", s); return s; }();
  return w;
}

}  // namespace

CpSet unicode_set(const std::string& key) {
  CpSet s;
  uni_get(key, s);
  return s;
}

namespace {

bool is_word_byte(int c) {
  return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '_';
}

bool is_line_term(uint32_t c) { return c == '\n' || c == '\r' || c == 0x85 || c == 0x2028 || c == 0x2029; }

void utf8(uint32_t cp, std::string& out) {
  if (cp < 0x80) { out.push_back((char)cp); return; }
  if (cp < 0x800) { out.push_back((char)(0xC0 | (cp >> 6))); out.push_back((char)(0x80 | (cp & 0x3F))); return; }
  if (cp < 0x10000) {
    out.push_back((char)(0xE0 | (cp >> 12))); out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back((char)(0x80 | (cp & 0x3F)));
    return;
  }
  out.push_back((char)(0xF0 | (cp >> 18))); out.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
  out.push_back((char)(0x80 | ((cp >> 6) & 0x3F))); out.push_back((char)(0x80 | (cp & 0x3F)));
}

// decode the code point starting at s[i] (lenient: a truncated / invalid sequence still yields a
// value); *len = its byte length
uint32_t decode_at(const uint8_t* s, int64_t n, int64_t i, int* len) {
  const uint8_t c = s[i];
  if (c < 0x80 || c < 0xC0) { *len = 1; return c; }
  const int k = c >= 0xF0 ? 4 : c >= 0xE0 ? 3 : 2;
  uint32_t cp = c & (0x7F >> k);
  int m = 1;
  for (; m < k && i + m < n; ++m) cp = (cp << 6) | (s[i + m] & 0x3F);
  *len = m;
  return cp;
}

// ------------------------------------------------------------------------------------------
// AST
// N_CSET: code-point set (parser output); N_SET: byte set (UTF-8-lowered AST only).
// N_GROUP .. N_MLANCHOR only exist in backtracking mode (Parser(..., bt = true)); the automaton
// path rejects their constructs as Unsupported before building them.
enum NT { N_EMPTY, N_SET, N_CSET, N_CAT, N_ALT, N_REP, N_ASSERT, N_GROUP, N_BACKREF, N_LOOK, N_ATOMIC, N_MLANCHOR };
struct Node {
  NT t = N_EMPTY;
  ByteSet set;
  CpSet cs;
  std::vector<int> kids;
  int lo = 0, hi = 0;      // REP (hi = -1: unbounded)
  uint32_t cond = CTX_ALL; // ASSERT
  bool uword = false;      // ASSERT: \b / \B with Unicode WORD semantics
  int idx = 0;             // GROUP / BACKREF: group number; MLANCHOR: 0 '^', 1 '$'
  bool behind = false;     // LOOK: lookbehind
  bool neg = false;        // LOOK: negative; MLANCHOR: UNIX_LINES
  bool ci = false;         // BACKREF: case-insensitive compare
  bool lazy = false;       // REP: reluctant (priority order matters inside atomic groups)
};

uint32_t mask_where(bool (*f)(int, int)) {
  uint32_t m = 0;
  for (int p = 0; p < 4; ++p)
    for (int n = 0; n < 6; ++n)
      if (f(p, n)) m |= 1u << ctx_index(p, n);
  return m;
}
bool f_bos(int p, int n) { return p == P_BOS && n != N_C; }
bool f_eol(int, int n) { return n == N_EOS || n == N_FT; }
bool f_eos(int, int n) { return n == N_EOS; }
bool f_wb(int p, int n) { return n != N_C && (p == P_W) != (n == N_W); }
bool f_nwb(int p, int n) { return n != N_C && (p == P_W) == (n == N_W); }
// MULTILINE '^' (Pattern.Caret): after BOS or a line terminator, never at the end of input
bool f_ml_caret(int p, int n) { return (p == P_BOS || p == P_T) && n != N_EOS && n != N_C; }
// MULTILINE '$' (Pattern.Dollar): before any line terminator or at the end
bool f_ml_dollar(int, int n) { return n == N_EOS || n == N_FT || n == N_T; }
// UNIX_LINES MULTILINE '^' (UnixCaret): lines hold no '\n', so only at BOS (not at the end)
bool f_ux_caret(int p, int n) { return p == P_BOS && n != N_EOS && n != N_C; }

struct Flags {
  bool ci = false, dotall = false, comments = false, multiline = false, unixl = false;
  bool ucase = false;    // UNICODE_CASE
  bool uclass = false;   // UNICODE_CHARACTER_CLASS
};

std::string upper_ascii(std::string s) {
  for (auto& c : s) c = (char)std::toupper((unsigned char)c);
  return s;
}
std::string lower_ascii(std::string s) {
  for (auto& c : s) c = (char)std::tolower((unsigned char)c);
  return s;
}

class Parser {
 public:
  // bt: backtracking mode -- capturing groups, backreferences, lookaround, atomic groups,
  // possessive quantifiers and MULTILINE anchors become nodes instead of Unsupported
  explicit Parser(const std::string& s, bool bt = false) : s_(s), bt_(bt) {}
  std::vector<Node> nodes;
  int ngroups = 0;
  int parse() {
    int r = parse_alt();
    if (i_ < s_.size()) {
      if (s_[i_] == ')') throw SyntaxError("Unmatched closing ')'");
      throw SyntaxError("unexpected character");
    }
    return r;
  }
  bool uses_wordb = false;
  bool uses_uword = false, uses_aword = false;   // \b with Unicode / ASCII word semantics
  bool needs_cp = false;                         // MULTILINE ^ / $ (code-point contexts)

 private:
  const std::string& s_;
  bool bt_ = false;
  size_t i_ = 0;
  Flags f_;
  std::map<std::string, int> names_;

  int add(Node n) { nodes.push_back(std::move(n)); return (int)nodes.size() - 1; }
  int mk_cset(const CpSet& c) { Node n; n.t = N_CSET; n.cs = c; return add(n); }
  int mk_assert(uint32_t c) { Node n; n.t = N_ASSERT; n.cond = c; return add(n); }
  int mk_cat(std::vector<int> k) {
    if (k.empty()) { Node n; n.t = N_EMPTY; return add(n); }
    if (k.size() == 1) return k[0];
    Node n; n.t = N_CAT; n.kids = std::move(k); return add(n);
  }
  int mk_alt(std::vector<int> k) {
    if (k.size() == 1) return k[0];
    Node n; n.t = N_ALT; n.kids = std::move(k); return add(n);
  }
  int mk_rep(int kid, int lo, int hi) { Node n; n.t = N_REP; n.kids = {kid}; n.lo = lo; n.hi = hi; return add(n); }

  bool eof() const { return i_ >= s_.size(); }
  int peek() const { return eof() ? -1 : (unsigned char)s_[i_]; }

  void skip_ws() {
    if (!f_.comments) return;
    while (!eof()) {
      char c = s_[i_];
      if (c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f' || c == '\x0b') { ++i_; continue; }
      if (c == '#') { while (!eof() && s_[i_] != '\n') ++i_; continue; }
      break;
    }
  }

  uint32_t read_cp() {  // decode one UTF-8 code point
    unsigned char c = s_[i_++];
    if (c < 0x80) return c;
    int n = c >= 0xF0 ? 3 : c >= 0xE0 ? 2 : 1;
    uint32_t cp = c & (0x3F >> n);
    for (int k = 0; k < n && !eof(); ++k) cp = (cp << 6) | ((unsigned char)s_[i_++] & 0x3F);
    return cp;
  }

  // ---- case folding (Java: CASE_INSENSITIVE folds ASCII letters only; with UNICODE_CASE it uses
  // Character.toUpperCase / toLowerCase; predefined classes and properties are not folded)
  void add_ci(CpSet& cs, uint32_t cp) {
    cs.add(cp);
    if (!f_.ci) return;
    if (!f_.ucase) {
      if (cp >= 'a' && cp <= 'z') cs.add(cp - 32);
      else if (cp >= 'A' && cp <= 'Z') cs.add(cp + 32);
      return;
    }
    // SingleU: ch matches when toLowerCase(toUpperCase(ch)) equals that of cp; walk the case graph
    const CaseMaps& M = case_maps();
    const uint32_t key = M.L(M.U(cp));
    std::vector<uint32_t> todo = {cp};
    std::set<uint32_t> seen = {cp};
    while (!todo.empty()) {
      const uint32_t x = todo.back();
      todo.pop_back();
      if (M.L(M.U(x)) == key) cs.add(x);
      auto it = M.adj.find(x);
      if (it == M.adj.end()) continue;
      for (uint32_t y : it->second)
        if (seen.insert(y).second) todo.push_back(y);
    }
  }
  void add_range_ci(CpSet& cs, uint32_t lo, uint32_t hi) {
    cs.add_range(lo, hi);
    if (!f_.ci) return;
    if (!f_.ucase) {   // CIRange: an ASCII ch matches when its ASCII upper / lower case is in range
      for (uint32_t c = 'a'; c <= 'z'; ++c) if (c >= lo && c <= hi) cs.add(c - 32);
      for (uint32_t c = 'A'; c <= 'Z'; ++c) if (c >= lo && c <= hi) cs.add(c + 32);
      return;
    }
    // CIRangeU: ch matches when ch, toUpperCase(ch) or toLowerCase(ch) is in range
    for (auto& p : case_maps().pairs)
      if (p.second >= lo && p.second <= hi) cs.add(p.first);
  }

  int hexval(int c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    throw SyntaxError("Illegal hexadecimal escape sequence");
  }

  // single-character escapes; i_ points after the backslash at the escape letter.
  bool char_escape(uint32_t& cp) {
    int c = peek();
    switch (c) {
      case 't': ++i_; cp = '\t'; return true;
      case 'n': ++i_; cp = '\n'; return true;
      case 'r': ++i_; cp = '\r'; return true;
      case 'f': ++i_; cp = '\f'; return true;
      case 'a': ++i_; cp = 7; return true;
      case 'e': ++i_; cp = 27; return true;
      case '0': {
        ++i_;
        uint32_t v = 0; int nd = 0;
        while (!eof() && nd < 3 && peek() >= '0' && peek() <= '7') {
          uint32_t nv = v * 8 + (peek() - '0');
          if (nv > 0377) break;
          v = nv; ++i_; ++nd;
        }
        if (nd == 0) throw SyntaxError("Illegal octal escape sequence");
        cp = v; return true;
      }
      case 'x': {
        ++i_;
        if (peek() == '{') {
          ++i_; uint32_t v = 0; int nd = 0;
          while (!eof() && peek() != '}') { v = v * 16 + hexval(peek()); ++i_; ++nd; if (v > CpSet::MAX) throw SyntaxError("Hexadecimal codepoint is too big"); }
          if (eof() || nd == 0) throw SyntaxError("Unclosed hexadecimal escape sequence");
          ++i_; cp = v; return true;
        }
        if (i_ + 2 > s_.size()) throw SyntaxError("Illegal hexadecimal escape sequence");
        cp = hexval(s_[i_]) * 16 + hexval(s_[i_ + 1]); i_ += 2; return true;
      }
      case 'u': {
        ++i_;
        if (i_ + 4 > s_.size()) throw SyntaxError("Illegal Unicode escape sequence");
        uint32_t v = 0;
        for (int k = 0; k < 4; ++k) v = v * 16 + hexval(s_[i_ + k]);
        i_ += 4;
        if (v >= 0xD800 && v < 0xDC00 && i_ + 6 <= s_.size() && s_[i_] == '\\' && s_[i_ + 1] == 'u') {
          uint32_t lo = 0;
          for (int k = 0; k < 4; ++k) lo = lo * 16 + hexval(s_[i_ + 2 + k]);
          if (lo >= 0xDC00 && lo < 0xE000) { i_ += 6; v = 0x10000 + ((v - 0xD800) << 10) + (lo - 0xDC00); }
        }
        cp = v; return true;
      }
      case 'c': {
        ++i_;
        if (eof()) throw SyntaxError("Illegal control escape sequence");
        cp = (uint32_t)(s_[i_++] ^ 64); return true;
      }
      default: break;
    }
    if (c >= 0 && c < 128 && !std::isalnum(c)) { ++i_; cp = c; return true; }
    if (c >= 128) { cp = read_cp(); return true; }
    return false;
  }

  // ---- \p{..} resolution (Pattern.family + CharPredicates, Java 21)
  bool for_property(const std::string& name, CpSet& out) {      // CharPredicates.forProperty
    if (f_.ci && uni_get("gci:" + name, out)) return true;
    return uni_get("gc:" + name, out);
  }
  bool for_unicode_property(const std::string& name, CpSet& out) {   // forUnicodeProperty (+ POSIX)
    const std::string u = upper_ascii(name);
    if (f_.ci && uni_get("upi:" + u, out)) return true;
    return uni_get("up:" + u, out);
  }
  bool for_posix_name(const std::string& name, CpSet& out) {
    static const std::set<std::string> posix = {"ALPHA", "LOWER", "UPPER", "SPACE", "PUNCT", "XDIGIT",
                                                "ALNUM", "CNTRL", "DIGIT", "BLANK", "GRAPH", "PRINT"};
    const std::string u = upper_ascii(name);
    if (!posix.count(u)) return false;
    return for_unicode_property(u, out);
  }
  CpSet script(const std::string& name) {
    CpSet s;
    if (!uni_get("sc:" + upper_ascii(name), s)) throw SyntaxError("Unknown character script name {" + name + "}");
    return s;
  }
  CpSet block(const std::string& name) {
    CpSet s;
    if (!uni_get("blk:" + upper_ascii(name), s)) throw SyntaxError("Unknown character block name {" + name + "}");
    return s;
  }
  CpSet property(const std::string& name) {
    CpSet s;
    const size_t eq = name.find('=');
    if (eq != std::string::npos) {
      const std::string key = lower_ascii(name.substr(0, eq)), value = name.substr(eq + 1);
      if (key == "sc" || key == "script") return script(value);
      if (key == "blk" || key == "block") return block(value);
      if ((key == "gc" || key == "general_category") && for_property(value, s)) return s;
      throw SyntaxError("Unknown Unicode property {name=<" + key + ">, value=<" + value + ">}");
    }
    if (name.rfind("In", 0) == 0) return block(name.substr(2));
    if (name.rfind("Is", 0) == 0) {
      const std::string sh = name.substr(2);
      if (for_unicode_property(sh, s) || for_property(sh, s)) return s;
      return script(sh);
    }
    if (f_.uclass && for_posix_name(name, s)) return s;
    if (for_property(name, s)) return s;
    throw SyntaxError("Unknown character property name {" + name + "}");
  }

  bool class_escape(CpSet& cs) {  // predefined classes; i_ at the letter
    int c = peek();
    CpSet t;
    bool neg = false;
    switch (c) {
      case 'd': case 'D':
        if (f_.uclass) uni_get("u:digit", t); else t.add_range('0', '9');
        neg = c == 'D'; break;
      case 's': case 'S':
        if (f_.uclass) uni_get("u:space", t); else { t.add_range('\t', '\r'); t.add(' '); }
        neg = c == 'S'; break;
      case 'w': case 'W':
        if (f_.uclass) t = unicode_word();
        else { t.add_range('a', 'z'); t.add_range('A', 'Z'); t.add_range('0', '9'); t.add('_'); }
        neg = c == 'W'; break;
      case 'h': case 'H':
        for (uint32_t x : {0x20u, 0x09u, 0xA0u, 0x1680u, 0x180Eu, 0x202Fu, 0x205Fu, 0x3000u}) t.add(x);
        t.add_range(0x2000, 0x200A); neg = c == 'H'; break;
      case 'v': case 'V':
        for (uint32_t x : {0x0Au, 0x0Bu, 0x0Cu, 0x0Du, 0x85u, 0x2028u, 0x2029u}) t.add(x);
        neg = c == 'V'; break;
      case 'p': case 'P': {
        ++i_;
        neg = c == 'P';
        std::string name;
        if (peek() == '{') {
          ++i_;
          while (!eof() && peek() != '}') name.push_back(s_[i_++]);
          if (eof()) throw SyntaxError("Unclosed character family");
          ++i_;
        } else {
          if (eof()) throw SyntaxError("Illegal character family");
          name.push_back(s_[i_++]);
        }
        if (!name.empty() && name[0] == '^') { neg = !neg; name = name.substr(1); }
        t = property(name);
        if (neg) t.negate();
        cs.unite(t);
        return true;
      }
      default: return false;
    }
    ++i_;
    if (neg) t.negate();
    cs.unite(t);
    return true;
  }

  CpSet parse_class() {  // at '['
    ++i_;
    bool neg = false;
    if (peek() == '^') { neg = true; ++i_; }
    CpSet cur;
    bool have_acc = false;
    CpSet acc;
    bool first = true;
    for (;;) {
      if (eof()) throw SyntaxError("Unclosed character class");
      int c = peek();
      if (c == ']' && !first) { ++i_; break; }
      first = false;
      if (c == '[') { CpSet sub = parse_class(); cur.unite(sub); continue; }
      if (c == '&' && i_ + 1 < s_.size() && s_[i_ + 1] == '&') {
        i_ += 2;
        if (!have_acc) { acc = cur; have_acc = true; } else acc.intersect(cur);
        cur = CpSet();
        continue;
      }
      uint32_t lo;
      if (c == '\\') {
        ++i_;
        if (eof()) throw SyntaxError("Unexpected internal error");
        if (peek() == 'Q') {
          ++i_;
          size_t e = s_.find("\\E", i_);
          size_t end = e == std::string::npos ? s_.size() : e;
          while (i_ < end) add_ci(cur, read_cp());
          i_ = e == std::string::npos ? s_.size() : e + 2;
          continue;
        }
        if (class_escape(cur)) continue;
        if (!char_escape(lo)) throw SyntaxError("Illegal/unsupported escape sequence in class");
      } else {
        lo = read_cp();
      }
      // range?
      if (peek() == '-' && i_ + 1 < s_.size() && s_[i_ + 1] != ']' && s_[i_ + 1] != '[') {
        ++i_;
        uint32_t hi;
        if (peek() == '\\') {
          ++i_;
          if (!char_escape(hi)) throw SyntaxError("Illegal character range");
        } else {
          hi = read_cp();
        }
        if (hi < lo) throw SyntaxError("Illegal character range");
        add_range_ci(cur, lo, hi);
      } else {
        add_ci(cur, lo);
      }
    }
    CpSet res = cur;
    if (have_acc) { acc.intersect(cur); res = acc; }
    if (neg) res.negate();
    return res;
  }

  int parse_alt() {
    std::vector<int> alts;
    alts.push_back(parse_cat());
    while (peek() == '|') { ++i_; alts.push_back(parse_cat()); }
    return mk_alt(alts);
  }

  bool parse_int(int& v) {
    size_t st = i_;
    long x = 0;
    while (!eof() && peek() >= '0' && peek() <= '9') { x = x * 10 + (peek() - '0'); if (x > 100000) x = 100000; ++i_; }
    v = (int)x;
    return i_ > st;
  }

  int parse_cat() {
    std::vector<int> items;
    for (;;) {
      skip_ws();
      int c = peek();
      if (c < 0 || c == '|' || c == ')') break;
      int atom = parse_atom();
      if (atom == -2) continue;  // flag-only group
      // quantifiers
      for (;;) {
        skip_ws();
        int q = peek();
        int lo, hi;
        if (q == '*') { lo = 0; hi = -1; ++i_; }
        else if (q == '+') { lo = 1; hi = -1; ++i_; }
        else if (q == '?') { lo = 0; hi = 1; ++i_; }
        else if (q == '{') {
          size_t save = i_;
          ++i_;
          if (!parse_int(lo)) { i_ = save; throw SyntaxError("Illegal repetition"); }
          hi = lo;
          if (peek() == ',') { ++i_; if (!parse_int(hi)) hi = -1; }
          if (peek() != '}') throw SyntaxError("Unclosed counted closure");
          ++i_;
          if (hi != -1 && hi < lo) throw SyntaxError("Illegal repetition range");
        } else break;
        bool lazy = false, possessive = false;
        if (peek() == '?') { ++i_; lazy = true; }                  // lazy: same language
        else if (peek() == '+') {
          if (!bt_) throw Unsupported("possessive quantifier");
          ++i_;
          possessive = true;
        }
        atom = mk_rep(atom, lo, hi);
        nodes[atom].lazy = lazy;
        if (possessive) { Node n; n.t = N_ATOMIC; n.kids = {atom}; atom = add(n); }
        break;  // Java does not allow stacked quantifiers (a** is an error); keep one
      }
      int q2 = peek();
      if (q2 == '*' || q2 == '+' || q2 == '?') throw SyntaxError("Dangling meta character");
      items.push_back(atom);
    }
    return mk_cat(items);
  }

  void parse_flags(Flags& fl, bool& ok_group) {
    bool neg = false;
    for (;;) {
      if (eof()) throw SyntaxError("Unknown inline modifier");
      int c = peek();
      if (c == ')' || c == ':') break;
      ++i_;
      if (c == '-') { neg = true; continue; }
      bool v = !neg;
      switch (c) {
        case 'i': fl.ci = v; break;
        case 's': fl.dotall = v; break;
        case 'x': fl.comments = v; break;
        case 'm': fl.multiline = v; break;
        case 'd': fl.unixl = v; break;
        case 'u': fl.ucase = v; break;
        case 'U': fl.uclass = v; fl.ucase = v; break;   // UNICODE_CHARACTER_CLASS implies UNICODE_CASE
        case 'c': break;                                 // CANON_EQ: no effect on composed input
        default: throw SyntaxError("Unknown inline modifier");
      }
    }
    ok_group = peek() == ':';
  }

  int parse_atom() {
    int c = peek();
    if (c == '(') {
      ++i_;
      Flags saved = f_;
      int group = 0;            // capturing group number (backtracking mode)
      int wrap = -1;            // 0 lookahead, 1 lookbehind, 2 atomic
      bool neg = false;
      if (peek() == '?') {
        ++i_;
        int d = peek();
        if (d == '=' || d == '!' || d == '>') {
          if (!bt_) throw Unsupported("lookahead/atomic group");
          ++i_;
          wrap = d == '>' ? 2 : 0;
          neg = d == '!';
        } else if (d == '<' && i_ + 1 < s_.size() && (s_[i_ + 1] == '=' || s_[i_ + 1] == '!')) {
          if (!bt_) throw Unsupported("lookbehind");
          neg = s_[i_ + 1] == '!';
          i_ += 2;
          wrap = 1;
        } else if (d == '<') {
          // named group
          size_t e = s_.find('>', i_);
          if (e == std::string::npos) throw SyntaxError("named capturing group is missing trailing '>'");
          const std::string name = s_.substr(i_ + 1, e - i_ - 1);
          if (name.empty() || !std::isalpha((unsigned char)name[0])) throw SyntaxError("capturing group name does not start with a Latin letter");
          if (names_.count(name)) throw SyntaxError("Named capturing group <" + name + "> is already defined");
          group = ++ngroups;
          names_[name] = group;
          i_ = e + 1;
        } else {
          bool grp = false;
          Flags nf = f_;
          parse_flags(nf, grp);
          if (!grp) {  // (?flags)  -> applies to the rest of the enclosing group
            ++i_;      // ')'
            f_ = nf;
            return -2;
          }
          ++i_;        // ':'
          f_ = nf;
        }
      } else {
        group = ++ngroups;      // plain '(' : capturing
      }
      int r = parse_alt();
      if (peek() != ')') throw SyntaxError("Unclosed group");
      ++i_;
      f_ = saved;
      if (bt_ && wrap >= 0) {
        Node n;
        n.t = wrap == 2 ? N_ATOMIC : N_LOOK;
        n.behind = wrap == 1;
        n.neg = neg;
        n.kids = {r};
        return add(n);
      }
      if (bt_ && group > 0) {
        Node n;
        n.t = N_GROUP;
        n.idx = group;
        n.kids = {r};
        return add(n);
      }
      return r;
    }
    if (c == '[') { CpSet cs = parse_class(); return mk_cset(cs); }
    if (c == '.') {
      ++i_;
      CpSet cs;
      cs.add_range(0, CpSet::MAX);
      if (!f_.dotall) {
        CpSet t;   // Java '.': every line terminator excluded (UNIX_LINES: only '\n')
        if (f_.unixl) t.add('\n');
        else for (uint32_t x : {0x0Au, 0x0Du, 0x85u, 0x2028u, 0x2029u}) t.add(x);
        t.negate();
        cs.intersect(t);
      }
      return mk_cset(cs);
    }
    if (c == '^') {
      ++i_;
      if (f_.multiline) {
        if (bt_) { Node n; n.t = N_MLANCHOR; n.idx = 0; n.neg = f_.unixl; return add(n); }
        if (f_.unixl) return mk_assert(mask_where(f_ux_caret));
        needs_cp = true;
        return mk_assert(mask_where(f_ml_caret));
      }
      return mk_assert(mask_where(f_bos));
    }
    if (c == '$') {
      ++i_;
      if (f_.multiline) {
        if (bt_) { Node n; n.t = N_MLANCHOR; n.idx = 1; n.neg = f_.unixl; return add(n); }
        if (f_.unixl) return mk_assert(mask_where(f_eos));
        needs_cp = true;
        return mk_assert(mask_where(f_ml_dollar));
      }
      return mk_assert(f_.unixl ? mask_where(f_eos) : mask_where(f_eol));
    }
    if (c == '*' || c == '+' || c == '?') throw SyntaxError("Dangling meta character");
    if (c == '{') throw SyntaxError("Illegal repetition");
    if (c == '\\') {
      ++i_;
      if (eof()) throw SyntaxError("Unexpected internal error");
      int e = peek();
      switch (e) {
        case 'b': case 'B': {
          ++i_;
          uses_wordb = true;
          (f_.uclass ? uses_uword : uses_aword) = true;
          const int a = mk_assert(mask_where(e == 'b' ? f_wb : f_nwb));
          nodes[a].uword = f_.uclass;
          return a;
        }
        case 'A': case 'G': ++i_; return mk_assert(mask_where(f_bos));
        case 'z': ++i_; return mk_assert(mask_where(f_eos));
        case 'Z': ++i_; return mk_assert(f_.unixl ? mask_where(f_eos) : mask_where(f_eol));
        case 'Q': {
          ++i_;
          size_t en = s_.find("\\E", i_);
          size_t end = en == std::string::npos ? s_.size() : en;
          std::vector<int> seq;
          while (i_ < end) seq.push_back(literal_node(read_cp()));
          i_ = en == std::string::npos ? s_.size() : en + 2;
          return mk_cat(seq);
        }
        case 'R': {
          ++i_;
          // (?:\r\n|[\n\x0B\f\r\x85  ]); lines never hold '\n', so no atomicity issue
          CpSet cr; cr.add('\r');
          CpSet nl; nl.add('\n');
          int crlf = mk_cat({mk_cset(cr), mk_cset(nl)});
          CpSet v; for (uint32_t x : {0x0Au, 0x0Bu, 0x0Cu, 0x0Du, 0x85u, 0x2028u, 0x2029u}) v.add(x);
          return mk_alt({crlf, mk_cset(v)});
        }
        case 'X': {
          ++i_;
          if (!bt_) throw Unsupported("\\X grapheme cluster");
          // approximation: (?>\r\n|\P{M}\p{M}*) (legacy grapheme cluster)
          CpSet m; uni_get("gc:M", m);
          CpSet nm = m; nm.negate();
          CpSet cr; cr.add('\r');
          CpSet nl; nl.add('\n');
          const int g = mk_alt({mk_cat({mk_cset(cr), mk_cset(nl)}), mk_cat({mk_cset(nm), mk_rep(mk_cset(m), 0, -1)})});
          Node n; n.t = N_ATOMIC; n.kids = {g};
          return add(n);
        }
        case 'N': throw Unsupported("\\N{name}");
        case 'k': {
          if (!bt_) throw Unsupported("named backreference");
          ++i_;
          if (peek() != '<') throw SyntaxError("\\k is not followed by '<' for named capturing group");
          size_t en = s_.find('>', i_);
          if (en == std::string::npos) throw SyntaxError("named capturing group is missing trailing '>'");
          const std::string name = s_.substr(i_ + 1, en - i_ - 1);
          auto it = names_.find(name);
          if (it == names_.end()) throw SyntaxError("named capturing group <" + name + "> does not exist");
          i_ = en + 1;
          Node n; n.t = N_BACKREF; n.idx = it->second; n.ci = f_.ci; return add(n);
        }
        default: break;
      }
      if (e >= '1' && e <= '9') {
        if (!bt_) throw Unsupported("backreference");
        // Java Pattern.ref: the first digit always, further digits while the group exists
        int ref = e - '0';
        ++i_;
        while (!eof() && peek() >= '0' && peek() <= '9') {
          const int nr = ref * 10 + (peek() - '0');
          if (nr > ngroups) break;
          ref = nr;
          ++i_;
        }
        Node n; n.t = N_BACKREF; n.idx = ref; n.ci = f_.ci; return add(n);
      }
      CpSet cs;
      if (class_escape(cs)) return mk_cset(cs);
      uint32_t cp;
      if (!char_escape(cp)) throw SyntaxError("Illegal/unsupported escape sequence");
      return literal_node(cp);
    }
    if (c == ')') throw SyntaxError("Unmatched closing ')'");
    return literal_node(read_cp());
  }

  int literal_node(uint32_t cp) {
    CpSet cs;
    add_ci(cs, cp);
    return mk_cset(cs);
  }
};

// ------------------------------------------------------------------------------------------
// UTF-8 lowering: code-point sets -> byte AST (for the byte DFA, the MFMA NFA and the backtracker)
//
// The non-ASCII part of a set is built as a trie over UTF-8 bytes: a byte whose whole code-point
// window (valid code points only: overlongs / beyond U+10FFFF are never in the input) lies in the
// set is "full" and is followed by free continuation bytes; a partial byte recurses into its
// continuation byte. Bytes with identical subtrees share one alternative. Automata follow a full
// byte by ONE self-looping continuation position (valid UTF-8 fixes the count, and no position can
// start on a continuation byte), so '.' / [^x] cost a handful of positions; the backtracker takes
// the exact continuation count.
class Lowerer {
 public:
  Lowerer(const std::vector<Node>& in, bool bt) : in_(in), bt_(bt) {}
  std::vector<Node> out;
  int lower(int id) {
    const Node& n = in_[id];
    if (n.t == N_CSET) return lower_cset(n.cs);
    Node c = n;
    c.cs = CpSet();
    for (auto& k : c.kids) k = lower(k);
    return add(std::move(c));
  }

 private:
  const std::vector<Node>& in_;
  bool bt_;
  struct Win { int b; uint32_t lo, hi, minv; int rem; };

  int add(Node n) { out.push_back(std::move(n)); return (int)out.size() - 1; }
  int mk_set(const ByteSet& b) { Node n; n.t = N_SET; n.set = b; return add(n); }
  int mk_cat(std::vector<int> k) { if (k.size() == 1) return k[0]; Node n; n.t = N_CAT; n.kids = std::move(k); return add(n); }
  int mk_alt(std::vector<int> k) { if (k.size() == 1) return k[0]; Node n; n.t = N_ALT; n.kids = std::move(k); return add(n); }
  int tail(int rem, bool any_len) {        // rem free continuation bytes
    ByteSet cont; cont.set_range(0x80, 0xBF);
    Node n; n.t = N_REP; n.kids = {mk_set(cont)};
    if (any_len) { n.lo = 1; n.hi = -1; } else { n.lo = rem; n.hi = rem; }
    return add(n);
  }
  static std::string sig_of(const ByteSet& b) {
    char buf[80];
    snprintf(buf, sizeof buf, "%016llx%016llx%016llx%016llx", (unsigned long long)b.w[0], (unsigned long long)b.w[1],
             (unsigned long long)b.w[2], (unsigned long long)b.w[3]);
    return buf;
  }

  // one trie level: the windows of the candidate bytes at this position; returns -1 if nothing
  int level(const CpSet& cs, const std::vector<Win>& wins, bool top, std::string& sig) {
    std::map<int, ByteSet> full;                         // rem -> bytes
    std::map<std::string, std::pair<ByteSet, int>> part; // subtree signature -> (bytes, subtree)
    for (const Win& w : wins) {
      const uint32_t vlo = std::max(w.lo, w.minv), vhi = std::min(w.hi, CpSet::MAX);
      if (vlo > vhi || !cs.touches(vlo, vhi)) continue;
      if (cs.covers(vlo, vhi)) { full[w.rem].set(w.b); continue; }
      // partial: recurse into the next (continuation) byte
      std::vector<Win> kids;
      const uint32_t span = (w.hi - w.lo + 1) / 64;
      for (int x = 0x80; x <= 0xBF; ++x) {
        const uint32_t lo = w.lo + (uint32_t)(x - 0x80) * span;
        kids.push_back({x, lo, lo + span - 1, w.minv, w.rem - 1});
      }
      std::string s;
      const int sub = level(cs, kids, false, s);
      if (sub < 0) continue;
      auto it = part.find(s);
      if (it == part.end()) part[s] = {ByteSet(), sub};
      part[s].first.set(w.b);
    }
    std::vector<int> alts;
    ByteSet merged;
    bool any_merged = false;
    for (auto& kv : full) {
      sig += "F" + std::to_string(kv.first) + sig_of(kv.second);
      if (kv.first == 0) alts.push_back(mk_set(kv.second));
      else if (top && !bt_) { merged = merged | kv.second; any_merged = true; }
      else alts.push_back(mk_cat({mk_set(kv.second), tail(kv.first, !bt_)}));
    }
    if (any_merged) alts.push_back(mk_cat({mk_set(merged), tail(1, true)}));
    for (auto& kv : part) {
      sig += "P" + sig_of(kv.second.first) + "(" + kv.first + ")";
      alts.push_back(mk_cat({mk_set(kv.second.first), kv.second.second}));
    }
    if (alts.empty()) return -1;
    return mk_alt(alts);
  }

  int lower_cset(const CpSet& cs) {
    ByteSet ascii;
    for (auto& p : cs.r)
      for (uint32_t c = p.first; c <= p.second && c < 128; ++c) ascii.set((int)c);
    std::vector<int> alts;
    if (!ascii.empty()) alts.push_back(mk_set(ascii));
    if (cs.touches(0x80, CpSet::MAX)) {
      std::vector<Win> leads;
      for (int b = 0xC0; b <= 0xDF; ++b) leads.push_back({b, (uint32_t)(b & 0x1F) << 6, ((uint32_t)(b & 0x1F) << 6) + 63, 0x80, 1});
      for (int b = 0xE0; b <= 0xEF; ++b) leads.push_back({b, (uint32_t)(b & 0x0F) << 12, ((uint32_t)(b & 0x0F) << 12) + 4095, 0x800, 2});
      for (int b = 0xF0; b <= 0xF7; ++b) leads.push_back({b, (uint32_t)(b & 0x07) << 18, ((uint32_t)(b & 0x07) << 18) + 0x3FFFF, 0x10000, 3});
      std::string sig;
      const int t = level(cs, leads, true, sig);
      if (t >= 0) alts.push_back(t);
    }
    if (alts.empty()) return mk_set(ByteSet());   // the empty set: a position that never matches
    return mk_alt(alts);
  }
};

// ------------------------------------------------------------------------------------------
// literal factor extraction (prefilter keys; ASCII-lowercased, a superset filter)
struct Lit {
  bool exact_ok = false;
  std::set<std::string> exact;
  bool fac_ok = false;
  std::set<std::string> fac;
};

constexpr size_t kMaxExact = 64;
constexpr size_t kMaxLitLen = 32;

int lower(int c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }

long quality(const std::set<std::string>& s) {
  if (s.empty()) return -1000000;
  size_t mn = 1000;
  for (auto& x : s) mn = std::min(mn, x.size());
  if (mn == 0) return -1000000;
  return (long)std::min<size_t>(mn, 8) * 1000 - (long)s.size();
}

void consider(Lit& L, const std::set<std::string>& cand) {
  if (quality(cand) <= -1000000) return;
  if (!L.fac_ok || quality(cand) > quality(L.fac)) { L.fac = cand; L.fac_ok = true; }
}

Lit lits(const std::vector<Node>& N, int id) {
  const Node& n = N[id];
  Lit r;
  switch (n.t) {
    case N_EMPTY: case N_ASSERT: case N_LOOK: case N_MLANCHOR:   // zero-width: no characters
      r.exact_ok = true; r.exact = {""}; return r;
    case N_GROUP: case N_ATOMIC: return lits(N, n.kids[0]);        // same strings (atomic: a subset)
    case N_BACKREF: return r;                                        // unknown text: breaks runs
    case N_SET: {
      std::set<int> ch;
      for (int b = 0; b < 256; ++b) if (n.set.test(b)) ch.insert(lower(b));
      if (!ch.empty() && ch.size() <= 4) { r.exact_ok = true; for (int c : ch) r.exact.insert(std::string(1, (char)c)); }
      return r;
    }
    case N_CSET: {   // a few code points: their UTF-8 strings (ASCII lower-cased)
      if (n.cs.empty() || n.cs.count() > 8) return r;
      std::set<std::string> ch;
      for (auto& p : n.cs.r)
        for (uint32_t c = p.first; c <= p.second; ++c) {
          std::string s;
          utf8(c, s);
          for (auto& x : s) x = (char)lower((unsigned char)x);
          ch.insert(s);
        }
      if (ch.size() <= 4) { r.exact_ok = true; r.exact = ch; }
      return r;
    }
    case N_CAT: {
      std::set<std::string> run = {""};
      bool run_ok = true, all_exact = true;
      for (int k : n.kids) {
        Lit c = lits(N, k);
        if (c.fac_ok) consider(r, c.fac);
        if (c.exact_ok) {
          // cross product
          size_t maxlen = 0;
          for (auto& a : run) maxlen = std::max(maxlen, a.size());
          size_t cm = 0;
          for (auto& b : c.exact) cm = std::max(cm, b.size());
          if (run_ok && run.size() * c.exact.size() <= kMaxExact && maxlen + cm <= kMaxLitLen) {
            std::set<std::string> nr;
            for (auto& a : run) for (auto& b : c.exact) nr.insert(a + b);
            run.swap(nr);
          } else {
            consider(r, run);
            all_exact = false;
            run = c.exact;
            run_ok = true;
          }
        } else {
          consider(r, run);
          all_exact = false;
          run = {""};
        }
      }
      consider(r, run);
      if (all_exact) { r.exact_ok = true; r.exact = run; }
      return r;
    }
    case N_ALT: {
      bool ex = true, fc = true;
      std::set<std::string> ue, uf;
      for (int k : n.kids) {
        Lit c = lits(N, k);
        if (c.exact_ok) { ue.insert(c.exact.begin(), c.exact.end()); } else ex = false;
        const std::set<std::string>* best = nullptr;
        if (c.exact_ok && quality(c.exact) > -1000000) best = &c.exact;
        if (c.fac_ok && (!best || quality(c.fac) > quality(*best))) best = &c.fac;
        if (best) uf.insert(best->begin(), best->end()); else fc = false;
      }
      if (ex && ue.size() <= kMaxExact) { r.exact_ok = true; r.exact = ue; }
      if (fc && uf.size() <= 256) { r.fac_ok = true; r.fac = uf; }
      return r;
    }
    case N_REP: {
      Lit c = lits(N, n.kids[0]);
      if (n.lo == 0) {
        if (n.hi == 1 && c.exact_ok && c.exact.size() + 1 <= kMaxExact) {
          r.exact_ok = true; r.exact = c.exact; r.exact.insert("");
        }
        return r;
      }
      if (c.exact_ok) consider(r, c.exact);
      if (c.fac_ok) consider(r, c.fac);
      if (n.lo == n.hi && c.exact_ok && n.lo <= 4) {
        std::set<std::string> run = {""};
        bool ok = true;
        for (int k = 0; k < n.lo && ok; ++k) {
          std::set<std::string> nr;
          for (auto& a : run) for (auto& b : c.exact) nr.insert(a + b);
          if (nr.size() > kMaxExact) ok = false;
          run.swap(nr);
        }
        if (ok) { r.exact_ok = true; r.exact = run; consider(r, run); }
      }
      return r;
    }
  }
  return r;
}

// ------------------------------------------------------------------------------------------
// Glushkov construction with boundary conditions (byte positions from N_SET, code-point positions
// from N_CSET)
struct Info {
  uint32_t nullable = 0;
  std::vector<Edge> first, last;
};

class Glushkov {
 public:
  // counters: bounded repeats of one code-point class become counted positions (Nfa::ctr; BPG
  // programs only -- the byte automata expand every repeat)
  Glushkov(const std::vector<Node>& N, int max_pos, bool counters = false)
      : N_(N), max_pos_(max_pos), counters_(counters) {}
  Nfa nfa;

  Info build(int id) {
    const Node& n = N_[id];
    Info r;
    switch (n.t) {
      case N_EMPTY: r.nullable = CTX_ALL; return r;
      case N_ASSERT: r.nullable = n.cond; return r;
      case N_SET: case N_CSET: {
        int p = nfa.npos++;
        if (nfa.npos > max_pos_) throw Unsupported("too many NFA positions");
        if (n.t == N_SET) nfa.cls.push_back(n.set); else nfa.ccls.push_back(n.cs);
        fol_.emplace_back();
        r.first.push_back({p, CTX_ALL});
        r.last.push_back({p, CTX_ALL});
        return r;
      }
      case N_CAT: {
        r = build(n.kids[0]);
        for (size_t k = 1; k < n.kids.size(); ++k) r = cat(r, build(n.kids[k]));
        return r;
      }
      case N_ALT: {
        r = build(n.kids[0]);
        for (size_t k = 1; k < n.kids.size(); ++k) {
          Info b = build(n.kids[k]);
          r.nullable |= b.nullable;
          r.first.insert(r.first.end(), b.first.begin(), b.first.end());
          r.last.insert(r.last.end(), b.last.begin(), b.last.end());
        }
        merge(r.first); merge(r.last);
        return r;
      }
      case N_REP: {
        int kid = n.kids[0];
        if (n.lo == 0 && n.hi == 0) { r.nullable = CTX_ALL; return r; }
        bool have = false;
        const int cset = counters_ && n.hi != -1 && n.hi - n.lo >= BPG_CTR_MIN ? single_cset(kid) : -1;
        if (cset >= 0) {
          // C{lo,hi} = lo plain copies of C, then ONE counted position for C{0, hi - lo}
          for (int k = 0; k < n.lo; ++k) {
            Info c = build(cset);
            r = have ? cat(r, c) : c;
            have = true;
          }
          Info c = build(cset);
          const int p = c.first[0].to;
          nfa.ctr.resize(nfa.npos, 0);
          nfa.ctr[p] = n.hi - n.lo;
          c.nullable = CTX_ALL;
          return have ? cat(r, c) : c;
        }
        for (int k = 0; k < n.lo; ++k) {
          bool lastcopy_loop = (n.hi == -1 && k == n.lo - 1);
          Info c = build(kid);
          if (lastcopy_loop) loop(c);
          r = have ? cat(r, c) : c;
          have = true;
        }
        if (n.hi == -1) {
          if (n.lo == 0) {
            Info c = build(kid);
            loop(c);
            c.nullable = CTX_ALL;
            r = have ? cat(r, c) : c;
            have = true;
          }
        } else {
          for (int k = n.lo; k < n.hi; ++k) {
            Info c = build(kid);
            c.nullable = CTX_ALL;
            r = have ? cat(r, c) : c;
            have = true;
          }
        }
        return r;
      }
      default:   // groups / backreferences / lookaround / atomic: backtracker-only nodes
        throw Unsupported("construct needs the backtracker");
    }
    return r;
  }

  void finish(const Info& top) {
    nfa.first = top.first;
    nfa.last = top.last;
    nfa.nullable = top.nullable;
    if (!nfa.ctr.empty()) nfa.ctr.resize(nfa.npos, 0);
    nfa.follow.resize(nfa.npos);
    for (int p = 0; p < nfa.npos; ++p) {
      auto& v = fol_[p];
      std::sort(v.begin(), v.end(), [](const Edge& a, const Edge& b) { return a.to < b.to; });
      std::vector<Edge>& o = nfa.follow[p];
      for (auto& e : v) {
        if (!o.empty() && o.back().to == e.to) o.back().cond |= e.cond;
        else o.push_back(e);
      }
      std::vector<Edge>().swap(v);
    }
  }

 private:
  const std::vector<Node>& N_;
  int max_pos_;
  bool counters_ = false;
  std::vector<std::vector<Edge>> fol_;

  // the N_CSET node a repeat's body reduces to (one character class, through single-child
  // concatenations / alternations), or -1
  int single_cset(int id) const {
    for (;;) {
      const Node& n = N_[id];
      if (n.t == N_CSET) return id;
      if ((n.t == N_CAT || n.t == N_ALT) && n.kids.size() == 1) { id = n.kids[0]; continue; }
      return -1;
    }
  }

  static void merge(std::vector<Edge>& v) {
    std::sort(v.begin(), v.end(), [](const Edge& a, const Edge& b) { return a.to < b.to; });
    std::vector<Edge> o;
    for (auto& e : v) {
      if (!o.empty() && o.back().to == e.to) o.back().cond |= e.cond;
      else o.push_back(e);
    }
    v.clear();
    for (auto& e : o) if (e.cond) v.push_back(e);
  }
  void link(const std::vector<Edge>& from, const std::vector<Edge>& to) {
    for (auto& a : from)
      for (auto& b : to) {
        uint32_t c = a.cond & b.cond;
        if (c) fol_[a.to].push_back({b.to, c});
      }
  }
  void loop(Info& c) { link(c.last, c.first); }
  Info cat(const Info& a, const Info& b) {
    Info r;
    r.nullable = a.nullable & b.nullable;
    r.first = a.first;
    for (auto& e : b.first) { uint32_t c = e.cond & a.nullable; if (c) r.first.push_back({e.to, c}); }
    r.last = b.last;
    for (auto& e : a.last) { uint32_t c = e.cond & b.nullable; if (c) r.last.push_back({e.to, c}); }
    link(a.last, b.first);
    merge(r.first); merge(r.last);
    return r;
  }
};

// a '$'-type condition (before-final-terminator vs plain) on a consuming edge: the automata only
// evaluate FT for acceptance, so such patterns go to the backtracker
bool ft_sensitive(uint32_t c) {
  for (int p = 0; p < 4; ++p) {
    const bool ft = (c >> ctx_index(p, N_FT)) & 1, nn = (c >> ctx_index(p, N_N)) & 1, nt = (c >> ctx_index(p, N_T)) & 1;
    if (ft != nn && ft != nt) return true;
  }
  return false;
}
void check_ft(const Nfa& nfa) {
  for (auto& e : nfa.first) if (ft_sensitive(e.cond)) throw Unsupported("end anchor inside pattern");
  for (auto& v : nfa.follow) for (auto& e : v) if (ft_sensitive(e.cond)) throw Unsupported("end anchor inside pattern");
}

// ------------------------------------------------------------------------------------------
// subset construction (byte DFAs). Ungated follow edges are precomputed as position bitsets, so
// a state's successor costs |state| word-ORs plus one AND per byte class instead of a walk of
// every follow list per class (bounded-gap NFAs have O(n^2) edges).
struct KeyHash {
  size_t operator()(const std::vector<uint64_t>& v) const {
    size_t h = 1469598103934665603ull;
    for (auto x : v) { h ^= x; h *= 1099511628211ull; h ^= h >> 29; }
    return h;
  }
};

struct SubsetTables {
  int np = 0, nw = 0;                                  // positions, bitset words
  std::vector<uint64_t> fu;                            // [np][nw] ungated follow bitsets
  std::vector<std::vector<Edge>> fg;                   // gated follow edges per position
  std::vector<uint64_t> first_u;                       // ungated first set
  std::vector<Edge> first_g;
  std::vector<uint64_t> cm;                            // [nclasses][nw] positions whose class holds the rep byte
  void init(int npos, const std::vector<const ByteSet*>& cls, const std::vector<std::vector<Edge>>& follow,
            const std::vector<Edge>& first, const std::vector<int>& rep) {
    np = npos;
    nw = (np + 63) / 64;
    fu.assign((size_t)np * nw, 0);
    fg.assign(np, {});
    for (int p = 0; p < np; ++p)
      for (auto& e : follow[p]) {
        if (e.cond == CTX_ALL) fu[(size_t)p * nw + (e.to >> 6)] |= 1ull << (e.to & 63);
        else fg[p].push_back(e);
      }
    first_u.assign(nw, 0);
    first_g.clear();
    for (auto& e : first) {
      if (e.cond == CTX_ALL) first_u[e.to >> 6] |= 1ull << (e.to & 63);
      else first_g.push_back(e);
    }
    cm.assign(rep.size() * nw, 0);
    for (size_t k = 0; k < rep.size(); ++k)
      for (int p = 0; p < np; ++p)
        if (cls[p]->test(rep[k])) cm[k * nw + (p >> 6)] |= 1ull << (p & 63);
  }
  // U = union of the ungated follow sets of the active positions
  void ungated(const std::vector<uint64_t>& A, std::vector<uint64_t>& U) const {
    std::fill(U.begin(), U.begin() + nw, 0);
    for (int w = 0; w < nw; ++w) {
      uint64_t m = A[w];
      while (m) {
        const int p = w * 64 + __builtin_ctzll(m);
        m &= m - 1;
        const uint64_t* f = fu.data() + (size_t)p * nw;
        for (int j = 0; j < nw; ++j) U[j] |= f[j];
      }
    }
  }
  // successor positions on class k (rep byte c) in context bit `bit`; returns whether any
  bool step(const std::vector<uint64_t>& A, const std::vector<uint64_t>& U, int k, int c, uint32_t bit,
            const std::vector<const ByteSet*>& cls, std::vector<uint64_t>& B) const {
    bool any = false;
    const uint64_t* m = cm.data() + (size_t)k * nw;
    for (int w = 0; w < nw; ++w) { B[w] = (U[w] | first_u[w]) & m[w]; any |= B[w] != 0; }
    for (int w = 0; w < nw; ++w) {
      uint64_t a = A[w];
      while (a) {
        const int p = w * 64 + __builtin_ctzll(a);
        a &= a - 1;
        for (auto& e : fg[p])
          if ((e.cond & bit) && cls[e.to]->test(c)) { B[e.to >> 6] |= 1ull << (e.to & 63); any = true; }
      }
    }
    for (auto& e : first_g)
      if ((e.cond & bit) && cls[e.to]->test(c)) { B[e.to >> 6] |= 1ull << (e.to & 63); any = true; }
    return any;
  }
};

int next_kind_of_byte(int c) { return is_word_byte(c) ? N_W : (c >= 0x80 && c <= 0xBF) ? N_C : N_N; }

Dfa build_dfa(const Nfa& nfa, bool uses_wordb, int max_states) {
  Dfa d;
  const int np = nfa.npos;
  const int nw = (np + 63) / 64 + 1;  // last word: prev kind
  // byte classes: signature = (membership in every distinct position class, word bit, cont bit)
  std::vector<ByteSet> dcls;
  for (auto& c : nfa.cls) {
    bool f = false;
    for (auto& x : dcls) if (x == c) { f = true; break; }
    if (!f) dcls.push_back(c);
  }
  std::map<std::vector<bool>, int> sig2cls;
  d.bytemap.assign(256, 0);
  std::vector<int> rep;
  for (int b = 0; b < 256; ++b) {
    std::vector<bool> sig;
    sig.reserve(dcls.size() + 2);
    for (auto& x : dcls) sig.push_back(x.test(b));
    sig.push_back(is_word_byte(b));
    sig.push_back(b >= 0x80 && b <= 0xBF);
    auto it = sig2cls.find(sig);
    int k;
    if (it == sig2cls.end()) { k = (int)rep.size(); sig2cls[sig] = k; rep.push_back(b); }
    else k = it->second;
    d.bytemap[b] = (uint8_t)k;
  }
  d.nclasses = (int)rep.size();
  if (d.nclasses > 256) throw Unsupported("too many byte classes");

  bool restartable = (nfa.nullable & CTX_NOT_BOS) != 0;
  for (auto& e : nfa.first) if (e.cond & CTX_NOT_BOS) restartable = true;
  d.anchored = !restartable;

  std::vector<const ByteSet*> clsp(np);
  for (int p = 0; p < np; ++p) clsp[p] = &nfa.cls[p];
  SubsetTables T;
  T.init(np, clsp, nfa.follow, nfa.first, rep);
  auto accepts = [&](const std::vector<uint64_t>& A, int prev, int next) {
    const uint32_t bit = 1u << ctx_index(prev, next);
    if (nfa.nullable & bit) return true;
    for (auto& e : nfa.last)
      if ((A[e.to >> 6] >> (e.to & 63) & 1) && (e.cond & bit)) return true;
    return false;
  };

  std::unordered_map<std::vector<uint64_t>, int, KeyHash> ids;
  std::vector<std::vector<uint64_t>> states;
  auto intern = [&](std::vector<uint64_t>& key) -> int {
    auto it = ids.find(key);
    if (it != ids.end()) return it->second;
    int id = (int)states.size() + 2;
    if (id >= max_states) throw Unsupported("DFA state limit");
    ids.emplace(key, id);
    states.push_back(key);
    return id;
  };
  std::vector<uint64_t> init(nw, 0);
  init[nw - 1] = P_BOS;
  intern(init);

  std::vector<std::vector<uint16_t>> rows;
  std::vector<uint8_t> acc;
  std::vector<uint64_t> U(nw, 0), B(nw, 0);
  for (size_t si = 0; si < states.size(); ++si) {
    const std::vector<uint64_t> A = states[si];
    const int prev = (int)A[nw - 1];
    uint8_t fl = 0;
    if (accepts(A, prev, N_EOS)) fl |= 1;
    if (accepts(A, prev, N_FT)) fl |= 2;
    acc.push_back(fl);
    std::vector<uint16_t> row(d.nclasses, 0);
    T.ungated(A, U);
    for (int k = 0; k < d.nclasses; ++k) {
      const int c = rep[k];
      const int nk = next_kind_of_byte(c);
      if (accepts(A, prev, nk)) { row[k] = 1; continue; }
      std::fill(B.begin(), B.end(), 0);
      const bool any = T.step(A, U, k, c, 1u << ctx_index(prev, nk), clsp, B);
      const int nprev = (nk == N_W && uses_wordb) ? P_W : P_N;
      if (!any && !restartable) { row[k] = 0; continue; }
      B[nw - 1] = (uint64_t)nprev;
      row[k] = (uint16_t)intern(B);
    }
    rows.push_back(std::move(row));
  }
  d.nstates = (int)states.size() + 2;
  d.trans.assign((size_t)d.nstates * d.nclasses, 0);
  d.accflags.assign(d.nstates, 0);
  for (int k = 0; k < d.nclasses; ++k) { d.trans[0 * d.nclasses + k] = 0; d.trans[1 * d.nclasses + k] = 1; }
  d.accflags[1] = 3;
  for (size_t si = 0; si < rows.size(); ++si) {
    for (int k = 0; k < d.nclasses; ++k) d.trans[(si + 2) * d.nclasses + k] = rows[si][k];
    d.accflags[si + 2] = acc[si];
  }
  return d;
}

}  // namespace

int final_terminator_len(const uint8_t* s, int64_t n) {
  if (n >= 1 && s[n - 1] == '\r') return 1;
  if (n >= 2 && s[n - 2] == 0xC2 && s[n - 1] == 0x85) return 2;
  if (n >= 3 && s[n - 3] == 0xE2 && s[n - 2] == 0x80 && (s[n - 1] == 0xA8 || s[n - 1] == 0xA9)) return 3;
  return 0;
}

bool dfa_find(const Dfa& d, const uint8_t* s, int64_t n) {
  int64_t ft = n - final_terminator_len(s, n);
  if (ft == n) ft = -1;
  int st = 2;
  const int nc = d.nclasses;
  for (int64_t t = 0; t < n; ++t) {
    if (t == ft && (d.accflags[st] & 2)) return true;
    st = d.trans[(size_t)st * nc + d.bytemap[s[t]]];
    if (st < 2) return st == 1;
  }
  return d.accflags[st] & 1;
}

namespace {
// required-literal factors of a parsed pattern -> out.literals (ASCII-lowercased OR-set)
void set_literals(Compiled& out, const std::vector<Node>& nodes, int root) {
  Lit L = lits(nodes, root);
  std::set<std::string> best;
  if (L.exact_ok && quality(L.exact) > -1000000) best = L.exact;
  if (L.fac_ok && (best.empty() || quality(L.fac) > quality(best))) best = L.fac;
  if (!best.empty()) {
    size_t mn = 1000;
    for (auto& x : best) mn = std::min(mn, x.size());
    if (mn >= 2) { out.has_literals = true; out.literals.assign(best.begin(), best.end()); }
  }
}

// a construct no automaton expresses: classify with the backtracking parser -- Java rejects the
// pattern (INVALID) or the native backtracker runs it (FALLBACK, bt_ok) -- and take its literals
// for the device prefilter
void classify_fallback(Compiled& out, const std::string& pattern, const std::string& why) {
  out.kind = Kind::FALLBACK;
  out.error = why;
  out.literals.clear();
  out.has_literals = false;
  try {
    Parser B(pattern, true);
    const int r = B.parse();
    set_literals(out, B.nodes, r);
    BtRegex check(pattern);
    out.bt_ok = true;
  } catch (const SyntaxError& e) {
    out.kind = Kind::INVALID;
    out.error = e.what();
    out.literals.clear();
    out.has_literals = false;
  } catch (const std::exception&) {
  }
}

// Regular RELAXATION of a backtracker-only regex: the AST of a SUPERSET language the automata run,
// so the GPU narrows the lines the host backtracker must check (literal-free regexes included):
// a group -> its body; a backreference -> a copy of its closed, case-sensitive group's body (the
// captured text is in that language), else any string; lookaround and MULTILINE anchors -> empty
// (they only restrict); atomic groups / possessive quantifiers -> plain (the same language or a
// superset). find() of the original implies find() of the relaxation.
class Relaxer {
 public:
  explicit Relaxer(const std::vector<Node>& in) : in_(in) {}
  std::vector<Node> out;
  int relax(int id) {
    const Node& n = in_[id];
    switch (n.t) {
      case N_GROUP: {
        open_.insert(n.idx);
        const int b = relax(n.kids[0]);
        open_.erase(n.idx);
        body_[n.idx] = b;
        return b;
      }
      case N_BACKREF: {
        auto it = body_.find(n.idx);
        if (!n.ci && it != body_.end() && !open_.count(n.idx)) return it->second;
        return any();
      }
      case N_LOOK: case N_MLANCHOR: { Node e; e.t = N_EMPTY; return add(e); }
      case N_ATOMIC: return relax(n.kids[0]);
      default: {
        Node c = n;
        for (auto& k : c.kids) k = relax(k);
        return add(c);
      }
    }
  }

 private:
  const std::vector<Node>& in_;
  std::map<int, int> body_;
  std::set<int> open_;
  int any_ = -1;
  int add(const Node& n) { out.push_back(n); return (int)out.size() - 1; }
  int any() {
    if (any_ < 0) {
      Node c; c.t = N_CSET; c.cs.add_range(0, CpSet::MAX);
      const int k = add(c);
      Node r; r.t = N_REP; r.kids = {k}; r.lo = 0; r.hi = -1;
      any_ = add(r);
    }
    return any_;
  }
};

Compiled compile_nodes(Compiled out, std::vector<Node> nodes, int root, int max_dfa_states, int max_positions,
                       bool want_bpg, const std::string& pattern);

// ---- find()-equivalence ----------------------------------------------------------------------
// The reference only asks find() (AnalysisService.java:95, ScoringService.java:281,300,330):
// whether SOME substring of the line is in L(R), i.e. membership of the line in Σ*·R·Σ*. There a
// LEADING repeat keeps only its minimum count: Σ*·X{m,n}·S = Σ*·X{m}·S, because the extra copies
// of X are matches of X at real text positions and fold into the Σ* prefix (any assertion inside
// them is still evaluated at the position it sits on); symmetrically for a TRAILING repeat and the
// Σ* suffix. X{0,n} and X* vanish, and the element after them becomes the leading one. This keeps
// repeated groups such as (?:ab.){0,1000}Z (= Z) or (?:ERROR \d+ ){1,300} (= ERROR \d+ ) on the
// automata instead of past the position limit. `lead`: the leading edge, else the trailing one.
// Returns whether node `id` now matches only the empty string (the caller moves on to the next
// element). The parser builds a tree (every node has one parent), so nodes are edited in place.
bool trim_edge(std::vector<Node>& N, int id, bool lead) {
  switch (N[id].t) {
    case N_EMPTY: return true;
    case N_REP: {
      if (N[id].lo == 0) {
        N[id] = Node();
        N[id].t = N_EMPTY;
        return true;
      }
      N[id].hi = N[id].lo;
      return false;
    }
    case N_GROUP: return trim_edge(N, N[id].kids[0], lead);
    case N_ALT: {                  // Σ*(A|B)S = Σ*AS ∪ Σ*BS: each alternative on its own
      bool all = true;
      const std::vector<int> kids = N[id].kids;
      for (int k : kids) all = trim_edge(N, k, lead) && all;
      return all;
    }
    case N_CAT: {
      const std::vector<int> kids = N[id].kids;
      const int n = (int)kids.size();
      for (int j = 0; j < n; ++j)
        if (!trim_edge(N, kids[lead ? j : n - 1 - j], lead)) return false;
      return true;
    }
    default: return false;         // a character, an assertion, a backtracker-only construct
  }
}

void trim_find(std::vector<Node>& N, int root) {
  trim_edge(N, root, true);
  trim_edge(N, root, false);
}

// ---- lookaround on the automata -------------------------------------------------------------
// A regex R0 · L1 · R1 · L2 · ... · LK · RK whose only non-regular-looking parts are clusters Ls of
// lookarounds between regular segments (R0 and RK may be empty) -- \bERROR\b(?!.*retry),
// (?=.*FATAL)ERR, (?<!a)b, (?<=a)b, (?<!\S)x(?!\S) -- still has a regular find() language, and
// Java matches it exactly as this definition says: the line matches iff there are positions
// p1 <= ... <= pK with
//   * R0 ending at p1 (Σ*·R0 accepts there; an empty R0: any position), Rs matching [ps, ps+1),
//     RK matching from pK (to any end),
//   * at each ps every lookbehind (?<=A) of Ls with some A match ending there, every (?<!A) none,
//     every lookahead (?=Y) matching from ps, every (?!Y) not.
// The find() DFA is built directly by a subset construction whose state is
//   (prev character kind, the unanchored position sets of Σ*R0 and of every lookbehind's Σ*A,
//    the set of live INSTANCES),
// an instance being (stage s, the anchored position set of Rs, one anchored set per lookahead of
// the clusters reached so far), each part DONE once it accepted or DEAD once empty. A segment
// that ends where the next cluster's lookbehinds hold moves a copy of its instance to the next
// stage (the instance goes on, looking for other ends). An instance succeeds when RK is DONE, every
// positive lookahead DONE and every negative one DEAD (at the end of the line a running part that
// does not accept there is DEAD); a negative lookahead that is DONE, or a positive one that is
// DEAD, drops it. Lookarounds and acceptance are only evaluated between whole characters (never
// before a UTF-8 continuation byte). No Unicode \b, no MULTILINE anchors and no '$'-type condition
// (final-terminator contexts) in any part; anything else -- nested lookarounds, backreferences,
// atomic groups, a construction past the state limit -- stays on the backtracker.
struct LookPart {
  Nfa nfa;
  std::vector<const ByteSet*> clsp;
  SubsetTables T;
  bool neg = false;                            // (?!Y) / (?<!A)
  std::unordered_map<std::vector<uint64_t>, int, KeyHash> ids;
  std::vector<std::vector<uint64_t>> sets;
  int intern(const std::vector<uint64_t>& s) {
    auto it = ids.find(s);
    if (it != ids.end()) return it->second;
    const int id = (int)sets.size();
    ids.emplace(s, id);
    sets.push_back(s);
    return id;
  }
  bool accepts(const std::vector<uint64_t>* A, uint32_t bit) const {   // A == nullptr: fresh (nothing consumed)
    if (!A) return (nfa.nullable & bit) != 0;
    for (auto& e : nfa.last)
      if (((*A)[e.to >> 6] >> (e.to & 63) & 1) && (e.cond & bit)) return true;
    return false;
  }
  // successors on class k (rep byte c) in context `bit`; `first`: also the first positions (a fresh
  // anchored part, or an unanchored part that restarts everywhere)
  std::vector<uint64_t> advance(const std::vector<uint64_t>* A, bool first, int k, int c, uint32_t bit) const {
    std::vector<uint64_t> B(T.nw, 0), U(T.nw, 0);
    const uint64_t* m = T.cm.data() + (size_t)k * T.nw;
    if (A) {
      T.ungated(*A, U);
      for (int w = 0; w < T.nw; ++w) {
        uint64_t a = (*A)[w];
        while (a) {
          const int p = w * 64 + __builtin_ctzll(a);
          a &= a - 1;
          for (auto& e : T.fg[p])
            if ((e.cond & bit) && clsp[e.to]->test(c)) B[e.to >> 6] |= 1ull << (e.to & 63);
        }
      }
    }
    if (first) {
      for (int w = 0; w < T.nw; ++w) U[w] |= T.first_u[w];
      for (auto& e : T.first_g)
        if ((e.cond & bit) && clsp[e.to]->test(c)) B[e.to >> 6] |= 1ull << (e.to & 63);
    }
    for (int w = 0; w < T.nw; ++w) B[w] |= U[w] & m[w];
    return B;
  }
};

constexpr int LK_FRESH = -1, LK_DONE = -2, LK_DEAD = -3;

bool any_ft(const Nfa& nfa) {
  if (ft_sensitive(nfa.nullable)) return true;
  for (auto& e : nfa.first) if (ft_sensitive(e.cond)) return true;
  for (auto& e : nfa.last) if (ft_sensitive(e.cond)) return true;
  for (auto& v : nfa.follow) for (auto& e : v) if (ft_sensitive(e.cond)) return true;
  return false;
}

class LookaroundDfa {
 public:
  LookaroundDfa(const std::vector<Node>& in, int root, int max_states, int max_positions, bool wordb)
      : in_(in), max_states_(max_states), max_pos_(max_positions), wordb_(wordb) {
    std::vector<int> items;
    flatten(root, items);
    // segments and clusters: R0 L1 R1 L2 R2 ... LK RK (contiguous lookarounds form one cluster)
    std::vector<std::vector<int>> segs(1), clus;
    for (int id : items) {
      if (in_[id].t == N_LOOK) {
        if (segs.size() == clus.size() + 1) clus.emplace_back();   // a new cluster after a segment
        clus.back().push_back(id);
      } else {
        if (segs.size() == clus.size()) segs.emplace_back();
        segs.back().push_back(id);
      }
    }
    K_ = (int)clus.size();
    if (K_ == 0) throw Unsupported("no lookaround");
    if (K_ > 4) throw Unsupported("more than 4 lookaround positions");
    segs.resize(K_ + 1);
    Lowerer Lw(plain_, false);
    auto part = [&](int cp_root, bool neg) {
      LookPart P;
      P.neg = neg;
      Glushkov G(Lw.out, max_pos_);
      Info top = G.build(Lw.lower(cp_root));
      G.finish(top);
      if (any_ft(G.nfa)) throw Unsupported("end anchor in a lookaround pattern");
      P.nfa = std::move(G.nfa);
      return P;
    };
    if (!segs[0].empty()) {
      const int c = cat(segs[0]);
      trim_edge(plain_, c, true);            // Σ*·R0: its leading repeat keeps its minimum
      main_.push_back(part(c, false));
      r0_ = 0;
    }
    seg_.assign(K_ + 1, -1);
    behind_.resize(K_ + 1);
    ahead_.resize(K_ + 1);
    for (int s = 1; s <= K_; ++s) {
      for (int id : clus[s - 1]) {
        const Node& n = in_[id];
        const int body = strip(n.kids[0]);
        if (n.behind) {
          behind_[s].push_back((int)main_.size());
          main_.push_back(part(body, n.neg));
        } else {
          trim_edge(plain_, body, false);    // Y·Σ*: a lookahead matches a prefix of the rest
          ahead_[s].push_back((int)ahd_.size());
          ahd_.push_back(part(body, n.neg));
        }
      }
      if (!segs[s].empty()) {
        const int c = cat(segs[s]);
        if (s == K_) trim_edge(plain_, c, false);   // RK·Σ*
        seg_[s] = (int)sgp_.size();
        sgp_.push_back(part(c, false));
      }
    }
  }

  Dfa build() {
    // byte classes: membership in every distinct position class of every part, word bit, cont bit
    std::vector<ByteSet> dcls;
    auto each = [&](auto&& f) { for (auto& p : main_) f(p); for (auto& p : sgp_) f(p); for (auto& p : ahd_) f(p); };
    each([&](LookPart& P) {
      for (auto& c : P.nfa.cls) {
        bool f = false;
        for (auto& x : dcls) if (x == c) { f = true; break; }
        if (!f) dcls.push_back(c);
      }
    });
    Dfa d;
    std::map<std::vector<bool>, int> sig2cls;
    d.bytemap.assign(256, 0);
    for (int b = 0; b < 256; ++b) {
      std::vector<bool> sig;
      for (auto& x : dcls) sig.push_back(x.test(b));
      sig.push_back(is_word_byte(b));
      sig.push_back(b >= 0x80 && b <= 0xBF);
      auto it = sig2cls.find(sig);
      int k;
      if (it == sig2cls.end()) { k = (int)rep_.size(); sig2cls[sig] = k; rep_.push_back(b); }
      else k = it->second;
      d.bytemap[b] = (uint8_t)k;
    }
    d.nclasses = (int)rep_.size();
    if (d.nclasses > 256) throw Unsupported("too many byte classes");
    each([&](LookPart& P) {
      P.clsp.resize(P.nfa.npos);
      for (int p = 0; p < P.nfa.npos; ++p) P.clsp[p] = &P.nfa.cls[p];
      P.T.init(P.nfa.npos, P.clsp, P.nfa.follow, P.nfa.first, rep_);
    });

    State s0;
    s0.prev = P_BOS;
    for (auto& P : main_) s0.main.push_back(P.intern(std::vector<uint64_t>(P.T.nw, 0)));
    intern(s0);
    std::vector<std::vector<uint16_t>> rows;
    std::vector<uint8_t> acc;
    for (size_t si = 0; si < states_.size(); ++si) {
      const State S = states_[si];
      acc.push_back(accepts_at_end(S) ? 1 : 0);
      std::vector<uint16_t> row(d.nclasses, 0);
      for (int k = 0; k < d.nclasses; ++k) row[k] = (uint16_t)step(S, k);
      rows.push_back(std::move(row));
    }
    d.nstates = (int)states_.size() + 2;
    d.trans.assign((size_t)d.nstates * d.nclasses, 0);
    d.accflags.assign(d.nstates, 0);
    for (int k = 0; k < d.nclasses; ++k) d.trans[1 * d.nclasses + k] = 1;
    d.accflags[1] = 3;
    for (size_t si = 0; si < rows.size(); ++si) {
      for (int k = 0; k < d.nclasses; ++k) d.trans[(si + 2) * d.nclasses + k] = rows[si][k];
      d.accflags[si + 2] = acc[si];
    }
    d.anchored = false;
    return d;
  }

 private:
  // an instance: [stage s (1..K), its segment's state, the state of every lookahead part (NOTYET
  // until its cluster is reached)]
  static constexpr int NOTYET = -4;
  struct State {
    int prev = P_BOS;
    std::vector<int> main;                      // set ids of the unanchored parts
    std::vector<std::vector<int>> insts;
    std::vector<int64_t> key() const {
      std::vector<int64_t> k{prev, (int64_t)main.size()};
      k.insert(k.end(), main.begin(), main.end());
      for (auto& t : insts) k.insert(k.end(), t.begin(), t.end());
      return k;
    }
  };
  struct VHash {
    size_t operator()(const std::vector<int64_t>& v) const {
      size_t h = 1469598103934665603ull;
      for (auto x : v) { h ^= (size_t)x; h *= 1099511628211ull; h ^= h >> 29; }
      return h;
    }
  };

  const std::vector<Node>& in_;
  std::vector<Node> plain_;                     // regular copies of the segments and the bodies
  int max_states_, max_pos_;
  bool wordb_;
  int K_ = 0, r0_ = -1;                         // clusters; main_ index of R0 (-1: empty)
  std::vector<LookPart> main_, sgp_, ahd_;      // unanchored (R0, lookbehinds), segments, lookaheads
  std::vector<int> seg_;                        // stage s -> sgp_ index (-1: empty segment)
  std::vector<std::vector<int>> behind_, ahead_;   // stage s -> its cluster's main_ / ahd_ indices
  std::vector<int> rep_;
  std::unordered_map<std::vector<int64_t>, int, VHash> sids_;
  std::vector<State> states_;

  void flatten(int id, std::vector<int>& items) {
    const Node& n = in_[id];
    if (n.t == N_CAT) { for (int k : n.kids) flatten(k, items); return; }
    if (n.t == N_GROUP) { flatten(n.kids[0], items); return; }
    items.push_back(id);
  }
  int add(Node n) { plain_.push_back(std::move(n)); return (int)plain_.size() - 1; }
  int cat(const std::vector<int>& items) {
    std::vector<int> k;
    for (int i : items) k.push_back(strip(i));
    if (k.size() == 1) return k[0];
    Node n; n.t = N_CAT; n.kids = std::move(k);
    return add(n);
  }
  // a regular copy of a sub-pattern: capturing groups are transparent (no backreference can refer
  // to them: those throw); lookaround, atomic groups, backreferences, MULTILINE anchors throw
  int strip(int id) {
    const Node& n = in_[id];
    switch (n.t) {
      case N_GROUP: return strip(n.kids[0]);
      case N_LOOK: throw Unsupported("nested lookaround");
      case N_ATOMIC: throw Unsupported("atomic group / possessive quantifier");
      case N_BACKREF: throw Unsupported("backreference");
      case N_MLANCHOR: throw Unsupported("MULTILINE anchor with lookaround");
      default: {
        Node c = n;
        for (auto& k : c.kids) k = strip(k);
        return add(c);
      }
    }
  }

  int intern(State& S) {
    std::sort(S.insts.begin(), S.insts.end());
    S.insts.erase(std::unique(S.insts.begin(), S.insts.end()), S.insts.end());
    const std::vector<int64_t> k = S.key();
    auto it = sids_.find(k);
    if (it != sids_.end()) return it->second;
    const int id = (int)states_.size() + 2;
    if (id >= max_states_ || id > 0xFFFF) throw Unsupported("DFA state limit");
    sids_.emplace(k, id);
    states_.push_back(S);
    return id;
  }

  static const std::vector<uint64_t>* set_of(const LookPart& P, int v) { return v >= 0 ? &P.sets[v] : nullptr; }
  static bool runs(int v) { return v >= 0 || v == LK_FRESH; }

  bool main_ends(const State& S, int j, uint32_t bit) const {
    return main_[j].accepts(&main_[j].sets[S.main[j]], bit) || (main_[j].nfa.nullable & bit);
  }
  // cluster s's lookbehinds hold here ((?<=A): some A ends here, (?<!A): none)
  bool behind_ok(const State& S, int s, uint32_t bit) const {
    for (int j : behind_[s])
      if (main_ends(S, j, bit) == main_[j].neg) return false;
    return true;
  }
  // an instance entering stage s here: its segment and cluster s's lookaheads start fresh
  std::vector<int> enter(std::vector<int> t, int s) const {
    t[0] = s;
    t[1] = seg_[s] < 0 ? LK_DONE : LK_FRESH;
    for (int j : ahead_[s]) t[2 + j] = LK_FRESH;
    return t;
  }
  bool alive(const std::vector<int>& t) const {
    for (size_t j = 0; j < ahd_.size(); ++j) {
      if (ahd_[j].neg && t[2 + j] == LK_DONE) return false;
      if (!ahd_[j].neg && t[2 + j] == LK_DEAD) return false;
    }
    return true;
  }
  bool success(const std::vector<int>& t) const {
    if (t[0] != K_ || t[1] != LK_DONE) return false;
    for (size_t j = 0; j < ahd_.size(); ++j)
      if (t[2 + j] != (ahd_[j].neg ? LK_DEAD : LK_DONE)) return false;
    return true;
  }

  // the instances at a character boundary (or the end) before the next character: lookaheads that
  // accept here are DONE, segments that end here move their instance on to the next stage (the
  // instance itself goes on looking for other ends), the last stage's segment is DONE. Returns the
  // live instances; `won` when one succeeded.
  std::vector<std::vector<int>> boundary(const State& S, uint32_t bit, bool& won) const {
    std::vector<std::vector<int>> work = S.insts, out;
    if ((r0_ < 0 || main_ends(S, r0_, bit)) && behind_ok(S, 1, bit))
      work.push_back(enter(std::vector<int>(2 + ahd_.size(), NOTYET), 1));
    won = false;
    while (!work.empty()) {
      std::vector<int> t = std::move(work.back());
      work.pop_back();
      for (size_t j = 0; j < ahd_.size(); ++j)
        if (runs(t[2 + j]) && ahd_[j].accepts(set_of(ahd_[j], t[2 + j]), bit)) t[2 + j] = LK_DONE;
      if (!alive(t)) continue;
      const int s = t[0];
      const bool ends = t[1] == LK_DONE || (runs(t[1]) && sgp_[seg_[s]].accepts(set_of(sgp_[seg_[s]], t[1]), bit));
      if (ends) {
        if (s == K_) {
          t[1] = LK_DONE;
        } else if (behind_ok(S, s + 1, bit)) {
          work.push_back(enter(t, s + 1));
        }
      }
      if (success(t)) { won = true; return out; }
      if (s < K_ && t[1] == LK_DONE) continue;     // an empty middle segment: only its next stage lives
      out.push_back(std::move(t));
    }
    return out;
  }

  bool accepts_at_end(const State& S) {
    bool won = false;
    std::vector<std::vector<int>> insts = boundary(S, 1u << ctx_index(S.prev, N_EOS), won);
    if (won) return true;
    for (auto& t : insts) {
      for (size_t j = 0; j < ahd_.size(); ++j)
        if (t[2 + j] != LK_DONE) t[2 + j] = LK_DEAD;      // nothing follows the end
      if (success(t)) return true;
    }
    return false;
  }

  int step(const State& S, int k) {
    const int c = rep_[k];
    const int nk = next_kind_of_byte(c);
    const uint32_t bit = 1u << ctx_index(S.prev, nk);
    std::vector<std::vector<int>> insts;
    if (nk != N_C) {                             // lookarounds sit between whole characters
      bool won = false;
      insts = boundary(S, bit, won);
      if (won) return 1;                         // ACCEPT
    } else {
      insts = S.insts;
    }
    State N;
    N.prev = (nk == N_W && wordb_) ? P_W : P_N;
    for (size_t j = 0; j < main_.size(); ++j)
      N.main.push_back(main_[j].intern(main_[j].advance(&main_[j].sets[S.main[j]], true, k, c, bit)));
    auto adv = [&](LookPart& P, int v) {
      std::vector<uint64_t> B = P.advance(set_of(P, v), v == LK_FRESH, k, c, bit);
      bool any = false;
      for (auto w : B) any |= w != 0;
      return any ? P.intern(B) : LK_DEAD;
    };
    for (auto& t : insts) {
      if (runs(t[1])) t[1] = adv(sgp_[seg_[t[0]]], t[1]);
      if (t[1] == LK_DEAD) continue;             // its segment can no longer end
      for (size_t j = 0; j < ahd_.size(); ++j)
        if (runs(t[2 + j])) t[2 + j] = adv(ahd_[j], t[2 + j]);
      if (!alive(t)) continue;
      if (success(t)) return 1;
      N.insts.push_back(std::move(t));
    }
    return intern(N);
  }
};

// A regex the automaton parser refused (lookaround, ...): its find() DFA when it is a lookaround
// cluster LookaroundDfa covers; throws Unsupported otherwise
void compile_lookaround(Compiled& out, const std::string& pattern, int max_dfa_states, int max_positions) {
  Parser B(pattern, true);
  const int r = B.parse();
  if (B.uses_uword) throw Unsupported("lookaround with Unicode \\b");
  LookaroundDfa L(B.nodes, r, max_dfa_states, max_positions, B.uses_wordb);
  Dfa d = L.build();
  set_literals(out, B.nodes, r);
  out.wordb = B.uses_wordb;
  out.uword = false;
  out.cp_only = false;
  out.dfa = std::move(d);
  out.kind = Kind::DFA;
  out.error.clear();
}

// "(?#relax)" + pattern: the automaton of the pattern's relaxation (Relaxer); FALLBACK if even that
// is not regular enough for the automata. Java rejects "(?#" (no comment groups), so no library
// regex starts with the marker.
Compiled compile_relaxed(const std::string& pattern, int max_dfa_states, int max_positions, bool want_bpg) {
  Compiled out;
  try {
    Parser B(pattern, true);
    const int r = B.parse();
    out.wordb = B.uses_wordb;
    out.uword = B.uses_uword;
    if (B.uses_uword && B.uses_aword) { out.kind = Kind::FALLBACK; out.error = "mixed \\b semantics"; return out; }
    out.cp_only = B.uses_uword;
    Relaxer Rx(B.nodes);
    const int root = Rx.relax(r);
    return compile_nodes(std::move(out), std::move(Rx.out), root, max_dfa_states, max_positions, want_bpg, pattern);
  } catch (const std::exception& e) {
    out.kind = Kind::FALLBACK;
    out.error = std::string("relaxation: ") + e.what();
    return out;
  }
}

Compiled compile_impl(const std::string& pattern, int max_dfa_states, int max_positions, bool want_bpg) {
  static const std::string kRelax = "(?#relax)";
  if (pattern.compare(0, kRelax.size(), kRelax) == 0)
    return compile_relaxed(pattern.substr(kRelax.size()), max_dfa_states, max_positions, want_bpg);
  Compiled out;
  std::vector<Node> nodes;
  int root;
  try {
    Parser P(pattern);
    root = P.parse();
    nodes = std::move(P.nodes);
    out.wordb = P.uses_wordb;
    out.uword = P.uses_uword;
    if (P.uses_uword && P.uses_aword) {
      classify_fallback(out, pattern, "\\b with both ASCII and Unicode word semantics");
      return out;
    }
    // Unicode \b needs the wordness of whole code points, MULTILINE anchors the line-terminator
    // contexts: only the code-point automaton has them
    out.cp_only = P.needs_cp || P.uses_uword;
  } catch (const SyntaxError& e) {
    out.kind = Kind::INVALID; out.error = e.what(); return out;
  } catch (const Unsupported& e) {
    classify_fallback(out, pattern, e.what());
    if (out.kind == Kind::FALLBACK) {
      // a lookaround cluster (the backtracker accepted the pattern, so Java does): its exact
      // find() DFA when the construction applies and fits
      try {
        Compiled lk = out;
        compile_lookaround(lk, pattern, max_dfa_states, max_positions);
        return lk;
      } catch (const std::exception& e2) {
        out.error += std::string("; lookaround DFA: ") + e2.what();
      }
    }
    return out;
  } catch (const std::exception& e) {
    out.kind = Kind::INVALID; out.error = e.what(); return out;
  }
  trim_find(nodes, root);   // (not for relaxations: the Relaxer shares one any-string node)
  return compile_nodes(std::move(out), std::move(nodes), root, max_dfa_states, max_positions, want_bpg, pattern);
}

Compiled compile_nodes(Compiled out, std::vector<Node> nodes, int root, int max_dfa_states, int max_positions,
                       bool want_bpg, const std::string& pattern) {
  set_literals(out, nodes, root);
  std::string why = out.cp_only ? "code-point contexts" : "";
  if (!out.cp_only) {
    try {
      Lowerer Lw(nodes, false);
      const int broot = Lw.lower(root);
      Glushkov G(Lw.out, max_positions);
      Info top = G.build(broot);
      G.finish(top);
      check_ft(G.nfa);
      out.nfa = std::move(G.nfa);
      out.byte_nfa = true;
      out.dfa = build_dfa(out.nfa, out.wordb, max_dfa_states);
      out.kind = Kind::DFA;
      return out;
    } catch (const Unsupported& e) {
      why = e.what();
      if (why == "end anchor inside pattern") { classify_fallback(out, pattern, why); return out; }
      out.dfa = Dfa();
    }
  }
  // DFA blow-up (bounded gaps, repeated groups) or code-point contexts: the code-point NFA
  out.kind = Kind::NFA;
  out.error = why;
  if (want_bpg) {
    // with counted positions first (bounded repeats of one class as one position + a count); a
    // program with more counted repeats than the walk keeps counts for is built expanded
    for (bool counters : {true, false}) {
      try {
        Glushkov G(nodes, BPG_MAX_POS, counters);
        Info top = G.build(root);
        G.finish(top);
        check_ft(G.nfa);
        out.bpg = bpg_program(G.nfa, out.uword);
        out.error = why;
        break;
      } catch (const Unsupported& e) {
        out.error = why + "; bpg: " + e.what();
        out.bpg.clear();
      }
    }
  }
  if (out.bpg.empty() && !out.byte_nfa) {
    // neither a program nor a byte NFA (for the MFMA engine): the backtracker
    out.nfa = Nfa();
    classify_fallback(out, pattern, out.error);
    return out;
  }
  try {
    BtRegex check(pattern);
    out.bt_ok = true;
  } catch (const std::exception&) {
  }
  return out;
}
}  // namespace

Compiled compile(const std::string& pattern, int max_dfa_states, int max_positions) {
  return compile_impl(pattern, max_dfa_states, max_positions, true);
}

// ------------------------------------------------------------------------------------------
// multi-regex DFA: subset construction over the union of the members' position NFAs
namespace {

struct Member {
  int off = 0;
  const Nfa* nfa = nullptr;
};

uint64_t member_accepts(const std::vector<Member>& M, const std::vector<uint64_t>& A, int prev, int next) {
  const uint32_t bit = 1u << ctx_index(prev, next);
  uint64_t m = 0;
  for (size_t r = 0; r < M.size(); ++r) {
    const Nfa& n = *M[r].nfa;
    bool ok = (n.nullable & bit) != 0;
    for (size_t i = 0; !ok && i < n.last.size(); ++i) {
      const int p = M[r].off + n.last[i].to;
      ok = ((A[p >> 6] >> (p & 63)) & 1) && (n.last[i].cond & bit);
    }
    if (ok) m |= 1ull << r;
  }
  return m;
}

}  // namespace

MultiDfa compile_multi(const std::vector<std::string>& patterns, int max_states) {
  if (patterns.empty() || patterns.size() > (size_t)MULTI_MAX_REGS) throw Unsupported("multi-DFA: 1..64 regexes");
  std::vector<Compiled> comp;
  comp.reserve(patterns.size());
  bool wordb = false;
  for (auto& p : patterns) {
    comp.push_back(compile_impl(p, 4, 4096, false));
    const Compiled& c = comp.back();
    if ((c.kind != Kind::DFA && c.kind != Kind::NFA) || !c.byte_nfa)
      throw Unsupported("multi-DFA member has no byte automaton");
    wordb |= c.wordb;
  }
  std::vector<Member> M(comp.size());
  int np = 0;
  for (size_t r = 0; r < comp.size(); ++r) {
    M[r].off = np;
    M[r].nfa = &comp[r].nfa;
    np += comp[r].nfa.npos;
  }
  std::vector<const ByteSet*> cls(np);
  std::vector<std::vector<Edge>> follow(np);
  std::vector<Edge> first;
  bool restartable = false;
  for (auto& m : M) {
    for (int p = 0; p < m.nfa->npos; ++p) {
      cls[m.off + p] = &m.nfa->cls[p];
      for (auto& e : m.nfa->follow[p]) follow[m.off + p].push_back({m.off + e.to, e.cond});
    }
    for (auto& e : m.nfa->first) {
      first.push_back({m.off + e.to, e.cond});
      if (e.cond & CTX_NOT_BOS) restartable = true;
    }
    if (m.nfa->nullable & CTX_NOT_BOS) restartable = true;
  }
  MultiDfa d;
  d.nregs = (int)M.size();
  // byte classes: (membership in every distinct position class, word byte, UTF-8 continuation)
  std::vector<ByteSet> dcls;
  for (int p = 0; p < np; ++p) {
    bool f = false;
    for (auto& x : dcls) if (x == *cls[p]) { f = true; break; }
    if (!f) dcls.push_back(*cls[p]);
  }
  std::map<std::vector<bool>, int> sig2cls;
  d.bytemap.assign(256, 0);
  std::vector<int> rep;
  for (int b = 0; b < 256; ++b) {
    std::vector<bool> sig;
    for (auto& x : dcls) sig.push_back(x.test(b));
    sig.push_back(is_word_byte(b));
    sig.push_back(b >= 0x80 && b <= 0xBF);
    auto it = sig2cls.find(sig);
    int k;
    if (it == sig2cls.end()) { k = (int)rep.size(); sig2cls[sig] = k; rep.push_back(b); }
    else k = it->second;
    d.bytemap[b] = (uint8_t)k;
  }
  d.nclasses = (int)rep.size();
  if (d.nclasses > 256) throw Unsupported("too many byte classes");
  SubsetTables T;
  T.init(np, cls, follow, first, rep);
  const int nw = T.nw + 1;   // last word: prev kind
  std::unordered_map<std::vector<uint64_t>, int, KeyHash> ids;
  std::vector<std::vector<uint64_t>> states;
  auto intern = [&](std::vector<uint64_t>& key) -> int {
    auto it = ids.find(key);
    if (it != ids.end()) return it->second;
    const int id = (int)states.size() + 1;       // 0 = DEAD
    if (id >= max_states || id > 0xFFFF) throw Unsupported("multi-DFA state limit");
    ids.emplace(key, id);
    states.push_back(key);
    return id;
  };
  std::vector<uint64_t> init(nw, 0);
  init[nw - 1] = P_BOS;
  intern(init);
  std::vector<uint32_t> rows;
  std::vector<uint64_t> racc, fin;
  std::vector<uint64_t> U(nw, 0), B(nw, 0);
  for (size_t si = 0; si < states.size(); ++si) {
    const std::vector<uint64_t> A = states[si];
    const int prev = (int)A[nw - 1];
    fin.push_back(member_accepts(M, A, prev, N_EOS));
    fin.push_back(member_accepts(M, A, prev, N_FT));
    uint64_t acc_k[6];
    for (int nk = 0; nk < 6; ++nk) acc_k[nk] = member_accepts(M, A, prev, nk);
    T.ungated(A, U);
    for (int k = 0; k < d.nclasses; ++k) {
      const int c = rep[k];
      const int nk = next_kind_of_byte(c);
      std::fill(B.begin(), B.end(), 0);
      const bool any = T.step(A, U, k, c, 1u << ctx_index(prev, nk), cls, B);
      uint32_t next = 0;
      if (any || restartable) {
        B[nw - 1] = (uint64_t)((nk == N_W && wordb) ? P_W : P_N);
        next = (uint32_t)intern(B);
      }
      rows.push_back(next);
      racc.push_back(acc_k[nk]);
    }
  }
  d.nstates = (int)states.size() + 1;
  d.trans.assign((size_t)d.nclasses, 0);            // DEAD row
  d.trans.insert(d.trans.end(), rows.begin(), rows.end());
  d.acc.assign((size_t)d.nclasses, 0);
  d.acc.insert(d.acc.end(), racc.begin(), racc.end());
  d.fin.assign(2, 0);
  d.fin.insert(d.fin.end(), fin.begin(), fin.end());
  return d;
}

uint64_t multi_find(const MultiDfa& d, const uint8_t* s, int64_t n) {
  int64_t ft = n - final_terminator_len(s, n);
  if (ft == n) ft = -1;
  uint32_t st = 1;
  uint64_t acc = 0;
  for (int64_t t = 0; t < n; ++t) {
    if (t == ft) acc |= d.fin[2 * st + 1];
    const size_t i = (size_t)st * d.nclasses + d.bytemap[s[t]];
    acc |= d.acc[i];
    st = d.trans[i];
  }
  return acc | d.fin[2 * st];
}

// ------------------------------------------------------------------------------------------
// bit-parallel Glushkov programs over code points (layout documented in csrc/kernels/bpg.h)
namespace {

constexpr int kBpgWidths[] = {1, 2, 3, 4, 6, 8, 12, 16, 24, 32};

struct Bits {
  int nw = 0;
  std::vector<uint64_t> w;
  explicit Bits(int n = 0) : nw((n + 63) / 64), w(nw, 0) {}
  void set(int p) { w[p >> 6] |= 1ull << (p & 63); }
  bool test(int p) const { return (w[p >> 6] >> (p & 63)) & 1; }
  bool any() const { for (auto x : w) if (x) return true; return false; }
  bool subset_of(const Bits& o) const { for (int i = 0; i < nw; ++i) if (w[i] & ~o.w[i]) return false; return true; }
  void orr(const Bits& o) { for (int i = 0; i < nw; ++i) w[i] |= o.w[i]; }
  void andnot(const Bits& o) { for (int i = 0; i < nw; ++i) w[i] &= ~o.w[i]; }
  bool operator==(const Bits& o) const { return w == o.w; }
};

// the kind of a code point at code-point level: W / N / T (a line terminator)
int cp_kind(uint32_t c, bool uword) {
  if (is_line_term(c)) return N_T;
  if (c < 128) return is_word_byte((int)c) ? N_W : N_N;
  return (uword && unicode_word().contains(c)) ? N_W : N_N;
}

}  // namespace

std::vector<uint64_t> bpg_program(const Nfa& nf, bool uword) {
  const int np = nf.npos;
  if (np <= 0) throw Unsupported("empty program");
  if (np > BPG_MAX_POS) throw Unsupported("more than 2048 positions");
  int W = 0;
  for (int w : kBpgWidths) if (w * 64 >= np) { W = w; break; }
  // ---- decomposition of the follow relation: shift, self, spread fields, exceptions (exact)
  std::vector<Bits> F(np, Bits(np));
  std::vector<std::pair<int, std::pair<uint32_t, Bits>>> gated;   // (src, (cond, targets))
  {
    std::map<std::pair<int, uint32_t>, Bits> g;
    for (int p = 0; p < np; ++p)
      for (auto& e : nf.follow[p]) {
        if (e.cond == CTX_ALL) F[p].set(e.to);
        else {
          auto it = g.find({p, e.cond});
          if (it == g.end()) it = g.emplace(std::make_pair(p, e.cond), Bits(np)).first;
          it->second.set(e.to);
        }
      }
    for (auto& kv : g) gated.push_back({kv.first.first, {kv.first.second, kv.second}});
  }
  Bits shift(np), selfl(np);
  std::vector<Bits> covered(np, Bits(np));
  for (int p = 0; p < np; ++p) {
    if (p + 1 < np && F[p].test(p + 1)) { shift.set(p); covered[p].set(p + 1); }
    if (F[p].test(p)) { selfl.set(p); covered[p].set(p); }
  }
  Bits src_all(np), R_all(np), lo_all(np), hi_all(np);
  for (int p = 0; p < np;) {
    // forward targets not yet covered
    bool fwd = false;
    int hi = -1, nR = 0;
    for (int q = p + 1; q < np; ++q)
      if (F[p].test(q)) { ++nR; hi = q; if (!covered[p].test(q)) fwd = true; }
    if (!fwd || hi - p < 1 || nR < 2) { ++p; continue; }
    Bits R(np);
    for (int q = p + 1; q <= hi; ++q) if (F[p].test(q)) R.set(q);
    // sources: every s in [p, hi] that reaches all targets above it (a field grows while they do)
    std::vector<int> src;
    for (int s = p; s <= hi; ++s) {
      Bits above = R;
      for (int q = 0; q <= s && q < np; ++q) if (above.test(q)) above.w[q >> 6] &= ~(1ull << (q & 63));
      if (above.subset_of(F[s])) src.push_back(s);
    }
    for (int s : src) {
      src_all.set(s);
      for (int q = s + 1; q <= hi; ++q) if (R.test(q)) covered[s].set(q);
    }
    R_all.orr(R);
    lo_all.set(p);
    hi_all.set(hi);
    p = hi + 1;
  }
  struct Exc { int src; uint32_t cond; Bits tos; };
  std::vector<Exc> exc;
  for (int p = 0; p < np; ++p) {
    Bits rest = F[p];
    rest.andnot(covered[p]);
    if (rest.any()) exc.push_back({p, CTX_ALL, rest});
    Bits extra = covered[p];
    extra.andnot(F[p]);
    if (extra.any()) throw Unsupported("bpg decomposition is not exact");
  }
  for (auto& g : gated) exc.push_back({g.first, g.second.first, g.second.second});
  std::sort(exc.begin(), exc.end(), [](const Exc& a, const Exc& b) { return a.src < b.src; });
  if ((int)exc.size() > BPG_MAX_EXC) throw Unsupported("too many exception edges");
  // ---- code-point classes: elementary intervals with the same (kind, membership) signature
  std::vector<uint32_t> cuts = {0, 128, CpSet::MAX + 1};
  for (int c = 1; c < 128; ++c) cuts.push_back((uint32_t)c);
  for (auto& cs : nf.ccls)
    for (auto& r : cs.r) { cuts.push_back(r.first); cuts.push_back(r.second + 1); }
  for (uint32_t t : {0x85u, 0x2028u, 0x2029u}) { cuts.push_back(t); cuts.push_back(t + 1); }
  if (uword)
    for (auto& r : unicode_word().r) { cuts.push_back(r.first); cuts.push_back(r.second + 1); }
  std::sort(cuts.begin(), cuts.end());
  cuts.erase(std::unique(cuts.begin(), cuts.end()), cuts.end());
  std::map<std::pair<int, std::vector<uint64_t>>, int> sig2cls;
  std::vector<Bits> rows;
  std::vector<uint16_t> amap(128, 0);
  std::vector<uint64_t> ranges;   // lo | cls << 21 | kind << 37
  int last_cls = -1, last_kind = -1;
  for (size_t i = 0; i + 1 < cuts.size(); ++i) {
    const uint32_t lo = cuts[i];   // [lo, cuts[i + 1]) has one signature (no cut inside)
    if (lo > CpSet::MAX) break;
    const int kind = cp_kind(lo, uword);
    Bits mem(W * 64);
    for (int p = 0; p < np; ++p) if (nf.ccls[p].contains(lo)) mem.set(p);
    auto key = std::make_pair(kind, mem.w);
    auto it = sig2cls.find(key);
    int k;
    if (it == sig2cls.end()) {
      k = (int)rows.size();
      if (k >= BPG_MAX_CLS) throw Unsupported("too many code-point classes");
      sig2cls[key] = k;
      rows.push_back(mem);
    } else {
      k = it->second;
    }
    if (lo < 128) { amap[lo] = (uint16_t)k; continue; }
    const int kd = kind == N_W ? 1 : kind == N_T ? 2 : 0;
    if (k == last_cls && kd == last_kind) continue;      // merged with the previous interval
    ranges.push_back((uint64_t)lo | ((uint64_t)k << 21) | ((uint64_t)kd << 37));
    last_cls = k;
    last_kind = kd;
  }
  const int ncls = (int)rows.size();
  // ---- counted positions (bounded repeats of one class): (position, bound) after the ranges
  std::vector<uint64_t> ctrs;
  for (int p = 0; p < (int)nf.ctr.size() && p < np; ++p)
    if (nf.ctr[p] > 0) ctrs.push_back((uint64_t)p | ((uint64_t)nf.ctr[p] << 16));
  if ((int)ctrs.size() > BPG_MAX_CTR) throw Unsupported("too many counted repeats");
  // ---- first / last per context, header flags
  std::vector<uint64_t> first((size_t)NCTX * W, 0), last((size_t)NCTX * W, 0);
  for (auto& e : nf.first)
    for (int c = 0; c < NCTX; ++c) if ((e.cond >> c) & 1) first[(size_t)c * W + (e.to >> 6)] |= 1ull << (e.to & 63);
  for (auto& e : nf.last)
    for (int c = 0; c < NCTX; ++c) if ((e.cond >> c) & 1) last[(size_t)c * W + (e.to >> 6)] |= 1ull << (e.to & 63);
  bool uniform = true;
  for (int c = 1; c < NCTX && uniform; ++c)
    for (int w = 0; w < W; ++w)
      if (first[(size_t)c * W + w] != first[w] || last[(size_t)c * W + w] != last[w]) { uniform = false; break; }
  const uint32_t nullable = nf.nullable & CTX_ALL;
  bool anchored = (nullable >> 6) == 0;                  // first set only after BOS (prev kind 0)
  for (size_t i = 6 * (size_t)W; i < first.size() && anchored; ++i) if (first[i]) anchored = false;
  const uint64_t E = exc.size();
  const uint64_t hdr = (uint64_t)W | (E << 8) | ((uint64_t)ncls << 20) | (anchored ? 1ull << 30 : 0) |
                       (uniform ? 1ull << 31 : 0) | ((uint64_t)nullable << 32) | (uword ? 1ull << 56 : 0) |
                       ((uint64_t)ctrs.size() << 57);
  std::vector<uint64_t> P;
  P.push_back(hdr);
  P.push_back(0);   // hdr2: nranges | total words << 32 (below)
  auto put = [&](const Bits& b) { for (int w = 0; w < W; ++w) P.push_back(w < b.nw ? b.w[w] : 0); };
  auto widen = [&](const Bits& b) { Bits o(W * 64); for (int w = 0; w < b.nw; ++w) o.w[w] = b.w[w]; return o; };
  put(widen(shift)); put(widen(selfl)); put(widen(src_all)); put(widen(R_all)); put(widen(lo_all)); put(widen(hi_all));
  P.insert(P.end(), first.begin(), first.end());
  P.insert(P.end(), last.begin(), last.end());
  for (int i = 0; i < 128; i += 4)
    P.push_back((uint64_t)amap[i] | ((uint64_t)amap[i + 1] << 16) | ((uint64_t)amap[i + 2] << 32) | ((uint64_t)amap[i + 3] << 48));
  for (auto& r : rows) put(r);
  for (auto& e : exc) {
    P.push_back((uint64_t)e.src | ((uint64_t)e.cond << 16));
    put(widen(e.tos));
  }
  P.insert(P.end(), ranges.begin(), ranges.end());
  P.insert(P.end(), ctrs.begin(), ctrs.end());
  P[1] = (uint64_t)ranges.size() | ((uint64_t)P.size() << 32);
  return P;
}

// ------------------------------------------------------------------------------------------
// backtracking VM (Java semantics for non-regular constructs)
namespace {

enum BOp : uint8_t { B_SET, B_SPLIT, B_JMP, B_SAVE, B_ASSERT, B_BREF, B_LOOK, B_ATOMIC, B_MARK, B_PROGRESS, B_ML,
                     B_MATCH };
struct BInst {
  BOp op;
  int x = 0, y = 0;        // SET: set id; SPLIT: preferred / other pc; JMP/SAVE/MARK/PROGRESS/BREF/LOOK/ATOMIC: arg
  uint32_t cond = 0;       // ASSERT
  bool f1 = false, f2 = false;   // BREF: ci; LOOK: behind, neg; ML: kind ($), unix lines; ASSERT: Unicode word
  int lo = 0, hi = 0;      // LOOK behind: byte-length bounds of the sub-pattern
};

constexpr int kMaxBtInsts = 1 << 18;

}  // namespace

struct BtRegex::Impl {
  std::vector<std::vector<BInst>> progs;   // [0] = main; sub-programs of lookaround / atomic groups
  std::vector<ByteSet> sets;
  int ncaps = 0, nmarks = 0;
  bool bos_only = false;                   // every match starts at BOS (leading \A / ^)
};

namespace {

struct BtCompiler {
  const std::vector<Node>& N;
  BtRegex::Impl& I;
  int total = 0;

  int new_prog() { I.progs.emplace_back(); return (int)I.progs.size() - 1; }
  int emit(int p, BInst in) {
    if (++total > kMaxBtInsts) throw Unsupported("backtracking program too large");
    I.progs[p].push_back(in);
    return (int)I.progs[p].size() - 1;
  }
  static constexpr int64_t INF = int64_t(1) << 40;
  void bounds(int id, int64_t& mn, int64_t& mx) const {
    const Node& n = N[id];
    switch (n.t) {
      case N_EMPTY: case N_ASSERT: case N_LOOK: case N_MLANCHOR: mn = mx = 0; return;
      case N_SET: case N_CSET: mn = mx = 1; return;
      case N_GROUP: case N_ATOMIC: bounds(n.kids[0], mn, mx); return;
      case N_BACKREF: mn = 0; mx = INF; return;
      case N_CAT: {
        mn = mx = 0;
        for (int k : n.kids) { int64_t a, b; bounds(k, a, b); mn += a; mx = (mx >= INF || b >= INF) ? INF : mx + b; }
        return;
      }
      case N_ALT: {
        mn = INF; mx = 0;
        for (int k : n.kids) { int64_t a, b; bounds(k, a, b); mn = std::min(mn, a); mx = std::max(mx, b); }
        return;
      }
      case N_REP: {
        int64_t a, b; bounds(n.kids[0], a, b);
        mn = a * n.lo;
        mx = (n.hi < 0 || b >= INF) ? (b == 0 ? 0 : INF) : b * n.hi;
        return;
      }
    }
    mn = 0; mx = INF;
  }
  void comp(int p, int id) {
    const Node& n = N[id];
    switch (n.t) {
      case N_EMPTY: case N_CSET: return;    // (N_CSET never reaches here: lowered)
      case N_SET: {
        BInst in{B_SET}; in.x = (int)I.sets.size(); I.sets.push_back(n.set); emit(p, in); return;
      }
      case N_CAT: for (int k : n.kids) comp(p, k); return;
      case N_ALT: {
        std::vector<int> jumps;
        for (size_t a = 0; a < n.kids.size(); ++a) {
          if (a + 1 < n.kids.size()) {
            const int sp = emit(p, BInst{B_SPLIT});
            I.progs[p][sp].x = sp + 1;
            comp(p, n.kids[a]);
            jumps.push_back(emit(p, BInst{B_JMP}));
            I.progs[p][sp].y = (int)I.progs[p].size();
          } else {
            comp(p, n.kids[a]);
          }
        }
        for (int j : jumps) I.progs[p][j].x = (int)I.progs[p].size();
        return;
      }
      case N_REP: {
        for (int k = 0; k < n.lo; ++k) comp(p, n.kids[0]);
        if (n.hi < 0) {   // loop; an empty iteration ends it (keeping its captures), as Java's Loop
          const int m = I.nmarks++;
          const int sp = emit(p, BInst{B_SPLIT});
          BInst mk{B_MARK}; mk.x = m; emit(p, mk);
          comp(p, n.kids[0]);
          BInst pr{B_PROGRESS}; pr.x = m;
          const int pi = emit(p, pr);
          BInst j{B_JMP}; j.x = sp; emit(p, j);
          const int out = (int)I.progs[p].size();
          I.progs[p][pi].y = out;
          I.progs[p][sp].x = n.lazy ? out : sp + 1;
          I.progs[p][sp].y = n.lazy ? sp + 1 : out;
        } else {
          std::vector<int> splits;
          for (int k = n.lo; k < n.hi; ++k) {
            splits.push_back(emit(p, BInst{B_SPLIT}));
            comp(p, n.kids[0]);
          }
          const int out = (int)I.progs[p].size();
          for (int sp : splits) {
            I.progs[p][sp].x = n.lazy ? out : sp + 1;
            I.progs[p][sp].y = n.lazy ? sp + 1 : out;
          }
        }
        return;
      }
      case N_ASSERT: { BInst in{B_ASSERT}; in.cond = n.cond; in.f1 = n.uword; emit(p, in); return; }
      case N_GROUP: {
        I.ncaps = std::max(I.ncaps, 2 * n.idx + 2);
        BInst a{B_SAVE}; a.x = 2 * n.idx; emit(p, a);
        comp(p, n.kids[0]);
        BInst b{B_SAVE}; b.x = 2 * n.idx + 1; emit(p, b);
        return;
      }
      case N_BACKREF: {
        I.ncaps = std::max(I.ncaps, 2 * n.idx + 2);
        BInst in{B_BREF}; in.x = n.idx; in.f1 = n.ci; emit(p, in); return;
      }
      case N_LOOK: case N_ATOMIC: {
        const int sub = new_prog();
        comp(sub, n.kids[0]);
        emit(sub, BInst{B_MATCH});
        BInst in{n.t == N_LOOK ? B_LOOK : B_ATOMIC};
        in.x = sub;
        if (n.t == N_LOOK) {
          in.f1 = n.behind;
          in.f2 = n.neg;
          if (n.behind) {
            int64_t mn, mx;
            bounds(n.kids[0], mn, mx);
            if (mx >= INF) throw SyntaxError("Look-behind group does not have an obvious maximum length");
            in.lo = (int)mn;
            in.hi = (int)mx;
          }
        }
        emit(p, in);
        return;
      }
      case N_MLANCHOR: { BInst in{B_ML}; in.f1 = n.idx == 1; in.f2 = n.neg; emit(p, in); return; }
    }
  }
};

struct BtRun {
  const BtRegex::Impl& I;
  const uint8_t* s;
  int64_t n, ft;
  int64_t steps = 0, budget;
  bool exhausted = false;

  uint32_t ctx_bit(int64_t i, bool uword) const {
    int prev, next;
    if (!uword) {
      prev = i == 0 ? P_BOS : (is_word_byte(s[i - 1]) ? P_W : P_N);
      if (i == n) next = N_EOS;
      else if (i == ft) next = N_FT;
      else next = next_kind_of_byte(s[i]);
    } else {   // Unicode WORD on whole code points
      if (i == 0) {
        prev = P_BOS;
      } else {
        int64_t j = i - 1;
        while (j > 0 && s[j] >= 0x80 && s[j] <= 0xBF) --j;
        int len;
        const uint32_t c = decode_at(s, n, j, &len);
        prev = (c < 128 ? is_word_byte((int)c) : unicode_word().contains(c)) ? P_W : P_N;
      }
      if (i == n) next = N_EOS;
      else if (i == ft) next = N_FT;
      else if (s[i] >= 0x80 && s[i] <= 0xBF) next = N_C;
      else {
        int len;
        const uint32_t c = decode_at(s, n, i, &len);
        next = (c < 128 ? is_word_byte((int)c) : unicode_word().contains(c)) ? N_W : N_N;
      }
    }
    return 1u << ctx_index(prev, next);
  }
  // line terminator (Java: \n \r U+0085 U+2028 U+2029) starting / ending at byte i
  bool term_at(int64_t i) const {
    if (i >= n) return false;
    const uint8_t c = s[i];
    if (c == '\n' || c == '\r') return true;
    if (c == 0xC2 && i + 1 < n && s[i + 1] == 0x85) return true;
    return c == 0xE2 && i + 2 < n && s[i + 1] == 0x80 && (s[i + 2] == 0xA8 || s[i + 2] == 0xA9);
  }
  bool term_before(int64_t i) const {
    if (i <= 0) return false;
    const uint8_t c = s[i - 1];
    if (c == '\n' || c == '\r') return true;
    if (c == 0x85 && i >= 2 && s[i - 2] == 0xC2) return true;
    return (c == 0xA8 || c == 0xA9) && i >= 3 && s[i - 3] == 0xE2 && s[i - 2] == 0x80;
  }
  bool ml_anchor(const BInst& in, int64_t i) const {
    if (!in.f1) {                                  // '^' (Pattern.Caret / UnixCaret)
      if (i == n) return false;                    // Perl: not at end of input, even after a newline
      if (i == 0) return true;
      if (in.f2) return s[i - 1] == '\n';
      if (!term_before(i)) return false;
      return !(s[i - 1] == '\r' && s[i] == '\n');
    }
    if (i == n) return true;                       // '$' (Pattern.Dollar multiline / UnixDollar)
    if (in.f2) return s[i] == '\n';
    if (s[i] == '\n') return !(i > 0 && s[i - 1] == '\r');
    return term_at(i);
  }

  struct Frame { int kind; int a; int64_t b; };   // 0: alternative (pc, pos); 1: cap undo; 2: mark undo

  // run program p from pos; req_end >= 0: only a match ending exactly there counts
  bool run(int p, int64_t pos, std::vector<int64_t>& caps, std::vector<int64_t>& marks, int64_t req_end,
           int64_t* end_out) {
    const std::vector<BInst>& code = I.progs[p];
    std::vector<Frame> st;
    int pc = 0;
    for (;;) {
      if (++steps > budget) { exhausted = true; return false; }
      const BInst& in = code[pc];
      bool ok = true;
      switch (in.op) {
        case B_SET:
          if (pos < n && I.sets[in.x].test(s[pos])) { ++pos; ++pc; } else ok = false;
          break;
        case B_SPLIT: st.push_back({0, in.y, pos}); pc = in.x; break;
        case B_JMP: pc = in.x; break;
        case B_SAVE: st.push_back({1, in.x, caps[in.x]}); caps[in.x] = pos; ++pc; break;
        case B_MARK: st.push_back({2, in.x, marks[in.x]}); marks[in.x] = pos; ++pc; break;
        case B_PROGRESS: pc = pos == marks[in.x] ? in.y : pc + 1; break;
        case B_ASSERT: if (ctx_bit(pos, in.f1) & in.cond) ++pc; else ok = false; break;
        case B_ML: if (ml_anchor(in, pos)) ++pc; else ok = false; break;
        case B_BREF: {
          const int64_t a = caps[2 * in.x], b = caps[2 * in.x + 1];
          if (a < 0 || b < 0) { ok = false; break; }
          const int64_t len = b - a;
          if (pos + len > n) { ok = false; break; }
          for (int64_t k = 0; k < len && ok; ++k) {
            int x = s[a + k], y = s[pos + k];
            if (in.f1) { x = (x >= 'A' && x <= 'Z') ? x + 32 : x; y = (y >= 'A' && y <= 'Z') ? y + 32 : y; }
            ok = x == y;
          }
          if (ok) { pos += len; ++pc; }
          break;
        }
        case B_LOOK: case B_ATOMIC: {
          std::vector<int64_t> c2 = caps, m2 = marks;
          int64_t e = -1;
          bool m = false;
          if (in.op == B_LOOK && in.f1) {          // lookbehind: every start within the length bounds
            for (int64_t j = pos - in.lo; j >= 0 && j >= pos - in.hi && !m; --j) {
              c2 = caps;
              m = run(in.x, j, c2, m2, pos, &e);
              if (exhausted) return false;
            }
          } else {
            m = run(in.x, pos, c2, m2, -1, &e);
            if (exhausted) return false;
          }
          if (in.op == B_LOOK && in.f2) m = !m;
          if (!m) { ok = false; break; }
          if (!(in.op == B_LOOK && in.f2))         // keep the group's captures (undoable)
            for (size_t k = 0; k < caps.size(); ++k)
              if (c2[k] != caps[k]) { st.push_back({1, (int)k, caps[k]}); caps[k] = c2[k]; }
          if (in.op == B_ATOMIC) pos = e;          // no backtracking into the atomic group
          ++pc;
          break;
        }
        case B_MATCH:
          if (req_end < 0 || pos == req_end) { if (end_out) *end_out = pos; return true; }
          ok = false;
          break;
      }
      if (ok) continue;
      for (;;) {                                   // backtrack
        if (st.empty()) return false;
        const Frame f = st.back();
        st.pop_back();
        if (f.kind == 1) caps[f.a] = f.b;
        else if (f.kind == 2) marks[f.a] = f.b;
        else { pc = f.a; pos = f.b; break; }
      }
    }
  }
};

}  // namespace

BtRegex::BtRegex(const std::string& pattern) {
  Parser P(pattern, true);
  const int root = P.parse();
  Lowerer Lw(P.nodes, true);
  const int broot = Lw.lower(root);
  auto impl = std::make_shared<Impl>();
  impl->ncaps = 2 * P.ngroups + 2;
  BtCompiler C{Lw.out, *impl};
  C.new_prog();
  C.comp(0, broot);
  C.emit(0, BInst{B_MATCH});
  const std::vector<BInst>& code = impl->progs[0];
  impl->bos_only = !code.empty() && code[0].op == B_ASSERT && code[0].cond == mask_where(f_bos);
  p_ = impl;
}

bool BtRegex::find(const uint8_t* s, int64_t n, int64_t budget, bool* exhausted) const {
  const Impl& I = *p_;
  BtRun R{I, s, n, -1, 0, budget};
  const int ftl = final_terminator_len(s, n);
  R.ft = ftl ? n - ftl : -1;
  std::vector<int64_t> caps(I.ncaps, -1), marks(std::max(I.nmarks, 1), -1);
  for (int64_t start = 0; start <= n; ++start) {
    if (start > 0 && start < n && s[start] >= 0x80 && s[start] <= 0xBF) continue;   // inside a code point
    std::fill(caps.begin(), caps.end(), -1);
    if (R.run(0, start, caps, marks, -1, nullptr)) return true;
    if (R.exhausted) break;
    if (I.bos_only) break;
  }
  if (exhausted) *exhausted = R.exhausted;
  return false;
}

}  // namespace lp
