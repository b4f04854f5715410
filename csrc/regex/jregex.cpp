// Java-regex -> literal factors + Glushkov NFA + byte DFA.  See jregex.h for the design.
#include "jregex.h"

#include <algorithm>
#include <cctype>
#include <cstring>
#include <map>
#include <set>
#include <unordered_map>

namespace lp {
namespace {

// ------------------------------------------------------------------------------------------
// code-point sets (ASCII bitmap + non-ASCII part: NONE / finite / ALL / PARTIAL)
struct CodeSet {
  uint64_t a[2] = {0, 0};          // ASCII 0..127
  enum Mode { FIN, ALL, PARTIAL } mode = FIN;
  std::set<uint32_t> cps;          // finite non-ASCII code points (mode FIN)

  void add(uint32_t cp) {
    if (cp < 128) { a[cp >> 6] |= 1ull << (cp & 63); return; }
    if (mode == FIN) { cps.insert(cp); if (cps.size() > 256) { mode = PARTIAL; cps.clear(); } }
  }
  void add_range(uint32_t lo, uint32_t hi) {
    for (uint32_t c = lo; c <= hi && c < 128; ++c) add(c);
    if (hi >= 128) {
      uint32_t l2 = std::max<uint32_t>(lo, 128);
      if (l2 <= 128 && hi >= 0x10FFFF) { mode = ALL; cps.clear(); return; }
      if (mode == ALL) return;
      if (hi - l2 > 256) { mode = PARTIAL; cps.clear(); return; }
      for (uint32_t c = l2; c <= hi; ++c) add(c);
    }
  }
  bool has_ascii(int c) const { return (a[c >> 6] >> (c & 63)) & 1; }
  void unite(const CodeSet& o) {
    a[0] |= o.a[0]; a[1] |= o.a[1];
    if (mode == ALL || o.mode == ALL) { mode = ALL; cps.clear(); return; }
    if (mode == PARTIAL || o.mode == PARTIAL) { mode = PARTIAL; cps.clear(); return; }
    for (auto c : o.cps) add(c);
  }
  void intersect(const CodeSet& o) {
    a[0] &= o.a[0]; a[1] &= o.a[1];
    if (o.mode == ALL) return;
    if (mode == ALL) { mode = o.mode; cps = o.cps; return; }
    if (mode == FIN && o.mode == FIN) {
      std::set<uint32_t> r;
      for (auto c : cps) if (o.cps.count(c)) r.insert(c);
      cps.swap(r);
      return;
    }
    mode = PARTIAL; cps.clear();
  }
  void negate() {
    a[0] = ~a[0]; a[1] = ~a[1];
    if (mode == ALL) { mode = FIN; cps.clear(); }
    else if (mode == FIN && cps.empty()) mode = ALL;
    else { mode = PARTIAL; cps.clear(); }
  }
};

// ------------------------------------------------------------------------------------------
// AST
// N_GROUP .. N_MLANCHOR only exist in backtracking mode (Parser(..., bt = true)); the automaton
// path rejects their constructs as Unsupported before building them.
enum NT { N_EMPTY, N_SET, N_CAT, N_ALT, N_REP, N_ASSERT, N_GROUP, N_BACKREF, N_LOOK, N_ATOMIC, N_MLANCHOR };
struct Node {
  NT t = N_EMPTY;
  ByteSet set;
  std::vector<int> kids;
  int lo = 0, hi = 0;      // REP (hi = -1: unbounded)
  uint16_t cond = CTX_ALL; // ASSERT
  int idx = 0;             // GROUP / BACKREF: group number; MLANCHOR: 0 '^', 1 '$'
  bool behind = false;     // LOOK: lookbehind
  bool neg = false;        // LOOK: negative
  bool ci = false;         // BACKREF: case-insensitive compare
  bool lazy = false;       // REP: reluctant (priority order matters inside atomic groups)
};

bool is_word_byte(int c) {
  return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '_';
}

uint16_t mask_where(bool (*f)(int, int)) {
  uint16_t m = 0;
  for (int p = 0; p < 3; ++p)
    for (int n = 0; n < 5; ++n)
      if (f(p, n)) m |= (uint16_t)(1u << ctx_index(p, n));
  return m;
}
bool f_bos(int p, int n) { return p == P_BOS && n != N_C; }
bool f_eol(int, int n) { return n == N_EOS || n == N_FT; }
bool f_eos(int, int n) { return n == N_EOS; }
bool f_wb(int p, int n) { return n != N_C && (p == P_W) != (n == N_W); }
bool f_nwb(int p, int n) { return n != N_C && (p == P_W) == (n == N_W); }

struct Flags { bool ci = false, dotall = false, comments = false, multiline = false, unixl = false; };

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

 private:
  const std::string& s_;
  bool bt_ = false;
  size_t i_ = 0;
  Flags f_;
  std::map<std::string, int> names_;

  int add(Node n) { nodes.push_back(std::move(n)); return (int)nodes.size() - 1; }
  int mk_set(const ByteSet& b) { Node n; n.t = N_SET; n.set = b; return add(n); }
  int mk_assert(uint16_t c) { Node n; n.t = N_ASSERT; n.cond = c; return add(n); }
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

  static void utf8(uint32_t cp, std::vector<int>& out) {
    if (cp < 0x80) { out.push_back(cp); return; }
    if (cp < 0x800) { out.push_back(0xC0 | (cp >> 6)); out.push_back(0x80 | (cp & 0x3F)); return; }
    if (cp < 0x10000) { out.push_back(0xE0 | (cp >> 12)); out.push_back(0x80 | ((cp >> 6) & 0x3F)); out.push_back(0x80 | (cp & 0x3F)); return; }
    out.push_back(0xF0 | (cp >> 18)); out.push_back(0x80 | ((cp >> 12) & 0x3F));
    out.push_back(0x80 | ((cp >> 6) & 0x3F)); out.push_back(0x80 | (cp & 0x3F));
  }

  void add_ci(CodeSet& cs, uint32_t cp) {
    cs.add(cp);
    if (f_.ci && cp < 128) {
      if (cp >= 'a' && cp <= 'z') cs.add(cp - 32);
      else if (cp >= 'A' && cp <= 'Z') cs.add(cp + 32);
    }
  }
  void add_range_ci(CodeSet& cs, uint32_t lo, uint32_t hi) {
    cs.add_range(lo, hi);
    if (f_.ci) for (uint32_t c = lo; c <= hi && c < 128; ++c) add_ci(cs, c);
  }

  // Lower a code-point set to an AST node over bytes.
  int set_node(const CodeSet& cs) {
    ByteSet b;
    for (int c = 0; c < 128; ++c) if (cs.has_ascii(c)) b.set(c);
    if (cs.mode == CodeSet::PARTIAL)
      throw Unsupported("character class with a partial non-ASCII range");
    if (cs.mode == CodeSet::ALL) {
      // any non-ASCII code point = lead byte followed by continuation bytes (valid UTF-8 input)
      b.set_range(0xC0, 0xFF);
      ByteSet cont; cont.set_range(0x80, 0xBF);
      int lead = mk_set(b);
      // at most 3 continuation bytes in valid UTF-8; the bound keeps lookbehind lengths finite
      int tail = mk_rep(mk_set(cont), 0, bt_ ? 3 : -1);
      if (bt_) {   // a code point is indivisible: backtracking must not give its bytes back
        Node n; n.t = N_ATOMIC; n.kids = {tail}; tail = add(n);
      }
      return mk_cat({lead, tail});
    }
    std::vector<int> alts;
    if (!b.empty() || cs.cps.empty()) alts.push_back(mk_set(b));
    for (auto cp : cs.cps) {
      std::vector<int> bytes; utf8(cp, bytes);
      std::vector<int> seq;
      for (int x : bytes) { ByteSet bb; bb.set(x); seq.push_back(mk_set(bb)); }
      alts.push_back(mk_cat(seq));
    }
    return mk_alt(alts);
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
          while (!eof() && peek() != '}') { v = v * 16 + hexval(peek()); ++i_; ++nd; }
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

  bool class_escape(CodeSet& cs) {  // predefined classes; i_ at the letter
    int c = peek();
    CodeSet t;
    bool neg = false;
    switch (c) {
      case 'd': case 'D': t.add_range('0', '9'); neg = c == 'D'; break;
      case 's': case 'S': for (uint32_t x : {' ', '\t', '\n', '\x0b', '\f', '\r'}) t.add(x); neg = c == 'S'; break;
      case 'w': case 'W': t.add_range('a', 'z'); t.add_range('A', 'Z'); t.add_range('0', '9'); t.add('_'); neg = c == 'W'; break;
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
        if (name.rfind("Is", 0) == 0) name = name.substr(2);
        auto R = [&](int lo, int hi) { t.add_range(lo, hi); };
        if (name == "Lower" || name == "javaLowerCase") { R('a', 'z'); if (f_.ci) R('A', 'Z'); }
        else if (name == "Upper" || name == "javaUpperCase") { R('A', 'Z'); if (f_.ci) R('a', 'z'); }
        else if (name == "ASCII") R(0, 127);
        else if (name == "Alpha") { R('a', 'z'); R('A', 'Z'); }
        else if (name == "Digit") R('0', '9');
        else if (name == "Alnum") { R('a', 'z'); R('A', 'Z'); R('0', '9'); }
        else if (name == "Punct") { R('!', '/'); R(':', '@'); R('[', '`'); R('{', '~'); }
        else if (name == "Graph") R('!', '~');
        else if (name == "Print") R(' ', '~');
        else if (name == "Blank") { t.add(' '); t.add('\t'); }
        else if (name == "Cntrl") { R(0, 0x1F); t.add(0x7F); }
        else if (name == "XDigit") { R('0', '9'); R('a', 'f'); R('A', 'F'); }
        else if (name == "Space" || name == "javaWhitespace") { for (uint32_t x : {' ', '\t', '\n', '\x0b', '\f', '\r'}) t.add(x); }
        else throw Unsupported("unicode property \\p{" + name + "}");
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

  CodeSet parse_class() {  // at '['
    ++i_;
    bool neg = false;
    if (peek() == '^') { neg = true; ++i_; }
    CodeSet cur;
    bool have_acc = false;
    CodeSet acc;
    bool first = true;
    for (;;) {
      if (eof()) throw SyntaxError("Unclosed character class");
      int c = peek();
      if (c == ']' && !first) { ++i_; break; }
      first = false;
      if (c == '[') { CodeSet sub = parse_class(); cur.unite(sub); continue; }
      if (c == '&' && i_ + 1 < s_.size() && s_[i_ + 1] == '&') {
        i_ += 2;
        if (!have_acc) { acc = cur; have_acc = true; } else acc.intersect(cur);
        cur = CodeSet();
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
    CodeSet res = cur;
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
        case 'u': break;   // UNICODE_CASE: ASCII behaviour identical; non-ASCII CI literals unsupported below
        case 'U': throw Unsupported("UNICODE_CHARACTER_CLASS");
        case 'c': throw Unsupported("CANON_EQ");
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
    if (c == '[') { CodeSet cs = parse_class(); return set_node(cs); }
    if (c == '.') {
      ++i_;
      CodeSet cs;
      cs.add_range(0, 127);
      cs.mode = CodeSet::ALL;
      if (!f_.dotall) {
        // Java: '.' excludes line terminators (\n \r; U+0085/U+2028/U+2029 are treated as ordinary
        // non-ASCII here — documented divergence). UNIX_LINES: only \n.
        cs.a[0] &= ~(1ull << '\n');
        if (!f_.unixl) cs.a[0] &= ~(1ull << '\r');
      }
      return set_node(cs);
    }
    if (c == '^') {
      ++i_;
      if (f_.multiline) {
        if (!bt_) throw Unsupported("MULTILINE ^");
        Node n; n.t = N_MLANCHOR; n.idx = 0; n.neg = f_.unixl; return add(n);
      }
      return mk_assert(mask_where(f_bos));
    }
    if (c == '$') {
      ++i_;
      if (f_.multiline) {
        if (!bt_) throw Unsupported("MULTILINE $");
        Node n; n.t = N_MLANCHOR; n.idx = 1; n.neg = f_.unixl; return add(n);
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
        case 'b': ++i_; uses_wordb = true; return mk_assert(mask_where(f_wb));
        case 'B': ++i_; uses_wordb = true; return mk_assert(mask_where(f_nwb));
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
          // (?:\r\n|[\n\x0B\f\r\x85  ])
          ByteSet cr; cr.set('\r'); ByteSet nl; nl.set('\n');
          int crlf = mk_cat({mk_set(cr), mk_set(nl)});
          CodeSet v; for (uint32_t x : {0x0Au, 0x0Bu, 0x0Cu, 0x0Du, 0x85u, 0x2028u, 0x2029u}) v.add(x);
          return mk_alt({crlf, set_node(v)});
        }
        case 'X': throw Unsupported("\\X grapheme cluster");
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
      CodeSet cs;
      if (class_escape(cs)) return set_node(cs);
      uint32_t cp;
      if (!char_escape(cp)) throw SyntaxError("Illegal/unsupported escape sequence");
      return literal_node(cp);
    }
    if (c == ')') throw SyntaxError("Unmatched closing ')'");
    return literal_node(read_cp());
  }

  int literal_node(uint32_t cp) {
    if (cp < 128) {
      CodeSet cs; add_ci(cs, cp);
      ByteSet b;
      for (int x = 0; x < 128; ++x) if (cs.has_ascii(x)) b.set(x);
      return mk_set(b);
    }
    std::vector<int> bytes; utf8(cp, bytes);
    std::vector<int> seq;
    for (int x : bytes) { ByteSet bb; bb.set(x); seq.push_back(mk_set(bb)); }
    return mk_cat(seq);
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
// Glushkov construction with boundary conditions
struct Info {
  uint16_t nullable = 0;
  std::vector<Edge> first, last;
};

class Glushkov {
 public:
  Glushkov(const std::vector<Node>& N, int max_pos) : N_(N), max_pos_(max_pos) {}
  Nfa nfa;
  std::vector<std::map<int, uint16_t>> fol;

  Info build(int id) {
    const Node& n = N_[id];
    Info r;
    switch (n.t) {
      case N_EMPTY: r.nullable = CTX_ALL; return r;
      case N_ASSERT: r.nullable = n.cond; return r;
      case N_SET: {
        int p = nfa.npos++;
        if (nfa.npos > max_pos_) throw Unsupported("too many NFA positions");
        nfa.cls.push_back(n.set);
        fol.emplace_back();
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
    nfa.follow.resize(nfa.npos);
    for (int p = 0; p < nfa.npos; ++p)
      for (auto& kv : fol[p]) nfa.follow[p].push_back({kv.first, kv.second});
  }

 private:
  const std::vector<Node>& N_;
  int max_pos_;

  static void merge(std::vector<Edge>& v) {
    std::map<int, uint16_t> m;
    for (auto& e : v) m[e.to] |= e.cond;
    v.clear();
    for (auto& kv : m) if (kv.second) v.push_back({kv.first, kv.second});
  }
  void link(const std::vector<Edge>& from, const std::vector<Edge>& to) {
    for (auto& a : from)
      for (auto& b : to) {
        uint16_t c = a.cond & b.cond;
        if (c) fol[a.to][b.to] |= c;
      }
  }
  void loop(Info& c) { link(c.last, c.first); }
  Info cat(const Info& a, const Info& b) {
    Info r;
    r.nullable = a.nullable & b.nullable;
    r.first = a.first;
    for (auto& e : b.first) { uint16_t c = e.cond & a.nullable; if (c) r.first.push_back({e.to, c}); }
    r.last = b.last;
    for (auto& e : a.last) { uint16_t c = e.cond & b.nullable; if (c) r.last.push_back({e.to, c}); }
    link(a.last, b.first);
    merge(r.first); merge(r.last);
    return r;
  }
};

// ------------------------------------------------------------------------------------------
// subset construction
struct KeyHash {
  size_t operator()(const std::vector<uint64_t>& v) const {
    size_t h = 1469598103934665603ull;
    for (auto x : v) { h ^= x; h *= 1099511628211ull; h ^= h >> 29; }
    return h;
  }
};

Dfa build_dfa(const Nfa& nfa, bool uses_wordb, int max_states) {
  Dfa d;
  const int np = nfa.npos;
  const int nw = (np + 63) / 64 + 1;  // last word: prev kind
  // byte classes: signature = (membership in every distinct position class, word bit)
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
    sig.reserve(dcls.size() + 1);
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

  // ACCEPT check helper
  auto accepts = [&](const std::vector<uint64_t>& A, int prev, int next) {
    uint16_t bit = (uint16_t)(1u << ctx_index(prev, next));
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

  d.trans.clear();
  d.accflags.clear();
  std::vector<std::vector<uint16_t>> rows;
  std::vector<uint8_t> acc;
  for (size_t si = 0; si < states.size(); ++si) {
    std::vector<uint64_t> A = states[si];
    int prev = (int)A[nw - 1];
    uint8_t fl = 0;
    if (accepts(A, prev, N_EOS)) fl |= 1;
    if (accepts(A, prev, N_FT)) fl |= 2;
    acc.push_back(fl);
    std::vector<uint16_t> row(d.nclasses, 0);
    for (int k = 0; k < d.nclasses; ++k) {
      int c = rep[k];
      int nk = is_word_byte(c) ? N_W : (c >= 0x80 && c <= 0xBF) ? N_C : N_N;
      if (accepts(A, prev, nk)) { row[k] = 1; continue; }
      uint16_t bit = (uint16_t)(1u << ctx_index(prev, nk));
      std::vector<uint64_t> B(nw, 0);
      bool any = false;
      for (int p = 0; p < np; ++p) {
        if (!(A[p >> 6] >> (p & 63) & 1)) continue;
        for (auto& e : nfa.follow[p])
          if ((e.cond & bit) && nfa.cls[e.to].test(c)) { B[e.to >> 6] |= 1ull << (e.to & 63); any = true; }
      }
      for (auto& e : nfa.first)
        if ((e.cond & bit) && nfa.cls[e.to].test(c)) { B[e.to >> 6] |= 1ull << (e.to & 63); any = true; }
      int nprev = (nk == N_W && uses_wordb) ? P_W : P_N;
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
// pattern (INVALID), the native backtracker runs it (FALLBACK, bt_ok), or only the Python oracle
// translation can (FALLBACK) -- and take its literals for the device prefilter
void classify_fallback(Compiled& out, const std::string& pattern, const std::string& why) {
  out.kind = Kind::FALLBACK;
  out.error = why;
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
}  // namespace

Compiled compile(const std::string& pattern, int max_dfa_states, int max_positions) {
  Compiled out;
  std::vector<Node> nodes;
  int root;
  bool wordb = false;
  try {
    Parser P(pattern);
    root = P.parse();
    nodes = std::move(P.nodes);
    wordb = P.uses_wordb;
    out.wordb = wordb;
  } catch (const SyntaxError& e) {
    out.kind = Kind::INVALID; out.error = e.what(); return out;
  } catch (const Unsupported& e) {
    classify_fallback(out, pattern, e.what());
    return out;
  } catch (const std::exception& e) {
    out.kind = Kind::INVALID; out.error = e.what(); return out;
  }
  set_literals(out, nodes, root);
  try {
    Glushkov G(nodes, max_positions);
    Info top = G.build(root);
    G.finish(top);
    out.nfa = std::move(G.nfa);
    // a '$'-type condition on a consuming edge cannot be represented by the DFA's FT handling
    auto ft_sensitive = [](uint16_t c) {
      for (int p = 0; p < 3; ++p) {
        bool ft = (c >> ctx_index(p, N_FT)) & 1, nn = (c >> ctx_index(p, N_N)) & 1;
        if (ft != nn) return true;
      }
      return false;
    };
    for (auto& e : out.nfa.first) if (ft_sensitive(e.cond)) throw Unsupported("end anchor inside pattern");
    for (auto& v : out.nfa.follow) for (auto& e : v) if (ft_sensitive(e.cond)) throw Unsupported("end anchor inside pattern");
  } catch (const Unsupported& e) {
    out.kind = Kind::FALLBACK;
    out.error = e.what();
    try {
      BtRegex check(pattern);
      out.bt_ok = true;
    } catch (const std::exception&) {
    }
    return out;
  }
  try {
    out.dfa = build_dfa(out.nfa, wordb, max_dfa_states);
    out.kind = Kind::DFA;
  } catch (const Unsupported& e) {
    out.kind = Kind::NFA; out.error = e.what();
    try {
      BtRegex check(pattern);
      out.bt_ok = true;
    } catch (const std::exception&) {
    }
  }
  return out;
}

// ------------------------------------------------------------------------------------------
// multi-regex DFA: subset construction over the union of the members' position NFAs
namespace {

struct Member {
  int off = 0;
  const Nfa* nfa = nullptr;
};

uint32_t member_accepts(const std::vector<Member>& M, const std::vector<uint64_t>& A, int prev, int next) {
  const uint16_t bit = (uint16_t)(1u << ctx_index(prev, next));
  uint32_t m = 0;
  for (size_t r = 0; r < M.size(); ++r) {
    const Nfa& n = *M[r].nfa;
    bool ok = (n.nullable & bit) != 0;
    for (size_t i = 0; !ok && i < n.last.size(); ++i) {
      const int p = M[r].off + n.last[i].to;
      ok = ((A[p >> 6] >> (p & 63)) & 1) && (n.last[i].cond & bit);
    }
    if (ok) m |= 1u << r;
  }
  return m;
}

}  // namespace

MultiDfa compile_multi(const std::vector<std::string>& patterns, int max_states) {
  if (patterns.empty() || patterns.size() > (size_t)MULTI_MAX_REGS) throw Unsupported("multi-DFA: 1..16 regexes");
  std::vector<Compiled> comp;
  comp.reserve(patterns.size());
  bool wordb = false;
  for (auto& p : patterns) {
    comp.push_back(compile(p, 4, 4096));
    const Compiled& c = comp.back();
    if (c.kind != Kind::DFA && c.kind != Kind::NFA) throw Unsupported("multi-DFA member is not an automaton regex");
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
  const int nw = (np + 63) / 64 + 1;   // last word: prev kind
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
  std::vector<uint32_t> rows, fin;
  for (size_t si = 0; si < states.size(); ++si) {
    const std::vector<uint64_t> A = states[si];
    const int prev = (int)A[nw - 1];
    fin.push_back(member_accepts(M, A, prev, N_EOS));
    fin.push_back(member_accepts(M, A, prev, N_FT));
    uint32_t acc_k[5];
    for (int nk = 0; nk < 5; ++nk) acc_k[nk] = member_accepts(M, A, prev, nk);
    for (int k = 0; k < d.nclasses; ++k) {
      const int c = rep[k];
      const int nk = is_word_byte(c) ? N_W : (c >= 0x80 && c <= 0xBF) ? N_C : N_N;
      const uint16_t bit = (uint16_t)(1u << ctx_index(prev, nk));
      std::vector<uint64_t> B(nw, 0);
      bool any = false;
      for (int p = 0; p < np; ++p) {
        if (!(A[p >> 6] >> (p & 63) & 1)) continue;
        for (auto& e : follow[p])
          if ((e.cond & bit) && cls[e.to]->test(c)) { B[e.to >> 6] |= 1ull << (e.to & 63); any = true; }
      }
      for (auto& e : first)
        if ((e.cond & bit) && cls[e.to]->test(c)) { B[e.to >> 6] |= 1ull << (e.to & 63); any = true; }
      uint32_t next = 0;
      if (any || restartable) {
        B[nw - 1] = (uint64_t)((nk == N_W && wordb) ? P_W : P_N);
        next = (uint32_t)intern(B);
      }
      rows.push_back(next | (acc_k[nk] << 16));
    }
  }
  d.nstates = (int)states.size() + 1;
  d.trans.assign((size_t)d.nclasses, 0);            // DEAD row
  d.trans.insert(d.trans.end(), rows.begin(), rows.end());
  d.fin.assign(2, 0);
  d.fin.insert(d.fin.end(), fin.begin(), fin.end());
  return d;
}

uint32_t multi_find(const MultiDfa& d, const uint8_t* s, int64_t n) {
  int64_t ft = n - final_terminator_len(s, n);
  if (ft == n) ft = -1;
  uint32_t st = 1, acc = 0;
  for (int64_t t = 0; t < n; ++t) {
    if (t == ft) acc |= d.fin[2 * st + 1];
    const uint32_t e = d.trans[(size_t)st * d.nclasses + d.bytemap[s[t]]];
    acc |= e >> 16;
    st = e & 0xFFFF;
  }
  return acc | d.fin[2 * st];
}

// ------------------------------------------------------------------------------------------
// backtracking VM (Java semantics for non-regular constructs)
namespace {

enum BOp : uint8_t { B_SET, B_SPLIT, B_JMP, B_SAVE, B_ASSERT, B_BREF, B_LOOK, B_ATOMIC, B_MARK, B_PROGRESS, B_ML,
                     B_MATCH };
struct BInst {
  BOp op;
  int x = 0, y = 0;        // SET: set id; SPLIT: preferred / other pc; JMP/SAVE/MARK/PROGRESS/BREF/LOOK/ATOMIC: arg
  uint16_t cond = 0;       // ASSERT
  bool f1 = false, f2 = false;   // BREF: ci; LOOK: behind, neg; ML: kind ($), unix lines
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
      case N_SET: mn = mx = 1; return;
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
      case N_EMPTY: return;
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
      case N_ASSERT: { BInst in{B_ASSERT}; in.cond = n.cond; emit(p, in); return; }
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

  uint16_t ctx_bit(int64_t i) const {
    const int prev = i == 0 ? P_BOS : (is_word_byte(s[i - 1]) ? P_W : P_N);
    int next;
    if (i == n) next = N_EOS;
    else if (i == ft) next = N_FT;
    else if (is_word_byte(s[i])) next = N_W;
    else if (s[i] >= 0x80 && s[i] <= 0xBF) next = N_C;
    else next = N_N;
    return (uint16_t)(1u << ctx_index(prev, next));
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
        case B_ASSERT: if (ctx_bit(pos) & in.cond) ++pc; else ok = false; break;
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
  auto impl = std::make_shared<Impl>();
  impl->ncaps = 2 * P.ngroups + 2;
  BtCompiler C{P.nodes, *impl};
  C.new_prog();
  C.comp(0, root);
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
