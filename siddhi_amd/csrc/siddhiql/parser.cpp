// Recursive-descent parser for the SiddhiQL subset on the pattern/sequence hot path.
//
// Grammar followed: modules/siddhi-query-compiler/src/main/antlr4/.../SiddhiQL.g4
//   partition            :155-157      pattern_stream / chains       :200-256
//   pattern_source        :258-290     sequence_stream / chains      :300-353
//   math_operation        :456-470     (precedence: NOT > * / % > + - > < > <= >= > == != > AND > OR)
//   attribute_reference   :488-495     time_value                     :661-669
// Tree shapes follow SiddhiQLBaseVisitorImpl.java:748-1260 (pattern), :1131-1260 (sequence), :1396-1435 and
// :2402-2418 (collect). '->' and ',' chains are left-associative (ANTLR4 left recursion); the sequence top
// level is Next(first, rest) as in visitEvery_sequence_source_chain (:1131).
#include "ast.h"

#include <cctype>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <functional>
#include <map>

namespace sql {

namespace {

enum class Tk { END, ID, INT, LONG, FLOAT, DOUBLE, STRING, SYM };

struct Token {
  Tk t;
  std::string s;  // identifier / symbol / literal text (strings unquoted)
  size_t pos;
};

std::string lower(std::string s) {
  for (auto& c : s) c = (char)std::tolower((unsigned char)c);
  return s;
}

std::vector<Token> lex(const std::string& src) {
  std::vector<Token> out;
  size_t i = 0, n = src.size();
  while (i < n) {
    char c = src[i];
    if (std::isspace((unsigned char)c)) { ++i; continue; }
    if (c == '-' && i + 1 < n && src[i + 1] == '-') {  // SINGLE_LINE_COMMENT
      while (i < n && src[i] != '\n') ++i;
      continue;
    }
    if (c == '/' && i + 1 < n && src[i + 1] == '*') {  // MULTILINE_COMMENT
      size_t e = src.find("*/", i + 2);
      i = (e == std::string::npos) ? n : e + 2;
      continue;
    }
    size_t start = i;
    if (std::isalpha((unsigned char)c) || c == '_') {
      while (i < n && (std::isalnum((unsigned char)src[i]) || src[i] == '_')) ++i;
      out.push_back({Tk::ID, src.substr(start, i - start), start});
      continue;
    }
    if (c == '`') {  // ID_QUOTES
      size_t e = src.find('`', i + 1);
      if (e == std::string::npos) throw ParseError("unterminated quoted identifier");
      out.push_back({Tk::ID, src.substr(i + 1, e - i - 1), start});
      i = e + 1;
      continue;
    }
    if (std::isdigit((unsigned char)c) || (c == '.' && i + 1 < n && std::isdigit((unsigned char)src[i + 1]))) {
      bool frac = false, exp = false;
      while (i < n && std::isdigit((unsigned char)src[i])) ++i;
      if (i < n && src[i] == '.' && i + 1 <= n) {
        // avoid treating "e1.price" style (no: digits cannot start an id) — plain decimal point
        frac = true;
        ++i;
        while (i < n && std::isdigit((unsigned char)src[i])) ++i;
      }
      if (i < n && (src[i] == 'e' || src[i] == 'E')) {
        size_t j = i + 1;
        if (j < n && (src[j] == '+' || src[j] == '-')) ++j;
        if (j < n && std::isdigit((unsigned char)src[j])) {
          exp = true;
          i = j;
          while (i < n && std::isdigit((unsigned char)src[i])) ++i;
        }
      }
      std::string num = src.substr(start, i - start);
      Tk t = (frac || exp) ? Tk::DOUBLE : Tk::INT;
      if (i < n) {
        char s = src[i];
        if ((s == 'L' || s == 'l') && !frac && !exp) { t = Tk::LONG; ++i; }
        else if (s == 'f' || s == 'F') { t = Tk::FLOAT; ++i; }
        else if (s == 'd' || s == 'D') { t = Tk::DOUBLE; ++i; }
      }
      // "1sec": ANTLR lexes INT then the unit keyword; a letter right after a number starts a new token
      out.push_back({t, num, start});
      continue;
    }
    if (c == '\'' || c == '"') {
      if (c == '"' && src.compare(i, 3, "\"\"\"") == 0) {
        size_t e = src.find("\"\"\"", i + 3);
        if (e == std::string::npos) throw ParseError("unterminated string");
        out.push_back({Tk::STRING, src.substr(i + 3, e - i - 3), start});
        i = e + 3;
        continue;
      }
      size_t e = src.find(c, i + 1);
      if (e == std::string::npos) throw ParseError("unterminated string");
      out.push_back({Tk::STRING, src.substr(i + 1, e - i - 1), start});
      i = e + 1;
      continue;
    }
    static const char* syms[] = {"->", "==", "!=", ">=", "<=", "(", ")", "[", "]", "<", ">", ",", ".", ";",
                                 "*", "+", "?", "-", "/", "%", "#", "@", ":", "=", "!"};
    bool matched = false;
    for (const char* s : syms) {
      size_t L = std::strlen(s);
      if (src.compare(i, L, s) == 0) {
        out.push_back({Tk::SYM, s, start});
        i += L;
        matched = true;
        break;
      }
    }
    if (!matched) throw ParseError(std::string("unexpected character '") + c + "'");
  }
  out.push_back({Tk::END, "", n});
  return out;
}

struct Parser {
  std::vector<Token> tk;
  size_t p = 0;
  App app;
  int anon_query = 0;

  const Token& peek(int k = 0) const { return tk[std::min(p + k, tk.size() - 1)]; }
  bool is_sym(const char* s, int k = 0) const { return peek(k).t == Tk::SYM && peek(k).s == s; }
  bool is_kw(const char* s, int k = 0) const { return peek(k).t == Tk::ID && lower(peek(k).s) == s; }
  bool accept_sym(const char* s) {
    if (is_sym(s)) { ++p; return true; }
    return false;
  }
  bool accept_kw(const char* s) {
    if (is_kw(s)) { ++p; return true; }
    return false;
  }
  [[noreturn]] void fail(const std::string& what) const {
    const Token& t = peek();
    throw ParseError("Syntax error at offset " + std::to_string(t.pos) + " near '" + t.s + "': " + what);
  }
  void expect_sym(const char* s) {
    if (!accept_sym(s)) fail(std::string("expected '") + s + "'");
  }
  void expect_kw(const char* s) {
    if (!accept_kw(s)) fail(std::string("expected '") + s + "'");
  }
  std::string ident() {
    if (peek().t != Tk::ID) fail("expected identifier");
    return tk[p++].s;
  }

  // ---- annotations ----
  struct Annotation {
    std::string name;  // e.g. "app:playback", "info"
    std::vector<std::pair<std::string, std::string>> elems;
  };
  Annotation annotation() {
    expect_sym("@");
    Annotation a;
    a.name = lower(ident());
    if (accept_sym(":")) a.name += ":" + lower(ident());
    if (accept_sym("(")) {
      if (!is_sym(")")) {
        do {
          std::string key, val;
          if (peek().t == Tk::ID && (is_sym("=", 1) || is_sym(".", 1))) {
            key = ident();
            while (accept_sym(".")) key += "." + ident();
            expect_sym("=");
          }
          if (peek().t == Tk::STRING || peek().t == Tk::INT || peek().t == Tk::ID) val = tk[p++].s;
          else fail("expected annotation value");
          a.elems.push_back({lower(key), val});
        } while (accept_sym(","));
      }
      expect_sym(")");
    }
    return a;
  }

  // ---- time ----
  bool at_time_unit(int k = 0) const {
    if (peek(k).t != Tk::ID) return false;
    std::string u = lower(peek(k).s);
    static const char* units[] = {"year", "years", "month", "months", "week", "weeks", "day", "days", "hour",
                                  "hours", "min", "minute", "minutes", "sec", "second", "seconds", "millisec",
                                  "millisecond", "milliseconds"};
    for (auto* x : units)
      if (u == x) return true;
    return false;
  }
  int64_t time_value() {
    // time_value (SiddhiQL.g4:661): a sequence of INT unit pairs; summed in milliseconds.
    int64_t total = 0;
    bool any = false;
    while (peek().t == Tk::INT && at_time_unit(1)) {
      int64_t v = std::stoll(tk[p++].s);
      std::string u = lower(tk[p++].s);
      int64_t ms;
      if (u.rfind("year", 0) == 0) ms = 365LL * 24 * 3600 * 1000;  // TimeConstant.year: 365 days
      else if (u.rfind("month", 0) == 0) ms = 30LL * 24 * 3600 * 1000;
      else if (u.rfind("week", 0) == 0) ms = 7LL * 24 * 3600 * 1000;
      else if (u.rfind("day", 0) == 0) ms = 24LL * 3600 * 1000;
      else if (u.rfind("hour", 0) == 0) ms = 3600LL * 1000;
      else if (u.rfind("millisec", 0) == 0) ms = 1;
      else if (u.rfind("min", 0) == 0) ms = 60LL * 1000;
      else ms = 1000;  // sec / second(s)
      total += v * ms;
      any = true;
    }
    if (!any) fail("expected time value");
    return total;
  }

  // ---- expressions (math_operation, SiddhiQL.g4:456-470) ----
  ExprP mk(ExprKind k) {
    auto e = std::make_unique<Expr>();
    e->kind = k;
    return e;
  }
  ExprP bin(ExprKind k, ExprP l, ExprP r) {
    auto e = mk(k);
    e->ch.push_back(std::move(l));
    e->ch.push_back(std::move(r));
    return e;
  }
  ExprP expr() { return or_expr(); }
  ExprP or_expr() {
    ExprP l = and_expr();
    while (accept_kw("or")) l = bin(ExprKind::OR, std::move(l), and_expr());
    return l;
  }
  ExprP and_expr() {
    ExprP l = eq_expr();
    while (accept_kw("and")) l = bin(ExprKind::AND, std::move(l), eq_expr());
    return l;
  }
  ExprP eq_expr() {
    ExprP l = rel_expr();
    for (;;) {
      if (accept_sym("==")) { auto e = bin(ExprKind::CMP, std::move(l), rel_expr()); e->cmp = CmpOp::EQ; l = std::move(e); }
      else if (accept_sym("!=")) { auto e = bin(ExprKind::CMP, std::move(l), rel_expr()); e->cmp = CmpOp::NE; l = std::move(e); }
      else break;
    }
    return l;
  }
  ExprP rel_expr() {
    ExprP l = add_expr();
    for (;;) {
      CmpOp op;
      if (accept_sym(">=")) op = CmpOp::GE;
      else if (accept_sym("<=")) op = CmpOp::LE;
      else if (accept_sym(">")) op = CmpOp::GT;
      else if (accept_sym("<")) op = CmpOp::LT;
      else break;
      auto e = bin(ExprKind::CMP, std::move(l), add_expr());
      e->cmp = op;
      l = std::move(e);
    }
    return l;
  }
  ExprP add_expr() {
    ExprP l = mul_expr();
    for (;;) {
      MathOp op;
      if (accept_sym("+")) op = MathOp::ADD;
      else if (accept_sym("-")) op = MathOp::SUB;
      else break;
      auto e = bin(ExprKind::MATH, std::move(l), mul_expr());
      e->math = op;
      l = std::move(e);
    }
    return l;
  }
  ExprP mul_expr() {
    ExprP l = unary();
    for (;;) {
      MathOp op;
      if (accept_sym("*")) op = MathOp::MUL;
      else if (accept_sym("/")) op = MathOp::DIV;
      else if (accept_sym("%")) op = MathOp::MOD;
      else break;
      auto e = bin(ExprKind::MATH, std::move(l), unary());
      e->math = op;
      l = std::move(e);
    }
    return l;
  }
  ExprP unary() {
    if (accept_kw("not")) {
      auto e = mk(ExprKind::NOT);
      e->ch.push_back(unary());
      return e;
    }
    return postfix(primary());
  }
  ExprP postfix(ExprP e) {
    // null_check: attribute_reference IS NULL
    if (is_kw("is") && is_kw("null", 1)) {
      p += 2;
      auto n = mk(ExprKind::IS_NULL);
      n->ch.push_back(std::move(e));
      return n;
    }
    return e;
  }
  ExprP number_const(bool neg) {
    const Token& t = tk[p++];
    auto e = mk(ExprKind::CONST);
    std::string txt = (neg ? "-" : "") + t.s;
    switch (t.t) {
      case Tk::INT: {
        long long v = std::stoll(txt);
        if (v < INT32_MIN || v > INT32_MAX) throw ParseError("int literal out of range: " + txt);
        e->ctype = AttrType::INT; e->ival = v; e->dval = (double)v; break;
      }
      case Tk::LONG: e->ctype = AttrType::LONG; e->ival = std::stoll(txt); e->dval = (double)e->ival; break;
      case Tk::FLOAT: e->ctype = AttrType::FLOAT; e->dval = (double)std::strtof(txt.c_str(), nullptr); break;
      case Tk::DOUBLE: e->ctype = AttrType::DOUBLE; e->dval = std::strtod(txt.c_str(), nullptr); break;
      default: fail("expected number");
    }
    return e;
  }
  bool is_number(int k = 0) const {
    Tk t = peek(k).t;
    return t == Tk::INT || t == Tk::LONG || t == Tk::FLOAT || t == Tk::DOUBLE;
  }
  ExprP primary() {
    if (accept_sym("(")) {
      ExprP e = expr();
      expect_sym(")");
      return e;
    }
    if ((is_sym("-") || is_sym("+")) && is_number(1)) {  // signed_*_value
      bool neg = is_sym("-");
      ++p;
      return number_const(neg);
    }
    if (peek().t == Tk::INT && at_time_unit(1)) {  // time_value constant → long ms
      auto e = mk(ExprKind::CONST);
      e->ctype = AttrType::LONG;
      e->ival = time_value();
      e->dval = (double)e->ival;
      return e;
    }
    if (is_number()) return number_const(false);
    if (peek().t == Tk::STRING) {
      auto e = mk(ExprKind::CONST);
      e->ctype = AttrType::STRING;
      e->sval = tk[p++].s;
      return e;
    }
    if (is_kw("true") || is_kw("false")) {
      auto e = mk(ExprKind::CONST);
      e->ctype = AttrType::BOOL;
      e->ival = is_kw("true") ? 1 : 0;
      ++p;
      return e;
    }
    if (is_kw("null")) {
      ++p;
      auto e = mk(ExprKind::CONST);
      e->cnull = true;
      e->ctype = AttrType::STRING;
      return e;
    }
    if (peek().t == Tk::ID) {
      if (is_sym("(", 1)) return function_call();
      if (is_sym(":", 1) && peek(2).t == Tk::ID && is_sym("(", 3))
        throw UnsupportedError("function calls are outside the hot-path subset: '" + peek().s + "'");
      // attribute_reference: name1 ('[' attribute_index ']')? '.' attribute_name | attribute_name
      auto e = mk(ExprKind::VAR);
      std::string first = ident();
      if (is_sym("[") || is_sym(".")) {
        e->stream_ref = first;
        if (accept_sym("[")) {
          e->index = attribute_index();
          expect_sym("]");
        }
        if (is_sym("#")) throw UnsupportedError("inner-stream attribute references are not supported");
        expect_sym(".");
        e->attr = ident();
      } else {
        e->attr = first;
      }
      return e;
    }
    fail("expected expression");
  }
  // function_operation (SiddhiQL.g4 function_operation: function_id '(' attribute_list? ')'). Of the built-in
  // functions only the instanceOf* type tests are in the subset (core/executor/function/
  // InstanceOf{Boolean,Double,Float,Integer,Long,String}FunctionExecutor.java: exactly one argument, BOOL result).
  ExprP function_call() {
    static const std::pair<const char*, AttrType> kInstanceOf[] = {
        {"instanceOfBoolean", AttrType::BOOL}, {"instanceOfDouble", AttrType::DOUBLE},
        {"instanceOfFloat", AttrType::FLOAT},  {"instanceOfInteger", AttrType::INT},
        {"instanceOfLong", AttrType::LONG},    {"instanceOfString", AttrType::STRING}};
    const std::string name = tk[p].s;
    for (auto& f : kInstanceOf) {
      if (name != f.first) continue;
      p += 2;  // name '('
      std::vector<ExprP> args;
      if (!is_sym(")")) {
        do args.push_back(expr());
        while (accept_sym(","));
      }
      expect_sym(")");
      if (args.size() != 1)
        throw ValidationError("Invalid no of arguments passed to " + name + "() function, required only 1, but found " +
                              std::to_string(args.size()));
      auto e = mk(ExprKind::INSTANCE_OF);
      e->ctype = f.second;
      e->ch.push_back(std::move(args[0]));
      return e;
    }
    throw UnsupportedError("function calls are outside the hot-path subset: '" + name + "'");
  }
  int attribute_index() {
    // visitAttribute_index (SiddhiQLBaseVisitorImpl.java:2323-2334): LAST → -2, LAST - k → -2 - k
    if (accept_kw("last")) {
      int idx = kLast;
      if (accept_sym("-")) {
        if (peek().t != Tk::INT) fail("expected integer after 'last -'");
        idx -= std::stoi(tk[p++].s);
      }
      return idx;
    }
    if (peek().t != Tk::INT) fail("expected attribute index");
    return std::stoi(tk[p++].s);
  }

  // ---- sources ----
  // basic_source: source basic_source_stream_handlers?  (filters only: '#'? '[' expression ']')
  // source: inner='#'? stream_id (SiddhiQL.g4 `source`); an inner stream keeps its '#' in the id
  std::string source_id() {
    if (accept_sym("#")) return "#" + ident();
    return ident();
  }
  void basic_source(StateElem& s) {
    s.stream_id = source_id();
    for (;;) {
      if (is_sym("#") && is_sym("[", 1)) ++p;
      if (accept_sym("[")) {
        s.filters.push_back(expr());
        expect_sym("]");
        continue;
      }
      if (is_sym("#")) throw UnsupportedError("windows / stream functions are outside the hot-path subset");
      break;
    }
  }
  // standard_stateful_source: (event '=')? basic_source
  StateP standard_stateful_source() {
    auto s = std::make_unique<StateElem>();
    s->kind = StateKind::STREAM;
    if (peek().t == Tk::ID && is_sym("=", 1)) {
      s->event_ref = ident();
      expect_sym("=");
    }
    basic_source(*s);
    return s;
  }
  // basic_absent_pattern_source: NOT basic_source for_time   (for_time optional in the logical forms)
  StateP absent_source(bool require_for) {
    expect_kw("not");
    auto s = std::make_unique<StateElem>();
    s->kind = StateKind::ABSENT;
    basic_source(*s);
    if (accept_kw("for")) {
      s->has_wait = true;
      s->wait_ms = time_value();
    } else if (require_for) {
      fail("expected 'for <time>' after absent stream");
    }
    return s;
  }
  StateP mk_logical(LogicalType t, StateP e1, StateP e2) {
    auto l = std::make_unique<StateElem>();
    l->kind = StateKind::LOGICAL;
    l->ltype = t;
    l->a = std::move(e1);
    l->b = std::move(e2);
    return l;
  }
  StateP mk_count(StateP s, int mn, int mx) {
    auto c = std::make_unique<StateElem>();
    c->kind = StateKind::COUNT;
    c->a = std::move(s);
    c->min_count = mn;
    c->max_count = mx;
    return c;
  }
  // collect: '<' (INT | INT? ':' INT?) '>'   (visitCollect :2402)
  StateP collect(StateP s) {
    expect_sym("<");
    int mn = kAny, mx = kAny;
    if (peek().t == Tk::INT && is_sym(">", 1)) {
      mn = mx = std::stoi(tk[p++].s);
    } else {
      if (peek().t == Tk::INT) mn = std::stoi(tk[p++].s);
      expect_sym(":");
      if (peek().t == Tk::INT) mx = std::stoi(tk[p++].s);
    }
    expect_sym(">");
    return mk_count(std::move(s), mn, mx);
  }
  // pattern_source / sequence_source: logical | collection | standard | logical_absent
  StateP source(bool sequence) {
    if (is_kw("not")) {
      // NOT basic_source (AND standard | for_time (AND|OR ...)?)   (visitLogical_absent_stateful_source :1000)
      StateP ab = absent_source(false);
      if (accept_kw("and")) {
        if (is_kw("not")) {
          StateP ab2 = absent_source(true);
          if (!ab->has_wait) fail("expected 'for <time>'");
          return mk_logical(LogicalType::AND, std::move(ab), std::move(ab2));  // logicalNotAnd(abs0, abs1)
        }
        StateP present = standard_stateful_source();
        return mk_logical(LogicalType::AND, std::move(ab), std::move(present));
      }
      if (accept_kw("or")) {
        if (!ab->has_wait) fail("expected 'for <time>'");
        if (is_kw("not")) {
          StateP ab2 = absent_source(true);
          return mk_logical(LogicalType::OR, std::move(ab), std::move(ab2));
        }
        StateP present = standard_stateful_source();
        return mk_logical(LogicalType::OR, std::move(ab), std::move(present));
      }
      if (!ab->has_wait) fail("expected 'for <time>' after absent stream");
      return ab;
    }
    StateP s = standard_stateful_source();
    if (is_kw("and") || is_kw("or")) {
      LogicalType t = is_kw("and") ? LogicalType::AND : LogicalType::OR;
      ++p;
      if (is_kw("not")) {
        StateP ab = absent_source(t == LogicalType::OR);
        // logicalNotAnd(absent, present) / logicalOr(absent, present): absent becomes element1
        return mk_logical(t, std::move(ab), std::move(s));
      }
      StateP s2 = standard_stateful_source();
      return mk_logical(t, std::move(s), std::move(s2));
    }
    if (is_sym("<")) return collect(std::move(s));
    if (sequence) {
      if (accept_sym("*")) return mk_count(std::move(s), 0, kAny);
      if (accept_sym("+")) return mk_count(std::move(s), 1, kAny);
      if (accept_sym("?")) return mk_count(std::move(s), 0, 1);
    }
    return s;
  }
  void maybe_within(StateElem& e) {
    if (accept_kw("within")) {
      e.has_within = true;
      e.within_ms = time_value();
    }
  }
  StateP mk_next(StateP a, StateP b) {
    auto n = std::make_unique<StateElem>();
    n->kind = StateKind::NEXT;
    n->a = std::move(a);
    n->b = std::move(b);
    return n;
  }
  StateP mk_every(StateP a) {
    auto n = std::make_unique<StateElem>();
    n->kind = StateKind::EVERY;
    n->a = std::move(a);
    return n;
  }

  // every_pattern_source_chain / pattern_source_chain (SiddhiQL.g4:205-218)
  StateP pattern_unit() {
    if (accept_kw("every")) {
      StateP inner;
      if (is_sym("(")) {
        ++p;
        inner = pattern_chain();
        expect_sym(")");
      } else {
        inner = source(false);
      }
      StateP ev = mk_every(std::move(inner));
      maybe_within(*ev);  // EveryStateElement.within (ignored by StateInputStreamParser.parse :263-282)
      return ev;
    }
    if (is_sym("(")) {
      ++p;
      StateP inner = pattern_chain();
      expect_sym(")");
      maybe_within(*inner);
      return inner;
    }
    StateP s = source(false);
    maybe_within(*s);
    return s;
  }
  // an element that is only `[every] not S for t` (chains of them included)
  static bool all_absent(const StateElem* e) {
    switch (e->kind) {
      case StateKind::ABSENT: return true;
      case StateKind::EVERY: return all_absent(e->a.get());
      case StateKind::NEXT: return all_absent(e->a.get()) && all_absent(e->b.get());
      default: return false;
    }
  }
  StateP pattern_chain() {
    StateP l = pattern_unit();
    int n = 1;
    while (accept_sym("->")) {
      l = mk_next(std::move(l), pattern_unit());
      ++n;
    }
    // left/right_absent_pattern_source (SiddhiQL.g4:224-238): a chain of absent elements needs a present one
    // (compiler AbsentPatternTestCase.java:56-61, `not A for t -> not B for t` is a SiddhiParserException)
    if (n > 1 && all_absent(l.get())) fail("an absent pattern chain needs at least one present (non-absent) element");
    return l;
  }
  // sequence_source_chain (SiddhiQL.g4:320-324)
  StateP sequence_unit() {
    if (is_sym("(")) {
      ++p;
      StateP inner = sequence_chain();
      expect_sym(")");
      maybe_within(*inner);
      return inner;
    }
    StateP s = source(true);
    maybe_within(*s);
    return s;
  }
  StateP sequence_chain() {
    StateP l = sequence_unit();
    while (accept_sym(",")) l = mk_next(std::move(l), sequence_unit());
    return l;
  }
  // every_sequence_source_chain: EVERY? sequence_source within_time? ',' sequence_source_chain
  StateP sequence_top() {
    bool every = accept_kw("every");
    StateP first;
    if (is_sym("(")) {  // EVERY? '(' chain ')' or a parenthesised logical-absent source
      ++p;
      first = sequence_chain();
      expect_sym(")");
    } else {
      first = source(true);
    }
    if (every) first = mk_every(std::move(first));
    maybe_within(*first);
    expect_sym(",");
    StateP rest = sequence_chain();
    return mk_next(std::move(first), std::move(rest));
  }

  // Decide pattern vs sequence vs single by scanning the query input to the first top-level
  // 'select'/'insert' keyword: '->' → pattern, top-level ',' → sequence.
  InputKind classify_input() {
    int depth = 0;
    bool has_arrow = false, has_comma = false, has_every = false;
    for (size_t k = p; k < tk.size(); ++k) {
      const Token& t = tk[k];
      if (t.t == Tk::END) break;
      if (t.t == Tk::SYM) {
        if (t.s == "(" || t.s == "[") ++depth;
        else if (t.s == ")" || t.s == "]") --depth;
        else if (t.s == "->") has_arrow = true;
        else if (t.s == "," && depth == 0) has_comma = true;
        else if (t.s == ";") break;
      } else if (t.t == Tk::ID && depth == 0) {
        std::string l = lower(t.s);
        if (l == "select" || l == "insert" || l == "output" || l == "return") break;
        if (l == "every" || l == "not" || l == "and" || l == "or") has_every = true;
      }
    }
    if (has_arrow) return InputKind::PATTERN;
    if (has_comma) return InputKind::SEQUENCE;
    if (has_every) return InputKind::PATTERN;
    return InputKind::SINGLE;
  }

  Query query(std::vector<Annotation>& anns) {
    Query q;
    for (auto& a : anns) {
      if (a.name == "info")
        for (auto& kv : a.elems)
          if (kv.first == "name") q.name = kv.second;
    }
    if (q.name.empty()) q.name = "query_" + std::to_string(++anon_query);
    expect_kw("from");
    // anonymous_stream (SiddhiQL.g4: `from from ... return` / `from (from ... return)`): a nested query
    if (is_kw("from") || (is_sym("(") && is_kw("from", 1)))
      throw UnsupportedError("anonymous (nested) query streams are outside the hot-path subset");
    q.input = classify_input();
    if (q.input == InputKind::SINGLE) {
      StateElem tmp;
      basic_source(tmp);
      q.stream_id = tmp.stream_id;
      q.filters = std::move(tmp.filters);
      if (is_kw("join") || is_kw("left") || is_kw("right") || is_kw("full") || is_kw("unidirectional") ||
          is_kw("as"))
        throw UnsupportedError("joins are outside the hot-path subset");
    } else if (q.input == InputKind::PATTERN) {
      q.state = pattern_chain();
    } else {
      q.state = sequence_top();
      // left/right_absent_sequence_source (SiddhiQL.g4:312-326): absent elements need a present one
      if (all_absent(q.state.get())) fail("an absent sequence needs at least one present (non-absent) element");
    }
    // query_section: select ... [having ...] (group by / order by / limit are out of scope)
    if (accept_kw("select")) {
      if (accept_sym("*")) {
        q.select_all = true;
      } else {
        do {
          OutputAttr oa;
          oa.expr = expr();
          if (accept_kw("as")) oa.rename = ident();
          else if (oa.expr->kind == ExprKind::VAR) oa.rename = oa.expr->attr;
          else fail("output attribute needs 'as <name>'");
          q.select.push_back(std::move(oa));
        } while (accept_sym(","));
      }
      if (is_kw("group")) throw UnsupportedError("group by is outside the hot-path subset");
      // having: a condition over the output attributes and the input events (QuerySelector.java:138-139)
      if (accept_kw("having")) q.having = expr();
      if (is_kw("order") || is_kw("limit"))
        throw UnsupportedError("order by / limit are outside the hot-path subset");
    } else {
      q.select_all = true;
    }
    if (is_kw("output")) throw UnsupportedError("output rate limiting is outside the hot-path subset");
    if (accept_kw("insert")) {
      if (accept_kw("current")) { expect_kw("events"); }
      else if (is_kw("expired") || is_kw("all")) throw UnsupportedError("only current events are supported");
      expect_kw("into");
      q.insert_into = source_id();
    } else if (is_kw("delete") || is_kw("update") || is_kw("return")) {
      throw UnsupportedError("table operations / return are outside the hot-path subset");
    } else {
      fail("expected 'insert into'");
    }
    return q;
  }

  StreamDef define_stream() {
    StreamDef d;
    d.id = ident();
    expect_sym("(");
    do {
      Attribute a;
      a.name = ident();
      std::string t = lower(ident());
      if (t == "int") a.type = AttrType::INT;
      else if (t == "long") a.type = AttrType::LONG;
      else if (t == "float") a.type = AttrType::FLOAT;
      else if (t == "double") a.type = AttrType::DOUBLE;
      else if (t == "string") a.type = AttrType::STRING;
      else if (t == "bool") a.type = AttrType::BOOL;
      else throw UnsupportedError("attribute type '" + t + "' is not supported");
      d.attrs.push_back(a);
    } while (accept_sym(","));
    expect_sym(")");
    return d;
  }

  void parse() {
    while (peek().t != Tk::END) {
      if (accept_sym(";")) continue;
      std::vector<Annotation> anns;
      while (is_sym("@")) anns.push_back(annotation());
      std::vector<Annotation> rest;
      for (auto& a : anns) {
        if (a.name == "app:name") {
          for (auto& kv : a.elems) app.name = kv.second;
        } else if (a.name == "app:playback") {
          for (auto& kv : a.elems)
            if (kv.first == "idle.time" || kv.first == "increment")
              throw UnsupportedError("@app:playback heartbeat parameters are not supported");
          app.playback = true;
        } else if (a.name == "app:statistics" || a.name == "app:description") {
          // observability / docs only
        } else {
          rest.push_back(a);
        }
      }
      if (peek().t == Tk::END) break;
      if (accept_kw("define")) {
        if (!accept_kw("stream")) throw UnsupportedError("only 'define stream' is supported (tables/windows/triggers/functions/aggregations are out of scope)");
        for (auto& a : rest)
          if (a.name == "async") throw UnsupportedError("@async streams are not supported");
        StreamDef d = define_stream();
        if (app.find_stream(d.id)) throw ValidationError("stream '" + d.id + "' is already defined");
        app.streams.push_back(std::move(d));
      } else if (accept_kw("partition")) {
        expect_kw("with");
        Partition part;
        expect_sym("(");
        do {
          PartitionWith pw;
          pw.key = expr();
          if (is_kw("as")) throw UnsupportedError("range partitions are not supported");
          expect_kw("of");
          pw.stream_id = ident();
          part.with.push_back(std::move(pw));
        } while (accept_sym(","));
        expect_sym(")");
        expect_kw("begin");
        while (!is_kw("end")) {
          if (accept_sym(";")) continue;
          std::vector<Annotation> qa;
          while (is_sym("@")) qa.push_back(annotation());
          part.queries.push_back(query(qa));
        }
        expect_kw("end");
        int pi = (int)app.partitions.size();
        for (size_t k = 0; k < part.queries.size(); ++k) app.order.push_back({pi, (int)k});
        app.partitions.push_back(std::move(part));
      } else if (is_kw("from")) {
        app.order.push_back({-1, (int)app.queries.size()});
        app.queries.push_back(query(rest));
      } else {
        fail("expected 'define', 'partition' or 'from'");
      }
    }
  }
};

}  // namespace

void collect_stream_ids(const StateElem* e, std::vector<std::string>& out) {
  switch (e->kind) {
    case StateKind::LOGICAL: collect_stream_ids(e->a.get(), out); collect_stream_ids(e->b.get(), out); break;
    case StateKind::COUNT: collect_stream_ids(e->a.get(), out); break;
    case StateKind::EVERY: collect_stream_ids(e->a.get(), out); break;
    case StateKind::NEXT: collect_stream_ids(e->a.get(), out); collect_stream_ids(e->b.get(), out); break;
    case StateKind::STREAM:
    case StateKind::ABSENT: out.push_back(e->stream_id); break;
  }
}

namespace {

void collect_refs(const StateElem* e, std::vector<std::pair<std::string, std::string>>& out) {
  switch (e->kind) {
    case StateKind::LOGICAL:
    case StateKind::NEXT: collect_refs(e->a.get(), out); collect_refs(e->b.get(), out); break;
    case StateKind::COUNT:
    case StateKind::EVERY: collect_refs(e->a.get(), out); break;
    case StateKind::STREAM:
    case StateKind::ABSENT: out.push_back({e->event_ref, e->stream_id}); break;
  }
}

// Type of a select expression (Java binary numeric promotion for arithmetic, as the executors'
// MathExpressionExecutor* classes return: double > float > long > int; compare / logic → BOOL).
AttrType infer_type(const Expr& x, const std::function<AttrType(const Expr&)>& var_type) {
  switch (x.kind) {
    case ExprKind::CONST: return x.ctype;
    case ExprKind::VAR: return var_type(x);
    case ExprKind::MATH: {
      const AttrType a = infer_type(*x.ch[0], var_type), b = infer_type(*x.ch[1], var_type);
      auto num = [](AttrType t) { return t == AttrType::INT || t == AttrType::LONG || t == AttrType::FLOAT || t == AttrType::DOUBLE; };
      if (!num(a) || !num(b)) throw ValidationError("arithmetic operands must be numeric");
      if (a == AttrType::DOUBLE || b == AttrType::DOUBLE) return AttrType::DOUBLE;
      if (a == AttrType::FLOAT || b == AttrType::FLOAT) return AttrType::FLOAT;
      if (a == AttrType::LONG || b == AttrType::LONG) return AttrType::LONG;
      return AttrType::INT;
    }
    default: return AttrType::BOOL;
  }
}

}  // namespace

// Validation common to both lowerings, in app order (SiddhiAppParser adds queries one by one): every stream a
// query reads is defined by `define stream` or by the `insert into` of an earlier query; an `insert into` of an
// undefined stream defines it from the query's output attributes (names and types: QueryParser →
// OutputParser / SiddhiApp.defineStream). Inner streams ('#name') exist only inside their partition
// (PartitionRuntime.addQuery :118-142, localStreamDefinitionMap).
App parse_app(const std::string& text) {
  Parser ps;
  ps.tk = lex(text);
  ps.parse();
  App& app = ps.app;
  auto find_in = [&](const std::string& id, int part) -> const StreamDef* {
    for (auto& s : app.streams)
      if (s.id == id && (id[0] != '#' || s.partition == part)) return &s;
    return nullptr;
  };
  auto check_stream = [&](const std::string& id, int part) -> const StreamDef* {
    if (id[0] == '#' && part < 0) throw ValidationError("inner stream '" + id + "' used outside a partition");
    const StreamDef* d = find_in(id, part);
    if (!d) throw ValidationError("stream '" + id + "' is not defined");
    return d;
  };
  for (auto& pt : app.partitions)
    for (auto& w : pt.with) {
      if (w.stream_id[0] == '#') throw ValidationError("partition key on inner stream '" + w.stream_id + "'");
      check_stream(w.stream_id, -1);
    }
  for (auto [pi, qi] : app.order) {
    Query& q = pi < 0 ? app.queries[qi] : app.partitions[pi].queries[qi];
    // input streams (copies: app.streams may grow below)
    std::vector<std::pair<std::string, StreamDef>> ins;  // (event reference, stream)
    if (q.input == InputKind::SINGLE) {
      ins.push_back({"", *check_stream(q.stream_id, pi)});
    } else {
      std::vector<std::pair<std::string, std::string>> refs;
      collect_refs(q.state.get(), refs);
      for (auto& r : refs) ins.push_back({r.first, *check_stream(r.second, pi)});
    }
    auto var_type = [&](const Expr& v) -> AttrType {
      for (auto& in : ins)
        if (v.stream_ref.empty() || v.stream_ref == in.first || v.stream_ref == in.second.id) {
          const int a = in.second.index_of(v.attr);
          if (a >= 0) return in.second.attrs[a].type;
        }
      throw ValidationError("attribute '" + v.attr + "' is not defined");
    };
    // the output schema (a select the lowerings reject, e.g. an unknown attribute or a duplicate name under
    // `select *`, is reported by them with the query's context; the AST itself stays valid)
    std::vector<Attribute> out;
    try {
      if (q.select_all) {
        for (auto& in : ins)
          for (auto& at : in.second.attrs) {
            bool dup = false;
            for (auto& o : out) dup |= o.name == at.name;
            if (!dup) out.push_back(at);
          }
      } else {
        for (auto& oa : q.select) out.push_back({oa.rename, infer_type(*oa.expr, var_type)});
      }
    } catch (const ValidationError&) {
      out.clear();
    }
    const std::string& id = q.insert_into;
    if (id[0] == '#' && pi < 0) throw ValidationError("inner stream '" + id + "' used outside a partition");
    if (const StreamDef* d = find_in(id, pi)) {
      if (!d->implicit && !out.empty() && d->attrs.size() != out.size())
        throw ValidationError("query '" + q.name + "' inserts " + std::to_string(out.size()) +
                              " attributes into stream '" + id + "' of " + std::to_string(d->attrs.size()));
    } else {
      if (id[0] == '#')
        for (auto& s : app.streams)
          if (s.id == id) throw UnsupportedError("inner stream '" + id + "' defined in two partitions");
      StreamDef nd;
      nd.id = id;
      nd.attrs = out;
      nd.implicit = true;
      nd.partition = id[0] == '#' ? pi : -1;
      app.streams.push_back(std::move(nd));
    }
  }
  return std::move(ps.app);
}

}  // namespace sql
