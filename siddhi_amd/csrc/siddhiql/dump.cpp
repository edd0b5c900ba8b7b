// Canonical JSON of a parsed SiddhiQL app: the tree SiddhiCompiler.parse returns
// (modules/siddhi-query-compiler/.../SiddhiCompiler.java:56 parse, :97 parseQuery), restricted to the subset
// this engine compiles. Used by sm_compile_dump (include/siddhi_amd.h) so the parser can be checked against the
// reference's own expected query trees (tests/golden/ast_kats.json, transcribed from siddhi-query-api
// PatternQueryTestCase / SequenceQueryTestCase and siddhi-query-compiler AbsentPatternTestCase).
//
// Shapes (one JSON object per node):
//   state   {"stream": id, "ref": e1?, "filters": [expr]}        StreamStateElement
//           {"not": {stream}, "for": ms?}                        AbsentStreamStateElement (waitingTime)
//           {"next": [a, b]}  {"every": a}  {"and"|"or": [a, b]}  Next / Every / Logical
//           {"count": a, "min": m, "max": M}                     CountStateElement (ANY = -1)
//           any state may carry "within": ms
//   expr    {"const": v, "type": T} | {"var": attr, "ref": s?, "index": i?} | {"cmp": op, "l": x, "r": y}
//           {"math": op, "l": x, "r": y} | {"and": [x, y]} | {"or": [x, y]} | {"not": x} | {"isnull": x}
#include <cstdio>
#include <sstream>

#include "ast.h"

namespace sql {

namespace {

void jstr(std::ostringstream& o, const std::string& s) {
  o << '"';
  for (char c : s) {
    if (c == '"' || c == '\\') o << '\\' << c;
    else if ((unsigned char)c < 0x20) {
      char b[8];
      snprintf(b, sizeof b, "\\u%04x", c);
      o << b;
    } else o << c;
  }
  o << '"';
}

const char* cmp_name(CmpOp c) {
  switch (c) {
    case CmpOp::EQ: return "==";
    case CmpOp::NE: return "!=";
    case CmpOp::LT: return "<";
    case CmpOp::LE: return "<=";
    case CmpOp::GT: return ">";
    default: return ">=";
  }
}

const char* math_name(MathOp m) {
  switch (m) {
    case MathOp::ADD: return "+";
    case MathOp::SUB: return "-";
    case MathOp::MUL: return "*";
    case MathOp::DIV: return "/";
    default: return "%";
  }
}

void expr(std::ostringstream& o, const Expr* e) {
  switch (e->kind) {
    case ExprKind::CONST:
      o << "{\"const\":";
      if (e->cnull) o << "null";
      else if (e->ctype == AttrType::STRING) jstr(o, e->sval);
      else if (e->ctype == AttrType::BOOL) o << (e->ival ? "true" : "false");
      else if (e->ctype == AttrType::FLOAT || e->ctype == AttrType::DOUBLE) {
        char b[64];
        snprintf(b, sizeof b, "%.17g", e->dval);
        o << b;
      } else o << e->ival;
      o << ",\"type\":\"" << attr_type_name(e->ctype) << "\"}";
      return;
    case ExprKind::VAR:
      o << "{\"var\":";
      jstr(o, e->attr);
      if (!e->stream_ref.empty()) {
        o << ",\"ref\":";
        jstr(o, e->stream_ref);
      }
      if (e->index != kNoIndex) o << ",\"index\":" << e->index;
      o << "}";
      return;
    case ExprKind::CMP:
      o << "{\"cmp\":\"" << cmp_name(e->cmp) << "\",\"l\":";
      expr(o, e->ch[0].get());
      o << ",\"r\":";
      expr(o, e->ch[1].get());
      o << "}";
      return;
    case ExprKind::MATH:
      o << "{\"math\":\"" << math_name(e->math) << "\",\"l\":";
      expr(o, e->ch[0].get());
      o << ",\"r\":";
      expr(o, e->ch[1].get());
      o << "}";
      return;
    case ExprKind::AND:
    case ExprKind::OR:
      o << (e->kind == ExprKind::AND ? "{\"and\":[" : "{\"or\":[");
      expr(o, e->ch[0].get());
      o << ",";
      expr(o, e->ch[1].get());
      o << "]}";
      return;
    case ExprKind::NOT:
      o << "{\"not\":";
      expr(o, e->ch[0].get());
      o << "}";
      return;
    case ExprKind::INSTANCE_OF:
      o << "{\"instanceof\":\"" << attr_type_name(e->ctype) << "\",\"arg\":";
      expr(o, e->ch[0].get());
      o << "}";
      return;
    default:
      o << "{\"isnull\":";
      expr(o, e->ch[0].get());
      o << "}";
      return;
  }
}

void stream_body(std::ostringstream& o, const StateElem* s) {
  o << "\"stream\":";
  jstr(o, s->stream_id);
  if (!s->event_ref.empty()) {
    o << ",\"ref\":";
    jstr(o, s->event_ref);
  }
  o << ",\"filters\":[";
  for (size_t k = 0; k < s->filters.size(); ++k) {
    if (k) o << ",";
    expr(o, s->filters[k].get());
  }
  o << "]";
}

void state(std::ostringstream& o, const StateElem* s) {
  o << "{";
  switch (s->kind) {
    case StateKind::STREAM: stream_body(o, s); break;
    case StateKind::ABSENT:
      o << "\"not\":{";
      stream_body(o, s);
      o << "}";
      if (s->has_wait) o << ",\"for\":" << s->wait_ms;
      break;
    case StateKind::NEXT:
      o << "\"next\":[";
      state(o, s->a.get());
      o << ",";
      state(o, s->b.get());
      o << "]";
      break;
    case StateKind::EVERY:
      o << "\"every\":";
      state(o, s->a.get());
      break;
    case StateKind::LOGICAL:
      o << (s->ltype == LogicalType::AND ? "\"and\":[" : "\"or\":[");
      state(o, s->a.get());
      o << ",";
      state(o, s->b.get());
      o << "]";
      break;
    case StateKind::COUNT:
      o << "\"count\":";
      state(o, s->a.get());
      o << ",\"min\":" << s->min_count << ",\"max\":" << s->max_count;
      break;
  }
  if (s->has_within) o << ",\"within\":" << s->within_ms;
  o << "}";
}

void query(std::ostringstream& o, const Query& q) {
  o << "{\"name\":";
  jstr(o, q.name);
  o << ",\"input\":\"" << (q.input == InputKind::SINGLE ? "single" : q.input == InputKind::PATTERN ? "pattern" : "sequence")
    << "\"";
  if (q.input == InputKind::SINGLE) {
    o << ",\"stream\":";
    jstr(o, q.stream_id);
    o << ",\"filters\":[";
    for (size_t k = 0; k < q.filters.size(); ++k) {
      if (k) o << ",";
      expr(o, q.filters[k].get());
    }
    o << "]";
  } else {
    o << ",\"state\":";
    state(o, q.state.get());
  }
  o << ",\"select\":";
  if (q.select_all) {
    o << "\"*\"";
  } else {
    o << "[";
    for (size_t k = 0; k < q.select.size(); ++k) {
      if (k) o << ",";
      o << "{\"as\":";
      jstr(o, q.select[k].rename);
      o << ",\"expr\":";
      expr(o, q.select[k].expr.get());
      o << "}";
    }
    o << "]";
  }
  if (q.having) {
    o << ",\"having\":";
    expr(o, q.having.get());
  }
  o << ",\"insert_into\":";
  jstr(o, q.insert_into);
  o << "}";
}

}  // namespace

std::string dump_app_json(const App& a) {
  std::ostringstream o;
  o << "{\"playback\":" << (a.playback ? "true" : "false") << ",\"streams\":[";
  for (size_t i = 0; i < a.streams.size(); ++i) {
    if (i) o << ",";
    o << "{\"id\":";
    jstr(o, a.streams[i].id);
    o << ",\"attrs\":[";
    for (size_t k = 0; k < a.streams[i].attrs.size(); ++k) {
      if (k) o << ",";
      o << "[";
      jstr(o, a.streams[i].attrs[k].name);
      o << ",\"" << attr_type_name(a.streams[i].attrs[k].type) << "\"]";
    }
    o << "]}";
  }
  o << "],\"queries\":[";
  for (size_t i = 0; i < a.queries.size(); ++i) {
    if (i) o << ",";
    query(o, a.queries[i]);
  }
  o << "],\"partitions\":[";
  for (size_t p = 0; p < a.partitions.size(); ++p) {
    if (p) o << ",";
    o << "{\"with\":[";
    for (size_t k = 0; k < a.partitions[p].with.size(); ++k) {
      if (k) o << ",";
      o << "{\"stream\":";
      jstr(o, a.partitions[p].with[k].stream_id);
      o << ",\"key\":";
      expr(o, a.partitions[p].with[k].key.get());
      o << "}";
    }
    o << "],\"queries\":[";
    for (size_t i = 0; i < a.partitions[p].queries.size(); ++i) {
      if (i) o << ",";
      query(o, a.partitions[p].queries[i]);
    }
    o << "]}";
  }
  o << "]}";
  return o.str();
}

}  // namespace sql
