// AST → device plan. See compiler.h for the reference files each part restates.
#include "compiler.h"

#include <algorithm>
#include <cstring>
#include <functional>
#include <set>

namespace sm {

using namespace sql;

int stream_index(const App& app, const std::string& id) {
  for (size_t i = 0; i < app.streams.size(); ++i)
    if (app.streams[i].id == id) return (int)i;
  return -1;
}

namespace {

bool numeric(int t) { return t == T_INT || t == T_LONG || t == T_FLOAT || t == T_DOUBLE; }

struct MetaStream {
  const StreamDef* def;
  std::string ref;
  int stream;
};

// ExpressionParser restated as a bytecode emitter.
struct Emitter {
  Dict& dict;
  std::vector<Instr>& code;
  std::vector<DVal>& consts;
  const std::vector<MetaStream>* metas = nullptr;  // state context
  const StreamDef* stream = nullptr;               // stream context
  int current_state = -1;
  int default_index = kCurrent;
  // collects VAR positions (for parity refs)
  std::vector<std::pair<int, int>>* var_refs = nullptr;

  // operand-stack slots the device evaluator (kernels/expr.h eval_prog) needs for x: a binary node keeps its
  // left value while the right operand is evaluated
  static int stack_need(const Expr& x) {
    if (x.ch.empty()) return 1;
    if (x.ch.size() == 1) return stack_need(*x.ch[0]);
    return std::max(stack_need(*x.ch[0]), 1 + stack_need(*x.ch[1]));
  }

  int level = 0;
  int emit(const Expr& x) {  // returns result type
    if (level == 0 && stack_need(x) > kMaxStack)
      throw UnsupportedError("expression nests deeper than the device evaluator's " + std::to_string(kMaxStack) +
                             "-entry operand stack");
    ++level;
    struct Leave {
      int& l;
      ~Leave() { --l; }
    } leave{level};
    return emit_node(x);
  }

  int emit_node(const Expr& x) {
    Instr in{};
    switch (x.kind) {
      case ExprKind::CONST: {
        DVal v{};
        v.null = x.cnull;
        int t = (int)x.ctype;
        if (t == T_FLOAT || t == T_DOUBLE) v.d = x.dval;
        else if (t == T_STRING) v.i = x.cnull ? -1 : dict.intern(x.sval);
        else v.i = x.ival;
        in.op = OP_CONST;
        in.a = (int)consts.size();
        in.t0 = t;
        consts.push_back(v);
        code.push_back(in);
        return t;
      }
      case ExprKind::VAR: return emit_var(x);
      case ExprKind::AND:
      case ExprKind::OR: {
        int a = emit(*x.ch[0]);
        int b = emit(*x.ch[1]);
        if (a != T_BOOL || b != T_BOOL) throw ValidationError("and/or operands should be of type BOOL");
        in.op = x.kind == ExprKind::AND ? OP_AND : OP_OR;
        in.t0 = T_BOOL;
        code.push_back(in);
        return T_BOOL;
      }
      case ExprKind::NOT: {
        if (emit(*x.ch[0]) != T_BOOL) throw ValidationError("not operand should be of type BOOL");
        in.op = OP_NOT;
        code.push_back(in);
        return T_BOOL;
      }
      case ExprKind::IS_NULL: {
        emit(*x.ch[0]);
        in.op = OP_ISNULL;
        code.push_back(in);
        return T_BOOL;
      }
      case ExprKind::INSTANCE_OF: {
        // InstanceOf*FunctionExecutor.execute(Object data): `data instanceof T`. An executor's value has its
        // static type (or is null), so the test is "not null" when the types agree and false otherwise.
        const size_t mark = code.size();
        if (emit(*x.ch[0]) == (int)x.ctype) {
          in.op = OP_ISNULL;
          code.push_back(in);
          Instr n{};
          n.op = OP_NOT;
          code.push_back(n);
        } else {
          code.resize(mark);  // the argument's value is never read (its references still count as refs)
          DVal v{};
          v.i = 0;
          in.op = OP_CONST;
          in.a = (int)consts.size();
          in.t0 = T_BOOL;
          consts.push_back(v);
          code.push_back(in);
        }
        return T_BOOL;
      }
      case ExprKind::CMP: {
        int a = emit(*x.ch[0]);
        int b = emit(*x.ch[1]);
        int ct;
        bool eq = x.cmp == CmpOp::EQ || x.cmp == CmpOp::NE;
        if (numeric(a) && numeric(b)) {
          if (a == T_DOUBLE || b == T_DOUBLE) ct = CT_DOUBLE;
          else if (a == T_FLOAT || b == T_FLOAT) ct = (eq && (a == T_LONG || b == T_LONG)) ? CT_DOUBLE : CT_FLOAT;
          else if (a == T_LONG || b == T_LONG) ct = CT_LONG;
          else ct = CT_INT;
        } else if ((a == T_STRING && b == T_STRING) || (a == T_BOOL && b == T_BOOL)) {
          if (!eq) throw ValidationError("compare operation not supported between non-numeric types");
          ct = CT_ID;
        } else {
          throw ValidationError(std::string("compare operation not supported between ") +
                                attr_type_name((AttrType)a) + " and " + attr_type_name((AttrType)b));
        }
        in.op = OP_CMP;
        in.sub = (int)x.cmp;  // CmpOp order == CMP_* order
        in.t0 = ct;
        in.t1 = a;
        in.t2 = b;
        code.push_back(in);
        return T_BOOL;
      }
      case ExprKind::MATH: {
        int a = emit(*x.ch[0]);
        int b = emit(*x.ch[1]);
        if (!numeric(a) || !numeric(b)) throw ValidationError("arithmetic operands must be numeric");
        int rt;
        if (a == T_DOUBLE || b == T_DOUBLE) rt = T_DOUBLE;
        else if (a == T_FLOAT || b == T_FLOAT) rt = T_FLOAT;
        else if (a == T_LONG || b == T_LONG) rt = T_LONG;
        else rt = T_INT;
        in.op = OP_MATH;
        in.sub = (int)x.math;
        in.t0 = rt;
        in.t1 = a;
        in.t2 = b;
        code.push_back(in);
        return rt;
      }
    }
    throw UnsupportedError("expression");
  }

  int emit_var(const Expr& x) {
    Instr in{};
    if (!metas) {  // MetaStreamEvent: the stream's own attribute (ExpressionParser.parseVariable :1232-1262)
      int a = stream->index_of(x.attr);
      if (a < 0) throw ValidationError("attribute '" + x.attr + "' is not defined in stream '" + stream->id + "'");
      in.op = OP_COL;
      in.a = a;
      in.t0 = (int)stream->attrs[a].type;
      code.push_back(in);
      if (var_refs) var_refs->push_back({-1, a});
      return in.t0;
    }
    // MetaStateEvent branch (:1263-1371)
    int pos = (x.index != kNoIndex) ? ((x.index <= kLast) ? x.index + 1 : x.index) : default_index;
    int chain = -1;
    const auto& ms = *metas;
    if (x.stream_ref.empty()) {
      if (current_state < 0) {
        for (size_t i = 0; i < ms.size(); ++i)
          if (ms[i].def->index_of(x.attr) >= 0) {
            if (chain >= 0) throw ValidationError("attribute '" + x.attr + "' is ambiguous across input streams");
            chain = (int)i;
          }
        if (chain < 0) throw ValidationError("attribute '" + x.attr + "' not found in any input stream");
      } else {
        chain = current_state;
        if (ms[chain].def->index_of(x.attr) < 0)
          throw ValidationError("attribute '" + x.attr + "' is not defined in stream '" + ms[chain].def->id + "'");
      }
    } else {
      for (size_t i = 0; i < ms.size(); ++i) {
        if (ms[i].ref.empty()) {
          if (ms[i].def->id == x.stream_ref) { chain = (int)i; break; }
        } else if (ms[i].ref == x.stream_ref) {
          chain = (int)i;
          if (current_state > -1 && !ms[current_state].ref.empty() && x.index != kNoIndex && x.index <= kLast &&
              x.stream_ref == ms[current_state].ref)
            pos = x.index;
          break;
        }
      }
      if (chain < 0) throw ValidationError("Stream with reference : " + x.stream_ref + " not found");
      if (ms[chain].def->index_of(x.attr) < 0)
        throw ValidationError("attribute '" + x.attr + "' is not defined in stream '" + ms[chain].def->id + "'");
    }
    int a = ms[chain].def->index_of(x.attr);
    in.op = OP_VAR;
    in.a = chain;
    in.b = pos;
    in.c = a;
    in.t0 = (int)ms[chain].def->attrs[a].type;
    code.push_back(in);
    if (var_refs) var_refs->push_back({chain, pos});
    return in.t0;
  }
};

// having (SelectorParser.generateHavingExecutor :214-228 → ExpressionParser.parseVariable with HAVING_STATE
// :1242-1275): a bare attribute name resolves to the query's output attribute first, and only when the output
// has no such attribute to the input events (state input) or nowhere (single-stream input: the output stream
// definition only). The output attribute's value is its select expression's value on the same event (the
// select is a pure function of the event), so the device program evaluates that expression in its place.
using OutAttrs = std::vector<std::pair<std::string, const Expr*>>;
ExprP having_subst(const Expr& x, const OutAttrs& outs, bool outputs_only) {
  if (x.kind == ExprKind::VAR && x.stream_ref.empty()) {
    for (auto& o : outs)
      if (o.first == x.attr) return having_subst(*o.second, {}, false);
    if (outputs_only) throw ValidationError("attribute '" + x.attr + "' is not an output attribute of the query");
  }
  auto e = std::make_unique<Expr>();
  e->kind = x.kind;
  e->ctype = x.ctype;
  e->cnull = x.cnull;
  e->ival = x.ival;
  e->dval = x.dval;
  e->sval = x.sval;
  e->stream_ref = x.stream_ref;
  e->index = x.index;
  e->attr = x.attr;
  e->cmp = x.cmp;
  e->math = x.math;
  for (auto& c : x.ch) e->ch.push_back(having_subst(*c, outs, outputs_only));
  return e;
}

struct Lowering {
  const App& app;
  Dict& dict;
  bool sequence;
  std::vector<MetaStream> metas;
  std::vector<DPre> pres;
  std::vector<DPost> posts;
  std::vector<DInner> inners;
  std::vector<DWithin> withins;
  std::vector<Instr> code;
  std::vector<DVal> consts;
  std::vector<std::pair<int64_t, std::vector<int>>> stack;  // within stack, index 0 = most recent
  std::vector<std::string> inner_stream;                     // per inner: first receiver stream id
  int nsched = 0;

  int new_pre(int kind) {
    DPre p{};
    p.kind = kind;
    p.sequence = sequence;
    p.stateId = -1;
    p.post = p.thisLast = p.partner = -1;
    p.sched = -1;
    p.waitingTime = -1;
    p.withinOff = (int)withins.size();
    p.withinCnt = (int)stack.size();
    for (auto& w : stack) {
      DWithin d{};
      d.t = w.first;
      d.n = (int)w.second.size();
      for (int k = 0; k < d.n && k < 2; ++k) d.ids[k] = w.second[k];
      withins.push_back(d);
    }
    pres.push_back(p);
    return (int)pres.size() - 1;
  }
  int new_post(int kind) {
    DPost p{};
    p.kind = kind;
    p.stateId = -1;
    p.nextPre = p.nextEveryPre = p.thisPre = p.callbackPre = p.partnerPre = p.partnerPost = -1;
    posts.push_back(p);
    return (int)posts.size() - 1;
  }
  void push_within(int64_t t, std::vector<int> ids) { stack.insert(stack.begin(), {t, std::move(ids)}); }
  void pop_within() { stack.erase(stack.begin()); }

  int inner(int kind, int first, int last, int a, int b, const std::string& sid) {
    DInner d{kind, first, last, a, b};
    inners.push_back(d);
    inner_stream.push_back(sid);
    return (int)inners.size() - 1;
  }

  // StateInputStreamParser.parse :132-432
  int parse(const StateElem* el, int pre, int post) {
    switch (el->kind) {
      case StateKind::STREAM:
      case StateKind::ABSENT: {
        const StreamDef* def = app.find_stream(el->stream_id);
        metas.push_back({def, el->event_ref, stream_index(app, el->stream_id)});
        if ((int)metas.size() > kMaxSlots) throw UnsupportedError("too many states in one pattern");
        int stateIndex = (int)metas.size() - 1;
        Emitter em{dict, code, consts};
        em.metas = &metas;
        em.current_state = stateIndex;
        em.default_index = kCurrent;
        int off = (int)code.size();
        for (size_t k = 0; k < el->filters.size(); ++k) {
          if (em.emit(*el->filters[k]) != T_BOOL) throw ValidationError("filter condition should be of type BOOL");
          if (k > 0) {
            Instr a{};
            a.op = OP_AND;
            code.push_back(a);
          }
        }
        int len = (int)code.size() - off;
        if (pre < 0) {
          if (el->has_within) push_within(el->within_ms, {-1});
          if (el->kind == StateKind::ABSENT) {
            pre = new_pre(PK_ABSENT_STREAM);
            pres[pre].waitingTime = el->wait_ms;
            pres[pre].sched = nsched++;
          } else {
            pre = new_pre(PK_STREAM);
          }
          if (el->has_within) pop_within();
        }
        pres[pre].stateId = stateIndex;
        pres[pre].progOff = off;
        pres[pre].progLen = len;
        pres[pre].trialCur = 1;
        for (int i = off; i < off + len; ++i)
          if (code[i].op == OP_VAR && code[i].a == stateIndex && code[i].b != kCurrent) pres[pre].trialCur = 0;
        if (post < 0) post = new_post(el->kind == StateKind::ABSENT ? PK_ABSENT_STREAM : PK_STREAM);
        posts[post].stateId = stateIndex;
        posts[post].thisPre = pre;
        pres[pre].post = post;
        pres[pre].thisLast = post;
        return inner(IK_STREAM, pre, post, -1, -1, el->stream_id);
      }
      case StateKind::NEXT: {
        int cur = parse(el->a.get(), -1, -1);
        if (el->has_within)
          push_within(el->within_ms, {pres[inners[cur].first].stateId, posts[inners[cur].last].stateId});
        int nxt = parse(el->b.get(), -1, -1);
        if (el->has_within) pop_within();
        set_next(inners[cur].last, inners[nxt].first);
        return inner(IK_NEXT, inners[cur].first, inners[nxt].last, cur, nxt, inner_stream[cur]);
      }
      case StateKind::EVERY: {
        int in = parse(el->a.get(), -1, -1);
        int last = inners[in].last;
        posts[last].nextEveryPre = inners[in].first;
        if (posts[last].kind == PK_LOGICAL || posts[last].kind == PK_ABSENT_LOGICAL)
          posts[posts[last].partnerPost].nextEveryPre = inners[in].first;
        return inner(IK_EVERY, inners[in].first, last, in, -1, inner_stream[in]);
      }
      case StateKind::LOGICAL: {
        if (el->has_within) push_within(el->within_ms, {-1});
        const StateElem* e1 = el->a.get();
        const StateElem* e2 = el->b.get();
        if (e1->kind != StateKind::STREAM && e1->kind != StateKind::ABSENT)
          throw UnsupportedError("logical operands must be stream states");
        bool a1 = e1->kind == StateKind::ABSENT, a2 = e2->kind == StateKind::ABSENT;
        int p1 = new_pre(a1 ? PK_ABSENT_LOGICAL : PK_LOGICAL);
        pres[p1].ltype = el->ltype == LogicalType::AND ? LT_AND : LT_OR;
        if (a1) {
          pres[p1].waitingTime = e1->has_wait ? e1->wait_ms : -1;
          pres[p1].sched = nsched++;
        }
        int o1 = new_post(a1 ? PK_ABSENT_LOGICAL : PK_LOGICAL);
        posts[o1].ltype = pres[p1].ltype;
        int p2 = new_pre(a2 ? PK_ABSENT_LOGICAL : PK_LOGICAL);
        pres[p2].ltype = pres[p1].ltype;
        if (a2) {
          pres[p2].waitingTime = e2->has_wait ? e2->wait_ms : -1;
          pres[p2].sched = nsched++;
        }
        int o2 = new_post(a2 ? PK_ABSENT_LOGICAL : PK_LOGICAL);
        posts[o2].ltype = pres[p1].ltype;
        if (el->has_within) pop_within();
        posts[o1].partnerPre = p2;
        posts[o2].partnerPre = p1;
        posts[o1].partnerPost = o2;
        posts[o2].partnerPost = o1;
        pres[p1].partner = p2;
        pres[p2].partner = p1;
        int in2 = parse(e2, p2, o2);
        int in1 = parse(e1, p1, o1);
        return inner(IK_LOGICAL, inners[in1].first, inners[in2].last, in1, in2, inner_stream[in2]);
      }
      case StateKind::COUNT: {
        int mn = el->min_count == kAny ? 0 : el->min_count;
        int mx = el->max_count == kAny ? INT32_MAX : el->max_count;
        if (el->has_within) push_within(el->within_ms, {-1});
        int cp = new_pre(PK_COUNT);
        pres[cp].minCount = mn;
        pres[cp].maxCount = mx;
        int co = new_post(PK_COUNT);
        posts[co].minCount = mn;
        posts[co].maxCount = mx;
        if (el->has_within) pop_within();
        if (el->a->kind != StateKind::STREAM) throw UnsupportedError("count operand must be a stream state");
        int in = parse(el->a.get(), cp, co);
        return inner(IK_COUNT, inners[in].first, inners[in].last, in, -1, inner_stream[in]);
      }
    }
    throw UnsupportedError("state element");
  }

  void set_next(int post, int next) {
    DPost& po = posts[post];
    if (po.kind == PK_LOGICAL || po.kind == PK_ABSENT_LOGICAL) {
      po.nextPre = next;
      posts[po.partnerPost].nextPre = next;
    } else if (po.kind == PK_COUNT) {
      po.nextPre = next;
      // CountPostStateProcessor.setNextStatePreProcessor :87-95 — evaluated here with isStartState as it
      // stands during parsing (false: setStartState runs later in QueryRuntime.init), so never taken.
      const DPre& tp = pres[po.thisPre];
      if (tp.isStart && tp.sequence && po.minCount == 0) posts[pres[next].post].callbackPre = po.thisPre;
    } else {
      po.nextPre = next;
    }
  }
};

}  // namespace

CompiledQuery compile_query(const App& app, const Query& q, int order, int partition, Dict& dict) {
  CompiledQuery cq;
  cq.name = q.name;
  cq.insert_into = q.insert_into;
  cq.order = order;
  cq.partition = partition;
  DQuery& h = cq.hdr;
  h.query_order = order;
  h.partitioned = partition >= 0;
  std::vector<DPre> pres;
  std::vector<DPost> posts;
  std::vector<DInner> inners;
  std::vector<DReceiver> recvs;
  std::vector<DWithin> withins;
  std::vector<Instr> code;
  std::vector<DVal> consts;
  std::vector<int32_t> sel;  // (off, len, type) triples
  std::vector<int32_t> refs; // (slot, idx) pairs
  std::vector<int32_t> init_order;

  if (q.input == InputKind::SINGLE) {
    h.kind = 0;
    int si = stream_index(app, q.stream_id);
    const StreamDef* def = &app.streams[si];
    h.stream = si;
    cq.streams.push_back(si);
    Emitter em{dict, code, consts};
    em.stream = def;
    h.filt_off = (int)code.size();
    for (size_t k = 0; k < q.filters.size(); ++k) {
      if (em.emit(*q.filters[k]) != T_BOOL) throw ValidationError("filter condition should be of type BOOL");
      if (k > 0) {
        Instr a{};
        a.op = OP_AND;
        code.push_back(a);
      }
    }
    if (q.having) {
      OutAttrs outs;
      std::vector<Expr> star;
      if (q.select_all) {
        star.resize(def->attrs.size());
        for (size_t k = 0; k < def->attrs.size(); ++k) {
          star[k].kind = ExprKind::VAR;
          star[k].attr = def->attrs[k].name;
          outs.push_back({def->attrs[k].name, &star[k]});
        }
      } else {
        for (auto& oa : q.select) outs.push_back({oa.rename, oa.expr.get()});
      }
      // QuerySelector drops the event after projection; with no aggregation that is one more filter
      if (em.emit(*having_subst(*q.having, outs, true)) != T_BOOL)
        throw ValidationError("having condition should be of type BOOL");
      if (!q.filters.empty()) {
        Instr a{};
        a.op = OP_AND;
        code.push_back(a);
      }
    }
    h.filt_len = (int)code.size() - h.filt_off;
    std::vector<std::pair<int, int>> vr;
    em.var_refs = &vr;
    auto add_sel = [&](const Expr& x, const std::string& name) {
      int off = (int)code.size();
      int t = em.emit(x);
      sel.push_back(off);
      sel.push_back((int)code.size() - off);
      sel.push_back(t);
      cq.sel_types.push_back(t);
      cq.sel_names.push_back(name);
    };
    if (q.select_all) {
      for (auto& a : def->attrs) {
        Expr v;
        v.kind = ExprKind::VAR;
        v.attr = a.name;
        add_sel(v, a.name);
      }
    } else {
      for (auto& oa : q.select) add_sel(*oa.expr, oa.rename);
    }
    for (auto& r : vr) {
      refs.push_back(r.first);
      refs.push_back(r.second);
    }
  } else {
    h.kind = q.input == InputKind::PATTERN ? 1 : 2;
    Lowering lw{app, dict, q.input == InputKind::SEQUENCE};
    int root = lw.parse(q.state.get(), -1, -1);
    // StateInputStreamParser.parseInputStream :124-125
    lw.pres[lw.inners[root].first].thisLast = lw.inners[root].last;
    // list-node operand caches (plan.h DPre.ncache): a trialCur stream / count state whose filter reads at most two
    // distinct operands of other states, each an earlier PK_STREAM state (its single-event chain is set before the
    // partial reaches this state and is changed afterwards only by that state's own processor, which has let the
    // partial go). Loads are keyed by (state, index, attribute, op).
    for (auto& P : lw.pres) {
      P.ncache = 0;
      P.cacheIns[0] = P.cacheIns[1] = -1;
      // (not in sequences: there a partial is mostly tried once before the next event resets it, and the fill would
      // be the same three dependent reads a trial makes, plus two words per node; measured: literal config 5 NFA
      // 17.4 -> 18.9 ms with the cache)
      if (P.sequence || !P.trialCur || P.progLen == 0 || (P.kind != PK_STREAM && P.kind != PK_COUNT)) continue;
      bool ok = true;
      int n = 0;
      for (int i = P.progOff; i < P.progOff + P.progLen && ok; ++i) {
        const Instr& in = lw.code[i];
        if (in.op != OP_VAR && in.op != OP_TS) continue;
        if (in.a == P.stateId) continue;  // own state: the incoming event (trialCur)
        const DPre* src = nullptr;
        for (auto& Q : lw.pres)
          if (Q.stateId == in.a) src = &Q;
        if (!src || src->kind != PK_STREAM || in.a >= P.stateId) {
          ok = false;
          break;
        }
        bool seen = false;
        for (int k = 0; k < n; ++k) {
          const Instr& c = lw.code[P.cacheIns[k]];
          seen |= c.op == in.op && c.a == in.a && c.b == in.b && c.c == in.c;
        }
        if (seen) continue;
        if (n == 2) ok = false;
        else P.cacheIns[n++] = i;
      }
      if (ok && n > 0) P.ncache = n;
      else P.cacheIns[0] = P.cacheIns[1] = -1;
    }
    // receivers :95-114
    std::vector<std::string> ids;
    collect_stream_ids(q.state.get(), ids);
    std::vector<std::string> uniq;
    for (auto& id : ids)
      if (std::find(uniq.begin(), uniq.end(), id) == uniq.end()) uniq.push_back(id);
    for (auto& id : uniq) {
      DReceiver r{};
      r.stream = stream_index(app, id);
      r.multi = std::count(ids.begin(), ids.end(), id) > 1;
      recvs.push_back(r);
      cq.streams.push_back(r.stream);
    }
    auto recv_of = [&](const std::string& id) -> DReceiver& {
      for (size_t k = 0; k < uniq.size(); ++k)
        if (uniq[k] == id) return recvs[k];
      throw std::runtime_error("receiver");
    };
    // QueryRuntime.init → setCommonProcessor: setQuerySelector, setStartState, init (:71-75)
    std::function<void(int)> set_qs = [&](int in) {
      const DInner& d = lw.inners[in];
      switch (d.kind) {
        case IK_STREAM:
        case IK_COUNT: lw.posts[d.last].hasNext = 1; break;
        case IK_NEXT: set_qs(d.b); break;
        case IK_EVERY: set_qs(d.a); break;
        case IK_LOGICAL: set_qs(d.b); set_qs(d.a); break;
      }
    };
    std::function<void(int)> set_start = [&](int in) {
      const DInner& d = lw.inners[in];
      switch (d.kind) {
        case IK_STREAM:
        case IK_COUNT: {
          DPre& p = lw.pres[d.first];
          p.isStart = 1;
          if ((p.kind == PK_LOGICAL || p.kind == PK_ABSENT_LOGICAL) && p.partner >= 0) lw.pres[p.partner].isStart = 1;
          break;
        }
        case IK_NEXT: set_start(d.a); break;
        case IK_EVERY: set_start(d.a); break;
        case IK_LOGICAL: set_start(d.b); set_start(d.a); break;
      }
    };
    std::vector<int> multi_procs_order[32];
    std::function<void(int)> init = [&](int in) {
      const DInner& d = lw.inners[in];
      switch (d.kind) {
        case IK_STREAM:
        case IK_COUNT: {
          DReceiver& r = recv_of(lw.inner_stream[in]);
          if (r.nstate >= kMaxProcs) throw UnsupportedError("too many states on one stream");
          if (r.multi) r.hasQuerySelector = lw.posts[lw.pres[d.first].post].hasNext;
          else r.hasQuerySelector = lw.posts[lw.pres[d.first].thisLast].hasNext;
          r.procs[r.nproc++] = d.first;  // setNext order
          r.stateProcs[r.nstate++] = d.first;
          if (!lw.sequence) init_order.push_back(d.first);
          break;
        }
        case IK_NEXT: init(d.a); init(d.b); break;
        case IK_EVERY: init(d.a); break;
        case IK_LOGICAL: init(d.b); init(d.a); break;
      }
    };
    set_qs(root);
    set_start(root);
    init(root);
    // Multi receivers process nextProcessors in reversed registration order (eventSequence)
    for (auto& r : recvs)
      if (r.multi) std::reverse(r.procs, r.procs + r.nproc);
    h.root_inner = root;
    // resetAndUpdate visiting orders (NextInnerStateRuntime.java:58-68: next.reset() then current.reset(),
    // current.update() then next.update(); LogicalInnerStateRuntime.java:62-70: inner2 only; Stream / Count /
    // Every: the first pre processor), flattened so the device loops over a constant list per event
    auto flatten = [&](bool reset, int32_t* out, int32_t& n) {
      std::vector<int> st{root};
      n = 0;
      while (!st.empty()) {
        const DInner& d = lw.inners[st.back()];
        st.pop_back();
        switch (d.kind) {
          case IK_STREAM:
          case IK_COUNT:
          case IK_EVERY:
            if (n >= 2 * kMaxSlots) throw UnsupportedError("inner runtime too large");
            out[n++] = d.first;
            break;
          case IK_NEXT:
            if (reset) { st.push_back(d.a); st.push_back(d.b); }
            else { st.push_back(d.b); st.push_back(d.a); }
            break;
          default: st.push_back(d.b); break;
        }
      }
    };
    flatten(true, h.reset_seq, h.nreset);
    flatten(false, h.update_seq, h.nupdate);
    // selector (SelectorParser :140-200): currentState UNKNOWN, default chain index 0
    Emitter em{dict, lw.code, lw.consts};
    em.metas = &lw.metas;
    em.current_state = -1;
    em.default_index = 0;
    std::vector<std::pair<int, int>> vr;
    em.var_refs = &vr;
    auto add_sel = [&](const Expr& x, const std::string& name) {
      int off = (int)lw.code.size();
      int t = em.emit(x);
      sel.push_back(off);
      sel.push_back((int)lw.code.size() - off);
      sel.push_back(t);
      cq.sel_types.push_back(t);
      cq.sel_names.push_back(name);
    };
    if (q.select_all) {
      std::set<std::string> seen;
      for (auto& m : lw.metas)
        for (auto& at : m.def->attrs) {
          if (!seen.insert(at.name).second) throw ValidationError("Duplicate attribute exist in streams");
          Expr v;
          v.kind = ExprKind::VAR;
          v.attr = at.name;
          add_sel(v, at.name);
        }
    } else {
      for (auto& oa : q.select) add_sel(*oa.expr, oa.rename);
    }
    for (auto& r : vr) {
      refs.push_back(r.first);
      refs.push_back(r.second);
    }
    if (q.having) {  // evaluated on the run record before the output is written (nfa_impl.h emit)
      OutAttrs outs;
      if (!q.select_all)
        for (auto& oa : q.select) outs.push_back({oa.rename, oa.expr.get()});
      em.var_refs = nullptr;
      h.having_off = (int)lw.code.size();
      if (em.emit(*having_subst(*q.having, outs, false)) != T_BOOL)
        throw ValidationError("having condition should be of type BOOL");
      h.having_len = (int)lw.code.size() - h.having_off;
    }
    for (auto& p : lw.pres)
      if (p.kind == PK_ABSENT_STREAM || p.kind == PK_ABSENT_LOGICAL) cq.has_absent = true;
    if (cq.has_absent && !app.playback)
      throw UnsupportedError("absent patterns ('not … for') require @app:playback (wall-clock timers are not reproducible)");
    h.nslots = (int)lw.metas.size();
    int maxattr = 0;
    for (int s = 0; s < h.nslots; ++s) {
      h.slot_nattr[s] = (int)lw.metas[s].def->attrs.size();
      h.slot_stream[s] = lw.metas[s].stream;
      maxattr = std::max(maxattr, h.slot_nattr[s]);
    }
    h.node_words = 4 + maxattr;  // hdr|next, ts, ordinal, null mask, attributes
    h.rec_words = 2 + (h.nslots + 1) / 2;
    h.nsched = lw.nsched;
    pres = lw.pres;
    posts = lw.posts;
    inners = lw.inners;
    withins = lw.withins;
    code = std::move(lw.code);
    consts = std::move(lw.consts);

    // ---- fast path detection: every e1=S[c1] -> e2=S[c2] (within T on e2), pattern, 2 slots
    const StateElem* root_el = q.state.get();
    if (q.input == InputKind::PATTERN && root_el->kind == StateKind::NEXT && !root_el->has_within &&
        root_el->a->kind == StateKind::EVERY && root_el->a->a->kind == StateKind::STREAM && !root_el->a->has_within &&
        !root_el->a->a->has_within && root_el->b->kind == StateKind::STREAM &&
        root_el->a->a->stream_id == root_el->b->stream_id && h.nslots == 2) {
      bool ok = !q.having;  // the closed form writes every match
      // selects may use any position; the closed form gives each output's e1/e2 single events
      for (size_t k = 0; k < refs.size(); k += 2)
        if (!(refs[k + 1] == 0 || refs[k + 1] == kCurrent)) ok = false;
      if (ok) {
        cq.fast_every_within = true;
        cq.fast_within = root_el->b->has_within ? root_el->b->within_ms : -1;
        cq.fast_c1_off = pres[0].progOff;
        cq.fast_c1_len = pres[0].progLen;
        cq.fast_c2_off = pres[1].progOff;
        cq.fast_c2_len = pres[1].progLen;
      }
    }
  }
  h.npre = (int)pres.size();
  h.npost = (int)posts.size();
  h.ninner = (int)inners.size();
  h.nrecv = (int)recvs.size();
  h.nwithin = (int)withins.size();
  h.nsel = (int)cq.sel_types.size();
  h.nrefs_vis = (int)refs.size() / 2;
  if (cq.fast_every_within) {  // hidden (e1, e2) ordinals for the NFA fallback of device batches
    refs.insert(refs.end(), {0, 0, 1, 0});
  }
  h.nrefs = (int)refs.size() / 2;
  h.nconst = (int)consts.size();
  // per-key state layout (int64 words)
  h.ks_pre = 0;
  int32_t kso = h.ks_pre;
  for (auto& p : pres) {
    p.ksOff = kso;
    kso += (p.kind == PK_ABSENT_STREAM || p.kind == PK_ABSENT_LOGICAL) ? kPreWordsAbsent : kPreWords;
  }
  h.ks_post = kso;
  if (h.npost > 62) throw UnsupportedError("more than 62 states in one query");
  h.ks_sched = h.ks_post + 1;  // the post processors' isEventReturned bits, one word
  h.ks_misc = h.ks_sched + h.nsched * (2 + kSchedCap);
  h.ks_words = h.ks_misc + 8;

  // pack blob
  auto align8 = [](size_t x) { return (x + 7) & ~size_t(7); };
  size_t off = align8(sizeof(DQuery));
  auto place = [&](size_t bytes) {
    size_t o = off;
    off = align8(off + bytes);
    return (int32_t)o;
  };
  h.off_pre = place(pres.size() * sizeof(DPre));
  h.off_post = place(posts.size() * sizeof(DPost));
  h.off_inner = place(inners.size() * sizeof(DInner));
  h.off_recv = place(recvs.size() * sizeof(DReceiver));
  h.off_within = place(withins.size() * sizeof(DWithin));
  h.off_code = place(code.size() * sizeof(Instr));
  h.off_const = place(consts.size() * sizeof(DVal));
  h.off_sel = place(sel.size() * sizeof(int32_t));
  h.off_refs = place(refs.size() * sizeof(int32_t));
  int32_t off_init = place((init_order.size() + 1) * sizeof(int32_t));
  cq.blob.assign(off, 0);
  char* b = cq.blob.data();
  auto put = [&](int32_t o, const void* src, size_t bytes) {
    if (bytes) memcpy(b + o, src, bytes);
  };
  put(h.off_pre, pres.data(), pres.size() * sizeof(DPre));
  put(h.off_post, posts.data(), posts.size() * sizeof(DPost));
  put(h.off_inner, inners.data(), inners.size() * sizeof(DInner));
  put(h.off_recv, recvs.data(), recvs.size() * sizeof(DReceiver));
  put(h.off_within, withins.data(), withins.size() * sizeof(DWithin));
  put(h.off_code, code.data(), code.size() * sizeof(Instr));
  put(h.off_const, consts.data(), consts.size() * sizeof(DVal));
  put(h.off_sel, sel.data(), sel.size() * sizeof(int32_t));
  put(h.off_refs, refs.data(), refs.size() * sizeof(int32_t));
  int32_t ninit = (int32_t)init_order.size();
  put(off_init, &ninit, sizeof(int32_t));
  put(off_init + 4, init_order.data(), init_order.size() * sizeof(int32_t));
  h.ks_misc = h.ks_misc;  // layout already set
  // the init list offset rides in pad fields of DQuery: store after header via filt fields for state queries
  if (h.kind != 0) h.filt_off = off_init;
  memcpy(b, &h, sizeof(DQuery));
  return cq;
}

CompiledPartition compile_partition(const App& app, const Partition& p, Dict& dict) {
  CompiledPartition cp;
  for (auto& w : p.with) {
    int si = stream_index(app, w.stream_id);
    if (std::find(cp.streams.begin(), cp.streams.end(), si) != cp.streams.end())
      throw UnsupportedError("multiple partition keys for one stream are not supported");
    std::vector<Instr> code;
    std::vector<DVal> consts;
    Emitter em{dict, code, consts};
    em.stream = &app.streams[si];
    int t = em.emit(*w.key);
    cp.streams.push_back(si);
    cp.key_code.push_back(std::move(code));
    cp.key_consts.push_back(std::move(consts));
    cp.key_type.push_back(t);
  }
  // all keys of one partition must share a key class (String.valueOf identity restated on int64 keys)
  auto cls = [](int t) { return (t == T_INT || t == T_LONG) ? 0 : t; };
  for (size_t k = 1; k < cp.key_type.size(); ++k)
    if (cls(cp.key_type[k]) != cls(cp.key_type[0]))
      throw UnsupportedError("partition keys of different types are not supported");
  return cp;
}

}  // namespace sm
