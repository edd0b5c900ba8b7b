// CPU DEBUG BUILD of the product's device NFA code (siddhi_amd/csrc/kernels/nfa_impl.h + expr.h), compiled
// with g++ and hd.h's shims so faults can be found with gdb / AddressSanitizer on the host instead of on the
// GPU. Test infrastructure only: the product library never contains or calls this code.
//
// It restates runtime.cpp's batch pipeline (record selection, partition-key slots in first-seen order,
// per-key lanes, output ordering) with host containers, runs every lane sequentially through nfa_lane(), and
// dumps outputs in the product's JSON shape, so tests can compare it with both the oracle and the GPU.
#include <algorithm>
#include <charconv>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../siddhi_amd/csrc/compiler.h"
#include "../../siddhi_amd/csrc/kernels/nfa_impl.h"

using namespace sm;

namespace {

struct Stage {
  const sql::StreamDef* def;
  std::vector<std::vector<int64_t>> cols;  // stored widened; views are rebuilt per flush with native widths
  std::vector<std::vector<uint8_t>> nulls;
  std::vector<int64_t> row_pos;
  int64_t rows = 0;
};

struct HQuery {
  CompiledQuery cq;
  const CompiledPartition* part = nullptr;
  std::unordered_map<int64_t, int32_t> slot_of;
  int32_t nslots = 0;
  std::vector<int64_t> ks, heap;
  int64_t state_slots = 0;
};

struct HostOut {
  OutRec r;
  std::vector<DVal> vals;
  std::vector<int64_t> refs;
  int q;
};

struct HApp {
  sql::App ast;
  Dict dict;
  std::vector<Stage> st;
  std::vector<CompiledPartition> parts;
  std::vector<std::unique_ptr<HQuery>> qs;
  std::vector<int32_t> ev_stream;
  std::vector<int64_t> ev_row, ev_ts, ev_clock, ev_ord, adv_pos, adv_clock, adv_wall;
  int64_t next_ord = 0;
  int64_t base = 0, clock = 0, clock_in = 0;
  int32_t heap_half = getenv("SM_HOST_HEAP_HALF") ? atoi(getenv("SM_HOST_HEAP_HALF")) : 1024;
  bool started = false;
  std::map<std::string, std::vector<std::string>> so, qo;
  std::string err;
};

void stage(HApp* a, int32_t s, int64_t row, int64_t ts, int wall) {
  int64_t p = (int64_t)a->ev_stream.size();
  a->ev_stream.push_back(s);
  a->ev_row.push_back(row);
  a->ev_ts.push_back(ts);
  a->ev_ord.push_back(s >= 0 ? a->next_ord++ : -1);
  if (a->ast.playback && s != NFA_START && ts >= a->clock) {
    a->clock = ts;
    a->adv_pos.push_back(p);
    a->adv_clock.push_back(ts);
    a->adv_wall.push_back(wall ? ts : -1);
  }
  a->ev_clock.push_back(a->clock);
}

struct HostColLoader {
  const NfaStream* st;
  int64_t row;
  StackVal var(const Instr& in) const {
    StackVal v{};
    int a = in.a;
    if (st->nulls[a] && st->nulls[a][row]) {
      v.null = 1;
      return v;
    }
    switch (st->types[a]) {
      case T_INT: v.i = ((const int32_t*)st->cols[a])[row]; break;
      case T_LONG: v.i = ((const int64_t*)st->cols[a])[row]; break;
      case T_FLOAT: v.d = (double)((const float*)st->cols[a])[row]; break;
      case T_DOUBLE: v.d = ((const double*)st->cols[a])[row]; break;
      case T_STRING: v.i = ((const int32_t*)st->cols[a])[row]; v.null = v.i < 0; break;
      default: v.i = ((const uint8_t*)st->cols[a])[row]; break;
    }
    return v;
  }
};

void json_val(std::ostringstream& o, const HApp* a, const DVal& v, int t) {
  if (v.null) { o << "null"; return; }
  switch (t) {
    case T_INT:
    case T_LONG: o << v.i; break;
    case T_BOOL: o << (v.i ? "true" : "false"); break;
    case T_FLOAT:
    case T_DOUBLE: {
      char b[64];
      auto r = std::to_chars(b, b + 64, v.d);
      std::string s(b, r.ptr);
      if (s.find_first_of(".eE") == std::string::npos) s += ".0";
      o << s;
      break;
    }
    default:
      if (v.i < 0 || v.i >= (int64_t)a->dict.strs.size()) o << "null";
      else o << '"' << a->dict.strs[v.i] << '"';
  }
}

void flush(HApp* a) {
  int64_t N = (int64_t)a->ev_stream.size();
  if (!N) return;
  // native-width column views
  std::vector<std::vector<std::vector<uint8_t>>> raw(a->st.size());
  std::vector<NfaStream> nst(a->st.size());
  for (size_t s = 0; s < a->st.size(); ++s) {
    Stage& S = a->st[s];
    NfaStream& d = nst[s];
    memset(&d, 0, sizeof(d));
    d.nattr = (int)S.def->attrs.size();
    raw[s].resize(d.nattr);
    for (int k = 0; k < d.nattr; ++k) {
      int t = (int)S.def->attrs[k].type;
      d.types[k] = t;
      auto& r = raw[s][k];
      int w = (t == T_LONG || t == T_DOUBLE) ? 8 : (t == T_BOOL ? 1 : 4);
      r.resize(std::max<int64_t>(S.rows, 1) * w);
      for (int64_t i = 0; i < S.rows; ++i) {
        int64_t x = S.cols[k][i];
        if (t == T_FLOAT) { float f = (float)__longlong_as_double(x); memcpy(&r[i * 4], &f, 4); }
        else if (w == 8) memcpy(&r[i * 8], &x, 8);
        else if (w == 4) { int32_t y = (int32_t)x; memcpy(&r[i * 4], &y, 4); }
        else r[i] = (uint8_t)x;
      }
      d.cols[k] = r.data();
      d.nulls[k] = S.nulls[k].empty() ? nullptr : S.nulls[k].data();
    }
  }
  std::vector<HostOut> outs;
  for (size_t qi = 0; qi < a->qs.size(); ++qi) {
    HQuery& q = *a->qs[qi];
    const DQuery& h = q.cq.hdr;
    const char* blob = q.cq.blob.data();
    int nsel = h.nsel, nrefs = h.nrefs;
    size_t stride = sizeof(OutRec) + nsel * sizeof(DVal) + nrefs * 8;
    if (h.kind == 0) {
      Stage& S = a->st[h.stream];
      const Instr* code = (const Instr*)(blob + h.off_code);
      const DVal* consts = (const DVal*)(blob + h.off_const);
      const int32_t* sel = (const int32_t*)(blob + h.off_sel);
      for (int64_t row = 0; row < S.rows; ++row) {
        HostColLoader ld{&nst[h.stream], row};
        if (h.filt_len && !truthy(eval_prog(code + h.filt_off, h.filt_len, consts, ld))) continue;
        HostOut o;
        memset(&o.r, 0, sizeof(o.r));
        int64_t p = S.row_pos[row];
        o.r.pos = p;
        o.r.phase = 1;
        o.r.query = h.query_order;
        o.r.ts = a->ev_ts[p];
        o.r.create = -1;
        for (int k = 0; k < nsel; ++k) {
          StackVal v = eval_prog(code + sel[3 * k], sel[3 * k + 1], consts, ld);
          DVal dv{};
          if (sel[3 * k + 2] == T_FLOAT || sel[3 * k + 2] == T_DOUBLE) dv.d = v.d;
          else dv.i = v.i;
          dv.null = v.null;
          o.vals.push_back(dv);
        }
        for (int k = 0; k < nrefs; ++k) o.refs.push_back(a->ev_ord[p]);
        o.q = (int)qi;
        outs.push_back(o);
      }
      continue;
    }
    std::vector<int64_t> pos;
    for (int64_t p = 0; p < N; ++p) {
      int s = a->ev_stream[p];
      if (s == NFA_START) {
        if (!h.partitioned) pos.push_back(p);
      } else if (s >= 0 && std::find(q.cq.streams.begin(), q.cq.streams.end(), s) != q.cq.streams.end()) {
        pos.push_back(p);
      }
    }
    std::vector<int64_t> key_off, key_pos;
    int64_t nkeys = 1;
    if (h.partitioned) {
      const CompiledPartition& cp = *q.part;
      std::vector<std::pair<int32_t, int64_t>> sp;  // slot, position
      for (int64_t p : pos) {
        int s = a->ev_stream[p];
        int k = (int)(std::find(cp.streams.begin(), cp.streams.end(), s) - cp.streams.begin());
        HostColLoader ld{&nst[s], a->ev_row[p]};
        StackVal v = eval_prog(cp.key_code[k].data(), (int)cp.key_code[k].size(), cp.key_consts[k].data(), ld);
        if (v.null) continue;
        int64_t key = (cp.key_type[k] == T_FLOAT || cp.key_type[k] == T_DOUBLE) ? __double_as_longlong(v.d) : v.i;
        auto it = q.slot_of.find(key);
        int32_t slot;
        if (it == q.slot_of.end()) {
          slot = q.nslots++;
          q.slot_of.emplace(key, slot);
        } else slot = it->second;
        sp.push_back({slot, p});
      }
      std::stable_sort(sp.begin(), sp.end(), [](auto& x, auto& y) { return x.first < y.first; });
      nkeys = q.nslots;
      key_off.assign(nkeys + 1, 0);
      for (auto& e : sp) key_off[e.first + 1]++;
      for (int64_t k = 0; k < nkeys; ++k) key_off[k + 1] += key_off[k];
      for (auto& e : sp) key_pos.push_back(e.second);
    } else {
      key_off = {0, (int64_t)pos.size()};
      key_pos = pos;
    }
    if (nkeys > q.state_slots) {  // ks rows are lane-interleaved (word-major): re-pitch each row; heap key-major
      auto grow = [&](std::vector<int64_t>& v, size_t words) {
        std::vector<int64_t> n((size_t)nkeys * words, 0);
        for (size_t w = 0; w < words; ++w)
          for (int64_t k = 0; k < q.state_slots; ++k) n[w * nkeys + k] = v[w * q.state_slots + k];
        v.swap(n);
      };
      grow(q.ks, (size_t)h.ks_words);
      q.heap.resize((size_t)nkeys * (2 * (size_t)a->heap_half + 64), 0);
      q.state_slots = nkeys;
    }
    std::vector<char> out((size_t)std::max<int64_t>(4096, 8 * (int64_t)pos.size() + 1024) * stride);
    unsigned count = 0;
    int err = 0;
    NfaBatch b{};
    b.ev_stream = a->ev_stream.data();
    b.ev_row = a->ev_row.data();
    b.ev_ts = a->ev_ts.data();
    b.ev_clock = a->ev_clock.data();
    b.ev_ord = a->ev_ord.data();
    b.streams = nst.data();
    b.adv_pos = a->adv_pos.data();
    b.adv_clock = a->adv_clock.data();
    b.adv_wall = a->adv_wall.data();
    b.nadv = (int64_t)a->adv_pos.size();
    b.clock_in = a->clock_in;
    b.key_off = key_off.data();
    b.key_pos = key_pos.empty() ? nullptr : key_pos.data();
    b.create_all = !h.partitioned;
    b.out = out.data();
    b.out_count = &count;
    b.out_cap = (uint32_t)(out.size() / stride);
    b.out_stride = (uint32_t)stride;
    {  // the compact LaneEv form under the device's rule (nfa.hip lane_compact_ok); SM_HOST_LANE_COMPACT=0 keeps 128 B
      const char* e = getenv("SM_HOST_LANE_COMPACT");
      int64_t lo = INT64_MAX, hi = -1;
      for (int64_t o : a->ev_ord)
        if (o >= 0) lo = std::min(lo, o), hi = std::max(hi, o);
      const bool ok = !(e && atoi(e) == 0) && h.node_words <= 8 && N < ((int64_t)1 << 31) && b.nadv < ((int64_t)1 << 31) &&
                      a->st.size() <= 127 && (hi < 0 || (uint64_t)(hi - lo) < kLeOrdMask);
      b.lane_compact = ok ? 1 : 0;
      b.lane_ord_base = hi < 0 ? 0 : lo;
    }
    std::vector<int64_t> lane_ev(std::max<size_t>(key_pos.size(), 1) * LaneEv::words(h.node_words, b.lane_compact));
    b.lane_ev = lane_ev.data();
    for (size_t k = 0; k < key_pos.size(); ++k) lane_event_record(b, key_pos[k], (int64_t)k, h.node_words, lane_ev.data());
    for (int32_t key = 0; key < nkeys; ++key) nfa_lane(b, blob, q.ks.data(), q.heap.data(), a->heap_half, q.state_slots, key, &err);
    if (err) throw std::runtime_error("nfa error flags " + std::to_string(err));
    for (unsigned k = 0; k < count; ++k) {
      const char* r = out.data() + (size_t)k * stride;
      HostOut o;
      memcpy(&o.r, r, sizeof(OutRec));
      o.vals.resize(nsel);
      memcpy(o.vals.data(), r + sizeof(OutRec), nsel * sizeof(DVal));
      o.refs.resize(nrefs);
      memcpy(o.refs.data(), r + sizeof(OutRec) + nsel * sizeof(DVal), nrefs * 8);
      o.q = (int)qi;
      outs.push_back(std::move(o));
    }
  }
  std::stable_sort(outs.begin(), outs.end(), [](const HostOut& x, const HostOut& y) {
    if (x.r.pos != y.r.pos) return x.r.pos < y.r.pos;
    if (x.r.phase != y.r.phase) return x.r.phase < y.r.phase;
    if (x.r.phase == 0) {
      if (x.r.time != y.r.time) return x.r.time < y.r.time;
      int gx = x.r.create >= 0, gy = y.r.create >= 0;
      if (gx != gy) return gx < gy;
      if (x.r.create != y.r.create) return x.r.create < y.r.create;
      if (x.r.query != y.r.query) return x.r.query < y.r.query;
      if (x.r.sched != y.r.sched) return x.r.sched < y.r.sched;
      return x.r.seq < y.r.seq;
    }
    if (x.r.query != y.r.query) return x.r.query < y.r.query;
    return x.r.seq < y.r.seq;
  });
  for (auto& o : outs) {
    const CompiledQuery& cq = a->qs[o.q]->cq;
    std::ostringstream s;
    s << "[" << o.r.ts << ",[";
    for (size_t k = 0; k < o.vals.size(); ++k) {
      if (k) s << ",";
      json_val(s, a, o.vals[k], cq.sel_types[k]);
    }
    s << "],[";
    for (size_t k = 0; k < o.refs.size(); ++k) s << (k ? "," : "") << o.refs[k];
    s << "]]";
    a->so[cq.insert_into].push_back(s.str());
    if (cq.partition < 0) {
      std::ostringstream qq;
      qq << "[" << o.r.ts << ",[[";
      for (size_t k = 0; k < o.vals.size(); ++k) {
        if (k) qq << ",";
        json_val(qq, a, o.vals[k], cq.sel_types[k]);
      }
      qq << "]]]";
      a->qo[cq.name].push_back(qq.str());
    }
  }
  a->base += N;
  a->clock_in = a->clock;
  a->ev_stream.clear(); a->ev_row.clear(); a->ev_ts.clear(); a->ev_clock.clear(); a->ev_ord.clear();
  a->adv_pos.clear(); a->adv_clock.clear(); a->adv_wall.clear();
  for (auto& S : a->st) {
    for (auto& c : S.cols) c.clear();
    for (auto& c : S.nulls) c.clear();
    S.row_pos.clear();
    S.rows = 0;
  }
}

}  // namespace

#ifdef SM_COUNT_ACCESS
namespace sm {
namespace {
int64_t g_access[8];
int g_phase;
int64_t g_phase_acc[2][16];
}
}  // namespace sm
extern "C" void h_access(int64_t* out) {
  for (int i = 0; i < 8; ++i) out[i] = sm::g_access[i];
}
extern "C" void h_access_phases(int64_t* out) {  // [kind][phase], kind 0 key-state, 1 heap
  for (int i = 0; i < 32; ++i) out[i] = sm::g_phase_acc[i / 16][i % 16];
}
#endif

extern "C" {

struct hv {
  int32_t type, is_null;
  int64_t i;
  double d;
  const char* s;
};

int h_create(const char* text, void** out, char* err, size_t len) {
  auto a = std::make_unique<HApp>();
  try {
    a->ast = sql::parse_app(text);
    for (auto& s : a->ast.streams) {
      Stage S;
      S.def = &s;
      S.cols.resize(s.attrs.size());
      S.nulls.resize(s.attrs.size());
      a->st.push_back(std::move(S));
    }
    for (auto& p : a->ast.partitions) a->parts.push_back(compile_partition(a->ast, p, a->dict));
    for (size_t o = 0; o < a->ast.order.size(); ++o) {
      auto [pi, qi] = a->ast.order[o];
      const sql::Query& qd = pi < 0 ? a->ast.queries[qi] : a->ast.partitions[pi].queries[qi];
      auto q = std::make_unique<HQuery>();
      q->cq = compile_query(a->ast, qd, (int)o, pi, a->dict);
      if (pi >= 0) {
        q->part = &a->parts[pi];
        for (int s : q->cq.streams)
          if (std::find(q->part->streams.begin(), q->part->streams.end(), s) == q->part->streams.end())
            throw sql::UnsupportedError("non-partitioned stream inside a partition is not supported");
        if (q->cq.hdr.kind == 0) throw sql::UnsupportedError("single-stream queries inside a partition");
      }
      a->qs.push_back(std::move(q));
    }
  } catch (const std::exception& e) {
    snprintf(err, len, "%s", e.what());
    if (dynamic_cast<const sql::ParseError*>(&e)) return 1;
    if (dynamic_cast<const sql::ValidationError*>(&e)) return 2;
    if (dynamic_cast<const sql::UnsupportedError*>(&e)) return 3;
    return 6;
  }
  *out = a.release();
  return 0;
}

void h_destroy(void* h) { delete (HApp*)h; }

void h_start(void* h) {
  HApp* a = (HApp*)h;
  if (a->started) return;
  a->started = true;
  stage(a, NFA_START, -1, a->clock, 0);
}

int h_send(void* h, const char* sid, int64_t ts, const hv* row) {
  HApp* a = (HApp*)h;
  int s = stream_index(a->ast, sid);
  Stage& S = a->st[s];
  for (size_t k = 0; k < S.def->attrs.size(); ++k) {
    int t = (int)S.def->attrs[k].type;
    int64_t x = 0;
    bool isnull = row[k].is_null;
    if (!isnull) {
      if (t == T_FLOAT) x = __double_as_longlong((double)(float)row[k].d);
      else if (t == T_DOUBLE) x = __double_as_longlong(row[k].d);
      else if (t == T_STRING) x = a->dict.intern(row[k].s ? row[k].s : "");
      else x = row[k].i;
    } else if (t == T_STRING) x = -1;
    S.cols[k].push_back(x);
    if (isnull && S.nulls[k].empty()) S.nulls[k].assign(S.rows, 0);
    if (!S.nulls[k].empty()) S.nulls[k].push_back(isnull);
  }
  S.row_pos.push_back((int64_t)a->ev_stream.size());
  stage(a, s, S.rows, ts, 0);
  S.rows++;
  return 0;
}

void h_advance(void* h, int64_t ts, int wall) {
  HApp* a = (HApp*)h;
  if (!a->ast.playback) return;
  stage(a, wall ? NFA_WALL : NFA_TICK, -1, ts, wall);
}

int h_flush(void* h, char* err, size_t len) {
  try {
    flush((HApp*)h);
  } catch (const std::exception& e) {
    snprintf(err, len, "%s", e.what());
    return 6;
  }
  return 0;
}

size_t h_dump(void* h, char* buf, size_t len) {
  HApp* a = (HApp*)h;
  std::ostringstream o;
  o << "{\"streams\":{";
  bool first = true;
  for (auto& kv : a->so) {
    o << (first ? "" : ",") << "\"" << kv.first << "\":[";
    first = false;
    for (size_t k = 0; k < kv.second.size(); ++k) o << (k ? "," : "") << kv.second[k];
    o << "]";
  }
  o << "},\"queries\":{";
  first = true;
  for (auto& kv : a->qo) {
    o << (first ? "" : ",") << "\"" << kv.first << "\":[";
    first = false;
    for (size_t k = 0; k < kv.second.size(); ++k) o << (k ? "," : "") << kv.second[k];
    o << "]";
  }
  o << "}}";
  std::string s = o.str();
  if (buf && len > s.size()) {
    memcpy(buf, s.data(), s.size());
    buf[s.size()] = 0;
  }
  return s.size();
}

}  // extern "C"
