// Host runtime + C ABI (include/siddhi_amd.h): SiddhiManager / SiddhiAppRuntime / InputHandler /
// callbacks restated over a batched device pipeline.
//
// send() stages events into per-stream host columns (the StreamJunction.sendData path,
// core/stream/StreamJunction.java:232); flush() uploads the batch once and runs every query on the GPU:
//   single-stream queries  → filter scan + projection kernels (stream_ops.hip)
//   pattern / sequence     → key grouping (stream_ops.hip) + NFA interpreter (nfa.hip)
// Outputs of all queries are ordered as the reference emits them (trigger position, timer phase, listener
// order, query order, emission order) and delivered to StreamCallback / QueryCallback on the calling thread.
#include <hip/hip_runtime.h>
#include <emmintrin.h>

#include <algorithm>
#include <array>
#include <charconv>
#include <chrono>
#include <cmath>
#include <cstring>
#include <deque>
#include <exception>
#include <functional>
#include <future>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <thread>
#include <string>
#include <type_traits>
#include <unordered_set>
#include <vector>

#include "../../include/siddhi_amd.h"
#include "compiler.h"
#include "kernels/fastpath.h"
#include "kernels/filter.h"
#include "kernels/nfa.h"
#include "kernels/primitives.h"
#include "kernels/stream_ops.h"
#include "kernels/partition.h"
#include "java_order.h"
#include "nfa_jit.h"
#include "siddhiql/ast.h"

namespace sm {
namespace {

thread_local std::string g_err;

struct DeviceError : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct TypeError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

int width_of(int t) {
  switch (t) {
    case T_INT: return 4;
    case T_LONG: return 8;
    case T_FLOAT: return 4;
    case T_DOUBLE: return 8;
    case T_STRING: return 4;
    default: return 1;
  }
}

// growable device buffer
struct DBuf {
  void* p = nullptr;
  size_t cap = 0;
  void* ensure(size_t bytes) {
    if (bytes > cap) {
      if (p) SM_HIP(hipFree(p));
      size_t c = std::max<size_t>(bytes, cap * 2);
      c = std::max<size_t>(c, 256);
      SM_HIP(hipMalloc(&p, c));
      cap = c;
    }
    return p;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  ~DBuf() { release(); }
};

struct StreamStage {
  const sql::StreamDef* def;
  std::vector<std::vector<uint8_t>> cols;
  std::vector<std::vector<uint8_t>> nulls;
  std::vector<bool> any_null;
  std::vector<int64_t> row_pos;
  int64_t rows = 0;
  // device copies for the current flush
  std::vector<DBuf> dcols, dnulls;
  DBuf drow_pos;
  DBuf drow_ts, drow_ord;  // flush_device: per-row event times and arrival ordinals
  void clear() {
    for (auto& c : cols) c.clear();
    for (auto& c : nulls) c.clear();
    std::fill(any_null.begin(), any_null.end(), false);
    row_pos.clear();
    rows = 0;
  }
};

// One output record read back from the device. Its selected values and reference ordinals stay in the record
// buffer it was read from (sm_app::out_arena, alive until the outputs are delivered): no allocation per output.
struct HostOut {
  OutRec r;
  const DVal* vals = nullptr;
  const int64_t* refs = nullptr;
  int nvals = 0, nrefs = 0;
  int qidx;
  int64_t e1 = -1, e2 = -1;  // closed-form queries: ordinals of the match's two events (hidden references)
  int64_t key_code = 0;      // partition queries: the instance's key code (an inner stream's routing key)
};

// Host copies of one query's device outputs (device_outputs), in its output order: the (e1, e2) tuples or a filter's
// rows (ordinals relative to base), the select values and the timestamps, all in sm_app::out_arena.
struct DevOut {
  int qi;
  int64_t m;
  const uint32_t* hp;
  const DVal* hv;       // values as DVal (nullptr in the compact form)
  const int64_t* hts;
  bool rows;
  int64_t base;
  const int64_t* hw = nullptr;  // compact form: one 64-bit word per value ...
  const uint8_t* hn = nullptr;  // ... and one byte of null flags per output (bit a: value a)
  // segments still in flight (round 5): outputs [seg_end[i-1], seg_end[i]) are in host memory once seg_ev[i] has
  // completed, so deliver_direct prepares the Events of a segment while later segments cross PCIe; empty = all copied
  std::vector<int64_t> seg_end;
  std::vector<hipEvent_t> seg_ev;
  hipEvent_t pairs_ev = nullptr;  // the (e1, e2) tuples (hp) are on the host
  void wait_all() const {
    for (hipEvent_t e : seg_ev) SM_HIP(hipEventSynchronize(e));
  }
};

struct Callback {
  sm_stream_callback scb = nullptr;
  sm_query_callback qcb = nullptr;
  sm_stream_columns_callback ccb = nullptr;  // a StreamCallback taking columns (sm_app_add_stream_columns_callback)
  void* user = nullptr;
};

template <typename F>
void parallel_for(size_t n, size_t grain, F&& f);

// A pinned host buffer (the app's output arena; a Pending in the views form owns the ones its views point into)
struct PinnedBuf {
  char* p = nullptr;
  size_t cap = 0;
};

// A growable array of trivially copyable elements whose growth does not initialise them (the Event arrays of a large
// output batch are filled by several threads right after they are sized).
template <typename T>
struct RawVec {
  static_assert(std::is_trivially_copyable<T>::value, "RawVec holds plain data");
  std::unique_ptr<T[]> p;
  size_t n = 0, cap = 0;
  size_t size() const { return n; }
  bool empty() const { return n == 0; }
  T* data() { return p.get(); }
  const T* data() const { return p.get(); }
  T& operator[](size_t i) { return p[i]; }
  T* begin() { return p.get(); }
  T* end() { return p.get() + n; }
  void resize(size_t m) {
    if (m > cap) {
      const size_t c = std::max(m, cap + cap / 2);
      std::unique_ptr<T[]> q(new T[c]);
      if (n) memcpy(q.get(), p.get(), n * sizeof(T));
      p.swap(q);
      cap = c;
    }
    n = m;
  }
  void push_back(const T& v) {
    resize(n + 1);
    p[n - 1] = v;
  }
  void clear() { n = 0; }
  void swap(RawVec& o) {
    p.swap(o.p);
    std::swap(n, o.n);
    std::swap(cap, o.cap);
  }
};

// One output chunk ready for the callbacks: the events one trigger (an input event or a scheduler firing) made
// one query emit, delivered as one StreamCallback.receive(Event[]) (StreamCallback.java:65-76) and one
// QueryCallback.receive(timestamp, in, removed) (QueryCallback.java:52-74). The chunks of one call share the arrays
// of a Pending (no allocation per chunk or per event): its callbacks are cbs[cb_off, cb_off + n_cbs) (the query's
// n_query_cbs QueryCallbacks first, then the output stream's StreamCallbacks), its events evs[ev_off, ev_off + n_ev).
struct PreparedChunk {
  int64_t ts = 0;
  uint32_t cb_off = 0, n_cbs = 0, n_query_cbs = 0;
  uint64_t ev_off = 0, n_ev = 0;
};

// The outputs of one call, prepared under the app lock with owned copies of everything the events point at, so
// the callbacks can run after the lock is released. Until finalise(), an event's data field holds the offset of its
// values in vals (vals still grows); finalise() turns the offsets into pointers once the call's outputs are complete.
struct Pending {
  RawVec<PreparedChunk> chunks;
  std::vector<Callback> cbs;
  RawVec<sm_event> evs;
  RawVec<sm_value> vals;
  std::vector<std::unique_ptr<std::string>> strs;  // owned STRING values (stable addresses)
  bool final_ = false;
  // uniform form (round 5, deliver_direct): every chunk of the call goes to the same callbacks (proto's cb fields), so
  // a chunk is only its first event's index (starts); its size is the distance to the next start and its timestamp
  // the last event's. 8 bytes per chunk instead of a 40-byte PreparedChunk, written and then read by the callbacks.
  bool uniform = false;
  PreparedChunk proto;
  RawVec<uint64_t> starts;
  // views form (round 6; uniform, and every callback of the call takes columns): no Events are built at all. Output
  // k's timestamp is cts[k], its select values cvals[k * cns ..] (8-byte words), its null bits cnul[k]: views of the
  // device outputs' pinned host copies, whose buffers this Pending owns until the callbacks have run (taken from the
  // app's output arena, given back afterwards: a callback's own send into the app gets buffers of its own)
  bool views = false;
  const int64_t* cts = nullptr;
  const int64_t* cvals = nullptr;
  const uint8_t* cnul = nullptr;
  int32_t cns = 0;
  int32_t ctypes[8] = {0};
  size_t cn = 0;
  std::vector<PinnedBuf> owned;
  // views of a bulk send's deferred copies (DevOut segments): outputs [seg_end[i-1], seg_end[i]) are on the host once
  // seg_ev[i] has completed, so the callbacks of the first chunks run while later segments still cross PCIe
  std::vector<int64_t> seg_end;
  std::vector<hipEvent_t> seg_ev;
  void wait_segments() {
    for (hipEvent_t e : seg_ev) SM_HIP(hipEventSynchronize(e));
    seg_ev.clear();
    seg_end.clear();
  }
  ~Pending() {
    for (hipEvent_t e : seg_ev) (void)hipEventSynchronize(e);  // copies into the owned buffers have landed
    for (auto& b : owned)
      if (b.p) (void)hipHostFree(b.p);
  }
  void swap(Pending& o) {
    chunks.swap(o.chunks);
    cbs.swap(o.cbs);
    evs.swap(o.evs);
    vals.swap(o.vals);
    strs.swap(o.strs);
    std::swap(final_, o.final_);
    std::swap(uniform, o.uniform);
    std::swap(proto, o.proto);
    starts.swap(o.starts);
    std::swap(views, o.views);
    std::swap(cts, o.cts);
    std::swap(cvals, o.cvals);
    std::swap(cnul, o.cnul);
    std::swap(cns, o.cns);
    std::swap(ctypes, o.ctypes);
    std::swap(cn, o.cn);
    owned.swap(o.owned);
    seg_end.swap(o.seg_end);
    seg_ev.swap(o.seg_ev);
  }
  void clear() {  // keeps the capacity (a bulk send reuses it chunk after chunk); owned buffers were given back
    chunks.clear();
    cbs.clear();
    evs.clear();
    vals.clear();
    strs.clear();
    final_ = false;
    uniform = false;
    starts.clear();
    views = false;
    cts = cvals = nullptr;
    cnul = nullptr;
    cn = 0;
    seg_end.clear();
    seg_ev.clear();
  }
  // the views as Events (uniform form kept): before another delivery of the same call needs them
  void devolve() {
    if (!views) return;
    wait_segments();
    evs.resize(cn);
    vals.resize(cn * (size_t)cns);
    parallel_for(cn, (size_t)1 << 16, [&](size_t lo, size_t hi) {
      for (size_t k = lo; k < hi; ++k) {
        for (int j = 0; j < cns; ++j) {
          sm_value& v = vals[k * cns + j];
          v.type = ctypes[j];
          v.is_null = (cnul[k] >> j) & 1;
          const int64_t w = v.is_null ? 0 : cvals[k * cns + j];
          v.i = 0;
          v.d = 0;
          if (ctypes[j] == T_FLOAT || ctypes[j] == T_DOUBLE) memcpy(&v.d, &w, 8);
          else v.i = w;
          v.s = nullptr;
        }
        evs[k] = sm_event{cts[k], (const sm_value*)(uintptr_t)(k * cns), (int32_t)cns};
      }
    });
    final_ = false;
    views = false;
  }
  // the uniform form as PreparedChunks (before a general deliver appends chunks of other callbacks)
  void expand() {
    devolve();
    if (!uniform) return;
    if (final_) {  // deliver_direct's streamed form holds pointers already: offsets again, vals may grow
      for (auto& e : evs) e.data = (const sm_value*)(uintptr_t)(e.data - vals.data());
      final_ = false;
    }
    const size_t n = starts.size();
    chunks.resize(n);
    for (size_t c = 0; c < n; ++c) {
      PreparedChunk ch = proto;
      ch.ev_off = starts[c];
      const size_t end = c + 1 < n ? starts[c + 1] : evs.size();
      ch.n_ev = end - ch.ev_off;
      ch.ts = evs[end - 1].timestamp;
      chunks[c] = ch;
    }
    starts.clear();
    uniform = false;
  }
  void finalise() {
    if (final_) return;
    for (auto& e : evs) e.data = vals.data() + (uintptr_t)e.data;
    final_ = true;
  }
};

struct QueryRt {
  CompiledQuery cq;
  DBuf blob;
  // state queries
  KeyTable keys;
  DBuf ks, heap;
  int64_t state_slots = 0;  // slots with allocated per-key state
  DBuf out;
  DBuf keyprogs;             // KeyProg array (device)
  std::vector<DBuf> keycode; // code / consts backing the key programs
  int nkeyprogs = 0;
  const CompiledPartition* part = nullptr;
  int pidx = -1;             // its partition
  bool bcast = false;        // reads a stream its partition does not key (sent to every instance)
  // device batch results
  DBuf dev_pairs;
  int64_t dev_n = 0;
  int64_t n_out = 0;         // output records read back since the counter was last taken
  FastState fast;            // v2 kernels' persistent look-back state
  FastCarry carry;           // open partials carried across device batches (closed-form queries)
  // dense partition-key ids for the closed form (remap_keys): 0 = not decided yet, 1 = keys become dense ids (the
  // carry holds ids), 2 = the raw key column is used
  int remap = 0;
  DenseKeys dense;
  bool nfa_used = false;     // host-API batches ran through the NFA kernel (partials live in ks / heap)
  bool nfa_mode = false;     // a closed-form query handed to the NFA kernel for good (nfa_device_batch)
  int level = 0;             // chaining depth: 0 reads input streams only, L reads a stream a level L-1 query fills
  int nfa_kernel_used = 0;   // 1 = query-specialised NFA kernel, 2 = interpreter (last batch this query ran on the NFA)
  int fast_path_used = 0;    // 5 = NFA kernel, 3 = bucket stack, 2 = onesweep form, 1 = general form (last device
                             // batch)
  // what sm_app_device_project needs of the last closed-form batch: its stream, event times, ordinals, and the
  // carry as it was before the batch (carried e1 rows)
  bool proj_ok = false;
  NfaStream proj_desc{};
  DBuf proj_desc_dev;
  const int64_t* proj_ts = nullptr;
  const int64_t* proj_ord = nullptr;
  int64_t proj_base = 0, proj_n = 0;
  DBuf prev_carry;
  int64_t prev_carry_n = 0;
  int prev_carry_w = 0;
  // a batch the NFA kernel ran (hand-over): its outputs' select values (dev_n x nsel DVal) then timestamps
  bool proj_nfa = false;
  DBuf nfa_proj;
  DBuf proj_out;  // device projection of a batch for its consumers (device_outputs)
  // the last device-events batch's output records in delivery order, pos = trigger ordinal (option "keep_outputs":
  // sm_app_copy_device_outputs, the multi-GPU merge)
  DBuf ev_out;
  int64_t ev_out_n = 0;
  uint32_t ev_out_stride = 0;
  // overflow pool of per-key arenas (NfaBatch::pool, Lane::promote): allocated words, words handed out
  DBuf pool, pool_top_dev;
  int64_t pool_words = 0;
  uint64_t pool_used = 0;
  int64_t pool_refused = 0;  // batches in which a promotion did not fit the pool (stat pool_refused:<query>)
  int64_t pool_compactions = 0;
  ~QueryRt() {
    carry.release();
    dense.release();
  }
};

// v2 eligibility: c2 may read one attribute only (of e1 / e2 slots), c1 only e1, no timestamp reads.
int fast_vattr(const CompiledQuery& cq, const std::vector<int32_t>& types) {
  const DQuery& h = cq.hdr;
  const Instr* code = (const Instr*)(cq.blob.data() + h.off_code);
  int vattr = -1;
  for (int k = 0; k < cq.fast_c2_len; ++k) {
    const Instr& in = code[cq.fast_c2_off + k];
    if (in.op == OP_TS || in.op == OP_COL) return -1;
    if (in.op == OP_VAR) {
      if (in.a < 0 || in.a > 1 || !(in.b == 0 || in.b == -1)) return -1;
      if (vattr >= 0 && in.c != vattr) return -1;
      vattr = in.c;
    }
  }
  for (int k = 0; k < cq.fast_c1_len; ++k) {
    const Instr& in = code[cq.fast_c1_off + k];
    if (in.op == OP_TS) return -1;
    if (in.op == OP_VAR && (in.a != 0 || !(in.b == 0 || in.b == -1))) return -1;
  }
  if (vattr < 0) vattr = 0;
  if (vattr >= (int)types.size() || types[vattr] == T_STRING || types[vattr] == T_BOOL) return -1;
  return vattr;
}

}  // namespace
}  // namespace sm

struct sm_manager {
  int dummy = 0;
};

struct sm_input {
  struct sm_app* app;
  int stream;
};

struct sm_app {
  std::mutex mu;
  // device-batch fast path knobs (sm_app_set_option "fast_general" / "fast_timing") and the last timings
  bool force_general_fast = false;
  int fast_stack = 0;  // option "fast_stack": 0 = automatic, 1 = always the bucket-stack kernels, 2 = never
  int key_remap = -1;  // option "key_remap": 1 = closed-form keys always become dense ids, 0 = never, -1 = when the
                       // first batch's key span exceeds the bucket-stack window (2^20)
  int max_level = 0;   // deepest query chaining level (0: no query reads a stream another query fills)
  std::vector<char> stream_fed;  // per stream: some query reads it and some query inserts into it
  // per partition: the streams it does not key that its queries read (broadcast to every instance), and the key
  // codes of its instances in creation order (the instances a broadcast event reaches)
  std::vector<std::vector<int>> part_bcast;
  std::vector<std::vector<int64_t>> part_keys;
  std::vector<std::vector<int32_t>> part_key_types;  // the key's attribute type per instance (its Java string form)
  std::vector<std::unordered_set<int64_t>> part_key_set;
  // per partition and stream it broadcasts: the partition receiver's place among that stream's junction receivers
  // (the app order of the partition's first query reading it: PartitionRuntime.addPartitionReceiver subscribes then)
  std::vector<std::map<int, int32_t>> part_bcast_group;
  bool fast_timing = false;
  bool fast_tm_ready = false;
  sm::FastTimings fast_tm{};
  sql::App ast;
  sm::Dict dict;
  std::vector<sm::StreamStage> streams;
  std::vector<std::unique_ptr<sm::QueryRt>> queries;  // app order
  std::vector<sm::CompiledPartition> parts;
  std::vector<std::unique_ptr<sm_input>> inputs;
  std::map<std::string, std::vector<sm::Callback>> stream_cbs, query_cbs;
  sm::Pending pending;  // outputs of the current call, delivered once the lock is released
  sm::Pending bulk_spare;  // the Event arrays of bulk sends, kept for the next one
  bool failed = false;                      // a batch failed half-way: matching state is inconsistent
  std::string failed_why;
  // batch staging
  std::vector<int32_t> ev_stream;
  std::vector<int64_t> ev_row, ev_ts, ev_clock, ev_ord;
  int64_t next_ordinal = 0;
  std::vector<int64_t> adv_pos, adv_clock, adv_wall;
  int64_t ordinal_base = 0;
  int64_t clock = 0;          // playback clock (EventTimeBasedMillisTimestampGenerator.lastEventTimestamp)
  int64_t clock_batch_in = 0;
  bool started = false;
  bool shut = false;
  int64_t batch_events = 1 << 20;
  int32_t heap_half = 1024;
  int64_t pool_init = (int64_t)1 << 25;  // option "pool_words": first size of a query's overflow pool (words)
  // NFA lanes in descending event-count order for batches with at least this many keys (0 = off;
  // SM_NFA_BALANCE=<min keys> / option "lane_balance"). A wave runs as long as its busiest lane; a wave's lanes then
  // stage and write back 64 scattered keys' state words and timer queues (more HBM traffic per launch), which the
  // shorter waves outweigh: round 4, config 5 literal 17.85 -> 17.7 ms (step unchanged with the sort), emitting
  // variant 147.1 -> 140.6 ms.
  int64_t lane_balance = (int64_t)1 << 16;
  int64_t out_records = 0;  // option "output_records" (0 = automatic)
  bool keep_outputs = false;  // option "keep_outputs": device-events batches keep their ordered output records
  int nfa_jit = -1;         // option "nfa_jit": 1 = query-specialised NFA kernels (nfa_jit.cpp), 0 = the
                            // interpreter, -1 = automatic (batches of 2^20 query records or more)
  uint64_t text_hash = 0;   // FNV-1a of the SiddhiQL text (snapshots restore only into the same app)
  bool collect = false;
  std::map<std::string, std::vector<std::string>> collected_streams;  // JSON fragments
  std::map<std::string, std::vector<std::string>> collected_queries;
  // output record buffers of the current call (HostOut points into them): pinned host memory, reused across calls
  struct OutArena {
    std::vector<sm::PinnedBuf> bufs;
    size_t next = 0;  // buffers in use by the current call
    // the buffers in use go to a Pending in the views form (its callbacks read them after the app lock is released)
    void lend(std::vector<sm::PinnedBuf>& to) {
      for (size_t i = 0; i < next; ++i) to.push_back(bufs[i]);
      bufs.erase(bufs.begin(), bufs.begin() + (ptrdiff_t)next);
      next = 0;
    }
    void give_back(std::vector<sm::PinnedBuf>& from) {
      for (auto& b : from) bufs.push_back(b);
      from.clear();
    }
    char* take(size_t bytes) {
      if (next == bufs.size()) bufs.emplace_back();
      sm::PinnedBuf& b = bufs[next++];
      if (b.cap < bytes) {
        if (b.p) SM_HIP(hipHostFree(b.p));
        b.p = nullptr;
        b.cap = std::max(bytes, b.cap * 2);
        SM_HIP(hipHostMalloc((void**)&b.p, b.cap, hipHostMallocDefault));
      }
      return b.p;
    }
    void clear() { next = 0; }
    ~OutArena() {
      for (auto& b : bufs)
        if (b.p) (void)hipHostFree(b.p);
    }
  } out_arena;
  // completion events of the output segments of the current call (DevOut::seg_ev), reused across calls
  struct EvPool {
    std::vector<hipEvent_t> evs;
    size_t next = 0;
    hipEvent_t take() {
      if (next == evs.size()) {
        hipEvent_t e;
        SM_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        evs.push_back(e);
      }
      return evs[next++];
    }
    void clear() { next = 0; }
    ~EvPool() {
      for (auto e : evs) (void)hipEventDestroy(e);
    }
  } out_events;
  // no JSON dump, no callback, no chaining: outputs are counted and stay in device memory, no HostOut is built
  bool outputs_unconsumed() const;
  bool need_outs = false;  // set while a caller reads the output records itself (nfa_device_batch)
  bool in_device_events = false;  // inside sm_app_process_device_events (keep_outputs applies)
  hipStream_t stream = nullptr;
  int device = 0;  // the HIP device the app was created on (helper threads select it)
  // bulk columnar sends (bulk_send_device): minimum events for the direct path (option "bulk_min"), events per chunk
  // (option "bulk_chunk"), the upload stream and the two chunk buffers (attributes, then event times)
  int64_t bulk_min = (int64_t)1 << 16;
  int64_t bulk_chunk = (int64_t)1 << 24;
  hipStream_t copy_stream = nullptr;
  std::vector<sm::DBuf> bulk[2];
  bool bulk_active = false;  // a bulk send is in progress (a callback's own large send is staged instead)
  bool defer_outputs = false;  // device_outputs leaves its copies in flight (DevOut segments): bulk sends only
  // host-side time of the output path since the last reset (stat "host_ms:<phase>"): 0 device batches (including
  // 1), 1 device projections copied out as records, 2 deliver (ordering + Event preparation), 3 callbacks of bulk
  // sends, 4 bulk sends waiting for their next chunk's upload
  double host_ms[5] = {0, 0, 0, 0, 0};
  sm::DBuf d_ev_stream, d_ev_row, d_ev_ts, d_ev_clock, d_ev_ord, d_adv_pos, d_adv_clock, d_adv_wall, d_adv_upto, d_streams,
      d_err, d_count,
      d_keyoff, scratch, d_rp, d_rp_streams;
  sm::Scratch sc;
};

namespace sm {
namespace {

void set_error(const std::string& m) { g_err = m; }

int status_of(const std::exception& e) {
  if (dynamic_cast<const sql::ParseError*>(&e)) return SM_E_PARSE;
  if (dynamic_cast<const sql::ValidationError*>(&e)) return SM_E_VALIDATION;
  if (dynamic_cast<const sql::UnsupportedError*>(&e)) return SM_E_UNSUPPORTED;
  if (dynamic_cast<const TypeError*>(&e)) return SM_E_TYPE;
  std::string w = e.what();
  if (w.rfind("HIP error", 0) == 0) return SM_E_DEVICE;
  return SM_E_RUNTIME;
}

template <typename F>
int guarded(F&& f) {
  try {
    f();
    return SM_OK;
  } catch (const std::exception& e) {
    set_error(e.what());
    return status_of(e);
  }
}

void run_callbacks(Pending& out);
void give_back(sm_app* a, Pending& out);

// Entry points that can produce outputs: run f under the app lock, then the callbacks of what it produced
// without it.
template <typename F>
int locked(sm_app* a, F&& f) {
  Pending out;
  int rc;
  {
    std::lock_guard<std::mutex> g(a->mu);
    rc = guarded([&] {
      if (a->failed) throw std::runtime_error(a->failed_why);
      f();
    });
    out.swap(a->pending);
  }
  run_callbacks(out);
  give_back(a, out);
  return rc;
}

void ensure_scratch(sm_app* a, size_t bytes) {
  if (a->sc.cap < bytes || !a->sc.base) {
    a->scratch.ensure(bytes);
    a->sc.base = (char*)a->scratch.p;
    a->sc.cap = a->scratch.cap;
  }
  a->sc.used = 0;
}

void build_app(sm_app* a) {
  a->streams.resize(a->ast.streams.size());
  for (size_t i = 0; i < a->ast.streams.size(); ++i) {
    StreamStage& st = a->streams[i];
    st.def = &a->ast.streams[i];
    size_t na = st.def->attrs.size();
    if (na > (size_t)kMaxAttrs) throw sql::UnsupportedError("stream has too many attributes");
    st.cols.resize(na);
    st.nulls.resize(na);
    st.any_null.assign(na, false);
    st.dcols.resize(na);
    st.dnulls.resize(na);
  }
  for (size_t pi = 0; pi < a->ast.partitions.size(); ++pi) {
    a->parts.push_back(compile_partition(a->ast, a->ast.partitions[pi], a->dict));
    // inner streams ('#name') of the partition carry their instance's key code in one extra LONG column, which
    // is their key program (PartitionRuntime routes them by the junction of stream id + key)
    for (size_t si = 0; si < a->ast.streams.size(); ++si) {
      const sql::StreamDef& d = a->ast.streams[si];
      if (d.id[0] != '#' || d.partition != (int)pi) continue;
      const int hidden = (int)d.attrs.size();
      if (hidden + 1 > kMaxAttrs) throw sql::UnsupportedError("inner stream has too many attributes");
      Instr in{};
      in.op = OP_COL;
      in.a = hidden;
      in.t0 = T_LONG;
      a->parts.back().streams.push_back((int)si);
      a->parts.back().key_code.push_back({in});
      a->parts.back().key_consts.push_back({});
      a->parts.back().key_type.push_back(T_LONG);
      StreamStage& st = a->streams[si];
      st.cols.resize(hidden + 1);
      st.nulls.resize(hidden + 1);
      st.any_null.assign(hidden + 1, false);
      st.dcols.resize(hidden + 1);
      st.dnulls.resize(hidden + 1);
    }
  }
  // query chaining: a query reading a stream other queries insert into runs one level after them, over the
  // input events merged with theirs (flush)
  std::vector<std::vector<int>> producers(a->ast.streams.size());
  a->stream_fed.assign(a->ast.streams.size(), 0);
  a->part_bcast.assign(a->ast.partitions.size(), {});
  a->part_keys.assign(a->ast.partitions.size(), {});
  a->part_key_types.assign(a->ast.partitions.size(), {});
  a->part_key_set.assign(a->ast.partitions.size(), {});
  a->part_bcast_group.assign(a->ast.partitions.size(), {});
  for (size_t o = 0; o < a->ast.order.size(); ++o) {
    auto [pi, qi] = a->ast.order[o];
    const sql::Query& qd = pi < 0 ? a->ast.queries[qi] : a->ast.partitions[pi].queries[qi];
    auto q = std::make_unique<QueryRt>();
    q->cq = compile_query(a->ast, qd, (int)o, pi, a->dict);
    if (pi >= 0) {
      q->part = &a->parts[pi];
      q->pidx = pi;
      CompiledPartition& cpm = a->parts[pi];
      for (int s : q->cq.streams)
        if (std::find(cpm.streams.begin(), cpm.streams.end(), s) == cpm.streams.end() ||
            std::find(a->part_bcast[pi].begin(), a->part_bcast[pi].end(), s) != a->part_bcast[pi].end()) {
          // a stream the partition does not key: every instance receives it (PartitionStreamReceiver :271-275).
          // The flush hands such a query one copy of each of these events per existing instance, carrying the
          // instance's key code in an extra column (the stream's key program here); instances are tracked on the
          // host, so the partition's keys must be columns
          if (q->cq.hdr.kind == 0)
            throw sql::UnsupportedError("a single-stream query inside a partition must read a keyed stream");
          for (size_t k = 0; k < cpm.key_code.size(); ++k)
            if (cpm.key_code[k].size() != 1 || cpm.key_code[k][0].op != OP_COL)
              throw sql::UnsupportedError("a partition whose queries read an unkeyed stream needs columns as keys");
          // The instances receive the event in the iteration order of a map keyed by streamId + String.valueOf(key)
          // (java_order.h). For an INT / LONG / STRING / BOOL key that string is exact; for FLOAT / DOUBLE it is
          // Java 8's Double.toString / Float.toString (sun.misc.FloatingDecimal), which is not always the shortest
          // round-trip digit string java_order.cpp writes, and no JVM here pins where they differ:
          // such an app is refused rather than given an order that cannot be pinned.
          for (int32_t kt : cpm.key_type)
            if (kt == T_FLOAT || kt == T_DOUBLE)
              throw sql::UnsupportedError(
                  "a partition keyed by a float / double attribute whose queries read an unkeyed stream (broadcast "
                  "order over Double.toString keys is not supported)");
          q->bcast = true;
          if (!a->part_bcast_group[pi].count(s)) a->part_bcast_group[pi][s] = q->cq.hdr.query_order;
          if (std::find(a->part_bcast[pi].begin(), a->part_bcast[pi].end(), s) == a->part_bcast[pi].end()) {
            Instr in{};
            in.op = OP_COL;
            in.a = (int)a->ast.streams[s].attrs.size();
            in.t0 = T_LONG;
            if (in.a + 1 > kMaxAttrs) throw sql::UnsupportedError("stream has too many attributes");
            cpm.streams.push_back(s);
            cpm.key_code.push_back({in});
            cpm.key_consts.push_back({});
            cpm.key_type.push_back(T_LONG);
            a->part_bcast[pi].push_back(s);
          }
        }
      if (q->cq.hdr.kind == 0) {
        // a filter inside a partition: the same rows as outside, minus those whose key is null (A17); the key is
        // read on the host, so it must be a column of the stream
        const CompiledPartition& cp = *q->part;
        const int k = (int)(std::find(cp.streams.begin(), cp.streams.end(), q->cq.hdr.stream) - cp.streams.begin());
        if (cp.key_code[k].size() != 1 || cp.key_code[k][0].op != OP_COL)
          throw sql::UnsupportedError("a single-stream query inside a partition needs a column as the key");
      }
    }
    const int out = sm::stream_index(a->ast, qd.insert_into);
    if (out >= 0) producers[out].push_back((int)a->queries.size());
    a->queries.push_back(std::move(q));
  }
  // Chaining levels by the producer / consumer relation (InsertIntoStreamCallback → StreamJunction.sendEvent →
  // the queries reading that stream), whether the stream was declared with `define stream` or named only by
  // `insert into`. The level merge (run_chained) places an inserted event before its root input event, which is
  // the reference's order when every reader of the stream was defined after its producers (the producer then sits
  // earlier on the root stream's junction); a reader defined before a producer of its stream is refused rather than
  // given another order.
  for (size_t qi = 0; qi < a->queries.size(); ++qi) {
    QueryRt& q = *a->queries[qi];
    for (int s : q.cq.streams) {
      if (producers[s].empty()) continue;
      a->stream_fed[s] = 1;
      for (int pq : producers[s]) {
        if (pq >= (int)qi)
          throw sql::UnsupportedError("query '" + q.cq.name + "' reads stream '" + a->ast.streams[s].id +
                                      "', which query '" + a->queries[pq]->cq.name +
                                      "' defined at or after it inserts into");
        q.level = std::max(q.level, a->queries[pq]->level + 1);
      }
    }
    a->max_level = std::max(a->max_level, q.level);
  }
  // an output must fit the stream it goes into (DefinitionParserHelper.validateOutputStream): checked for the streams
  // the parser defined from `insert into` and for every stream another query reads
  for (size_t s = 0; s < producers.size(); ++s) {
    if (!a->ast.streams[s].implicit && !a->stream_fed[s]) continue;
    const auto& at = a->ast.streams[s].attrs;
    for (int pq : producers[s]) {
      const CompiledQuery& cq = a->queries[pq]->cq;
      bool same = at.size() == cq.sel_types.size();
      for (size_t k = 0; same && k < at.size(); ++k) same = (int)at[k].type == cq.sel_types[k];
      if (!same) throw sql::ValidationError("query '" + cq.name + "' output does not match stream '" + a->ast.streams[s].id + "'");
    }
  }
}

void upload_app(sm_app* a) {
  SM_HIP(hipGetDevice(&a->device));
  SM_HIP(hipStreamCreateWithFlags(&a->stream, hipStreamNonBlocking));
  for (auto& q : a->queries) {
    q->blob.ensure(q->cq.blob.size());
    SM_HIP(hipMemcpyAsync(q->blob.p, q->cq.blob.data(), q->cq.blob.size(), hipMemcpyHostToDevice, a->stream));
    if (q->part) {
      // key programs of the partition's streams
      const CompiledPartition& cp = *q->part;
      std::vector<KeyProg> kps(cp.streams.size());
      q->keycode.resize(cp.streams.size() * 2);
      for (size_t k = 0; k < cp.streams.size(); ++k) {
        size_t cb = std::max<size_t>(cp.key_code[k].size() * sizeof(Instr), 16);
        size_t kb = std::max<size_t>(cp.key_consts[k].size() * sizeof(DVal), 16);
        q->keycode[2 * k].ensure(cb);
        q->keycode[2 * k + 1].ensure(kb);
        if (!cp.key_code[k].empty())
          SM_HIP(hipMemcpyAsync(q->keycode[2 * k].p, cp.key_code[k].data(), cp.key_code[k].size() * sizeof(Instr),
                                hipMemcpyHostToDevice, a->stream));
        if (!cp.key_consts[k].empty())
          SM_HIP(hipMemcpyAsync(q->keycode[2 * k + 1].p, cp.key_consts[k].data(),
                                cp.key_consts[k].size() * sizeof(DVal), hipMemcpyHostToDevice, a->stream));
        kps[k].stream = cp.streams[k];
        kps[k].len = (int)cp.key_code[k].size();
        kps[k].type = cp.key_type[k];
        kps[k].code = (const Instr*)q->keycode[2 * k].p;
        kps[k].consts = (const DVal*)q->keycode[2 * k + 1].p;
      }
      q->keyprogs.ensure(kps.size() * sizeof(KeyProg));
      SM_HIP(hipMemcpyAsync(q->keyprogs.p, kps.data(), kps.size() * sizeof(KeyProg), hipMemcpyHostToDevice, a->stream));
      q->nkeyprogs = (int)kps.size();
      q->keys.reserve(1, a->stream);
    }
  }
  SM_HIP(hipStreamSynchronize(a->stream));
}

// ---- JSON (parity dump) in the same shape as the oracle's
void json_val(std::ostringstream& o, const sm_app* a, const DVal& v, int t) {
  if (v.null) {
    o << "null";
    return;
  }
  switch (t) {
    case T_INT:
    case T_LONG: o << v.i; break;
    case T_BOOL: o << (v.i ? "true" : "false"); break;
    case T_FLOAT:
    case T_DOUBLE: {
      if (std::isnan(v.d)) { o << "\"NaN\""; break; }
      if (std::isinf(v.d)) { o << (v.d > 0 ? "\"Infinity\"" : "\"-Infinity\""); break; }
      char b[64];
      auto r = std::to_chars(b, b + 64, v.d);
      std::string s(b, r.ptr);
      if (s.find_first_of(".eE") == std::string::npos) s += ".0";
      o << s;
      break;
    }
    default: {
      if (v.i < 0 || v.i >= (int64_t)a->dict.strs.size()) {
        o << "null";
        break;
      }
      o << '"';
      for (char c : a->dict.strs[v.i]) {
        if (c == '"' || c == '\\') o << '\\' << c;
        else if ((unsigned char)c < 0x20) {
          char b[8];
          snprintf(b, 8, "\\u%04x", c);
          o << b;
        } else o << c;
      }
      o << '"';
    }
  }
}

// Host threads for the output path: the process's CPU share (OMP_NUM_THREADS where the launcher sets it, e.g. 16 on
// the GPU box, whose nproc shows the whole machine), at most 16.
int host_threads() {
  static const int t = [] {
    int n = (int)std::thread::hardware_concurrency();
    if (const char* e = getenv("OMP_NUM_THREADS")) n = std::min(n > 0 ? n : 1 << 30, std::max(1, atoi(e)));
    return std::max(1, std::min(n, 16));
  }();
  return t;
}

// f(lo, hi) over [0, n) on up to host_threads() threads, at least `grain` items each.
template <typename F>
void parallel_for(size_t n, size_t grain, F&& f) {
  const size_t t = std::min<size_t>((size_t)host_threads(), std::max<size_t>(n / std::max<size_t>(grain, 1), 1));
  if (t <= 1) {
    f((size_t)0, n);
    return;
  }
  // an exception in a worker (a failed HIP call while it waits for an output segment) is rethrown on the calling
  // thread after every worker has joined, so the entry point reports it instead of the process terminating
  std::vector<std::exception_ptr> err(t);
  std::vector<std::thread> th;
  th.reserve(t - 1);
  for (size_t w = 1; w < t; ++w)
    th.emplace_back([&, w] {
      try {
        f(n * w / t, n * (w + 1) / t);
      } catch (...) {
        err[w] = std::current_exception();
      }
    });
  try {
    f((size_t)0, n / t);
  } catch (...) {
    err[0] = std::current_exception();
  }
  for (auto& x : th) x.join();
  for (auto& e : err)
    if (e) std::rethrow_exception(e);
}

void to_sm_values(const sm_app* a, const DVal* vals, int nvals, const CompiledQuery& cq, sm_value* out) {
  for (int k = 0; k < nvals; ++k) {
    sm_value& v = out[k];
    int t = cq.sel_types[k];
    v.type = t;
    v.is_null = vals[k].null;
    v.i = 0;
    v.d = 0;
    v.s = nullptr;
    if (v.is_null) continue;
    if (t == T_FLOAT || t == T_DOUBLE) v.d = vals[k].d;
    else if (t == T_STRING) {
      int64_t id = vals[k].i;
      if (id < 0 || id >= (int64_t)a->dict.strs.size()) v.is_null = 1;
      else v.s = a->dict.strs[id].c_str();
    } else v.i = vals[k].i;
  }
}

// the same from the compact device form: raw 64-bit words and a byte of null flags (bit k: value k)
void to_sm_values_compact(const sm_app* a, const int64_t* w, uint8_t nulls, int nvals, const CompiledQuery& cq,
                          sm_value* out) {
  for (int k = 0; k < nvals; ++k) {
    sm_value& v = out[k];
    const int t = cq.sel_types[k];
    v.type = t;
    v.is_null = (nulls >> k) & 1;
    v.i = 0;
    v.d = 0;
    v.s = nullptr;
    if (v.is_null) continue;
    if (t == T_FLOAT || t == T_DOUBLE) memcpy(&v.d, &w[k], 8);
    else if (t == T_STRING) {
      const int64_t id = w[k];
      if (id < 0 || id >= (int64_t)a->dict.strs.size()) v.is_null = 1;
      else v.s = a->dict.strs[id].c_str();
    } else v.i = w[k];
  }
}

// Outputs in the reference's emission order (trigger position, timer phase, listener order, query order,
// emission order), grouped into one chunk per (trigger, emitting query instance): the collect dump is appended
// here, the callbacks run later (run_callbacks) outside the app lock.
}  // namespace
}  // namespace sm

bool sm_app::outputs_unconsumed() const {
  if (collect || need_outs || max_level > 0) return false;
  for (auto& q : queries) {
    auto it = stream_cbs.find(q->cq.insert_into);
    if (it != stream_cbs.end() && !it->second.empty()) return false;
    auto qt = query_cbs.find(q->cq.name);
    if (q->cq.partition < 0 && qt != query_cbs.end() && !qt->second.empty()) return false;
  }
  return true;
}

namespace sm {
namespace {

bool out_before(const OutRec& x, const OutRec& y) {
  if (x.pos != y.pos) return x.pos < y.pos;
  if (x.phase != y.phase) return x.phase < y.phase;
  if (x.phase == 0) {
    if (x.time != y.time) return x.time < y.time;
    int gx = x.create >= 0, gy = y.create >= 0;  // non-partitioned listeners registered first
    if (gx != gy) return gx < gy;
    if (x.create != y.create) return x.create < y.create;
    if (x.query != y.query) return x.query < y.query;
    return x.sched < y.sched;
  }
  // data phase: the trigger's junction receivers in subscription order (query order); a partition receiver hands a
  // broadcast event to its instances one after another (time = the instance's rank in the receiver's
  // ConcurrentHashMap iteration + 1, sched = the receiver's place), each instance's queries in query order
  const int32_t gx = x.time ? x.sched : x.query, gy = y.time ? y.sched : y.query;
  if (gx != gy) return gx < gy;
  if (x.time != y.time) return x.time < y.time;
  return x.query < y.query;
}

// The callbacks one output chunk of query cq goes to, in the reference's order: OutputRateLimiter.sendToCallBacks
// (core/query/output/ratelimit/OutputRateLimiter.java:61-73) calls the query's QueryCallbacks first, then hands the
// chunk to the output stream's junction, whose StreamCallbacks receive it. Returns {first index in pd.cbs, number of
// QueryCallbacks, number of callbacks}.
std::array<int64_t, 3> query_callbacks(sm_app* a, const CompiledQuery& cq) {
  Pending& pd = a->pending;
  std::array<int64_t, 3> at{(int64_t)pd.cbs.size(), 0, 0};
  if (cq.partition < 0) {  // partition clones do not inherit QueryCallbacks (PartitionRuntime)
    auto qt = a->query_cbs.find(cq.name);
    if (qt != a->query_cbs.end())
      for (auto& cb : qt->second)
        if (cb.qcb) pd.cbs.push_back(cb);
  }
  at[1] = (int64_t)pd.cbs.size() - at[0];
  auto it = a->stream_cbs.find(cq.insert_into);
  if (it != a->stream_cbs.end())
    for (auto& cb : it->second)
      if (cb.scb || cb.ccb) pd.cbs.push_back(cb);
  at[2] = (int64_t)pd.cbs.size() - at[0];
  return at;
}

void deliver(sm_app* a, std::vector<HostOut>& outs) {
  if (a->outputs_unconsumed()) {  // nothing to hand out: the outputs were only counted
    a->out_arena.clear();
    return;
  }
  const auto t0 = std::chrono::steady_clock::now();
  struct Tm {
    sm_app* a;
    std::chrono::steady_clock::time_point t0;
    ~Tm() { a->host_ms[2] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); }
  } tm{a, t0};
  auto key_less = [](const OutRec& x, const OutRec& y) { return out_before(x, y); };
  const auto before = [&](const HostOut& x, const HostOut& y) {
    if (key_less(x.r, y.r)) return true;
    if (key_less(y.r, x.r)) return false;
    return x.r.seq < y.r.seq;
  };
  // the device orders one query's records already (order_outputs); several queries' outputs still interleave here
  if (!std::is_sorted(outs.begin(), outs.end(), before)) std::stable_sort(outs.begin(), outs.end(), before);
  std::vector<std::array<int64_t, 3>> qcb(a->queries.size(), std::array<int64_t, 3>{-1, 0, 0});
  // pass 1 (in order): chunks, the collect dump, and each output's place in the Event arrays; pass 2 (threads): the
  // Events themselves
  Pending& pd = a->pending;
  std::vector<int64_t> voff(outs.size(), -1), eoff(outs.size(), -1);
  size_t nvals = pd.vals.size(), nevs = pd.evs.size();
  bool strings = false;
  size_t i = 0;
  while (i < outs.size()) {
    size_t j = i + 1;  // the chunk: same trigger and emitting query instance
    while (j < outs.size() && outs[j].qidx == outs[i].qidx && !key_less(outs[i].r, outs[j].r) &&
           !key_less(outs[j].r, outs[i].r))
      ++j;
    const CompiledQuery& cq = a->queries[outs[i].qidx]->cq;
    // this query's callbacks, appended to pd.cbs once per deliver()
    auto& at = qcb[outs[i].qidx];
    if (at[0] < 0) at = query_callbacks(a, cq);
    const size_t nsel = cq.sel_types.size();
    PreparedChunk ch;
    ch.ts = outs[j - 1].r.ts;  // QueryCallback.receiveStreamEvent: the chunk's last event's timestamp
    ch.cb_off = (uint32_t)at[0];
    ch.n_cbs = (uint32_t)at[2];
    ch.n_query_cbs = (uint32_t)at[1];
    ch.ev_off = nevs;
    ch.n_ev = j - i;
    if (ch.n_cbs)
      for (int t : cq.sel_types) strings |= t == T_STRING;
    for (size_t k = i; k < j; ++k) {
      HostOut& h = outs[k];
      if (a->collect) {
        std::ostringstream o;
        o << "[" << h.r.ts << ",[";
        for (int q = 0; q < h.nvals; ++q) {
          if (q) o << ",";
          json_val(o, a, h.vals[q], cq.sel_types[q]);
        }
        o << "],[";
        for (int q = 0; q < h.nrefs; ++q) {
          if (q) o << ",";
          o << h.refs[q];
        }
        o << "]]";
        a->collected_streams[cq.insert_into].push_back(o.str());
        if (cq.partition < 0) {
          std::ostringstream qo;
          qo << "[" << h.r.ts << ",[[";
          for (int q = 0; q < h.nvals; ++q) {
            if (q) qo << ",";
            json_val(qo, a, h.vals[q], cq.sel_types[q]);
          }
          qo << "]]]";
          a->collected_queries[cq.name].push_back(qo.str());
        }
      }
      if (ch.n_cbs == 0) continue;
      voff[k] = (int64_t)nvals;
      eoff[k] = (int64_t)nevs++;
      nvals += nsel;
    }
    if (ch.n_cbs) {
      pd.expand();
      pd.chunks.push_back(ch);
    }
    i = j;
  }
  pd.vals.resize(nvals);
  pd.evs.resize(nevs);
  parallel_for(outs.size(), (size_t)1 << 16, [&](size_t lo, size_t hi) {
    for (size_t k = lo; k < hi; ++k) {
      if (eoff[k] < 0) continue;
      const HostOut& h = outs[k];
      to_sm_values(a, h.vals, h.nvals, a->queries[h.qidx]->cq, pd.vals.data() + voff[k]);
      pd.evs[eoff[k]] = sm_event{h.r.ts, (const sm_value*)(uintptr_t)voff[k], (int32_t)h.nvals};
    }
  });
  if (strings)  // STRING values are owned by the pending outputs (the dictionary may change before the callbacks)
    for (size_t k = 0; k < outs.size(); ++k)
      for (int q = 0; eoff[k] >= 0 && q < outs[k].nvals; ++q) {
        sm_value& v = pd.vals[voff[k] + q];
        if (v.type == T_STRING && !v.is_null) {
          pd.strs.push_back(std::make_unique<std::string>(v.s));
          v.s = pd.strs.back()->c_str();
        }
      }
  a->out_arena.clear();  // the chunks own copies of everything they hand out
}

// Callbacks of the prepared chunks, on the calling thread, with the app lock released: a callback may send into
// the same app (its outputs are delivered inside that send, as in the reference). Reference behaviour for a
// callback that throws (caught and logged, StreamCallback.java:92-99) is the binding's business: C callbacks
// cannot throw across the ABI.
// A columns StreamCallback on a chunk of Events (the forms other than the views): the chunk's columns built for the call
void call_columns(const Callback& cb, const sm_event* evs, size_t n) {
  const int32_t ns = n ? evs[0].n : 0;
  std::vector<int64_t> ts(n), w((size_t)n * ns);
  std::vector<uint8_t> nb(n, 0);
  for (size_t k = 0; k < n; ++k) {
    ts[k] = evs[k].timestamp;
    for (int j = 0; j < ns; ++j) {
      const sm_value& v = evs[k].data[j];
      if (v.is_null) nb[k] |= (uint8_t)(1u << j);
      if (v.type == T_FLOAT || v.type == T_DOUBLE) memcpy(&w[k * ns + j], &v.d, 8);
      else w[k * ns + j] = v.is_null ? 0 : v.i;
    }
  }
  cb.ccb(cb.user, n, ts.data(), w.data(), nb.data(), ns);
}

// the pinned buffers a views-form Pending held go back to the app's output arena
void give_back(sm_app* a, Pending& out) {
  if (out.owned.empty()) return;
  out.wait_segments();  // no copy into the buffers is still in flight
  std::lock_guard<std::mutex> g(a->mu);
  a->out_arena.give_back(out.owned);
}

void run_callbacks(Pending& out) {
  if (out.chunks.empty() && !(out.uniform && !out.starts.empty())) return;
  if (out.views) {  // every callback takes columns: views of the outputs, chunk by chunk (Pending::views)
    const PreparedChunk& p = out.proto;
    const size_t n = out.starts.size(), ne = out.cn;
    const uint64_t* st = out.starts.data();
    const int32_t ns = out.cns;
    size_t ready = out.seg_end.empty() ? ne : 0, seg = 0;
    for (size_t k = 0; k < n; ++k) {
      const size_t b = st[k], e = k + 1 < n ? st[k + 1] : ne;
      while (e > ready) {  // the chunk's outputs are on the host once their segments' copies have completed
        SM_HIP(hipEventSynchronize(out.seg_ev[seg]));
        ready = (size_t)out.seg_end[seg++];
      }
      for (uint32_t c = 0; c < p.n_cbs; ++c) {
        const Callback& cb = out.cbs[p.cb_off + c];
        cb.ccb(cb.user, e - b, out.cts + b, out.cvals + b * ns, out.cnul + b, ns);
      }
    }
    return;
  }
  if (!out.final_) {  // Pending::finalise on the host threads
    sm_value* vals = out.vals.data();
    sm_event* evs = out.evs.data();
    parallel_for(out.evs.size(), (size_t)1 << 16, [&](size_t lo, size_t hi) {
      for (size_t k = lo; k < hi; ++k) evs[k].data = vals + (uintptr_t)evs[k].data;
    });
    out.final_ = true;
  }
  if (out.uniform) {
    const PreparedChunk& p = out.proto;
    const size_t n = out.starts.size(), ne = out.evs.size();
    const uint64_t* st = out.starts.data();
    const sm_event* ev0 = out.evs.data();
    if (p.n_cbs == 1 && p.n_query_cbs == 0 && !out.cbs[p.cb_off].ccb) {  // one StreamCallback: no per-chunk dispatch
      const Callback& cb = out.cbs[p.cb_off];
      const sm_stream_callback f = cb.scb;
      void* const u = cb.user;
      for (size_t k = 0; k < n; ++k) {
        const size_t b = st[k], e = k + 1 < n ? st[k + 1] : ne;
        f(u, ev0 + b, e - b);
      }
      return;
    }
    for (size_t k = 0; k < n; ++k) {
      const size_t b = st[k], e = k + 1 < n ? st[k + 1] : ne;
      for (uint32_t c = 0; c < p.n_cbs; ++c) {
        const Callback& cb = out.cbs[p.cb_off + c];
        if (c < p.n_query_cbs) cb.qcb(cb.user, ev0[e - 1].timestamp, ev0 + b, e - b, nullptr, 0);
        else if (cb.ccb) call_columns(cb, ev0 + b, e - b);
        else cb.scb(cb.user, ev0 + b, e - b);
      }
    }
    return;
  }
  for (auto& ch : out.chunks) {
    const sm_event* evs = out.evs.data() + ch.ev_off;
    for (uint32_t c = 0; c < ch.n_cbs; ++c) {
      const Callback& cb = out.cbs[ch.cb_off + c];
      if (c < ch.n_query_cbs) cb.qcb(cb.user, ch.ts, evs, ch.n_ev, nullptr, 0);
      else if (cb.ccb) call_columns(cb, evs, ch.n_ev);
      else cb.scb(cb.user, evs, ch.n_ev);
    }
  }
}

void read_outputs(sm_app* a, int qidx, const void* dev, int64_t n, std::vector<HostOut>& outs) {
  if (n <= 0) return;
  a->queries[qidx]->n_out += n;
  // no callback, no dump, no chaining: the records stay in device memory (sm_app_copy_device_outputs), counted
  if (a->outputs_unconsumed()) return;
  const CompiledQuery& cq = a->queries[qidx]->cq;
  size_t stride = sizeof(OutRec) + cq.hdr.nsel * sizeof(DVal) + cq.hdr.nrefs * sizeof(int64_t);
  char* host = a->out_arena.take((size_t)n * stride);
  SM_HIP(hipMemcpyAsync(host, dev, (size_t)n * stride, hipMemcpyDeviceToHost, a->stream));
  SM_HIP(hipStreamSynchronize(a->stream));
  outs.reserve(outs.size() + (size_t)n);
  for (int64_t k = 0; k < n; ++k) {
    const char* b = host + (size_t)k * stride;
    HostOut h;
    memcpy(&h.r, b, sizeof(OutRec));
    h.vals = (const DVal*)(b + sizeof(OutRec));
    h.nvals = cq.hdr.nsel;
    const int64_t* rf = (const int64_t*)(b + sizeof(OutRec) + cq.hdr.nsel * sizeof(DVal));
    h.refs = rf;
    h.nrefs = cq.hdr.nrefs_vis;
    if (cq.hdr.nrefs == cq.hdr.nrefs_vis + 2) {
      h.e1 = rf[cq.hdr.nrefs_vis];
      h.e2 = rf[cq.hdr.nrefs_vis + 1];
    }
    h.qidx = qidx;
    outs.push_back(h);
  }
}

void ensure_state(sm_app* a, QueryRt& q, int64_t nkeys) {
  if (nkeys <= q.state_slots) return;
  int64_t cap = std::max<int64_t>(nkeys, q.state_slots * 2);
  cap = std::max<int64_t>(cap, 16);
  const DQuery& h = q.cq.hdr;
  size_t ks_bytes = (size_t)cap * h.ks_words * 8;
  size_t heap_words = 2 * (size_t)a->heap_half + 64;
  size_t heap_bytes = (size_t)cap * heap_words * 8;
  void *nks = nullptr, *nheap = nullptr;
  SM_HIP(hipMalloc(&nks, ks_bytes));
  SM_HIP(hipMalloc(&nheap, heap_bytes));
  SM_HIP(hipMemsetAsync(nks, 0, ks_bytes, a->stream));
  if (q.state_slots > 0) {  // ks: lane-interleaved rows (word-major, one column per key), re-pitched; heap: key-major
    SM_HIP(hipMemcpy2DAsync(nks, (size_t)cap * 8, q.ks.p, (size_t)q.state_slots * 8, (size_t)q.state_slots * 8,
                            (size_t)h.ks_words, hipMemcpyDeviceToDevice, a->stream));
    SM_HIP(hipMemcpyAsync(nheap, q.heap.p, (size_t)q.state_slots * heap_words * 8, hipMemcpyDeviceToDevice, a->stream));
  }
  SM_HIP(hipStreamSynchronize(a->stream));
  q.ks.release();
  q.heap.release();
  q.ks.p = nks;
  q.ks.cap = ks_bytes;
  q.heap.p = nheap;
  q.heap.cap = heap_bytes;
  q.state_slots = cap;
}

// The query's overflow pool holds at least `words` words, the first `keep` of them preserved (a promoted key's heap
// is addressed by its pool offset, so growing copies the used prefix into the larger buffer).
void ensure_pool(sm_app* a, QueryRt& q, int64_t words, int64_t keep) {
  if (!q.pool_top_dev.p) {  // {words handed out, largest failed request of the batch}
    q.pool_top_dev.ensure(16);
    SM_HIP(hipMemsetAsync(q.pool_top_dev.p, 0, 16, a->stream));
  }
  if (words <= q.pool_words) return;
  void* np = nullptr;
  SM_HIP(hipMalloc(&np, (size_t)words * 8));
  keep = std::min(keep, q.pool_words);
  if (keep > 0) SM_HIP(hipMemcpyAsync(np, q.pool.p, (size_t)keep * 8, hipMemcpyDeviceToDevice, a->stream));
  SM_HIP(hipStreamSynchronize(a->stream));
  q.pool.release();
  q.pool.p = np;
  q.pool.cap = (size_t)words * 8;
  q.pool_words = words;
}

template <typename T>
void upload(sm_app* a, DBuf& d, const std::vector<T>& v) {
  d.ensure(std::max<size_t>(v.size() * sizeof(T), 16));
  if (!v.empty()) SM_HIP(hipMemcpyAsync(d.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, a->stream));
}

// Stream count the lane-events and key-lookup kernels are told (they copy at most kLdsStreams descriptors into LDS;
// A/B: SM_LDS_STREAMS=0 passes "too many", so they read the descriptors from device memory). Measured on config 5
// (5 streams): grouping 7.0 -> 6.8 ms, lane events 6.8 -> 6.5 ms.
int lds_stream_count(int nstreams) {
  static const char* e = getenv("SM_LDS_STREAMS");
  return (e && e[0] == '0') ? (1 << 30) : nstreams;
}

// Device-side view of one batch in arrival order (uploaded by flush, or built on the device by
// sm_app_process_device_events).
struct EvArrays {
  const int32_t* ev_stream;
  const int64_t* ev_row;
  const int64_t* ev_ts;
  const int64_t* ev_clock;
  const int64_t* ev_ord;
  const NfaStream* streams;
  const int64_t* adv_pos;
  const int64_t* adv_clock;
  const int64_t* adv_wall;
  const int64_t* adv_upto;  // per position: advance points at positions <= it
  int64_t nadv;
  int64_t clock_in;
};

// Reclaim the overflow pool at a batch boundary: Lane::promote claims a fresh region whenever a key
// outgrows its current heap and abandons the old one, so a pool that only grew would keep every region a key ever
// used. Every promoted key's live objects move to a new pool region sized for them, or back to the key's own arena
// when they fit a quarter of it (nfa_pool_lane, two passes); the old pool is then entirely dead and freed.
void compact_pool(sm_app* a, QueryRt& q, int64_t nkeys, hipStream_t hs) {
  if (!q.pool.p || q.pool_used == 0 || nkeys <= 0) return;
  DBuf off, top;
  off.ensure((size_t)nkeys * 8);
  top.ensure(8);
  SM_HIP(hipMemsetAsync(top.p, 0, 8, hs));
  launch_pool_compact(0, (const char*)q.blob.p, (int64_t*)q.ks.p, (int64_t*)q.heap.p, a->heap_half, q.state_slots,
                      (int32_t)nkeys, (int64_t*)q.pool.p, nullptr, (unsigned long long*)top.p, (int64_t*)off.p, hs);
  uint64_t need = 0;
  SM_HIP(hipMemcpyAsync(&need, top.p, 8, hipMemcpyDeviceToHost, hs));
  SM_HIP(hipStreamSynchronize(hs));
  const int64_t words = std::max<int64_t>(2 * (int64_t)need + 4096, (int64_t)1 << 16);
  void* np = nullptr;
  SM_HIP(hipMalloc(&np, (size_t)words * 8));
  launch_pool_compact(1, (const char*)q.blob.p, (int64_t*)q.ks.p, (int64_t*)q.heap.p, a->heap_half, q.state_slots,
                      (int32_t)nkeys, (int64_t*)q.pool.p, (int64_t*)np, nullptr, (int64_t*)off.p, hs);
  SM_HIP(hipGetLastError());
  SM_HIP(hipMemcpyAsync(q.pool_top_dev.p, &need, 8, hipMemcpyHostToDevice, hs));
  SM_HIP(hipStreamSynchronize(hs));
  q.pool.release();
  q.pool.p = np;
  q.pool.cap = (size_t)words * 8;
  q.pool_words = words;
  q.pool_used = need;
  ++q.pool_compactions;
}

// One pattern / sequence query over a batch: select its streams' records, group them by partition key, run the
// NFA kernel (one lane per key) and read its output records back for ordered delivery.
void run_pattern_query(sm_app* a, int qi, const EvArrays& ev, int64_t N, std::vector<HostOut>& outs, hipStream_t hs,
                       FastTimings* tm = nullptr) {
  QueryRt& q = *a->queries[qi];
  const DQuery& h = q.cq.hdr;
  size_t stride = sizeof(OutRec) + h.nsel * sizeof(DVal) + h.nrefs * sizeof(int64_t);
  uint64_t mask = 0;
  for (int s : q.cq.streams) mask |= (1ull << s);
  bool partitioned = h.partitioned;
  int64_t* pos = (int64_t*)a->sc.take(N * 8);
  int64_t nq = select_records(ev.ev_stream, N, mask, !partitioned, pos, a->sc, hs);
  if (tm) tm->mark("nfa_select", hs);
  int64_t* key_pos = pos;
  int64_t* key_off = nullptr;
  int64_t nkeys = 1;
  if (partitioned) {
    int64_t nv = group_by_key(q.keys, pos, nq, ev.ev_stream, ev.ev_row, lds_stream_count((int)a->streams.size()),
                              ev.streams, (const KeyProg*)q.keyprogs.p, q.nkeyprogs, &key_pos,
                              &key_off, a->sc, hs, nq == N /* select_records kept every position: pos[i] = i */);
    nq = nv;
    nkeys = q.keys.nslots;
  } else {
    key_off = (int64_t*)a->sc.take(16);
    int64_t ho[2] = {0, nq};
    SM_HIP(hipMemcpyAsync(key_off, ho, 16, hipMemcpyHostToDevice, hs));
  }
  if (tm) tm->mark("nfa_group", hs);
  if (nkeys == 0) return;
  ensure_state(a, q, nkeys);
  // output record capacity: option "output_records", else 8 per record (capped at 2^26 records); overflow
  // is detected by the kernel and reported as an error naming the option
  int64_t cap = a->out_records > 0 ? a->out_records : std::min<int64_t>(std::max<int64_t>(4096, 8 * nq + 1024), 1 << 26);
  q.out.ensure((size_t)cap * stride);
  NfaBatch b{};
  b.ev_stream = ev.ev_stream;
  b.ev_row = ev.ev_row;
  b.ev_ts = ev.ev_ts;
  b.ev_clock = ev.ev_clock;
  b.ev_ord = ev.ev_ord;
  b.streams = ev.streams;
  b.adv_pos = ev.adv_pos;
  b.adv_clock = ev.adv_clock;
  b.adv_wall = ev.adv_wall;
  b.adv_upto = ev.adv_upto;
  b.nadv = ev.nadv;
  b.clock_in = ev.clock_in;
  if (h.nsched > 0 && ev.nadv > 0 && ev.nadv < INT32_MAX) {
    // timers: the clock index of the advance points (timer_fire finds a timer's due point with one load instead of a
    // gallop), for a clock span of at most 2^26 values (256 MB of int32); wider spans keep the gallop. The span's two
    // ends are read back here: that waits for the work queued before it on the stream, which the NFA
    // launch below waits for anyway, so the host loses one launch latency per batch, not device time
    int64_t ends[2];
    SM_HIP(hipMemcpyAsync(&ends[0], ev.adv_clock, 8, hipMemcpyDeviceToHost, hs));
    SM_HIP(hipMemcpyAsync(&ends[1], ev.adv_clock + ev.nadv - 1, 8, hipMemcpyDeviceToHost, hs));
    SM_HIP(hipStreamSynchronize(hs));
    const int64_t span = ends[1] - ends[0] + 1;
    static const bool cidx_on = !(getenv("SM_NFA_CLOCK_INDEX") && getenv("SM_NFA_CLOCK_INDEX")[0] == '0');
    if (cidx_on && span > 0 && span <= ((int64_t)1 << 26) && a->sc.used + (size_t)span * 4 + (64 << 20) < a->sc.cap) {
      int32_t* cidx = (int32_t*)a->sc.take((size_t)span * 4);
      launch_clock_index(ev.adv_clock, ev.nadv, ends[0], span, cidx, hs);
      b.adv_cidx = cidx;
      b.adv_cmin = ends[0];
      b.adv_cspan = span;
    }
  }
  b.key_off = key_off;
  b.key_pos = key_pos;
  b.lane_compact = lane_compact_ok(b, N, h.node_words, (int)a->ast.streams.size(), a->sc, hs, &b.lane_ord_base) ? 1 : 0;
  b.lane_ev = (const int64_t*)a->sc.take((size_t)std::max<int64_t>(nq, 1) * LaneEv::words(h.node_words, b.lane_compact) * 8);
  b.create_all = !partitioned;
  b.out = q.out.p;
  b.out_count = (uint32_t*)a->d_count.p;
  b.out_cap = (uint32_t)cap;
  b.out_stride = (uint32_t)stride;
  {  // room for every promotion this batch can make: a promoted region holds at most ~32x the words the batch
     // allocates (8x live per semispace, two semispaces, keys promoted at a quarter of their arena), and a batch
     // allocates at most a record, a chain node and a list node per event; capped at option pool_words
    const int64_t bound = (int64_t)q.pool_used + 32 * nq * (int64_t)(h.rec_words + h.node_words + 2) + 4096;
    ensure_pool(a, q, std::max<int64_t>(q.pool_words, std::min<int64_t>(bound, a->pool_init)), (int64_t)q.pool_used);
  }
  b.pool = (int64_t*)q.pool.p;
  b.pool_top = (unsigned long long*)q.pool_top_dev.p;
  b.pool_cap = q.pool_words;
  SM_HIP(hipMemsetAsync((uint64_t*)q.pool_top_dev.p + 1, 0, 8, hs));
  SM_HIP(hipMemsetAsync(a->d_count.p, 0, 4, hs));
  SM_HIP(hipMemsetAsync(a->d_err.p, 0, 4, hs));
  launch_lane_events(b, N, nq, h.node_words, (int32_t*)a->sc.take((size_t)std::max<int64_t>(N, 1) * 4),
                     lds_stream_count((int)a->streams.size()), hs);
  if (tm) tm->mark("nfa_setup", hs);
  if (partitioned && a->lane_balance > 0 && nkeys >= a->lane_balance && a->sc.used + (size_t)nkeys * 24 + (4 << 20) < a->sc.cap) {
    uint32_t* perm = (uint32_t*)a->sc.take((size_t)nkeys * 4);
    launch_lane_balance(key_off, (int32_t)nkeys, perm, a->sc, hs);
    b.lane_perm = perm;
  }
  void* jit = nullptr;
  if (nfa_jit_wanted(a->nfa_jit, nq)) {
    try {
      jit = nfa_jit_function(q.cq.blob, b.lane_compact);
    } catch (const std::exception& e) {
      // the automatic mode falls back to the interpreter (same semantics); an explicit nfa_jit = 1 reports it
      if (a->nfa_jit == 1) throw;
      fprintf(stderr, "[siddhi_amd] query '%s': query-specialised NFA kernel unavailable, using the interpreter (%s)\n",
              q.cq.name.c_str(), e.what());
      a->nfa_jit = 0;
    }
  }
  q.nfa_kernel_used = jit ? 1 : 2;
  if (jit)
    launch_nfa_jit(jit, nfa_jit_lds_bytes(q.cq.blob), b, (int64_t*)q.ks.p, (int64_t*)q.heap.p, a->heap_half,
                   q.state_slots, (int32_t)nkeys, (int32_t*)a->d_err.p, hs);
  else
    launch_nfa(b, (const char*)q.blob.p, (int64_t*)q.ks.p, (int64_t*)q.heap.p, a->heap_half, q.state_slots,
               (int32_t)nkeys, (int32_t*)a->d_err.p, hs);
  SM_HIP(hipGetLastError());
  if (tm) tm->mark("nfa", hs);
  uint32_t hc = 0;
  int32_t he = 0;
  SM_HIP(hipMemcpyAsync(&hc, a->d_count.p, 4, hipMemcpyDeviceToHost, hs));
  SM_HIP(hipMemcpyAsync(&he, a->d_err.p, 4, hipMemcpyDeviceToHost, hs));
  uint64_t ptop[2] = {0, 0};
  SM_HIP(hipMemcpyAsync(ptop, q.pool_top_dev.p, 16, hipMemcpyDeviceToHost, hs));
  SM_HIP(hipStreamSynchronize(hs));
  q.pool_used = ptop[0];
  const int64_t want = (int64_t)ptop[1];  // largest promotion the pool could not take this batch (0: none failed)
  if (want > 0) ++q.pool_refused;
  // keep the pool at most half full for the next batch's promotions, with room for the largest refused one: reclaim
  // dead regions first (compact_pool), grow only if the live partial matches and that request need it
  if (((int64_t)q.pool_used + want) * 2 > q.pool_words) compact_pool(a, q, nkeys, hs);
  if (((int64_t)q.pool_used + want) * 2 > q.pool_words)
    ensure_pool(a, q, std::max<int64_t>(2 * q.pool_words, 2 * ((int64_t)q.pool_used + want)), (int64_t)q.pool_used);
  if (he) {
    std::string why;
    if (he & NFA_ERR_ARENA)
      why += " one event allocated more partial-match state than its key's arena had free, or the overflow pool is "
             "full (raise option heap_words or pool_words);";
    if (he & NFA_ERR_TIMERS) why += " timer queue full;";
    if (he & NFA_ERR_OUTPUT) why += " output buffer full (raise option output_records);";
    if (he & NFA_ERR_NPE) why += " NullPointerException/IllegalStateException path of the reference;";
    throw std::runtime_error("query '" + q.cq.name + "':" + why);
  }
  const int64_t nout = std::min<int64_t>(hc, cap);
  // lanes claim output slots with an atomic, so the records are unordered across lanes: order a large set on the
  // device (a few radix passes) instead of sorting it on the host
  const char* recs = (const char*)q.out.p;
  const size_t need = (size_t)nout * (48 + stride) + (16 << 20);  // keys, indices, ordered copy, sort passes
  const bool keep = a->keep_outputs && a->in_device_events;
  if ((nout >= 2048 || (keep && nout > 1)) && a->sc.used + need <= a->sc.cap) {
    recs = order_outputs(recs, nout, (uint32_t)stride, ev.ev_clock, a->sc, hs);
    SM_HIP(hipStreamSynchronize(hs));
  }
  if (keep) {  // the ordered records with their triggers' global ordinals (sm_app_copy_device_outputs)
    if (nout > 1 && recs == (const char*)q.out.p)
      throw std::runtime_error("query '" + q.cq.name + "': too many output records to order for keep_outputs");
    q.ev_out.ensure(std::max<size_t>((size_t)nout * stride, 16));
    if (nout) SM_HIP(hipMemcpyAsync(q.ev_out.p, recs, (size_t)nout * stride, hipMemcpyDeviceToDevice, hs));
    trigger_ordinals((char*)q.ev_out.p, nout, (uint32_t)stride, ev.ev_ord, hs);
    q.ev_out_n = nout;
    q.ev_out_stride = (uint32_t)stride;
  }
  read_outputs(a, qi, recs, nout, outs);
}

// Scratch of one batch: record selection + key grouping (~96 B per record) and the LaneEv records of the widest
// pattern query.
size_t batch_scratch(const sm_app* a, int64_t N) {
  int64_t lane_words = 0;
  for (auto& q : a->queries)
    if (q->cq.hdr.kind != 0) lane_words = std::max<int64_t>(lane_words, LaneEv::words(q->cq.hdr.node_words));
  return (size_t)N * (100 + 8 * (size_t)lane_words) + (64 << 20);
}

// A closed-form query handed to the general NFA kernel for the rest of its life (QueryRt::nfa_mode) when a device
// batch leaves the closed form's premise: event time decreasing inside the batch or against the carried state,
// a condition outside the v2 kernels' envelope with partials to carry, or matching state already held by the NFA
// (host-API events). The reference has no such switch: it always runs the NFA (StreamPreStateProcessor
// processAndReturn :274-327), and the closed form is only a shortcut of it for monotone event time.
// The carried open partials move into the NFA state by replaying their e1 events in front of the batch, in
// arrival order: each replayed event passes c1 again and re-creates its partial, and as an e2 candidate it meets
// only replayed partials of its own key that it already failed when it first arrived (a partial is still open
// only because every later event of its key failed c2 without expiring it: isExpired :102-121), so the replay
// emits nothing. The batch's matches go to dev_pairs as in the closed form: (e1, e2) relative to ordinal_base,
// in reference order.
int64_t nfa_device_batch(sm_app* a, int qi, int s, size_t n, const int64_t* d_ts, const void* const* d_cols,
                         const int64_t* d_ordinals, int64_t ordinal_base, hipStream_t hs, std::vector<HostOut>* douts) {
  QueryRt& q = *a->queries[qi];
  const auto& attrs = a->streams[s].def->attrs;
  const int nattr = (int)attrs.size();
  const int64_t nc = q.nfa_mode ? 0 : q.carry.n;
  const int64_t N = nc + (int64_t)n;
  q.nfa_mode = true;
  q.carry.reset();  // its partials are handed over below; a failure from here on marks the app failed
  if (N == 0) return 0;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  size_t off = 0;
  std::vector<size_t> col_off(nattr);
  for (int k = 0; k < nattr; ++k) {
    col_off[k] = off;
    off += al((size_t)N * width_of((int)attrs[k].type));
  }
  const size_t ts_off = off;
  off += al((size_t)N * 8);
  const size_t ord_off = off;
  off += al((size_t)N * 8);
  const size_t sid_off = off;
  off += al((size_t)N * 4);
  a->d_rp.ensure(off);
  char* base = (char*)a->d_rp.p;
  if (nc > 0) {  // the carried rows become the first nc entries of the columns, on the device
    if (nattr > kMaxAttrs) throw std::runtime_error("stream has more attributes than the device path supports");
    CarryCols cc{};
    cc.nattr = nattr;
    cc.width = q.carry.width;
    for (int k = 0; k < nattr; ++k) {
      cc.types[k] = (int)attrs[k].type;
      cc.cols[k] = base + col_off[k];
    }
    cc.ts = (int64_t*)(base + ts_off);
    cc.ord = (int64_t*)(base + ord_off);
    carry_rows_to_columns((const int64_t*)q.carry.rows, nc, cc, hs);
  }
  for (int k = 0; k < nattr; ++k) {
    const size_t cw = width_of((int)attrs[k].type);
    if (n) SM_HIP(hipMemcpyAsync(base + col_off[k] + nc * cw, d_cols[k], n * cw, hipMemcpyDeviceToDevice, hs));
  }
  if (n) SM_HIP(hipMemcpyAsync(base + ts_off + nc * 8, d_ts, n * 8, hipMemcpyDeviceToDevice, hs));
  if (d_ordinals) {
    if (n) SM_HIP(hipMemcpyAsync(base + ord_off + nc * 8, d_ordinals, n * 8, hipMemcpyDeviceToDevice, hs));
  } else {
    iota_i64((int64_t*)(base + ord_off) + nc, (int64_t)n, ordinal_base, hs);
  }
  SM_HIP(hipMemsetD32Async((hipDeviceptr_t)(base + sid_off), s, (size_t)N, hs));
  std::vector<NfaStream> nst(a->streams.size());
  memset(nst.data(), 0, nst.size() * sizeof(NfaStream));
  nst[s].nattr = nattr;
  for (int k = 0; k < nattr; ++k) {
    nst[s].types[k] = (int)attrs[k].type;
    nst[s].cols[k] = base + col_off[k];
  }
  a->d_rp_streams.ensure(nst.size() * sizeof(NfaStream));
  SM_HIP(hipMemcpyAsync(a->d_rp_streams.p, nst.data(), nst.size() * sizeof(NfaStream), hipMemcpyHostToDevice, hs));
  for (DBuf* d : {&a->d_ev_row, &a->d_ev_clock, &a->d_ev_ord, &a->d_adv_pos, &a->d_adv_clock, &a->d_adv_wall,
                  &a->d_adv_upto})
    d->ensure((size_t)N * 8);
  a->d_err.ensure(16);
  a->d_count.ensure(16);
  ensure_scratch(a, batch_scratch(a, N));
  a->sc.used = 0;
  const int32_t* sid = (const int32_t*)(base + sid_off);
  const int64_t* ts = (const int64_t*)(base + ts_off);
  int64_t clock_out = a->clock;  // the closed form leaves the playback clock alone: so does its fallback
  const int64_t nadv = build_event_index(N, sid, (int32_t)a->streams.size(), ts, (const int64_t*)(base + ord_off), 0,
                                         a->ast.playback, a->clock, nullptr /* rows = positions */, (int64_t*)a->d_ev_ord.p,
                                         (int64_t*)a->d_ev_clock.p, (int64_t*)a->d_adv_pos.p,
                                         (int64_t*)a->d_adv_clock.p, (int64_t*)a->d_adv_wall.p,
                                         (int64_t*)a->d_adv_upto.p, &clock_out, a->sc, hs);
  const EvArrays ev{sid, nullptr, ts, (const int64_t*)a->d_ev_clock.p,
                    (const int64_t*)a->d_ev_ord.p, (const NfaStream*)a->d_rp_streams.p, (const int64_t*)a->d_adv_pos.p,
                    (const int64_t*)a->d_adv_clock.p, (const int64_t*)a->d_adv_wall.p, (const int64_t*)a->d_adv_upto.p,
                    nadv, a->clock};
  std::vector<HostOut> outs;
  a->sc.used = 0;
  a->need_outs = true;
  struct Reset {
    bool& f;
    ~Reset() { f = false; }
  } reset_need{a->need_outs};
  run_pattern_query(a, qi, ev, N, outs, hs);
  std::stable_sort(outs.begin(), outs.end(), [](const HostOut& x, const HostOut& y) {
    return x.r.pos != y.r.pos ? x.r.pos < y.r.pos : x.r.seq < y.r.seq;
  });
  std::vector<uint32_t> pairs(outs.size() * 2);
  for (size_t k = 0; k < outs.size(); ++k) {
    if (outs[k].r.pos < nc || outs[k].e1 < 0 || outs[k].e2 < 0)
      throw std::runtime_error("query '" + q.cq.name + "': internal error in the hand-over of carried partials");
    pairs[2 * k] = (uint32_t)(outs[k].e1 - ordinal_base);
    pairs[2 * k + 1] = (uint32_t)(outs[k].e2 - ordinal_base);
  }
  q.dev_pairs.ensure(std::max<size_t>(pairs.size() * 4, 16));
  if (!pairs.empty())
    SM_HIP(hipMemcpyAsync(q.dev_pairs.p, pairs.data(), pairs.size() * 4, hipMemcpyHostToDevice, hs));
  // the outputs' Event data for sm_app_device_project (the closed form projects on demand; here the NFA kernel
  // already evaluated the select list)
  const size_t ns = (size_t)q.cq.hdr.nsel, m = outs.size();
  std::vector<DVal> pv(m * ns);
  std::vector<int64_t> pts(m);
  for (size_t k = 0; k < m; ++k) {
    if (ns) memcpy(pv.data() + k * ns, outs[k].vals, ns * sizeof(DVal));
    pts[k] = outs[k].r.ts;
  }
  q.nfa_proj.ensure(std::max<size_t>(m * (ns * sizeof(DVal) + 8), 16));
  if (m) {
    if (ns) SM_HIP(hipMemcpyAsync(q.nfa_proj.p, pv.data(), m * ns * sizeof(DVal), hipMemcpyHostToDevice, hs));
    SM_HIP(hipMemcpyAsync((char*)q.nfa_proj.p + m * ns * sizeof(DVal), pts.data(), m * 8, hipMemcpyHostToDevice, hs));
  }
  SM_HIP(hipStreamSynchronize(hs));
  if (douts)  // the trigger of each output is its e2 (a data event): global ordinal as the delivery position
    for (HostOut& h : outs) {
      h.r.pos = h.e2;
      douts->push_back(h);
    }
  return (int64_t)m;
}

// Whether anything takes query q's outputs: the collect dump, a StreamCallback on its output stream, or a
// QueryCallback (not inherited by partition clones).
bool outputs_consumed(const sm_app* a, const QueryRt& q) {
  if (a->collect) return true;
  auto it = a->stream_cbs.find(q.cq.insert_into);
  if (it != a->stream_cbs.end() && !it->second.empty()) return true;
  auto qt = a->query_cbs.find(q.cq.name);
  return q.cq.partition < 0 && qt != a->query_cbs.end() && !qt->second.empty();
}

// The outputs of query qi's last device batch (closed-form matches or a filter's kept rows) as HostOut records for
// deliver(): QuerySelector.processNoGroupBy (:124-167) on the device (pair_project), one copy to the host, then
// OutputRateLimiter.sendToCallBacks (:61) → StreamCallback.receive (:65) / QueryCallback through deliver(). Each
// output's trigger is its e2 (a filter: its row), so deliver() makes one chunk per input event, as a sequence of
// InputHandler.send calls would. The host copies the records point into live in sm_app::out_arena.
void device_outputs(sm_app* a, int qi, hipStream_t hs, std::vector<DevOut>& outs) {
  const auto t0 = std::chrono::steady_clock::now();
  QueryRt& q = *a->queries[qi];
  const int64_t m = q.dev_n;
  if (m <= 0 || !q.proj_ok) return;
  const CompiledQuery& cq = q.cq;
  const bool rows = cq.hdr.kind == 0;
  const int ns = cq.hdr.nsel;
  const size_t np = (size_t)m * (rows ? 1 : 2);
  uint32_t* hp = (uint32_t*)a->out_arena.take(np * 4);
  SM_HIP(hipMemcpyAsync(hp, q.dev_pairs.p, np * 4, hipMemcpyDeviceToHost, hs));
  hipEvent_t pairs_ev = nullptr;
  if (a->defer_outputs) {
    pairs_ev = a->out_events.take();
    SM_HIP(hipEventRecord(pairs_ev, hs));
  }
  // values, then timestamps: pinned, reused across calls (sm_app::out_arena), not zero-filled. Up to 8 select
  // values cross PCIe in the compact form (8 bytes per value + one byte of null flags per output instead of a
  // 16-byte DVal per value)
  const bool compact = ns > 0 && ns <= 8;
  const size_t vbytes = compact ? (size_t)ns * 8 + 1 : (size_t)ns * sizeof(DVal);
  char* hb = (char*)a->out_arena.take((size_t)m * (vbytes + 8) + 16);
  int64_t* hts = (int64_t*)hb;
  char* hvals = hb + (size_t)m * 8;  // DVal array, or words then null bytes
  q.proj_desc_dev.ensure(sizeof(NfaStream));
  SM_HIP(hipMemcpyAsync(q.proj_desc_dev.p, &q.proj_desc, sizeof(NfaStream), hipMemcpyHostToDevice, hs));
  // deferred (bulk sends, round 5): segments of 2^20 outputs, each with a completion event instead of one final
  // synchronisation, so that deliver_direct prepares the Events of a segment while the later ones are copied
  const bool defer = a->defer_outputs;
  const int64_t chunk = std::min<int64_t>(m, (int64_t)1 << (defer ? 20 : 22));
  q.proj_out.ensure((size_t)chunk * (vbytes + 8) + 16);
  std::vector<int64_t> seg_end;
  std::vector<hipEvent_t> seg_ev;
  int64_t* dts = (int64_t*)q.proj_out.p;
  char* dvals = (char*)q.proj_out.p + (size_t)chunk * 8;
  // the carried partials' e1 order, once for every segment (pair_project_carry_order)
  a->sc.used = 0;
  const uint32_t *ck = nullptr, *ci = nullptr;
  if (q.prev_carry_n > 0 && !rows)
    pair_project_carry_order((const int64_t*)q.prev_carry.p, q.prev_carry_n, q.prev_carry_w, q.proj_base, a->sc, hs,
                             &ck, &ci);
  const size_t sc_base = a->sc.used;
  for (int64_t k0 = 0; k0 < m; k0 += chunk) {
    const int64_t c = std::min(chunk, m - k0);
    a->sc.used = sc_base;
    int64_t* dw = compact ? (int64_t*)dvals : nullptr;
    uint8_t* dn = compact ? (uint8_t*)(dvals + (size_t)chunk * ns * 8) : nullptr;
    // stream order keeps segment k's copies ahead of segment k + 1's projection into the same device buffers
    pair_project((const uint32_t*)q.dev_pairs.p + (rows ? k0 : 2 * k0), c, (const NfaStream*)q.proj_desc_dev.p,
                 q.proj_ord, q.proj_n, q.proj_base, q.proj_ts, (const int64_t*)q.prev_carry.p, q.prev_carry_n,
                 q.prev_carry_w, (const char*)q.blob.p, compact ? nullptr : (DVal*)dvals, dts, a->sc, hs, rows, dw, dn,
                 ck, ci, !defer);
    if (compact) {
      SM_HIP(hipMemcpyAsync(hvals + (size_t)k0 * ns * 8, dw, (size_t)c * ns * 8, hipMemcpyDeviceToHost, hs));
      SM_HIP(hipMemcpyAsync(hvals + (size_t)m * ns * 8 + k0, dn, (size_t)c, hipMemcpyDeviceToHost, hs));
    } else if (ns) {
      SM_HIP(hipMemcpyAsync(hvals + (size_t)k0 * ns * sizeof(DVal), dvals, (size_t)c * ns * sizeof(DVal),
                            hipMemcpyDeviceToHost, hs));
    }
    SM_HIP(hipMemcpyAsync(hts + k0, dts, (size_t)c * 8, hipMemcpyDeviceToHost, hs));
    if (defer) {
      seg_end.push_back(k0 + c);
      seg_ev.push_back(a->out_events.take());
      SM_HIP(hipEventRecord(seg_ev.back(), hs));
    }
  }
  if (!defer) SM_HIP(hipStreamSynchronize(hs));
  DevOut d{qi, m, hp, compact ? nullptr : (const DVal*)hvals, hts, rows, q.proj_base};
  if (compact) {
    d.hw = (const int64_t*)hvals;
    d.hn = (const uint8_t*)(hvals + (size_t)m * ns * 8);
  }
  d.seg_end.swap(seg_end);
  d.seg_ev.swap(seg_ev);
  d.pairs_ev = pairs_ev;
  outs.push_back(d);
  q.n_out += m;
  a->host_ms[1] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// HostOut records of device outputs (the general deliver(): several queries' outputs to interleave, or NFA records
// to merge with): the trigger of each output is its e2 (a filter: its row), the hidden references its e1 / e2.
void materialize(sm_app* a, const DevOut& d, std::vector<HostOut>& outs) {
  const CompiledQuery& cq = a->queries[d.qi]->cq;
  const int ns = cq.hdr.nsel, nr = cq.hdr.nrefs_vis;
  const int32_t* rslots = (const int32_t*)(cq.blob.data() + cq.hdr.off_refs);
  int64_t* hrf = (int64_t*)a->out_arena.take((size_t)std::max<int64_t>(d.m * nr, 1) * 8);
  const DVal* hv = d.hv;
  if (d.hw) {  // compact form: HostOut points at DVals
    DVal* v = (DVal*)a->out_arena.take((size_t)std::max<int64_t>(d.m * ns, 1) * sizeof(DVal));
    parallel_for((size_t)d.m, (size_t)1 << 16, [&](size_t lo, size_t hi) {
      for (size_t k = lo; k < hi; ++k)
        for (int j = 0; j < ns; ++j) {
          DVal& x = v[k * ns + j];
          x.i = d.hw[k * ns + j];
          x.null = (d.hn[k] >> j) & 1;
          x.pad = 0;
        }
    });
    hv = v;
  }
  const size_t base = outs.size();
  outs.resize(base + (size_t)d.m);
  parallel_for((size_t)d.m, (size_t)1 << 16, [&](size_t lo, size_t hi) {
    for (size_t k = lo; k < hi; ++k) {
      const int64_t e1 = d.base + (int32_t)d.hp[d.rows ? k : 2 * k];
      const int64_t e2 = d.base + (int32_t)d.hp[d.rows ? k : 2 * k + 1];
      int64_t* rf = hrf + k * nr;
      for (int r = 0; r < nr; ++r) rf[r] = rslots[2 * r] == 0 ? e1 : e2;
      HostOut& h = outs[base + k];
      memset(&h.r, 0, sizeof(h.r));
      h.r.pos = e2;
      h.r.create = -1;
      h.r.ts = d.hts[k];
      h.r.phase = 1;
      h.r.query = cq.hdr.query_order;
      h.r.seq = (int32_t)k;
      h.vals = hv + k * ns;
      h.nvals = ns;
      h.refs = rf;
      h.nrefs = nr;
      h.qidx = d.qi;
      h.e1 = e1;
      h.e2 = e2;
    }
  });
}

// One query's device outputs straight into Events (deliver_device when nothing else interleaves with them and no
// dump is collected): they are in reference order already (e2, then e1; a filter's rows in order), one chunk per
// trigger = per run of equal e2. No HostOut, no comparison sort; the Events are built by several threads.
void deliver_direct(sm_app* a, const DevOut& d) {
  const auto t0 = std::chrono::steady_clock::now();
  const CompiledQuery& cq = a->queries[d.qi]->cq;
  const int ns = cq.hdr.nsel;
  Pending& pd = a->pending;
  const std::array<int64_t, 3> at = query_callbacks(a, cq);
  if (at[2] == 0) {
    d.wait_all();  // the copies in flight land in buffers the next call reuses
    return;
  }
  const size_t m = (size_t)d.m;
  auto trig = [&](size_t k) { return d.rows ? d.hp[k] : d.hp[2 * k + 1]; };
  // the call's only outputs: the uniform chunk form (Pending::starts); otherwise PreparedChunks after what is there
  const bool uni = pd.chunks.empty() && !pd.uniform && pd.evs.size() == 0;
  if (!uni) pd.expand();
  const size_t c0 = pd.chunks.size(), e0 = pd.evs.size(), v0 = pd.vals.size();
  pd.evs.resize(e0 + m);
  pd.vals.resize(v0 + m * ns);
  // chunk starts (one per trigger) from the tuples, which cross PCIe first: counted per unit (a slice of the outputs),
  // then the Events written at their ranks. With deferred copies (DevOut segments) every segment is cut into one unit
  // per thread and thread t takes units t, t + T, ...: all threads build the Events of a segment as soon as it has
  // landed, while the later segments are still being copied (a thread waits only for the segment of its next unit)
  if (d.pairs_ev) SM_HIP(hipEventSynchronize(d.pairs_ev));
  const size_t T = std::min<size_t>((size_t)host_threads(), std::max<size_t>(m >> 16, 1));
  const size_t U = T * std::max<size_t>(d.seg_end.size(), 1);
  std::vector<size_t> cnt(U + 1, 0);
  parallel_for(T, 1, [&](size_t lo, size_t hi) {
    for (size_t t = lo; t < hi; ++t)
      for (size_t u = t; u < U; u += T) {
        size_t c = 0;
        for (size_t k = m * u / U; k < m * (u + 1) / U; ++k) c += k == 0 || trig(k) != trig(k - 1);
        cnt[u + 1] = c;
      }
  });
  for (size_t u = 0; u < U; ++u) cnt[u + 1] += cnt[u];
  bool strings = false;
  for (int t : cq.sel_types) strings |= t == T_STRING;
  // the views form (round 6): every callback of the chunks takes columns (sm_app_add_stream_columns_callback), so
  // no Event is built: the chunk starts only, and the callbacks get views of the pinned copies, whose buffers the
  // Pending takes from the output arena until they have run (Pending::views)
  bool cols_only = uni && d.hw && !strings && ns <= 8 && at[1] == 0;
  for (int64_t c = at[0]; c < at[0] + at[2] && cols_only; ++c) cols_only = pd.cbs[(size_t)c].ccb != nullptr;
  if (cols_only) {
    pd.evs.resize(e0);
    pd.vals.resize(v0);
    pd.uniform = true;
    pd.proto = PreparedChunk{};
    pd.proto.cb_off = (uint32_t)at[0];
    pd.proto.n_cbs = (uint32_t)at[2];
    pd.starts.resize(cnt[U]);
    parallel_for(T, 1, [&](size_t lo, size_t hi) {
      for (size_t t = lo; t < hi; ++t)
        for (size_t u = t; u < U; u += T) {
          size_t c = cnt[u];
          for (size_t k = m * u / U; k < m * (u + 1) / U; ++k)
            if (k == 0 || trig(k) != trig(k - 1)) pd.starts[c++] = k;
        }
    });
    pd.seg_end = d.seg_end;  // the values may still be crossing PCIe: run_callbacks waits segment by segment
    pd.seg_ev = d.seg_ev;
    pd.views = true;
    pd.cts = d.hts;
    pd.cvals = d.hw;
    pd.cnul = d.hn;
    pd.cns = ns;
    for (int j = 0; j < ns; ++j) pd.ctypes[j] = cq.sel_types[j];
    pd.cn = m;
    a->out_arena.lend(pd.owned);
    a->host_ms[2] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return;
  }
  // the streamed form: one query's compact values without strings are written with non-temporal stores (gigabytes
  // of Events that the next accesses read from DRAM anyway: no read-for-ownership of every line), the events holding
  // their final pointers (the call's vals do not grow again before the callbacks; Pending::expand undoes it)
  const bool streamed = uni && d.hw && !strings && ns <= 8;
  int64_t w0[8] = {0};
  bool isf[8] = {false};
  for (int j = 0; j < ns && streamed; ++j) {
    w0[j] = (int64_t)(uint32_t)cq.sel_types[j];
    isf[j] = cq.sel_types[j] == T_FLOAT || cq.sel_types[j] == T_DOUBLE;
  }
  if (uni) {
    pd.uniform = true;
    pd.proto = PreparedChunk{};
    pd.proto.cb_off = (uint32_t)at[0];
    pd.proto.n_cbs = (uint32_t)at[2];
    pd.proto.n_query_cbs = (uint32_t)at[1];
    pd.starts.resize(cnt[U]);
  } else {
    pd.chunks.resize(c0 + cnt[U]);
  }
  parallel_for(T, 1, [&](size_t lo, size_t hi) {
    for (size_t t = lo; t < hi; ++t) {
      size_t ready = d.seg_end.empty() ? m : 0;  // outputs known to be on the host
      for (size_t u = t; u < U; u += T) {
        size_t c = c0 + cnt[u];
        const size_t kb = m * u / U, ke = m * (u + 1) / U;
        for (size_t k = kb; k < ke; ++k) {
          if (k >= ready) {
            for (size_t i = 0; i < d.seg_end.size(); ++i)
              if ((size_t)d.seg_end[i] > k) {
                SM_HIP(hipEventSynchronize(d.seg_ev[i]));
                ready = (size_t)d.seg_end[i];
                break;
              }
          }
          if (streamed) {
            sm_value* v = pd.vals.data() + v0 + k * ns;
            long long* vw = (long long*)v;
            const uint8_t nb = d.hn[k];
            for (int j = 0; j < ns; ++j) {
              const bool nul = (nb >> j) & 1;
              const long long x = nul ? 0 : (long long)d.hw[k * ns + j];
              _mm_stream_si64(vw + 4 * j, (long long)(w0[j] | ((int64_t)nul << 32)));  // type, is_null
              _mm_stream_si64(vw + 4 * j + 1, isf[j] ? 0 : x);                        // i
              _mm_stream_si64(vw + 4 * j + 2, isf[j] ? x : 0);                        // d (the double's bits)
              _mm_stream_si64(vw + 4 * j + 3, 0);                                     // s
            }
            long long* ew = (long long*)(pd.evs.data() + e0 + k);
            _mm_stream_si64(ew, (long long)d.hts[k]);
            _mm_stream_si64(ew + 1, (long long)(uintptr_t)v);
            _mm_stream_si64(ew + 2, (long long)(uint32_t)ns);
          } else {
            if (d.hw) to_sm_values_compact(a, d.hw + k * ns, d.hn[k], ns, cq, pd.vals.data() + v0 + k * ns);
            else to_sm_values(a, d.hv + k * ns, ns, cq, pd.vals.data() + v0 + k * ns);
            pd.evs[e0 + k] = sm_event{d.hts[k], (const sm_value*)(uintptr_t)(v0 + k * ns), (int32_t)ns};
          }
          if (k == 0 || trig(k) != trig(k - 1)) {
            if (uni) {
              pd.starts[c++] = k;
              continue;
            }
            PreparedChunk& ch = pd.chunks[c++];
            ch.cb_off = (uint32_t)at[0];
            ch.n_cbs = (uint32_t)at[2];
            ch.n_query_cbs = (uint32_t)at[1];
            ch.ev_off = e0 + k;
          }
        }
      }
    }
    if (streamed) _mm_sfence();  // the streamed lines are visible before the callbacks read them
  });
  if (streamed) pd.final_ = true;
  const size_t nch = uni ? c0 : pd.chunks.size();
  parallel_for(nch - c0, (size_t)1 << 16, [&](size_t lo, size_t hi) {  // sizes and timestamps (the last event's)
    for (size_t c = c0 + lo; c < c0 + hi; ++c) {
      PreparedChunk& ch = pd.chunks[c];
      const size_t end = c + 1 < nch ? pd.chunks[c + 1].ev_off : e0 + m;
      ch.n_ev = end - ch.ev_off;
      ch.ts = pd.evs[end - 1].timestamp;
    }
  });
  if (strings)  // STRING values are owned by the pending outputs (the dictionary may change before the callbacks)
    for (size_t k = v0; k < pd.vals.size(); ++k) {
      sm_value& v = pd.vals[k];
      if (v.type == T_STRING && !v.is_null) {
        pd.strs.push_back(std::make_unique<std::string>(v.s));
        v.s = pd.strs.back()->c_str();
      }
    }
  a->host_ms[2] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// Host side of one batch in arrival order: the staged input (flush), or a chaining level's merged batch.
struct EvHost {
  std::vector<int32_t>* stream;
  std::vector<int64_t>*row, *ts, *clock, *ord, *adv_pos, *adv_clock, *adv_wall;
};

// Key code (the int64 the key table hashes: key_lookup_kernel) of a row's key column, false if it is null.
bool host_key_code(const StreamStage& st, int col, int64_t row, int64_t* code) {
  if (st.any_null[col] && st.nulls[col][row]) return false;
  const uint8_t* b = st.cols[col].data();
  const int t = col < (int)st.def->attrs.size() ? (int)st.def->attrs[col].type : T_LONG;
  switch (t) {
    case T_INT:
    case T_STRING: { int32_t x; memcpy(&x, b + row * 4, 4); *code = x; break; }
    case T_LONG: memcpy(code, b + row * 8, 8); break;
    case T_FLOAT: {
      float f;
      memcpy(&f, b + row * 4, 4);
      double d = f;
      if (d != d) d = std::numeric_limits<double>::quiet_NaN();
      memcpy(code, &d, 8);
      if (d != d) *code = 0x7ff8000000000000ll;
      break;
    }
    case T_DOUBLE: {
      double d;
      memcpy(&d, b + row * 8, 8);
      memcpy(code, &d, 8);
      if (d != d) *code = 0x7ff8000000000000ll;
      break;
    }
    default: *code = b[row]; break;
  }
  return true;
}

// A batch assembled on the host (chaining levels, broadcast copies): per-stream rows plus the arrival-order
// arrays. Streams listed in `hidden` get one more column (a LONG key code) than the rows they copy.
struct BatchBuilder {
  std::vector<StreamStage> stages;
  std::vector<int32_t> stream;
  std::vector<int64_t> row, ts, clock, ord, adv_pos, adv_clock, adv_wall;
  EvHost ev() { return EvHost{&stream, &row, &ts, &clock, &ord, &adv_pos, &adv_clock, &adv_wall}; }
  void init(const std::vector<StreamStage>& like, const std::vector<int>& hidden = {}) {
    stages.resize(like.size());
    for (size_t s = 0; s < like.size(); ++s) {
      StreamStage& d = stages[s];
      d.def = like[s].def;
      size_t nc = like[s].cols.size();
      if (std::find(hidden.begin(), hidden.end(), (int)s) != hidden.end()) ++nc;
      d.cols.resize(nc);
      d.nulls.resize(nc);
      d.any_null.assign(nc, false);
      d.dcols.resize(nc);
      d.dnulls.resize(nc);
    }
  }
  static int width(const StreamStage& st, int k) {
    return k < (int)st.def->attrs.size() ? width_of((int)st.def->attrs[k].type) : 8;
  }
  // a new event record; its row (if any) is appended with put_bytes / copy_row
  int64_t put(int32_t s, int64_t t, int64_t clk, int64_t o) {
    const int64_t pos = (int64_t)stream.size();
    stream.push_back(s);
    ts.push_back(t);
    clock.push_back(clk);
    ord.push_back(o);
    if (s < 0) {
      row.push_back(-1);
    } else {
      StreamStage& d = stages[s];
      row.push_back(d.rows++);
      d.row_pos.push_back(pos);
    }
    return pos;
  }
  void put_bytes(int s, size_t k, const uint8_t* b, int w, bool nul) {
    StreamStage& d = stages[s];
    d.cols[k].insert(d.cols[k].end(), b, b + w);
    d.nulls[k].push_back(nul ? 1 : 0);
    if (nul) d.any_null[k] = true;
  }
  void copy_row(int s, const StreamStage& src, int64_t r) {
    for (size_t k = 0; k < src.cols.size(); ++k) {
      const int w = width(src, (int)k);
      put_bytes(s, k, src.cols[k].data() + r * w, w, src.any_null[k] && src.nulls[k][r]);
    }
  }
};

// Upload a batch for the query kernels; the returned view is valid until the next upload.
EvArrays upload_batch(sm_app* a, std::vector<StreamStage>& stages, const EvHost& e) {
  const int64_t N = (int64_t)e.stream->size();
  std::vector<NfaStream> nst(stages.size());
  for (size_t s = 0; s < stages.size(); ++s) {
    StreamStage& st = stages[s];
    NfaStream& d = nst[s];
    memset(&d, 0, sizeof(d));
    d.nattr = (int)st.cols.size();  // an extra key column included
    for (int k = 0; k < d.nattr; ++k) {
      d.types[k] = k < (int)st.def->attrs.size() ? (int)st.def->attrs[k].type : T_LONG;
      upload(a, st.dcols[k], st.cols[k]);
      d.cols[k] = st.dcols[k].p;
      if (st.any_null[k]) {
        upload(a, st.dnulls[k], st.nulls[k]);
        d.nulls[k] = (const uint8_t*)st.dnulls[k].p;
      }
    }
    upload(a, st.drow_pos, st.row_pos);
  }
  upload(a, a->d_streams, nst);
  upload(a, a->d_ev_stream, *e.stream);
  upload(a, a->d_ev_row, *e.row);
  upload(a, a->d_ev_ts, *e.ts);
  upload(a, a->d_ev_clock, *e.clock);
  upload(a, a->d_ev_ord, *e.ord);
  upload(a, a->d_adv_pos, *e.adv_pos);
  upload(a, a->d_adv_clock, *e.adv_clock);
  upload(a, a->d_adv_wall, *e.adv_wall);
  std::vector<int64_t> upto(N);
  size_t j = 0;
  for (int64_t p = 0; p < N; ++p) {
    while (j < e.adv_pos->size() && (*e.adv_pos)[j] <= p) ++j;
    upto[p] = (int64_t)j;
  }
  upload(a, a->d_adv_upto, upto);
  SM_HIP(hipStreamSynchronize(a->stream));
  a->d_err.ensure(16);
  a->d_count.ensure(16);
  ensure_scratch(a, batch_scratch(a, N));
  return EvArrays{(const int32_t*)a->d_ev_stream.p, (const int64_t*)a->d_ev_row.p, (const int64_t*)a->d_ev_ts.p,
                  (const int64_t*)a->d_ev_clock.p, (const int64_t*)a->d_ev_ord.p, (const NfaStream*)a->d_streams.p,
                  (const int64_t*)a->d_adv_pos.p, (const int64_t*)a->d_adv_clock.p, (const int64_t*)a->d_adv_wall.p,
                  (const int64_t*)a->d_adv_upto.p, (int64_t)e.adv_pos->size(), a->clock_batch_in};
}

// Instances of partition pi in creation order after the events of a batch: `keys` / `kset` start as the
// instances before the batch; each keyed event (a key column that is not null) of a new key appends one.
// at[p] = instances existing when position p is delivered (its own instance included).
void walk_instances(const sm_app* a, int pi, const std::vector<StreamStage>& stages, const EvHost& e,
                    std::vector<int64_t>& keys, std::vector<int32_t>& types, std::unordered_set<int64_t>& kset,
                    std::vector<int64_t>* at) {
  const CompiledPartition& cp = a->parts[pi];
  const std::vector<int>& bc = a->part_bcast[pi];
  const int64_t N = (int64_t)e.stream->size();
  if (at) at->resize(N);
  for (int64_t p = 0; p < N; ++p) {
    const int s = (*e.stream)[p];
    if (s >= 0 && a->ast.streams[s].id[0] != '#' && std::find(bc.begin(), bc.end(), s) == bc.end()) {
      const auto it = std::find(cp.streams.begin(), cp.streams.end(), s);
      if (it != cp.streams.end()) {
        int64_t code;
        const int col = cp.key_code[it - cp.streams.begin()][0].a;
        if (host_key_code(stages[s], col, (*e.row)[p], &code) && kset.insert(code).second) {
          keys.push_back(code);
          types.push_back(col < (int)stages[s].def->attrs.size() ? (int32_t)stages[s].def->attrs[col].type : T_LONG);
        }
      }
    }
    if (at) (*at)[p] = (int64_t)keys.size();
  }
}

// A query reading a stream its partition does not key, over a copy of the batch in which each such event is
// repeated once per instance existing at that point, in the order PartitionStreamReceiver.send (:271-275) visits
// them: cachedStreamJunctionMap.values(), a ConcurrentHashMap keyed by streamId + String.valueOf(key) and filled in
// creation order (java_order.h). The copy's extra column holds the instance's key code. Its outputs move back to
// the original event's position, ranked by the copy's place in that iteration (OutRec.time = rank + 1) under the
// partition receiver's place among the stream's receivers (OutRec.sched).
void run_bcast_query(sm_app* a, int qi, std::vector<StreamStage>& stages, const EvHost& e, std::vector<HostOut>& outs) {
  QueryRt& q = *a->queries[qi];
  const int pi = q.pidx;
  const std::vector<int>& bc = a->part_bcast[pi];
  std::vector<int64_t> keys = a->part_keys[pi];
  std::vector<int32_t> ktypes = a->part_key_types[pi];
  std::unordered_set<int64_t> kset = a->part_key_set[pi];
  std::vector<int64_t> at;
  walk_instances(a, pi, stages, e, keys, ktypes, kset, &at);
  // the receiver's junction map per broadcast stream, grown in creation order as the batch creates instances
  struct Chm {
    JavaChmOrder map;
    std::vector<int> order;
    size_t ordered = 0;  // map size `order` was taken at
  };
  std::map<int, Chm> chm;
  auto instance_order = [&](int s, int64_t count) -> const std::vector<int>& {
    Chm& c = chm[s];
    while ((int64_t)c.map.size() < count) {
      const size_t k = c.map.size();
      const std::string ks = ktypes[k] == T_STRING
                                 ? (keys[k] >= 0 && keys[k] < (int64_t)a->dict.strs.size() ? a->dict.strs[keys[k]] : "")
                                 : java_value_string(ktypes[k], keys[k]);
      c.map.put(a->ast.streams[s].id + ks);
    }
    if (c.ordered != c.map.size() || c.order.empty()) {
      c.order = c.map.order();
      c.ordered = c.map.size();
    }
    return c.order;
  };
  BatchBuilder b;
  b.init(stages, bc);
  const int64_t N = (int64_t)e.stream->size();
  std::vector<int64_t> map, rank;
  std::vector<int64_t> newpos(N);
  for (int64_t p = 0; p < N; ++p) {
    const int s = (*e.stream)[p];
    const bool rep = s >= 0 && std::find(bc.begin(), bc.end(), s) != bc.end();
    const int64_t copies = rep ? at[p] : 1;
    const std::vector<int>* ord = rep && copies > 0 ? &instance_order(s, copies) : nullptr;
    newpos[p] = (int64_t)b.stream.size();
    for (int64_t k = 0; k < copies; ++k) {
      b.put(s, (*e.ts)[p], (*e.clock)[p], (*e.ord)[p]);
      map.push_back(p);
      rank.push_back(rep ? k : -1);
      if (s < 0) continue;
      b.copy_row(s, stages[s], (*e.row)[p]);
      if (rep) b.put_bytes(s, stages[s].cols.size(), (const uint8_t*)&keys[(*ord)[k]], 8, false);
    }
  }
  for (size_t k = 0; k < e.adv_pos->size(); ++k) {
    b.adv_pos.push_back(newpos[(*e.adv_pos)[k]]);
    b.adv_clock.push_back((*e.adv_clock)[k]);
    b.adv_wall.push_back((*e.adv_wall)[k]);
  }
  const EvArrays ev = upload_batch(a, b.stages, b.ev());
  const size_t first = outs.size();
  a->sc.used = 0;
  run_pattern_query(a, qi, ev, (int64_t)b.stream.size(), outs, a->stream);
  q.nfa_used = true;
  std::vector<int64_t> slot_keys(q.keys.nslots);
  if (!slot_keys.empty())
    SM_HIP(hipMemcpy(slot_keys.data(), q.keys.slot_keys, slot_keys.size() * 8, hipMemcpyDeviceToHost));
  for (size_t i = first; i < outs.size(); ++i) {
    HostOut& h = outs[i];
    if (h.r.key >= 0 && h.r.key < (int32_t)slot_keys.size()) h.key_code = slot_keys[h.r.key];
    const int64_t r = rank[h.r.pos];
    const int s = (*e.stream)[map[h.r.pos]];
    h.r.pos = map[h.r.pos];
    if (r >= 0 && h.r.phase == 1) {
      h.r.time = r + 1;
      h.r.sched = a->part_bcast_group[pi].at(s);
    } else if (r >= 0) {
      h.r.seq = (int32_t)(r * (1 << 20) + h.r.seq);
    }
  }
}

// Upload one batch and run the queries of chaining level `level` over it; their outputs (positions in this
// batch) are appended to outs. Outputs of a partition query carry their instance's key code (key_code).
void run_level(sm_app* a, std::vector<StreamStage>& stages, const EvHost& e, int level, std::vector<HostOut>& outs) {
  const int64_t N = (int64_t)e.stream->size();
  const EvArrays ev = upload_batch(a, stages, e);
  for (size_t qi = 0; qi < a->queries.size(); ++qi) {
    QueryRt& q = *a->queries[qi];
    if (q.level != level || q.bcast) continue;
    const DQuery& h = q.cq.hdr;
    a->sc.used = 0;
    q.proj_ok = q.proj_nfa = false;  // host-staged outputs: nothing for sm_app_device_project
    size_t stride = sizeof(OutRec) + h.nsel * sizeof(DVal) + h.nrefs * sizeof(int64_t);
    const size_t first = outs.size();
    if (h.kind == 0) {
      StreamStage& st = stages[h.stream];
      if (st.rows == 0) continue;
      const NfaStream* sd = (const NfaStream*)a->d_streams.p + h.stream;
      int64_t* rows = (int64_t*)a->sc.take(st.rows * 8);
      const char* blob = (const char*)q.blob.p;
      const DQuery* hd = &h;
      int64_t nm = filter_rows(sd, st.rows, (const Instr*)(blob + hd->off_code) + h.filt_off, h.filt_len,
                               (const DVal*)(blob + hd->off_const), rows, a->sc, a->stream);
      q.out.ensure(std::max<size_t>((size_t)nm * stride, 16));
      project_rows(sd, rows, nm, (const int64_t*)st.drow_pos.p, (const int64_t*)a->d_ev_ts.p, (const int64_t*)a->d_ev_ord.p, blob,
                   h.query_order, (char*)q.out.p, (uint32_t)stride, a->stream);
      read_outputs(a, (int)qi, q.out.p, nm, outs);
      if (q.part) {
        // PartitionStreamReceiver drops an event whose key is null before any instance sees it
        const CompiledPartition& cp = *q.part;
        const int k = (int)(std::find(cp.streams.begin(), cp.streams.end(), h.stream) - cp.streams.begin());
        const int col = cp.key_code[k][0].a;
        size_t w = first;
        for (size_t i = first; i < outs.size(); ++i) {
          int64_t code;
          if (!host_key_code(st, col, (*e.row)[outs[i].r.pos], &code)) continue;
          outs[i].key_code = code;
          if (w != i) outs[w] = std::move(outs[i]);
          ++w;
        }
        outs.resize(w);
      }
      continue;
    }
    run_pattern_query(a, (int)qi, ev, N, outs, a->stream);
    for (int s : q.cq.streams)
      if (stages[s].rows > 0) q.nfa_used = true;
    if (q.part && outs.size() > first) {  // instance key of each output (its lane's key slot)
      std::vector<int64_t> keys(q.keys.nslots);
      if (!keys.empty())
        SM_HIP(hipMemcpy(keys.data(), q.keys.slot_keys, keys.size() * 8, hipMemcpyDeviceToHost));
      for (size_t i = first; i < outs.size(); ++i)
        if (outs[i].r.key >= 0 && outs[i].r.key < (int32_t)keys.size()) outs[i].key_code = keys[outs[i].r.key];
    }
  }
  for (size_t qi = 0; qi < a->queries.size(); ++qi)  // their batches replace the uploaded one: last
    if (a->queries[qi]->level == level && a->queries[qi]->bcast) run_bcast_query(a, (int)qi, stages, e, outs);
}

bool out_before(const OutRec& x, const OutRec& y);

// Query chaining (InsertIntoStreamCallback → StreamJunction.sendEvent → the reading queries, depth first, before
// the junction moves on to its next receiver). Every event and output gets an order key:
//   input event at position p: (p, 2); an output: its trigger's key (an input event's: (p)), then
//   (phase 1: 1, query, seq | timer phase 0: 0, time, listener group, create, query, scheduler, seq);
//   an event a query inserts into a stream later queries read: the key of that output.
// Level L runs over the previous level's batch merged with the events level L-1's queries inserted, in key
// order: an inserted event precedes its root input event, because every query reading it was defined (and so
// subscribed to that event's stream) after the query inserting it; it keeps the trigger's playback clock
// (sendEvent does not advance it) and has no arrival ordinal. Outputs are delivered in key order.
void run_chained(sm_app* a, std::vector<HostOut>& outs) {
  using Key = std::vector<int64_t>;
  struct Level {
    std::vector<StreamStage> stages;
    std::vector<int32_t> stream;
    std::vector<int64_t> row, ts, clock, ord, adv_pos, adv_clock, adv_wall;
    std::vector<Key> key;
    EvHost ev() { return EvHost{&stream, &row, &ts, &clock, &ord, &adv_pos, &adv_clock, &adv_wall}; }
  };
  auto out_key = [](const Key& trig, const OutRec& r) {
    Key k = trig.size() == 2 && trig[1] == 2 ? Key{trig[0]} : trig;
    if (r.phase == 1) k.insert(k.end(), {1, r.time ? r.sched : r.query, r.time, r.query, r.seq});
    else k.insert(k.end(), {0, r.time, r.create >= 0 ? 1 : 0, r.create, r.query, r.sched, r.seq});
    return k;
  };
  std::vector<std::unique_ptr<Level>> lv;
  std::vector<StreamStage>* pst = &a->streams;
  EvHost pe{&a->ev_stream, &a->ev_row, &a->ev_ts, &a->ev_clock, &a->ev_ord, &a->adv_pos, &a->adv_clock, &a->adv_wall};
  std::vector<Key> pkey(a->ev_stream.size());
  for (size_t p = 0; p < pkey.size(); ++p) pkey[p] = Key{(int64_t)p, 2};
  std::vector<Key> okey(outs.size());
  size_t done = 0;  // outputs whose key is known
  auto key_outs = [&](const std::vector<Key>& ek) {
    okey.resize(outs.size());
    for (; done < outs.size(); ++done) okey[done] = out_key(ek[outs[done].r.pos], outs[done].r);
  };
  key_outs(pkey);
  size_t lstart = 0;
  for (int L = 1; L <= a->max_level; ++L) {
    const size_t lend = outs.size();
    // this level's new events: outputs of level L-1 into streams a query reads
    std::vector<size_t> der;
    for (size_t i = lstart; i < lend; ++i) {
      const int s = stream_index(a->ast, a->queries[outs[i].qidx]->cq.insert_into);
      if (s >= 0 && a->stream_fed[s]) der.push_back(i);
    }
    lstart = lend;
    std::stable_sort(der.begin(), der.end(), [&](size_t x, size_t y) { return okey[x] < okey[y]; });
    auto nl = std::make_unique<Level>();
    nl->stages.resize(pst->size());
    for (size_t s = 0; s < pst->size(); ++s) {
      StreamStage& d = nl->stages[s];
      const StreamStage& o = (*pst)[s];
      d.def = o.def;
      d.cols.resize(o.cols.size());
      d.nulls.resize(o.cols.size());
      d.any_null.assign(o.cols.size(), false);
      d.dcols.resize(o.cols.size());
      d.dnulls.resize(o.cols.size());
    }
    const int64_t Np = (int64_t)pe.stream->size();
    std::vector<int64_t> map(Np);
    auto col_width = [](const StreamStage& st, int k) {
      return k < (int)st.def->attrs.size() ? width_of((int)st.def->attrs[k].type) : 8;
    };
    auto put_event = [&](int32_t s, int64_t ts, int64_t clk, int64_t ord, const Key& k) {
      nl->stream.push_back(s);
      nl->ts.push_back(ts);
      nl->clock.push_back(clk);
      nl->ord.push_back(ord);
      nl->key.push_back(k);
      if (s < 0) {
        nl->row.push_back(-1);
        return;
      }
      StreamStage& d = nl->stages[s];
      nl->row.push_back(d.rows);
      d.row_pos.push_back((int64_t)nl->stream.size() - 1);
      ++d.rows;
    };
    auto copy_event = [&](int64_t p) {
      const int32_t s = (*pe.stream)[p];
      map[p] = (int64_t)nl->stream.size();
      const int64_t r = (*pe.row)[p];
      put_event(s, (*pe.ts)[p], (*pe.clock)[p], (*pe.ord)[p], pkey[p]);
      if (s < 0) return;
      StreamStage& d = nl->stages[s];
      const StreamStage& o = (*pst)[s];
      for (size_t k = 0; k < o.cols.size(); ++k) {
        const int w = col_width(o, (int)k);
        d.cols[k].insert(d.cols[k].end(), o.cols[k].begin() + r * w, o.cols[k].begin() + (r + 1) * w);
        const uint8_t nul = o.any_null[k] ? o.nulls[k][r] : 0;
        d.nulls[k].push_back(nul);
        if (nul) d.any_null[k] = true;
      }
    };
    auto derived_event = [&](size_t oi) {
      const HostOut& h = outs[oi];
      const int s = stream_index(a->ast, a->queries[h.qidx]->cq.insert_into);
      put_event(s, h.r.ts, (*pe.clock)[h.r.pos], -1, okey[oi]);
      StreamStage& d = nl->stages[s];
      const size_t na = d.def->attrs.size();
      for (size_t k = 0; k < d.cols.size(); ++k) {
        uint8_t b[8];
        int w;
        uint8_t nul = 0;
        if (k < na) {
          const int t = (int)d.def->attrs[k].type;
          w = width_of(t);
          const DVal& v = h.vals[k];
          nul = v.null ? 1 : 0;
          if (t == T_FLOAT) {
            const float f = (float)v.d;
            memcpy(b, &f, 4);
          } else if (t == T_DOUBLE) {
            memcpy(b, &v.d, 8);
          } else if (t == T_LONG) {
            memcpy(b, &v.i, 8);
          } else if (t == T_BOOL) {
            b[0] = (uint8_t)(v.i != 0);
          } else {
            const int32_t x = (int32_t)v.i;
            memcpy(b, &x, 4);
          }
        } else {  // inner stream: the producing instance's key code
          w = 8;
          memcpy(b, &h.key_code, 8);
        }
        d.cols[k].insert(d.cols[k].end(), b, b + w);
        d.nulls[k].push_back(nul);
        if (nul) d.any_null[k] = true;
      }
    };
    size_t di = 0;
    for (int64_t p = 0; p < Np; ++p) {
      while (di < der.size() && okey[der[di]] < pkey[p]) derived_event(der[di++]);
      copy_event(p);
    }
    while (di < der.size()) derived_event(der[di++]);
    for (size_t k = 0; k < pe.adv_pos->size(); ++k) {
      nl->adv_pos.push_back(map[(*pe.adv_pos)[k]]);
      nl->adv_clock.push_back((*pe.adv_clock)[k]);
      nl->adv_wall.push_back((*pe.adv_wall)[k]);
    }
    run_level(a, nl->stages, nl->ev(), L, outs);
    key_outs(nl->key);
    pst = &nl->stages;
    pkey = nl->key;
    lv.push_back(std::move(nl));
    pe = lv.back()->ev();
  }
  // delivery order: by key; one position per (trigger, query) so that deliver keeps it and groups its chunks
  std::vector<size_t> ord(outs.size());
  for (size_t i = 0; i < ord.size(); ++i) ord[i] = i;
  std::stable_sort(ord.begin(), ord.end(), [&](size_t x, size_t y) { return okey[x] < okey[y]; });
  std::vector<HostOut> sorted;
  sorted.reserve(outs.size());
  int64_t rank = -1;
  for (size_t k = 0; k < ord.size(); ++k) {
    const Key& cur = okey[ord[k]];
    if (k == 0 || !std::equal(cur.begin(), cur.end() - 1, okey[ord[k - 1]].begin(), okey[ord[k - 1]].end() - 1)) ++rank;
    sorted.push_back(std::move(outs[ord[k]]));
    sorted.back().r.pos = rank;
    sorted.back().r.phase = 1;
  }
  outs.swap(sorted);
}

// The device-batch path of one stream (sm_app_process_device_batch, and host-API batches of apps whose queries all
// take it: flush_device): every query reading stream s runs over the n events (columns, event times and ordinals
// in device memory) on hs; the outputs that have consumers are appended to douts (host copies in out_arena).
void device_batch_stream(sm_app* a, int s, size_t n, const int64_t* d_ts, const void* const* d_cols,
                         const int64_t* d_ordinals, int64_t ordinal_base, hipStream_t hs, std::vector<HostOut>& douts,
                         std::vector<DevOut>& draw) {
  if (a->max_level > 0)
    throw sql::UnsupportedError("apps whose queries read streams other queries fill run through the host API");
  for (auto& bc : a->part_bcast)
    if (!bc.empty()) throw sql::UnsupportedError("partitions reading unkeyed streams run through the host API");
  for (auto& qp : a->queries)
    if (qp->cq.hdr.kind != 0 && !qp->cq.fast_every_within &&
        std::find(qp->cq.streams.begin(), qp->cq.streams.end(), s) != qp->cq.streams.end())
      throw sql::UnsupportedError("device batches support filter queries and `every e1 -> e2 within T` patterns; "
                                  "query '" + qp->cq.name + "' takes sm_app_process_device_events or the host API");
  StreamStage& st = a->streams[s];
  NfaStream d;
  memset(&d, 0, sizeof(d));
  d.nattr = (int)st.def->attrs.size();
  for (int k = 0; k < d.nattr; ++k) {
    d.types[k] = (int)st.def->attrs[k].type;
    d.cols[k] = d_cols[k];
  }
  a->d_streams.ensure(sizeof(NfaStream));
  SM_HIP(hipMemcpyAsync(a->d_streams.p, &d, sizeof(NfaStream), hipMemcpyHostToDevice, hs));
  size_t need = 64 << 20;  // filter queries: mask words + block counts; patterns: records, pairs, counts
  for (auto& qp : a->queries) {
    const CompiledQuery& cq = qp->cq;
    if (std::find(cq.streams.begin(), cq.streams.end(), s) == cq.streams.end()) continue;
    // patterns: records / staging / pairs (64 B per event), carry-out candidates (32 B each) and the carried
    // partials' working arrays, plus the bucket-stack spill rings and bounded buffers
    const size_t nc = (size_t)qp->carry.n, wc = (size_t)std::max(qp->carry.width, 4);
    need = std::max(need, cq.hdr.kind == 0 ? n / 8 + n / 1024 + (64 << 20)
                                           : n * 68 + std::min<size_t>(n + nc, (size_t)1 << 26) * 32 +
                                                 nc * (160 + 8 * wc) + ((size_t)640 << 20));
  }
  ensure_scratch(a, need);
  for (size_t qi = 0; qi < a->queries.size(); ++qi) {
    QueryRt& q = *a->queries[qi];
    const CompiledQuery& cq = q.cq;
    if (std::find(cq.streams.begin(), cq.streams.end(), s) == cq.streams.end()) continue;
    a->sc.used = 0;
    const char* blob = (const char*)q.blob.p;
    const bool consumed = outputs_consumed(a, q);
    q.proj_ok = q.proj_nfa = false;
    q.proj_desc = d;
    q.proj_ts = d_ts;
    q.proj_ord = d_ordinals;
    q.proj_base = ordinal_base;
    q.proj_n = (int64_t)n;
    if (cq.hdr.kind == 0) {
      q.dev_pairs.ensure(std::max<size_t>(n * 4, 16));
      bool typed = false;
      q.dev_n = filter_device(d, (const NfaStream*)a->d_streams.p, (int64_t)n,
                              (const Instr*)(blob + cq.hdr.off_code) + cq.hdr.filt_off,
                              (const Instr*)(cq.blob.data() + cq.hdr.off_code) + cq.hdr.filt_off, cq.hdr.filt_len,
                              (const DVal*)(blob + cq.hdr.off_const), (const DVal*)(cq.blob.data() + cq.hdr.off_const),
                              d_ordinals, ordinal_base, (uint32_t*)q.dev_pairs.p, a->sc, hs,
                              a->fast_timing ? &a->fast_tm : nullptr, &typed);
      q.fast_path_used = typed ? 4 : 3;
      q.prev_carry_n = 0;
      q.proj_ok = true;
      if (consumed) device_outputs(a, (int)qi, hs, draw);
      continue;
    }
    if (q.nfa_mode || q.nfa_used) {  // matching state held by the NFA kernel
      q.dev_n = nfa_device_batch(a, (int)qi, s, n, d_ts, d_cols, d_ordinals, ordinal_base, hs,
                                 consumed ? &douts : nullptr);
      q.fast_path_used = 5;
      q.proj_nfa = true;
      continue;
    }
    FastArgs fa{};
    fa.n = (int64_t)n;
    fa.ts = d_ts;
    fa.st = (const NfaStream*)a->d_streams.p;
    fa.key = cq.partition >= 0 ? (const KeyProg*)q.keyprogs.p : nullptr;
    if (fa.key) {
      const CompiledPartition& cp = *q.part;
      int idx = (int)(std::find(cp.streams.begin(), cp.streams.end(), s) - cp.streams.begin());
      fa.key = (const KeyProg*)q.keyprogs.p + idx;
    }
    fa.code = (const Instr*)(blob + cq.hdr.off_code);
    fa.consts = (const DVal*)(blob + cq.hdr.off_const);
    fa.c1_off = cq.fast_c1_off;
    fa.c1_len = cq.fast_c1_len;
    fa.c2_off = cq.fast_c2_off;
    fa.c2_len = cq.fast_c2_len;
    fa.within = cq.fast_within;
    fa.ordinals = d_ordinals;
    fa.ordinal_base = ordinal_base;
    q.dev_pairs.ensure(std::max<size_t>((n + (size_t)q.carry.n) * 8, 16));
    std::vector<int32_t> types(d.types, d.types + d.nattr);
    FastHostInfo hi;
    hi.cols = d_cols;
    hi.types = types.data();
    hi.vattr = fast_vattr(cq, types);
    hi.c2_host = (const Instr*)(cq.blob.data() + cq.hdr.off_code) + cq.fast_c2_off;
    hi.c2_len = cq.fast_c2_len;
    hi.c1_host = (const Instr*)(cq.blob.data() + cq.hdr.off_code) + cq.fast_c1_off;
    hi.c1_len = cq.fast_c1_len;
    if (hi.vattr >= 0) hi.vtype = types[hi.vattr];
    hi.nattr = d.nattr;
    if (fa.key) {
      const CompiledPartition& cp = *q.part;
      int idx = (int)(std::find(cp.streams.begin(), cp.streams.end(), s) - cp.streams.begin());
      const auto& kc = cp.key_code[idx];
      if (kc.size() == 1 && kc[0].op == OP_COL) {
        hi.key_col = kc[0].a;
        hi.key_type = types[hi.key_col];
      }
    }
    // partition keys as dense ids (any key domain): decided at the query's first closed-form batch, then kept, since
    // the carried partials hold ids; ValuePartitionExecutor (core/partition/executor/ValuePartitionExecutor.java:34-39)
    // keys by any value, so a sparse 64-bit id must not leave the closed form
    if (fa.key && hi.key_col >= 0 && !a->force_general_fast && n > 0) {
      if (q.remap == 0 && !q.carry.active) {
        // option "key_remap", or (automatic) ids when the first batch's key span exceeds the bucket-stack window
        // (2^20): the batch runs on the values with remap_span set, and its prep pass reports a wider span
        // (FAST_KEY_SPAN) before anything changes
        if (a->key_remap >= 0) q.remap = a->key_remap ? 1 : 2;
        else hi.remap_span = (int64_t)1 << 20;
      }
      if (q.remap == 1) {  // the pipelines read the ids instead of the key column (the column keeps its values)
        int32_t* dk = (int32_t*)a->sc.take(n * 4);
        remap_keys(q.dense, hi.cols[hi.key_col], hi.key_type, (int64_t)n, dk, hs);
        hi.dense_keys = dk;
      }
    }
    q.prev_carry_n = q.carry.n;
    q.prev_carry_w = q.carry.width;
    if (q.carry.n > 0) {
      const size_t cb = (size_t)q.carry.n * q.carry.width * 8;
      q.prev_carry.ensure(cb);
      SM_HIP(hipMemcpyAsync(q.prev_carry.p, q.carry.rows, cb, hipMemcpyDeviceToDevice, hs));
    }
    int64_t m = FAST_OUTSIDE;
    if (!a->force_general_fast)
      m = fast_every_within_v2(fa, hi, q.fast, q.carry, (uint32_t*)q.dev_pairs.p, (int64_t)(n + q.carry.n), a->sc, hs,
                               a->fast_timing ? &a->fast_tm : nullptr, a->fast_stack);
    if (m == FAST_KEY_SPAN && q.remap != 1 && a->key_remap < 0 && fa.key && hi.key_col >= 0) {
      // the first batch's keys span more than the bucket-stack window, or a later batch's keys leave the span the
      // first batch showed: dense ids from here on, for the carried partials' keys too (each key's rows stay one
      // run, so the carry keeps its grouping)
      q.remap = 1;
      hi.remap_span = 0;
      remap_carry_keys(q.dense, q.carry.rows, q.carry.n, q.carry.width, a->sc, hs);
      if (q.carry.n > 0)
        SM_HIP(hipMemcpyAsync(q.prev_carry.p, q.carry.rows, (size_t)q.carry.n * q.carry.width * 8,
                              hipMemcpyDeviceToDevice, hs));
      int32_t* dk = (int32_t*)a->sc.take(n * 4);
      remap_keys(q.dense, hi.cols[hi.key_col], hi.key_type, (int64_t)n, dk, hs);
      hi.dense_keys = dk;
      m = fast_every_within_v2(fa, hi, q.fast, q.carry, (uint32_t*)q.dev_pairs.p, (int64_t)(n + q.carry.n), a->sc, hs,
                               a->fast_timing ? &a->fast_tm : nullptr, a->fast_stack);
    }
    if (q.remap == 0 && hi.remap_span > 0 && m != FAST_OUTSIDE) q.remap = 2;  // the span fitted: values from here on
    q.fast_path_used = q.fast.last_path;
    if (m == FAST_OUTSIDE && a->force_general_fast && q.carry.n == 0) {
      // diagnostic (option "fast_general"): the stateless general closed form, one batch at a time
      m = fast_every_within(fa, (uint32_t*)q.dev_pairs.p, (int64_t)n, a->sc, hs, a->fast_timing ? &a->fast_tm : nullptr);
      q.fast_path_used = 1;
    } else if (m < 0) {
      // event time not monotone, or a condition outside the v2 envelope: the NFA kernel takes the query over
      // (carried partials included) and keeps it, so later batches and host events see one matching state
      m = nfa_device_batch(a, (int)qi, s, n, d_ts, d_cols, d_ordinals, ordinal_base, hs, consumed ? &douts : nullptr);
      q.fast_path_used = 5;
      q.proj_nfa = true;
    }
    q.dev_n = m;
    q.proj_ok = q.fast_path_used != 5 && m >= 0;
    if (q.proj_ok && consumed) device_outputs(a, (int)qi, hs, draw);
  }
}

// Outputs of device-batch queries to their consumers (deliver() hands them out even when only the collect dump
// takes them).
void deliver_device(sm_app* a, std::vector<HostOut>& douts, std::vector<DevOut>& draw) {
  if (!douts.empty() || !draw.empty()) {
    a->need_outs = true;
    struct Reset {
      bool& f;
      ~Reset() { f = false; }
    } reset_need{a->need_outs};
    if (douts.empty() && draw.size() == 1 && !a->collect) {
      deliver_direct(a, draw[0]);
    } else {
      for (const DevOut& d : draw) {
        d.wait_all();
        materialize(a, d, douts);
      }
      deliver(a, douts);
    }
  }
  a->out_arena.clear();
  a->out_events.clear();
}

// Whether a host-API batch (the staged events of sm_input_send / sm_input_send_columns) can take the device-batch
// path, stream by stream: every query is a filter or an `every e1 -> e2 within T` pattern (so no query reads the
// playback clock or has timers, and each reads one stream), no query reads another query's output, no partition
// broadcasts, and no staged value is null (device columns carry no null masks). The closed form then runs on the
// host's events exactly as on a device batch, with one carry: InputHandler.send(Event[]) (InputHandler.java:64-68)
// feeds the same receivers as any other send.
bool app_device_ok(const sm_app* a) {
  if (a->max_level > 0) return false;
  for (auto& bc : a->part_bcast)
    if (!bc.empty()) return false;
  for (auto& q : a->queries)
    if (q->cq.hdr.kind != 0 && !q->cq.fast_every_within) return false;
  return true;
}

bool host_batch_device_ok(const sm_app* a) {
  if (!app_device_ok(a)) return false;
  for (auto& st : a->streams)
    if (st.rows > 0)
      for (size_t k = 0; k < st.any_null.size(); ++k)
        if (st.any_null[k]) return false;
  return true;
}

// A host-API batch through the device-batch path (host_batch_device_ok): per stream, its staged columns, its events'
// times and arrival ordinals are uploaded and device_batch_stream runs every query reading it; the outputs of all
// streams are delivered together in reference order (deliver() orders them by trigger ordinal, then query).
// Heartbeats and the start record carry no event: no query of such an app reads them.
void flush_device(sm_app* a) {
  std::vector<HostOut> douts;
  std::vector<DevOut> draw;
  a->out_arena.clear();
  for (size_t s = 0; s < a->streams.size(); ++s) {
    StreamStage& st = a->streams[s];
    if (st.rows == 0) continue;
    bool read = false;
    for (auto& q : a->queries) read |= std::find(q->cq.streams.begin(), q->cq.streams.end(), (int)s) != q->cq.streams.end();
    if (!read) continue;
    const int64_t R = st.rows;
    std::vector<int64_t> rts(R), rord(R);
    bool contiguous = true;
    for (int64_t r = 0; r < R; ++r) {
      const int64_t p = st.row_pos[r];
      rts[r] = a->ev_ts[p];
      rord[r] = a->ev_ord[p];
      contiguous &= rord[r] == rord[0] + r;
    }
    std::vector<const void*> dc(st.cols.size());
    for (size_t k = 0; k < st.cols.size(); ++k) {
      upload(a, st.dcols[k], st.cols[k]);
      dc[k] = st.dcols[k].p;
    }
    upload(a, st.drow_ts, rts);
    if (!contiguous) upload(a, st.drow_ord, rord);
    device_batch_stream(a, (int)s, (size_t)R, (const int64_t*)st.drow_ts.p, dc.data(),
                        contiguous ? nullptr : (const int64_t*)st.drow_ord.p, rord[0], a->stream, douts, draw);
  }
  SM_HIP(hipStreamSynchronize(a->stream));
  deliver_device(a, douts, draw);
}


void flush(sm_app* a);

// InputHandler.send(Event[]) (InputHandler.java:64-68) of a large columnar batch (sm_input_send_columns, at least
// bulk_min events, no nulls, no STRING attribute) for an app whose queries all take the device-batch path
// (app_device_ok): the columns go from the caller's memory straight to the device in chunks of bulk_chunk events,
// without host staging, and each chunk runs through device_batch_stream with the next arrival ordinals (one carry, so
// partials span the chunks as they span sends in the reference). A helper thread uploads chunk c + 1 on its own HIP
// stream while chunk c is processed. Each chunk is processed under the app lock and its outputs go to the callbacks
// before the next chunk (with the lock released, so a callback may send into the app: what it sends is staged and
// runs before the next chunk). Returns a status like the locked entry points.
int bulk_send_device(sm_app* a, int s, size_t n, const int64_t* ts, const void* const* cols) {
  const int nattr = (int)a->streams[s].def->attrs.size();
  std::vector<size_t> w(nattr);
  for (int k = 0; k < nattr; ++k) w[k] = (size_t)width_of((int)a->streams[s].def->attrs[k].type);
  const size_t B = std::min(n, (size_t)std::max<int64_t>(a->bulk_chunk, 1));
  const size_t nchunks = (n + B - 1) / B;
  const int dev = a->device;
  std::future<void> next;
  auto upload_chunk = [a, dev, nattr, &w, ts, cols](size_t lo, size_t len, int b) {
    SM_HIP(hipSetDevice(dev));
    hipStream_t cs = a->copy_stream;
    for (int k = 0; k < nattr; ++k)
      SM_HIP(hipMemcpyAsync(a->bulk[b][k].p, (const char*)cols[k] + lo * w[k], len * w[k], hipMemcpyHostToDevice, cs));
    SM_HIP(hipMemcpyAsync(a->bulk[b][nattr].p, ts + lo, len * 8, hipMemcpyHostToDevice, cs));
    SM_HIP(hipStreamSynchronize(cs));
  };
  Pending out;  // the chunks' outputs; its arrays are reused from chunk to chunk and from call to call
  {
    std::lock_guard<std::mutex> g(a->mu);
    out.swap(a->bulk_spare);
  }
  struct Done {  // the upload in flight finishes before the buffers can be reused or freed
    sm_app* a;
    std::future<void>& f;
    Pending& out;
    ~Done() {
      if (f.valid()) f.wait();
      std::lock_guard<std::mutex> g(a->mu);
      a->bulk_active = false;
      out.clear();
      a->bulk_spare.swap(out);
    }
  } done{a, next, out};
  int rc = SM_OK;
  std::vector<HostOut> douts;
  std::vector<DevOut> draw;
  using clk = std::chrono::steady_clock;
  auto ms_since = [](clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); };
  for (size_t c = 0; c < nchunks && rc == SM_OK; ++c) {
    {
      std::lock_guard<std::mutex> g(a->mu);
      out.clear();
      a->pending.swap(out);  // a->pending is empty between calls: it takes the reused arrays
      rc = guarded([&] {
        if (a->failed) throw std::runtime_error(a->failed_why);
        flush(a);  // events staged before this chunk (earlier sends, or callbacks of the previous chunk) come first
        if (c == 0) {
          if (!a->copy_stream) SM_HIP(hipStreamCreateWithFlags(&a->copy_stream, hipStreamNonBlocking));
          for (int b = 0; b < 2; ++b) {
            a->bulk[b].resize(nattr + 1);
            for (int k = 0; k < nattr; ++k) a->bulk[b][k].ensure(B * w[k]);
            a->bulk[b][nattr].ensure(B * 8);
          }
          next = std::async(std::launch::async, upload_chunk, (size_t)0, B, 0);
        }
        const size_t lo = c * B, len = std::min(B, n - lo);
        const int b = (int)(c & 1);
        const auto tw = clk::now();
        next.get();  // chunk c is on the device (rethrows an upload error)
        a->host_ms[4] += ms_since(tw);
        if (c + 1 < nchunks) next = std::async(std::launch::async, upload_chunk, lo + B, std::min(B, n - lo - B), b ^ 1);
        std::vector<const void*> dc(nattr);
        for (int k = 0; k < nattr; ++k) dc[k] = a->bulk[b][k].p;
        douts.clear();
        draw.clear();
        a->out_arena.clear();
        try {
          const auto td = clk::now();
          // outputs cross PCIe in segments while the first ones become Events (DevOut::seg_ev, deliver_direct)
          a->defer_outputs = true;
          struct Undefer {
            sm_app* a;
            ~Undefer() {
              // no copy outlives the call, unless the call's Pending holds views of them (it waits for them itself)
              if (a->defer_outputs && a->pending.seg_ev.empty()) (void)hipStreamSynchronize(a->stream);
              a->defer_outputs = false;
            }
          } undefer{a};
          device_batch_stream(a, s, len, (const int64_t*)a->bulk[b][nattr].p, dc.data(), nullptr, a->next_ordinal,
                              a->stream, douts, draw);
          a->host_ms[0] += ms_since(td);
          deliver_device(a, douts, draw);
        } catch (const std::exception& e) {
          a->failed = true;
          a->failed_why = std::string("a batch failed half-way (") + e.what() +
                          "); the matching state is inconsistent: restore a snapshot or reset the app";
          throw;
        }
        a->next_ordinal += (int64_t)len;
        a->ordinal_base += (int64_t)len;
        if (a->ast.playback)  // StreamJunction.sendData :232-237: the clock follows the largest event time so far
          for (size_t i = lo; i < lo + len; ++i) a->clock = std::max(a->clock, ts[i]);
        a->clock_batch_in = a->clock;
      });
      out.swap(a->pending);
    }
    const auto tc = clk::now();
    run_callbacks(out);
    give_back(a, out);
    a->host_ms[3] += ms_since(tc);
  }
  return rc;
}

void flush(sm_app* a) {
  const int64_t N = (int64_t)a->ev_stream.size();
  if (N == 0) return;
  std::vector<HostOut> outs;
  // the batch is consumed whatever happens below: a query that fails half-way leaves the matching state
  // inconsistent (earlier queries advanced, outputs lost), so the app refuses further events until it is restored
  // or reset, instead of running the same events again
  struct BatchDone {
    sm_app* a;
    int64_t N;
    bool ok = false;
    ~BatchDone() {
      a->ordinal_base += N;
      a->clock_batch_in = a->clock;
      a->ev_stream.clear();
      a->ev_row.clear();
      a->ev_ts.clear();
      a->ev_clock.clear();
      a->ev_ord.clear();
      a->adv_pos.clear();
      a->adv_clock.clear();
      a->adv_wall.clear();
      for (auto& st : a->streams) st.clear();
    }
  } done{a, N};
  try {
    if (host_batch_device_ok(a)) {
      flush_device(a);
      return;
    }
    // the NFA kernel runs this batch: a closed-form query whose stream has events here hands its carried partials
    // over first (nfa_device_batch without new events replays them into the NFA state) and stays on the NFA
    for (size_t qi = 0; qi < a->queries.size(); ++qi) {
      QueryRt& q = *a->queries[qi];
      if (!q.cq.fast_every_within || q.nfa_mode || q.nfa_used || q.carry.n == 0) continue;
      const int s = q.cq.streams.at(0);
      if (a->streams[s].rows > 0) nfa_device_batch(a, (int)qi, s, 0, nullptr, nullptr, nullptr, 0, a->stream, nullptr);
    }
    const EvHost e0{&a->ev_stream, &a->ev_row, &a->ev_ts, &a->ev_clock, &a->ev_ord, &a->adv_pos, &a->adv_clock,
                    &a->adv_wall};
    run_level(a, a->streams, e0, 0, outs);
    if (a->max_level > 0) run_chained(a, outs);
    for (size_t pi = 0; pi < a->part_bcast.size(); ++pi)  // instances this batch created, for later broadcasts
      if (!a->part_bcast[pi].empty())
        walk_instances(a, (int)pi, a->streams, e0, a->part_keys[pi], a->part_key_types[pi], a->part_key_set[pi],
                       nullptr);
  } catch (const std::exception& e) {
    a->failed = true;
    a->failed_why = std::string("a batch failed half-way (") + e.what() +
                    "); the matching state is inconsistent: restore a snapshot or reset the app";
    throw;
  }
  deliver(a, outs);
}

// StreamJunction.sendData :232-237: the playback clock advances (and listeners fire) only when ts >= clock
void stage_record(sm_app* a, int32_t stream, int64_t row, int64_t ts, int wall) {
  int64_t p = (int64_t)a->ev_stream.size();
  a->ev_stream.push_back(stream);
  a->ev_row.push_back(row);
  a->ev_ts.push_back(ts);
  a->ev_ord.push_back(stream >= 0 ? a->next_ordinal++ : -1);
  if (a->ast.playback && stream != NFA_START) {
    if (ts >= a->clock) {
      a->clock = ts;
      a->adv_pos.push_back(p);
      a->adv_clock.push_back(ts);
      a->adv_wall.push_back(wall ? ts : -1);
    }
  }
  a->ev_clock.push_back(a->clock);
}

void maybe_autoflush(sm_app* a) {
  if ((int64_t)a->ev_stream.size() >= a->batch_events) flush(a);
}

void put_value(StreamStage& st, int k, const sm_value& v, sm_app* a) {
  int t = (int)st.def->attrs[k].type;
  auto& col = st.cols[k];
  size_t w = width_of(t);
  size_t off = col.size();
  col.resize(off + w);
  uint8_t* dst = col.data() + off;
  bool isnull = v.is_null != 0;
  if (!isnull && v.type != t) throw TypeError("value type does not match attribute '" + st.def->attrs[k].name + "'");
  switch (t) {
    case T_INT: { int32_t x = isnull ? 0 : (int32_t)v.i; memcpy(dst, &x, 4); break; }
    case T_LONG: { int64_t x = isnull ? 0 : v.i; memcpy(dst, &x, 8); break; }
    case T_FLOAT: { float x = isnull ? 0.f : (float)v.d; memcpy(dst, &x, 4); break; }
    case T_DOUBLE: { double x = isnull ? 0.0 : v.d; memcpy(dst, &x, 8); break; }
    case T_STRING: { int32_t x = isnull ? -1 : a->dict.intern(v.s ? v.s : ""); memcpy(dst, &x, 4); break; }
    default: { uint8_t x = isnull ? 0 : (v.i ? 1 : 0); *dst = x; break; }
  }
  if (isnull || st.any_null[k]) {
    if (!st.any_null[k]) {
      st.any_null[k] = true;
      st.nulls[k].assign(st.rows, 0);
    }
    st.nulls[k].push_back(isnull ? 1 : 0);
  }
}

std::string dump_json(sm_app* a) {
  std::ostringstream o;
  o << "{\"streams\":{";
  bool first = true;
  for (auto& kv : a->collected_streams) {
    if (!first) o << ",";
    first = false;
    o << "\"" << kv.first << "\":[";
    for (size_t k = 0; k < kv.second.size(); ++k) o << (k ? "," : "") << kv.second[k];
    o << "]";
  }
  o << "},\"queries\":{";
  first = true;
  for (auto& kv : a->collected_queries) {
    if (!first) o << ",";
    first = false;
    o << "\"" << kv.first << "\":[";
    for (size_t k = 0; k < kv.second.size(); ++k) o << (k ? "," : "") << kv.second[k];
    o << "]";
  }
  o << "}}";
  return o.str();
}

}  // namespace
}  // namespace sm

using namespace sm;

// snapshot encoding helpers (sm_app_snapshot / sm_app_restore)
namespace {
constexpr char kSnapMagic[8] = {'S', 'M', 'S', 'N', 'A', 'P', '0', '5'};

struct SnapWriter {
  std::vector<uint8_t> b;
  void raw(const void* p, size_t n) { b.insert(b.end(), (const uint8_t*)p, (const uint8_t*)p + n); }
  template <typename T> void put(T v) { raw(&v, sizeof(T)); }
};
struct SnapReader {
  const uint8_t* p;
  size_t n, o = 0;
  void raw(void* d, size_t k) {
    if (o + k > n) throw std::runtime_error("CannotRestoreSiddhiAppStateException: snapshot truncated");
    memcpy(d, p + o, k);
    o += k;
  }
  template <typename T> T get() {
    T v;
    raw(&v, sizeof(T));
    return v;
  }
};

uint64_t fnv1a(const std::string& s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
  return h;
}
}  // namespace

extern "C" {

const char* sm_last_error(void) { return sm::g_err.c_str(); }

// The StreamCallback of the reference's performance samples (modules/siddhi-samples/performance-samples: receive()
// adds events.length to a counter), as a native function: `user` points at an int64 count.
void sm_count_events_callback(void* user, const sm_event* events, size_t n) {
  (void)events;
  *(int64_t*)user += (int64_t)n;
}
const char* sm_version(void) { return "siddhi_amd 0.1 (gfx950)"; }

int sm_manager_create(sm_manager** out) {
  *out = new sm_manager();
  return SM_OK;
}
void sm_manager_destroy(sm_manager* m) { delete m; }

int sm_app_create(sm_manager* m, const char* siddhiql, sm_app** out) {
  (void)m;
  *out = nullptr;
  auto a = std::make_unique<sm_app>();
  int rc = guarded([&] {
    a->ast = sql::parse_app(siddhiql ? siddhiql : "");
    a->text_hash = fnv1a(siddhiql ? siddhiql : "");
    build_app(a.get());
    int dev = 0;
    if (hipGetDeviceCount(&dev) != hipSuccess || dev == 0)
      throw std::runtime_error("HIP error: no MI355X device visible (the engine has no CPU fallback)");
    upload_app(a.get());
    if (const char* e = getenv("SIDDHI_AMD_HEAP_WORDS")) a->heap_half = std::max(256, atoi(e));
    if (const char* e = getenv("SM_NFA_BALANCE")) a->lane_balance = atoll(e);
  });
  if (rc == SM_OK) *out = a.release();
  return rc;
}

int sm_compile_dump(const char* siddhiql, char* buf, size_t cap, size_t* len) {
  return guarded([&] {
    const std::string j = sql::dump_app_json(sql::parse_app(siddhiql ? siddhiql : ""));
    *len = j.size();
    if (buf && cap > j.size()) {
      memcpy(buf, j.data(), j.size());
      buf[j.size()] = 0;
    }
  });
}

int sm_nfa_jit_compile(const char* siddhiql, int query, char* log, size_t cap, size_t* code_size) {
  int rc = guarded([&] {
    const sql::App ast = sql::parse_app(siddhiql ? siddhiql : "");
    if (query < 0 || (size_t)query >= ast.order.size()) throw std::runtime_error("no such query");
    Dict dict;
    auto [pi, qi] = ast.order[query];
    const sql::Query& qd = pi < 0 ? ast.queries[qi] : ast.partitions[pi].queries[qi];
    const CompiledQuery cq = compile_query(ast, qd, query, pi, dict);
    // SM_NFA_JIT_COMPACT=0/1: compile for that LaneEv form as a constant, as a batch launch does (tools/jit_precompile.py
    // fills the code-object cache this way on the build host); unset: the form is read at run time
    const char* cf = getenv("SM_NFA_JIT_COMPACT");
    const std::vector<char> code = nfa_jit_compile(cq.blob, cf && *cf ? (atoi(cf) ? 1 : 0) : -1);
    if (code_size) *code_size = code.size();
    if (const char* path = getenv("SM_NFA_JIT_CO")) {
      if (FILE* f = fopen(path, "wb")) {
        fwrite(code.data(), 1, code.size(), f);
        fclose(f);
      }
    }
  });
  if (log && cap) {
    const std::string& m = sm::g_err;
    const size_t n = std::min(cap - 1, m.size());
    memcpy(log, m.data(), n);
    log[n] = 0;
  }
  return rc;
}

void sm_app_destroy(sm_app* a) {
  if (!a) return;
  for (auto& q : a->queries) q->keys.release();
  if (a->stream) (void)hipStreamDestroy(a->stream);
  if (a->copy_stream) (void)hipStreamDestroy(a->copy_stream);
  delete a;
}

int sm_app_start(sm_app* a) {
  return locked(a, [&] {
    if (a->started) return;
    a->started = true;
    // absent start-state processors of non-partitioned queries schedule their first timer at start()
    stage_record(a, NFA_START, -1, a->clock, 0);
  });
}

int sm_app_flush(sm_app* a) {
  return locked(a, [&] { flush(a); });
}

int sm_app_shutdown(sm_app* a) {
  return locked(a, [&] {
    if (a->shut) return;
    flush(a);
    a->shut = true;
  });
}

int sm_app_input_handler(sm_app* a, const char* stream_id, sm_input** out) {
  std::lock_guard<std::mutex> g(a->mu);
  return guarded([&] {
    int s = stream_index(a->ast, stream_id ? stream_id : "");
    if (s < 0) throw sql::ValidationError(std::string("stream '") + (stream_id ? stream_id : "") + "' is not defined");
    if (a->ast.streams[s].id[0] == '#')
      throw sql::ValidationError(std::string("inner stream '") + stream_id + "' is only visible inside its partition");
    auto in = std::make_unique<sm_input>();
    in->app = a;
    in->stream = s;
    *out = in.get();
    a->inputs.push_back(std::move(in));
  });
}

int sm_input_send(sm_input* in, int64_t ts, const sm_value* row, size_t n) {
  sm_app* a = in->app;
  return locked(a, [&] {
    StreamStage& st = a->streams[in->stream];
    if (n != st.def->attrs.size()) throw TypeError("row has " + std::to_string(n) + " values, stream '" + st.def->id +
                                                   "' has " + std::to_string(st.def->attrs.size()) + " attributes");
    // the whole row is checked before any column grows (a rejected row leaves the staged columns aligned)
    for (size_t k = 0; k < n; ++k)
      if (!row[k].is_null && row[k].type != (int)st.def->attrs[k].type)
        throw TypeError("value type does not match attribute '" + st.def->attrs[k].name + "'");
    for (size_t k = 0; k < n; ++k) put_value(st, (int)k, row[k], a);
    st.row_pos.push_back((int64_t)a->ev_stream.size());
    stage_record(a, in->stream, st.rows, ts, 0);
    st.rows++;
    maybe_autoflush(a);
  });
}

int sm_input_send_columns(sm_input* in, size_t n, const int64_t* ts, const void* const* cols,
                          const uint8_t* const* null_flags) {
  sm_app* a = in->app;
  bool bulk = false;
  const int rc = locked(a, [&] {
    StreamStage& st = a->streams[in->stream];
    size_t na = st.def->attrs.size();
    bool nulls = false, strings = false;
    for (size_t k = 0; k < na; ++k) {
      nulls |= null_flags && null_flags[k];
      strings |= (int)st.def->attrs[k].type == T_STRING;
    }
    bulk = (int64_t)n >= a->bulk_min && !nulls && !strings && !a->bulk_active && app_device_ok(a);
    if (bulk) {
      a->bulk_active = true;
      return;
    }
    for (size_t i = 0; i < n; ++i) {
      for (size_t k = 0; k < na; ++k) {
        sm_value v{};
        int t = (int)st.def->attrs[k].type;
        v.type = t;
        v.is_null = null_flags && null_flags[k] && null_flags[k][i];
        switch (t) {
          case T_INT: v.i = ((const int32_t*)cols[k])[i]; break;
          case T_LONG: v.i = ((const int64_t*)cols[k])[i]; break;
          case T_FLOAT: v.d = ((const float*)cols[k])[i]; break;
          case T_DOUBLE: v.d = ((const double*)cols[k])[i]; break;
          case T_STRING: v.s = ((const char* const*)cols[k])[i]; v.is_null |= v.s == nullptr; break;
          default: v.i = ((const uint8_t*)cols[k])[i]; break;
        }
        put_value(st, (int)k, v, a);
      }
      st.row_pos.push_back((int64_t)a->ev_stream.size());
      stage_record(a, in->stream, st.rows, ts[i], 0);
      st.rows++;
      maybe_autoflush(a);
    }
  });
  if (rc != SM_OK || !bulk) return rc;
  return bulk_send_device(a, in->stream, n, ts, cols);
}

int sm_app_stream_schema(sm_app* a, const char* stream_id, int32_t* types, size_t cap, size_t* n) {
  std::lock_guard<std::mutex> g(a->mu);
  return guarded([&] {
    int s = stream_index(a->ast, stream_id ? stream_id : "");
    if (s < 0) throw sql::ValidationError(std::string("stream '") + (stream_id ? stream_id : "") + "' is not defined");
    const auto& at = a->ast.streams[s].attrs;
    *n = at.size();
    for (size_t k = 0; k < at.size() && k < cap; ++k) types[k] = (int32_t)at[k].type;
  });
}

int sm_app_advance_time(sm_app* a, int64_t ts) {
  return locked(a, [&] {
    if (!a->ast.playback) return;
    stage_record(a, NFA_TICK, -1, ts, 0);
  });
}

int sm_app_advance_wallclock(sm_app* a, int64_t ts) {
  return locked(a, [&] {
    if (!a->ast.playback) return;
    stage_record(a, NFA_WALL, -1, ts, 1);
  });
}

int sm_app_add_stream_callback(sm_app* a, const char* stream_id, sm_stream_callback cb, void* user) {
  std::lock_guard<std::mutex> g(a->mu);
  return guarded([&] {
    Callback c;
    c.scb = cb;
    c.user = user;
    a->stream_cbs[stream_id].push_back(c);
  });
}

int sm_app_add_stream_columns_callback(sm_app* a, const char* stream_id, sm_stream_columns_callback cb, void* user) {
  std::lock_guard<std::mutex> g(a->mu);
  return guarded([&] {
    const int s = sm::stream_index(a->ast, stream_id);
    if (s >= 0) {
      const auto& attrs = a->ast.streams[s].attrs;
      if (attrs.size() > 8) throw sql::UnsupportedError("columns callbacks take streams of at most 8 attributes");
      for (auto& at : attrs)
        if (at.type == sql::AttrType::STRING)
          throw sql::UnsupportedError("columns callbacks take streams without STRING attributes");
    }
    Callback c;
    c.ccb = cb;
    c.user = user;
    a->stream_cbs[stream_id].push_back(c);
  });
}

void sm_count_columns_callback(void* user, size_t n, const int64_t* ts, const int64_t* values, const uint8_t* null_bits,
                               int32_t nsel) {
  (void)ts;
  (void)values;
  (void)null_bits;
  (void)nsel;
  *(int64_t*)user += (int64_t)n;
}

int sm_app_add_query_callback(sm_app* a, const char* query_name, sm_query_callback cb, void* user) {
  std::lock_guard<std::mutex> g(a->mu);
  return guarded([&] {
    bool found = false;
    for (auto& q : a->queries)
      if (q->cq.name == query_name) found = true;
    if (!found) throw sql::ValidationError(std::string("No query with name ") + query_name + " exists");
    Callback c;
    c.qcb = cb;
    c.user = user;
    a->query_cbs[query_name].push_back(c);
  });
}

int sm_app_set_collect(sm_app* a, int collect) {
  std::lock_guard<std::mutex> g(a->mu);
  a->collect = collect != 0;
  return SM_OK;
}

size_t sm_app_dump_outputs(sm_app* a, char* buf, size_t len) {
  std::lock_guard<std::mutex> g(a->mu);
  std::string s = dump_json(a);
  if (buf && len > s.size()) {
    memcpy(buf, s.data(), s.size());
    buf[s.size()] = 0;
  }
  return s.size();
}

int sm_app_set_option(sm_app* a, const char* key, int64_t value) {
  std::lock_guard<std::mutex> g(a->mu);
  return guarded([&] {
    std::string k = key ? key : "";
    if (k == "heap_words") {
      for (auto& q : a->queries)
        if (q->state_slots) throw std::runtime_error("heap_words must be set before the first flush");
      a->heap_half = (int32_t)std::max<int64_t>(256, value);
    } else if (k == "pool_words") {
      a->pool_init = std::max<int64_t>(1 << 16, value);
    } else if (k == "fast_general") {
      a->force_general_fast = value != 0;
    } else if (k == "fast_stack") {
      a->fast_stack = (int)std::min<int64_t>(std::max<int64_t>(value, 0), 2);
    } else if (k == "fast_timing") {
      if (value && !a->fast_tm_ready) {
        for (auto& e : a->fast_tm.ev) SM_HIP(hipEventCreate(&e));
        for (auto& e : a->fast_tm.mk) SM_HIP(hipEventCreate(&e));
        a->fast_tm_ready = true;
      }
      a->fast_timing = value != 0;
    } else if (k == "lane_balance") {
      a->lane_balance = value;
    } else if (k == "nfa_jit") {
      a->nfa_jit = value < 0 ? -1 : (value != 0);
    } else if (k == "reset") {
      // drop every partition instance, partial match, pending timer and the playback clock, keeping the device
      // allocations: the state of a freshly created runtime of the same app (bench / test helper)
      a->ev_stream.clear();
      a->ev_row.clear();
      a->ev_ts.clear();
      a->ev_clock.clear();
      a->ev_ord.clear();
      a->adv_pos.clear();
      a->adv_clock.clear();
      a->adv_wall.clear();
      for (auto& st : a->streams) st.clear();
      for (auto& q : a->queries) {
        if (q->keys.tslots) SM_HIP(hipMemsetAsync(q->keys.tslots, 0, (size_t)q->keys.cap * 4, a->stream));
        q->keys.nslots = 0;
        if (q->state_slots) SM_HIP(hipMemsetAsync(q->ks.p, 0, (size_t)q->state_slots * q->cq.hdr.ks_words * 8, a->stream));
        if (q->pool_top_dev.p) SM_HIP(hipMemsetAsync(q->pool_top_dev.p, 0, 8, a->stream));
        q->pool_used = 0;
        q->dev_n = 0;
        q->carry.reset();
        q->dense.clear(a->stream);
        q->remap = 0;
      }
      SM_HIP(hipStreamSynchronize(a->stream));
      a->clock = a->clock_batch_in = 0;
      a->next_ordinal = a->ordinal_base = 0;
      for (double& t : a->host_ms) t = 0;
      a->started = false;
      a->failed = false;
      a->failed_why.clear();
      for (auto& q : a->queries) q->nfa_used = q->nfa_mode = false;
      for (auto& k : a->part_keys) k.clear();
      for (auto& k : a->part_key_types) k.clear();
      for (auto& k : a->part_key_set) k.clear();
      if (value) {  // reset and start again
        a->started = true;
        stage_record(a, NFA_START, -1, a->clock, 0);
      }
    } else if (k == "output_records") {
      a->out_records = std::max<int64_t>(0, value);
    } else if (k == "key_remap") {
      a->key_remap = value < 0 ? -1 : (value != 0);
    } else if (k == "keep_outputs") {
      a->keep_outputs = value != 0;
    } else if (k == "bulk_min") {
      a->bulk_min = std::max<int64_t>(1, value);
    } else if (k == "bulk_chunk") {
      a->bulk_chunk = std::max<int64_t>(1, value);
    } else if (k == "batch_events") {
      a->batch_events = std::max<int64_t>(1, value);
    } else {
      throw std::invalid_argument("unknown option " + k);
    }
  });
}

int sm_app_process_device_batch(sm_app* a, const char* stream_id, size_t n, const int64_t* d_ts,
                                const void* const* d_cols, const int64_t* d_ordinals, int64_t ordinal_base,
                                void* hip_stream) {
  return locked(a, [&] {
    int s = stream_index(a->ast, stream_id ? stream_id : "");
    if (s < 0) throw sql::ValidationError("unknown stream");
    flush(a);  // staged host events come first (arrival order)
    hipStream_t hs = hip_stream ? (hipStream_t)hip_stream : a->stream;
    // no stream given: the batch may still be in the making on any stream of the caller (the app's own stream does
    // not wait for the legacy default stream), so all device work completes before it is read
    if (!hip_stream) SM_HIP(hipDeviceSynchronize());
    std::vector<HostOut> douts;               // this batch's outputs for their consumers: NFA records
    std::vector<DevOut> draw;                 // and host copies of closed-form / filter device outputs
    a->out_arena.clear();
    try {
      device_batch_stream(a, s, n, d_ts, d_cols, d_ordinals, ordinal_base, hs, douts, draw);
      deliver_device(a, douts, draw);
    } catch (const std::exception& e) {
      a->failed = true;
      a->failed_why = std::string("a device batch failed half-way (") + e.what() +
                      "); the matching state is inconsistent: restore a snapshot or reset the app";
      throw;
    }
  });
}

// Interleaved multi-stream batch already resident in HBM: the device form of a sequence of InputHandler.send
// calls (InputHandler.java:53 → StreamJunction.sendData :232) over streams that share one schema. Staged host
// events are flushed first, so arrival order across both entry points is kept. Pattern / sequence queries run
// through the general NFA kernel exactly as in flush(); outputs are delivered to callbacks in reference order.
int sm_app_process_device_events(sm_app* a, size_t n, const int32_t* d_stream_idx, const int64_t* d_ts,
                                 const void* const* d_cols, const int64_t* d_ordinals, int64_t ordinal_base,
                                 void* hip_stream) {
  return locked(a, [&] {
    flush(a);
    if (n == 0) return;
    if (a->max_level > 0)
      throw sql::UnsupportedError("apps whose queries read streams other queries fill run through the host API");
    for (auto& bc : a->part_bcast)
      if (!bc.empty()) throw sql::UnsupportedError("partitions reading unkeyed streams run through the host API");
    hipStream_t hs = hip_stream ? (hipStream_t)hip_stream : a->stream;
    // no stream given: the batch may still be in the making on any stream of the caller (the app's own stream does
    // not wait for the legacy default stream), so all device work completes before it is read
    if (!hip_stream) SM_HIP(hipDeviceSynchronize());
    // every stream a query reads must carry the batch schema (the schema of the first such stream)
    const std::vector<sql::Attribute>* schema = nullptr;
    for (auto& qp : a->queries) {
      if (qp->cq.hdr.kind == 0)
        throw sql::UnsupportedError("interleaved device batches run pattern / sequence queries; filter query '" +
                                    qp->cq.name + "' takes sm_app_process_device_batch");
      for (int s : qp->cq.streams) {
        const auto& at = a->streams[s].def->attrs;
        if (!schema) schema = &at;
        bool same = at.size() == schema->size();
        for (size_t k = 0; same && k < at.size(); ++k) same = at[k].type == (*schema)[k].type;
        if (!same)
          throw sql::ValidationError("stream '" + a->streams[s].def->id +
                                     "' does not share the interleaved batch schema");
      }
    }
    if (!schema) return;
    std::vector<NfaStream> nst(a->streams.size());
    for (size_t s = 0; s < a->streams.size(); ++s) {
      NfaStream& d = nst[s];
      memset(&d, 0, sizeof(d));
      const auto& at = a->streams[s].def->attrs;
      bool same = at.size() == schema->size();
      for (size_t k = 0; same && k < at.size(); ++k) same = at[k].type == (*schema)[k].type;
      if (!same) continue;  // never read: no query of this app selects it
      d.nattr = (int)at.size();
      for (int k = 0; k < d.nattr; ++k) {
        d.types[k] = (int)at[k].type;
        d.cols[k] = d_cols[k];
      }
    }
    a->d_streams.ensure(nst.size() * sizeof(NfaStream));
    SM_HIP(hipMemcpyAsync(a->d_streams.p, nst.data(), nst.size() * sizeof(NfaStream), hipMemcpyHostToDevice, hs));
    const int64_t N = (int64_t)n;
    for (DBuf* d : {&a->d_ev_row, &a->d_ev_clock, &a->d_ev_ord, &a->d_adv_pos, &a->d_adv_clock, &a->d_adv_wall,
                    &a->d_adv_upto})
      d->ensure((size_t)N * 8);
    a->d_err.ensure(16);
    a->d_count.ensure(16);
    ensure_scratch(a, batch_scratch(a, N));
    a->sc.used = 0;
    FastTimings* tm = a->fast_timing ? &a->fast_tm : nullptr;
    if (tm) {
      tm->nmk = 0;
      tm->mark("start", hs);
    }
    int64_t clock_out = a->clock;
    const int64_t nadv = build_event_index(
        N, d_stream_idx, (int32_t)a->streams.size(), d_ts, d_ordinals, ordinal_base, a->ast.playback, a->clock,
        nullptr /* rows = positions */, d_ordinals ? nullptr : (int64_t*)a->d_ev_ord.p /* given ordinals are read in place */,
        (int64_t*)a->d_ev_clock.p, (int64_t*)a->d_adv_pos.p, (int64_t*)a->d_adv_clock.p, (int64_t*)a->d_adv_wall.p,
        (int64_t*)a->d_adv_upto.p, &clock_out, a->sc, hs);
    if (tm) tm->mark("event_index", hs);
    // the event ordinals: the caller's array when given (a heartbeat's entry is never read as an event's ordinal)
    const EvArrays ev{d_stream_idx, nullptr, d_ts, (const int64_t*)a->d_ev_clock.p,
                      d_ordinals ? d_ordinals : (const int64_t*)a->d_ev_ord.p, (const NfaStream*)a->d_streams.p,
                      (const int64_t*)a->d_adv_pos.p,
                      (const int64_t*)a->d_adv_clock.p, (const int64_t*)a->d_adv_wall.p, (const int64_t*)a->d_adv_upto.p,
                      nadv, a->clock};
    std::vector<HostOut> outs;
    a->in_device_events = true;
    struct Reset {
      bool& f;
      ~Reset() { f = false; }
    } reset_in{a->in_device_events};
    for (size_t qi = 0; qi < a->queries.size(); ++qi) {
      a->sc.used = 0;
      a->queries[qi]->n_out = 0;
      a->queries[qi]->ev_out_n = 0;
      run_pattern_query(a, (int)qi, ev, N, outs, hs, tm);
      a->queries[qi]->dev_n = a->queries[qi]->n_out;
    }
    a->clock = clock_out;
    a->clock_batch_in = a->clock;
    if (!d_ordinals) a->next_ordinal = std::max<int64_t>(a->next_ordinal, ordinal_base + N);
    deliver(a, outs);
  });
}

// ---- persistence: SiddhiAppRuntime.snapshot() :548 / restore(byte[]) :560 (core/SiddhiAppRuntime.java). The
// snapshot holds what the reference's Snapshotables hold for the hot path: every partition instance (key table),
// each instance's pending / new-and-every partial matches with their event chains (per-key state words + heap,
// StreamPreStateProcessor.currentState :339-353), pending scheduler timers (Scheduler.currentState), the
// playback clock and the arrival ordinal, plus the string dictionary the device values refer to. Closed-form
// queries fed by device batches keep their open partials as carry rows instead (FastCarry): those rows, the
// last batch's event time and the query's hand-over flags are part of the snapshot too. Staged events are flushed
// first, so the snapshot is taken at a batch boundary.

int sm_app_snapshot(sm_app* a, uint8_t* buf, size_t cap, size_t* len) {
  return locked(a, [&] {
    flush(a);
    SnapWriter w;
    w.raw(kSnapMagic, 8);
    w.put<uint64_t>(a->text_hash);
    w.put<int64_t>(a->clock);
    w.put<int64_t>(a->clock_batch_in);
    w.put<int64_t>(a->next_ordinal);
    w.put<int64_t>(a->ordinal_base);
    w.put<uint8_t>(a->started);
    w.put<int32_t>(a->heap_half);
    w.put<uint32_t>((uint32_t)a->dict.strs.size());
    for (auto& str : a->dict.strs) {
      w.put<uint32_t>((uint32_t)str.size());
      w.raw(str.data(), str.size());
    }
    w.put<uint32_t>((uint32_t)a->part_keys.size());  // partition instances (broadcast targets), creation order
    for (size_t pi = 0; pi < a->part_keys.size(); ++pi) {
      const auto& k = a->part_keys[pi];
      w.put<uint64_t>(k.size());
      w.raw(k.data(), k.size() * 8);
      w.raw(a->part_key_types[pi].data(), k.size() * 4);
    }
    w.put<uint32_t>((uint32_t)a->queries.size());
    const size_t heap_words = 2 * (size_t)a->heap_half + 64;
    for (auto& qp : a->queries) {
      QueryRt& q = *qp;
      const int32_t n = q.cq.hdr.kind == 0 ? 0 : q.keys.nslots ? q.keys.nslots : (int32_t)std::min<int64_t>(q.state_slots, 1);
      const int32_t kw = q.cq.hdr.ks_words;
      w.put<int32_t>(q.cq.hdr.partitioned ? q.keys.nslots : -1);
      w.put<int32_t>(n);
      w.put<int32_t>(kw);
      if (q.cq.hdr.partitioned && q.keys.nslots) {
        std::vector<int64_t> keys(q.keys.nslots);
        SM_HIP(hipMemcpy(keys.data(), q.keys.slot_keys, keys.size() * 8, hipMemcpyDeviceToHost));
        w.raw(keys.data(), keys.size() * 8);
      }
      if (n > 0) {
        // per-key state words: lane-interleaved with stride state_slots on the device, packed to stride n here
        std::vector<int64_t> ks((size_t)n * kw);
        SM_HIP(hipMemcpy2D(ks.data(), (size_t)n * 8, q.ks.p, (size_t)q.state_slots * 8, (size_t)n * 8, (size_t)kw,
                           hipMemcpyDeviceToHost));
        w.raw(ks.data(), ks.size() * 8);
        std::vector<int64_t> heap((size_t)n * heap_words);
        SM_HIP(hipMemcpy(heap.data(), q.heap.p, heap.size() * 8, hipMemcpyDeviceToHost));
        w.raw(heap.data(), heap.size() * 8);
      }
      // the overflow pool's used prefix (promoted keys' heaps, addressed by pool offset)
      const uint64_t pu = std::min<uint64_t>(q.pool_used, (uint64_t)q.pool_words);
      w.put<uint64_t>(pu);
      if (pu) {
        std::vector<int64_t> pool(pu);
        SM_HIP(hipMemcpy(pool.data(), q.pool.p, pu * 8, hipMemcpyDeviceToHost));
        w.raw(pool.data(), pu * 8);
      }
      w.put<uint8_t>((uint8_t)(q.nfa_used | (q.nfa_mode << 1) | (q.carry.active << 2)));
      w.put<int32_t>(q.remap);  // dense key ids: the id -> key array (the carry's keys are ids)
      w.put<int64_t>(q.dense.nslots);
      if (q.dense.nslots) {
        std::vector<int64_t> keys((size_t)q.dense.nslots);
        SM_HIP(hipMemcpy(keys.data(), q.dense.slot_keys, keys.size() * 8, hipMemcpyDeviceToHost));
        w.raw(keys.data(), keys.size() * 8);
      }
      w.put<int64_t>(q.carry.ts_last);
      w.put<int64_t>(q.carry.n);
      w.put<int32_t>(q.carry.width);
      if (q.carry.n > 0) {
        std::vector<int64_t> rows((size_t)q.carry.n * q.carry.width);
        SM_HIP(hipMemcpy(rows.data(), q.carry.rows, rows.size() * 8, hipMemcpyDeviceToHost));
        w.raw(rows.data(), rows.size() * 8);
      }
    }
    *len = w.b.size();
    if (buf && cap >= w.b.size()) memcpy(buf, w.b.data(), w.b.size());
    else if (buf) throw std::invalid_argument("snapshot buffer too small");
  });
}

int sm_app_restore(sm_app* a, const uint8_t* buf, size_t len) {
  std::lock_guard<std::mutex> g(a->mu);
  return guarded([&] {
    SnapReader r{buf, len};
    char magic[8];
    r.raw(magic, 8);
    if (memcmp(magic, kSnapMagic, 8) != 0) throw std::runtime_error("CannotRestoreSiddhiAppStateException: not a snapshot");
    if (r.get<uint64_t>() != a->text_hash)
      throw std::runtime_error("CannotRestoreSiddhiAppStateException: snapshot of a different Siddhi app");
    // drop staged records (a START marker included): the snapshot's state replaces them
    a->ev_stream.clear();
    a->ev_row.clear();
    a->ev_ts.clear();
    a->ev_clock.clear();
    a->ev_ord.clear();
    a->adv_pos.clear();
    a->adv_clock.clear();
    a->adv_wall.clear();
    for (auto& st : a->streams) st.clear();
    a->failed = false;
    a->failed_why.clear();
    for (auto& q : a->queries) q->carry.reset();
    a->clock = r.get<int64_t>();
    a->clock_batch_in = r.get<int64_t>();
    a->next_ordinal = r.get<int64_t>();
    a->ordinal_base = r.get<int64_t>();
    a->started = r.get<uint8_t>() != 0;
    const int32_t half = r.get<int32_t>();
    const uint32_t nd = r.get<uint32_t>();
    Dict d;
    for (uint32_t i = 0; i < nd; ++i) {
      std::string str(r.get<uint32_t>(), '\0');
      r.raw(&str[0], str.size());
      d.intern(str);
    }
    for (size_t i = 0; i < a->dict.strs.size(); ++i)  // ids baked into the compiled plan must agree
      if (i >= d.strs.size() || d.strs[i] != a->dict.strs[i])
        throw std::runtime_error("CannotRestoreSiddhiAppStateException: string dictionary mismatch");
    a->dict = d;
    if (r.get<uint32_t>() != a->part_keys.size()) throw std::runtime_error("CannotRestoreSiddhiAppStateException: plan mismatch");
    for (size_t pi = 0; pi < a->part_keys.size(); ++pi) {
      a->part_keys[pi].resize(r.get<uint64_t>());
      r.raw(a->part_keys[pi].data(), a->part_keys[pi].size() * 8);
      a->part_key_types[pi].resize(a->part_keys[pi].size());
      r.raw(a->part_key_types[pi].data(), a->part_keys[pi].size() * 4);
      a->part_key_set[pi] = std::unordered_set<int64_t>(a->part_keys[pi].begin(), a->part_keys[pi].end());
    }
    if (r.get<uint32_t>() != a->queries.size())
      throw std::runtime_error("CannotRestoreSiddhiAppStateException: query count mismatch");
    for (auto& qp : a->queries)
      if (qp->state_slots && half != a->heap_half)
        throw std::runtime_error("CannotRestoreSiddhiAppStateException: heap_words differs from the running app");
    a->heap_half = half;
    const size_t heap_words = 2 * (size_t)a->heap_half + 64;
    for (auto& qp : a->queries) {
      QueryRt& q = *qp;
      const int32_t nkeys = r.get<int32_t>();
      const int32_t n = r.get<int32_t>();
      const int32_t kw = r.get<int32_t>();
      if (kw != q.cq.hdr.ks_words) throw std::runtime_error("CannotRestoreSiddhiAppStateException: plan mismatch");
      if (nkeys >= 0) {
        std::vector<int64_t> keys(nkeys);
        r.raw(keys.data(), keys.size() * 8);
        q.keys.load(keys.data(), nkeys, a->stream);
      }
      if (n > 0) {
        ensure_state(a, q, n);
        std::vector<int64_t> ks((size_t)n * kw);
        r.raw(ks.data(), ks.size() * 8);
        SM_HIP(hipMemset(q.ks.p, 0, (size_t)q.state_slots * kw * 8));
        SM_HIP(hipMemcpy2D(q.ks.p, (size_t)q.state_slots * 8, ks.data(), (size_t)n * 8, (size_t)n * 8, (size_t)kw,
                           hipMemcpyHostToDevice));
        std::vector<int64_t> heap((size_t)n * heap_words);
        r.raw(heap.data(), heap.size() * 8);
        SM_HIP(hipMemcpy(q.heap.p, heap.data(), heap.size() * 8, hipMemcpyHostToDevice));
      } else if (q.state_slots) {
        SM_HIP(hipMemset(q.ks.p, 0, (size_t)q.state_slots * kw * 8));
      }
      const uint64_t pu = r.get<uint64_t>();
      if (pu) {
        std::vector<int64_t> pool(pu);
        r.raw(pool.data(), pu * 8);
        ensure_pool(a, q, std::max<int64_t>(a->pool_init, 2 * (int64_t)pu), 0);
        SM_HIP(hipMemcpy(q.pool.p, pool.data(), pu * 8, hipMemcpyHostToDevice));
      } else {
        ensure_pool(a, q, 0, 0);
      }
      q.pool_used = pu;
      SM_HIP(hipMemcpy(q.pool_top_dev.p, &q.pool_used, 8, hipMemcpyHostToDevice));
      const uint8_t fl = r.get<uint8_t>();
      q.nfa_used = fl & 1;
      q.nfa_mode = (fl >> 1) & 1;
      q.carry.reset();
      q.carry.active = (fl >> 2) & 1;
      q.remap = r.get<int32_t>();
      const int64_t nd = r.get<int64_t>();
      if (q.remap < 0 || q.remap > 2 || nd < 0 || nd > INT32_MAX)
        throw std::runtime_error("CannotRestoreSiddhiAppStateException: bad key ids");
      std::vector<int64_t> dkeys((size_t)nd);
      if (nd) r.raw(dkeys.data(), (size_t)nd * 8);
      q.dense.load(dkeys.data(), nd, a->stream);
      q.carry.ts_last = r.get<int64_t>();
      const int64_t cn = r.get<int64_t>();
      const int32_t cw = r.get<int32_t>();
      if (cn < 0 || cw < 0 || (cn > 0 && cw < 3)) throw std::runtime_error("CannotRestoreSiddhiAppStateException: bad carry");
      if (cn > 0) {
        std::vector<int64_t> rows((size_t)cn * cw);
        r.raw(rows.data(), rows.size() * 8);
        q.carry.reserve(cn, cw);
        SM_HIP(hipMemcpy(q.carry.rows, rows.data(), rows.size() * 8, hipMemcpyHostToDevice));
        q.carry.n = cn;
      }
      q.carry.width = cw;
    }
    if (r.o != len) throw std::runtime_error("CannotRestoreSiddhiAppStateException: trailing bytes");
  });
}

}  // extern "C"

// Scratch of the app-less multi-GPU helpers, one per device (a process may drive several devices).
namespace {
struct HelperScratch {
  std::mutex mu;
  sm::DBuf buf;
  sm::Scratch sc;
};

HelperScratch& helper_scratch(size_t need) {
  static std::mutex mu;
  static std::map<int, std::unique_ptr<HelperScratch>> per_dev;
  int dev = 0;
  SM_HIP(hipGetDevice(&dev));
  HelperScratch* h;
  {
    std::lock_guard<std::mutex> g(mu);
    auto& p = per_dev[dev];
    if (!p) p = std::make_unique<HelperScratch>();
    h = p.get();
  }
  h->mu.lock();  // released by the caller (HelperLock)
  if (h->buf.cap < need) h->buf.ensure(need);
  h->sc.base = (char*)h->buf.p;
  h->sc.cap = h->buf.cap;
  h->sc.used = 0;
  return *h;
}

struct HelperLock {
  HelperScratch& h;
  ~HelperLock() { h.mu.unlock(); }
};
}  // namespace

extern "C" {

// Multi-GPU key exchange helper (no app handle): stable partition of a device batch by owner rank.
int sm_partition_by_owner(const void* d_keys, int key_width, size_t n, uint32_t world, int ncols,
                          const int32_t* widths, const int32_t* strides, const void* const* d_src,
                          void* const* d_dst, uint64_t* counts, void* hip_stream) {
  return guarded([&] {
    if (ncols < 0 || ncols > sm::kMaxPartCols) throw std::invalid_argument("ncols out of range");
    if (key_width != 4 && key_width != 8)
      throw std::invalid_argument("key width must be 4 or 8 bytes (widen narrower integer keys)");
    sm::PartCols pc{};
    pc.n = ncols;
    for (int c = 0; c < ncols; ++c) {
      if (widths[c] != 1 && widths[c] != 2 && widths[c] != 4 && widths[c] != 8)
        throw std::invalid_argument("column width must be 1, 2, 4 or 8 bytes");
      const int32_t st = strides ? strides[c] : widths[c];
      if (st < widths[c]) throw std::invalid_argument("column stride smaller than its width");
      if (((uintptr_t)d_dst[c] | (uintptr_t)st) % widths[c])
        throw std::invalid_argument("packed field not aligned to its width");
      pc.width[c] = widths[c];
      pc.stride[c] = st;
      pc.src[c] = d_src[c];
      pc.dst[c] = d_dst[c];
    }
    HelperScratch& h = helper_scratch((size_t)world * ((n + 4095) / 4096 + 1) * 4 + (16 << 20));
    HelperLock lk{h};
    sm::partition_by_owner(d_keys, key_width, (int64_t)n, world, pc, counts, h.sc, (hipStream_t)hip_stream);
  });
}

int sm_merge_heartbeats(size_t n, const int64_t* d_ord, const int32_t* d_sid, const int64_t* d_ts, int ncols,
                        const int32_t* widths, const void* const* d_src, size_t m, const int64_t* d_tick_ord,
                        const int64_t* d_tick_ts, int32_t* d_sid_out, int64_t* d_ts_out, int64_t* d_ord_out,
                        void* const* d_dst, size_t* n_out, void* hip_stream) {
  return guarded([&] {
    if (ncols < 0 || ncols > sm::kMaxPartCols) throw std::invalid_argument("ncols out of range");
    sm::MergeOut o{};
    o.ncols = ncols;
    for (int c = 0; c < ncols; ++c) {
      o.width[c] = widths[c];
      o.src[c] = d_src[c];
      o.dst[c] = d_dst[c];
    }
    o.sid = d_sid_out;
    o.ts = d_ts_out;
    o.ord = d_ord_out;
    HelperScratch& h = helper_scratch((size_t)m * 4 + (16 << 20));
    HelperLock lk{h};
    *n_out = (size_t)sm::merge_heartbeats(d_ord, d_sid, d_ts, (int64_t)n, d_tick_ord, d_tick_ts, (int64_t)m, o, h.sc,
                                          (hipStream_t)hip_stream);
  });
}

int sm_unpack_records(const void* d_rec, size_t m, int rec_bytes, int ncols, const int32_t* offsets,
                      const int32_t* widths, void* const* d_dst, int ord_field, int nsrc, const uint64_t* run_counts,
                      const int64_t* src_first, int64_t* d_ordinals, void* hip_stream) {
  return guarded([&] {
    if (ncols < 0 || ncols > sm::kMaxPartCols) throw std::invalid_argument("ncols out of range");
    if (rec_bytes <= 0 || rec_bytes > 64 || rec_bytes % 8) throw std::invalid_argument("record size must be 8..64 bytes, a multiple of 8");
    if ((uintptr_t)d_rec % 8) throw std::invalid_argument("record buffer not 8-byte aligned");
    sm::UnpackCols u{};
    u.n = ncols;
    u.rec_words = rec_bytes / 8;
    for (int c = 0; c < ncols; ++c) {
      if (widths[c] != 1 && widths[c] != 2 && widths[c] != 4 && widths[c] != 8)
        throw std::invalid_argument("field width must be 1, 2, 4 or 8 bytes");
      if (offsets[c] < 0 || offsets[c] + widths[c] > rec_bytes || offsets[c] % widths[c])
        throw std::invalid_argument("field outside the record or not aligned to its width");
      u.off[c] = offsets[c];
      u.width[c] = widths[c];
      u.dst[c] = d_dst ? d_dst[c] : nullptr;
    }
    u.ord_field = -1;
    if (ord_field >= 0) {
      if (ord_field >= ncols || widths[ord_field] != 4) throw std::invalid_argument("ordinal field must be a 4-byte field");
      if (nsrc <= 0 || nsrc > sm::kMaxOwners || !run_counts || !src_first || !d_ordinals)
        throw std::invalid_argument("ordinal field needs 1..64 source runs, their first ordinals and an output");
      uint64_t end = 0;
      for (int r = 0; r < nsrc; ++r) {
        end += run_counts[r];
        u.run_end[r] = (int64_t)end;
        u.src_first[r] = src_first[r];
      }
      if (end != m) throw std::invalid_argument("source run counts do not add up to the record count");
      u.ord_field = ord_field;
      u.nsrc = nsrc;
      u.ord_out = d_ordinals;
    }
    sm::unpack_records((const uint64_t*)d_rec, (int64_t)m, u, (hipStream_t)hip_stream);
    SM_HIP(hipGetLastError());
  });
}

int sm_order_matches(const uint64_t* d_pairs, size_t n, int64_t lo, int64_t hi, uint64_t* d_out, void* hip_stream) {
  return guarded([&] {
    if (n == 0) return;
    if (d_pairs == d_out) throw std::invalid_argument("order_matches: output must not alias the input");
    HelperScratch& h = helper_scratch((size_t)std::max<int64_t>(hi - lo, 0) * 4 + (16 << 20));
    HelperLock lk{h};
    sm::order_matches(d_pairs, (int64_t)n, lo, hi, d_out, h.sc, (hipStream_t)hip_stream);
  });
}

// Multi-GPU output merge (siddhi_amd/shard.py order_outputs): runs of output records, each in delivery order, into
// the reference's delivery order. Records as sm_app_copy_device_outputs writes them (pos = trigger ordinal).
static_assert(sizeof(sm_out_rec) == sizeof(sm::OutRec) && offsetof(sm_out_rec, phase) == offsetof(sm::OutRec, phase),
              "sm_out_rec mirrors the device output record");

int sm_order_outputs(const void* d_recs, size_t n, size_t stride, void* d_out, void* hip_stream) {
  return guarded([&] {
    if (n == 0) return;
    if (stride < sizeof(sm::OutRec) || stride % 8) throw std::invalid_argument("order_outputs: bad record stride");
    if (d_recs == d_out) throw std::invalid_argument("order_outputs: output must not alias the input");
    HelperScratch& h = helper_scratch(n * 48 + (32 << 20));
    HelperLock lk{h};
    sm::order_outputs((const char*)d_recs, (int64_t)n, (uint32_t)stride, nullptr, h.sc, (hipStream_t)hip_stream, 62,
                      (char*)d_out);
    SM_HIP(hipStreamSynchronize((hipStream_t)hip_stream));
  });
}

int sm_app_copy_device_outputs(sm_app* a, const char* query_name, void* d_dst, size_t cap_bytes, size_t* n,
                               size_t* stride, void* hip_stream) {
  std::lock_guard<std::mutex> g(a->mu);
  return guarded([&] {
    if (!a->keep_outputs) throw std::invalid_argument("copy_device_outputs needs option keep_outputs = 1");
    for (auto& q : a->queries)
      if (q->cq.name == query_name) {
        const size_t st = sizeof(OutRec) + q->cq.hdr.nsel * sizeof(DVal) + q->cq.hdr.nrefs * sizeof(int64_t);
        const size_t bytes = (size_t)q->ev_out_n * st;
        *n = (size_t)q->ev_out_n;
        if (stride) *stride = st;
        if (!d_dst) return;
        if (bytes > cap_bytes) throw std::invalid_argument("copy_device_outputs: destination too small");
        if (bytes) SM_HIP(hipMemcpyAsync(d_dst, q->ev_out.p, bytes, hipMemcpyDeviceToDevice, (hipStream_t)hip_stream));
        return;
      }
    throw sql::ValidationError(std::string("No query with name ") + query_name);
  });
}

int sm_app_get_stat(sm_app* a, const char* key, double* out) {
  std::lock_guard<std::mutex> g(a->mu);
  return guarded([&] {
    std::string k = key ? key : "";
    if (k.rfind("output_events:", 0) == 0) {  // output events of the last device batch
      for (auto& q : a->queries)
        if (q->cq.name == k.substr(14)) {
          *out = (double)q->dev_n;
          return;
        }
      throw sql::ValidationError("No query with name " + k.substr(14));
    }
    if (k.rfind("nfa_state:", 0) == 0) {  // 1 = the query's matching state is held by the NFA kernel from now on
      for (auto& q : a->queries)
        if (q->cq.name == k.substr(10)) {
          *out = (q->nfa_mode || q->nfa_used) ? 1.0 : 0.0;
          return;
        }
      throw sql::ValidationError("No query with name " + k.substr(10));
    }
    if (k.rfind("nfa_kernel:", 0) == 0) {  // 1 = query-specialised kernel, 2 = interpreter, 0 = not run
      for (auto& q : a->queries)
        if (q->cq.name == k.substr(11)) {
          *out = q->nfa_kernel_used;
          return;
        }
      throw sql::ValidationError("No query with name " + k.substr(11));
    }
    for (const char* pk : {"pool_words:", "pool_used:", "pool_compactions:", "pool_refused:"}) {  // overflow pool
      const std::string pre = pk;
      if (k.rfind(pre, 0) == 0) {
        for (auto& q : a->queries)
          if (q->cq.name == k.substr(pre.size())) {
            *out = pre == "pool_words:" ? (double)q->pool_words
                 : pre == "pool_used:"  ? (double)q->pool_used
                 : pre == "pool_refused:" ? (double)q->pool_refused
                                        : (double)q->pool_compactions;
            return;
          }
        throw sql::ValidationError("No query with name " + k.substr(pre.size()));
      }
    }
    if (k.rfind("fast_path:", 0) == 0) {
      for (auto& q : a->queries)
        if (q->cq.name == k.substr(10)) {
          *out = q->fast_path_used;
          return;
        }
      throw sql::ValidationError("No query with name " + k.substr(10));
    }
    if (k == "fast_ms:group" || k == "fast_ms:walk" || k == "fast_ms:order") {
      if (!a->fast_tm_ready) throw std::invalid_argument("fast_timing option is off");
      int i = k == "fast_ms:group" ? 0 : k == "fast_ms:walk" ? 1 : 2;
      float ms = 0;
      SM_HIP(hipEventElapsedTime(&ms, a->fast_tm.ev[i], a->fast_tm.ev[i + 1]));
      *out = ms;
      return;
    }
    // per-kernel totals of the last device batch: "kernel_ms:<label>" / "kernel_calls:<label>" (fast_timing)
    if (k.rfind("kernel_ms:", 0) == 0 || k.rfind("kernel_calls:", 0) == 0) {
      if (!a->fast_tm_ready) throw std::invalid_argument("fast_timing option is off");
      const bool calls = k[7] == 'c';
      const std::string label = k.substr(calls ? 13 : 10);
      double tot = 0;
      int cnt = 0;
      for (int i = 1; i < a->fast_tm.nmk; ++i)
        if (label == a->fast_tm.label[i]) {
          float ms = 0;
          SM_HIP(hipEventElapsedTime(&ms, a->fast_tm.mk[i - 1], a->fast_tm.mk[i]));
          tot += ms;
          ++cnt;
        }
      *out = calls ? cnt : tot;
      return;
    }
    if (k.rfind("host_ms:", 0) == 0) {
      static const char* names[5] = {"device", "outputs", "deliver", "callbacks", "upload_wait"};
      for (int i = 0; i < 5; ++i)
        if (k.substr(8) == names[i]) {
          *out = a->host_ms[i];
          return;
        }
    }
    throw std::invalid_argument("unknown stat " + k);
  });
}

int sm_app_copy_device_matches(sm_app* a, const char* query_name, void* d_dst, size_t cap_bytes, size_t* n,
                               void* hip_stream) {
  std::lock_guard<std::mutex> g(a->mu);
  return guarded([&] {
    for (auto& q : a->queries)
      if (q->cq.name == query_name) {
        const size_t bytes = (size_t)q->dev_n * (q->cq.hdr.kind == 0 ? 4 : 8);
        if (bytes > cap_bytes) throw std::invalid_argument("copy_device_matches: destination too small");
        if (bytes) SM_HIP(hipMemcpyAsync(d_dst, q->dev_pairs.p, bytes, hipMemcpyDeviceToDevice, (hipStream_t)hip_stream));
        *n = (size_t)q->dev_n;
        return;
      }
    throw sql::ValidationError(std::string("No query with name ") + query_name);
  });
}

// QuerySelector.processNoGroupBy (core/query/selector/QuerySelector.java:124-167) for the outputs of the last
// closed-form device batch, on the device: the select list of each (e1, e2) match, in output order.
int sm_app_device_project(sm_app* a, const char* query_name, sm_dval* d_values, size_t cap_values, int64_t* d_ts,
                          size_t* n, int32_t* nsel, void* hip_stream) {
  static_assert(sizeof(sm_dval) == sizeof(DVal), "sm_dval mirrors the device value");
  return locked(a, [&] {
    QueryRt* q = nullptr;
    for (auto& qp : a->queries)
      if (qp->cq.name == query_name) q = qp.get();
    if (!q) throw sql::ValidationError(std::string("No query with name ") + query_name);
    if (!q->proj_ok && !q->proj_nfa)
      throw sql::UnsupportedError("query '" + q->cq.name + "': no device batch to project (host-API events deliver "
                                  "Event data to callbacks)");
    const int64_t m = q->dev_n;
    const int32_t ns = q->cq.hdr.nsel;
    if (n) *n = (size_t)m;
    if (nsel) *nsel = ns;
    if (!d_values) return;
    if ((size_t)m * (size_t)ns > cap_values) throw std::invalid_argument("d_values holds fewer than n * nsel values");
    hipStream_t hs = hip_stream ? (hipStream_t)hip_stream : a->stream;
    if (q->proj_nfa) {  // the NFA kernel evaluated the select list already (nfa_device_batch)
      if (m && ns)
        SM_HIP(hipMemcpyAsync(d_values, q->nfa_proj.p, (size_t)m * ns * sizeof(DVal), hipMemcpyDeviceToDevice, hs));
      if (m && d_ts)
        SM_HIP(hipMemcpyAsync(d_ts, (char*)q->nfa_proj.p + (size_t)m * ns * sizeof(DVal), (size_t)m * 8,
                              hipMemcpyDeviceToDevice, hs));
      SM_HIP(hipStreamSynchronize(hs));
      return;
    }
    q->proj_desc_dev.ensure(sizeof(NfaStream));
    SM_HIP(hipMemcpyAsync(q->proj_desc_dev.p, &q->proj_desc, sizeof(NfaStream), hipMemcpyHostToDevice, hs));
    ensure_scratch(a, (size_t)q->prev_carry_n * 16 + ((size_t)64 << 20));
    a->sc.used = 0;
    pair_project((const uint32_t*)q->dev_pairs.p, m, (const NfaStream*)q->proj_desc_dev.p, q->proj_ord, q->proj_n,
                 q->proj_base, q->proj_ts, (const int64_t*)q->prev_carry.p, q->prev_carry_n, q->prev_carry_w,
                 (const char*)q->blob.p, (DVal*)d_values, d_ts, a->sc, hs, q->cq.hdr.kind == 0);
  });
}

int sm_app_device_matches(sm_app* a, const char* query_name, const uint32_t** d_pairs, size_t* n) {
  std::lock_guard<std::mutex> g(a->mu);
  return guarded([&] {
    for (auto& q : a->queries)
      if (q->cq.name == query_name) {
        *d_pairs = (const uint32_t*)q->dev_pairs.p;
        *n = (size_t)q->dev_n;
        return;
      }
    throw sql::ValidationError(std::string("No query with name ") + query_name);
  });
}

}  // extern "C"
