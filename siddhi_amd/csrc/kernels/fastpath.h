// Host entry of the closed-form `every e1 -> e2 within T` kernels (fastpath.hip: general form;
// fastpath3.hip: keyed bandwidth form for single-column keys and a single compared attribute).
#pragma once
#include "nfa.h"
#include "primitives.h"
#include "stream_ops.h"

namespace sm {

struct FastArgs {
  int64_t n;
  const int64_t* ts;          // device, event timestamps
  const NfaStream* st;        // device stream descriptor (columns)
  const KeyProg* key;         // device key program or nullptr (non-partitioned)
  const Instr* code;          // device bytecode of the query
  const DVal* consts;
  int c1_off, c1_len, c2_off, c2_len;
  int64_t within;             // -1 = none
  const int64_t* ordinals;    // device or nullptr
  int64_t ordinal_base;
};

// Host-side facts about the plan and the batch used to pick the v2 kernels.
struct FastHostInfo {
  const void* const* cols;    // host array of device column pointers
  const int32_t* types;       // column types
  int key_col = -1;           // partition key is this column (-1: expression or none)
  int key_type = 0;
  int vattr = -1;             // the only attribute c2 reads (-1: not eligible)
  int vtype = 0;
  const Instr* c2_host = nullptr;  // host copy of the c2 program (specialisation of the walk's compare)
  int c2_len = 0;
  const Instr* c1_host = nullptr;  // host copy of the c1 program (c1 on the compared attribute: no bit mask)
  int c1_len = 0;
  int nattr = 0;              // attributes of the stream (carried partial rows)
  const int32_t* dense_keys = nullptr;  // device: the key column as dense ids (remap_keys), read instead of the column
  int64_t remap_span = 0;  // > 0: a key span above it returns FAST_KEY_SPAN (the caller gives the keys dense ids)
};

// Device facts cached across batches by the v2 kernels.
struct FastState {
  int cus = 0;              // compute units of the device
  int sort_wgs_per_cu = 0;  // resident down-sweep workgroups per CU (persistent-chunk grid)
  int walk_wgs_per_cu = 0;  // resident walk workgroups per CU
  int last_path = 0;        // pipeline of the last batch: 2 = sort / walk, 3 = bucket stack
};

struct FastTimings {          // optional HIP events: [0] start, [1] keyed sort done, [2] walk done, [3] end
  hipEvent_t ev[4];
  // per-launch marks of the v2 pipeline: mk[0] before the first kernel, mk[k] after the k-th, label[k] its kernel
  static constexpr int kMaxMarks = 32;
  hipEvent_t mk[kMaxMarks];
  const char* label[kMaxMarks];
  int nmk = 0;
  void mark(const char* l, hipStream_t s) {
    if (nmk < kMaxMarks) {
      label[nmk] = l;
      (void)hipEventRecord(mk[nmk++], s);
    }
  }
};

// Open partials carried across device batches of one query: the pending list of the e2 pre-processor, which the
// reference keeps between InputHandler.send calls (StreamPreStateProcessor.java:208-221 addState, :268-271
// updateState, :274-327 processAndReturn). One row per partial = its e1 event:
//   [key, global ordinal, event time, attribute 0 .. nattr-1 (canonical 64-bit: integers as int64, FLOAT /
//   DOUBLE as double bits)]
// sorted by (key, ordinal). As in the reference, a partial stays pending until an event of its own key either
// matches it or finds it expired (isExpired :102-121); keys that see no event keep their partials.
struct FastCarry {
  int64_t* rows = nullptr;  // device, n rows of `width` words
  int64_t n = 0, cap = 0;   // rows / allocated rows
  int width = 0;            // 3 + nattr
  bool active = false;      // a device batch has run for this query: ts_last is valid
  int64_t ts_last = 0;      // event time of the last event of the last batch
  void reserve(int64_t rows_needed, int w);
  void release();
  void reset() {
    n = 0;
    active = false;
    ts_last = 0;
  }
};

int64_t fast_every_within(const FastArgs& a, uint32_t* pairs_out, int64_t pairs_cap, Scratch& sc, hipStream_t s,
                          FastTimings* tm = nullptr);

// Results of fast_every_within_v2 besides M >= 0.
enum : int64_t { FAST_OUTSIDE = -1, FAST_NON_MONOTONE = -2, FAST_KEY_SPAN = -3 };

// FAST_OUTSIDE: outside the v2 envelope (caller falls back to fast_every_within); FAST_NON_MONOTONE: event time
// decreases inside the batch or against the carried state (the closed form does not apply: the caller takes the
// general NFA path); FAST_KEY_SPAN: the partition keys (carried ones included) span more than 2^30 values, or more
// than hi.remap_span when that is set (the caller may give them dense ids and run the batch again; nothing was
// changed). Match pairs are relative to a.ordinal_base; an e1 carried from an earlier batch has a
// negative (int32) relative ordinal. The carry is read and replaced.
int64_t fast_every_within_v2(const FastArgs& a, const FastHostInfo& hi, FastState& fs, FastCarry& carry,
                             uint32_t* pairs_out, int64_t pairs_cap, Scratch& sc, hipStream_t s,
                             FastTimings* tm = nullptr, int stack_mode = 0);

// ---- internal: the bucket-stack pipeline (stack.hip), entered by fast_every_within_v2 after key pass 0 ----

// Facts about a batch once key pass 0 has scattered its 16-byte records {key - kmin | c1 << 31, ordinal - base,
// value code, ts - ts0} into kBins buckets by the low key digit (fastpath3.hip).
struct StackPlan {
  const void* rec;          // uint4 records, bucket order
  const uint32_t* dbase;    // bucket starts
  int64_t n;
  int64_t omax;             // largest relative ordinal of the batch
  int H;                    // in-bucket keys (key span >> kRB, rounded up)
  int64_t kmin;
  int op;                   // CMP_* of `e2.x OP e1.x`
  bool fp;                  // compared as floating point
  bool exact_codes;         // value codes decide every comparison
  int vtype, vattr, vmode;
  int64_t vmin;
  const void* vcol;
  int64_t within;
  int64_t ts0, ts_last;
  int32_t o0;               // relative ordinal of the batch's first event: carried partials lie before it
};

// M >= 0, or -1 when the batch must take the sort / walk pipeline instead (a key's open partials overflowed the
// stack, a slice's match log filled, a NaN compared value): neither pairs_out nor the carry was touched then.
int64_t stack_pipeline(const StackPlan& p, const FastArgs& a, const FastHostInfo& hi, FastState& fs, FastCarry& carry,
                       uint32_t* pairs_out, int64_t pairs_cap, Scratch& sc, hipStream_t s, FastTimings* tm);

// Carry-out candidates (4 words each: key, global ordinal, event time, source = batch row >= 0 or -(old carry
// row) - 1) → the new carry rows, sorted by (key, ordinal). `old` is read before carry.rows is replaced.
void build_carry(const int64_t* cand, int64_t ncand, const NfaStream* st, int nattr, FastCarry& carry, Scratch& sc,
                 hipStream_t s, int key_bits = 64, int64_t kmin = 0, bool key_runs_ordered = false);

// On-device projection of m closed-form outputs (pairs = the device tuples of the last batch): the query's select
// programs (blob_dev = its device plan) → out[k * nsel + a], and e2's event time → ts_out[k] (may be null). An e1
// carried from an earlier batch reads its row of prev_carry (the carry as it was before the batch: nc rows of cw
// words). The batch's columns / ts / ordinals must still be resident. rows = true: `pairs` are a filter query's
// kept rows (m u32, ordinal - base), each output reading its own row.
void pair_project(const uint32_t* pairs, int64_t m, const NfaStream* st_dev, const int64_t* ord, int64_t n,
                  int64_t base, const int64_t* ts, const int64_t* prev_carry, int64_t nc, int cw, const char* blob_dev,
                  DVal* out, int64_t* ts_out, Scratch& sc, hipStream_t s, bool rows = false,
                  int64_t* words = nullptr, uint8_t* nulls = nullptr,  // words / nulls: compact form (nsel <= 8)
                  const uint32_t* carry_keys = nullptr, const uint32_t* carry_idx = nullptr, bool sync = true);
// The carried partials' e1 ordinals sorted for pair_project (carry_keys / carry_idx, nc each, in sc): a caller
// projecting one batch's outputs in several launches sorts them once (round 5: device_outputs' segments)
void pair_project_carry_order(const int64_t* prev_carry, int64_t nc, int cw, int64_t base, Scratch& sc, hipStream_t s,
                              const uint32_t** carry_keys, const uint32_t** carry_idx);

}  // namespace sm
