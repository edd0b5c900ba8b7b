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
};

// Device facts cached across batches by the v2 kernels.
struct FastState {
  int cus = 0;              // compute units of the device
  int sort_wgs_per_cu = 0;  // resident down-sweep workgroups per CU (persistent-chunk grid)
  int walk_wgs_per_cu = 0;  // resident walk workgroups per CU
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

int64_t fast_every_within(const FastArgs& a, uint32_t* pairs_out, int64_t pairs_cap, Scratch& sc, hipStream_t s,
                          FastTimings* tm = nullptr);

// -1: outside the v2 envelope (caller falls back to fast_every_within)
int64_t fast_every_within_v2(const FastArgs& a, const FastHostInfo& hi, FastState& fs, uint32_t* pairs_out,
                             int64_t pairs_cap, Scratch& sc, hipStream_t s, FastTimings* tm = nullptr);

}  // namespace sm
