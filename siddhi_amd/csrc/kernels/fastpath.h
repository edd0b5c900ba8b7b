// Host entry of the closed-form `every e1 -> e2 within T` kernel (fastpath.hip).
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

struct FastTimings {          // optional HIP events bracketing the phases (group / scan / order)
  hipEvent_t ev[4];
};

int64_t fast_every_within(const FastArgs& a, uint32_t* pairs_out, int64_t pairs_cap, Scratch& sc, hipStream_t s,
                          FastTimings* tm = nullptr);

}  // namespace sm
