// Device-batch FilterProcessor (filter.hip): typed conjunction form + bytecode-interpreter form, both two
// streaming passes (count + write) around a block-count scan.
#pragma once
#include <cstring>
#include <vector>

#include "fastpath.h"
#include "nfa.h"
#include "primitives.h"

namespace sm {

constexpr int kFilterMaxLeaves = 4;

struct FilterLeaf {  // `x CMP y` with exactly one of x, y a column
  Instr cmp;
  bool is_col[2];
  int idx[2];  // column index or constant index
};

struct FilterLeaves {
  int n = 0;
  FilterLeaf leaf[kFilterMaxLeaves];
};

// Is `code` (postfix) a conjunction of at most kFilterMaxLeaves `column CMP constant` leaves over numeric
// columns? Fills `out` when it is.
bool filter_leaves(const Instr* code, int len, const DVal* consts, const int32_t* types, int nattr,
                   FilterLeaves& out);

// Rows [0, n) of one stream; writes the kept rows (uint32, ordinals[row] - ordinal_base when ordinals is given)
// to `out` in arrival order and returns their count. code/consts are given as device copies (interpreter
// form) and host copies (leaf analysis). `tm` (optional) receives per-launch marks "filter_count",
// "filter_scan", "filter_write"; *typed tells whether the conjunction form ran.
int64_t filter_device(const NfaStream& st_host, const NfaStream* st_dev, int64_t n, const Instr* code_dev,
                      const Instr* code_host, int len, const DVal* consts_dev, const DVal* consts_host,
                      const int64_t* ordinals, int64_t ordinal_base, uint32_t* out, Scratch& sc, hipStream_t s,
                      FastTimings* tm, bool* typed);

}  // namespace sm
