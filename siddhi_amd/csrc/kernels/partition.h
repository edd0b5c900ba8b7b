// Stable partition of a columnar batch by owner rank (multi-GPU key exchange); see partition.hip.
#pragma once
#include <vector>

#include "primitives.h"

namespace sm {

constexpr int kMaxOwners = 64;
constexpr int kMaxPartCols = 16;

struct PartCols {
  int32_t n;
  int32_t width[kMaxPartCols];  // bytes per element: 1, 2, 4 or 8
  const void* src[kMaxPartCols];
  void* dst[kMaxPartCols];
};

void partition_by_owner(const void* keys, int key_width, int64_t n, uint32_t world, const PartCols& cols,
                        uint64_t* counts_host, Scratch& sc, hipStream_t s);

}  // namespace sm
