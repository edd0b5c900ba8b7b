// Hand-written data-movement primitives for gfx950 (wave64):
//   * exclusive_scan_u32 / u64      — reduce-then-scan over 256-thread blocks
//   * radix_sort_pairs<K>           — stable LSD radix sort, 8-bit digits, (K key, uint32 value) pairs;
//                                     in-block stable ranking by wave64 ballot peer masks, one pass =
//                                     upsweep histogram + digit-major scan + ranked scatter
// Used for partition-key grouping (the reference's PartitionStreamReceiver → per-key junction routing,
// core/partition/PartitionStreamReceiver.java:156-168) and for ordering match tuples by trigger event.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdexcept>
#include <string>

namespace sm {

#define SM_HIP(x)                                                                          \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess)                                                                  \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e_) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__));                 \
  } while (0)

// Scratch allocator handed to primitives: a device arena carved on demand by the runtime.
struct Scratch {
  char* base = nullptr;
  size_t cap = 0;
  size_t used = 0;
  void* take(size_t bytes) {
    size_t off = (used + 255) & ~size_t(255);
    if (off + bytes > cap) throw std::runtime_error("device scratch exhausted");
    used = off + bytes;
    return base + off;
  }
};

void exclusive_scan_u32(uint32_t* data, size_t n, Scratch& sc, hipStream_t s, uint32_t* total_dev = nullptr);
void exclusive_scan_u64(uint64_t* data, size_t n, Scratch& sc, hipStream_t s, uint64_t* total_dev = nullptr);

// Stable sort of (keys, vals) by key bits [begin_bit, end_bit). Ping-pongs between the two buffer pairs;
// returns true when the result ended up in (keys_alt, vals_alt). vals may be null (keys only).
template <typename K>
bool radix_sort_pairs(K* keys, K* keys_alt, uint32_t* vals, uint32_t* vals_alt, size_t n, int begin_bit,
                      int end_bit, Scratch& sc, hipStream_t s);

}  // namespace sm
