// Decoupled look-back primitives (single-pass prefix over tiles) shared by the onesweep radix passes and the
// walk's match compaction. Status word per (tile, counter): epoch(30) | flag(2) | value(32); flag 1 = tile
// aggregate, 2 = inclusive prefix. Words carry the launch's epoch, so they are never re-zeroed between launches
// (R2 form of cdna_hip_programming.md Guideline 16: the data IS the flag, agent-scope atomics on both sides).
// Every spin is bounded (kSpinLimit) and reports through *err.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sm {

constexpr unsigned long long kSpinLimit = 1ull << 26;

__device__ __forceinline__ void st_put(unsigned long long* p, uint32_t epoch, uint32_t flag, uint32_t v) {
  __hip_atomic_store(p, ((unsigned long long)epoch << 34) | ((unsigned long long)flag << 32) | v, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// exclusive prefix of `cnt` over all earlier tiles for one lane-owned counter
__device__ __forceinline__ uint32_t lookback(unsigned long long* status, int64_t stride, int64_t tile, uint32_t epoch,
                                             uint32_t cnt, unsigned int* err) {
  if (tile == 0) {
    st_put(status, epoch, 2, cnt);
    return 0;
  }
  st_put(status + tile * stride, epoch, 1, cnt);
  uint32_t excl = 0;
  int64_t p = tile - 1;
  unsigned long long spins = 0;
  while (true) {
    unsigned long long s = __hip_atomic_load(status + p * stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t flag = (uint32_t)(s >> 32) & 3u;
    if ((uint32_t)(s >> 34) != epoch || flag == 0) {
      if (++spins > kSpinLimit) {
        atomicOr(err, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    excl += (uint32_t)s;
    if (flag == 2) break;
    --p;
  }
  st_put(status + tile * stride, epoch, 2, excl + cnt);
  return excl;
}

// Windowed look-back for one lane-owned counter: the W nearest unresolved predecessors are read with W
// independent loads per step (cross-XCD agent-scope loads cost ~1 us each, so a one-at-a-time walk over the
// tiles still in flight serialises on that latency).
template <int W>
__device__ __forceinline__ uint32_t lookback_win(unsigned long long* status, int64_t stride, int64_t tile,
                                                 uint32_t epoch, uint32_t cnt, unsigned int* err) {
  if (tile == 0) {
    st_put(status, epoch, 2, cnt);
    return 0;
  }
  st_put(status + tile * stride, epoch, 1, cnt);
  uint32_t excl = 0;
  int64_t top = tile - 1;
  unsigned long long spins = 0;
  while (true) {
    unsigned long long sv[W];
#pragma unroll
    for (int k = 0; k < W; ++k) {
      const int64_t p = top - k;
      sv[k] = p >= 0 ? __hip_atomic_load(status + p * stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                     : ((unsigned long long)epoch << 34) | (2ull << 32);  // virtual inclusive 0 before tile 0
    }
    int adv = W;
    bool done = false;
#pragma unroll
    for (int k = 0; k < W; ++k) {
      if (adv == W && !done) {
        const uint32_t flag = (uint32_t)(sv[k] >> 32) & 3u;
        if ((uint32_t)(sv[k] >> 34) != epoch || flag == 0) {
          adv = k;
        } else {
          excl += (uint32_t)sv[k];
          if (flag == 2) done = true;
        }
      }
    }
    if (done) break;
    top -= adv;
    if (adv == 0) {
      if (++spins > kSpinLimit) {
        atomicOr(err, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  st_put(status + tile * stride, epoch, 2, excl + cnt);
  return excl;
}

// Wave-parallel look-back for one tile counter, run by ONE full wave: lane l reads predecessor top - l, so a
// step resolves up to 64 tiles. Returns the exclusive prefix (wave-uniform).
__device__ __forceinline__ uint32_t lookback_wave(unsigned long long* status, int64_t tile, uint32_t epoch,
                                                  uint32_t cnt, unsigned int* err) {
  const int lane = threadIdx.x & 63;
  if (tile == 0) {
    if (lane == 0) st_put(status, epoch, 2, cnt);
    return 0;
  }
  if (lane == 0) st_put(status + tile, epoch, 1, cnt);
  uint32_t excl = 0;
  int64_t top = tile - 1;
  unsigned long long spins = 0;
  while (true) {
    const int64_t p = top - lane;
    const unsigned long long sv =
        p >= 0 ? __hip_atomic_load(status + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
               : ((unsigned long long)epoch << 34) | (2ull << 32);
    const uint32_t flag = ((uint32_t)(sv >> 34) == epoch) ? ((uint32_t)(sv >> 32) & 3u) : 0u;
    const uint64_t incl = __ballot(flag == 2);
    const uint64_t zero = __ballot(flag == 0);
    const uint64_t stop = incl | zero;
    const int f = stop ? __ffsll((unsigned long long)stop) - 1 : 64;  // first lane that stops the walk
    // lanes below f, plus lane f when it holds an inclusive prefix. Written as a lane mask: the equivalent
    // `lane < f || (lane == f && ((incl >> f) & 1))` is miscompiled by ROCm 7.2 hipcc for gfx950 (lane f
    // drops out; reproduced by tests/native/lookback_check.hip).
    const uint64_t below = f >= 64 ? ~0ull : ((1ull << f) - 1ull);
    const uint64_t take = below | ((f < 64 && ((incl >> f) & 1ull)) ? (1ull << f) : 0ull);
    uint32_t v = ((take >> lane) & 1ull) ? (uint32_t)sv : 0u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    excl += v;
    if (f < 64 && ((incl >> f) & 1ull)) break;
    top -= f;
    if (f == 0) {
      if (++spins > kSpinLimit) {
        if (lane == 0) atomicOr(err, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  if (lane == 0) st_put(status + tile, epoch, 2, excl + cnt);
  return excl;
}

}  // namespace sm
