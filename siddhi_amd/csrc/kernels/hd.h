// Device-code portability header. Under hipcc: HIP runtime. Under a plain host compiler (g++): shims so the
// SAME device source (expr.h, nfa_impl.h) builds as a single-threaded CPU debug binary for gdb / sanitizers
// (tests/native/) — the product library itself is always built by hipcc for gfx950.
#pragma once
#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#else
#include <cmath>
#include <cstdint>
#include <cstring>
#define __device__
#define __host__
#define __global__
#define __forceinline__ inline
#define __launch_bounds__(...)
typedef struct ihipStream_t* hipStream_t;
#ifndef SM_HOST_EMU
inline unsigned atomicAdd(unsigned* p, unsigned v) {
  unsigned o = *p;
  *p += v;
  return o;
}
inline unsigned long long atomicAdd(unsigned long long* p, unsigned long long v) {
  unsigned long long o = *p;
  *p += v;
  return o;
}
inline int atomicOr(int* p, int v) {
  int o = *p;
  *p |= v;
  return o;
}
inline unsigned long long atomicCAS(unsigned long long* p, unsigned long long cmp, unsigned long long v) {
  unsigned long long o = *p;
  if (o == cmp) *p = v;
  return o;
}
inline unsigned long long atomicMax(unsigned long long* p, unsigned long long v) {
  unsigned long long o = *p;
  if (v > o) *p = v;
  return o;
}
#else
// Wave emulator (tests/native/stack_emu.cpp, test infrastructure): every GPU thread of a workgroup is a fiber of one
// host thread; wave64 operations and __syncthreads are barriers of the fibers of a wave / the workgroup (the
// emulator's scheduler runs fibers until they reach one); __shared__ arrays are statics (one workgroup runs at a
// time). Only convergent wave operations are supported (every lane of the wave reaches the same sequence of them),
// which is how the emulated kernels use them.
#include <memory>
struct sm_dim3 {
  unsigned x = 0, y = 0, z = 0;
};
extern sm_dim3 threadIdx, blockIdx, gridDim, blockDim;  // threadIdx: the running fiber's
namespace sm_emu {
void wave_sync();   // all 64 lanes of the running fiber's wave
void block_sync();  // every fiber of the workgroup
extern unsigned long long (*wave_buf)[64];  // exchange slots of each wave
inline int lane() { return (int)(threadIdx.x & 63); }
inline unsigned long long* buf() { return wave_buf[threadIdx.x >> 6]; }
}  // namespace sm_emu
#define __shared__ static
#define __noinline__ __attribute__((noinline))
struct uint2 {
  unsigned x, y;
};
struct uint4 {
  unsigned x, y, z, w;
};
inline uint2 make_uint2(unsigned x, unsigned y) { return {x, y}; }
inline uint4 make_uint4(unsigned x, unsigned y, unsigned z, unsigned w) { return {x, y, z, w}; }
inline void __syncthreads() { sm_emu::block_sync(); }
inline unsigned long long __ballot(int pred) {
  unsigned long long* b = sm_emu::buf();
  b[sm_emu::lane()] = pred != 0;
  sm_emu::wave_sync();
  unsigned long long m = 0;
  for (int l = 0; l < 64; ++l) m |= (b[l] ? 1ull : 0ull) << l;
  sm_emu::wave_sync();
  return m;
}
inline int __any(int pred) { return __ballot(pred) != 0; }
template <typename T>
inline T sm_emu_exchange(T v, int src) {
  unsigned long long* b = sm_emu::buf();
  unsigned long long u = 0;
  memcpy(&u, &v, sizeof(T));
  b[sm_emu::lane()] = u;
  sm_emu::wave_sync();
  const unsigned long long r = b[src & 63];
  sm_emu::wave_sync();
  T out;
  memcpy(&out, &r, sizeof(T));
  return out;
}
template <typename T>
inline T __shfl(T v, int src, int = 64) { return sm_emu_exchange(v, src); }
template <typename T>
inline T __shfl_up(T v, unsigned d, int = 64) {
  const int l = sm_emu::lane();
  const T r = sm_emu_exchange(v, l >= (int)d ? l - (int)d : l);
  return l >= (int)d ? r : v;
}
inline int __popcll(unsigned long long x) { return __builtin_popcountll(x); }
inline int __popc(unsigned x) { return __builtin_popcount(x); }
inline unsigned atomicAdd(unsigned* p, unsigned v) { return __atomic_fetch_add(p, v, __ATOMIC_SEQ_CST); }
inline unsigned long long atomicAdd(unsigned long long* p, unsigned long long v) {
  return __atomic_fetch_add(p, v, __ATOMIC_SEQ_CST);
}
inline unsigned atomicOr(unsigned* p, unsigned v) { return __atomic_fetch_or(p, v, __ATOMIC_SEQ_CST); }
inline int atomicOr(int* p, int v) { return __atomic_fetch_or(p, v, __ATOMIC_SEQ_CST); }
inline unsigned long long atomicCAS(unsigned long long* p, unsigned long long cmp, unsigned long long v) {
  __atomic_compare_exchange_n(p, &cmp, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST);
  return cmp;
}
inline unsigned long long atomicMax(unsigned long long* p, unsigned long long v) {
  unsigned long long o = __atomic_load_n(p, __ATOMIC_SEQ_CST);
  while (v > o && !__atomic_compare_exchange_n(p, &o, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) {
  }
  return o;
}
inline unsigned __float_as_uint(float f) {
  unsigned u;
  memcpy(&u, &f, 4);
  return u;
}
#endif
inline long long __double_as_longlong(double d) {
  long long x;
  memcpy(&x, &d, 8);
  return x;
}
struct longlong2 {
  long long x, y;
};
inline longlong2 make_longlong2(long long x, long long y) { return {x, y}; }
inline double __longlong_as_double(long long x) {
  double d;
  memcpy(&d, &x, 8);
  return d;
}
#endif
