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
inline unsigned atomicAdd(unsigned* p, unsigned v) {
  unsigned o = *p;
  *p += v;
  return o;
}
inline int atomicOr(int* p, int v) {
  int o = *p;
  *p |= v;
  return o;
}
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
