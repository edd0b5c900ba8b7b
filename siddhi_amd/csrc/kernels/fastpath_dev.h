// Device helpers shared by the keyed fast-path kernels (fastpath3.hip: sort / walk pipeline; stack.hip:
// bucket-stack pipeline): record value codes, compare specialisation, wave64 ranking primitives.
#pragma once
#include <type_traits>

#include "expr.h"
#include "nfa.h"

namespace sm {
namespace {

#ifndef SM_RB
#define SM_RB 10
#endif
constexpr int kRB = SM_RB;  // radix bits per pass
constexpr int kBins = 1 << kRB;
constexpr uint32_t kKeyMask = 0x7fffffffu;

constexpr uint32_t kNanCode = 0xffffffffu;  // value code of a NaN (FLOAT / DOUBLE): always compared exactly

// value-code modes
enum : int { VC_I32 = 0, VC_F32 = 1, VC_F64 = 2, VC_I64R = 3, VC_I64H = 4 };

struct Ctrl {
  unsigned long long kmin, kmax;  // sign-biased key range
  unsigned long long omax;        // max relative ordinal
  unsigned long long vmin, vmax;  // sign-biased range of a LONG compared attribute
  unsigned int bad_ts, bad_ord;   // ts decreasing / ordinals not increasing
  long long ts0, ts_last;
  long long o0;  // relative ordinal of the batch's first event
};

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its global stores
// (__syncthreads() may also drain vmcnt, which exposes every round of scattered stores). No kernel here exchanges
// global data between the waves of a workgroup.
__device__ __forceinline__ void lds_barrier() {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
#else  // host wave emulator (hd.h SM_HOST_EMU): a workgroup barrier
  __syncthreads();
#endif
}

// Lockstep point of a wave: a no-op on the GPU (the lanes of a wave execute each instruction together), a wave
// barrier under the host wave emulator, where the lanes are threads: placed between an LDS read every lane makes
// and a write one lane makes to the same word (the rank-counting idiom), which SIMD order serialises on the GPU.
__device__ __forceinline__ void wave_lockstep() {
#if !defined(__HIP_DEVICE_COMPILE__) && defined(SM_HOST_EMU)
  (void)__ballot(1);
#endif
}

// gfx950 bit / dot instructions, with plain restatements for the host wave emulator
__device__ __forceinline__ uint32_t sm_sbfe1(uint32_t d, int b) {  // bit b of d as 0 or ~0
#if defined(__HIP_DEVICE_COMPILE__)
  return (uint32_t)__builtin_amdgcn_sbfe((int)d, b, 1);
#else
  return ((d >> b) & 1u) ? 0xffffffffu : 0u;
#endif
}
__device__ __forceinline__ uint32_t sm_and_not_xor(uint32_t a, uint32_t b, uint32_t c) {  // a & ~(b ^ c)
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x90);  // a = 0xF0, b = 0xCC, c = 0xAA
#else
  return a & ~(b ^ c);
#endif
}
__device__ __forceinline__ uint32_t sm_udot4(uint32_t a, uint32_t b, uint32_t c) {  // sum of byte products + c
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_udot4(a, b, c, false);
#else
  uint32_t s = c;
  for (int k = 0; k < 4; ++k) s += ((a >> (8 * k)) & 255u) * ((b >> (8 * k)) & 255u);
  return s;
#endif
}

// Lanes of this wave whose kRB-bit digit equals this lane's (valid lanes only): one ballot per bit, and per
// bit one v_bitop3 per half, peers &= bit ? ballot : ~ballot  ==  peers & ~(ballot ^ sext(bit)).
__device__ __forceinline__ uint64_t peer_mask(uint32_t d, bool valid) {
  const uint64_t v = __ballot(valid);
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
#pragma unroll
  for (int bb = 0; bb < kRB; ++bb) {
    const uint32_t m = sm_sbfe1(d, bb);  // 0 or ~0
    const uint64_t bal = __ballot(m != 0u);
    lo = sm_and_not_xor(lo, (uint32_t)bal, m);
    hi = sm_and_not_xor(hi, (uint32_t)(bal >> 32), m);
  }
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

__device__ __forceinline__ uint64_t lanemask_lt() {
  const int lane = threadIdx.x & 63;
  return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

__device__ __forceinline__ StackVal col_value(const NfaStream* st, int a, int64_t row) {
  StackVal v;
  v.i = 0;
  v.d = 0;
  v.null = 0;
  switch (st->types[a]) {
    case T_INT: v.i = ((const int32_t*)st->cols[a])[row]; break;
    case T_LONG: v.i = ((const int64_t*)st->cols[a])[row]; break;
    case T_FLOAT: v.d = (double)((const float*)st->cols[a])[row]; break;
    case T_DOUBLE: v.d = ((const double*)st->cols[a])[row]; break;
    case T_STRING: v.i = ((const int32_t*)st->cols[a])[row]; v.null = v.i < 0; break;
    default: v.i = ((const uint8_t*)st->cols[a])[row]; break;
  }
  return v;
}

// One attribute column resolved once per kernel (its pointer and type out of the NfaStream descriptor), so a loop
// of column reads does not reload the descriptor after every store (the compiler cannot prove the stores miss it)
struct ColRef {
  const void* p;
  int t;
  __device__ __forceinline__ StackVal at(int64_t row) const {
    StackVal v;
    v.i = 0;
    v.d = 0;
    v.null = 0;
    switch (t) {
      case T_INT: v.i = ((const int32_t*)p)[row]; break;
      case T_LONG: v.i = ((const int64_t*)p)[row]; break;
      case T_FLOAT: v.d = (double)((const float*)p)[row]; break;
      case T_DOUBLE: v.d = ((const double*)p)[row]; break;
      case T_STRING: v.i = ((const int32_t*)p)[row]; v.null = v.i < 0; break;
      default: v.i = ((const uint8_t*)p)[row]; break;
    }
    return v;
  }
};
__device__ __forceinline__ ColRef col_ref(const NfaStream* st, int a) { return ColRef{st->cols[a], st->types[a]}; }

// canonical 64-bit image of an attribute value (double bits for FLOAT/DOUBLE, integer otherwise)
__device__ __forceinline__ uint64_t canon(const StackVal& v, int type) {
  return (type == T_FLOAT || type == T_DOUBLE) ? (uint64_t)__double_as_longlong(v.d) : (uint64_t)v.i;
}
__device__ __forceinline__ StackVal uncanon(uint64_t bits, int type) {
  StackVal v;
  v.null = 0;
  if (type == T_FLOAT || type == T_DOUBLE) v.d = __longlong_as_double((long long)bits);
  else v.i = (int64_t)bits;
  return v;
}

// monotone 32-bit value code (see the header)
template <typename VT>
__device__ __forceinline__ uint32_t vcode(VT v, int mode, int64_t vmin) {
  if constexpr (std::is_same<VT, int32_t>::value) {
    return (uint32_t)v ^ 0x80000000u;
  } else if constexpr (std::is_same<VT, float>::value) {
    if (v != v) return kNanCode;
    const uint32_t b = v == 0.0f ? 0u : __float_as_uint(v);  // -0.0 == 0.0
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
  } else if constexpr (std::is_same<VT, double>::value) {
    if (v != v) return kNanCode;
    const uint64_t b = v == 0.0 ? 0ull : (uint64_t)__double_as_longlong(v);
    const uint64_t m = (b >> 63) ? ~b : (b | 0x8000000000000000ull);
    return (uint32_t)(m >> 32);
  } else {  // int64
    if (mode == VC_I64R) return (uint32_t)(v - vmin);
    return (uint32_t)(((uint64_t)v ^ 0x8000000000000000ull) >> 32);
  }
}

// A condition program decoded once per thread: its kernel-uniform instructions and constants stay in scalar
// registers across loops instead of being re-read every iteration.
struct Cond {
  const Instr* code;
  int len;
  const DVal* consts;
  bool simple;  // `x CMP y` with x, y variables or constants
  Instr a, b, op;
  StackVal ka, kb;
};

__device__ __forceinline__ StackVal const_val(const DVal* consts, int k) {
  const DVal c = consts[k];
  StackVal v;
  v.i = c.i;
  v.d = c.d;
  v.null = c.null;
  return v;
}

__device__ __forceinline__ Cond make_cond(const Instr* code, int len, const DVal* consts) {
  Cond c;
  c.code = code;
  c.len = len;
  c.consts = consts;
  c.simple = len == 3 && code[2].op == OP_CMP && code[0].op != OP_CMP && code[1].op != OP_CMP &&
             code[0].op != OP_MATH && code[1].op != OP_MATH && code[0].op != OP_NOT && code[1].op != OP_NOT;
  if (c.simple) {
    c.a = code[0];
    c.b = code[1];
    c.op = code[2];
    if (c.a.op == OP_CONST) c.ka = const_val(consts, c.a.a);
    if (c.b.op == OP_CONST) c.kb = const_val(consts, c.b.a);
  }
  return c;
}

template <typename Ld>
__device__ __forceinline__ bool eval(const Cond& c, const Ld& ld) {
  if (c.len == 0) return true;
  if (c.simple) {
    const StackVal l = c.a.op == OP_CONST ? c.ka : ld.var(c.a);
    const StackVal r = c.b.op == OP_CONST ? c.kb : ld.var(c.b);
    if (l.null || r.null) return c.op.sub == CMP_NE;
    return do_compare(c.op, l, r);
  }
  return truthy(eval_prog(c.code, c.len, c.consts, ld));
}

// c.simple (or empty) conditions only: no interpreter stack in the caller
template <typename Ld>
__device__ __forceinline__ bool eval_simple(const Cond& c, const Ld& ld) {
  if (c.len == 0) return true;
  const StackVal l = c.a.op == OP_CONST ? c.ka : ld.var(c.a);
  const StackVal r = c.b.op == OP_CONST ? c.kb : ld.var(c.b);
  if (l.null || r.null) return c.op.sub == CMP_NE;
  return do_compare(c.op, l, r);
}

template <int OP, typename T>
__device__ __forceinline__ bool cmp_fixed(T x, T y) {
  if constexpr (OP == CMP_EQ) return x == y;
  else if constexpr (OP == CMP_NE) return x != y;
  else if constexpr (OP == CMP_LT) return x < y;
  else if constexpr (OP == CMP_LE) return x <= y;
  else if constexpr (OP == CMP_GT) return x > y;
  else return x >= y;
}

// e1-only program on an original row (c1)
struct RowLoader {
  const NfaStream* st;
  int64_t row;
  __device__ StackVal var(const Instr& in) const {
    if (in.op == OP_COL) return col_value(st, in.a, row);
    return col_value(st, in.c, row);
  }
};

// c2 over the carried attribute: slot 0 = e1, slot 1 = e2 (host checked every variable reads `vattr`)
struct PairLoader {
  uint64_t v1, v2;
  int type;
  __device__ StackVal var(const Instr& in) const { return uncanon(in.a == 0 ? v1 : v2, type); }
};

// Unkeyed walk: c2 on canonical 64-bit values, as a fixed compare `e2.x OP e1.x` (OP >= 0; FP: compared as
// double, else as int64) or the generic condition program (OP < 0).
template <int OP, bool FP>
struct C2 {
  Cond c;
  int vtype;
  __device__ __forceinline__ bool operator()(uint64_t v1, uint64_t v2) const {
    if constexpr (OP < 0) {
      return eval(c, PairLoader{v1, v2, vtype});
    } else {
      if constexpr (FP) return cmp_fixed<OP>(__longlong_as_double((long long)v2), __longlong_as_double((long long)v1));
      else return cmp_fixed<OP>((int64_t)v2, (int64_t)v1);
    }
  }
};

// Keyed walk: c2 = `e2.x OP e1.x` on value codes; equal inexact codes and NaN go to the exact column values.
template <int OP, bool FP>
struct C2Code {
  bool exact_codes;  // the code mode is exact (INT, FLOAT, rebased LONG)
  int vtype;
  const void* vcol;
  const int64_t* ord;  // ordinals of the batch rows (nullptr: row = relative ordinal)
  int64_t obase, n;
  __device__ int64_t row_of(uint32_t o) const {  // rows are in ordinal order
    if (!ord) return o;
    const int64_t want = (int64_t)o + obase;
    int64_t lo = 0, hi = n - 1;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (ord[mid] < want) lo = mid + 1;
      else hi = mid;
    }
    return lo;
  }
  __device__ bool exact(uint32_t o1, uint32_t o2) const {
    const int64_t r1 = row_of(o1), r2 = row_of(o2);
    if constexpr (FP) {
      double x1, x2;
      if (vtype == T_FLOAT) {
        x1 = ((const float*)vcol)[r1];
        x2 = ((const float*)vcol)[r2];
      } else {
        x1 = ((const double*)vcol)[r1];
        x2 = ((const double*)vcol)[r2];
      }
      return cmp_fixed<OP>(x2, x1);
    } else {
      int64_t x1, x2;
      if (vtype == T_INT) {
        x1 = ((const int32_t*)vcol)[r1];
        x2 = ((const int32_t*)vcol)[r2];
      } else {
        x1 = ((const int64_t*)vcol)[r1];
        x2 = ((const int64_t*)vcol)[r2];
      }
      return cmp_fixed<OP>(x2, x1);
    }
  }
  __device__ __forceinline__ bool operator()(uint32_t c1, uint32_t o1, uint32_t c2, uint32_t o2) const {
    if (!needs_exact(c1, c2)) return cmp_fixed<OP>(c2, c1);
    return exact(o1, o2);
  }
  // the codes alone do not decide the comparison (equal inexact codes, or a NaN)
  __device__ __forceinline__ bool needs_exact(uint32_t c1, uint32_t c2) const {
    const bool nan = FP & ((c1 == kNanCode) | (c2 == kNanCode));
    return nan | (!exact_codes & (c1 == c2));
  }
};

// Chunk g of a pass: [g * per, g * per + len_g); len_g = seg_len[g] when given, else the uniform split of n.
__device__ __forceinline__ void chunk_range(int g, int64_t n, int64_t per, const uint32_t* seg_len, int64_t& lo,
                                            int64_t& len) {
  lo = (int64_t)g * per;
  if (seg_len) {
    len = seg_len[g];
  } else {
    len = n - lo;
    if (len > per) len = per;
    if (len < 0) len = 0;
  }
}

}  // namespace
}  // namespace sm
