// Device-side bytecode evaluation shared by the filter, projection, fast-path and NFA kernels.
// Semantics follow the reference's expression executors:
//   compare:  core/executor/condition/compare/**  (null → false; NotEqual null → true,
//             NotEqualCompareConditionExpressionExecutor.java)
//   and/or:   AndConditionExpressionExecutor.java:66-76, OrConditionExpressionExecutor.java:65-76 (null → false)
//   not:      NotConditionExpressionExecutor.java:43-50 (not null → true)
//   math:     core/executor/math/** (result type by promotion; x/0 and x%0 → null; Java int wrap-around)
#pragma once
#include "hd.h"

#include "../plan.h"

namespace sm {

// One operand: integer-typed values live in i, FLOAT / DOUBLE ones in d (the instruction's static types pick
// the member, see do_compare / do_math), so the two share storage and an operand is 16 bytes.
struct StackVal {
  union {
    int64_t i;
    double d;
  };
  int null;
};

__device__ __forceinline__ bool cmp_apply(int op, int c) {  // c = -1 / 0 / 1 ; unordered handled by caller
  switch (op) {
    case CMP_EQ: return c == 0;
    case CMP_NE: return c != 0;
    case CMP_LT: return c < 0;
    case CMP_LE: return c <= 0;
    case CMP_GT: return c > 0;
    default: return c >= 0;
  }
}

template <typename T>
__device__ __forceinline__ bool cmp_typed(int op, T x, T y) {
  switch (op) {
    case CMP_EQ: return x == y;
    case CMP_NE: return x != y;
    case CMP_LT: return x < y;
    case CMP_LE: return x <= y;
    case CMP_GT: return x > y;
    default: return x >= y;
  }
}

__device__ __forceinline__ bool is_fp(int t) { return t == T_FLOAT || t == T_DOUBLE; }

__device__ __forceinline__ bool do_compare(const Instr& in, const StackVal& l, const StackVal& r) {
  switch (in.t0) {
    case CT_INT: return cmp_typed<int32_t>(in.sub, (int32_t)l.i, (int32_t)r.i);
    case CT_LONG: return cmp_typed<int64_t>(in.sub, l.i, r.i);
    case CT_ID: return cmp_typed<int64_t>(in.sub, l.i, r.i);
    case CT_FLOAT: {
      float x = is_fp(in.t1) ? (float)l.d : (float)l.i;
      float y = is_fp(in.t2) ? (float)r.d : (float)r.i;
      return cmp_typed<float>(in.sub, x, y);
    }
    default: {
      double x = is_fp(in.t1) ? l.d : (double)l.i;
      double y = is_fp(in.t2) ? r.d : (double)r.i;
      return cmp_typed<double>(in.sub, x, y);
    }
  }
}

__device__ __forceinline__ StackVal do_math(const Instr& in, const StackVal& l, const StackVal& r) {
  StackVal o;
  o.null = 1;
  o.i = 0;
  o.d = 0;
  if (l.null || r.null) return o;
  switch (in.t0) {
    case T_DOUBLE: {
      double x = is_fp(in.t1) ? l.d : (double)l.i;
      double y = is_fp(in.t2) ? r.d : (double)r.i;
      double z;
      switch (in.sub) {
        case M_ADD: z = x + y; break;
        case M_SUB: z = x - y; break;
        case M_MUL: z = x * y; break;
        case M_DIV: if (y == 0.0) return o; z = x / y; break;
        default: if (y == 0.0) return o; z = fmod(x, y); break;
      }
      o.d = z;
      break;
    }
    case T_FLOAT: {
      float x = is_fp(in.t1) ? (float)l.d : (float)l.i;
      float y = is_fp(in.t2) ? (float)r.d : (float)r.i;
      float z;
      switch (in.sub) {
        case M_ADD: z = x + y; break;
        case M_SUB: z = x - y; break;
        case M_MUL: z = x * y; break;
        case M_DIV: if (y == 0.0f) return o; z = x / y; break;
        default: if (y == 0.0f) return o; z = fmodf(x, y); break;
      }
      o.d = (double)z;
      break;
    }
    case T_LONG: {
      int64_t x = l.i, y = r.i, z;
      switch (in.sub) {
        case M_ADD: z = (int64_t)((uint64_t)x + (uint64_t)y); break;
        case M_SUB: z = (int64_t)((uint64_t)x - (uint64_t)y); break;
        case M_MUL: z = (int64_t)((uint64_t)x * (uint64_t)y); break;
        case M_DIV: if (y == 0) return o; z = (x == INT64_MIN && y == -1) ? INT64_MIN : x / y; break;
        default: if (y == 0) return o; z = (y == -1) ? 0 : x % y; break;
      }
      o.i = z;
      break;
    }
    default: {
      int32_t x = (int32_t)l.i, y = (int32_t)r.i, z;
      switch (in.sub) {
        case M_ADD: z = (int32_t)((uint32_t)x + (uint32_t)y); break;
        case M_SUB: z = (int32_t)((uint32_t)x - (uint32_t)y); break;
        case M_MUL: z = (int32_t)((uint32_t)x * (uint32_t)y); break;
        case M_DIV: if (y == 0) return o; z = (x == INT32_MIN && y == -1) ? INT32_MIN : x / y; break;
        default: if (y == 0) return o; z = (y == -1) ? 0 : x % y; break;
      }
      o.i = z;
      break;
    }
  }
  o.null = 0;
  return o;
}

// Column loader for stream context: typed SoA columns.
struct ColCtx {
  const void* const* cols;  // per attribute base pointer
  const int32_t* types;     // per attribute type
  int64_t row;
  __device__ StackVal load(int a) const {
    StackVal v;
    v.null = 0;
    v.i = 0;
    v.d = 0;
    switch (types[a]) {
      case T_INT: v.i = ((const int32_t*)cols[a])[row]; break;
      case T_LONG: v.i = ((const int64_t*)cols[a])[row]; break;
      case T_FLOAT: v.d = (double)((const float*)cols[a])[row]; break;
      case T_DOUBLE: v.d = ((const double*)cols[a])[row]; break;
      case T_STRING: {
        int32_t id = ((const int32_t*)cols[a])[row];
        v.i = id;
        v.null = id < 0;
        break;
      }
      default: v.i = ((const uint8_t*)cols[a])[row]; break;
    }
    return v;
  }
};

// Generic evaluation. Loader must provide StackVal var(const Instr&) for OP_VAR / OP_COL.
// SM_NFA_JIT_INLINE_ALL: the plan's programs are constants there; unrolled, the operand stack becomes registers
#ifdef SM_NFA_JIT_INLINE_ALL
#define SM_EXPR_INL __attribute__((always_inline))
#define SM_EXPR_UNROLL _Pragma("unroll")
#else
#define SM_EXPR_INL
#define SM_EXPR_UNROLL
#endif
template <typename Loader>
SM_EXPR_INL __device__ StackVal eval_prog(const Instr* code, int len, const DVal* consts, const Loader& ld) {
  StackVal st[kMaxStack];
  int sp = 0;
  SM_EXPR_UNROLL
  for (int pc = 0; pc < len; ++pc) {
    const Instr in = code[pc];
    switch (in.op) {
      case OP_CONST: {
        const DVal c = consts[in.a];
        if (in.t0 == T_FLOAT || in.t0 == T_DOUBLE) st[sp].d = c.d;
        else st[sp].i = c.i;
        st[sp].null = c.null;
        ++sp;
        break;
      }
      case OP_COL:
      case OP_VAR:
      case OP_TS:
        st[sp++] = ld.var(in);
        break;
      case OP_CMP: {
        StackVal r = st[--sp];
        StackVal l = st[--sp];
        StackVal o;
        o.d = 0;
        o.null = 0;
        if (l.null || r.null) o.i = (in.sub == CMP_NE);
        else o.i = do_compare(in, l, r);
        st[sp++] = o;
        break;
      }
      case OP_MATH: {
        StackVal r = st[--sp];
        StackVal l = st[--sp];
        st[sp++] = do_math(in, l, r);
        break;
      }
      case OP_AND: {
        StackVal r = st[--sp];
        StackVal l = st[--sp];
        StackVal o;
        o.d = 0;
        o.null = 0;
        o.i = (!l.null && l.i) && (!r.null && r.i);
        st[sp++] = o;
        break;
      }
      case OP_OR: {
        StackVal r = st[--sp];
        StackVal l = st[--sp];
        StackVal o;
        o.d = 0;
        o.null = 0;
        o.i = (!l.null && l.i) || (!r.null && r.i);
        st[sp++] = o;
        break;
      }
      case OP_NOT: {
        StackVal l = st[--sp];
        StackVal o;
        o.d = 0;
        o.null = 0;
        o.i = !(!l.null && l.i);
        st[sp++] = o;
        break;
      }
      default: {  // OP_ISNULL
        StackVal l = st[--sp];
        StackVal o;
        o.d = 0;
        o.null = 0;
        o.i = l.null ? 1 : 0;
        st[sp++] = o;
        break;
      }
    }
  }
  return st[0];
}

__device__ __forceinline__ bool truthy(const StackVal& v) { return !v.null && v.i != 0; }

}  // namespace sm
