// Closed-form kernel for `[partition with (k of S)] from every e1=S[c1] -> e2=S[c2(e1,e2)] within T`
// (SURVEY.md §8(a) A12). With non-decreasing event time the reference's processor chain
// (StreamPreStateProcessor.processAndReturn :274-327 on e2 before e1 for each event — reversed
// PatternMultiProcessStreamReceiver order :39-45 — plus `within` expiry :102-121 and the every back-edge
// StreamPostStateProcessor.process :66-68) is equivalent, per partial spawned by event i (c1(i)), to
//     j*(i) = min { j > i : key_j = key_i, c2(i, j), ts_j - ts_i <= T }
// and the selector emits (i, j*) ordered by j*, then i. This file computes exactly that on the device:
//   1. stable group of the events by key (radix sort of rebased keys)           [partitioned only]
//   2. c1 flags per event; forward scan per partial inside its key run
//   3. compaction of matches in key-run order, stable radix sort by j → reference order
#include "expr.h"
#include "fastpath.h"

namespace sm {

namespace {

inline dim3 grid_for(int64_t n, int t = 256) { return dim3((unsigned)((n + t - 1) / t)); }

__device__ __forceinline__ StackVal load_col(const NfaStream* st, int a, int64_t row) {
  StackVal v;
  v.i = 0;
  v.d = 0;
  v.null = 0;
  if (st->nulls[a] && st->nulls[a][row]) {
    v.null = 1;
    return v;
  }
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

// OP_VAR for a two-slot run record whose slots each hold one event (e1 = row1, e2 = row2).
struct PairLoader {
  const NfaStream* st;
  int64_t row1, row2;
  __device__ StackVal var(const Instr& in) const {
    StackVal v;
    v.i = 0;
    v.d = 0;
    v.null = 1;
    int64_t row = (in.a == 0) ? row1 : row2;
    if (row < 0 || !(in.b == 0 || in.b == -1)) return v;  // one-element chains: index 0 / CURRENT only
    return load_col(st, in.c, row);
  }
};

struct KeyLoader {
  const NfaStream* st;
  int64_t row;
  __device__ StackVal var(const Instr& in) const { return load_col(st, in.a, row); }
};

__global__ void fp_keys_kernel(const NfaStream* __restrict__ st, int64_t n, const KeyProg* __restrict__ kp,
                               int64_t* __restrict__ keys, uint8_t* __restrict__ valid) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  KeyLoader ld{st, i};
  StackVal v = eval_prog(kp->code, kp->len, kp->consts, ld);
  int64_t key;
  if (kp->type == T_FLOAT || kp->type == T_DOUBLE) {
    double d = v.d;
    if (d != d) d = __longlong_as_double(0x7ff8000000000000ll);
    key = __double_as_longlong(d);
  } else {
    key = v.i;
  }
  keys[i] = key;
  valid[i] = !v.null;
}

__global__ void fp_minmax_kernel(const int64_t* __restrict__ keys, int64_t n, unsigned long long* __restrict__ mm) {
  uint64_t lo = ~0ull, hi = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t u = (uint64_t)keys[i] ^ 0x8000000000000000ull;
    lo = u < lo ? u : lo;
    hi = u > hi ? u : hi;
  }
  // wave reduce then one atomic per wave
  for (int o = 32; o > 0; o >>= 1) {
    uint64_t a = __shfl_down(lo, o, 64), b = __shfl_down(hi, o, 64);
    lo = a < lo ? a : lo;
    hi = b > hi ? b : hi;
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMin(&mm[0], (unsigned long long)lo);
    atomicMax(&mm[1], (unsigned long long)hi);
  }
}

// rebased sort key; events with a null key sort after every valid key and are ignored
__global__ void fp_rebase_kernel(const int64_t* __restrict__ keys, const uint8_t* __restrict__ valid, int64_t n,
                                 uint64_t lo, uint64_t null_key, uint64_t* __restrict__ sk, uint32_t* __restrict__ idx) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  sk[i] = valid[i] ? (((uint64_t)keys[i] ^ 0x8000000000000000ull) - lo) : null_key;
  idx[i] = (uint32_t)i;
}

__global__ void fp_ts_check_kernel(const int64_t* __restrict__ ts, int64_t n, uint32_t* __restrict__ bad) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > 0 && i < n && ts[i] < ts[i - 1]) atomicOr(bad, 1u);
}

// One thread per event in key-run order: if the event spawns a partial (c1), scan forward within its run.
__global__ void fp_scan_kernel(const NfaStream* __restrict__ st, const int64_t* __restrict__ ts, int64_t n,
                               const uint32_t* __restrict__ perm, const uint64_t* __restrict__ skey,
                               uint64_t null_key, const Instr* __restrict__ code, const DVal* __restrict__ consts,
                               int c1_off, int c1_len, int c2_off, int c2_len, int64_t within,
                               uint32_t* __restrict__ match_v, uint8_t* __restrict__ has) {
  int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= n) return;
  has[u] = 0;
  const uint64_t k = skey ? skey[u] : 0;
  if (skey && k == null_key) return;
  const int64_t i = perm ? perm[u] : u;
  if (c1_len > 0) {
    PairLoader l1{st, i, -1};
    if (!truthy(eval_prog(code + c1_off, c1_len, consts, l1))) return;
  }
  const int64_t ti = ts[i];
  for (int64_t v = u + 1; v < n; ++v) {
    if (skey && skey[v] != k) return;
    const int64_t j = perm ? perm[v] : v;
    int64_t d = ts[j] - ti;
    if (within >= 0 && (d < 0 ? -d : d) > within) return;
    bool ok = true;
    if (c2_len > 0) {
      PairLoader l2{st, i, j};
      ok = truthy(eval_prog(code + c2_off, c2_len, consts, l2));
    }
    if (ok) {
      match_v[u] = (uint32_t)j;
      has[u] = 1;
      return;
    }
  }
}

__global__ void fp_u8_to_u32(const uint8_t* __restrict__ f, int64_t n, uint32_t* __restrict__ o) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) o[i] = f[i];
}

// matches in key-run order → (sort key = j position, value = i position)
__global__ void fp_emit_kernel(const uint8_t* __restrict__ has, const uint32_t* __restrict__ excl, int64_t n,
                               const uint32_t* __restrict__ perm, const uint32_t* __restrict__ match_v,
                               uint32_t* __restrict__ mj, uint32_t* __restrict__ mi) {
  int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= n || !has[u]) return;
  uint32_t o = excl[u];
  mj[o] = match_v[u];
  mi[o] = perm ? perm[u] : (uint32_t)u;
}

// final tuples relative to ordinal_base (explicit ordinals for sharded streams)
__global__ void fp_pairs_kernel(const uint32_t* __restrict__ mj, const uint32_t* __restrict__ mi, int64_t m,
                                const int64_t* __restrict__ ordinals, int64_t base, uint32_t* __restrict__ pairs) {
  int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= m) return;
  uint32_t i = mi[k], j = mj[k];
  pairs[2 * k] = ordinals ? (uint32_t)(ordinals[i] - base) : i;
  pairs[2 * k + 1] = ordinals ? (uint32_t)(ordinals[j] - base) : j;
}

}  // namespace

int64_t fast_every_within(const FastArgs& a, uint32_t* pairs_out, int64_t pairs_cap, Scratch& sc, hipStream_t s,
                          FastTimings* tm) {
  const int64_t n = a.n;
  if (n == 0) return 0;
  if (n >= 0xffffffffll) throw std::runtime_error("fast path: batch larger than 2^32 events");
  size_t mark = sc.used;
  uint32_t* bad = (uint32_t*)sc.take(4);
  SM_HIP(hipMemsetAsync(bad, 0, 4, s));
  hipLaunchKernelGGL(fp_ts_check_kernel, grid_for(n), dim3(256), 0, s, a.ts, n, bad);
  uint32_t* perm = nullptr;
  uint64_t* skey = nullptr;
  uint64_t null_key = ~0ull;
  if (a.key) {
    int64_t* keys = (int64_t*)sc.take(n * 8);
    uint8_t* valid = (uint8_t*)sc.take(n);
    hipLaunchKernelGGL(fp_keys_kernel, grid_for(n), dim3(256), 0, s, a.st, n, a.key, keys, valid);
    unsigned long long* mm = (unsigned long long*)sc.take(16);
    unsigned long long init[2] = {~0ull, 0ull};
    SM_HIP(hipMemcpyAsync(mm, init, 16, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(fp_minmax_kernel, dim3((unsigned)std::min<int64_t>(2048, (n + 255) / 256)), dim3(256), 0, s,
                       keys, n, mm);
    unsigned long long hmm[2];
    SM_HIP(hipMemcpyAsync(hmm, mm, 16, hipMemcpyDeviceToHost, s));
    SM_HIP(hipStreamSynchronize(s));
    uint64_t span = hmm[1] >= hmm[0] ? hmm[1] - hmm[0] : 0;
    int bits = 0;
    while (bits < 64 && (span >> bits) != 0) ++bits;
    // null keys get span+1 (one more bit when needed)
    null_key = span + 1;
    while (bits < 64 && (null_key >> bits) != 0) ++bits;
    uint64_t* sk = (uint64_t*)sc.take(n * 8);
    uint64_t* sk2 = (uint64_t*)sc.take(n * 8);
    uint32_t* si = (uint32_t*)sc.take(n * 4);
    uint32_t* si2 = (uint32_t*)sc.take(n * 4);
    hipLaunchKernelGGL(fp_rebase_kernel, grid_for(n), dim3(256), 0, s, keys, valid, n, (uint64_t)hmm[0], null_key, sk,
                       si);
    if (tm) SM_HIP(hipEventRecord(tm->ev[0], s));
    bool alt = radix_sort_pairs<uint64_t>(sk, sk2, si, si2, n, 0, std::max(bits, 1), sc, s);
    if (tm) SM_HIP(hipEventRecord(tm->ev[1], s));
    skey = alt ? sk2 : sk;
    perm = alt ? si2 : si;
  } else if (tm) {
    SM_HIP(hipEventRecord(tm->ev[0], s));
    SM_HIP(hipEventRecord(tm->ev[1], s));
  }
  uint32_t* match_v = (uint32_t*)sc.take(n * 4);
  uint8_t* has = (uint8_t*)sc.take(n);
  hipLaunchKernelGGL(fp_scan_kernel, grid_for(n), dim3(256), 0, s, a.st, a.ts, n, perm, skey, null_key, a.code,
                     a.consts, a.c1_off, a.c1_len, a.c2_off, a.c2_len, a.within, match_v, has);
  if (tm) SM_HIP(hipEventRecord(tm->ev[2], s));
  uint32_t* ex = (uint32_t*)sc.take(n * 4);
  uint32_t* total = (uint32_t*)sc.take(4);
  hipLaunchKernelGGL(fp_u8_to_u32, grid_for(n), dim3(256), 0, s, has, n, ex);
  exclusive_scan_u32(ex, n, sc, s, total);
  uint32_t hb = 0, hm = 0;
  SM_HIP(hipMemcpyAsync(&hb, bad, 4, hipMemcpyDeviceToHost, s));
  SM_HIP(hipMemcpyAsync(&hm, total, 4, hipMemcpyDeviceToHost, s));
  SM_HIP(hipStreamSynchronize(s));
  if (hb) {
    sc.used = mark;
    throw std::runtime_error("fast path requires non-decreasing event timestamps within a device batch");
  }
  if ((int64_t)hm > pairs_cap) {
    sc.used = mark;
    throw std::runtime_error("match buffer too small");
  }
  uint32_t* mj = (uint32_t*)sc.take(std::max<uint32_t>(hm, 1) * 4);
  uint32_t* mi = (uint32_t*)sc.take(std::max<uint32_t>(hm, 1) * 4);
  uint32_t* mj2 = (uint32_t*)sc.take(std::max<uint32_t>(hm, 1) * 4);
  uint32_t* mi2 = (uint32_t*)sc.take(std::max<uint32_t>(hm, 1) * 4);
  hipLaunchKernelGGL(fp_emit_kernel, grid_for(n), dim3(256), 0, s, has, ex, n, perm, match_v, mj, mi);
  int jbits = 0;
  while (jbits < 32 && ((uint64_t)(n - 1) >> jbits) != 0) ++jbits;
  bool alt = false;
  alt = radix_sort_pairs<uint32_t>(mj, mj2, mi, mi2, hm, 0, std::max(jbits, 1), sc, s);
  const uint32_t* fj = alt ? mj2 : mj;
  const uint32_t* fi = alt ? mi2 : mi;
  if (hm) hipLaunchKernelGGL(fp_pairs_kernel, grid_for(hm), dim3(256), 0, s, fj, fi, (int64_t)hm, a.ordinals,
                             a.ordinal_base, pairs_out);
  if (tm) SM_HIP(hipEventRecord(tm->ev[3], s));
  sc.used = mark;
  return hm;
}

}  // namespace sm
