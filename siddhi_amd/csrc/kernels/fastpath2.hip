// Bandwidth-shaped closed form for `[partition with (k of S)] from every e1=S[c1] -> e2=S[c2] within T`
// (derivation and citations in fastpath.hip). For each event i with c1(i):
//     j*(i) = min { j > i : key_j = key_i, c2(i, j), ts_j - ts_i <= T },   output (i, j*) ordered by (j*, i).
//
// Pipeline (all device-resident, two host syncs per batch):
//   prep     key min/max, ts monotonicity + span, max relative ordinal           (reads key + ts)
//   hist     per-digit histograms of the rebased key for every sort pass          (reads key)
//   fwd_k    onesweep LSD pass k (10-bit digits) moving the 20-byte record
//            {key|c1<<31 : u32, ordinal : u32, c2 attribute : u64, ts - ts0 : u32}; pass 0 builds the record
//            from the original columns (c1 evaluated here, once per event)
//   walk     one lane per record in key order: forward scan inside the key run until c2 holds or the window
//            closes; matches are compacted in record order with a decoupled look-back → (j, i) u32 pairs
//   jhist    per-digit histograms of j
//   jsort_k  onesweep LSD passes over the (j, i) pairs; the last pass writes the interleaved output
// Every onesweep pass: dynamic tile ids (forward progress for the look-back), stable in-tile ranking by
// wave64 ballot peer masks, per-(tile, digit) look-back on epoch-tagged 8-byte status words (agent-scope
// atomics both sides, so no status memset per pass), LDS exchange so that each digit run leaves the tile as
// contiguous stores.
#include "expr.h"
#include "fastpath.h"

namespace sm {

namespace {

constexpr int kBlock = 512;
constexpr int kWaves = kBlock / 64;
constexpr int kItems = 16;
constexpr int kTile = kBlock * kItems;  // 8192 records per onesweep tile
constexpr int kRB = 10;                 // radix bits per pass
constexpr int kBins = 1 << kRB;
constexpr int kBinsPerThread = kBins / kBlock;
constexpr uint32_t kKeyMask = 0x7fffffffu;
constexpr int kWalkBlock = 256;
constexpr int kWalkItems = 8;
constexpr int kWalkTile = kWalkBlock * kWalkItems;
constexpr unsigned long long kSpinLimit = 1ull << 26;

static_assert(kBins % kBlock == 0, "bins per thread");

struct Ctrl {
  unsigned long long kmin, kmax;  // sign-biased key range
  unsigned long long omax;        // max relative ordinal
  unsigned int bad_ts, nulls, err, nmatch;
  unsigned int tile_ctr[16];
  long long ts0, ts_last;
};

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

// canonical 64-bit image of an attribute value (double bits for FLOAT/DOUBLE, integer otherwise)
__device__ __forceinline__ uint64_t canon(const StackVal& v, int type) {
  return (type == T_FLOAT || type == T_DOUBLE) ? (uint64_t)__double_as_longlong(v.d) : (uint64_t)v.i;
}
__device__ __forceinline__ StackVal uncanon(uint64_t bits, int type) {
  StackVal v;
  v.null = 0;
  if (type == T_FLOAT || type == T_DOUBLE) {
    v.d = __longlong_as_double((long long)bits);
    v.i = 0;
  } else {
    v.i = (int64_t)bits;
    v.d = 0;
  }
  return v;
}

template <typename Ld>
__device__ __forceinline__ StackVal operand(const Instr& in, const DVal* consts, const Ld& ld) {
  if (in.op == OP_CONST) {
    const DVal c = consts[in.a];
    StackVal v;
    v.i = c.i;
    v.d = c.d;
    v.null = c.null;
    return v;
  }
  return ld.var(in);
}

// Condition program → bool, with the common `x CMP y` shape evaluated without the interpreter stack.
template <typename Ld>
__device__ __forceinline__ bool eval_cond(const Instr* code, int len, const DVal* consts, const Ld& ld) {
  if (len == 0) return true;
  if (len == 3 && code[2].op == OP_CMP && code[0].op != OP_CMP && code[1].op != OP_CMP &&
      code[0].op != OP_MATH && code[1].op != OP_MATH && code[0].op != OP_NOT && code[1].op != OP_NOT) {
    const StackVal l = operand(code[0], consts, ld), r = operand(code[1], consts, ld);
    if (l.null || r.null) return code[2].sub == CMP_NE;
    return do_compare(code[2], l, r);
  }
  return truthy(eval_prog(code, len, consts, ld));
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

// ---------------------------------------------------------------- prep / histograms

__global__ void prep_kernel(const void* __restrict__ kcol, int ktype, const int64_t* __restrict__ ts,
                            const int64_t* __restrict__ ord, int64_t obase, int64_t n, Ctrl* __restrict__ c) {
  unsigned long long lo = ~0ull, hi = 0, om = 0;
  unsigned int bad = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (kcol) {
      int64_t k = ktype == T_INT ? (int64_t)((const int32_t*)kcol)[i] : ((const int64_t*)kcol)[i];
      unsigned long long u = (unsigned long long)k ^ 0x8000000000000000ull;
      lo = u < lo ? u : lo;
      hi = u > hi ? u : hi;
    }
    if (i > 0 && ts[i] < ts[i - 1]) bad = 1;
    if (ord) {
      unsigned long long o = (unsigned long long)(ord[i] - obase);
      om = o > om ? o : om;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long a = __shfl_down(lo, o, 64), b = __shfl_down(hi, o, 64), d = __shfl_down(om, o, 64);
    lo = a < lo ? a : lo;
    hi = b > hi ? b : hi;
    om = d > om ? d : om;
  }
  bad = __any(bad) ? 1u : 0u;
  if ((threadIdx.x & 63) == 0) {
    if (kcol) {
      atomicMin(&c->kmin, lo);
      atomicMax(&c->kmax, hi);
    }
    if (ord) atomicMax(&c->omax, om);
    if (bad) atomicOr(&c->bad_ts, 1u);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    c->ts0 = ts[0];
    c->ts_last = ts[n - 1];
    if (!ord) c->omax = (unsigned long long)(n - 1);
  }
}

// digit histograms of the rebased key for `npass` passes → hist[pass][kBins]
__global__ void __launch_bounds__(kBlock) key_hist_kernel(const void* __restrict__ kcol, int ktype, int64_t kmin,
                                                          int64_t n, int npass, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[4][kBins];
  for (int k = threadIdx.x; k < 4 * kBins; k += kBlock) (&h[0][0])[k] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t k = ktype == T_INT ? (int64_t)((const int32_t*)kcol)[i] : ((const int64_t*)kcol)[i];
    uint32_t r = (uint32_t)(k - kmin);
    for (int p = 0; p < npass; ++p) atomicAdd(&h[p][(r >> (p * kRB)) & (kBins - 1)], 1u);
  }
  __syncthreads();
  for (int p = 0; p < npass; ++p)
    for (int d = threadIdx.x; d < kBins; d += kBlock)
      if (h[p][d]) atomicAdd(&hist[p * kBins + d], h[p][d]);
}

// digit histograms of u32 values (j) whose count lives on the device
__global__ void __launch_bounds__(kBlock) u32_hist_kernel(const uint32_t* __restrict__ v, const unsigned int* n_dev,
                                                          int npass, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[4][kBins];
  for (int k = threadIdx.x; k < 4 * kBins; k += kBlock) (&h[0][0])[k] = 0;
  __syncthreads();
  const int64_t n = *n_dev;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t r = v[i];
    for (int p = 0; p < npass; ++p) atomicAdd(&h[p][(r >> (p * kRB)) & (kBins - 1)], 1u);
  }
  __syncthreads();
  for (int p = 0; p < npass; ++p)
    for (int d = threadIdx.x; d < kBins; d += kBlock)
      if (h[p][d]) atomicAdd(&hist[p * kBins + d], h[p][d]);
}

// in-place exclusive scan of each pass's histogram (one block per pass)
__global__ void __launch_bounds__(kBlock) hist_scan_kernel(uint32_t* __restrict__ hist) {
  __shared__ uint32_t lw[kWaves];
  uint32_t* h = hist + blockIdx.x * kBins;
  uint32_t v[kBinsPerThread], s = 0;
  for (int k = 0; k < kBinsPerThread; ++k) {
    v[k] = h[threadIdx.x * kBinsPerThread + k];
    s += v[k];
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t inc = s;
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t u = __shfl_up(inc, o, 64);
    if (lane >= o) inc += u;
  }
  if (lane == 63) lw[w] = inc;
  __syncthreads();
  uint32_t run = inc - s;
  for (int k = 0; k < w; ++k) run += lw[k];
  for (int k = 0; k < kBinsPerThread; ++k) {
    h[threadIdx.x * kBinsPerThread + k] = run;
    run += v[k];
  }
}

// ---------------------------------------------------------------- onesweep pass

// record sources / sinks
struct OrigSrc {  // pass 0 of the keyed sort: builds the record from the original columns
  const NfaStream* st;
  const void* kcol;
  int ktype;
  int64_t kmin;
  const Instr* c1;
  int c1_len;
  const DVal* consts;
  int vattr, vtype;
  const int64_t* ts;
  int64_t ts0;
  const int64_t* ord;
  int64_t obase;
  __device__ uint32_t key(int64_t p) const {
    int64_t k = ktype == T_INT ? (int64_t)((const int32_t*)kcol)[p] : ((const int64_t*)kcol)[p];
    RowLoader ld{st, p};
    const bool c = eval_cond(c1, c1_len, consts, ld);
    return (uint32_t)(k - kmin) | (c ? 0x80000000u : 0u);
  }
  __device__ uint32_t f0(int64_t p) const { return ord ? (uint32_t)(ord[p] - obase) : (uint32_t)p; }
  __device__ uint64_t f1(int64_t p) const { return canon(col_value(st, vattr, p), vtype); }
  __device__ uint32_t f2(int64_t p) const { return (uint32_t)(ts[p] - ts0); }
};

struct RecSoA {  // keyed record, structure of arrays
  uint32_t* k;
  uint32_t* f0;
  uint64_t* f1;
  uint32_t* f2;
};

struct RecSrc {
  const uint32_t* k;
  const uint32_t* f0;
  const uint64_t* f1;
  const uint32_t* f2;
  __device__ uint32_t key(int64_t p) const { return k[p]; }
  __device__ uint32_t g0(int64_t p) const { return f0[p]; }
};

// status word: epoch(30) | flag(2) | value(32); flag 1 = tile aggregate, 2 = inclusive prefix
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

// Shared onesweep core: ranks the tile's keys, runs the per-digit look-back and leaves, in LDS, for every
// record its local sorted position and every digit's global base. MODE selects the record layout moved.
//   MODE 0: keyed record, source = original columns (OrigSrc), sink = RecSoA
//   MODE 1: keyed record, source = RecSrc, sink = RecSoA
//   MODE 2: (j, i) pairs, source/sink = two u32 arrays
//   MODE 3: (j, i) pairs, source = two u32 arrays, sink = interleaved (i, j) u32 pairs
template <int MODE, typename Src>
__global__ void __launch_bounds__(kBlock) onesweep_kernel(Src src, RecSoA dst, uint32_t* __restrict__ dj,
                                                          uint32_t* __restrict__ di, uint64_t* __restrict__ dpairs,
                                                          int64_t n_host, const unsigned int* n_dev, int shift,
                                                          const uint32_t* __restrict__ gstart,
                                                          unsigned long long* __restrict__ status, uint32_t epoch,
                                                          unsigned int* __restrict__ tile_ctr,
                                                          unsigned int* __restrict__ err) {
  __shared__ uint64_t xbuf[kTile];
  __shared__ uint16_t wcnt[kWaves][kBins];
  __shared__ uint32_t tstart[kBins];
  __shared__ uint32_t gbase[kBins];
  __shared__ uint32_t lw[kWaves];
  __shared__ uint32_t sh_tile;
  uint32_t* xb32 = (uint32_t*)xbuf;

  const int64_t n = n_dev ? (int64_t)*n_dev : n_host;
  if (threadIdx.x == 0) sh_tile = atomicAdd(tile_ctr, 1u);
  for (int k = threadIdx.x; k < kWaves * kBins; k += kBlock) (&wcnt[0][0])[k] = 0;
  __syncthreads();
  const int64_t tile = sh_tile;
  const int64_t base = tile * kTile;
  if (base >= n) return;
  const int tile_n = (int)((n - base) < kTile ? (n - base) : kTile);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = lanemask_lt();

  uint32_t keys[kItems];
  uint32_t lp[kItems];  // rank within (wave, digit), then local sorted position
#pragma unroll
  for (int k = 0; k < kItems; ++k) {
    const int e = w * 64 * kItems + k * 64 + lane;
    const bool valid = e < tile_n;
    uint32_t key = 0;
    if (valid) key = src.key(base + e);
    keys[k] = key;
    const uint32_t d = ((key & kKeyMask) >> shift) & (kBins - 1);
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < kRB; ++b) {
      const bool bit = (d >> b) & 1u;
      const uint64_t bal = __ballot(bit);
      peers &= bit ? bal : ~bal;
    }
    uint32_t old = 0;
    if (valid) old = wcnt[w][d];
    const uint32_t below = (uint32_t)__popcll(peers & lt);
    if (valid && below == 0) wcnt[w][d] = (uint16_t)(old + (uint32_t)__popcll(peers));
    lp[k] = old + below;
  }
  __syncthreads();

  // per digit: wave offsets (exclusive, in place) and the tile count
  uint32_t cnt[kBinsPerThread];
  uint32_t csum = 0;
#pragma unroll
  for (int b = 0; b < kBinsPerThread; ++b) {
    const int d = threadIdx.x * kBinsPerThread + b;
    uint32_t run = 0;
    for (int q = 0; q < kWaves; ++q) {
      const uint32_t c = wcnt[q][d];
      wcnt[q][d] = (uint16_t)run;
      run += c;
    }
    cnt[b] = run;
    csum += run;
  }
  // block exclusive scan of the tile counts over digits → tstart
  {
    uint32_t inc = csum;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(inc, o, 64);
      if (lane >= o) inc += u;
    }
    if (lane == 63) lw[w] = inc;
    __syncthreads();
    uint32_t run = inc - csum;
    for (int q = 0; q < w; ++q) run += lw[q];
#pragma unroll
    for (int b = 0; b < kBinsPerThread; ++b) {
      const int d = threadIdx.x * kBinsPerThread + b;
      tstart[d] = run;
      run += cnt[b];
    }
  }
  // decoupled look-back per digit
#pragma unroll
  for (int b = 0; b < kBinsPerThread; ++b) {
    const int d = threadIdx.x * kBinsPerThread + b;
    const uint32_t excl = lookback(status + d, kBins, tile, epoch, cnt[b], err);
    gbase[d] = gstart[d] + excl;
  }
  __syncthreads();

  // local sorted positions; key exchange
#pragma unroll
  for (int k = 0; k < kItems; ++k) {
    const int e = w * 64 * kItems + k * 64 + lane;
    if (e < tile_n) {
      const uint32_t d = ((keys[k] & kKeyMask) >> shift) & (kBins - 1);
      lp[k] += tstart[d] + wcnt[w][d];
      xb32[lp[k]] = keys[k];
    }
  }
  __syncthreads();
  uint32_t dest[kItems];
#pragma unroll
  for (int r = 0; r < kItems; ++r) {
    const int s = r * kBlock + threadIdx.x;
    if (s < tile_n) {
      const uint32_t key = xb32[s];
      const uint32_t d = ((key & kKeyMask) >> shift) & (kBins - 1);
      dest[r] = gbase[d] + (uint32_t)s - tstart[d];
      if (MODE == 0 || MODE == 1) dst.k[dest[r]] = key;
      if (MODE == 2) dj[dest[r]] = key;
    }
  }

  if constexpr (MODE == 3) {  // (j, i) → interleaved (i, j): one 8-byte exchange
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const int e = w * 64 * kItems + k * 64 + lane;
      if (e < tile_n) xbuf[lp[k]] = ((uint64_t)keys[k] << 32) | src.g0(base + e);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
      const int s = r * kBlock + threadIdx.x;
      if (s < tile_n) dpairs[dest[r]] = xbuf[s];
    }
    return;
  } else {
    // payload field 0 (u32)
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const int e = w * 64 * kItems + k * 64 + lane;
      if (e < tile_n) {
        if constexpr (MODE == 0) xb32[lp[k]] = src.f0(base + e);
        else xb32[lp[k]] = src.g0(base + e);
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
      const int s = r * kBlock + threadIdx.x;
      if (s < tile_n) {
        if (MODE == 2) di[dest[r]] = xb32[s];
        else dst.f0[dest[r]] = xb32[s];
      }
    }
    if constexpr (MODE == 0 || MODE == 1) {
      // payload field 1 (u64)
      __syncthreads();
#pragma unroll
      for (int k = 0; k < kItems; ++k) {
        const int e = w * 64 * kItems + k * 64 + lane;
        if (e < tile_n) {
          if constexpr (MODE == 0) xbuf[lp[k]] = src.f1(base + e);
          else xbuf[lp[k]] = src.f1[base + e];
        }
      }
      __syncthreads();
#pragma unroll
      for (int r = 0; r < kItems; ++r) {
        const int s = r * kBlock + threadIdx.x;
        if (s < tile_n) dst.f1[dest[r]] = xbuf[s];
      }
      // payload field 2 (u32)
      __syncthreads();
#pragma unroll
      for (int k = 0; k < kItems; ++k) {
        const int e = w * 64 * kItems + k * 64 + lane;
        if (e < tile_n) {
          if constexpr (MODE == 0) xb32[lp[k]] = src.f2(base + e);
          else xb32[lp[k]] = src.f2[base + e];
        }
      }
      __syncthreads();
#pragma unroll
      for (int r = 0; r < kItems; ++r) {
        const int s = r * kBlock + threadIdx.x;
        if (s < tile_n) dst.f2[dest[r]] = xb32[s];
      }
    }
  }
}

struct PairSrc {
  const uint32_t* j;
  const uint32_t* i;
  __device__ uint32_t key(int64_t p) const { return j[p]; }
  __device__ uint32_t g0(int64_t p) const { return i[p]; }
};

// ---------------------------------------------------------------- walk

struct WalkArgs {
  // keyed (sorted records) or original columns
  const uint32_t* k;
  const uint32_t* f0;
  const uint64_t* f1;
  const uint32_t* f2;
  const NfaStream* st;
  const int64_t* ts;
  const int64_t* ord;
  int64_t obase;
  const Instr* c1;
  int c1_len;
  const Instr* c2;
  int c2_len;
  const DVal* consts;
  int vattr, vtype;
  int64_t within;
  int64_t n;
};

template <bool KEYED>
__global__ void __launch_bounds__(kWalkBlock) walk_kernel(WalkArgs a, uint32_t* __restrict__ mj,
                                                          uint32_t* __restrict__ mi,
                                                          unsigned long long* __restrict__ status, uint32_t epoch,
                                                          unsigned int* __restrict__ tile_ctr,
                                                          unsigned int* __restrict__ nmatch,
                                                          unsigned int* __restrict__ err) {
  __shared__ uint32_t wtot[kWalkBlock / 64];
  __shared__ uint32_t sh_tile, sh_base;
  if (threadIdx.x == 0) sh_tile = atomicAdd(tile_ctr, 1u);
  __syncthreads();
  const int64_t tile = sh_tile;
  const int64_t base = tile * kWalkTile;
  const int64_t n = a.n;
  if (base >= n) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = lanemask_lt();
  uint32_t jv[kWalkItems], iv[kWalkItems];
  uint64_t hm[kWalkItems];
  uint32_t mine = 0;  // matches of this wave before item k (running, wave-uniform)
  uint32_t woff[kWalkItems];
#pragma unroll
  for (int k = 0; k < kWalkItems; ++k) {
    const int64_t u = base + w * 64 * kWalkItems + k * 64 + lane;
    bool has = false;
    uint32_t j = 0, i = 0;
    if (u < n) {
      if constexpr (KEYED) {
        const uint32_t ku = a.k[u];
        if (ku >> 31) {
          const uint32_t key = ku & kKeyMask, tu = a.f2[u];
          const uint64_t vu = a.f1[u];
          for (int64_t v = u + 1; v < n; ++v) {
            const uint32_t kv = a.k[v];
            if ((kv & kKeyMask) != key) break;
            if (a.within >= 0 && (int64_t)(a.f2[v] - tu) > a.within) break;
            PairLoader ld{vu, a.f1[v], a.vtype};
            if (eval_cond(a.c2, a.c2_len, a.consts, ld)) {
              has = true;
              j = a.f0[v];
              i = a.f0[u];
              break;
            }
          }
        }
      } else {
        RowLoader rl{a.st, u};
        if (eval_cond(a.c1, a.c1_len, a.consts, rl)) {
          const int64_t tu = a.ts[u];
          const uint64_t vu = canon(col_value(a.st, a.vattr, u), a.vtype);
          for (int64_t v = u + 1; v < n; ++v) {
            const int64_t d = a.ts[v] - tu;
            if (a.within >= 0 && (d < 0 ? -d : d) > a.within) break;
            PairLoader ld{vu, canon(col_value(a.st, a.vattr, v), a.vtype), a.vtype};
            if (eval_cond(a.c2, a.c2_len, a.consts, ld)) {
              has = true;
              j = a.ord ? (uint32_t)(a.ord[v] - a.obase) : (uint32_t)v;
              i = a.ord ? (uint32_t)(a.ord[u] - a.obase) : (uint32_t)u;
              break;
            }
          }
        }
      }
    }
    const uint64_t bal = __ballot(has);
    hm[k] = bal;
    woff[k] = mine + (uint32_t)__popcll(bal & lt);
    mine += (uint32_t)__popcll(bal);
    jv[k] = j;
    iv[k] = i;
  }
  if (lane == 0) wtot[w] = mine;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int q = 0; q < kWalkBlock / 64; ++q) {
      const uint32_t c = wtot[q];
      wtot[q] = t;
      t += c;
    }
    const uint32_t excl = lookback(status, 1, tile, epoch, t, err);
    sh_base = excl;
    if (base + kWalkTile >= n) *nmatch = excl + t;  // last tile publishes the total
  }
  __syncthreads();
  const uint32_t ob = sh_base + wtot[w];
#pragma unroll
  for (int k = 0; k < kWalkItems; ++k) {
    if ((hm[k] >> lane) & 1ull) {
      mj[ob + woff[k]] = jv[k];
      mi[ob + woff[k]] = iv[k];
    }
  }
}

inline int bits_for(uint64_t v) {
  int b = 0;
  while (b < 64 && (v >> b) != 0) ++b;
  return b;
}

}  // namespace

// Returns -1 when the batch is outside the v2 envelope (caller takes the general path).
int64_t fast_every_within_v2(const FastArgs& a, const FastHostInfo& hi, FastState& fs, uint32_t* pairs_out,
                             int64_t pairs_cap, Scratch& sc, hipStream_t s, FastTimings* tm) {
  const int64_t n = a.n;
  if (n == 0) return 0;
  if (n >= 0x7fffffffll || hi.vattr < 0) return -1;
  const bool keyed = a.key != nullptr;
  if (keyed && (hi.key_col < 0 || !(hi.key_type == T_INT || hi.key_type == T_LONG))) return -1;
  size_t mark = sc.used;
  Ctrl* c = (Ctrl*)sc.take(sizeof(Ctrl));
  {
    Ctrl init{};
    init.kmin = ~0ull;
    SM_HIP(hipMemcpyAsync(c, &init, sizeof(Ctrl), hipMemcpyHostToDevice, s));
  }
  const void* kcol = keyed ? hi.cols[hi.key_col] : nullptr;
  const unsigned grid_rd = (unsigned)std::min<int64_t>(2048, (n + 511) / 512);
  if (tm) SM_HIP(hipEventRecord(tm->ev[0], s));
  hipLaunchKernelGGL(prep_kernel, dim3(grid_rd), dim3(512), 0, s, kcol, hi.key_type, a.ts, a.ordinals,
                     a.ordinal_base, n, c);
  Ctrl hc;
  SM_HIP(hipMemcpyAsync(&hc, c, sizeof(Ctrl), hipMemcpyDeviceToHost, s));
  SM_HIP(hipStreamSynchronize(s));
  auto bail = [&]() -> int64_t {
    sc.used = mark;
    return -1;
  };
  if (a.within >= 0) {
    if (hc.bad_ts) {
      sc.used = mark;
      throw std::runtime_error("fast path requires non-decreasing event timestamps within a device batch");
    }
    if ((unsigned long long)(hc.ts_last - hc.ts0) >= 0xffffffffull) return bail();
  }
  if (hc.omax >= 0x7fffffffull) return bail();
  int kbits = 0;
  int64_t kmin = 0;
  if (keyed) {
    const uint64_t span = hc.kmax - hc.kmin;
    kbits = std::max(1, bits_for(span));
    if (kbits > 30) return bail();
    kmin = (int64_t)(hc.kmin ^ 0x8000000000000000ull);
  }
  const int fpass = keyed ? (kbits + kRB - 1) / kRB : 0;
  const int jbits = std::max(1, bits_for(hc.omax));
  const int jpass = (jbits + kRB - 1) / kRB;

  // persistent look-back status (epoch-tagged, zeroed once at allocation)
  const int64_t tiles = (n + kTile - 1) / kTile;
  const int64_t wtiles = (n + kWalkTile - 1) / kWalkTile;
  const size_t need = (size_t)std::max<int64_t>(tiles * kBins, wtiles) * 8;
  if (fs.status_bytes < need) {
    if (fs.status) SM_HIP(hipFree(fs.status));
    SM_HIP(hipMalloc(&fs.status, need));
    SM_HIP(hipMemsetAsync(fs.status, 0, need, s));
    fs.status_bytes = need;
  }
  unsigned long long* status = (unsigned long long*)fs.status;
  uint32_t* hist = (uint32_t*)sc.take(sizeof(uint32_t) * kBins * 8);
  SM_HIP(hipMemsetAsync(hist, 0, sizeof(uint32_t) * kBins * 8, s));
  unsigned int* ctr = &c->tile_ctr[0];
  int ctr_used = 0;

  // record buffers
  RecSoA A{}, B{};
  uint32_t *mj = nullptr, *mi = nullptr, *pj = nullptr, *pi = nullptr;
  const unsigned sort_grid = (unsigned)tiles;
  if (keyed) {
    A.k = (uint32_t*)sc.take(n * 4);
    A.f0 = (uint32_t*)sc.take(n * 4);
    A.f1 = (uint64_t*)sc.take(n * 8);
    A.f2 = (uint32_t*)sc.take(n * 4);
    B.k = (uint32_t*)sc.take(n * 4);
    B.f0 = (uint32_t*)sc.take(n * 4);
    B.f1 = (uint64_t*)sc.take(n * 8);
    B.f2 = (uint32_t*)sc.take(n * 4);
    hipLaunchKernelGGL(key_hist_kernel, dim3(grid_rd), dim3(kBlock), 0, s, kcol, hi.key_type, kmin, n, fpass, hist);
    hipLaunchKernelGGL(hist_scan_kernel, dim3(fpass), dim3(kBlock), 0, s, hist);
    OrigSrc os{a.st, kcol, hi.key_type, kmin, a.code + a.c1_off, a.c1_len, a.consts, hi.vattr, hi.vtype, a.ts,
               hc.ts0, a.ordinals, a.ordinal_base};
    hipLaunchKernelGGL((onesweep_kernel<0, OrigSrc>), dim3(sort_grid), dim3(kBlock), 0, s, os, A, nullptr, nullptr,
                       nullptr, n, nullptr, 0, hist, status, ++fs.epoch, ctr + ctr_used++, &c->err);
    RecSoA* cur = &A;
    RecSoA* nxt = &B;
    for (int p = 1; p < fpass; ++p) {
      RecSrc rs{cur->k, cur->f0, cur->f1, cur->f2};
      hipLaunchKernelGGL((onesweep_kernel<1, RecSrc>), dim3(sort_grid), dim3(kBlock), 0, s, rs, *nxt, nullptr,
                         nullptr, nullptr, n, nullptr, p * kRB, hist + p * kBins, status, ++fs.epoch,
                         ctr + ctr_used++, &c->err);
      std::swap(cur, nxt);
    }
    if (tm) SM_HIP(hipEventRecord(tm->ev[1], s));
    WalkArgs wa{cur->k, cur->f0, cur->f1, cur->f2, a.st, a.ts, a.ordinals, a.ordinal_base,
                a.code + a.c1_off, a.c1_len, a.code + a.c2_off, a.c2_len, a.consts, hi.vattr, hi.vtype,
                a.within, n};
    // (j, i) into the dead buffer; ping-pong partner carved from it too (n*8 + n*8 <= 20n)
    mj = (uint32_t*)nxt->k;
    mi = nxt->f0;
    pj = (uint32_t*)nxt->f1;
    pi = (uint32_t*)nxt->f1 + n;
    hipLaunchKernelGGL((walk_kernel<true>), dim3((unsigned)wtiles), dim3(kWalkBlock), 0, s, wa, mj, mi, status,
                       ++fs.epoch, ctr + ctr_used++, &c->nmatch, &c->err);
  } else {
    if (tm) SM_HIP(hipEventRecord(tm->ev[1], s));
    mj = (uint32_t*)sc.take(n * 4);
    mi = (uint32_t*)sc.take(n * 4);
    pj = (uint32_t*)sc.take(n * 4);
    pi = (uint32_t*)sc.take(n * 4);
    WalkArgs wa{nullptr, nullptr, nullptr, nullptr, a.st, a.ts, a.ordinals, a.ordinal_base,
                a.code + a.c1_off, a.c1_len, a.code + a.c2_off, a.c2_len, a.consts, hi.vattr, hi.vtype,
                a.within, n};
    hipLaunchKernelGGL((walk_kernel<false>), dim3((unsigned)wtiles), dim3(kWalkBlock), 0, s, wa, mj, mi, status,
                       ++fs.epoch, ctr + ctr_used++, &c->nmatch, &c->err);
  }
  if (tm) SM_HIP(hipEventRecord(tm->ev[2], s));

  // order by j: LSD passes over (j, i); the last one writes the interleaved output
  uint32_t* jh = hist + 4 * kBins;
  hipLaunchKernelGGL(u32_hist_kernel, dim3(grid_rd), dim3(kBlock), 0, s, mj, &c->nmatch, jpass, jh);
  hipLaunchKernelGGL(hist_scan_kernel, dim3(jpass), dim3(kBlock), 0, s, jh);
  uint32_t *cj = mj, *ci = mi, *nj = pj, *ni = pi;
  for (int p = 0; p < jpass; ++p) {
    PairSrc ps{cj, ci};
    if (p == jpass - 1) {
      hipLaunchKernelGGL((onesweep_kernel<3, PairSrc>), dim3(sort_grid), dim3(kBlock), 0, s, ps, RecSoA{}, nullptr,
                         nullptr, (uint64_t*)pairs_out, n, &c->nmatch, p * kRB, jh + p * kBins, status, ++fs.epoch,
                         ctr + ctr_used++, &c->err);
    } else {
      hipLaunchKernelGGL((onesweep_kernel<2, PairSrc>), dim3(sort_grid), dim3(kBlock), 0, s, ps, RecSoA{}, nj, ni,
                         nullptr, n, &c->nmatch, p * kRB, jh + p * kBins, status, ++fs.epoch, ctr + ctr_used++,
                         &c->err);
      std::swap(cj, nj);
      std::swap(ci, ni);
    }
  }
  if (tm) SM_HIP(hipEventRecord(tm->ev[3], s));
  SM_HIP(hipMemcpyAsync(&hc, c, sizeof(Ctrl), hipMemcpyDeviceToHost, s));
  SM_HIP(hipStreamSynchronize(s));
  sc.used = mark;
  if (hc.err) throw std::runtime_error("fast path: look-back did not converge (device error)");
  if ((int64_t)hc.nmatch > pairs_cap) throw std::runtime_error("match buffer too small");
  (void)ctr_used;
  return (int64_t)hc.nmatch;
}

}  // namespace sm
