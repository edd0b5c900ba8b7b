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
#include "lookback.h"

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
constexpr int kWalkHalo = 256;  // records staged past the tile for scans that leave it
constexpr int kWalkLds = kWalkTile + kWalkHalo;
constexpr int kLookW = 8;  // look-back window (independent status loads per step)

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

// A condition program decoded once per thread: its kernel-uniform instructions and constants stay in scalar
// registers across the scan loops instead of being re-read every iteration.
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
// canonical 64-bit image of a typed column value (as canon(), with the column type fixed at compile time)
template <typename VT>
__device__ __forceinline__ uint64_t canon_t(VT v) {
  if constexpr (std::is_floating_point<VT>::value) return (uint64_t)__double_as_longlong((double)v);
  else return (uint64_t)(int64_t)v;
}

// Pass 0 of the keyed sort: builds the record from the original columns. Key and compared-attribute column
// types are template parameters (no per-element type switch in the unrolled item loops); c1 is evaluated by
// c1(), once per event, outside the unrolled loops.
template <typename KT, typename VT>
struct OrigSrc {
  static constexpr bool kC1 = true;
  const NfaStream* st;
  const KT* kcol;
  const VT* vcol;
  int64_t kmin;
  const Instr* c1p;
  int c1_len;
  const DVal* consts;
  const int64_t* ts;
  int64_t ts0;
  const int64_t* ord;
  int64_t obase;
  __device__ uint32_t key(int64_t p) const { return (uint32_t)((int64_t)kcol[p] - kmin); }
  __device__ bool c1(int64_t p) const {
    RowLoader ld{st, p};
    return eval_cond(c1p, c1_len, consts, ld);
  }
  __device__ uint32_t f0(int64_t p) const { return ord ? (uint32_t)(ord[p] - obase) : (uint32_t)p; }
  __device__ uint64_t f1(int64_t p) const { return canon_t(vcol[p]); }
  __device__ uint32_t f2(int64_t p) const { return (uint32_t)(ts[p] - ts0); }
};

struct RecSoA {  // keyed record, structure of arrays
  uint32_t* k;
  uint32_t* f0;
  uint64_t* f1;
  uint32_t* f2;
};

struct RecSrc {
  static constexpr bool kC1 = false;
  const uint32_t* k;
  const uint32_t* f0;
  const uint64_t* f1;
  const uint32_t* f2;
  __device__ uint32_t key(int64_t p) const { return k[p]; }
  __device__ uint32_t g0(int64_t p) const { return f0[p]; }
};

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
  __shared__ uint32_t xb32[kTile];  // exchange buffer, one 32-bit field at a time (u64 fields in two halves)
  __shared__ uint16_t wcnt[kWaves][kBins];
  __shared__ uint32_t tstart[kBins];
  __shared__ uint32_t gbase[kBins];
  __shared__ uint32_t tcnt[kBins];
  __shared__ uint32_t lw[kWaves];
  __shared__ uint32_t sh_tile;

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

  uint32_t c1m = 0;  // c1 flag of each item (bit k), evaluated in a rolled loop to keep the code compact
  if constexpr (Src::kC1) {
#pragma unroll 1
    for (int k = 0; k < kItems; ++k) {
      const int e = w * 64 * kItems + k * 64 + lane;
      if (e < tile_n && src.c1(base + e)) c1m |= 1u << k;
    }
  }
  uint32_t keys[kItems];
  uint32_t lp[kItems];  // rank within (wave, digit), then local sorted position
#pragma unroll
  for (int k = 0; k < kItems; ++k) {
    const int e = w * 64 * kItems + k * 64 + lane;
    const bool valid = e < tile_n;
    uint32_t key = 0;
    if (valid) key = src.key(base + e) | (((c1m >> k) & 1u) << 31);
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
  // decoupled look-back per digit; lanes take consecutive digits so each status read is coalesced
#pragma unroll
  for (int b = 0; b < kBinsPerThread; ++b) tcnt[threadIdx.x * kBinsPerThread + b] = cnt[b];
  __syncthreads();
#pragma unroll
  for (int b = 0; b < kBinsPerThread; ++b) {
    const int d = b * kBlock + threadIdx.x;
    const uint32_t excl = lookback_win<kLookW>(status + d, kBins, tile, epoch, tcnt[d], err);
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

  if constexpr (MODE == 3) {  // (j, i) → interleaved (i, j): j is already in xb32 at the sorted slots
    uint32_t jj[kItems];
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
      const int s = r * kBlock + threadIdx.x;
      jj[r] = s < tile_n ? xb32[s] : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const int e = w * 64 * kItems + k * 64 + lane;
      if (e < tile_n) xb32[lp[k]] = src.g0(base + e);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
      const int s = r * kBlock + threadIdx.x;
      if (s < tile_n) dpairs[dest[r]] = ((uint64_t)jj[r] << 32) | xb32[s];
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
      // payload field 1 (u64), low then high half
      uint32_t hi[kItems];
      __syncthreads();
#pragma unroll
      for (int k = 0; k < kItems; ++k) {
        const int e = w * 64 * kItems + k * 64 + lane;
        if (e < tile_n) {
          uint64_t x;
          if constexpr (MODE == 0) x = src.f1(base + e);
          else x = src.f1[base + e];
          xb32[lp[k]] = (uint32_t)x;
          hi[k] = (uint32_t)(x >> 32);
        }
      }
      __syncthreads();
      uint32_t lo[kItems];
#pragma unroll
      for (int r = 0; r < kItems; ++r) {
        const int s = r * kBlock + threadIdx.x;
        lo[r] = s < tile_n ? xb32[s] : 0u;
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < kItems; ++k) {
        const int e = w * 64 * kItems + k * 64 + lane;
        if (e < tile_n) xb32[lp[k]] = hi[k];
      }
      __syncthreads();
#pragma unroll
      for (int r = 0; r < kItems; ++r) {
        const int s = r * kBlock + threadIdx.x;
        if (s < tile_n) dst.f1[dest[r]] = ((uint64_t)xb32[s] << 32) | lo[r];
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
  static constexpr bool kC1 = false;
  const uint32_t* j;
  const uint32_t* i;
  __device__ uint32_t key(int64_t p) const { return j[p]; }
  __device__ uint32_t g0(int64_t p) const { return i[p]; }
};

// ---------------------------------------------------------------- walk
//
// One lane per record (tile order = record order, so the look-back compaction keeps matches in record order).
// The tile's records plus a halo of the next kWalkHalo records are staged into LDS with coalesced loads; every
// forward scan reads LDS and leaves it only when a key run (keyed) or a window (unkeyed) runs past the halo,
// where it continues from global memory. A scan stops at the first event satisfying c2 (match), at the end of
// the key run, or when the window closes.

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
struct WalkLds;
template <>
struct WalkLds<true> {
  uint64_t v[kWalkLds];
  uint32_t k[kWalkLds];
  uint32_t t[kWalkLds];
};
template <>
struct WalkLds<false> {
  uint64_t v[kWalkLds];
  int64_t t[kWalkLds];
};

// Forward scan of one partial (record lu of the tile, keyed: c1 already known to hold). Returns the position
// of the first event satisfying c2 inside the key run (keyed) and the window, or -1.
// c2 as a fixed compare `e2.x OP e1.x` over the carried attribute (OP >= 0; FP: compared as double, else as
// int64 — exact for every column type the spec admits), or the generic condition program (OP < 0).
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

template <bool KEYED, typename CF>
__device__ __forceinline__ int64_t scan_partial(const WalkArgs& a, const WalkLds<KEYED>& L, const CF& c2,
                                                int64_t base, int64_t lend, int lu) {
  const int64_t n = a.n;
  const uint64_t vu = L.v[lu];
  int64_t v = base + lu + 1;
  if constexpr (KEYED) {
    const uint32_t key = L.k[lu] & kKeyMask, tu = L.t[lu];
    for (; v < lend; ++v) {  // staged records
      const int lv = (int)(v - base);
      if ((L.k[lv] & kKeyMask) != key || (a.within >= 0 && (int64_t)(L.t[lv] - tu) > a.within)) return -1;
      if (c2(vu, L.v[lv])) return v;
    }
    for (; v < n; ++v) {  // the key run continues past the halo
      if ((a.k[v] & kKeyMask) != key || (a.within >= 0 && (int64_t)(a.f2[v] - tu) > a.within)) return -1;
      if (c2(vu, a.f1[v])) return v;
    }
  } else {
    const int64_t tu = L.t[lu];
    for (; v < lend; ++v) {
      const int64_t d = L.t[v - base] - tu;
      if (a.within >= 0 && (d < 0 ? -d : d) > a.within) return -1;
      if (c2(vu, L.v[v - base])) return v;
    }
    for (; v < n; ++v) {
      const int64_t d = a.ts[v] - tu;
      if (a.within >= 0 && (d < 0 ? -d : d) > a.within) return -1;
      if (c2(vu, canon(col_value(a.st, a.vattr, v), a.vtype))) return v;
    }
  }
  return -1;
}

template <bool KEYED, int OP, bool FP>
__global__ void __launch_bounds__(kWalkBlock) walk_kernel(WalkArgs a, uint32_t* __restrict__ mj,
                                                          uint32_t* __restrict__ mi,
                                                          unsigned long long* __restrict__ status, uint32_t epoch,
                                                          unsigned int* __restrict__ tile_ctr,
                                                          unsigned int* __restrict__ nmatch,
                                                          unsigned int* __restrict__ err) {
  __shared__ WalkLds<KEYED> L;
  __shared__ uint32_t sj[kWalkItems][kWalkBlock];      // matched position of each item (valid where bal bit set)
  __shared__ uint64_t sbal[kWalkBlock / 64][kWalkItems];
  __shared__ uint32_t wtot[kWalkBlock / 64];
  __shared__ uint32_t sh_tile, sh_base;
  if (threadIdx.x == 0) sh_tile = atomicAdd(tile_ctr, 1u);
  __syncthreads();
  const int64_t tile = sh_tile;
  const int64_t base = tile * kWalkTile;
  const int64_t n = a.n;
  if (base >= n) return;
  const int nload = (int)((n - base) < kWalkLds ? (n - base) : kWalkLds);
  for (int e = threadIdx.x; e < nload; e += kWalkBlock) {
    const int64_t p = base + e;
    if constexpr (KEYED) {
      L.k[e] = a.k[p];
      L.t[e] = a.f2[p];
      L.v[e] = a.f1[p];
    } else {
      L.t[e] = a.ts[p];
      L.v[e] = canon(col_value(a.st, a.vattr, p), a.vtype);
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = lanemask_lt();
  const int64_t lend = base + nload;
  C2<OP, FP> c2;
  if constexpr (OP < 0) c2.c = make_cond(a.c2, a.c2_len, a.consts);
  c2.vtype = a.vtype;
  Cond c1;
  if constexpr (!KEYED) c1 = make_cond(a.c1, a.c1_len, a.consts);
  uint32_t mine = 0;  // matches of this wave (wave-uniform)
  // items in a rolled loop (one copy of the scan code); per-item results go through LDS
#pragma unroll 1
  for (int k = 0; k < kWalkItems; ++k) {
    const int lu = w * 64 * kWalkItems + k * 64 + lane;
    const int64_t u = base + lu;
    int64_t hit = -1;
    if (u < n) {
      bool c1u;
      if constexpr (KEYED) c1u = (L.k[lu] >> 31) != 0;
      else c1u = eval(c1, RowLoader{a.st, u});
      if (c1u) hit = scan_partial<KEYED>(a, L, c2, base, lend, lu);
    }
    const uint64_t bal = __ballot(hit >= 0);
    if (hit >= 0) sj[k][threadIdx.x] = (uint32_t)(hit - base);  // < 2^31: offset inside or past the tile
    if (lane == 0) sbal[w][k] = bal;
    mine += (uint32_t)__popcll(bal);
  }
  if (lane == 0) wtot[w] = mine;
  __syncthreads();
  if (threadIdx.x < 64) {
    uint32_t t = 0, mywt = 0;
    for (int q = 0; q < kWalkBlock / 64; ++q) {
      const uint32_t c = wtot[q];
      if (q == lane) mywt = t;
      t += c;
    }
    const uint32_t excl = lookback_wave(status, tile, epoch, t, err);
    if (lane < kWalkBlock / 64) wtot[lane] = mywt;
    if (lane == 0) {
      sh_base = excl;
      if (base + kWalkTile >= n) *nmatch = excl + t;  // last tile publishes the total
    }
  }
  __syncthreads();
  uint32_t ob = sh_base + wtot[w];
#pragma unroll 1
  for (int k = 0; k < kWalkItems; ++k) {
    const uint64_t bal = sbal[w][k];
    if ((bal >> lane) & 1ull) {
      const uint32_t pos = ob + (uint32_t)__popcll(bal & lt);
      const int64_t u = base + w * 64 * kWalkItems + k * 64 + lane;
      const int64_t v = base + sj[k][threadIdx.x];
      if constexpr (KEYED) {
        mj[pos] = a.f0[v];
        mi[pos] = a.f0[u];
      } else {
        mj[pos] = a.ord ? (uint32_t)(a.ord[v] - a.obase) : (uint32_t)v;
        mi[pos] = a.ord ? (uint32_t)(a.ord[u] - a.obase) : (uint32_t)u;
      }
    }
    ob += (uint32_t)__popcll(bal);
  }
}

inline int bits_for(uint64_t v) {
  int b = 0;
  while (b < 64 && (v >> b) != 0) ++b;
  return b;
}

}  // namespace

template <typename KT, typename VT>
void launch_pass0_t(const FastHostInfo& hi, const FastArgs& a, const void* kcol, int64_t kmin, int64_t ts0,
                    unsigned grid, hipStream_t s, RecSoA dst, const uint32_t* hist, unsigned long long* status,
                    uint32_t epoch, unsigned int* ctr, unsigned int* err) {
  OrigSrc<KT, VT> os{a.st, (const KT*)kcol, (const VT*)hi.cols[hi.vattr], kmin, a.code + a.c1_off, a.c1_len,
                     a.consts, a.ts, ts0, a.ordinals, a.ordinal_base};
  hipLaunchKernelGGL((onesweep_kernel<0, OrigSrc<KT, VT>>), dim3(grid), dim3(kBlock), 0, s, os, dst, nullptr,
                     nullptr, nullptr, a.n, nullptr, 0, hist, status, epoch, ctr, err);
}

template <typename KT>
void launch_pass0_k(const FastHostInfo& hi, const FastArgs& a, const void* kcol, int64_t kmin, int64_t ts0,
                    unsigned grid, hipStream_t s, RecSoA dst, const uint32_t* hist, unsigned long long* status,
                    uint32_t epoch, unsigned int* ctr, unsigned int* err) {
  switch (hi.vtype) {
    case T_INT: launch_pass0_t<KT, int32_t>(hi, a, kcol, kmin, ts0, grid, s, dst, hist, status, epoch, ctr, err); break;
    case T_LONG: launch_pass0_t<KT, int64_t>(hi, a, kcol, kmin, ts0, grid, s, dst, hist, status, epoch, ctr, err); break;
    case T_FLOAT: launch_pass0_t<KT, float>(hi, a, kcol, kmin, ts0, grid, s, dst, hist, status, epoch, ctr, err); break;
    case T_DOUBLE: launch_pass0_t<KT, double>(hi, a, kcol, kmin, ts0, grid, s, dst, hist, status, epoch, ctr, err); break;
    default: throw std::runtime_error("fast path: unsupported compared-attribute type");
  }
}

void launch_pass0(const FastHostInfo& hi, const FastArgs& a, const void* kcol, int64_t kmin, int64_t ts0,
                  unsigned grid, hipStream_t s, RecSoA dst, const uint32_t* hist, unsigned long long* status,
                  uint32_t epoch, unsigned int* ctr, unsigned int* err) {
  if (hi.key_type == T_INT) launch_pass0_k<int32_t>(hi, a, kcol, kmin, ts0, grid, s, dst, hist, status, epoch, ctr, err);
  else launch_pass0_k<int64_t>(hi, a, kcol, kmin, ts0, grid, s, dst, hist, status, epoch, ctr, err);
}

// Compare spec of c2 for the walk: op * 2 + fp, normalised to `e2.x OP e1.x`, or -1 (generic program).
// Admitted: `eK.x CMP eL.x` over the carried attribute, one operand per slot, compared in its own type.
int c2_spec(const FastHostInfo& hi) {
  if (!hi.c2_host || hi.c2_len != 3) return -1;
  const Instr* c = hi.c2_host;
  if (c[0].op != OP_VAR || c[1].op != OP_VAR || c[2].op != OP_CMP) return -1;
  if (c[0].c != hi.vattr || c[1].c != hi.vattr || c[0].a == c[1].a) return -1;
  const int ct = c[2].t0;
  const bool ok = (hi.vtype == T_DOUBLE && ct == CT_DOUBLE) || (hi.vtype == T_FLOAT && ct == CT_FLOAT) ||
                  (hi.vtype == T_INT && ct == CT_INT) || (hi.vtype == T_LONG && ct == CT_LONG);
  if (!ok) return -1;
  int op = c[2].sub;
  if (c[0].a == 0) {  // e1 OP e2  →  e2 OP' e1
    static const int flip[6] = {CMP_EQ, CMP_NE, CMP_GT, CMP_GE, CMP_LT, CMP_LE};
    op = flip[op];
  }
  const bool fp = hi.vtype == T_DOUBLE || hi.vtype == T_FLOAT;
  return op * 2 + (fp ? 1 : 0);
}

template <bool KEYED, int OP, bool FP>
void launch_walk_t(int64_t tiles, hipStream_t s, const WalkArgs& wa, uint32_t* mj, uint32_t* mi,
                   unsigned long long* status, uint32_t epoch, unsigned int* ctr, unsigned int* nmatch,
                   unsigned int* err) {
  hipLaunchKernelGGL((walk_kernel<KEYED, OP, FP>), dim3((unsigned)tiles), dim3(kWalkBlock), 0, s, wa, mj, mi, status,
                     epoch, ctr, nmatch, err);
}

template <bool KEYED>
void launch_walk(int spec, int64_t tiles, hipStream_t s, const WalkArgs& wa, uint32_t* mj, uint32_t* mi,
                 unsigned long long* status, uint32_t epoch, unsigned int* ctr, unsigned int* nmatch,
                 unsigned int* err) {
#define SM_WALK(OP, FP) launch_walk_t<KEYED, OP, FP>(tiles, s, wa, mj, mi, status, epoch, ctr, nmatch, err)
  switch (spec) {
    case CMP_EQ * 2: SM_WALK(CMP_EQ, false); break;
    case CMP_EQ * 2 + 1: SM_WALK(CMP_EQ, true); break;
    case CMP_NE * 2: SM_WALK(CMP_NE, false); break;
    case CMP_NE * 2 + 1: SM_WALK(CMP_NE, true); break;
    case CMP_LT * 2: SM_WALK(CMP_LT, false); break;
    case CMP_LT * 2 + 1: SM_WALK(CMP_LT, true); break;
    case CMP_LE * 2: SM_WALK(CMP_LE, false); break;
    case CMP_LE * 2 + 1: SM_WALK(CMP_LE, true); break;
    case CMP_GT * 2: SM_WALK(CMP_GT, false); break;
    case CMP_GT * 2 + 1: SM_WALK(CMP_GT, true); break;
    case CMP_GE * 2: SM_WALK(CMP_GE, false); break;
    case CMP_GE * 2 + 1: SM_WALK(CMP_GE, true); break;
    default: SM_WALK(-1, false); break;
  }
#undef SM_WALK
}

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
  if (tm) {
    SM_HIP(hipEventRecord(tm->ev[0], s));
    tm->nmk = 0;
    tm->mark("start", s);
  }
  auto tmark = [&](const char* l) {
    if (tm) tm->mark(l, s);
  };
  hipLaunchKernelGGL(prep_kernel, dim3(grid_rd), dim3(512), 0, s, kcol, hi.key_type, a.ts, a.ordinals,
                     a.ordinal_base, n, c);
  tmark("prep");
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
    tmark("key_hist");
    hipLaunchKernelGGL(hist_scan_kernel, dim3(fpass), dim3(kBlock), 0, s, hist);
    tmark("hist_scan");
    launch_pass0(hi, a, kcol, kmin, hc.ts0, sort_grid, s, A, hist, status, ++fs.epoch, ctr + ctr_used++, &c->err);
    tmark("key_pass0");
    RecSoA* cur = &A;
    RecSoA* nxt = &B;
    for (int p = 1; p < fpass; ++p) {
      RecSrc rs{cur->k, cur->f0, cur->f1, cur->f2};
      hipLaunchKernelGGL((onesweep_kernel<1, RecSrc>), dim3(sort_grid), dim3(kBlock), 0, s, rs, *nxt, nullptr,
                         nullptr, nullptr, n, nullptr, p * kRB, hist + p * kBins, status, ++fs.epoch,
                         ctr + ctr_used++, &c->err);
      tmark("key_pass");
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
    launch_walk<true>(c2_spec(hi), wtiles, s, wa, mj, mi, status, ++fs.epoch, ctr + ctr_used++, &c->nmatch, &c->err);
    tmark("walk");
  } else {
    if (tm) SM_HIP(hipEventRecord(tm->ev[1], s));
    mj = (uint32_t*)sc.take(n * 4);
    mi = (uint32_t*)sc.take(n * 4);
    pj = (uint32_t*)sc.take(n * 4);
    pi = (uint32_t*)sc.take(n * 4);
    WalkArgs wa{nullptr, nullptr, nullptr, nullptr, a.st, a.ts, a.ordinals, a.ordinal_base,
                a.code + a.c1_off, a.c1_len, a.code + a.c2_off, a.c2_len, a.consts, hi.vattr, hi.vtype,
                a.within, n};
    launch_walk<false>(c2_spec(hi), wtiles, s, wa, mj, mi, status, ++fs.epoch, ctr + ctr_used++, &c->nmatch, &c->err);
    tmark("walk");
  }
  if (tm) SM_HIP(hipEventRecord(tm->ev[2], s));

  // order by j: LSD passes over (j, i); the last one writes the interleaved output
  uint32_t* jh = hist + 4 * kBins;
  hipLaunchKernelGGL(u32_hist_kernel, dim3(grid_rd), dim3(kBlock), 0, s, mj, &c->nmatch, jpass, jh);
  tmark("j_hist");
  hipLaunchKernelGGL(hist_scan_kernel, dim3(jpass), dim3(kBlock), 0, s, jh);
  tmark("hist_scan");
  uint32_t *cj = mj, *ci = mi, *nj = pj, *ni = pi;
  for (int p = 0; p < jpass; ++p) {
    PairSrc ps{cj, ci};
    if (p == jpass - 1) {
      hipLaunchKernelGGL((onesweep_kernel<3, PairSrc>), dim3(sort_grid), dim3(kBlock), 0, s, ps, RecSoA{}, nullptr,
                         nullptr, (uint64_t*)pairs_out, n, &c->nmatch, p * kRB, jh + p * kBins, status, ++fs.epoch,
                         ctr + ctr_used++, &c->err);
      tmark("j_pass_last");
    } else {
      hipLaunchKernelGGL((onesweep_kernel<2, PairSrc>), dim3(sort_grid), dim3(kBlock), 0, s, ps, RecSoA{}, nj, ni,
                         nullptr, n, &c->nmatch, p * kRB, jh + p * kBins, status, ++fs.epoch, ctr + ctr_used++,
                         &c->err);
      tmark("j_pass");
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
