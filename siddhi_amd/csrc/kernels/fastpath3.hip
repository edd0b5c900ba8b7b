// Bandwidth-shaped closed form for `[partition with (k of S)] from every e1=S[c1] -> e2=S[c2] within T`
// (derivation and citations in fastpath.hip). For each event i with c1(i):
//     j*(i) = min { j > i : key_j = key_i, c2(i, j), ts_j - ts_i <= T },   output (i, j*) ordered by (j*, i).
//
// Every pass is a reduce-then-scan pass over G persistent workgroups, each owning one contiguous chunk of the
// input (no inter-workgroup waiting inside a launch: a decoupled look-back walks the status words of the
// tiles still in flight one cross-XCD load at a time, which on MI355X cost more than the data movement):
//   prep      key min/max, ts monotonicity + span, max relative ordinal               (reads key + ts)
//   up_key    per-chunk digit counts of the rebased key (pass 0 from the key column, later passes from the
//             record keys)                                                              (reads 4 B/event)
//   scan      per digit, exclusive over chunks; digit bases                             (G x 1024 counts)
//   down_*    per chunk, tile by tile: stable in-tile ranking by wave64 ballot peer masks, LDS exchange so
//             that each digit run leaves the tile as contiguous stores, running per-digit chunk offsets in LDS.
//             Key pass 0 builds the 20-byte record {key|c1<<31 : u32, ordinal : u32, c2 attribute : u64,
//             ts - ts0 : u32} from the original columns (c1 evaluated here, once per event).
//   walk      per chunk, tile by tile: records + halo staged in LDS, one lane per record with a lane-private
//             queue of its records; forward scan inside the key run until c2 holds or the window closes;
//             matches compacted chunk-locally (staging) with the digit-0 counts of j as a side product
//   down_j    LSD passes over the (j, i) pairs by j; the first reads the chunk-local staging, the last writes
//             the interleaved (i, j) output
#include <type_traits>
#include <vector>

#include "expr.h"
#include "fastpath.h"

namespace sm {

namespace {

constexpr int kBlock = 512;
constexpr int kWaves = kBlock / 64;
constexpr int kItems = 8;
constexpr int kTile = kBlock * kItems;  // 4096 elements per down-sweep tile
constexpr int kRB = 10;                 // radix bits per pass
constexpr int kBins = 1 << kRB;
constexpr int kBinsPerThread = kBins / kBlock;
constexpr uint32_t kKeyMask = 0x7fffffffu;
constexpr int kUpUnroll = 8;            // independent loads in flight per thread in the up-sweeps
constexpr int kWalkBlock = 256;
constexpr int kWalkItems = 4;
constexpr int kWalkTile = kWalkBlock * kWalkItems;  // 1024 records per walk tile
constexpr int kWalkHalo = 256;                      // records staged past the tile for scans that leave it
constexpr int kWalkLds = kWalkTile + kWalkHalo;
constexpr int kWalkWaves = kWalkBlock / 64;

static_assert(kBins % kBlock == 0, "bins per thread");
static_assert(kTile % kWalkTile == 0, "walk tiles nest in sort tiles");

struct Ctrl {
  unsigned long long kmin, kmax;  // sign-biased key range
  unsigned long long omax;        // max relative ordinal
  unsigned int bad_ts, pad;
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
template <typename VT>
__device__ __forceinline__ uint64_t canon_t(VT v) {
  if constexpr (std::is_floating_point<VT>::value) return (uint64_t)__double_as_longlong((double)v);
  else return (uint64_t)(int64_t)v;
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

// ---------------------------------------------------------------- prep

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

// ---------------------------------------------------------------- up-sweeps and scans

template <typename KT>
struct KeyColDigits {  // rebased key from the original key column
  const KT* kcol;
  int64_t kmin;
  __device__ uint32_t key(int64_t p) const { return (uint32_t)((int64_t)kcol[p] - kmin); }
};
struct U32Digits {  // record keys / j values
  const uint32_t* v;
  __device__ uint32_t key(int64_t p) const { return v[p]; }
};

// per-chunk digit counts → cnt[d * G + g]
template <typename DS>
__global__ void __launch_bounds__(kBlock) upsweep_kernel(DS src, int64_t n, int64_t per, int G, int shift,
                                                         uint32_t* __restrict__ cnt) {
  __shared__ uint32_t h[kBins];
  for (int d = threadIdx.x; d < kBins; d += kBlock) h[d] = 0;
  __syncthreads();
  int64_t lo, len;
  chunk_range(blockIdx.x, n, per, nullptr, lo, len);
  const int64_t hi = lo + len;
  for (int64_t b = lo; b < hi; b += (int64_t)kBlock * kUpUnroll) {
    uint32_t k[kUpUnroll];
#pragma unroll
    for (int u = 0; u < kUpUnroll; ++u) {
      const int64_t p = b + u * kBlock + threadIdx.x;
      k[u] = p < hi ? src.key(p) : 0xffffffffu;
    }
#pragma unroll
    for (int u = 0; u < kUpUnroll; ++u)
      if (b + u * kBlock + threadIdx.x < hi) atomicAdd(&h[((k[u] & kKeyMask) >> shift) & (kBins - 1)], 1u);
  }
  __syncthreads();
  for (int d = threadIdx.x; d < kBins; d += kBlock) cnt[(int64_t)d * G + blockIdx.x] = h[d];
}

// one block per digit: exclusive scan over the G chunk counts in place, digit total → tot[d]
__global__ void __launch_bounds__(256) scan_chunks_kernel(uint32_t* __restrict__ cnt, int G,
                                                          uint32_t* __restrict__ tot) {
  __shared__ uint32_t lw[4];
  __shared__ uint32_t carry;
  uint32_t* row = cnt + (int64_t)blockIdx.x * G;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int b = 0; b < G; b += 256) {
    const int g = b + threadIdx.x;
    const uint32_t v = g < G ? row[g] : 0u;
    uint32_t inc = v;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(inc, o, 64);
      if (lane >= o) inc += u;
    }
    if (lane == 63) lw[w] = inc;
    __syncthreads();
    uint32_t run = carry + inc - v;
    for (int q = 0; q < w; ++q) run += lw[q];
    if (g < G) row[g] = run;
    __syncthreads();
    if (threadIdx.x == 255) carry = run + v;
    __syncthreads();
  }
  if (threadIdx.x == 0) tot[blockIdx.x] = carry;
}

// exclusive scan of the kBins digit totals in place (one block)
__global__ void __launch_bounds__(kBlock) digit_base_kernel(uint32_t* __restrict__ tot) {
  __shared__ uint32_t lw[kWaves];
  uint32_t v[kBinsPerThread], s = 0;
  for (int k = 0; k < kBinsPerThread; ++k) {
    v[k] = tot[threadIdx.x * kBinsPerThread + k];
    s += v[k];
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t inc = s;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(inc, o, 64);
    if (lane >= o) inc += u;
  }
  if (lane == 63) lw[w] = inc;
  __syncthreads();
  uint32_t run = inc - s;
  for (int k = 0; k < w; ++k) run += lw[k];
  for (int k = 0; k < kBinsPerThread; ++k) {
    tot[threadIdx.x * kBinsPerThread + k] = run;
    run += v[k];
  }
}

// ---------------------------------------------------------------- down-sweep

// Pass 0 of the keyed sort: builds the record from the original columns. Key and compared-attribute column
// types are template parameters; c1 is evaluated by c1(), once per event, outside the unrolled loops.
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

struct PairSrc {
  static constexpr bool kC1 = false;
  const uint32_t* j;
  const uint32_t* i;
  __device__ uint32_t key(int64_t p) const { return j[p]; }
  __device__ uint32_t g0(int64_t p) const { return i[p]; }
};

// Down-sweep of one LSD pass over chunk blockIdx.x (persistent: tile by tile, running per-digit offsets).
//   MODE 0: keyed record from the original columns (OrigSrc) → RecSoA
//   MODE 1: keyed record (RecSrc) → RecSoA
//   MODE 2: (j, i) pairs → two u32 arrays
//   MODE 3: (j, i) pairs → interleaved (i, j) u32 pairs (last pass)
template <int MODE, typename Src>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4))) downsweep_kernel(Src src, RecSoA dst, uint32_t* __restrict__ dj,
                                                           uint32_t* __restrict__ di, uint64_t* __restrict__ dpairs,
                                                           int64_t n, int64_t per, const uint32_t* seg_len, int G,
                                                           int shift, const uint32_t* __restrict__ cnt,
                                                           const uint32_t* __restrict__ dbase) {
  __shared__ uint32_t xb32[kTile];  // exchange buffer, one 32-bit field at a time (u64 fields in two halves)
  __shared__ uint16_t wcnt[kWaves][kBins];
  __shared__ uint32_t tstart[kBins];
  __shared__ uint32_t run[kBins];  // next output position of each digit for this chunk
  __shared__ uint16_t sdig[kTile];  // digit of the element at each sorted slot (destinations are recomputed
                                    // per exchange from LDS instead of living in registers)
  __shared__ uint32_t lw[kWaves];

  int64_t lo, len;
  chunk_range(blockIdx.x, n, per, seg_len, lo, len);
  for (int d = threadIdx.x; d < kBins; d += kBlock) run[d] = dbase[d] + cnt[(int64_t)d * G + blockIdx.x];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = lanemask_lt();
  Cond c1;
  if constexpr (Src::kC1) c1 = make_cond(src.c1p, src.c1_len, src.consts);

  for (int64_t base = lo; base < lo + len; base += kTile) {
    const int tile_n = (int)((lo + len - base) < kTile ? (lo + len - base) : kTile);
    // every load of the tile is issued up front (one exposed memory latency per tile, not one per field)
    uint32_t keys[kItems], p0[kItems], p2[kItems];
    uint64_t p1[kItems];
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const int e = w * 64 * kItems + k * 64 + lane;
      if (e < tile_n) {
        const int64_t p = base + e;
        keys[k] = src.key(p);
        if constexpr (MODE == 0) {
          p0[k] = src.f0(p);
          p1[k] = src.f1(p);
          p2[k] = src.f2(p);
        } else if constexpr (MODE == 1) {
          p0[k] = src.f0[p];
          p1[k] = src.f1[p];
          p2[k] = src.f2[p];
        } else {
          p0[k] = src.g0(p);
        }
      }
    }
    __syncthreads();  // previous tile's readers of wcnt / xb32 / sdig / run are done
    for (int k = threadIdx.x; k < kWaves * kBins; k += kBlock) (&wcnt[0][0])[k] = 0;
    if constexpr (Src::kC1) {  // c1 flag of each item → key bit 31, evaluated in a rolled loop
#pragma unroll 1
      for (int k = 0; k < kItems; ++k) {
        const int e = w * 64 * kItems + k * 64 + lane;
        if (e < tile_n && eval(c1, RowLoader{src.st, base + e})) keys[k] |= 0x80000000u;
      }
    }
    __syncthreads();

    uint32_t lp[kItems];  // rank within (wave, digit), then local sorted position
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const int e = w * 64 * kItems + k * 64 + lane;
      const bool valid = e < tile_n;
      const uint32_t d = valid ? ((keys[k] & kKeyMask) >> shift) & (kBins - 1) : 0u;
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
    uint32_t cnt_t[kBinsPerThread];
    uint32_t csum = 0;
#pragma unroll
    for (int b = 0; b < kBinsPerThread; ++b) {
      const int d = threadIdx.x * kBinsPerThread + b;
      uint32_t r = 0;
      for (int q = 0; q < kWaves; ++q) {
        const uint32_t c = wcnt[q][d];
        wcnt[q][d] = (uint16_t)r;
        r += c;
      }
      cnt_t[b] = r;
      csum += r;
    }
    {  // block exclusive scan of the tile counts over digits → tstart
      uint32_t inc = csum;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(inc, o, 64);
        if (lane >= o) inc += u;
      }
      if (lane == 63) lw[w] = inc;
      __syncthreads();
      uint32_t r = inc - csum;
      for (int q = 0; q < w; ++q) r += lw[q];
#pragma unroll
      for (int b = 0; b < kBinsPerThread; ++b) {
        tstart[threadIdx.x * kBinsPerThread + b] = r;
        r += cnt_t[b];
      }
    }
    __syncthreads();

    // local sorted positions; key exchange; slot digits
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
    auto dest_of = [&](int s) -> uint32_t {
      const uint32_t d = sdig[s];
      return run[d] + (uint32_t)s - tstart[d];
    };
    uint32_t jj[kItems];  // MODE 3: j of the sorted slots
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
      const int s = r * kBlock + threadIdx.x;
      if (s < tile_n) {
        const uint32_t key = xb32[s];
        const uint32_t d = ((key & kKeyMask) >> shift) & (kBins - 1);
        sdig[s] = (uint16_t)d;
        const uint32_t dst_pos = run[d] + (uint32_t)s - tstart[d];
        if constexpr (MODE == 0 || MODE == 1) dst.k[dst_pos] = key;
        if constexpr (MODE == 2) dj[dst_pos] = key;
        if constexpr (MODE == 3) jj[r] = key;
      }
    }
    // payload exchanges: scatter the field into sorted slots, then coalesced stores by slot
    auto exchange = [&](const uint32_t (&v)[kItems], auto&& store) {
      __syncthreads();
#pragma unroll
      for (int k = 0; k < kItems; ++k) {
        const int e = w * 64 * kItems + k * 64 + lane;
        if (e < tile_n) xb32[lp[k]] = v[k];
      }
      __syncthreads();
#pragma unroll
      for (int r = 0; r < kItems; ++r) {
        const int s = r * kBlock + threadIdx.x;
        if (s < tile_n) store(r, s, xb32[s]);
      }
    };
    if constexpr (MODE == 3) {  // (j, i) → interleaved (i, j)
      exchange(p0, [&](int r, int s, uint32_t x) { dpairs[dest_of(s)] = ((uint64_t)jj[r] << 32) | x; });
    } else if constexpr (MODE == 2) {
      exchange(p0, [&](int, int s, uint32_t x) { di[dest_of(s)] = x; });
    } else {
      exchange(p0, [&](int, int s, uint32_t x) { dst.f0[dest_of(s)] = x; });
      uint32_t* f1w = (uint32_t*)dst.f1;  // u64 field as two 32-bit halves
      uint32_t half[kItems];
#pragma unroll
      for (int k = 0; k < kItems; ++k) half[k] = (uint32_t)p1[k];
      exchange(half, [&](int, int s, uint32_t x) { f1w[2 * (size_t)dest_of(s)] = x; });
#pragma unroll
      for (int k = 0; k < kItems; ++k) half[k] = (uint32_t)(p1[k] >> 32);
      exchange(half, [&](int, int s, uint32_t x) { f1w[2 * (size_t)dest_of(s) + 1] = x; });
      exchange(p2, [&](int, int s, uint32_t x) { dst.f2[dest_of(s)] = x; });
    }
    __syncthreads();  // every destination computed from run[] before it advances
#pragma unroll
    for (int b = 0; b < kBinsPerThread; ++b) run[threadIdx.x * kBinsPerThread + b] += cnt_t[b];
  }
}

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
struct WalkLds;
template <>
struct WalkLds<true> {
  uint64_t v[kWalkLds];
  uint32_t k[kWalkLds];
  uint32_t t[kWalkLds];
  uint32_t o[kWalkLds];
};
template <>
struct WalkLds<false> {
  uint64_t v[kWalkLds];
  int64_t t[kWalkLds];
};

// Chunk blockIdx.x, tile by tile. One lane per record of the tile; each lane works through its kWalkItems
// records as a private queue (a lane whose scan ends takes its next record at once, so a wave runs for the
// longest per-lane total instead of kWalkItems x the longest single scan). Scans read the staged records; one
// that runs past them is finished from global memory (rare: key runs / windows longer than the halo).
// Matches are compacted in record order into the chunk's staging region [lo, lo + count); the chunk's match
// count goes to mcount[g] and the digit-0 counts of j to jcnt[d * G + g] (the first j pass needs no up-sweep).
template <bool KEYED, int OP, bool FP>
__global__ void __launch_bounds__(kWalkBlock) walk_kernel(WalkArgs a, int64_t per, int G,
                                                          uint32_t* __restrict__ stj, uint32_t* __restrict__ sti,
                                                          uint32_t* __restrict__ mcount,
                                                          uint32_t* __restrict__ jcnt) {
  __shared__ WalkLds<KEYED> L;
  __shared__ uint32_t sj[kWalkItems][kWalkBlock];  // per item: matched position - tile base (or resume point)
  __shared__ uint64_t sbal[kWalkWaves][kWalkItems];
  __shared__ uint32_t wtot[kWalkWaves];
  __shared__ uint32_t jh[kBins];
  __shared__ uint32_t sh_run;

  const int64_t n = a.n;
  int64_t lo, len;
  chunk_range(blockIdx.x, n, per, nullptr, lo, len);
  const int64_t hi = lo + len;
  for (int d = threadIdx.x; d < kBins; d += kWalkBlock) jh[d] = 0;
  if (threadIdx.x == 0) sh_run = 0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = lanemask_lt();
  C2<OP, FP> c2;
  if constexpr (OP < 0) c2.c = make_cond(a.c2, a.c2_len, a.consts);
  c2.vtype = a.vtype;
  Cond c1;
  if constexpr (!KEYED) c1 = make_cond(a.c1, a.c1_len, a.consts);

  for (int64_t base = lo; base < hi; base += kWalkTile) {
    __syncthreads();  // previous tile's LDS readers are done
    const int nload = (int)((n - base) < kWalkLds ? (n - base) : kWalkLds);
    for (int e = threadIdx.x; e < nload; e += kWalkBlock) {
      const int64_t p = base + e;
      if constexpr (KEYED) {
        L.k[e] = a.k[p];
        L.t[e] = a.f2[p];
        L.v[e] = a.f1[p];
        L.o[e] = a.f0[p];
      } else {
        L.t[e] = a.ts[p];
        L.v[e] = canon(col_value(a.st, a.vattr, p), a.vtype);
      }
    }
    __syncthreads();
    const int lend = nload;  // staged positions are [0, lend) relative to base
    uint32_t c1m = 0;        // c1 of each item (bit k)
#pragma unroll 1
    for (int k = 0; k < kWalkItems; ++k) {
      const int lu = w * 64 * kWalkItems + k * 64 + lane;
      if (base + lu < hi) {
        bool c;
        if constexpr (KEYED) c = (L.k[lu] >> 31) != 0;
        else c = eval(c1, RowLoader{a.st, base + lu});
        if (c) c1m |= 1u << k;
      }
    }
    // lane-private queue over the items with c1
    uint32_t hasm = 0, openm = 0;
    uint32_t todo = c1m;
    int k = -1, v = 0;
    uint64_t vu = 0;
    int64_t tu = 0;
    uint32_t key = 0;
    auto take = [&]() -> bool {
      if (!todo) return false;
      k = __ffs(todo) - 1;
      todo &= todo - 1;
      const int lu = w * 64 * kWalkItems + k * 64 + lane;
      vu = L.v[lu];
      tu = L.t[lu];
      if constexpr (KEYED) key = L.k[lu] & kKeyMask;
      v = lu + 1;
      return true;
    };
    bool live = take();
    while (__any(live)) {
      if (live) {
        if (v >= lend) {  // leaves the staged records: finish from global memory below
          if (base + v < n) {
            openm |= 1u << k;
            sj[k][threadIdx.x] = (uint32_t)v;
          }
          live = take();
        } else {
          bool stop;
          if constexpr (KEYED) {
            stop = (L.k[v] & kKeyMask) != key || (a.within >= 0 && (int64_t)(L.t[v] - (uint32_t)tu) > a.within);
          } else {
            const int64_t d = L.t[v] - tu;
            stop = a.within >= 0 && (d < 0 ? -d : d) > a.within;
          }
          if (stop) {
            live = take();
          } else if (c2(vu, L.v[v])) {
            hasm |= 1u << k;
            sj[k][threadIdx.x] = (uint32_t)v;
            live = take();
          } else {
            ++v;
          }
        }
      }
    }
    // scans that ran past the staged records
#pragma unroll 1
    while (openm) {
      const int kk = __ffs(openm) - 1;
      openm &= openm - 1;
      const int luu = w * 64 * kWalkItems + kk * 64 + lane;
      const uint64_t vuu = L.v[luu];
      for (int64_t p = base + sj[kk][threadIdx.x]; p < n; ++p) {
        if constexpr (KEYED) {
          if ((a.k[p] & kKeyMask) != (L.k[luu] & kKeyMask) ||
              (a.within >= 0 && (int64_t)(a.f2[p] - L.t[luu]) > a.within))
            break;
          if (c2(vuu, a.f1[p])) {
            hasm |= 1u << kk;
            sj[kk][threadIdx.x] = (uint32_t)(p - base);
            break;
          }
        } else {
          const int64_t d = a.ts[p] - L.t[luu];
          if (a.within >= 0 && (d < 0 ? -d : d) > a.within) break;
          if (c2(vuu, canon(col_value(a.st, a.vattr, p), a.vtype))) {
            hasm |= 1u << kk;
            sj[kk][threadIdx.x] = (uint32_t)(p - base);
            break;
          }
        }
      }
    }
    uint32_t mine = 0;
#pragma unroll 1
    for (int q = 0; q < kWalkItems; ++q) {
      const uint64_t bal = __ballot((hasm >> q) & 1u);
      if (lane == 0) sbal[w][q] = bal;
      mine += (uint32_t)__popcll(bal);
    }
    if (lane == 0) wtot[w] = mine;
    __syncthreads();
    uint32_t ob = sh_run, tot = 0;
    for (int q = 0; q < kWalkWaves; ++q) {
      if (q < w) ob += wtot[q];
      tot += wtot[q];
    }
#pragma unroll 1
    for (int q = 0; q < kWalkItems; ++q) {
      const uint64_t bal = sbal[w][q];
      if ((bal >> lane) & 1ull) {
        const int64_t pos = lo + ob + (uint32_t)__popcll(bal & lt);
        const int luq = w * 64 * kWalkItems + q * 64 + lane;
        const uint32_t jv = sj[q][threadIdx.x];
        uint32_t jo, io;
        if constexpr (KEYED) {
          jo = jv < (uint32_t)lend ? L.o[jv] : a.f0[base + jv];
          io = L.o[luq];
        } else {
          const int64_t vj = base + jv, ui = base + luq;
          jo = a.ord ? (uint32_t)(a.ord[vj] - a.obase) : (uint32_t)vj;
          io = a.ord ? (uint32_t)(a.ord[ui] - a.obase) : (uint32_t)ui;
        }
        stj[pos] = jo;
        sti[pos] = io;
        atomicAdd(&jh[jo & (kBins - 1)], 1u);
      }
      ob += (uint32_t)__popcll(bal);
    }
    __syncthreads();  // every wave read sh_run / wtot
    if (threadIdx.x == 0) sh_run += tot;
  }
  __syncthreads();
  if (threadIdx.x == 0) mcount[blockIdx.x] = sh_run;
  for (int d = threadIdx.x; d < kBins; d += kWalkBlock) jcnt[(int64_t)d * G + blockIdx.x] = jh[d];
}

inline int bits_for(uint64_t v) {
  int b = 0;
  while (b < 64 && (v >> b) != 0) ++b;
  return b;
}

// Compare spec of c2 for the walk: op * 2 + fp, normalised to `e2.x OP e1.x`, or -1 (generic program).
// Admitted: `eK.x CMP eL.x` over the carried attribute, one operand per slot, compared in its own type.
int c2_spec(const FastHostInfo& hi) {
  if (!hi.c2_host || hi.c2_len != 3) return -1;
  const Instr* c = hi.c2_host;
  if (c[0].op != OP_VAR || c[1].op != OP_VAR || c[2].op != OP_CMP) return -1;
  if (c[0].c != hi.vattr || c[1].c != hi.vattr || c[0].a == c[1].a) return -1;
  if (!(c[0].b == 0 || c[0].b == -1) || !(c[1].b == 0 || c[1].b == -1)) return -1;
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
void launch_walk_t(int G, hipStream_t s, const WalkArgs& wa, int64_t per, uint32_t* stj, uint32_t* sti,
                   uint32_t* mcount, uint32_t* jcnt) {
  hipLaunchKernelGGL((walk_kernel<KEYED, OP, FP>), dim3(G), dim3(kWalkBlock), 0, s, wa, per, G, stj, sti, mcount,
                     jcnt);
}

template <bool KEYED>
void launch_walk(int spec, int G, hipStream_t s, const WalkArgs& wa, int64_t per, uint32_t* stj, uint32_t* sti,
                 uint32_t* mcount, uint32_t* jcnt) {
#define SM_WALK(OP, FP) launch_walk_t<KEYED, OP, FP>(G, s, wa, per, stj, sti, mcount, jcnt)
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

template <typename KT, typename VT>
void launch_down0_t(const FastHostInfo& hi, const FastArgs& a, const void* kcol, int64_t kmin, int64_t ts0, int G,
                    int64_t per, hipStream_t s, RecSoA dst, const uint32_t* cnt, const uint32_t* dbase) {
  OrigSrc<KT, VT> os{a.st, (const KT*)kcol, (const VT*)hi.cols[hi.vattr], kmin, a.code + a.c1_off, a.c1_len,
                     a.consts, a.ts, ts0, a.ordinals, a.ordinal_base};
  hipLaunchKernelGGL((downsweep_kernel<0, OrigSrc<KT, VT>>), dim3(G), dim3(kBlock), 0, s, os, dst, nullptr, nullptr,
                     nullptr, a.n, per, nullptr, G, 0, cnt, dbase);
}

template <typename KT>
void launch_down0_k(const FastHostInfo& hi, const FastArgs& a, const void* kcol, int64_t kmin, int64_t ts0, int G,
                    int64_t per, hipStream_t s, RecSoA dst, const uint32_t* cnt, const uint32_t* dbase) {
  switch (hi.vtype) {
    case T_INT: launch_down0_t<KT, int32_t>(hi, a, kcol, kmin, ts0, G, per, s, dst, cnt, dbase); break;
    case T_LONG: launch_down0_t<KT, int64_t>(hi, a, kcol, kmin, ts0, G, per, s, dst, cnt, dbase); break;
    case T_FLOAT: launch_down0_t<KT, float>(hi, a, kcol, kmin, ts0, G, per, s, dst, cnt, dbase); break;
    case T_DOUBLE: launch_down0_t<KT, double>(hi, a, kcol, kmin, ts0, G, per, s, dst, cnt, dbase); break;
    default: throw std::runtime_error("fast path: unsupported compared-attribute type");
  }
}

int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

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
  auto bail = [&]() -> int64_t {
    sc.used = mark;
    return -1;
  };
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

  // persistent chunking: G workgroups (as many as the down-sweep keeps resident), chunks of whole sort tiles
  if (fs.cus == 0) {
    int dev = 0;
    SM_HIP(hipGetDevice(&dev));
    SM_HIP(hipDeviceGetAttribute(&fs.cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  if (fs.sort_wgs_per_cu == 0) {
    int b = 0;
    SM_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, downsweep_kernel<1, RecSrc>, kBlock, 0));
    fs.sort_wgs_per_cu = std::max(1, b);
    b = 0;
    SM_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, walk_kernel<true, CMP_GT, true>, kWalkBlock, 0));
    fs.walk_wgs_per_cu = std::max(1, b);
  }
  // sort passes: kOversub chunks per resident workgroup (balances the tail); walk: one chunk per resident
  // workgroup, whole walk tiles (the first j pass runs over the walk's chunks)
  constexpr int kOversub = 2;
  const int64_t tiles = (n + kTile - 1) / kTile;
  const int G = (int)std::max<int64_t>(1, std::min<int64_t>(tiles, (int64_t)kOversub * fs.sort_wgs_per_cu * fs.cus));
  const int64_t per = round_up((n + G - 1) / G, kTile);
  const int64_t wtiles = (n + kWalkTile - 1) / kWalkTile;
  const int Gw = (int)std::max<int64_t>(1, std::min<int64_t>(wtiles, (int64_t)fs.walk_wgs_per_cu * fs.cus));
  const int64_t perw = round_up((n + Gw - 1) / Gw, kWalkTile);
  uint32_t* cnt = (uint32_t*)sc.take(sizeof(uint32_t) * kBins * std::max(G, Gw));
  uint32_t* dbase = (uint32_t*)sc.take(sizeof(uint32_t) * kBins);
  uint32_t* mcount = (uint32_t*)sc.take(sizeof(uint32_t) * Gw);
  auto scan_counts = [&](int g) {
    hipLaunchKernelGGL(scan_chunks_kernel, dim3(kBins), dim3(256), 0, s, cnt, g, dbase);
    hipLaunchKernelGGL(digit_base_kernel, dim3(1), dim3(kBlock), 0, s, dbase);
    tmark("scan");
  };

  RecSoA A{}, B{};
  uint32_t *stj = nullptr, *sti = nullptr;  // walk staging (chunk-local compaction)
  uint32_t *pj = nullptr, *pi = nullptr, *qj = nullptr, *qi = nullptr;  // j-sort ping-pong
  WalkArgs wa{};
  wa.st = a.st;
  wa.ts = a.ts;
  wa.ord = a.ordinals;
  wa.obase = a.ordinal_base;
  wa.c1 = a.code + a.c1_off;
  wa.c1_len = a.c1_len;
  wa.c2 = a.code + a.c2_off;
  wa.c2_len = a.c2_len;
  wa.consts = a.consts;
  wa.vattr = hi.vattr;
  wa.vtype = hi.vtype;
  wa.within = a.within;
  wa.n = n;
  const int spec = c2_spec(hi);
  if (keyed) {
    A.k = (uint32_t*)sc.take(n * 4);
    A.f0 = (uint32_t*)sc.take(n * 4);
    A.f1 = (uint64_t*)sc.take(n * 8);
    A.f2 = (uint32_t*)sc.take(n * 4);
    B.k = (uint32_t*)sc.take(n * 4);
    B.f0 = (uint32_t*)sc.take(n * 4);
    B.f1 = (uint64_t*)sc.take(n * 8);
    B.f2 = (uint32_t*)sc.take(n * 4);
    // key pass 0 from the original columns
    if (hi.key_type == T_INT)
      hipLaunchKernelGGL((upsweep_kernel<KeyColDigits<int32_t>>), dim3(G), dim3(kBlock), 0, s,
                         KeyColDigits<int32_t>{(const int32_t*)kcol, kmin}, n, per, G, 0, cnt);
    else
      hipLaunchKernelGGL((upsweep_kernel<KeyColDigits<int64_t>>), dim3(G), dim3(kBlock), 0, s,
                         KeyColDigits<int64_t>{(const int64_t*)kcol, kmin}, n, per, G, 0, cnt);
    tmark("key_up");
    scan_counts(G);
    if (hi.key_type == T_INT) launch_down0_k<int32_t>(hi, a, kcol, kmin, hc.ts0, G, per, s, A, cnt, dbase);
    else launch_down0_k<int64_t>(hi, a, kcol, kmin, hc.ts0, G, per, s, A, cnt, dbase);
    tmark("key_pass0");
    RecSoA* cur = &A;
    RecSoA* nxt = &B;
    for (int p = 1; p < fpass; ++p) {
      hipLaunchKernelGGL((upsweep_kernel<U32Digits>), dim3(G), dim3(kBlock), 0, s, U32Digits{cur->k}, n, per, G,
                         p * kRB, cnt);
      tmark("key_up");
      scan_counts(G);
      RecSrc rs{cur->k, cur->f0, cur->f1, cur->f2};
      hipLaunchKernelGGL((downsweep_kernel<1, RecSrc>), dim3(G), dim3(kBlock), 0, s, rs, *nxt, nullptr, nullptr,
                         nullptr, n, per, nullptr, G, p * kRB, cnt, dbase);
      tmark("key_pass");
      std::swap(cur, nxt);
    }
    if (tm) SM_HIP(hipEventRecord(tm->ev[1], s));
    wa.k = cur->k;
    wa.f0 = cur->f0;
    wa.f1 = cur->f1;
    wa.f2 = cur->f2;
    // staging in the dead record buffer; j ping-pong: nxt->f1 (2n u32) and, after the walk, cur->k / cur->f0
    stj = nxt->k;
    sti = nxt->f0;
    pj = (uint32_t*)nxt->f1;
    pi = (uint32_t*)nxt->f1 + n;
    qj = cur->k;
    qi = cur->f0;
    launch_walk<true>(spec, Gw, s, wa, perw, stj, sti, mcount, cnt);
  } else {
    if (tm) SM_HIP(hipEventRecord(tm->ev[1], s));
    stj = (uint32_t*)sc.take(n * 4);
    sti = (uint32_t*)sc.take(n * 4);
    pj = (uint32_t*)sc.take(n * 4);
    pi = (uint32_t*)sc.take(n * 4);
    qj = (uint32_t*)sc.take(n * 4);
    qi = (uint32_t*)sc.take(n * 4);
    launch_walk<false>(spec, Gw, s, wa, perw, stj, sti, mcount, cnt);
  }
  tmark("walk");
  if (tm) SM_HIP(hipEventRecord(tm->ev[2], s));

  // order by j: LSD passes over (j, i); the first reads the walk's chunk-local staging (its digit-0 counts
  // came from the walk), the last writes the interleaved output
  std::vector<uint32_t> hm(Gw);
  SM_HIP(hipMemcpyAsync(hm.data(), mcount, sizeof(uint32_t) * Gw, hipMemcpyDeviceToHost, s));
  scan_counts(Gw);
  SM_HIP(hipStreamSynchronize(s));
  int64_t M = 0;
  for (int g = 0; g < Gw; ++g) M += hm[g];
  if (M > pairs_cap) {
    sc.used = mark;
    throw std::runtime_error("match buffer too small");
  }
  if (M > 0) {
    const int64_t perM = round_up((M + G - 1) / G, kTile);
    uint32_t *cj = stj, *ci = sti;
    uint32_t* outs[2][2] = {{pj, pi}, {qj, qi}};
    for (int p = 0; p < jpass; ++p) {
      const bool last = p == jpass - 1;
      if (p > 0) {
        hipLaunchKernelGGL((upsweep_kernel<U32Digits>), dim3(G), dim3(kBlock), 0, s, U32Digits{cj}, M, perM, G,
                           p * kRB, cnt);
        tmark("j_up");
        scan_counts(G);
      }
      const int64_t nn = p == 0 ? n : M;
      const int64_t pp = p == 0 ? perw : perM;
      const uint32_t* seg = p == 0 ? mcount : nullptr;
      const int gg = p == 0 ? Gw : G;
      PairSrc ps{cj, ci};
      if (last) {
        hipLaunchKernelGGL((downsweep_kernel<3, PairSrc>), dim3(gg), dim3(kBlock), 0, s, ps, RecSoA{}, nullptr, nullptr,
                           (uint64_t*)pairs_out, nn, pp, seg, gg, p * kRB, cnt, dbase);
        tmark("j_pass_last");
      } else {
        uint32_t* nj = outs[p & 1][0];
        uint32_t* ni = outs[p & 1][1];
        hipLaunchKernelGGL((downsweep_kernel<2, PairSrc>), dim3(gg), dim3(kBlock), 0, s, ps, RecSoA{}, nj, ni, nullptr,
                           nn, pp, seg, gg, p * kRB, cnt, dbase);
        tmark("j_pass");
        cj = nj;
        ci = ni;
      }
    }
  }
  if (tm) SM_HIP(hipEventRecord(tm->ev[3], s));
  SM_HIP(hipStreamSynchronize(s));
  sc.used = mark;
  return M;
}

}  // namespace sm
