// Bandwidth-shaped closed form for `[partition with (k of S)] from every e1=S[c1] -> e2=S[c2] within T`
// (derivation and citations in fastpath.hip). For each event i with c1(i):
//     j*(i) = min { j > i : key_j = key_i, c2(i, j), ts_j - ts_i <= T },   output (i, j*) ordered by (j*, i).
//
// Every pass is a reduce-then-scan pass over G persistent workgroups, each owning one contiguous chunk of the
// input (no inter-workgroup waiting inside a launch: a decoupled look-back walks the status words of the
// tiles still in flight one cross-XCD load at a time, which on MI355X cost more than the data movement):
//   prep      key min/max, ts monotonicity + span, max relative ordinal, compared-attribute range
//   up_key    per-chunk digit counts of the rebased key (pass 0 from the key column, later passes from the
//             records)
//   scan      per digit, exclusive over chunks; digit bases                             (G x kBins counts)
//   down_*    per chunk, tile by tile: stable in-tile ranking by wave64 ballot peer masks, LDS exchange so
//             that each digit run leaves the tile as contiguous stores, running per-digit chunk offsets in LDS.
//             Key pass 0 builds the 16-byte keyed record (below) from the original columns (c1 evaluated
//             there, once per event).
//   walk      keyed: per chunk, tile by tile: records + halo staged in LDS, one lane per record with a
//             lane-private queue of its records; forward scan inside the key run until c2 holds or the window
//             closes; matches compacted chunk-locally (staging) with the digit-0 counts of j as a side product.
//             Unkeyed (no partition): the same over the original columns.
//   down_j    LSD passes over the (j, i) pairs by j; the first reads the chunk-local staging, the last writes
//             the output.
//
// Keyed record: ONE 16-byte element {key | c1 << 31, ordinal, value code, ts - ts0}. The scatter of every pass
// is the cost that matters (each tile sends its elements to kBins digit runs); one aligned 16-byte stream per
// element writes runs 4x longer than four 32-bit field arrays would. The value code is a monotone 32-bit image
// of the compared attribute: exact for INT, FLOAT and for LONG batches whose range spans < 2^32; for DOUBLE
// (and wide LONG) it is the high half of the order-preserving 64-bit image, so `code2 != code1` decides any
// comparison and equal codes (or NaN) fall back to the exact column values (rare; the record's ordinal gives
// the row).
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "expr.h"
#include "fastpath.h"
#include "fastpath_dev.h"
#include "pass0_dev.h"

#ifndef SM_ORIG_NT_LOAD
#define SM_ORIG_NT_LOAD 1  // A/B build flag: nontemporal column loads in key pass 0 (OrigSrc; 13.56 -> 13.32 ms)
#endif

namespace sm {

namespace {

#ifndef SM_SB
#define SM_SB 512
#endif
#ifndef SM_SI
#define SM_SI 8
#endif
constexpr int kBlock = SM_SB;
constexpr int kWaves = kBlock / 64;
constexpr int kItems = SM_SI;
constexpr int kTile = kBlock * kItems;  // 4096 elements per down-sweep tile
constexpr int kBinsPerThread = kBins >= kBlock ? kBins / kBlock : 1;  // digits owned per thread
constexpr int kUpUnroll = 8;  // independent loads in flight per thread in the up-sweeps
#ifndef SM_WB
#define SM_WB 512
#endif
#ifndef SM_WI
#define SM_WI 4
#endif
constexpr int kWalkBlock = SM_WB;
constexpr int kWalkItems = SM_WI;
constexpr int kWalkTile = kWalkBlock * kWalkItems;  // 1024 records per walk tile
constexpr int kWalkHalo = 256;                      // records staged past the tile for scans that leave it
constexpr int kWalkLds = kWalkTile + kWalkHalo;
constexpr int kWalkWaves = kWalkBlock / 64;
constexpr int kUnkeyedBudget = 32;  // private (per-lane) scan steps of an unkeyed record before the wave helps

static_assert(kBins % kBlock == 0 || kBlock % kBins == 0, "bins per thread");
static_assert(kTile % kWalkTile == 0, "walk tiles nest in sort tiles");

// Diagnostic build only (tests/native/micro_sort.hip defines SM_STAMPS): per-wave s_memtime stamps at phase
// boundaries of the down-sweep tile loop, summed into sm_stamps[] (shares, not absolute times).
#ifdef SM_STAMPS
__device__ unsigned long long sm_stamps[16];
#define SM_STAMP(i)                                                            \
  do {                                                                         \
    __builtin_amdgcn_sched_barrier(0);                                         \
    unsigned long long t_;                                                     \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
    __builtin_amdgcn_sched_barrier(0);                                         \
    if ((i) > 0) st_acc[(i) - 1] += t_ - st_last;                              \
    st_last = t_;                                                              \
  } while (0)
#define SM_STAMP_DECL                \
  unsigned long long st_acc[8] = {}; \
  unsigned long long st_last = 0
#define SM_STAMP_FLUSH                                                    \
  do {                                                                    \
    if ((threadIdx.x & 63) == 0)                                          \
      for (int q_ = 0; q_ < 8; ++q_) atomicAdd(&sm_stamps[q_], st_acc[q_]); \
  } while (0)
#else
#define SM_STAMP(i) \
  do {              \
  } while (0)
#define SM_STAMP_DECL
#define SM_STAMP_FLUSH \
  do {                 \
  } while (0)
#endif


// ---------------------------------------------------------------- prep

// One read of the key, ts (and ordinal / LONG attribute) columns per event, per chunk of the sort grid:
//   * key min/max, ts monotonicity, max relative ordinal, ordinals increasing, LONG attribute range → Ctrl
//   * MASK: c1 of every event as a bit mask (bit p & 63 of word p >> 6; ballot per wave). Keyed batches whose
//     c1 reads only the compared attribute skip it: the pass-0 down-sweep evaluates c1 on the value it loads.
//   * per-chunk counts of the pass-0 digit. Keys are rebased by kmin rounded down to a multiple of kBins, so
//     the low digit of the rebased key is the low digit of the key itself and needs no kmin yet.
// Tiles of kTile events (kItems per thread, every load of the tile issued before any is used).
// EXTRA: an ordinal column or a LONG compared attribute is read too (without them, their registers are not held:
// 134 -> fewer VGPRs, two workgroups per CU instead of one)
template <typename KT, bool MASK, bool EXTRA>
__global__ void __launch_bounds__(kBlock) prep_kernel(const KT* __restrict__ kcol, const int64_t* __restrict__ vlong,
                                                      const int64_t* __restrict__ ts, const int64_t* __restrict__ ord,
                                                      int64_t obase, int64_t n, int64_t per, int G,
                                                      const NfaStream* __restrict__ st, const Instr* __restrict__ c1code,
                                                      int c1len, const DVal* __restrict__ consts,
                                                      uint64_t* __restrict__ c1mask, uint32_t* __restrict__ cnt,
                                                      Ctrl* __restrict__ c) {
  __shared__ uint32_t h[kBins];
  for (int d = threadIdx.x; d < kBins; d += kBlock) h[d] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t lo0, len;
  chunk_range(blockIdx.x, n, per, nullptr, lo0, len);
  const int64_t hi0 = lo0 + len;
  unsigned long long lo = ~0ull, hi = 0, om = 0, vlo = ~0ull, vhi = 0;
  unsigned int bad = 0, bado = 0;
  for (int64_t base = lo0; base < hi0; base += kTile) {
    KT kk[kItems];
    int64_t tt[kItems], oo[kItems], vv[kItems], tp[kItems], op[kItems];
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const int64_t p = base + w * 64 * kItems + k * 64 + lane;
      if (p < hi0) {
        if (kcol) kk[k] = __builtin_nontemporal_load(kcol + p);
        tt[k] = __builtin_nontemporal_load(ts + p);
        if (EXTRA && ord) oo[k] = ord[p];
        if (EXTRA && vlong) vv[k] = vlong[p];
        if (lane == 0 && p > 0) {  // the element before each wave-item (other lanes take it from lane - 1)
          tp[k] = ts[p - 1];
          if (EXTRA && ord) op[k] = ord[p - 1];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const int64_t p = base + w * 64 * kItems + k * 64 + lane;
      const bool in = p < hi0;
      int64_t pt = __shfl_up(tt[k], 1, 64);
      if (lane == 0) pt = p > 0 ? tp[k] : tt[k];
      if (in && tt[k] < pt) bad = 1;
      if (EXTRA && ord) {
        int64_t po = __shfl_up(oo[k], 1, 64);
        if (lane == 0) po = p > 0 ? op[k] : oo[k] - 1;
        if (in) {
          const unsigned long long o = (unsigned long long)(oo[k] - obase);
          om = o > om ? o : om;
          if (oo[k] <= po) bado = 1;
        }
      }
      if (in && kcol) {
        const unsigned long long u = (unsigned long long)(int64_t)kk[k] ^ 0x8000000000000000ull;
        lo = u < lo ? u : lo;
        hi = u > hi ? u : hi;
        atomicAdd(&h[(uint32_t)kk[k] & (kBins - 1)], 1u);
      }
      if (EXTRA && in && vlong) {
        const unsigned long long u = (unsigned long long)vv[k] ^ 0x8000000000000000ull;
        vlo = u < vlo ? u : vlo;
        vhi = u > vhi ? u : vhi;
      }
    }
    if constexpr (MASK) {
      const Cond c1 = make_cond(c1code, c1len, consts);
      if (c1.simple) {
        // `x CMP y`: every operand load of the tile issued before the first compare (the interpreter loop below
        // waits on one row's loads at a time); the operand columns resolved once (ColRef)
        const ColRef ca = c1.a.op == OP_CONST ? ColRef{nullptr, 0} : col_ref(st, c1.a.op == OP_COL ? c1.a.a : c1.a.c);
        const ColRef cb = c1.b.op == OP_CONST ? ColRef{nullptr, 0} : col_ref(st, c1.b.op == OP_COL ? c1.b.a : c1.b.c);
        StackVal l[kItems], r[kItems];
#pragma unroll
        for (int k = 0; k < kItems; ++k) {
          const int64_t p = base + w * 64 * kItems + k * 64 + lane;
          if (p < hi0) {
            l[k] = c1.a.op == OP_CONST ? c1.ka : ca.at(p);
            r[k] = c1.b.op == OP_CONST ? c1.kb : cb.at(p);
          }
        }
#pragma unroll
        for (int k = 0; k < kItems; ++k) {
          const int64_t p = base + w * 64 * kItems + k * 64 + lane;
          if (p - lane >= hi0) break;
          const bool cv = p < hi0 && ((l[k].null || r[k].null) ? c1.op.sub == CMP_NE : do_compare(c1.op, l[k], r[k]));
          const uint64_t bal = __ballot(cv);
          if (lane == 0) c1mask[p >> 6] = bal;
        }
        continue;
      }
#pragma unroll 1
      for (int k = 0; k < kItems; ++k) {
        const int64_t p = base + w * 64 * kItems + k * 64 + lane;
        if (p - lane >= hi0) break;
        const bool cv = p < hi0 && eval(c1, RowLoader{st, p});
        const uint64_t bal = __ballot(cv);
        if (lane == 0) c1mask[p >> 6] = bal;
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long x = __shfl_down(lo, o, 64), y = __shfl_down(hi, o, 64), z = __shfl_down(om, o, 64);
    unsigned long long e = __shfl_down(vlo, o, 64), f = __shfl_down(vhi, o, 64);
    lo = x < lo ? x : lo;
    hi = y > hi ? y : hi;
    om = z > om ? z : om;
    vlo = e < vlo ? e : vlo;
    vhi = f > vhi ? f : vhi;
  }
  bad = __any(bad) ? 1u : 0u;
  bado = __any(bado) ? 1u : 0u;
  if (lane == 0) {
    if (kcol) {
      atomicMin(&c->kmin, lo);
      atomicMax(&c->kmax, hi);
    }
    if (vlong) {
      atomicMin(&c->vmin, vlo);
      atomicMax(&c->vmax, vhi);
    }
    if (ord) atomicMax(&c->omax, om);
    if (bad) atomicOr(&c->bad_ts, 1u);
    if (bado) atomicOr(&c->bad_ord, 1u);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    c->ts0 = ts[0];
    c->ts_last = ts[n - 1];
    c->o0 = ord ? ord[0] - obase : 0;
    if (!ord) c->omax = (unsigned long long)(n - 1);
  }
  __syncthreads();
  if (kcol)
    for (int d = threadIdx.x; d < kBins; d += kBlock) cnt[(int64_t)d * G + blockIdx.x] = h[d];
}

// ---------------------------------------------------------------- up-sweeps and scans

template <typename KT>
struct KeyColDigits {  // rebased key from the original key column
  const KT* kcol;
  int64_t kmin;
  __device__ uint32_t key(int64_t p) const { return (uint32_t)((int64_t)kcol[p] - kmin); }
};
struct RecDigits {  // keys of keyed records (word 0 of each 16-byte record)
  const uint4* r;
  __device__ uint32_t key(int64_t p) const { return ((const uint32_t*)r)[4 * p]; }
};
struct PairDigits {  // j of (j << 32) | i pairs
  const uint64_t* q;
  __device__ uint32_t key(int64_t p) const { return (uint32_t)(q[p] >> 32); }
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
      k[u] = p < hi ? src.key(p) : 0u;
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
    const int d = threadIdx.x * kBinsPerThread + k;
    v[k] = d < kBins ? tot[d] : 0u;
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
    if (threadIdx.x * kBinsPerThread + k < kBins) tot[threadIdx.x * kBinsPerThread + k] = run;
    run += v[k];
  }
}

// ---------------------------------------------------------------- down-sweep

// c1 over the compared attribute's value alone (slot-0 variables and stream columns all read that attribute)
template <typename VT>
struct ValLoader {
  VT v;
  __device__ StackVal var(const Instr&) const {
    StackVal r;
    r.i = 0;
    r.d = 0;
    r.null = 0;
    if constexpr (std::is_floating_point<VT>::value) r.d = (double)v;
    else r.i = (int64_t)v;
    return r;
  }
};

// Pass 0 of the keyed sort: builds the record from the original columns. Key and compared-attribute column
// types are template parameters. c1 comes from prep's bit mask, or (c1_inline: c1 reads only the compared
// attribute) is evaluated here on the loaded value.
template <typename KT, typename VT>
struct OrigSrc {
  const NfaStream* st;
  const KT* kcol;
  const VT* vcol;
  int64_t kmin;
  int vmode;
  int64_t vmin;
  const uint64_t* c1mask;
  const int64_t* ts;
  int64_t ts0;
  const int64_t* ord;
  int64_t obase;
  const Instr* c1code;
  int c1len;
  const DVal* consts;
  bool c1_inline;
  Cond c1;
  __device__ void init() {
    if (c1_inline) c1 = make_cond(c1code, c1len, consts);
  }
  __device__ uint32_t c1_bit(VT v, uint64_t m, int64_t p) const {
    if (c1_inline) return eval_simple(c1, ValLoader<VT>{v}) ? 1u : 0u;
    return (uint32_t)(m >> (p & 63)) & 1u;
  }
  __device__ uint4 rec(int64_t p) const {
    uint4 r;
    const VT v = vcol[p];
    const uint64_t m = c1_inline ? 0ull : c1mask[p >> 6];
    r.x = (uint32_t)((int64_t)kcol[p] - kmin) | (c1_bit(v, m, p) << 31);
    r.y = ord ? (uint32_t)(ord[p] - obase) : (uint32_t)p;
    r.z = vcode<VT>(v, vmode, vmin);
    r.w = (uint32_t)(ts[p] - ts0);
    return r;
  }
  // raw column values of one event (loads in flight until split() uses them) + its c1 mask word
  struct Raw {
    KT k;
    VT v;
    int64_t t, o;
    uint64_t m;
  };
  __device__ Raw load(int64_t p) const {
    Raw r;
#if SM_ORIG_NT_LOAD
    // read-once columns: nontemporal loads keep the L2 for the pass's scattered record stores (as RecSrc)
    r.k = __builtin_nontemporal_load(kcol + p);
    r.v = __builtin_nontemporal_load(vcol + p);
    r.t = __builtin_nontemporal_load(ts + p);
    r.o = ord ? __builtin_nontemporal_load(ord + p) - obase : p;
#else
    r.k = kcol[p];
    r.v = vcol[p];
    r.t = ts[p];
    r.o = ord ? ord[p] - obase : p;
#endif
    r.m = c1_inline ? 0ull : c1mask[p >> 6];
    return r;
  }
  __device__ void split(const Raw& r, int64_t p, uint64_t& a, uint64_t& b) const {
    const uint32_t c1 = c1_bit(r.v, r.m, p);
    a = (uint64_t)((uint32_t)((int64_t)r.k - kmin) | (c1 << 31)) | ((uint64_t)(uint32_t)r.o << 32);
    b = (uint64_t)vcode<VT>(r.v, vmode, vmin) | ((uint64_t)(uint32_t)(r.t - ts0) << 32);
  }
  __device__ uint4 record(const Raw& r, int64_t p) const {  // pass0_kernel (pass0_dev.h)
    const uint32_t c1 = c1_bit(r.v, r.m, p);
    return make_uint4((uint32_t)((int64_t)r.k - kmin) | (c1 << 31), (uint32_t)r.o, vcode<VT>(r.v, vmode, vmin),
                      (uint32_t)(r.t - ts0));
  }
  __device__ void flush() {}
};

struct RecSrc {
  const uint4* r;
  __device__ void init() {}
  typedef unsigned int Raw __attribute__((ext_vector_type(4)));
  // read-once stream: nontemporal loads keep the L2 for the scattered stores (PMC: -10 % pass time)
  __device__ uint4 rec(int64_t p) const {
    const Raw v = __builtin_nontemporal_load((const Raw*)r + p);
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  __device__ Raw load(int64_t p) const { return __builtin_nontemporal_load((const Raw*)r + p); }
  __device__ void split(const Raw& v, int64_t, uint64_t& a, uint64_t& b) const {
    a = (uint64_t)v.x | ((uint64_t)v.y << 32);
    b = (uint64_t)v.z | ((uint64_t)v.w << 32);
  }
};

struct PairSrc {  // (j << 32) | i
  const uint64_t* q;
  __device__ void init() {}
  using Raw = uint64_t;
  __device__ Raw load(int64_t p) const { return __builtin_nontemporal_load(q + p); }
  __device__ void split(const Raw& v, int64_t, uint64_t& a, uint64_t&) const { a = v; }
};

// Down-sweep of one LSD pass over chunk blockIdx.x (persistent: tile by tile, running per-digit offsets).
//   MODE 0: keyed record from the original columns (OrigSrc) → records
//   MODE 1: keyed records (RecSrc) → records
//   MODE 2: (j << 32) | i pairs → pairs (the last pass writes the output: in memory the (i, j) u32 pairs)
template <int MODE, typename Src>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4)))
downsweep_kernel(Src src, uint4* __restrict__ drec, uint64_t* __restrict__ dpairs, int64_t n, int64_t per,
                 const uint32_t* seg_len, int G, int shift, const uint32_t* __restrict__ cnt,
                 const uint32_t* __restrict__ dbase) {
  __shared__ uint64_t xb64[kTile];  // exchange buffer: records in two 64-bit halves, pairs whole
  __shared__ uint16_t wcnt[kWaves][kBins];
  __shared__ uint32_t tstart[kBins];
  __shared__ uint32_t run[kBins];  // next output position of each digit for this chunk
  __shared__ uint32_t lw[kWaves];

  int64_t lo, len;
  chunk_range(blockIdx.x, n, per, seg_len, lo, len);
  src.init();
  for (int d = threadIdx.x; d < kBins; d += kBlock) run[d] = dbase[d] + cnt[(int64_t)d * G + blockIdx.x];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = lanemask_lt();
  SM_STAMP_DECL;

  for (int64_t base = lo; base < lo + len; base += kTile) {
    SM_STAMP(0);
    const int tile_n = (int)((lo + len - base) < kTile ? (lo + len - base) : kTile);
    // every load of the tile is issued up front (one exposed memory latency per tile)
    uint64_t a[kItems], b[kItems];  // records: a = key | ordinal << 32, b = code | ts << 32; pairs: a only
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const int e = w * 64 * kItems + k * 64 + lane;
      if (e < tile_n) {
        const int64_t p = base + e;
        if constexpr (MODE <= 1) {
          const uint4 r = src.rec(p);
          a[k] = (uint64_t)r.x | ((uint64_t)r.y << 32);
          b[k] = (uint64_t)r.z | ((uint64_t)r.w << 32);
        } else {
          a[k] = __builtin_nontemporal_load(src.q + p);
        }
      }
    }
    lds_barrier();  // previous tile's readers of wcnt / xb64 / run are done
    for (int k = threadIdx.x; k < kWaves * kBins; k += kBlock) (&wcnt[0][0])[k] = 0;
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): every load of the tile retired (known to the compiler, so no
                                         // later vmcnt wait for them lands behind this tile's stores)
    lds_barrier();
    SM_STAMP(1);

    uint32_t lp[kItems];  // rank within (wave, digit), then local sorted position
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const int e = w * 64 * kItems + k * 64 + lane;
      const bool valid = e < tile_n;
      const uint32_t key = MODE <= 1 ? (uint32_t)a[k] : (uint32_t)(a[k] >> 32);
      const uint32_t d = valid ? ((key & kKeyMask) >> shift) & (kBins - 1) : 0u;
      const uint64_t peers = peer_mask(d, valid);
      uint32_t old = 0;
      if (valid) old = wcnt[w][d];
      const uint32_t below = (uint32_t)__popcll(peers & lt);
      if (valid && below == 0) wcnt[w][d] = (uint16_t)(old + (uint32_t)__popcll(peers));
      lp[k] = old + below;
    }
    lds_barrier();
    SM_STAMP(2);

    // per digit: wave offsets (exclusive, in place) and the tile count
    uint32_t cnt_t[kBinsPerThread];
    uint32_t csum = 0;
#pragma unroll
    for (int bb = 0; bb < kBinsPerThread; ++bb) {
      const int d = threadIdx.x * kBinsPerThread + bb;
      uint32_t r = 0;
      if (d < kBins)
        for (int q = 0; q < kWaves; ++q) {
          const uint32_t c = wcnt[q][d];
          wcnt[q][d] = (uint16_t)r;
          r += c;
        }
      cnt_t[bb] = r;
      csum += r;
    }
    {  // block exclusive scan of the tile counts over digits → tstart
      uint32_t inc = csum;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(inc, o, 64);
        if (lane >= o) inc += u;
      }
      if (lane == 63) lw[w] = inc;
      lds_barrier();
      uint32_t r = inc - csum;
      for (int q = 0; q < w; ++q) r += lw[q];
#pragma unroll
      for (int bb = 0; bb < kBinsPerThread; ++bb) {
        if (threadIdx.x * kBinsPerThread + bb < kBins) tstart[threadIdx.x * kBinsPerThread + bb] = r;
        r += cnt_t[bb];
      }
    }
    lds_barrier();
    SM_STAMP(3);

    // local sorted positions; the first exchange carries the key, so each sorted slot learns its digit and
    // destination from it
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const int e = w * 64 * kItems + k * 64 + lane;
      if (e < tile_n) {
        const uint32_t key = MODE <= 1 ? (uint32_t)a[k] : (uint32_t)(a[k] >> 32);
        const uint32_t d = ((key & kKeyMask) >> shift) & (kBins - 1);
        lp[k] += tstart[d] + wcnt[w][d];
        xb64[lp[k]] = a[k];
      }
    }
    lds_barrier();
    uint32_t dest[kItems];
    uint64_t sa[kItems];  // records: first half of the slot's record
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
      const int s = r * kBlock + threadIdx.x;
      if (s < tile_n) {
        const uint64_t x = xb64[s];
        const uint32_t key = MODE <= 1 ? (uint32_t)x : (uint32_t)(x >> 32);
        const uint32_t d = ((key & kKeyMask) >> shift) & (kBins - 1);
        dest[r] = run[d] + (uint32_t)s - tstart[d];
        if constexpr (MODE <= 1) sa[r] = x;
        else dpairs[dest[r]] = x;
      }
    }
    SM_STAMP(4);
    if constexpr (MODE <= 1) {  // second half, then one 16-byte store per record
      lds_barrier();
#pragma unroll
      for (int k = 0; k < kItems; ++k) {
        const int e = w * 64 * kItems + k * 64 + lane;
        if (e < tile_n) xb64[lp[k]] = b[k];
      }
      lds_barrier();
#pragma unroll
      for (int r = 0; r < kItems; ++r) {
        const int s = r * kBlock + threadIdx.x;
        if (s < tile_n) {
          const uint64_t y = xb64[s];
          drec[dest[r]] = make_uint4((uint32_t)sa[r], (uint32_t)(sa[r] >> 32), (uint32_t)y, (uint32_t)(y >> 32));
        }
      }
    }
    SM_STAMP(5);
    lds_barrier();  // every destination computed from run[] before it advances
#pragma unroll
    for (int bb = 0; bb < kBinsPerThread; ++bb)
      if (threadIdx.x * kBinsPerThread + bb < kBins) run[threadIdx.x * kBinsPerThread + bb] += cnt_t[bb];
    SM_STAMP(6);
  }
  SM_STAMP_FLUSH;
}

// Write-combining down-sweep (same pass semantics as downsweep_kernel). A tile sends about 4 elements to each of
// its kBins digit runs, so plain scattered stores leave most 64-byte segments of the output partly written by
// one tile and finished by the next; with 64 workgroups per XCD each holding 1024 runs open, the L2 evicts those
// partial lines in between and the pass writes ~1.7x its bytes (PMC: TCC_EA0_WRREQ / _64B). Here a tile stores
// only elements whose 64-byte segment is complete in this chunk's view; the tail of each run (< one segment) is
// carried in LDS to the next tile, and the last tile of the chunk flushes everything. Loads of tile t+1 are
// issued as soon as tile t's elements are in LDS, so they overlap tile t's stores.
#ifndef SM_WCB
#define SM_WCB 1024
#endif
constexpr int kWcBlock = SM_WCB;
constexpr int kWcWaves = kWcBlock / 64;
constexpr int kWcItems = kTile / kWcBlock;
constexpr int kWcBPT = kBins >= kWcBlock ? kBins / kWcBlock : 1;  // digits owned per thread
static_assert(kTile % kWcBlock == 0, "write-combining tile");

template <int MODE, typename Src>
__global__ void __launch_bounds__(kWcBlock)
downsweep_wc_kernel(Src src, uint4* __restrict__ drec, uint64_t* __restrict__ dpairs, int64_t n, int64_t per,
                    const uint32_t* seg_len, int G, int shift, const uint32_t* __restrict__ cnt,
                    const uint32_t* __restrict__ dbase) {
  constexpr int S = MODE <= 1 ? 4 : 8;   // elements per 64-byte segment
  constexpr int CW = MODE <= 1 ? 2 : 1;  // 64-bit words per element
  __shared__ uint64_t xb64[kTile];
  __shared__ uint16_t wcnt[kWcWaves][kBins];
  __shared__ uint32_t tstart[kBins + 1];
  __shared__ uint32_t run[kBins];  // next output position of each digit for this chunk
  __shared__ uint32_t cst[kBins];  // first carried position of each digit: carry = [cst, run)
  __shared__ uint64_t carry[kBins * (S - 1) * CW];
  __shared__ uint32_t lw[kWcWaves];

  int64_t lo, len;
  chunk_range(blockIdx.x, n, per, seg_len, lo, len);
  src.init();
  for (int d = threadIdx.x; d < kBins; d += kWcBlock) {
    const uint32_t r0 = dbase[d] + cnt[(int64_t)d * G + blockIdx.x];
    run[d] = r0;
    cst[d] = r0;
  }
  if (threadIdx.x == 0) tstart[kBins] = 0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = lanemask_lt();
  SM_STAMP_DECL;

  typename Src::Raw raw[kWcItems];
  auto load_tile = [&](int64_t base) {
    const int64_t rem = lo + len - base;
    const int tn = rem < kTile ? (int)rem : kTile;
#pragma unroll
    for (int k = 0; k < kWcItems; ++k) {
      const int e = w * 64 * kWcItems + k * 64 + lane;
      if (e < tn) raw[k] = src.load(base + e);
    }
  };
  if (len > 0) load_tile(lo);

  for (int64_t base = lo; base < lo + len; base += kTile) {
    SM_STAMP(0);
    const int tile_n = (int)((lo + len - base) < kTile ? (lo + len - base) : kTile);
    const bool last = base + kTile >= lo + len;
    uint64_t a[kWcItems], b[kWcItems];
#pragma unroll
    for (int k = 0; k < kWcItems; ++k) {
      const int e = w * 64 * kWcItems + k * 64 + lane;
      if (e < tile_n) src.split(raw[k], base + e, a[k], b[k]);
    }
    lds_barrier();  // previous tile's readers of wcnt / xb64 / run / tstart are done
    for (int k = threadIdx.x; k < kWcWaves * kBins; k += kWcBlock) (&wcnt[0][0])[k] = 0;
    lds_barrier();
    SM_STAMP(1);

    uint32_t lp[kWcItems];  // rank within (wave, digit), then local sorted position
#pragma unroll
    for (int k = 0; k < kWcItems; ++k) {
      const int e = w * 64 * kWcItems + k * 64 + lane;
      const bool valid = e < tile_n;
      const uint32_t key = MODE <= 1 ? (uint32_t)a[k] : (uint32_t)(a[k] >> 32);
      const uint32_t d = valid ? ((key & kKeyMask) >> shift) & (kBins - 1) : 0u;
      const uint64_t peers = peer_mask(d, valid);
      uint32_t old = 0;
      if (valid) old = wcnt[w][d];
      const uint32_t below = (uint32_t)__popcll(peers & lt);
      if (valid && below == 0) wcnt[w][d] = (uint16_t)(old + (uint32_t)__popcll(peers));
      lp[k] = old + below;
    }
    lds_barrier();
    SM_STAMP(2);

    // per digit: wave offsets (exclusive, in place) and the tile count
    uint32_t cnt_t[kWcBPT];
    uint32_t csum = 0;
#pragma unroll
    for (int bb = 0; bb < kWcBPT; ++bb) {
      const int d = threadIdx.x * kWcBPT + bb;
      uint32_t r = 0;
      if (d < kBins)
        for (int q = 0; q < kWcWaves; ++q) {
          const uint32_t c = wcnt[q][d];
          wcnt[q][d] = (uint16_t)r;
          r += c;
        }
      cnt_t[bb] = r;
      csum += r;
    }
    {  // block exclusive scan of the tile counts over digits → tstart
      uint32_t inc = csum;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(inc, o, 64);
        if (lane >= o) inc += u;
      }
      if (lane == 63) lw[w] = inc;
      lds_barrier();
      uint32_t r = inc - csum;
      for (int q = 0; q < w; ++q) r += lw[q];
#pragma unroll
      for (int bb = 0; bb < kWcBPT; ++bb) {
        if (threadIdx.x * kWcBPT + bb < kBins) tstart[threadIdx.x * kWcBPT + bb] = r;
        r += cnt_t[bb];
      }
      if (threadIdx.x == kWcBlock - 1) tstart[kBins] = r;
    }
    lds_barrier();
    SM_STAMP(3);

    // local sorted positions; the first exchange carries the key, so each sorted slot learns its digit,
    // its destination and whether its segment completes in this tile
#pragma unroll
    for (int k = 0; k < kWcItems; ++k) {
      const int e = w * 64 * kWcItems + k * 64 + lane;
      if (e < tile_n) {
        const uint32_t key = MODE <= 1 ? (uint32_t)a[k] : (uint32_t)(a[k] >> 32);
        const uint32_t d = ((key & kKeyMask) >> shift) & (kBins - 1);
        lp[k] += tstart[d] + wcnt[w][d];
        xb64[lp[k]] = a[k];
      }
    }
    if constexpr (MODE == 2)
      if (!last) load_tile(base + kTile);  // a[] is in LDS: the next tile's loads overlap this tile's stores
    lds_barrier();
    uint32_t dest[kWcItems], lim[kWcItems], ncs[kWcItems], dg[kWcItems];
    uint64_t sa[kWcItems];
#pragma unroll
    for (int r = 0; r < kWcItems; ++r) {
      const int s = r * kWcBlock + threadIdx.x;
      if (s < tile_n) {
        const uint64_t x = xb64[s];
        const uint32_t key = MODE <= 1 ? (uint32_t)x : (uint32_t)(x >> 32);
        const uint32_t d = ((key & kKeyMask) >> shift) & (kBins - 1);
        const uint32_t ts_ = tstart[d], rn = run[d];
        dest[r] = rn + (uint32_t)s - ts_;
        const uint32_t l = last ? 0xffffffffu : ((rn + tstart[d + 1] - ts_) & ~(uint32_t)(S - 1));
        lim[r] = l;
        const uint32_t c0 = cst[d];
        ncs[r] = c0 > l ? c0 : l;
        dg[r] = d;
        sa[r] = x;
      }
    }
    // carried elements of each digit whose segment completes now (or the chunk ends) leave first; the slots they
    // free are refilled only after the next barrier
    auto flush_old = [&]() {
#pragma unroll
      for (int bb = 0; bb < kWcBPT; ++bb) {
        const int d = threadIdx.x * kWcBPT + bb;
        if (d < kBins) {
          const uint32_t c0 = cst[d], rn = run[d];
          const uint32_t l = (rn + cnt_t[bb]) & ~(uint32_t)(S - 1);
          if (rn != c0 && (last || l > c0)) {
            for (uint32_t q = 0; q < rn - c0; ++q) {
              const uint64_t* cw = &carry[((uint32_t)d * (S - 1) + q) * CW];
              if constexpr (MODE <= 1) drec[c0 + q] = make_uint4((uint32_t)cw[0], (uint32_t)(cw[0] >> 32),
                                                                 (uint32_t)cw[1], (uint32_t)(cw[1] >> 32));
              else dpairs[c0 + q] = cw[0];
            }
          }
        }
      }
    };
    SM_STAMP(4);
    if constexpr (MODE <= 1) {  // second half, then one 16-byte store (or carry) per record
      lds_barrier();
#pragma unroll
      for (int k = 0; k < kWcItems; ++k) {
        const int e = w * 64 * kWcItems + k * 64 + lane;
        if (e < tile_n) xb64[lp[k]] = b[k];
      }
      if (!last) load_tile(base + kTile);
      flush_old();
      lds_barrier();
#pragma unroll
      for (int r = 0; r < kWcItems; ++r) {
        const int s = r * kWcBlock + threadIdx.x;
        if (s < tile_n) {
          const uint64_t y = xb64[s];
          if (dest[r] < lim[r]) {
            drec[dest[r]] = make_uint4((uint32_t)sa[r], (uint32_t)(sa[r] >> 32), (uint32_t)y, (uint32_t)(y >> 32));
          } else {
            uint64_t* cw = &carry[(dg[r] * (S - 1) + (dest[r] - ncs[r])) * CW];
            cw[0] = sa[r];
            cw[1] = y;
          }
        }
      }
    } else {
      flush_old();
      lds_barrier();
#pragma unroll
      for (int r = 0; r < kWcItems; ++r) {
        const int s = r * kWcBlock + threadIdx.x;
        if (s < tile_n) {
          if (dest[r] < lim[r]) dpairs[dest[r]] = sa[r];
          else carry[dg[r] * (S - 1) + (dest[r] - ncs[r])] = sa[r];
        }
      }
    }
    SM_STAMP(5);
    lds_barrier();  // every destination computed from run[] / cst[] before they advance
#pragma unroll
    for (int bb = 0; bb < kWcBPT; ++bb) {
      const int d = threadIdx.x * kWcBPT + bb;
      if (d < kBins) {
        const uint32_t rn = run[d] + cnt_t[bb];
        const uint32_t l = rn & ~(uint32_t)(S - 1);
        run[d] = rn;
        if (l > cst[d]) cst[d] = l;
      }
    }
    SM_STAMP(6);
  }
  SM_STAMP_FLUSH;
}

// ---------------------------------------------------------------- walk

struct WalkArgs {
  const uint4* rec;  // keyed: sorted records
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
  bool exact_codes;
  const uint64_t* c1mask;  // unkeyed: c1 bits of the events
  // carry out: partials still pending at the end (their key's events ran out before a match or expiry)
  int64_t kmin, ts0;
  int64_t* cand;
  uint32_t* cand_n;
  uint32_t cand_cap;
  uint32_t* err;
};

template <bool KEYED>
struct WalkLds;
template <>
struct WalkLds<true> {
  uint4 r[kWalkLds];  // {key | c1 << 31, ordinal, value code, ts}: one ds_read_b128 per record
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
__global__ void __launch_bounds__(kWalkBlock) __attribute__((amdgpu_waves_per_eu(6))) walk_kernel(WalkArgs a, int64_t per, int G,
                                                          uint64_t* __restrict__ stq, uint32_t* __restrict__ mcount,
                                                          uint32_t* __restrict__ jcnt) {
  __shared__ WalkLds<KEYED> L;
  __shared__ uint32_t sj[kWalkItems][kWalkBlock];  // per item: matched position - tile base (or resume point)
  __shared__ uint64_t sbal[kWalkWaves][kWalkItems];
  __shared__ uint32_t wtot[kWalkWaves];
  __shared__ uint32_t jh[kBins];
  __shared__ uint32_t sh_run;
  // unkeyed ordered compare (`e2.x OP e1.x`, OP one of < <= > >=): per block of kSkipBlk staged records the value
  // that would satisfy c2 for the most e1 (max for > / >=, min for < / <=, NaN excluded), so a scan can step over a
  // whole block none of whose records can match (event time is non-decreasing: a block that holds the window's end
  // and no match ends the scan like the first record after it)
  constexpr bool kSkip = !KEYED && (OP == CMP_LT || OP == CMP_LE || OP == CMP_GT || OP == CMP_GE);
  constexpr int kSkipBlk = 16;
  __shared__ uint64_t bx[kSkip ? kWalkLds / kSkipBlk : 1];

  const int64_t n = a.n;
  int64_t lo, len;
  chunk_range(blockIdx.x, n, per, nullptr, lo, len);
  const int64_t hi = lo + len;
  for (int d = threadIdx.x; d < kBins; d += kWalkBlock) jh[d] = 0;
  if (threadIdx.x == 0) sh_run = 0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = lanemask_lt();
  C2<OP, FP> c2;  // unkeyed
  if constexpr (!KEYED && OP < 0) c2.c = make_cond(a.c2, a.c2_len, a.consts);
  c2.vtype = a.vtype;
  C2Code<OP, FP> cc{a.exact_codes, a.vtype, a.st->cols[a.vattr], a.ord, a.obase, n};  // keyed
  const ColRef vref = KEYED ? ColRef{nullptr, 0} : col_ref(a.st, a.vattr);  // unkeyed: the compared column

  // keyed: the next tile's records are loaded into registers while the current tile is scanned
  constexpr int kPre = (kWalkLds + kWalkBlock - 1) / kWalkBlock;
  uint4 pre[kPre];
  auto prefetch = [&](int64_t b) {
#pragma unroll
    for (int q = 0; q < kPre; ++q) {
      const int64_t p = b + q * kWalkBlock + threadIdx.x;
      if (q * kWalkBlock + threadIdx.x < kWalkLds && p < n) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 v = __builtin_nontemporal_load((const u32x4*)a.rec + p);
        pre[q] = make_uint4(v.x, v.y, v.z, v.w);
      }
    }
  };
  if constexpr (KEYED) prefetch(lo);
  SM_STAMP_DECL;

  for (int64_t base = lo; base < hi; base += kWalkTile) {
    SM_STAMP(0);
    lds_barrier();  // previous tile's LDS readers are done
    const int nload = (int)((n - base) < kWalkLds ? (n - base) : kWalkLds);
    if constexpr (KEYED) {
#pragma unroll
      for (int q = 0; q < kPre; ++q) {
        const int e = q * kWalkBlock + threadIdx.x;
        if (e < nload) {
          L.r[e] = pre[q];
        }
      }
      if (base + kWalkTile < hi) prefetch(base + kWalkTile);
    } else {
      for (int e = threadIdx.x; e < nload; e += kWalkBlock) {
        const int64_t p = base + e;
        L.t[e] = a.ts[p];
        L.v[e] = canon(vref.at(p), a.vtype);
      }
    }
    lds_barrier();
    if constexpr (kSkip) {
      for (int b = threadIdx.x; b < nload / kSkipBlk; b += kWalkBlock) {
        constexpr bool kMax = OP == CMP_GT || OP == CMP_GE;
        if constexpr (FP) {
          double x = kMax ? -__builtin_inf() : __builtin_inf();
          for (int e = 0; e < kSkipBlk; ++e) {
            const double y = __longlong_as_double((long long)L.v[b * kSkipBlk + e]);
            if (kMax ? y > x : y < x) x = y;  // NaN never replaces (and never matches)
          }
          bx[b] = (uint64_t)__double_as_longlong(x);
        } else {
          int64_t x = kMax ? INT64_MIN : INT64_MAX;
          for (int e = 0; e < kSkipBlk; ++e) {
            const int64_t y = (int64_t)L.v[b * kSkipBlk + e];
            if (kMax ? y > x : y < x) x = y;
          }
          bx[b] = (uint64_t)x;
        }
      }
      lds_barrier();
    }
    SM_STAMP(1);
    const int lend = nload;  // staged positions are [0, lend) relative to base
    uint32_t c1m = 0;        // c1 of each item (bit k)
#pragma unroll 1
    for (int k = 0; k < kWalkItems; ++k) {
      const int lu = w * 64 * kWalkItems + k * 64 + lane;
      if (base + lu < hi) {
        bool c;
        if constexpr (KEYED) c = (L.r[lu].x >> 31) != 0;
        else c = (a.c1mask[(base + lu) >> 6] >> ((base + lu) & 63)) & 1ull;
        if (c) c1m |= 1u << k;
      }
    }
    // lane-private queue over the items with c1. The loop body is written branch-light (selects, one
    // predicated take): every live lane advances its scan by one record per iteration.
    uint32_t hasm = 0, openm = 0, pendm = 0;  // matched / scan left the staged records / key's events ran out
    uint32_t todo = c1m;
    int k = 0, v = 0, steps = 0;
    uint64_t vu = 0;
    int64_t tu = 0;
    uint32_t key = 0, cu = 0, ou = 0;
    bool live = false;
    int vstart = 0;
    auto take = [&]() {
      live = todo != 0;
      k = live ? __ffs(todo) - 1 : 0;
      todo &= todo - 1;
      const int lu = w * 64 * kWalkItems + k * 64 + lane;
      if constexpr (KEYED) {
        const uint4 r = L.r[lu];
        key = r.x & kKeyMask;
        ou = r.y;
        cu = r.z;
        tu = r.w;
      } else {
        tu = L.t[lu];
        vu = L.v[lu];
      }
      v = lu + 1;
      vstart = v;
      steps = 0;
    };
    SM_STAMP(2);
    take();
    while (__any(live)) {
      // unkeyed scans run until c2 holds or the window closes (up to window-many events: no key run bounds them),
      // so a lane scans privately for kUnkeyedBudget records and leaves the rest to the wave-cooperative finish
      const bool inb = v < lend && (KEYED || (kSkip ? steps : v - vstart) < kUnkeyedBudget);
      // a whole block without a possible match: step over it (its window end, if any, is seen at the next record)
      bool skip = false;
      if constexpr (kSkip) skip = live && inb && (v % kSkipBlk) == 0 && v + kSkipBlk <= lend && !c2(vu, bx[v / kSkipBlk]);
      const int vv = inb ? v : lend - 1;
      bool stop, hit, kchg = false;
      if constexpr (KEYED) {
        // straight-line step: one ds_read_b128, conditions combined without short-circuit branches; the rare
        // exact comparisons run afterwards for the lanes that need them
        const uint4 r = L.r[vv];
        const bool expired = (a.within >= 0) & ((int64_t)(r.w - (uint32_t)tu) > a.within);
        kchg = inb & (((r.x ^ key) & kKeyMask) != 0u);
        stop = (!inb) | kchg | expired;
        const bool ex = live & !stop & cc.needs_exact(cu, r.z);
        hit = live & !stop & !ex & cmp_fixed<OP>(r.z, cu);
        if (__any(ex))
          if (ex) hit = cc.exact(ou, r.y);
      } else {
        const int64_t d = L.t[vv] - tu;
        stop = !skip && (!inb || (a.within >= 0 && (d < 0 ? -d : d) > a.within));
        hit = live && !skip && !stop && c2(vu, L.v[vv]);
      }
      const bool open = live && !inb && base + v < n;  // leaves the staged records: finished from global below
      const bool pend = live && (kchg || (!inb && base + v >= n));  // the key's events (or the batch) ran out
      hasm |= hit ? (1u << k) : 0u;
      openm |= open ? (1u << k) : 0u;
      pendm |= pend ? (1u << k) : 0u;
      if (hit || open) sj[k][threadIdx.x] = (uint32_t)v;
      const bool done = live && (stop || hit);
      v += skip ? kSkipBlk : 1;
      ++steps;
      if (done) take();
    }
    SM_STAMP(3);
    if constexpr (!KEYED) {
      // wave-cooperative finish of the open scans: one scan at a time, 64 consecutive candidates per step (one
      // ballot each), so a window of W events costs W / 64 steps instead of W steps on one lane
      uint64_t pend = __ballot(openm != 0);
#pragma unroll 1
      while (pend) {
        const int src = __ffsll((unsigned long long)pend) - 1;
        const uint32_t om = __shfl(openm, src, 64);
        const int kk = __ffs(om) - 1;
        const int luu = w * 64 * kWalkItems + kk * 64 + src;
        const int64_t t0 = L.t[luu];
        const uint64_t v0 = L.v[luu];
        int64_t found = -1;
        bool ran_out = true;  // no expiring event before the end of the batch
        for (int64_t p = base + sj[kk][w * 64 + src]; p < n; p += 64) {
          const int64_t q = p + lane;
          bool stp = q >= n, hit = false;
          if (!stp) {
            const int64_t d = a.ts[q] - t0;
            stp = a.within >= 0 && (d < 0 ? -d : d) > a.within;
            if (!stp) hit = c2(v0, canon(vref.at(q), a.vtype));
          }
          const uint64_t hb = __ballot(hit), any = __ballot(stp) | hb;
          if (any) {
            const int f = __ffsll((unsigned long long)any) - 1;
            if ((hb >> f) & 1ull) found = p + f;
            ran_out = found < 0 && p + f >= n;
            break;
          }
        }
        if (lane == src) {
          if (found >= 0) {
            hasm |= 1u << kk;
            sj[kk][threadIdx.x] = (uint32_t)(found - base);
          } else if (ran_out) {
            pendm |= 1u << kk;
          }
          openm &= ~(1u << kk);
        }
        pend = __ballot(openm != 0);
      }
    }
    // scans that ran past the staged records
#pragma unroll 1
    while (openm) {
      const int kk = __ffs(openm) - 1;
      openm &= openm - 1;
      const int luu = w * 64 * kWalkItems + kk * 64 + lane;
      bool ran_out = true;
      for (int64_t p = base + sj[kk][threadIdx.x]; p < n; ++p) {
        bool hit;
        if constexpr (KEYED) {
          const uint4 r = a.rec[p];
          const uint4 ru = L.r[luu];
          if ((r.x & kKeyMask) != (ru.x & kKeyMask)) break;  // the key's events ran out: pending
          if (a.within >= 0 && (int64_t)(r.w - ru.w) > a.within) {
            ran_out = false;
            break;
          }
          hit = cc(ru.z, ru.y, r.z, r.y);
        } else {
          const int64_t d = a.ts[p] - L.t[luu];
          if (a.within >= 0 && (d < 0 ? -d : d) > a.within) {
            ran_out = false;
            break;
          }
          hit = c2(L.v[luu], canon(vref.at(p), a.vtype));
        }
        if (hit) {
          hasm |= 1u << kk;
          sj[kk][threadIdx.x] = (uint32_t)(p - base);
          ran_out = false;
          break;
        }
      }
      if (ran_out) pendm |= 1u << kk;
    }
    SM_STAMP(4);
    // carry out: partials still pending at the end of the batch (wave-aggregated append)
    if (__any(pendm != 0)) {
      const uint32_t np = (uint32_t)__popc(pendm);
      uint32_t inc = np;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(inc, o, 64);
        if (lane >= o) inc += u;
      }
      uint32_t cb = 0;
      if (lane == 63 && inc) cb = atomicAdd(a.cand_n, inc);
      cb = __shfl(cb, 63, 64) + inc - np;
      for (uint32_t pm = pendm; pm; pm &= pm - 1) {
        const int q = __ffs(pm) - 1;
        const int luq = w * 64 * kWalkItems + q * 64 + lane;
        int64_t key = 0, ordg, tsg, row;
        if constexpr (KEYED) {
          const uint4 r = L.r[luq];
          key = a.kmin + (int64_t)(r.x & kKeyMask);
          ordg = (int64_t)r.y + a.obase;
          tsg = (int64_t)r.w + a.ts0;
          row = cc.row_of(r.y);
        } else {
          row = base + luq;
          ordg = a.ord ? a.ord[row] : a.obase + row;
          tsg = L.t[luq];
        }
        if (cb < a.cand_cap) {
          int64_t* c = a.cand + 4 * (int64_t)cb;
          c[0] = key;
          c[1] = ordg;
          c[2] = tsg;
          c[3] = row;
        } else {
          atomicOr(a.err, 1u);
        }
        ++cb;
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
    lds_barrier();
    SM_STAMP(5);
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
          jo = jv < (uint32_t)lend ? L.r[jv].y : ((const uint32_t*)(a.rec + base + jv))[1];
          io = L.r[luq].y;
        } else {
          const int64_t vj = base + jv, ui = base + luq;
          jo = a.ord ? (uint32_t)(a.ord[vj] - a.obase) : (uint32_t)vj;
          io = a.ord ? (uint32_t)(a.ord[ui] - a.obase) : (uint32_t)ui;
        }
        stq[pos] = ((uint64_t)jo << 32) | io;
        atomicAdd(&jh[jo & (kBins - 1)], 1u);
      }
      ob += (uint32_t)__popcll(bal);
    }
    lds_barrier();  // every wave read sh_run / wtot
    if (threadIdx.x == 0) sh_run += tot;
    SM_STAMP(6);
  }
  SM_STAMP_FLUSH;
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
void launch_walk_t(int G, hipStream_t s, const WalkArgs& wa, int64_t per, uint64_t* stq, uint32_t* mcount,
                   uint32_t* jcnt) {
  hipLaunchKernelGGL((walk_kernel<KEYED, OP, FP>), dim3(G), dim3(kWalkBlock), 0, s, wa, per, G, stq, mcount, jcnt);
}

template <bool KEYED>
void launch_walk(int spec, int G, hipStream_t s, const WalkArgs& wa, int64_t per, uint64_t* stq, uint32_t* mcount,
                 uint32_t* jcnt) {
#define SM_WALK(OP, FP) launch_walk_t<KEYED, OP, FP>(G, s, wa, per, stq, mcount, jcnt)
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
    default:
      if constexpr (KEYED) throw std::logic_error("keyed walk needs a compare spec");
      else SM_WALK(-1, false);
      break;
  }
#undef SM_WALK
}

// ---------------------------------------------------------------- j order by output tiles (round 6)
// The unkeyed walk leaves its (j << 32) | i pairs chunk by chunk in i order; the output wants (j, i) order (the
// reference emits at e2's arrival, the partials it completes oldest first). A match's j is at most D ordinals after
// its i, and in the config-3 shape D is small (`within 1 sec` over one event per ms: D <= 1000). Then the pairs whose
// j falls in an output tile of kJtTile ordinals all have i in [tile start - D, tile end): one workgroup per tile reads
// that i range (binary search in the walk chunks that cover it), keeps the pairs whose j is in the tile, and places
// them by a stable counting sort on j in LDS, i order kept within a j. That replaces the LSD j passes (an up-sweep and
// a scatter of every pair per 10 bits of j) with one count pass and one read of about (kJtTile + D) / kJtTile of the
// pairs. Batches with D > kJtDMax, or a tile with more than kJtCap pairs, keep the LSD passes.
constexpr int kJtB = 11;
constexpr uint32_t kJtTile = 1u << kJtB;  // output ordinals per tile
constexpr uint32_t kJtCap = 4096;         // pairs a tile's workgroup holds in LDS
constexpr uint32_t kJtDMax = 4 * kJtTile;
constexpr int kJtThreads = 256;

// Pairs per output tile (cnt[t], t = j >> kJtB, runs of equal tiles within a wave counted once), the largest j - i,
// and where each i-tile's pairs start: P[u] = the staging index of the first pair with i >= u * kJtTile, for the
// tiles whose first ordinal falls in this chunk's ordinal range [ord of its first event, ord of the next chunk's)
// (ordinals rise with the batch position, so the chunks' ranges partition the ordinals; a tile with no pair in its
// chunk points at the chunk's end). A tile's workgroup then finds its input with two loads instead of searches.
__global__ void __launch_bounds__(1024) jt_count_kernel(const uint64_t* __restrict__ stq,
                                                       const uint32_t* __restrict__ mcount, int64_t perw, int Gw,
                                                       const int64_t* __restrict__ ord, int64_t obase, int64_t n,
                                                       uint32_t T, uint32_t* __restrict__ cnt,
                                                       uint32_t* __restrict__ dmax, uint32_t* __restrict__ P) {
  constexpr uint32_t kLoc = 256;  // output tiles from the chunk's first one counted in LDS, flushed once
  __shared__ uint32_t lcnt[kLoc];
  const int g = blockIdx.x, lane = threadIdx.x & 63;
  const int64_t p0 = (int64_t)g * perw, p1 = p0 + perw;
  if (p0 >= n) return;
  for (uint32_t x = threadIdx.x; x < kLoc; x += blockDim.x) lcnt[x] = 0;
  __syncthreads();
  auto ord_at = [&](int64_t p) { return ord ? (uint32_t)(ord[p] - obase) : (uint32_t)p; };
  const uint32_t c0 = ord_at(p0);
  const uint32_t tbase = c0 >> kJtB;  // a pair's e2 is after its e1: no tile below this one
  const uint32_t u_first = (c0 + kJtTile - 1) >> kJtB;  // tiles whose first ordinal is in this chunk's range
  const uint32_t u_end = p1 < n ? (ord_at(p1) + kJtTile - 1) >> kJtB : T;
  const uint64_t* q = stq + p0;
  const uint32_t m = mcount[g];
  const uint32_t xbase = (uint32_t)p0;
  if (g == 0 && threadIdx.x == 0) P[T] = (uint32_t)((int64_t)Gw * perw < 0xffffffffll ? Gw * perw : 0xffffffffll);
  if (m == 0) {
    for (uint32_t u = u_first + threadIdx.x; u < u_end; u += blockDim.x) P[u] = xbase;
    return;  // (uniform: nothing was counted)
  }
  uint32_t dm = 0;
  constexpr int kLd = 8;  // pairs per thread whose loads are in flight together
  for (uint32_t b0 = (threadIdx.x >> 6) * 64u; b0 < m; b0 += blockDim.x * kLd) {
    uint64_t vv[kLd];
#pragma unroll
    for (int r = 0; r < kLd; ++r) {
      const uint32_t k = b0 + r * blockDim.x + lane;
      vv[r] = k < m ? q[k] : 0ull;
    }
#pragma unroll
    for (int r = 0; r < kLd; ++r) {
    const uint32_t b = b0 + r * blockDim.x;
    const uint32_t k = b + lane;
    const bool valid = k < m;
    const uint64_t v = vv[r];
    const uint32_t j = (uint32_t)(v >> 32), i = (uint32_t)v;
    if (valid && j - i > dm) dm = j - i;
    const uint32_t t = valid ? j >> kJtB : 0xffffffffu;
    const uint32_t tp = __shfl_up(t, 1, 64);
    const bool head = valid && (lane == 0 || t != tp);
    const uint64_t hm = __ballot(head);
    const uint32_t nv = (uint32_t)__popcll(__ballot(valid));
    const uint64_t after = lane == 63 ? 0ull : hm >> (lane + 1);
    const uint32_t next = after ? (uint32_t)lane + 1u + (uint32_t)__builtin_ctzll(after) : nv;
    if (head) {
      if (t - tbase < kLoc) atomicAdd(&lcnt[t - tbase], next - (uint32_t)lane);
      else atomicAdd(&cnt[t], next - (uint32_t)lane);
    }
    const uint32_t ip = __shfl_up(i, 1, 64);  // the previous pair's i (lane 0: from memory)
    if (valid) {  // i-tiles that start after the previous pair's i and at or before this one's: they start here
      const uint32_t ui = i >> kJtB;
      const uint32_t up = k == 0 ? u_first : (((lane == 0 ? (uint32_t)q[k - 1] : ip)) >> kJtB) + 1u;
      for (uint32_t u = up > u_first ? up : u_first; u <= ui && u < u_end; ++u) P[u] = xbase + k;
      if (k == m - 1)
        for (uint32_t u = (ui + 1 > u_first ? ui + 1 : u_first); u < u_end; ++u) P[u] = xbase + m;
    }
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t x = __shfl_xor(dm, o, 64);
    dm = x > dm ? x : dm;
  }
  if (lane == 0) atomicMax(dmax, dm);
  __syncthreads();
  for (uint32_t x = threadIdx.x; x < kLoc; x += blockDim.x)
    if (lcnt[x] && tbase + x < T) atomicAdd(&cnt[tbase + x], lcnt[x]);
}

// output tile blockIdx.x: off[t] = pairs before the tile (exclusive scan of the counts over T + 1 entries); its input
// is the staging range [P[i-tile of t0 - D], P[t + 1]), walk chunk by chunk (pairs at [g perw, g perw + mcount[g]))
constexpr int kJtLd = 8;  // staged pairs per thread and load round (their loads are in flight together)
__global__ void __launch_bounds__(kJtThreads) jt_place_kernel(const uint64_t* __restrict__ stq,
                                                              const uint32_t* __restrict__ mcount, int64_t perw,
                                                              const uint32_t* __restrict__ P,
                                                              const uint32_t* __restrict__ off, uint32_t D,
                                                              uint64_t* __restrict__ out, uint32_t* __restrict__ err) {
  constexpr int kJtW = kJtThreads / 64;
  __shared__ uint64_t a[kJtCap];
  __shared__ __attribute__((aligned(4))) uint16_t cw[kJtW][kJtTile];  // per (wave, j): count, then cursor
  __shared__ uint32_t wsum[kJtThreads / 64];
  __shared__ uint32_t wrc[kJtLd][kJtThreads / 64];
  __shared__ uint32_t s_n;
  const int t = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t K = off[t + 1] - off[t];
  if (K == 0) return;
  if (K > kJtCap) {  // the whole batch takes the LSD passes
    if (tid == 0) atomicOr(err, 1u);
    return;
  }
  const uint32_t t0 = (uint32_t)t << kJtB, t1 = t0 + kJtTile;
  const uint32_t lo_i = t0 > D ? t0 - D : 0u;
  const uint32_t x0 = P[lo_i >> kJtB], x1 = P[t + 1];
  for (uint32_t x = tid; x < kJtW * kJtTile / 2; x += kJtThreads) ((uint32_t*)&cw[0][0])[x] = 0;
  if (tid == 0) s_n = 0;
  const uint64_t lt = lanemask_lt();
  lds_barrier();
  for (uint32_t g = x0 / (uint32_t)perw; x0 < x1 && g <= (x1 - 1) / (uint32_t)perw; ++g) {
    const uint32_t gb = g * (uint32_t)perw;
    const uint32_t b0 = x0 > gb ? x0 - gb : 0u;
    const uint32_t m = mcount[g];
    const uint32_t b1 = x1 - gb < m ? x1 - gb : m;
    const uint64_t* q = stq + gb;
    for (uint32_t b = b0; b < b1; b += kJtThreads * kJtLd) {  // the tile's pairs, compacted in i order
      uint64_t v[kJtLd];
#pragma unroll
      for (int r = 0; r < kJtLd; ++r) {
        const uint32_t k = b + r * kJtThreads + tid;
        v[r] = k < b1 ? q[k] : 0ull;
      }
      // the round's selected pairs in (r, wave, lane) order = i order: per (r, wave) counts, then one prefix
      uint64_t bal[kJtLd];
#pragma unroll
      for (int r = 0; r < kJtLd; ++r) {
        const uint32_t k = b + r * kJtThreads + tid;
        const uint32_t j = (uint32_t)(v[r] >> 32);
        bal[r] = __ballot(k < b1 && j >= t0 && j < t1);
        if (lane == 0) wrc[r][w] = (uint32_t)__popcll(bal[r]);
      }
      lds_barrier();
      uint32_t run = s_n;
#pragma unroll
      for (int r = 0; r < kJtLd; ++r) {
        uint32_t o = run;
#pragma unroll
        for (int x = 0; x < kJtThreads / 64; ++x) {
          if (x < w) o += wrc[r][x];
          run += wrc[r][x];
        }
        if ((bal[r] >> lane) & 1ull) {
          const uint32_t idx = o + (uint32_t)__popcll(bal[r] & lt);
          if (idx < kJtCap) a[idx] = v[r];
        }
      }
      lds_barrier();  // every thread read s_n and the counts
      if (tid == 0) s_n = run;
      lds_barrier();
    }
  }
  if (s_n != K) {  // the counts and the tile's pairs disagree: never expected; the LSD passes take the batch
    if (tid == 0) atomicOr(err, 2u);
    return;
  }
  // stable placement by all waves: wave w takes the quarter [q0, q1) of the tile's pairs; per (wave, j) counts, then
  // per (wave, j) cursors = j's start + the counts of the earlier quarters, so each wave places its pairs after every
  // earlier pair of the same j
  const uint32_t q0 = (uint32_t)(((uint64_t)K * (uint32_t)w) / kJtW);
  const uint32_t q1 = (uint32_t)(((uint64_t)K * (uint32_t)(w + 1)) / kJtW);
  uint32_t* cw32 = (uint32_t*)&cw[0][0];
  for (uint32_t x = q0 + lane; x < q1; x += 64) {
    const uint32_t jo = (uint32_t)(a[x] >> 32) - t0;
    atomicAdd(&cw32[w * (kJtTile / 2) + (jo >> 1)], 1u << (16 * (jo & 1)));
  }
  lds_barrier();
  {  // thread tid owns kPer consecutive j's: totals, block scan, per-wave cursors
    constexpr int kPer = kJtTile / kJtThreads;
    uint32_t tot[kPer], s = 0;
#pragma unroll
    for (int x = 0; x < kPer; ++x) {
      const uint32_t jo = tid * kPer + x;
      tot[x] = 0;
#pragma unroll
      for (int v = 0; v < kJtW; ++v) tot[x] += cw[v][jo];
      s += tot[x];
    }
    uint32_t inc = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(inc, o, 64);
      if (lane >= o) inc += u;
    }
    if (lane == 63) wsum[w] = inc;
    lds_barrier();
    uint32_t base = inc - s;
    for (int x = 0; x < w; ++x) base += wsum[x];
#pragma unroll
    for (int x = 0; x < kPer; ++x) {
      const uint32_t jo = tid * kPer + x;
      uint32_t st = base;
#pragma unroll
      for (int v = 0; v < kJtW; ++v) {
        const uint32_t c = cw[v][jo];
        cw[v][jo] = (uint16_t)st;
        st += c;
      }
      base += tot[x];
    }
  }
  lds_barrier();
  uint64_t* o = out + off[t];
  for (uint32_t b = q0; b < q1; b += 64) {
    const uint32_t k = b + lane;
    const bool valid = k < q1;
    const uint64_t v = valid ? a[k] : 0ull;
    const uint32_t jo = valid ? (uint32_t)(v >> 32) - t0 : 0u;
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int bb = 0; bb < kJtB; ++bb) {
      const uint64_t bl = __ballot((jo >> bb) & 1u);
      peers &= ((jo >> bb) & 1u) ? bl : ~bl;
    }
    const uint32_t below = (uint32_t)__popcll(peers & lt);
    const uint32_t c = valid ? (uint32_t)cw[w][jo] : 0u;
    wave_lockstep();
    if (valid && below == 0) cw[w][jo] = (uint16_t)(c + (uint32_t)__popcll(peers));
    wave_lockstep();
    if (valid) o[c + below] = v;
  }
}

// j order by tiles: on by default; SM_JTILE=0 keeps the LSD passes (A/B and tests; read per batch)
bool jtile_on() {
  const char* e = getenv("SM_JTILE");
  return !(e && e[0] == '0');
}

// record passes with the write-combining down-sweep (SM_SORT_WC=0 selects the plain one, for comparison)
bool sort_wc() {
  static const bool on = [] {
    const char* e = getenv("SM_SORT_WC");
    return !(e && e[0] == '0');
  }();
  return on;
}

// pair (j-order) passes with the write-combining down-sweep: SM_JPASS_WC=1 for the passes after the first,
// 2 for all of them, 0 (default) none
int jpass_wc() {
  static const int v = [] {
    const char* e = getenv("SM_JPASS_WC");
    return e ? atoi(e) : 0;
  }();
  return v;
}

// c1 reads only the compared attribute (slot-0 variables / stream columns of vattr): evaluated in pass 0
bool c1_inline(const FastHostInfo& hi, const FastArgs& a) {
  if (!hi.c1_host || hi.c1_len != a.c1_len) return false;
  if (hi.c1_len != 0) {  // the device side evaluates `x CMP y` (make_cond's simple form) only
    const Instr* c = hi.c1_host;
    auto leaf = [](const Instr& in) { return in.op != OP_CMP && in.op != OP_MATH && in.op != OP_NOT; };
    if (hi.c1_len != 3 || c[2].op != OP_CMP || !leaf(c[0]) || !leaf(c[1])) return false;
  }
  for (int k = 0; k < hi.c1_len; ++k) {
    const Instr& in = hi.c1_host[k];
    if (in.op == OP_TS) return false;
    if (in.op == OP_VAR && (in.a != 0 || in.c != hi.vattr)) return false;
    if (in.op == OP_COL && in.a != hi.vattr) return false;
  }
  return true;
}

template <typename KT, typename VT>
void launch_down0_t(const FastHostInfo& hi, const FastArgs& a, const void* kcol, int64_t kmin, int vmode, int64_t vmin,
                    const uint64_t* c1mask, int64_t ts0, int G, int64_t per, hipStream_t s, uint4* dst,
                    const uint32_t* cnt, const uint32_t* dbase) {
  OrigSrc<KT, VT> os{a.st, (const KT*)kcol, (const VT*)hi.cols[hi.vattr], kmin, vmode, vmin, c1mask, a.ts, ts0,
                     a.ordinals, a.ordinal_base, a.code + a.c1_off, a.c1_len, a.consts, c1_inline(hi, a)};
  static const bool p0v2 = !(getenv("SM_PASS0_V2") && getenv("SM_PASS0_V2")[0] == '0');
  if (sort_wc() && p0v2)  // pass0_dev.h (A/B: SM_PASS0_V2=0 runs the generic write-combining down-sweep)
    hipLaunchKernelGGL((pass0_kernel<OrigSrc<KT, VT>>), dim3(G), dim3(kP0Block), 0, s, os, dst, a.n, per, G, cnt, dbase);
  else if (sort_wc())
    hipLaunchKernelGGL((downsweep_wc_kernel<0, OrigSrc<KT, VT>>), dim3(G), dim3(kWcBlock), 0, s, os, dst, nullptr, a.n,
                       per, nullptr, G, 0, cnt, dbase);
  else
    hipLaunchKernelGGL((downsweep_kernel<0, OrigSrc<KT, VT>>), dim3(G), dim3(kBlock), 0, s, os, dst, nullptr, a.n, per,
                       nullptr, G, 0, cnt, dbase);
}

template <typename KT>
void launch_down0_k(const FastHostInfo& hi, const FastArgs& a, const void* kcol, int64_t kmin, int vmode, int64_t vmin,
                    const uint64_t* m, int64_t ts0, int G, int64_t per, hipStream_t s, uint4* dst,
                    const uint32_t* cnt, const uint32_t* dbase) {
  switch (hi.vtype) {
    case T_INT: launch_down0_t<KT, int32_t>(hi, a, kcol, kmin, vmode, vmin, m, ts0, G, per, s, dst, cnt, dbase); break;
    case T_LONG: launch_down0_t<KT, int64_t>(hi, a, kcol, kmin, vmode, vmin, m, ts0, G, per, s, dst, cnt, dbase); break;
    case T_FLOAT: launch_down0_t<KT, float>(hi, a, kcol, kmin, vmode, vmin, m, ts0, G, per, s, dst, cnt, dbase); break;
    case T_DOUBLE: launch_down0_t<KT, double>(hi, a, kcol, kmin, vmode, vmin, m, ts0, G, per, s, dst, cnt, dbase); break;
    default: throw std::runtime_error("fast path: unsupported compared-attribute type");
  }
}

int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

// ---- carried partials on the walk pipeline

struct ResolveArgs {
  const int64_t* crow;  // carry rows [key, ordinal, ts, values...]
  int64_t nc;
  int w, vattr, vtype, vmode;
  int64_t vmin;
  bool exact_codes;
  const uint4* rec;  // keyed: records sorted by key
  const NfaStream* st;
  const int64_t* ts;
  const int64_t* ord;
  int64_t obase, n, kmin, span, ts0, within;
  uint64_t* cpair;  // per carried partial: (j << 32) | (e1 ordinal - base), or ~0
  int64_t* cand;
  uint32_t* cand_n;
  uint32_t cand_cap;
  uint32_t* err;
};

// One thread per carried partial: the first event of its key in this batch that matches it (reference:
// processAndReturn over the pending list, StreamPreStateProcessor.java:274-327), finds it expired (dropped), or
// none (still pending: carry-out candidate).
template <bool KEYED, int OP, bool FP>
__global__ void resolve_kernel(ResolveArgs r) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= r.nc) return;
  const int64_t* row = r.crow + i * r.w;
  const int64_t key = row[0], oc = row[1], tc = row[2];
  const StackVal vc = uncanon((uint64_t)row[3 + r.vattr], r.vtype);
  r.cpair[i] = ~0ull;
  if (oc - r.obase < INT32_MIN) atomicOr(r.err, 2u);  // not expressible as a 32-bit relative ordinal
  auto pending = [&]() {
    const uint32_t q = atomicAdd(r.cand_n, 1u);
    if (q < r.cand_cap) {
      int64_t* c = r.cand + 4 * (int64_t)q;
      c[0] = key;
      c[1] = oc;
      c[2] = tc;
      c[3] = -i - 1;
    } else {
      atomicOr(r.err, 1u);
    }
  };
  int64_t p = 0, kr = 0;
  uint32_t code = 0;
  if constexpr (KEYED) {
    kr = key - r.kmin;
    if (kr < 0 || kr > r.span) {  // no event of this key in the batch
      pending();
      return;
    }
    int64_t lo = 0, hi = r.n;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if ((int64_t)(r.rec[mid].x & kKeyMask) < kr) lo = mid + 1;
      else hi = mid;
    }
    p = lo;
    switch (r.vtype) {
      case T_INT: code = vcode<int32_t>((int32_t)vc.i, r.vmode, r.vmin); break;
      case T_LONG: code = vcode<int64_t>(vc.i, r.vmode, r.vmin); break;
      case T_FLOAT: code = vcode<float>((float)vc.d, r.vmode, r.vmin); break;
      default: code = vcode<double>(vc.d, r.vmode, r.vmin); break;
    }
  }
  for (; p < r.n; ++p) {
    int64_t tj, rowj = p;
    uint32_t oj, cj = 0;
    if constexpr (KEYED) {
      const uint4 e = r.rec[p];
      if ((int64_t)(e.x & kKeyMask) != kr) break;
      tj = (int64_t)e.w + r.ts0;
      oj = e.y;
      cj = e.z;
      rowj = -1;
    } else {
      tj = r.ts[p];
      oj = r.ord ? (uint32_t)(r.ord[p] - r.obase) : (uint32_t)p;
    }
    const int64_t dt = tj - tc;
    if (r.within >= 0 && (dt < 0 ? -dt : dt) > r.within) return;  // expired at this event: dropped
    bool hit;
    const bool nan = FP & ((code == kNanCode) | (cj == kNanCode));
    if (KEYED && !nan && (r.exact_codes || code != cj)) {
      hit = cmp_fixed<OP>(cj, code);
    } else {
      if (rowj < 0) {  // keyed: the row of ordinal oj
        rowj = oj;
        if (r.ord) {
          const int64_t want = (int64_t)oj + r.obase;
          int64_t lo = 0, hi = r.n - 1;
          while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (r.ord[mid] < want) lo = mid + 1;
            else hi = mid;
          }
          rowj = lo;
        }
      }
      const StackVal vj = col_value(r.st, r.vattr, rowj);
      if constexpr (FP) hit = cmp_fixed<OP>(vj.d, vc.d);
      else hit = cmp_fixed<OP>(vj.i, vc.i);
    }
    if (hit) {
      r.cpair[i] = ((uint64_t)oj << 32) | (uint32_t)(oc - r.obase);
      return;
    }
  }
  pending();
}

template <bool KEYED, int OP, bool FP>
void launch_resolve_t(const ResolveArgs& r, hipStream_t s) {
  hipLaunchKernelGGL((resolve_kernel<KEYED, OP, FP>), dim3((unsigned)((r.nc + 255) / 256)), dim3(256), 0, s, r);
}

void launch_resolve(bool keyed, int spec, const ResolveArgs& r, hipStream_t s) {
#define SM_RES(OP, FP) (keyed ? launch_resolve_t<true, OP, FP>(r, s) : launch_resolve_t<false, OP, FP>(r, s))
  switch (spec) {
    case CMP_EQ * 2: SM_RES(CMP_EQ, false); break;
    case CMP_EQ * 2 + 1: SM_RES(CMP_EQ, true); break;
    case CMP_NE * 2: SM_RES(CMP_NE, false); break;
    case CMP_NE * 2 + 1: SM_RES(CMP_NE, true); break;
    case CMP_LT * 2: SM_RES(CMP_LT, false); break;
    case CMP_LT * 2 + 1: SM_RES(CMP_LT, true); break;
    case CMP_LE * 2: SM_RES(CMP_LE, false); break;
    case CMP_LE * 2 + 1: SM_RES(CMP_LE, true); break;
    case CMP_GT * 2: SM_RES(CMP_GT, false); break;
    case CMP_GT * 2 + 1: SM_RES(CMP_GT, true); break;
    case CMP_GE * 2: SM_RES(CMP_GE, false); break;
    case CMP_GE * 2 + 1: SM_RES(CMP_GE, true); break;
    default: throw std::logic_error("carried partials need a fixed compare");
  }
#undef SM_RES
}

__global__ void pair_flag_kernel(const uint64_t* __restrict__ cp, int64_t n, uint32_t* __restrict__ f) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) f[i] = cp[i] != ~0ull ? 1u : 0u;
}

// sign-flipped e1 word: (j, e1) sorts in signed e1 order (a carried e1 may lie before the ordinal base)
__global__ void pair_compact_kernel(const uint64_t* __restrict__ cp, const uint32_t* __restrict__ pos, int64_t n,
                                    uint64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && cp[i] != ~0ull) out[pos[i]] = cp[i] ^ 0x80000000ull;
}

// merge of the walk's (j, i)-ordered pairs with the carried partials' pairs (also (j, i)-ordered); for equal j the
// carried ones (older e1) come first
__global__ void merge_main_kernel(const uint64_t* __restrict__ mq, int64_t m, const uint64_t* __restrict__ cq,
                                  int64_t mc, uint64_t* __restrict__ out) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= m) return;
  const uint64_t v = mq[k];
  const uint32_t j = (uint32_t)(v >> 32);
  int64_t lo = 0, hi = mc;  // carried pairs with j_c <= j
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((uint32_t)(cq[mid] >> 32) <= j) lo = mid + 1;
    else hi = mid;
  }
  out[k + lo] = v;
}

__global__ void merge_carried_kernel(const uint64_t* __restrict__ cq, int64_t mc, const uint64_t* __restrict__ mq,
                                     int64_t m, uint64_t* __restrict__ out) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= mc) return;
  const uint64_t v = cq[k] ^ 0x80000000ull;
  const uint32_t j = (uint32_t)(v >> 32);
  int64_t lo = 0, hi = m;  // walk pairs with j_w < j
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((uint32_t)(mq[mid] >> 32) < j) lo = mid + 1;
    else hi = mid;
  }
  out[k + lo] = v;
}

}  // namespace

// Returns -1 when the batch is outside the v2 envelope (caller takes the general path).
int64_t fast_every_within_v2(const FastArgs& a, const FastHostInfo& hi, FastState& fs, FastCarry& carry,
                             uint32_t* pairs_out, int64_t pairs_cap, Scratch& sc, hipStream_t s, FastTimings* tm,
                             int stack_mode) {
  const int64_t n = a.n;
  if (n == 0) return 0;
  if (n >= 0x7fffffffll || hi.vattr < 0) return FAST_OUTSIDE;
  const bool keyed = a.key != nullptr;
  if (keyed && (hi.key_col < 0 || !(hi.key_type == T_INT || hi.key_type == T_LONG))) return FAST_OUTSIDE;
  const int spec = c2_spec(hi);
  if (keyed && spec < 0) return FAST_OUTSIDE;  // keyed records carry value codes: fixed compares only
  if (carry.n > 0 && spec < 0) return FAST_OUTSIDE;
  size_t mark = sc.used;
  auto bail = [&]() -> int64_t {
    sc.used = mark;
    return FAST_OUTSIDE;
  };
  Ctrl* c = (Ctrl*)sc.take(sizeof(Ctrl));
  {
    Ctrl init{};
    init.kmin = ~0ull;
    init.vmin = ~0ull;
    SM_HIP(hipMemcpyAsync(c, &init, sizeof(Ctrl), hipMemcpyHostToDevice, s));
  }
  const void* kcol = keyed ? (hi.dense_keys ? (const void*)hi.dense_keys : hi.cols[hi.key_col]) : nullptr;
  const int key_type = hi.dense_keys ? T_INT : hi.key_type;
  const int64_t* vlong = (keyed && hi.vtype == T_LONG) ? (const int64_t*)hi.cols[hi.vattr] : nullptr;
  if (tm) {
    SM_HIP(hipEventRecord(tm->ev[0], s));
    tm->nmk = 0;
    tm->mark("start", s);
  }
  auto tmark = [&](const char* l) {
    if (tm) tm->mark(l, s);
  };

  // persistent chunking: G workgroups (as many as the down-sweep keeps resident), chunks of whole sort tiles
  if (fs.cus == 0) {
    int dev = 0;
    SM_HIP(hipGetDevice(&dev));
    SM_HIP(hipDeviceGetAttribute(&fs.cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  if (fs.sort_wgs_per_cu == 0) {
    int b = 0;
    if (sort_wc()) SM_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, downsweep_wc_kernel<1, RecSrc>, kWcBlock, 0));
    else SM_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, downsweep_kernel<1, RecSrc>, kBlock, 0));
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
  uint64_t* c1mask = (uint64_t*)sc.take(((n + 63) / 64) * 8);
  auto scan_counts = [&](int g) {
    hipLaunchKernelGGL(scan_chunks_kernel, dim3(kBins), dim3(256), 0, s, cnt, g, dbase);
    hipLaunchKernelGGL(digit_base_kernel, dim3(1), dim3(kBlock), 0, s, dbase);
    tmark("scan");
  };

  // column facts + c1 mask + pass-0 digit counts, one pass
  const bool mask = !keyed || !c1_inline(hi, a);
#define SM_PREP2(KT, M, X)                                                                                          \
  hipLaunchKernelGGL((prep_kernel<KT, M, X>), dim3(G), dim3(kBlock), 0, s, (const KT*)kcol, vlong, a.ts, a.ordinals, \
                     a.ordinal_base, n, per, G, a.st, a.code + a.c1_off, a.c1_len, a.consts, c1mask, cnt, c)
#define SM_PREP(KT, M)                  \
  do {                                  \
    if (a.ordinals || vlong)            \
      SM_PREP2(KT, M, true);            \
    else                                \
      SM_PREP2(KT, M, false);           \
  } while (0)
  if (key_type == T_LONG && keyed) {
    if (mask) SM_PREP(int64_t, true);
    else SM_PREP(int64_t, false);
  } else {
    if (mask) SM_PREP(int32_t, true);
    else SM_PREP(int32_t, false);
  }
#undef SM_PREP
#undef SM_PREP2
  tmark("prep");
  Ctrl hc;
  SM_HIP(hipMemcpyAsync(&hc, c, sizeof(Ctrl), hipMemcpyDeviceToHost, s));
  SM_HIP(hipStreamSynchronize(s));
  if (a.within >= 0) {
    // the closed form needs non-decreasing event time, inside the batch and after the carried state
    if (hc.bad_ts || (carry.active && hc.ts0 < carry.ts_last)) {
      sc.used = mark;
      return FAST_NON_MONOTONE;
    }
    if ((unsigned long long)(hc.ts_last - hc.ts0) >= 0xffffffffull) return bail();
  }
  if (hc.omax >= 0x7fffffffull || hc.bad_ord) return bail();
  int kbits = 0;
  int64_t kmin = 0;
  uint64_t kspan = 0;
  if (keyed) {
    kmin = (int64_t)(hc.kmin ^ 0x8000000000000000ull);
    kmin &= ~(int64_t)(kBins - 1);  // rebase on a digit boundary (prep counted digit 0 of the raw key)
    kspan = (uint64_t)((int64_t)(hc.kmax ^ 0x8000000000000000ull) - kmin);
    kbits = std::max(1, bits_for(kspan));
    if (kbits > 30 || (hi.remap_span > 0 && kspan > (uint64_t)hi.remap_span)) {
      sc.used = mark;
      return FAST_KEY_SPAN;
    }
  }
  // value code of the compared attribute
  int vmode = VC_I32;
  int64_t vmin = 0;
  bool exact_codes = true;
  switch (hi.vtype) {
    case T_INT: vmode = VC_I32; break;
    case T_FLOAT: vmode = VC_F32; break;
    case T_DOUBLE: vmode = VC_F64; exact_codes = false; break;
    default:
      // rebased codes need every compared value (carried partials too) inside the batch's range
      if (keyed && carry.n == 0 && hc.vmax - hc.vmin <= 0xffffffffull) {
        vmode = VC_I64R;
        vmin = (int64_t)(hc.vmin ^ 0x8000000000000000ull);
      } else {
        vmode = VC_I64H;
        exact_codes = false;
      }
  }
  const int fpass = keyed ? (kbits + kRB - 1) / kRB : 0;
  const int jbits = std::max(1, bits_for(hc.omax));
  const int jpass = (jbits + kRB - 1) / kRB;
  auto finish = [&](int64_t m) {
    carry.ts_last = carry.active ? std::max<int64_t>(carry.ts_last, hc.ts_last) : (int64_t)hc.ts_last;
    carry.active = true;
    sc.used = mark;
    return m;
  };

  uint64_t* stq = nullptr;                // walk staging (chunk-local compaction), (j << 32) | i
  uint64_t *pq = nullptr, *qq = nullptr;  // j-sort ping-pong
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
  wa.exact_codes = exact_codes;
  wa.c1mask = c1mask;
  wa.kmin = kmin;
  wa.ts0 = hc.ts0;
  // carry-out candidates of the walk pipeline: pending partials of the batch + carried ones still pending
  const int64_t nc = carry.n;
  const int64_t cand_cap = std::min<int64_t>(n + nc, (int64_t)1 << 26) + 1024;
  uint32_t* cflags = (uint32_t*)sc.take(16);  // [0] candidates, [1] overflow
  SM_HIP(hipMemsetAsync(cflags, 0, 16, s));
  int64_t* cand = nullptr;
  uint4* cur = nullptr;
  if (keyed) {
    uint4* A = (uint4*)sc.take(n * 16);
    uint4* B = (uint4*)sc.take(n * 16);
    // key pass 0 from the original columns (its digit counts came from prep)
    scan_counts(G);
    if (key_type == T_INT)
      launch_down0_k<int32_t>(hi, a, kcol, kmin, vmode, vmin, c1mask, hc.ts0, G, per, s, A, cnt, dbase);
    else launch_down0_k<int64_t>(hi, a, kcol, kmin, vmode, vmin, c1mask, hc.ts0, G, per, s, A, cnt, dbase);
    tmark("key_pass0");
    // bucket-stack pipeline when the per-bucket keys fill a workgroup (stack.hip); it falls back here otherwise
    const int H = (int)std::min<uint64_t>(kspan >> kRB, 1ull << 20) + 1;
    const bool order_op = spec >= 0 && (spec >> 1) != CMP_EQ && (spec >> 1) != CMP_NE;
    const bool ts_ok = a.within < 0 || (a.within < (1ll << 30) && hc.ts_last - hc.ts0 < (1ll << 30));
    if (stack_mode != 2 && order_op && ts_ok && H <= kBins && (stack_mode == 1 || H >= kBins / 2)) {
      StackPlan sp{};
      sp.rec = A;
      sp.dbase = dbase;
      sp.n = n;
      sp.omax = (int64_t)hc.omax;
      sp.H = H;
      sp.kmin = kmin;
      sp.op = spec >> 1;
      sp.fp = (spec & 1) != 0;
      sp.exact_codes = exact_codes;
      sp.vtype = hi.vtype;
      sp.vattr = hi.vattr;
      sp.vmode = vmode;
      sp.vmin = vmin;
      sp.vcol = hi.cols[hi.vattr];
      sp.within = a.within;
      sp.ts0 = hc.ts0;
      sp.ts_last = hc.ts_last;
      sp.o0 = (int32_t)hc.o0;
      const int64_t m = stack_pipeline(sp, a, hi, fs, carry, pairs_out, pairs_cap, sc, s, tm);
      if (m >= 0) {
        fs.last_path = 3;
        if (tm) {
          SM_HIP(hipEventRecord(tm->ev[1], s));
          SM_HIP(hipEventRecord(tm->ev[2], s));
          SM_HIP(hipEventRecord(tm->ev[3], s));
        }
        return finish(m);
      }
    }
    cand = (int64_t*)sc.take((size_t)cand_cap * 32);
    cur = A;
    uint4* nxt = B;
    for (int p = 1; p < fpass; ++p) {
      hipLaunchKernelGGL((upsweep_kernel<RecDigits>), dim3(G), dim3(kBlock), 0, s, RecDigits{cur}, n, per, G,
                         p * kRB, cnt);
      tmark("key_up");
      scan_counts(G);
      if (sort_wc())
        hipLaunchKernelGGL((downsweep_wc_kernel<1, RecSrc>), dim3(G), dim3(kWcBlock), 0, s, RecSrc{cur}, nxt, nullptr, n,
                           per, nullptr, G, p * kRB, cnt, dbase);
      else
        hipLaunchKernelGGL((downsweep_kernel<1, RecSrc>), dim3(G), dim3(kBlock), 0, s, RecSrc{cur}, nxt, nullptr, n,
                           per, nullptr, G, p * kRB, cnt, dbase);
      tmark("key_pass");
      std::swap(cur, nxt);
    }
    if (tm) SM_HIP(hipEventRecord(tm->ev[1], s));
    wa.rec = cur;
    wa.cand = cand;
    wa.cand_n = cflags;
    wa.cand_cap = (uint32_t)cand_cap;
    wa.err = cflags + 1;
    // staging + one ping-pong buffer in the dead record buffer (2 x 8n of its 16n bytes); the other in `cur`
    // once the walk is done
    stq = (uint64_t*)nxt;
    pq = (uint64_t*)nxt + n;
    qq = (uint64_t*)cur;
    launch_walk<true>(spec, Gw, s, wa, perw, stq, mcount, cnt);
  } else {
    if (tm) SM_HIP(hipEventRecord(tm->ev[1], s));
    cand = (int64_t*)sc.take((size_t)cand_cap * 32);
    wa.cand = cand;
    wa.cand_n = cflags;
    wa.cand_cap = (uint32_t)cand_cap;
    wa.err = cflags + 1;
    stq = (uint64_t*)sc.take(n * 8);
    pq = (uint64_t*)sc.take(n * 8);
    qq = (uint64_t*)sc.take(n * 8);
    launch_walk<false>(spec, Gw, s, wa, perw, stq, mcount, cnt);
  }
  fs.last_path = 2;
  tmark("walk");
  // j order by output tiles (unkeyed walk, jt_place_kernel): pairs per tile and the largest j - i, read back with the
  // match counts below
  const int64_t jt_T = keyed ? 0 : (int64_t)(hc.omax >> kJtB) + 1;
  const bool jt_try = !keyed && jtile_on() && jt_T <= ((int64_t)1 << 22) && (int64_t)Gw * perw < 0xffffffffll;
  uint32_t* jt_cnt = nullptr;
  uint32_t* jt_misc = nullptr;  // [0] largest j - i, [1] placement error
  uint32_t* jt_P = nullptr;      // staging index where each i-tile's pairs start (T + 1 entries)
  if (jt_try) {
    jt_cnt = (uint32_t*)sc.take((size_t)(jt_T + 1) * 4);
    jt_misc = (uint32_t*)sc.take(8);
    jt_P = (uint32_t*)sc.take((size_t)(jt_T + 1) * 4);
    SM_HIP(hipMemsetAsync(jt_cnt, 0, (size_t)(jt_T + 1) * 4, s));
    SM_HIP(hipMemsetAsync(jt_misc, 0, 8, s));
    hipLaunchKernelGGL(jt_count_kernel, dim3(Gw), dim3(1024), 0, s, stq, mcount, perw, Gw, a.ordinals, a.ordinal_base,
                       n, (uint32_t)jt_T, jt_cnt, jt_misc, jt_P);
    tmark("j_count");
  }
  if (tm) SM_HIP(hipEventRecord(tm->ev[2], s));

  // carried partials against this batch (before the walk's records are overwritten by the j passes)
  uint64_t* cps = nullptr;
  int64_t Mc = 0;
  if (nc > 0) {
    uint64_t* cpair = (uint64_t*)sc.take((size_t)nc * 8);
    ResolveArgs ra{};
    ra.crow = carry.rows;
    ra.nc = nc;
    ra.w = carry.width;
    ra.vattr = hi.vattr;
    ra.vtype = hi.vtype;
    ra.vmode = vmode;
    ra.vmin = vmin;
    ra.exact_codes = exact_codes;
    ra.rec = cur;
    ra.st = a.st;
    ra.ts = a.ts;
    ra.ord = a.ordinals;
    ra.obase = a.ordinal_base;
    ra.n = n;
    ra.kmin = kmin;
    ra.span = (int64_t)kspan;
    ra.ts0 = hc.ts0;
    ra.within = a.within;
    ra.cpair = cpair;
    ra.cand = cand;
    ra.cand_n = cflags;
    ra.cand_cap = (uint32_t)cand_cap;
    ra.err = cflags + 1;
    launch_resolve(keyed, spec, ra, s);
    uint32_t* fl = (uint32_t*)sc.take((size_t)nc * 4 + 4);
    hipLaunchKernelGGL(pair_flag_kernel, dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, s, cpair, nc, fl);
    exclusive_scan_u32(fl, (size_t)nc, sc, s, fl + nc);
    uint32_t hmc = 0;
    SM_HIP(hipMemcpyAsync(&hmc, fl + nc, 4, hipMemcpyDeviceToHost, s));
    SM_HIP(hipStreamSynchronize(s));
    Mc = hmc;
    if (Mc > 0) {
      cps = (uint64_t*)sc.take((size_t)Mc * 8);
      uint64_t* cps2 = (uint64_t*)sc.take((size_t)Mc * 8);
      hipLaunchKernelGGL(pair_compact_kernel, dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, s, cpair, fl, nc, cps);
      // (j, i) order
      if (radix_sort_pairs<uint64_t>(cps, cps2, nullptr, nullptr, (size_t)Mc, 0, 64, sc, s)) cps = cps2;
    }
  }

  // order by j: LSD passes over the (j, i) pairs; the first reads the walk's chunk-local staging (its digit-0
  // counts came from the walk), the last writes the output
  std::vector<uint32_t> hm(Gw);
  SM_HIP(hipMemcpyAsync(hm.data(), mcount, sizeof(uint32_t) * Gw, hipMemcpyDeviceToHost, s));
  scan_counts(Gw);
  uint32_t hcf[2];
  SM_HIP(hipMemcpyAsync(hcf, cflags, 8, hipMemcpyDeviceToHost, s));
  uint32_t hjd = 0xffffffffu;
  if (jt_try) SM_HIP(hipMemcpyAsync(&hjd, jt_misc, 4, hipMemcpyDeviceToHost, s));
  SM_HIP(hipStreamSynchronize(s));
  if (hcf[1]) {
    sc.used = mark;
    throw std::runtime_error((hcf[1] & 2) ? "a carried partial lies more than 2^31 events before the batch's ordinal "
                                            "base (match tuples are 32-bit ordinals relative to it)"
                                          : "fast path: more than 2^26 partial matches pending at the end of a device "
                                            "batch");
  }
  int64_t M = 0;
  for (int g = 0; g < Gw; ++g) M += hm[g];
  if (M + Mc > pairs_cap) {
    sc.used = mark;
    throw std::runtime_error("match buffer too small");
  }
  uint64_t* mainq = (uint64_t*)pairs_out;
  bool jt_done = false;
  if (M > 0 && jt_try && hjd <= kJtDMax) {
    uint64_t* tgt = Mc == 0 ? (uint64_t*)pairs_out : pq;
    exclusive_scan_u32(jt_cnt, (size_t)jt_T + 1, sc, s);
    hipLaunchKernelGGL(jt_place_kernel, dim3((unsigned)jt_T), dim3(kJtThreads), 0, s, stq, mcount, perw, jt_P, jt_cnt,
                       hjd, tgt, jt_misc + 1);
    tmark("j_tile");
    uint32_t herr = 0;
    SM_HIP(hipMemcpyAsync(&herr, jt_misc + 1, 4, hipMemcpyDeviceToHost, s));
    SM_HIP(hipStreamSynchronize(s));
    if (herr == 0) {
      jt_done = true;
      mainq = tgt;
    }
  }
  if (M > 0 && !jt_done) {
    const int64_t perM = round_up((M + G - 1) / G, kTile);
    const uint64_t* cq = stq;
    uint64_t* outs[2] = {pq, qq};
    for (int p = 0; p < jpass; ++p) {
      const bool last = p == jpass - 1;
      if (p > 0) {
        hipLaunchKernelGGL((upsweep_kernel<PairDigits>), dim3(G), dim3(kBlock), 0, s, PairDigits{cq}, M, perM, G,
                           p * kRB, cnt);
        tmark("j_up");
        scan_counts(G);
      }
      const int64_t nn = p == 0 ? n : M;
      const int64_t pp = p == 0 ? perw : perM;
      const uint32_t* seg = p == 0 ? mcount : nullptr;
      const int gg = p == 0 ? Gw : G;
      uint64_t* nq = (last && Mc == 0) ? (uint64_t*)pairs_out : outs[p & 1];
      if (jpass_wc() > (p == 0 ? 1 : 0))
        hipLaunchKernelGGL((downsweep_wc_kernel<2, PairSrc>), dim3(gg), dim3(kWcBlock), 0, s, PairSrc{cq}, nullptr, nq,
                           nn, pp, seg, gg, p * kRB, cnt, dbase);
      else
        hipLaunchKernelGGL((downsweep_kernel<2, PairSrc>), dim3(gg), dim3(kBlock), 0, s, PairSrc{cq}, nullptr, nq, nn,
                           pp, seg, gg, p * kRB, cnt, dbase);
      tmark(last ? "j_pass_last" : "j_pass");
      cq = nq;
    }
    mainq = (uint64_t*)cq;
  }
  if (Mc > 0) {  // merge the carried partials' matches in: for equal j they come first (older e1)
    const int64_t tot = M + Mc;
    (void)tot;
    if (M > 0)
      hipLaunchKernelGGL(merge_main_kernel, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, s, mainq, M, cps, Mc,
                         (uint64_t*)pairs_out);
    hipLaunchKernelGGL(merge_carried_kernel, dim3((unsigned)((Mc + 255) / 256)), dim3(256), 0, s, cps, Mc, mainq, M,
                       (uint64_t*)pairs_out);
    tmark("carry_merge");
  }
  if (tm) SM_HIP(hipEventRecord(tm->ev[3], s));
  // carry out
  build_carry(cand, hcf[0], a.st, hi.nattr, carry, sc, s);
  SM_HIP(hipStreamSynchronize(s));
  return finish(M + Mc);
}

}  // namespace sm
