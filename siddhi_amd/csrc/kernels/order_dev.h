// Order kernel of the bucket-stack pipeline (stack.hip): the stack kernel leaves each bucket's matches in its
// staging run in arrival order of j (pops of one j consecutive, oldest e1 first: StreamPreStateProcessor
// .processAndReturn :274-327 walks the pending list oldest first), with the run's offset of every ordinal tile
// (mt[t][d]: matches of bucket d whose j precedes tile t). The output is every (i, j) in (j, then pending order),
// the reference's emission order. A j belongs to exactly one bucket (its key's), so one tile's output is the
// interleaving of the buckets' segments by j, and a j's matches are one run inside one segment.
//
// order2_kernel (round 6, the default; SM_ORDER_V1=1 builds the round-3 order_kernel of stack.hip). That kernel
// kept the segments in registers from their load to their placement and waited, once per tile, for the segment
// loads and (gfx9's vmcnt counts loads and stores in order) for the previous tile's output stores: one workgroup per
// CU spent most of each tile waiting on memory. Here the segments pass through LDS, and the next tile's loads are in
// flight while this tile is counted and placed:
//   * an LDS input image holds the tile's segments, bucket after bucket (offsets: a block scan of the lengths; a
//     staging index per image entry, written with the tile's descriptor);
//   * at the top of each tile every thread issues the loads of the next tile's image entries (eight per thread,
//     lane-consecutive: a wave instruction reads 64 consecutive entries of about eleven segments) and of an mt row
//     two tiles ahead; they land in the input image after this tile's placement, before its output stores;
//   * count: each thread takes eight consecutive image entries; the first match of each j-run stores the run length
//     in a u16 per ordinal (plain stores: no other bucket has that j); block scan of the counts; placement of each
//     match at offset(j) + its rank in the run into an LDS output image, written out coalesced.
// A tile with more matches than the images hold (dense matches: kOC2 per 2^kTB ordinals) takes a slower exact path:
// one thread per bucket, LDS atomic counts, direct placement in HBM.
#pragma once
#include "stack_dev.h"

namespace sm {
namespace {

struct OrderArgs {
  const uint64_t* stage;
  const uint32_t* sbase;
  const uint32_t* mt;  // [t][d]: matches of bucket d whose j precedes tile t (ntiles + 1 rows)
  int64_t ntiles;
  uint64_t* out;
};

#ifndef SM_ORDER2_GT
#define SM_ORDER2_GT 32  // A/B build flag: consecutive tiles per order2 workgroup (the pipeline's prologue is per group)
#endif
constexpr int kGT2 = SM_ORDER2_GT;
// the two images (8-byte matches) and the next tile's staging index per entry (4 bytes) in what the counts and the
// scan words leave of 160 KB
constexpr int kOC2 = ((160 * 1024 - kOT * 2 - 256) / 20) & ~7;
constexpr int kLP = (kOC2 + kOB - 1) / kOB;  // image entries per thread
static_assert(kOT == 8 * kOB, "eight u16 counts (one 16-byte LDS word) per thread in the scan");
static_assert(kBins == kOB && kOB == 1024, "one bucket per thread");
static_assert(kLP == 8 && kOC2 % kLP == 0 && kOC2 <= kLP * kOB, "a thread's block of the image: eight entries, whole");
static_assert(kOC2 < 65536 && (size_t)kOT * 4 <= (size_t)kOC2 * 8, "u16 offsets; the u32 overflow counts alias the input image");

__device__ __forceinline__ uint32_t o2_j(uint64_t v) { return (uint32_t)(v >> 32); }
// LDS position of image entry e: within each 64-byte block of eight entries the four 16-byte chunks are XOR-swizzled
// by bits 4-5 of e, so that the 16-byte reads of a thread's block (lane stride 64 bytes) fall in distinct banks,
// while consecutive lanes landing consecutive entries still fill whole blocks
__device__ __forceinline__ uint32_t o2_pos(uint32_t e) { return e ^ (((e >> 4) & 3u) << 1); }
// a value the compiler cannot see through: keeps address arithmetic at its use instead of hoisted (and spilled)
__device__ __forceinline__ uint32_t o2_opaque(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(x));
#endif
  return x;
}

#ifndef SM_ORDER2_STAMPS
#define SM_ORDER2_STAMPS 0  // diagnostic build flag: shader clocks per phase of order2_kernel, summed over waves
#endif
#if SM_ORDER2_STAMPS
__device__ unsigned long long g_o2_stamps[8];
#endif
#if SM_ORDER2_STAMPS && defined(__HIP_DEVICE_COMPILE__)
#define SM_O2_CLOCK() __builtin_amdgcn_s_memtime()
#else
#define SM_O2_CLOCK() 0ull
#endif
#define SM_O2_PHASE(i)                              \
  do {                                              \
    if (SM_ORDER2_STAMPS) {                         \
      const unsigned long long t_ = SM_O2_CLOCK();  \
      o2_acc[i] += t_ - o2_last;                    \
      o2_last = t_;                                 \
    }                                               \
  } while (0)

__global__ void __launch_bounds__(kOB) order2_kernel(OrderArgs a) {
  __shared__ __attribute__((aligned(16))) uint64_t inb[kOC2];   // the tile's segments, bucket after bucket
  __shared__ __attribute__((aligned(16))) uint64_t obuf[kOC2];  // the tile's output
  __shared__ __attribute__((aligned(16))) uint16_t c16[kOT];    // run length of each ordinal's j, then its offset
  __shared__ uint32_t src[kOC2];                                // the next tile to load: staging index of each entry
  __shared__ uint32_t lw[kOB / 64];
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t sb = a.sbase[tid];
  const int64_t T = a.ntiles;
  const uint32_t* inj = (const uint32_t*)inb + 1;  // j of image entry e: inj[2 o2_pos(e)]
  unsigned long long o2_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, o2_last = SM_O2_CLOCK();
  // phases: 0 prologue 6 issue 1 count 2 scan 3 place 7 land 4 output writes 5 descriptor

  // descriptor of bucket tid's segment [lo, hi) of its run (block scan: one barrier; the writes become visible at
  // the caller's next barrier); returns the tile's total
  auto desc = [&](uint32_t lo, uint32_t hi) {
    const uint32_t len = hi - lo;
    uint32_t tt;
    const uint32_t ib = block_excl(len, lw, &tt);
    if (tt <= (uint32_t)kOC2)  // image entry -> staging index
      for (uint32_t k = 0; k < len; ++k) src[ib + k] = sb + lo + k;
    return tt;
  };
  // the described tile's image entries tid + k kOB into registers (consecutive lanes: consecutive entries, mostly
  // of one segment); issued without waiting
  uint64_t v[kLP];
  auto issue = [&](uint32_t tt) {
    // branch-free, so that every LDS lookup is issued before the first load: an entry past the tile's end reads
    // the tile's last entry again (a cache hit) and is not landed
    uint32_t x[kLP];
#pragma unroll
    for (int k = 0; k < kLP; ++k) x[k] = src[(uint32_t)(tid + k * kOB) < tt ? (uint32_t)(tid + k * kOB) : tt - 1u];
#pragma unroll
    for (int k = 0; k < kLP; ++k) v[k] = a.stage[x[k]];
  };
  auto land = [&](uint32_t tt) {
#pragma unroll
    for (int k = 0; k < kLP; ++k) {
      const uint32_t e = (uint32_t)(tid + k * kOB);
      if (e < tt) inb[o2_pos(e)] = v[k];
    }
  };

  for (int64_t tb = (int64_t)blockIdx.x * kGT2; tb < T; tb += (int64_t)gridDim.x * kGT2) {
    const int64_t te = tb + kGT2 < T ? tb + kGT2 : T;
    lds_barrier();  // the previous group's readers of lw, the descriptors and the images are done
    // mA, mB, mC: bucket tid's run offsets of tiles t, t + 1, t + 2
    uint32_t mA = a.mt[tb * kBins + tid];
    uint32_t mB = a.mt[(tb + 1) * kBins + tid];
    uint32_t mC = tb + 1 < te ? a.mt[(tb + 2) * kBins + tid] : mB;
    uint32_t tcur;
    (void)block_excl(mA, lw, &tcur);
    int64_t out = tcur;  // matches whose j precedes the tile
    for (int k = tid; k < kOT / 8; k += kOB) ((uint4*)c16)[k] = make_uint4(0, 0, 0, 0);
    lds_barrier();  // lw's readers are done
    tcur = desc(mA, mB);
    lds_barrier();  // the descriptor is visible
    if (tcur != 0u && tcur <= (uint32_t)kOC2) {
      issue(tcur);
      land(tcur);
    }
    lds_barrier();  // the image is filled; the descriptor's readers are done
    uint32_t tnext = tb + 1 < te ? desc(mB, mC) : 0u;
    lds_barrier();  // the next descriptor is visible
    SM_O2_PHASE(0);

    for (int64_t t = tb; t < te; ++t) {
      const uint32_t j0 = (uint32_t)(t << kTB);
      const bool ovf = tcur > (uint32_t)kOC2;
      const bool more = t + 1 < te && tnext != 0u && tnext <= (uint32_t)kOC2;
      // the mt row after the next tile, then the next tile's entries: in flight during this tile's count, scan and
      // placement (the row first: the wait for the entries at the hand-over then covers it, before any store)
      uint32_t mD = t + 2 < te ? a.mt[(t + 3) * kBins + tid] : mC;  // t + 3 <= te <= T: the row exists
      if (more) issue(tnext);
      SM_O2_PHASE(6);
      if (!ovf) {
        // runs: thread tid takes the kLP consecutive entries [e0, e0 + kLP) (kLP / 2 16-byte reads); run starts, run
        // lengths and ranks come from register compares, LDS only at the block's edges (a run crossing one: rare).
        // The entry before a run's first is another j: of this bucket, or of another bucket, which never has it.
        const uint32_t e0 = (uint32_t)tid * kLP;
        uint32_t jj[kLP], rk8[kLP];
        if (e0 < tcur) {
          const uint4* b4 = (const uint4*)inb + e0 / 2;
          const int sw = (tid >> 1) & 3;  // o2_pos's chunk swizzle of this block
#pragma unroll
          for (int q = 0; q < kLP / 2; ++q) {
            const uint4 x = b4[q ^ sw];
            jj[2 * q] = x.y;
            jj[2 * q + 1] = x.w;
          }
          const uint32_t nv = tcur - e0 < (uint32_t)kLP ? tcur - e0 : (uint32_t)kLP;  // valid entries of the block
          // rank of each entry in its run (the first one's run may come from the block before)
          uint32_t r0 = 0;
          if (e0 > 0 && inj[2 * o2_pos(e0 - 1)] == jj[0]) {
            const uint32_t eo = o2_opaque(e0);  // no hoisted (spilled) addresses: a scratch reload would wait for
            r0 = 1;                             // the next tile's loads in flight
            while (r0 < eo && inj[2 * o2_pos(eo - r0 - 1)] == jj[0]) ++r0;
          }
          rk8[0] = r0;
#pragma unroll
          for (int k = 1; k < kLP; ++k) rk8[k] = jj[k] == jj[k - 1] ? rk8[k - 1] + 1u : 0u;
          // length of the run from each entry to its end (the last one's may go on into the next block)
          uint32_t ln[kLP];
          {
            uint32_t x = 0;
            if (nv == (uint32_t)kLP && e0 + kLP < tcur && inj[2 * o2_pos(e0 + kLP)] == jj[kLP - 1]) {
              const uint32_t eo = o2_opaque(e0 + kLP), to = o2_opaque(tcur);
              x = 1;
              while (eo + x < to && inj[2 * o2_pos(eo + x)] == jj[kLP - 1]) ++x;
            }
            ln[kLP - 1] = 1u + x;
          }
#pragma unroll
          for (int k = kLP - 2; k >= 0; --k) ln[k] = 1u + ((uint32_t)(k + 1) < nv && jj[k + 1] == jj[k] ? ln[k + 1] : 0u);
#pragma unroll
          for (int k = 0; k < kLP; ++k)
            if ((uint32_t)k < nv && rk8[k] == 0u) c16[jj[k] - j0] = (uint16_t)ln[k];
        }
        lds_barrier();
        SM_O2_PHASE(1);
        {  // offsets: eight ordinals per thread (packed u16 sums: the tile's total is below 2^16)
          uint4* c4 = (uint4*)c16 + tid;
          const uint4 c = *c4;
          const uint32_t s2 = c.x + c.y + c.z + c.w;
          uint32_t tt;
          uint32_t r = block_excl((s2 & 0xffffu) + (s2 >> 16), lw, &tt);
          uint32_t h[4] = {c.x, c.y, c.z, c.w}, o[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const uint32_t lo = r, hi = r + (h[k] & 0xffffu);
            r = hi + (h[k] >> 16);
            o[k] = lo | (hi << 16);
          }
          *c4 = make_uint4(o[0], o[1], o[2], o[3]);
        }
        lds_barrier();
        SM_O2_PHASE(2);
        // placement: offset of the j + rank in its run
        if (e0 < tcur) {
          const uint32_t nv = tcur - e0 < (uint32_t)kLP ? tcur - e0 : (uint32_t)kLP;
          uint32_t off[kLP];
#pragma unroll
          for (int k = 0; k < kLP; ++k) off[k] = c16[(jj[k] - j0) & (kOT - 1)];
          const uint4* b4 = (const uint4*)inb + e0 / 2;
          const int sw = (tid >> 1) & 3;
#pragma unroll
          for (int q = 0; q < kLP / 2; ++q) {
            const uint4 x = b4[q ^ sw];
            if ((uint32_t)(2 * q) < nv) obuf[off[2 * q] + rk8[2 * q]] = ((uint64_t)x.y << 32) | x.x;
            if ((uint32_t)(2 * q + 1) < nv) obuf[off[2 * q + 1] + rk8[2 * q + 1]] = ((uint64_t)x.w << 32) | x.z;
          }
        }
        lds_barrier();
        SM_O2_PHASE(3);
      } else {  // more matches than the images hold: one thread per bucket, straight from HBM
        uint32_t* c32 = (uint32_t*)inb;
        for (int k = tid; k < kOT / 4; k += kOB) ((uint4*)c32)[k] = make_uint4(0, 0, 0, 0);
        lds_barrier();
        const uint32_t s = sb + mA, n = mB - mA;
        for (uint32_t k = 0; k < n; ++k) atomicAdd(&c32[o2_j(a.stage[s + k]) - j0], 1u);
        lds_barrier();
        {
          uint4* c4 = (uint4*)c32 + 2 * tid;
          const uint4 x = c4[0], y = c4[1];
          uint32_t tt;
          uint32_t r = block_excl(x.x + x.y + x.z + x.w + y.x + y.y + y.z + y.w, lw, &tt);
          uint4 ox, oy;
          ox.x = r;
          ox.y = ox.x + x.x;
          ox.z = ox.y + x.y;
          ox.w = ox.z + x.z;
          oy.x = ox.w + x.w;
          oy.y = oy.x + y.x;
          oy.z = oy.y + y.y;
          oy.w = oy.z + y.z;
          c4[0] = ox;
          c4[1] = oy;
        }
        lds_barrier();
        uint32_t pj = 0xffffffffu, rk = 0;
        for (uint32_t k = 0; k < n; ++k) {
          const uint64_t x = a.stage[s + k];
          const uint32_t j = o2_j(x);
          rk = j == pj ? rk + 1u : 0u;
          pj = j;
          a.out[out + c32[j - j0] + rk] = x;
        }
        lds_barrier();  // the counts' readers are done before the next tile's entries land
      }
      // hand-over: the next tile's entries into the image (their loads were issued before this tile's output
      // stores, so the wait does not include those), then this tile's output, and clear the counts
      if (more) land(tnext);
      mD = o2_opaque(mD);  // waited for here, with the entries, not after this tile's stores
      SM_O2_PHASE(7);
      SM_O2_PHASE(7);
      if (!ovf)
        for (uint32_t k = tid; k < tcur; k += kOB) a.out[out + k] = obuf[k];
      for (int k = tid; k < kOT / 8; k += kOB) ((uint4*)c16)[k] = make_uint4(0, 0, 0, 0);
      SM_O2_PHASE(4);
      out += tcur;
      tcur = tnext;
      mA = mB;
      mB = mC;
      // the descriptor of tile t + 2 (its block scan's lw readers are past the placement barrier; the entries of
      // tile t + 1 were looked up through the old descriptor before this point)
      tnext = t + 2 < te ? desc(mC, mD) : 0u;
      mC = mD;
      lds_barrier();  // image, counts and descriptor ready for the next tile
      SM_O2_PHASE(5);
    }
  }
#if SM_ORDER2_STAMPS && defined(__HIP_DEVICE_COMPILE__)
  if (lane == 0)
    for (int i = 0; i < 8; ++i) atomicAdd(&g_o2_stamps[i], o2_acc[i]);
#endif
}

}  // namespace
}  // namespace sm
