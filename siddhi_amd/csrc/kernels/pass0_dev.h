// Key pass 0 of the keyed fast path (round 3): the stable 1024-way scatter of 16-byte keyed records by the key's
// low digit, built from the original columns (Src: OrigSrc in fastpath3.hip). Same pass semantics and the same
// write-combining as downsweep_wc_kernel<0> (fastpath3.hip: a tile stores only records whose 64-byte segment of the
// output completes in this chunk; the < 4 records left of a digit's run are carried in LDS to the next tile and the
// chunk's last tile flushes them), with less LDS traffic per record:
//   * per (digit, wave) counts are one 32-byte row per digit ([digit][wave] u16): a digit's tile count and the
//     records of its earlier waves come from two 16-byte reads and packed 16-bit dot products, where the old layout
//     walked the 16 waves per digit with 32 LDS operations;
//   * the record moves through LDS once (16-byte slots, 64 KB per 4096-record tile) instead of as two 8-byte halves.
// A header of its own so the kernel also runs under the host wave emulator (tests/native/pass0_emu.cpp).
#pragma once
#include "fastpath_dev.h"

namespace sm {
namespace {

constexpr int kP0Block = 1024;               // threads; thread d owns digit d in the per-digit steps
constexpr int kP0Waves = kP0Block / 64;      // 16: one u16 count per wave in a digit's 32-byte row
constexpr int kP0Items = 4;                  // records per thread per tile
constexpr int kP0Tile = kP0Block * kP0Items;  // 4096
constexpr int kP0Seg = 4;                    // records per 64-byte output segment
static_assert(kBins == kP0Block && kP0Waves == 16, "one digit per thread, 16 waves");

__device__ __forceinline__ uint32_t sm_udot2(uint32_t a, uint32_t b, uint32_t c) {  // sum of u16 products + c
#if defined(__HIP_DEVICE_COMPILE__)
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b), c, false);
#else
  return c + (a & 0xffffu) * (b & 0xffffu) + (a >> 16) * (b >> 16);
#endif
}

// block-wide exclusive scan of one value per thread; the total through *tot
__device__ __forceinline__ uint32_t p0_block_excl(uint32_t v, uint32_t* lw, uint32_t* tot) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(inc, o, 64);
    if (lane >= o) inc += u;
  }
  if (lane == 63) lw[w] = inc;
  lds_barrier();
  uint32_t r = inc - v, t = 0;
  for (int q = 0; q < kP0Waves; ++q) {
    const uint32_t x = lw[q];
    if (q < w) r += x;
    t += x;
  }
  *tot = t;
  return r;
}

// sum of the u16 counts of waves [0, w) in a digit's row (8 words, two waves each)
__device__ __forceinline__ uint32_t p0_before(const uint4& r0, const uint4& r1, int w) {
  const uint32_t word[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t m = 2 * i + 1 < w ? 0xffffffffu : (2 * i < w ? 0x0000ffffu : 0u);
    s = sm_udot2(word[i] & m, 0x00010001u, s);
  }
  return s;
}

// Chunk blockIdx.x = [blockIdx.x * per, + per) of the batch, tile by tile. cnt[d * G + g] = records of digit d in
// chunks before g (scan_chunks), dbase[d] = records of digits before d: chunk g's first position for digit d is
// dbase[d] + cnt[d * G + g].
template <typename Src>
__global__ void __launch_bounds__(kP0Block) pass0_kernel(Src src, uint4* __restrict__ drec, int64_t n, int64_t per,
                                                          int G, const uint32_t* __restrict__ cnt,
                                                          const uint32_t* __restrict__ dbase) {
  __shared__ __attribute__((aligned(16))) uint4 xb[kP0Tile];
  __shared__ __attribute__((aligned(16))) uint16_t wc[kBins][kP0Waves];
  __shared__ uint32_t tstart[kBins + 1];
  __shared__ uint32_t run[kBins];  // next output position of each digit for this chunk
  __shared__ uint32_t cst[kBins];  // first position of the digit's incomplete segment: carried = [cst, run)
  __shared__ __attribute__((aligned(16))) uint4 carry[kBins][kP0Seg - 1];
  __shared__ uint32_t lw[kP0Waves];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint64_t lt = lanemask_lt();
  const int64_t lo = (int64_t)blockIdx.x * per;
  int64_t len = n - lo;
  if (len > per) len = per;
  if (len < 0) len = 0;
  src.init();
  uint4* row = (uint4*)&wc[tid][0];  // digit tid's count row, zeroed for the first tile here, then after each
                                     // tile's placement (its last reader), so no barrier opens a tile
  {
    const uint32_t r0 = dbase[tid] + cnt[(int64_t)tid * G + blockIdx.x];
    run[tid] = r0;
    cst[tid] = r0;
    row[0] = make_uint4(0, 0, 0, 0);
    row[1] = make_uint4(0, 0, 0, 0);
  }
  lds_barrier();
  typename Src::Raw raw[kP0Items];
  auto load_tile = [&](int64_t base) {
    const int64_t rem = lo + len - base;
    const int tn = rem < kP0Tile ? (int)rem : kP0Tile;
#pragma unroll
    for (int k = 0; k < kP0Items; ++k) {
      const int e = w * 64 * kP0Items + k * 64 + lane;
      if (e < tn) raw[k] = src.load(base + e);
    }
  };
  if (len > 0) load_tile(lo);

  for (int64_t base = lo; base < lo + len; base += kP0Tile) {
    const int tile_n = (int)((lo + len - base) < kP0Tile ? (lo + len - base) : kP0Tile);
    const bool last = base + kP0Tile >= lo + len;
    uint4 rec[kP0Items];
#pragma unroll
    for (int k = 0; k < kP0Items; ++k) {
      const int e = w * 64 * kP0Items + k * 64 + lane;
      if (e < tile_n) rec[k] = src.record(raw[k], base + e);
    }
    // (the previous tile's readers of xb / tstart / run / cst / carry finished before its closing barrier)

    // stable rank within (wave, digit): wave64 ballot peer masks, in arrival order
    uint32_t dg[kP0Items], lp[kP0Items];
#pragma unroll
    for (int k = 0; k < kP0Items; ++k) {
      const int e = w * 64 * kP0Items + k * 64 + lane;
      const bool valid = e < tile_n;
      dg[k] = valid ? rec[k].x & (kBins - 1) : 0u;
      const uint64_t peers = peer_mask(dg[k], valid);
      uint32_t old = 0;
      if (valid) old = wc[dg[k]][w];
      wave_lockstep();
      const uint32_t below = (uint32_t)__popcll(peers & lt);
      if (valid && below == 0) wc[dg[k]][w] = (uint16_t)(old + (uint32_t)__popcll(peers));
      wave_lockstep();
      lp[k] = old + below;
    }
    lds_barrier();

    // digit tid: its tile count and the tile's digit starts (block scan)
    uint32_t ct;
    {
      const uint4 r0 = row[0], r1 = row[1];
      ct = 0;
      const uint32_t word[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
#pragma unroll
      for (int i = 0; i < 8; ++i) ct = sm_udot2(word[i], 0x00010001u, ct);
      uint32_t tot;
      tstart[tid] = p0_block_excl(ct, lw, &tot);
      if (tid == 0) tstart[kBins] = tot;
    }
    const uint32_t rn = run[tid], c0 = cst[tid];
    const uint32_t lim = last ? 0xffffffffu : ((rn + ct) & ~(uint32_t)(kP0Seg - 1));
    lds_barrier();

    // the tile into LDS grouped by digit (arrival order within a digit)
#pragma unroll
    for (int k = 0; k < kP0Items; ++k) {
      const int e = w * 64 * kP0Items + k * 64 + lane;
      if (e < tile_n) {
        const uint4* rr = (const uint4*)&wc[dg[k]][0];
        xb[tstart[dg[k]] + p0_before(rr[0], rr[1], w) + lp[k]] = rec[k];
      }
    }
    if (!last) load_tile(base + kP0Tile);  // the next tile's loads overlap this tile's stores
    // carried records of digit tid whose segment completes now (or the chunk ends) leave first
    if (rn != c0 && (last || lim > c0))
      for (uint32_t q = 0; q < rn - c0; ++q) drec[c0 + q] = carry[tid][q];
    lds_barrier();  // xb complete; the carry slots read above may be refilled; the count rows are read no more
    row[0] = make_uint4(0, 0, 0, 0);
    row[1] = make_uint4(0, 0, 0, 0);

    // one 16-byte store per record, or into the carry when its segment is not complete in this chunk yet
#pragma unroll
    for (int r = 0; r < kP0Items; ++r) {
      const int s = r * kP0Block + tid;
      if (s < tile_n) {
        const uint4 x = xb[s];
        const uint32_t d = x.x & (kBins - 1);
        const uint32_t rd = run[d], td = tstart[d];
        const uint32_t dest = rd + (uint32_t)s - td;
        const uint32_t ld = last ? 0xffffffffu : ((rd + tstart[d + 1] - td) & ~(uint32_t)(kP0Seg - 1));
        if (dest < ld) {
          drec[dest] = x;
        } else {
          const uint32_t cd = cst[d];
          carry[d][dest - (cd > ld ? cd : ld)] = x;
        }
      }
    }
    lds_barrier();  // every destination computed from run / cst before they advance
    run[tid] = rn + ct;
    if (lim != 0xffffffffu && lim > c0) cst[tid] = lim;
  }
  src.flush();
}

}  // namespace
}  // namespace sm
