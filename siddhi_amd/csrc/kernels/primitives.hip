// Scan and stable LSD radix sort for gfx950 (wave64). See primitives.h.
#include "primitives.h"

namespace sm {

namespace {

constexpr int kScanThreads = 256;
constexpr int kScanItems = 16;
constexpr int kScanTile = kScanThreads * kScanItems;

template <typename T>
__device__ __forceinline__ T wave_incl_scan(T v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    T u = __shfl_up(v, o, 64);
    if (lane >= o) v += u;
  }
  return v;
}

// Block-wide exclusive scan of one value per thread; returns (exclusive prefix, block total).
template <typename T>
__device__ __forceinline__ T block_excl_scan(T v, T* lds_waves, T& total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  T inc = wave_incl_scan(v);
  if (lane == 63) lds_waves[w] = inc;
  __syncthreads();
  T wbase = 0, tot = 0;
  for (int k = 0; k < (int)(blockDim.x >> 6); ++k) {
    if (k < w) wbase += lds_waves[k];
    tot += lds_waves[k];
  }
  __syncthreads();
  total = tot;
  return wbase + inc - v;
}

template <typename T>
__global__ void scan_reduce_kernel(const T* __restrict__ in, size_t n, T* __restrict__ partials) {
  __shared__ T lw[kScanThreads / 64];
  size_t base = (size_t)blockIdx.x * kScanTile;
  T s = 0;
  for (int k = 0; k < kScanItems; ++k) {
    size_t i = base + (size_t)k * kScanThreads + threadIdx.x;
    if (i < n) s += in[i];
  }
  T tot;
  block_excl_scan(s, lw, tot);
  if (threadIdx.x == 0) partials[blockIdx.x] = tot;
}

template <typename T>
__global__ void scan_apply_kernel(T* __restrict__ data, size_t n, const T* __restrict__ offsets,
                                  T* __restrict__ total_out) {
  __shared__ T lw[kScanThreads / 64];
  size_t base = (size_t)blockIdx.x * kScanTile + (size_t)threadIdx.x * kScanItems;
  T v[kScanItems];
  T s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    size_t i = base + k;
    v[k] = (i < n) ? data[i] : 0;
    s += v[k];
  }
  T tot;
  T run = block_excl_scan(s, lw, tot) + (offsets ? offsets[blockIdx.x] : 0);
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    size_t i = base + k;
    if (i < n) data[i] = run;
    run += v[k];
  }
  if (total_out && blockIdx.x == gridDim.x - 1 && threadIdx.x == blockDim.x - 1) *total_out = run;
}

template <typename T>
void exclusive_scan_impl(T* data, size_t n, Scratch& sc, hipStream_t s, T* total_dev) {
  if (n == 0) {
    if (total_dev) SM_HIP(hipMemsetAsync(total_dev, 0, sizeof(T), s));
    return;
  }
  size_t nb = (n + kScanTile - 1) / kScanTile;
  if (nb == 1) {
    hipLaunchKernelGGL(scan_apply_kernel<T>, dim3(1), dim3(kScanThreads), 0, s, data, n, (const T*)nullptr,
                       total_dev);
    return;
  }
  size_t mark = sc.used;
  T* partials = (T*)sc.take(nb * sizeof(T));
  hipLaunchKernelGGL(scan_reduce_kernel<T>, dim3(nb), dim3(kScanThreads), 0, s, data, n, partials);
  exclusive_scan_impl<T>(partials, nb, sc, s, (T*)nullptr);
  hipLaunchKernelGGL(scan_apply_kernel<T>, dim3(nb), dim3(kScanThreads), 0, s, data, n, (const T*)partials,
                     total_dev);
  sc.used = mark;
}

// ---------------------------------------------------------------- radix sort
constexpr int kRsThreads = 256;  // 4 waves
constexpr int kRsItems = 16;     // items per lane
constexpr int kRsWaveTile = 64 * kRsItems;
constexpr int kRsTile = kRsThreads * kRsItems;  // 4096

template <typename K>
__global__ __launch_bounds__(kRsThreads) void rs_upsweep(const K* __restrict__ keys, size_t n, int shift, int bits,
                                                         uint32_t* __restrict__ hist, uint32_t nblocks) {
  __shared__ uint32_t cnt[256];
  cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t dmask = (1u << bits) - 1;
  size_t base = (size_t)blockIdx.x * kRsTile;
  for (int k = 0; k < kRsItems; ++k) {
    size_t i = base + (size_t)k * kRsThreads + threadIdx.x;
    if (i < n) atomicAdd(&cnt[(uint32_t)(keys[i] >> shift) & dmask], 1u);
  }
  __syncthreads();
  hist[(size_t)threadIdx.x * nblocks + blockIdx.x] = cnt[threadIdx.x];
}

// Stable scatter of one 4096-item tile by its digit. Ranks within (wave, digit) come from ballot peer masks; the
// tile is then regrouped in LDS by digit (digit-major, arrival order within a digit) and leaves as contiguous digit
// runs, so consecutive lanes store consecutive addresses (about 16 items of 4 + 4 bytes per run at 256 digits):
// one or two lines per run instead of one line touched per lane and store instruction.
template <typename K>
__global__ __launch_bounds__(kRsThreads) void rs_downsweep(const K* __restrict__ kin, K* __restrict__ kout,
                                                           const uint32_t* __restrict__ vin,
                                                           uint32_t* __restrict__ vout, size_t n, int shift,
                                                           int bits, const uint32_t* __restrict__ hist,
                                                           uint32_t nblocks) {
  __shared__ uint32_t wcount[4][256];
  __shared__ uint32_t wbase[4][256];
  __shared__ uint32_t gbase[256];
  __shared__ uint32_t tstart[256];
  __shared__ uint32_t wsum[4];
  __shared__ K lkey[kRsTile];
  __shared__ uint32_t lval[kRsTile];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int k = 0; k < 4; ++k) wcount[k][threadIdx.x] = 0;
  __syncthreads();
  const uint32_t dmask = (1u << bits) - 1;
  const size_t tbeg = (size_t)blockIdx.x * kRsTile;
  const size_t wbeg = tbeg + (size_t)w * kRsWaveTile;
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  K key[kRsItems];
  uint32_t val[kRsItems];
  uint32_t lrank[kRsItems];
#pragma unroll
  for (int it = 0; it < kRsItems; ++it) {
    size_t i = wbeg + (size_t)it * 64 + lane;
    bool valid = i < n;
    key[it] = valid ? kin[i] : (K)0;
    val[it] = (valid && vin) ? vin[i] : 0u;
    uint32_t d = (uint32_t)(key[it] >> shift) & dmask;
    uint64_t peers = __ballot(valid);
    for (int b = 0; b < bits; ++b) {
      uint64_t bb = __ballot((d >> b) & 1u);
      peers &= ((d >> b) & 1u) ? bb : ~bb;
    }
    uint32_t r = (uint32_t)__popcll(peers & lt_mask);
    uint32_t before = wcount[w][d];
    __builtin_amdgcn_wave_barrier();
    if (valid && r == 0) wcount[w][d] = before + (uint32_t)__popcll(peers);
    __builtin_amdgcn_wave_barrier();
    lrank[it] = valid ? before + r : 0xffffffffu;
  }
  __syncthreads();
  {
    // digit threadIdx.x: its items before each wave, its tile start (block scan of the tile's digit counts)
    uint32_t acc = 0;
    for (int k = 0; k < 4; ++k) {
      wbase[k][threadIdx.x] = acc;
      acc += wcount[k][threadIdx.x];
    }
    gbase[threadIdx.x] = hist[(size_t)threadIdx.x * nblocks + blockIdx.x];
    uint32_t inc = acc;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(inc, o, 64);
      if (lane >= o) inc += u;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t off = 0;
    for (int k = 0; k < w; ++k) off += wsum[k];
    tstart[threadIdx.x] = off + inc - acc;
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < kRsItems; ++it) {
    if (lrank[it] == 0xffffffffu) continue;
    const uint32_t d = (uint32_t)(key[it] >> shift) & dmask;
    const uint32_t slot = tstart[d] + wbase[w][d] + lrank[it];
    lkey[slot] = key[it];
    lval[slot] = val[it];
  }
  __syncthreads();
  const uint32_t tn = n - tbeg < (size_t)kRsTile ? (uint32_t)(n - tbeg) : (uint32_t)kRsTile;
#pragma unroll 4
  for (uint32_t sl = threadIdx.x; sl < tn; sl += kRsThreads) {
    const K k = lkey[sl];
    const uint32_t d = (uint32_t)(k >> shift) & dmask;
    const size_t dest = (size_t)gbase[d] + (sl - tstart[d]);
    kout[dest] = k;
    if (vout) vout[dest] = lval[sl];
  }
}

}  // namespace

void exclusive_scan_u32(uint32_t* data, size_t n, Scratch& sc, hipStream_t s, uint32_t* total_dev) {
  exclusive_scan_impl<uint32_t>(data, n, sc, s, total_dev);
}
void exclusive_scan_u64(uint64_t* data, size_t n, Scratch& sc, hipStream_t s, uint64_t* total_dev) {
  exclusive_scan_impl<uint64_t>(data, n, sc, s, total_dev);
}

template <typename K>
bool radix_sort_pairs(K* keys, K* keys_alt, uint32_t* vals, uint32_t* vals_alt, size_t n, int begin_bit,
                      int end_bit, Scratch& sc, hipStream_t s) {
  if (n == 0 || end_bit <= begin_bit) return false;
  if (n > 0xffffffffull) throw std::runtime_error("radix_sort_pairs: more than 2^32 items");
  uint32_t nblocks = (uint32_t)((n + kRsTile - 1) / kRsTile);
  size_t mark = sc.used;
  uint32_t* hist = (uint32_t*)sc.take((size_t)256 * nblocks * sizeof(uint32_t));
  K *ki = keys, *ko = keys_alt;
  uint32_t *vi = vals, *vo = vals_alt;
  bool alt = false;
  for (int b = begin_bit; b < end_bit; b += 8) {
    int bits = std::min(8, end_bit - b);
    hipLaunchKernelGGL(rs_upsweep<K>, dim3(nblocks), dim3(kRsThreads), 0, s, ki, n, b, bits, hist, nblocks);
    exclusive_scan_u32(hist, (size_t)256 * nblocks, sc, s);
    hipLaunchKernelGGL(rs_downsweep<K>, dim3(nblocks), dim3(kRsThreads), 0, s, ki, ko, vi, vo, n, b, bits, hist,
                       nblocks);
    std::swap(ki, ko);
    std::swap(vi, vo);
    alt = !alt;
  }
  sc.used = mark;
  return alt;
}

template bool radix_sort_pairs<uint32_t>(uint32_t*, uint32_t*, uint32_t*, uint32_t*, size_t, int, int, Scratch&,
                                         hipStream_t);
template bool radix_sort_pairs<uint64_t>(uint64_t*, uint64_t*, uint32_t*, uint32_t*, size_t, int, int, Scratch&,
                                         hipStream_t);

}  // namespace sm
