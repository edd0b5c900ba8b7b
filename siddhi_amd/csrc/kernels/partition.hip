// Stable partition of a columnar batch by owning rank (key_owner: hash of the key) for the multi-GPU key exchange
// (PartitionStreamReceiver.receive core/partition/PartitionStreamReceiver.java:156 routes each event to the
// runtime of its key; across GPUs the key's owner rank plays that role). A counting sort with world <= 64 buckets:
//   1. per 4096-event tile: events per owner                                  -> cnt[owner * tiles + tile]
//   2. exclusive scan of cnt (owner-major)                                      -> first slot of (owner, tile)
//   3. per tile, events in arrival order: rank within (tile, owner) from wave ballots, then every column is
//      copied to its slot. Within an owner the output keeps arrival order, so rank r receives its rows in
//      global arrival order once the ranks' slices are concatenated.
// HBM traffic: key 4-8 B (pass 1) + every column read and written once (pass 3).
#include "partition.h"

namespace sm {
namespace {

constexpr int kPThreads = 256, kPItems = 16, kPTile = kPThreads * kPItems;

template <typename K>
__device__ __forceinline__ uint32_t owner_of(K k, uint32_t world) {
  return key_owner((int64_t)k, world);
}

template <typename K>
__global__ __launch_bounds__(kPThreads) void owner_count_kernel(const K* __restrict__ keys, int64_t n, uint32_t world,
                                                                uint32_t ntiles, uint32_t* __restrict__ cnt) {
  __shared__ uint32_t c[kMaxOwners];
  if (threadIdx.x < kMaxOwners) c[threadIdx.x] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kPTile;
  for (int k = 0; k < kPItems; ++k) {
    const int64_t i = base + (int64_t)k * kPThreads + threadIdx.x;
    if (i < n) atomicAdd(&c[owner_of(keys[i], world)], 1u);
  }
  __syncthreads();
  if (threadIdx.x < world) cnt[(int64_t)threadIdx.x * ntiles + blockIdx.x] = c[threadIdx.x];
}

template <typename K>
__global__ __launch_bounds__(kPThreads) void owner_scatter_kernel(const K* __restrict__ keys, int64_t n,
                                                                  uint32_t world, uint32_t ntiles,
                                                                  const uint32_t* __restrict__ start, PartCols cols) {
  __shared__ uint32_t run[kMaxOwners];                   // next slot of each owner for this tile
  __shared__ uint32_t wc[kPThreads / 64][kMaxOwners];    // per-wave counts of the current round
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (threadIdx.x < world) run[threadIdx.x] = start[(int64_t)threadIdx.x * ntiles + blockIdx.x];
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  const int64_t base = (int64_t)blockIdx.x * kPTile;
  for (int k = 0; k < kPItems; ++k) {
    const int64_t i = base + (int64_t)k * kPThreads + threadIdx.x;
    const bool in = i < n;
    const uint32_t o = in ? owner_of(keys[i], world) : 0u;
    // lanes of this wave with the same owner, via one ballot per owner bit
    uint64_t peers = __ballot(in);
    for (uint32_t b = 1; b < world; b <<= 1) {
      const uint64_t bb = __ballot((o & b) != 0);
      peers &= (o & b) ? bb : ~bb;
    }
    const uint32_t below = (uint32_t)__popcll(peers & lt);
    __syncthreads();  // run[] of the previous round is final; wc may be reused
    if (threadIdx.x < kPThreads / 64 * kMaxOwners) (&wc[0][0])[threadIdx.x] = 0;
    __syncthreads();
    if (in && below == 0) wc[w][o] = (uint32_t)__popcll(peers);
    __syncthreads();
    if (in) {
      uint32_t slot = run[o] + below;
      for (int q = 0; q < w; ++q) slot += wc[q][o];
      for (int c = 0; c < cols.n; ++c) {
        char* d = (char*)cols.dst[c] + (size_t)slot * cols.stride[c];
        switch (cols.width[c]) {
          case 4: *(uint32_t*)d = ((const uint32_t*)cols.src[c])[i]; break;
          case 8: *(uint64_t*)d = ((const uint64_t*)cols.src[c])[i]; break;
          case 2: *(uint16_t*)d = ((const uint16_t*)cols.src[c])[i]; break;
          default: *(uint8_t*)d = ((const uint8_t*)cols.src[c])[i]; break;
        }
      }
    }
    __syncthreads();
    if (threadIdx.x < world) {
      uint32_t t = 0;
      for (int q = 0; q < kPThreads / 64; ++q) t += wc[q][threadIdx.x];
      run[threadIdx.x] += t;
    }
  }
}

template <typename K>
void partition_impl(const K* keys, int64_t n, uint32_t world, const PartCols& cols, uint64_t* counts_host,
                    Scratch& sc, hipStream_t s) {
  const uint32_t ntiles = (uint32_t)((n + kPTile - 1) / kPTile);
  size_t mark = sc.used;
  uint32_t* cnt = (uint32_t*)sc.take((size_t)world * ntiles * 4 + 4);
  hipLaunchKernelGGL(owner_count_kernel<K>, dim3(ntiles), dim3(kPThreads), 0, s, keys, n, world, ntiles, cnt);
  // per-owner totals before the scan turns the counts into slots
  std::vector<uint32_t> h((size_t)world * ntiles);
  SM_HIP(hipMemcpyAsync(h.data(), cnt, h.size() * 4, hipMemcpyDeviceToHost, s));
  exclusive_scan_u32(cnt, (size_t)world * ntiles, sc, s);
  hipLaunchKernelGGL(owner_scatter_kernel<K>, dim3(ntiles), dim3(kPThreads), 0, s, keys, n, world, ntiles,
                     (const uint32_t*)cnt, cols);
  SM_HIP(hipStreamSynchronize(s));
  for (uint32_t o = 0; o < world; ++o) {
    uint64_t t = 0;
    for (uint32_t b = 0; b < ntiles; ++b) t += h[(size_t)o * ntiles + b];
    counts_host[o] = t;
  }
  sc.used = mark;
}

// per pair: one more match of its e2
__global__ void e2_count_kernel(const uint64_t* __restrict__ p, int64_t n, int64_t lo, uint32_t* __restrict__ cnt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) atomicAdd(&cnt[(int64_t)(p[i] >> 32) - lo], 1u);
}

// per pair: its place = matches of earlier e2 (scanned counts) + its rank among its e2's matches, which sit
// consecutively (one source run, e1 order) just before it
__global__ void e2_place_kernel(const uint64_t* __restrict__ p, int64_t n, int64_t lo, const uint32_t* __restrict__ off,
                                uint64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t v = p[i];
  const uint32_t j = (uint32_t)(v >> 32);
  int64_t r = 0;
  while (i - r - 1 >= 0 && (uint32_t)(p[i - r - 1] >> 32) == j) ++r;
  out[off[(int64_t)j - lo] + r] = v;
}

// Playback heartbeats of a rank (multi-GPU config 5): the received events (global ordinals ascending) merged with
// the global clock-advance points (ascending ordinals), a point at an ordinal this rank holds dropped (that event
// advances the clock itself). Merge path by binary search: a kept point's place = kept points before it + events
// with smaller ordinals; an event's place = its index + kept points with smaller ordinals.
__device__ __forceinline__ int64_t lower_bound_i64(const int64_t* __restrict__ a, int64_t n, int64_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__global__ void tick_keep_kernel(const int64_t* __restrict__ ord, int64_t n, const int64_t* __restrict__ tord,
                                 int64_t m, uint32_t* __restrict__ keep) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const int64_t lb = lower_bound_i64(ord, n, tord[j]);
  keep[j] = (lb < n && ord[lb] == tord[j]) ? 0u : 1u;
}

__global__ void tick_place_kernel(const int64_t* __restrict__ ord, int64_t n, const int64_t* __restrict__ tord,
                                  const int64_t* __restrict__ tts, int64_t m, const uint32_t* __restrict__ kpos,
                                  MergeOut o) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m || kpos[j + 1] == kpos[j]) return;  // dropped
  const int64_t p = (int64_t)kpos[j] + lower_bound_i64(ord, n, tord[j]);
  o.sid[p] = -1;
  o.ts[p] = tts[j];
  o.ord[p] = tord[j];  // the ordinal of the event that advanced the clock: the trigger of the timers it fires
  for (int c = 0; c < o.ncols; ++c) {
    char* d = (char*)o.dst[c];
    if (o.width[c] == 4) ((uint32_t*)d)[p] = 0u;
    else ((uint64_t*)d)[p] = 0ull;
  }
}

__global__ void event_place_kernel(const int64_t* __restrict__ ord, const int32_t* __restrict__ sid,
                                   const int64_t* __restrict__ ts, int64_t n, const int64_t* __restrict__ tord,
                                   int64_t m, const uint32_t* __restrict__ kpos, MergeOut o) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t p = i + (int64_t)kpos[lower_bound_i64(tord, m, ord[i])];
  o.sid[p] = sid[i];
  o.ts[p] = ts[i];
  o.ord[p] = ord[i];
  for (int c = 0; c < o.ncols; ++c) {
    const char* sc = (const char*)o.src[c];
    char* d = (char*)o.dst[c];
    if (o.width[c] == 4) ((uint32_t*)d)[p] = ((const uint32_t*)sc)[i];
    else ((uint64_t*)d)[p] = ((const uint64_t*)sc)[i];
  }
}

}  // namespace

int64_t merge_heartbeats(const int64_t* ord, const int32_t* sid, const int64_t* ts, int64_t n, const int64_t* tord,
                         const int64_t* tts, int64_t m, const MergeOut& o, Scratch& sc, hipStream_t s) {
  for (int c = 0; c < o.ncols; ++c)
    if (o.width[c] != 4 && o.width[c] != 8) throw std::invalid_argument("heartbeat merge: columns of 4 or 8 bytes");
  if (o.ncols > kMaxPartCols) throw std::invalid_argument("too many columns");
  const size_t mark = sc.used;
  uint32_t* kpos = (uint32_t*)sc.take((size_t)(m + 1) * 4);
  uint32_t kept = 0;
  if (m > 0) {
    hipLaunchKernelGGL(tick_keep_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, ord, n, tord, m, kpos);
    exclusive_scan_u32(kpos, (size_t)m, sc, s, kpos + m);
    SM_HIP(hipMemcpyAsync(&kept, kpos + m, 4, hipMemcpyDeviceToHost, s));
    hipLaunchKernelGGL(tick_place_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, ord, n, tord, tts, m,
                       (const uint32_t*)kpos, o);
  } else {
    SM_HIP(hipMemsetAsync(kpos, 0, 4, s));
  }
  if (n > 0)
    hipLaunchKernelGGL(event_place_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, ord, sid, ts, n, tord,
                       m, (const uint32_t*)kpos, o);
  SM_HIP(hipStreamSynchronize(s));
  sc.used = mark;
  return n + (int64_t)kept;
}

void order_matches(const uint64_t* pairs, int64_t n, int64_t lo, int64_t hi, uint64_t* out, Scratch& sc,
                   hipStream_t s) {
  if (n == 0) return;
  if (hi <= lo || hi - lo >= (int64_t)UINT32_MAX) throw std::invalid_argument("ordinal slice out of range");
  const size_t mark = sc.used;
  uint32_t* cnt = (uint32_t*)sc.take((size_t)(hi - lo) * 4 + 4);
  SM_HIP(hipMemsetAsync(cnt, 0, (size_t)(hi - lo) * 4, s));
  const dim3 g((unsigned)((n + 255) / 256));
  hipLaunchKernelGGL(e2_count_kernel, g, dim3(256), 0, s, pairs, n, lo, cnt);
  exclusive_scan_u32(cnt, (size_t)(hi - lo), sc, s);
  hipLaunchKernelGGL(e2_place_kernel, g, dim3(256), 0, s, pairs, n, lo, (const uint32_t*)cnt, out);
  SM_HIP(hipStreamSynchronize(s));
  sc.used = mark;
}

void partition_by_owner(const void* keys, int key_width, int64_t n, uint32_t world, const PartCols& cols,
                        uint64_t* counts_host, Scratch& sc, hipStream_t s) {
  if (world == 0 || world > (uint32_t)kMaxOwners) throw std::invalid_argument("world size must be 1..64");
  if (n >= (int64_t)UINT32_MAX) throw std::invalid_argument("partition batch too large (>= 2^32 events)");
  if (cols.n > kMaxPartCols) throw std::invalid_argument("too many columns");
  if (n == 0) {
    for (uint32_t o = 0; o < world; ++o) counts_host[o] = 0;
    return;
  }
  if (key_width == 4) partition_impl<int32_t>((const int32_t*)keys, n, world, cols, counts_host, sc, s);
  else if (key_width == 8) partition_impl<int64_t>((const int64_t*)keys, n, world, cols, counts_host, sc, s);
  else throw std::invalid_argument("partition keys must be 4- or 8-byte integers");
}

namespace {
// one thread per record: its words are loaded once (the wave's loads cover consecutive records, so every line is
// used whole), each field goes to its column with a coalesced store
__global__ void __launch_bounds__(256) unpack_records_kernel(const uint64_t* __restrict__ rec, int64_t m,
                                                             UnpackCols u) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  uint64_t w[8];
#pragma unroll
  for (int k = 0; k < 8; ++k)
    if (k < u.rec_words) w[k] = rec[i * u.rec_words + k];
  for (int c = 0; c < u.n; ++c) {
    const int o = u.off[c], wd = u.width[c];
    uint64_t x = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (k == (o >> 3)) x = w[k];
    x >>= (o & 7) * 8;
    if (c == u.ord_field) {
      // source run of record i (runs in rank order): its slice's first ordinal + the in-slice offset
      int lo = 0, hi = u.nsrc - 1;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (i < u.run_end[mid]) hi = mid;
        else lo = mid + 1;
      }
      u.ord_out[i] = u.src_first[lo] + (int64_t)(uint32_t)x;
    }
    void* d = u.dst[c];
    if (!d) continue;
    if (wd == 8) ((uint64_t*)d)[i] = x;
    else if (wd == 4) ((uint32_t*)d)[i] = (uint32_t)x;
    else if (wd == 2) ((uint16_t*)d)[i] = (uint16_t)x;
    else ((uint8_t*)d)[i] = (uint8_t)x;
  }
}
}  // namespace

void unpack_records(const uint64_t* rec, int64_t m, const UnpackCols& u, hipStream_t s) {
  if (m <= 0) return;
  hipLaunchKernelGGL(unpack_records_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, rec, m, u);
}

}  // namespace sm
