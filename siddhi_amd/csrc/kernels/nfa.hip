// HIP launch wrapper of the NFA interpreter (implementation in nfa_impl.h).
#include "nfa_impl.h"
#include "primitives.h"

#include <algorithm>
#include <cstdlib>

namespace sm {
namespace {

// SM_NFA_WAVES (A/B builds): minimum waves per SIMD the register allocator must leave room for
#ifdef SM_NFA_WAVES
#define SM_NFA_ATTR __attribute__((amdgpu_waves_per_eu(SM_NFA_WAVES)))
#else
#define SM_NFA_ATTR
#endif

__global__ SM_NFA_ATTR void nfa_kernel(NfaBatch b, const char* __restrict__ blob, int64_t* ks_all, int64_t* heap_all,
                           int32_t heap_half, int64_t lanes, int32_t nkeys, int32_t* err_out) {
  const int lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= nkeys) return;
  const int key = b.lane_perm ? (int)b.lane_perm[lane] : lane;
  nfa_lane(b, blob, ks_all, heap_all, heap_half, lanes, key, err_out);
}

__global__ void pool_compact_kernel(int pass, const char* __restrict__ blob, int64_t* ks_all, int64_t* heap_all,
                                    int32_t heap_half, int64_t lanes, int32_t nkeys, int64_t* old_pool,
                                    int64_t* new_pool, unsigned long long* new_top, int64_t* new_off) {
  const int key = blockIdx.x * blockDim.x + threadIdx.x;
  if (key >= nkeys) return;
  nfa_pool_lane(blob, ks_all, heap_all, heap_half, lanes, key, pass, old_pool, new_pool, new_top, new_off);
}

// Gather each record of the query's batch, in key order, into its LaneEv record: a lane then reads one
// contiguous record per event instead of chasing key_pos -> stream / row / ts / clock / ordinal / columns.
// Key order -> batch position is a permutation (key_pos); build the records in batch-position order instead, so
// the column reads are coalesced and each record (one line-sized store burst) goes to its key-order slot.
__global__ void lane_index_kernel(const int64_t* __restrict__ key_pos, int64_t nq, int32_t* __restrict__ inv) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < nq) inv[key_pos[k]] = (int32_t)k;
}

__global__ void lane_events_kernel(NfaBatch b, int64_t n, const int32_t* __restrict__ inv, int32_t node_words,
                                   int64_t* __restrict__ out) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const int32_t k = inv[p];
  if (k >= 0) lane_event_record(b, p, k, node_words, out);
}

// The common record shapes (16 words = one 128-byte line; the compact form, 8 words = 64 bytes): each thread builds
// the record of its batch position in LDS, then groups of WORDS / 2 lanes store one record each (16 B per lane), so a
// wave's store instruction writes whole records (8 lines / 16 half-lines) instead of touching 64 (one 16-byte piece
// of each of 64 scattered records per instruction).
constexpr int kLeBlock = 256;
template <int WORDS>
__global__ void __launch_bounds__(kLeBlock) lane_events_lds_kernel(NfaBatch b, int64_t n, const int32_t* __restrict__ inv,
                                                                   int32_t node_words, int nstreams,
                                                                   int64_t* __restrict__ out) {
  constexpr int kStride = WORDS + 2;  // words per LDS row: 2 of padding (rows start on rotating banks)
  constexpr int kPieces = WORDS / 2;  // 16-byte pieces per record
  __shared__ int64_t lrec[kLeBlock * kStride];
  __shared__ int32_t lk[kLeBlock];
  __shared__ NfaStream lst[kLdsStreams];  // the batch's stream descriptors (each record reads its stream's)
  const int tid = threadIdx.x;
  if (nstreams <= kLdsStreams) {
    const int words = nstreams * (int)(sizeof(NfaStream) / 8);
    for (int q = tid; q < words; q += kLeBlock) ((uint64_t*)lst)[q] = ((const uint64_t*)b.streams)[q];
    __syncthreads();
    b.streams = lst;
  }
  const int64_t p = (int64_t)blockIdx.x * kLeBlock + tid;
  const int32_t k = p < n ? inv[p] : -1;
  lk[tid] = k;
  if (k >= 0) lane_event_record(b, p, 0, node_words, lrec + tid * kStride);
  __syncthreads();
  const int piece = tid % kPieces;
#pragma unroll 4
  for (int r = tid / kPieces; r < kLeBlock; r += kLeBlock / kPieces) {
    const int32_t kr = lk[r];
    if (kr >= 0) {
      const longlong2 v = *(const longlong2*)(lrec + r * kStride + 2 * piece);
      *((longlong2*)(out + (int64_t)kr * WORDS) + piece) = v;
    }
  }
}

// lo / hi of the data events' ordinals (markers carry -1): one atomic pair per workgroup
// range of the data events' ordinals (a heartbeat's entry, stream < 0, carries no event ordinal and is skipped)
__global__ void __launch_bounds__(256) ord_range_kernel(const int64_t* __restrict__ ord, const int32_t* __restrict__ sid,
                                                        int64_t n, unsigned long long* __restrict__ mm) {
  uint64_t lo = ~0ull, hi = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t o = ord[i];
    if (o >= 0 && sid[i] >= 0) {
      lo = (uint64_t)o < lo ? (uint64_t)o : lo;
      hi = (uint64_t)o > hi ? (uint64_t)o : hi;
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t l2 = __shfl_xor(lo, off, 64), h2 = __shfl_xor(hi, off, 64);
    lo = l2 < lo ? l2 : lo;
    hi = h2 > hi ? h2 : hi;
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMin(&mm[0], (unsigned long long)lo);
    atomicMax(&mm[1], (unsigned long long)hi);
  }
}

// sort key of slot k: 65535 - min(events of k in this batch, 65535) (descending count)
__global__ void lane_count_kernel(const int64_t* __restrict__ key_off, int32_t nkeys, uint32_t* __restrict__ ck,
                                  uint32_t* __restrict__ slot) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nkeys) return;
  const int64_t c = key_off[k + 1] - key_off[k];
  ck[k] = 65535u - (uint32_t)(c < 65535 ? c : 65535);
  slot[k] = (uint32_t)k;
}

__global__ void clock_index_kernel(const int64_t* __restrict__ clk, int64_t n, int64_t cmin, int64_t span,
                                   int32_t* __restrict__ idx) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= span) return;
  const int64_t x = cmin + c;
  int64_t lo = 0, hi = n;  // first a with clk[a] >= x
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (clk[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  idx[c] = (int32_t)lo;
}

}  // namespace

void launch_clock_index(const int64_t* adv_clock, int64_t nadv, int64_t cmin, int64_t span, int32_t* idx,
                        hipStream_t s) {
  if (span <= 0) return;
  hipLaunchKernelGGL(clock_index_kernel, dim3((unsigned)((span + 255) / 256)), dim3(256), 0, s, adv_clock, nadv, cmin,
                     span, idx);
}

void launch_lane_balance(const int64_t* key_off, int32_t nkeys, uint32_t* perm, Scratch& sc, hipStream_t s) {
  if (nkeys <= 0) return;
  size_t mark = sc.used;
  uint32_t* ck = (uint32_t*)sc.take((size_t)nkeys * 4);
  uint32_t* ck2 = (uint32_t*)sc.take((size_t)nkeys * 4);
  uint32_t* v2 = (uint32_t*)sc.take((size_t)nkeys * 4);
  hipLaunchKernelGGL(lane_count_kernel, dim3((unsigned)((nkeys + 255) / 256)), dim3(256), 0, s, key_off, nkeys, ck,
                     perm);
  if (radix_sort_pairs<uint32_t>(ck, ck2, perm, v2, (size_t)nkeys, 0, 16, sc, s))
    SM_HIP(hipMemcpyAsync(perm, v2, (size_t)nkeys * 4, hipMemcpyDeviceToDevice, s));
  sc.used = mark;
}

void launch_lane_events(const NfaBatch& b, int64_t n, int64_t nq, int32_t node_words, int32_t* inv_scratch,
                        int nstreams, hipStream_t s) {
  if (nq <= 0) return;
  if (nq >= INT32_MAX) throw std::runtime_error("query batch too large for the lane-event index (>= 2^31 records)");
  // positions outside the query's records stay -1; when the query keeps every record, lane_index writes them all
  if (nq < n) SM_HIP(hipMemsetAsync(inv_scratch, 0xff, (size_t)n * 4, s));
  hipLaunchKernelGGL(lane_index_kernel, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, s, b.key_pos, nq,
                     inv_scratch);
  if (b.lane_compact)
    hipLaunchKernelGGL(lane_events_lds_kernel<8>, dim3((unsigned)((n + kLeBlock - 1) / kLeBlock)), dim3(kLeBlock), 0, s,
                       b, n, (const int32_t*)inv_scratch, node_words, nstreams, (int64_t*)b.lane_ev);
  else if (LaneEv::words(node_words) == 16)
    hipLaunchKernelGGL(lane_events_lds_kernel<16>, dim3((unsigned)((n + kLeBlock - 1) / kLeBlock)), dim3(kLeBlock), 0,
                       s, b, n, (const int32_t*)inv_scratch, node_words, nstreams, (int64_t*)b.lane_ev);
  else
    hipLaunchKernelGGL(lane_events_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, b, n,
                       (const int32_t*)inv_scratch, node_words, (int64_t*)b.lane_ev);
}

bool lane_compact_ok(const NfaBatch& b, int64_t n, int32_t node_words, int nstreams, Scratch& sc, hipStream_t s,
                     int64_t* ord_base) {
  static const char* env = getenv("SM_LANE_COMPACT");  // A/B: 0 keeps the 128-byte records
  if (env && atoi(env) == 0) return false;
  if (node_words > 8 || n >= ((int64_t)1 << 31) || b.nadv >= ((int64_t)1 << 31) || nstreams > 127) return false;
  *ord_base = 0;
  if (n == 0) return true;
  const size_t mark = sc.used;
  unsigned long long* mm = (unsigned long long*)sc.take(16);
  const unsigned long long init[2] = {~0ull, 0ull};
  SM_HIP(hipMemcpyAsync(mm, init, 16, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(ord_range_kernel, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 1024)), dim3(256), 0, s,
                     b.ev_ord, b.ev_stream, n, mm);
  unsigned long long h[2];
  SM_HIP(hipMemcpyAsync(h, mm, 16, hipMemcpyDeviceToHost, s));
  SM_HIP(hipStreamSynchronize(s));
  sc.used = mark;
  if (h[0] > h[1]) return true;  // no data event
  if (h[1] - h[0] >= kLeOrdMask) return false;
  *ord_base = (int64_t)h[0];
  return true;
}

void launch_pool_compact(int pass, const char* blob_dev, int64_t* ks, int64_t* heap, int32_t heap_half, int64_t lanes,
                         int32_t nkeys, int64_t* old_pool, int64_t* new_pool, unsigned long long* new_top,
                         int64_t* new_off, hipStream_t s) {
  if (nkeys <= 0) return;
  hipLaunchKernelGGL(pool_compact_kernel, dim3((unsigned)((nkeys + 255) / 256)), dim3(256), 0, s, pass, blob_dev, ks,
                     heap, heap_half, lanes, nkeys, old_pool, new_pool, new_top, new_off);
}

void launch_nfa(const NfaBatch& b, const char* blob_dev, int64_t* ks, int64_t* heap, int32_t heap_half,
                int64_t lanes, int32_t nkeys, int32_t* err_dev, hipStream_t s) {
  if (nkeys <= 0) return;
  int threads = 64;
  int blocks = (nkeys + threads - 1) / threads;
  hipLaunchKernelGGL(nfa_kernel, dim3(blocks), dim3(threads), 0, s, b, blob_dev, ks, heap, heap_half, lanes, nkeys,
                     err_dev);
}

}  // namespace sm
