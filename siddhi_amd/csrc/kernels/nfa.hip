// HIP launch wrapper of the NFA interpreter (implementation in nfa_impl.h).
#include "nfa_impl.h"
#include "primitives.h"

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

// The common record shape (16 words = one 128-byte line): each thread builds the record of its batch position in
// LDS, then groups of 8 lanes store one record each (8 x 16 B), so a wave's store instruction writes 8 whole lines
// instead of touching 64 (one 16-byte piece of each of 64 scattered records per instruction).
constexpr int kLeBlock = 256;
constexpr int kLeStride = 18;  // words per LDS row: 16 + 2 of padding (rows start on rotating banks)
__global__ void __launch_bounds__(kLeBlock) lane_events16_kernel(NfaBatch b, int64_t n, const int32_t* __restrict__ inv,
                                                               int32_t node_words, int64_t* __restrict__ out) {
  __shared__ int64_t lrec[kLeBlock * kLeStride];
  __shared__ int32_t lk[kLeBlock];
  const int tid = threadIdx.x;
  const int64_t p = (int64_t)blockIdx.x * kLeBlock + tid;
  const int32_t k = p < n ? inv[p] : -1;
  lk[tid] = k;
  if (k >= 0) lane_event_record(b, p, 0, node_words, lrec + tid * kLeStride);
  __syncthreads();
  const int piece = tid & 7;
#pragma unroll 4
  for (int r = tid >> 3; r < kLeBlock; r += kLeBlock / 8) {
    const int32_t kr = lk[r];
    if (kr >= 0) {
      const longlong2 v = *(const longlong2*)(lrec + r * kLeStride + 2 * piece);
      *((longlong2*)(out + (int64_t)kr * 16) + piece) = v;
    }
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

}  // namespace

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
                        hipStream_t s) {
  if (nq <= 0) return;
  if (nq >= INT32_MAX) throw std::runtime_error("query batch too large for the lane-event index (>= 2^31 records)");
  // positions outside the query's records stay -1; when the query keeps every record, lane_index writes them all
  if (nq < n) SM_HIP(hipMemsetAsync(inv_scratch, 0xff, (size_t)n * 4, s));
  hipLaunchKernelGGL(lane_index_kernel, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, s, b.key_pos, nq,
                     inv_scratch);
  if (LaneEv::words(node_words) == 16)
    hipLaunchKernelGGL(lane_events16_kernel, dim3((unsigned)((n + kLeBlock - 1) / kLeBlock)), dim3(kLeBlock), 0, s, b,
                       n, (const int32_t*)inv_scratch, node_words, (int64_t*)b.lane_ev);
  else
    hipLaunchKernelGGL(lane_events_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, b, n,
                       (const int32_t*)inv_scratch, node_words, (int64_t*)b.lane_ev);
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
