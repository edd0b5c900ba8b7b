// HIP launch wrapper of the NFA interpreter (implementation in nfa_impl.h).
#include "nfa_impl.h"

namespace sm {
namespace {

__global__ void nfa_kernel(NfaBatch b, const char* __restrict__ blob, int64_t* ks_all, int64_t* heap_all,
                           int32_t heap_half, int64_t lanes, int32_t nkeys, int32_t* err_out) {
  int key = blockIdx.x * blockDim.x + threadIdx.x;
  if (key >= nkeys) return;
  nfa_lane(b, blob, ks_all, heap_all, heap_half, lanes, key, err_out);
}

}  // namespace

void launch_nfa(const NfaBatch& b, const char* blob_dev, int64_t* ks, int64_t* heap, int32_t heap_half,
                int64_t lanes, int32_t nkeys, int32_t* err_dev, hipStream_t s) {
  if (nkeys <= 0) return;
  int threads = 64;
  int blocks = (nkeys + threads - 1) / threads;
  hipLaunchKernelGGL(nfa_kernel, dim3(blocks), dim3(threads), 0, s, b, blob_dev, ks, heap, heap_half, lanes, nkeys,
                     err_dev);
}

}  // namespace sm
