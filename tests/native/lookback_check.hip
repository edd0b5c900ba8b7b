// Standalone GPU check + timing of the look-back primitives (kernels/lookback.h): every tile's exclusive
// prefix must equal the host prefix sum, for the serial, windowed and wave-parallel forms.
// Build: hipcc --offload-arch=gfx950 -O3 -o build/lookback_check lookback_check.hip ; run on the GPU box.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../siddhi_amd/csrc/kernels/lookback.h"

using namespace sm;

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(2);                                                                \
    }                                                                         \
  } while (0)

__host__ __device__ inline uint32_t cnt_of(uint32_t tile, uint32_t d) {
  uint32_t x = tile * 2654435761u ^ (d * 40503u + 17u);
  x ^= x >> 13;
  x *= 0x5bd1e995u;
  x ^= x >> 15;
  return x % 97u;
}

constexpr int kD = 1024;  // counters per tile for the per-digit forms

template <int FORM>
__global__ void __launch_bounds__(512) k_digits(unsigned long long* status, uint32_t epoch, unsigned* ctr,
                                                uint32_t* out, unsigned* err) {
  __shared__ unsigned sh;
  if (threadIdx.x == 0) sh = atomicAdd(ctr, 1u);
  __syncthreads();
  const uint32_t tile = sh;
  for (int d = threadIdx.x; d < kD; d += blockDim.x) {
    uint32_t e;
    if (FORM == 0) e = lookback(status + d, kD, tile, epoch, cnt_of(tile, d), err);
    else e = lookback_win<8>(status + d, kD, tile, epoch, cnt_of(tile, d), err);
    out[(size_t)tile * kD + d] = e;
  }
}

__global__ void __launch_bounds__(256) k_wave(unsigned long long* status, uint32_t epoch, unsigned* ctr,
                                              uint32_t* out, unsigned* err) {
  __shared__ unsigned sh;
  if (threadIdx.x == 0) sh = atomicAdd(ctr, 1u);
  __syncthreads();
  const uint32_t tile = sh;
  if (threadIdx.x < 64) {
    const uint32_t e = lookback_wave(status, tile, epoch, cnt_of(tile, 0), err);
    if (threadIdx.x == 0) out[tile] = e;
  }
}


int main(int argc, char** argv) {
  const int tiles = argc > 1 ? atoi(argv[1]) : 20000;
  unsigned long long* status;
  unsigned *ctr, *err;
  uint32_t* out;
  CK(hipMalloc(&status, (size_t)tiles * kD * 8));
  CK(hipMemset(status, 0, (size_t)tiles * kD * 8));
  CK(hipMalloc(&ctr, 16 * 4));
  CK(hipMalloc(&err, 4));
  CK(hipMalloc(&out, (size_t)tiles * kD * 4));
  std::vector<uint32_t> h((size_t)tiles * kD);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  int fails = 0;
  for (int form = 0; form < 3; ++form) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipMemset(ctr, 0, 64));
      CK(hipMemset(err, 0, 4));
      const uint32_t epoch = 1 + form * 2 + rep;
      CK(hipEventRecord(a));
      if (form == 0) hipLaunchKernelGGL(k_digits<0>, dim3(tiles), dim3(512), 0, 0, status, epoch, ctr, out, err);
      if (form == 1) hipLaunchKernelGGL(k_digits<1>, dim3(tiles), dim3(512), 0, 0, status, epoch, ctr, out, err);
      if (form == 2) hipLaunchKernelGGL(k_wave, dim3(tiles), dim3(256), 0, 0, status, epoch, ctr, out, err);
      CK(hipEventRecord(b));
      CK(hipDeviceSynchronize());
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      unsigned herr = 0;
      CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
      const int nd = form == 2 ? 1 : kD;
      CK(hipMemcpy(h.data(), out, (size_t)tiles * kD * 4, hipMemcpyDeviceToHost));
      int bad = 0;
      for (int d = 0; d < nd; ++d) {
        uint32_t run = 0;
        for (int t = 0; t < tiles; ++t) {
          const uint32_t got = form == 2 ? h[t] : h[(size_t)t * kD + d];
          if (got != run && bad++ < 5) printf("  form %d digit %d tile %d: got %u want %u\n", form, d, t, got, run);
          run += cnt_of(t, d);
        }
      }
      printf("form %d (%s) tiles %d: %.3f ms, err=%u, %s\n", form,
             form == 0 ? "serial" : form == 1 ? "window8" : "wave", tiles, ms, herr, bad ? "MISMATCH" : "ok");
      fails += bad != 0 || herr != 0;
    }
  }
  printf(fails ? "FAILED\n" : "PASSED\n");
  return fails ? 1 : 0;
}
