// Micro-benchmark of the fast path's LSD passes (test infrastructure, diagnostic): one key-record pass
// (MODE 1) and one pair pass (MODE 2) over synthetic data, timed with HIP events, plus the phase shares of
// the down-sweep tile loop from s_memtime stamps (SM_STAMPS build; read the shares, not the times).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -DSM_STAMPS -I../../siddhi_amd/csrc -o build/micro_sort
//        micro_sort.hip   (tests/native/Makefile target micro)
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "kernels/fastpath3.hip"

using namespace sm;

#define CK(x) SM_HIP(x)

__global__ void fill_kernel(uint4* r, int64_t n, int kbits) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + 12345;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  r[i] = make_uint4((uint32_t)(z & ((1u << kbits) - 1)) | ((z >> 40) & 1 ? 0x80000000u : 0u), (uint32_t)i,
                    (uint32_t)(z >> 32), (uint32_t)(i / 10000));
}

__global__ void fill_pairs(uint64_t* q, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + 777;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z ^= z >> 31;
  q[i] = ((z % (uint64_t)n) << 32) | (uint32_t)i;
}

static const char* kPhase[6] = {"loads+zero", "rank", "digit scan", "key xchg+store", "payload xchg", "tail"};

static void report_stamps(const char* what) {
#ifdef SM_STAMPS
  unsigned long long h[16];
  CK(hipMemcpyFromSymbol(h, HIP_SYMBOL(sm_stamps), sizeof(h)));
  unsigned long long tot = 0;
  for (int i = 0; i < 6; ++i) tot += h[i];
  printf("  %s phase shares:", what);
  for (int i = 0; i < 6; ++i) printf(" %s %.1f%%", kPhase[i], tot ? 100.0 * h[i] / tot : 0.0);
  printf("\n");
  unsigned long long z[16] = {};
  CK(hipMemcpyToSymbol(HIP_SYMBOL(sm_stamps), z, sizeof(z)));
#else
  (void)what;
#endif
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 100000000;
  const int kbits = argc > 2 ? atoi(argv[2]) : 20;
  int dev = 0, cus = 0, wpc = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&wpc, downsweep_kernel<1, RecSrc>, kBlock, 0));
  const int G = (int)std::min<int64_t>((n + kTile - 1) / kTile, 2LL * wpc * cus);
  const int64_t per = round_up((n + G - 1) / G, kTile);
  printf("n=%lld cus=%d wgs/cu=%d G=%d per=%lld\n", (long long)n, cus, wpc, G, (long long)per);
  uint4 *A, *B;
  CK(hipMalloc(&A, n * 16));
  CK(hipMalloc(&B, n * 16));
  uint32_t *cnt, *dbase;
  CK(hipMalloc(&cnt, 4ull * kBins * G));
  CK(hipMalloc(&dbase, 4ull * kBins));
  hipLaunchKernelGGL(fill_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, A, n, kbits);
  hipEvent_t e0, e1, e2, e3;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&e2));
  CK(hipEventCreate(&e3));
  for (int shift = 0; shift < kbits; shift += kRB) {
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL((upsweep_kernel<RecDigits>), dim3(G), dim3(kBlock), 0, 0, RecDigits{A}, n, per, G, shift, cnt);
      CK(hipEventRecord(e1));
      hipLaunchKernelGGL(scan_chunks_kernel, dim3(kBins), dim3(256), 0, 0, cnt, G, dbase);
      hipLaunchKernelGGL(digit_base_kernel, dim3(1), dim3(kBlock), 0, 0, dbase);
      CK(hipEventRecord(e2));
      hipLaunchKernelGGL((downsweep_kernel<1, RecSrc>), dim3(G), dim3(kBlock), 0, 0, RecSrc{A}, B, nullptr, n, per,
                         nullptr, G, shift, cnt, dbase);
      CK(hipEventRecord(e3));
      CK(hipDeviceSynchronize());
      float up = 0, sc = 0, dn = 0;
      CK(hipEventElapsedTime(&up, e0, e1));
      CK(hipEventElapsedTime(&sc, e1, e2));
      CK(hipEventElapsedTime(&dn, e2, e3));
      printf("record pass shift %d: up %.3f ms (%.0f GB/s)  scan %.3f ms  down %.3f ms (%.0f GB/s)\n", shift, up,
             n * 4 / (up * 1e-3) / 1e9, sc, dn, n * 32 / (dn * 1e-3) / 1e9);
      report_stamps("record");
    }
  }
  // pairs pass
  uint64_t *P, *Q;
  CK(hipMalloc(&P, n * 8));
  CK(hipMalloc(&Q, n * 8));
  hipLaunchKernelGGL(fill_pairs, dim3((n + 255) / 256), dim3(256), 0, 0, P, n);
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((upsweep_kernel<PairDigits>), dim3(G), dim3(kBlock), 0, 0, PairDigits{P}, n, per, G, 0, cnt);
    hipLaunchKernelGGL(scan_chunks_kernel, dim3(kBins), dim3(256), 0, 0, cnt, G, dbase);
    hipLaunchKernelGGL(digit_base_kernel, dim3(1), dim3(kBlock), 0, 0, dbase);
    CK(hipEventRecord(e2));
    hipLaunchKernelGGL((downsweep_kernel<2, PairSrc>), dim3(G), dim3(kBlock), 0, 0, PairSrc{P}, nullptr, Q, n, per,
                       nullptr, G, 0, cnt, dbase);
    CK(hipEventRecord(e3));
    CK(hipDeviceSynchronize());
    float dn = 0;
    CK(hipEventElapsedTime(&dn, e2, e3));
    printf("pair pass: down %.3f ms (%.0f GB/s)\n", dn, n * 16 / (dn * 1e-3) / 1e9);
    report_stamps("pair");
  }
  return 0;
}
