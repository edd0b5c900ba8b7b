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

// sorted keyed records shaped like config 4 after the key sort: runs of R records per key, ordinals increasing
// within a run, ts = ordinal / 10000, random value codes, c1 on ~80 %
__global__ void fill_sorted(uint4* r, int64_t n, int64_t K) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t R = n / K;
  const int64_t key = i / R, j = i % R;
  const uint64_t ord = (uint64_t)(j * K + key);
  uint64_t z = ord * 0x9E3779B97F4A7C15ull + 99;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z ^= z >> 31;
  const bool c1 = (z % 100) >= 20;
  r[i] = make_uint4((uint32_t)key | (c1 ? 0x80000000u : 0u), (uint32_t)ord, (uint32_t)(z >> 32),
                    (uint32_t)(ord / 10000));
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
static const char* kWalkPhase[6] = {"stage", "c1", "scan", "open scans", "ballots", "output"};
static const char** gPhase = kPhase;

static void report_stamps(const char* what) {
#ifdef SM_STAMPS
  unsigned long long h[16];
  CK(hipMemcpyFromSymbol(h, HIP_SYMBOL(sm_stamps), sizeof(h)));
  unsigned long long tot = 0;
  for (int i = 0; i < 6; ++i) tot += h[i];
  printf("  %s phase shares:", what);
  for (int i = 0; i < 6; ++i) printf(" %s %.1f%%", gPhase[i], tot ? 100.0 * h[i] / tot : 0.0);
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
  // write-combining record passes
  {
    int wwc = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&wwc, downsweep_wc_kernel<1, RecSrc>, kWcBlock, 0));
    const int Gc = (int)std::min<int64_t>((n + kTile - 1) / kTile, 2LL * wwc * cus);
    const int64_t perc = round_up((n + Gc - 1) / Gc, kTile);
    printf("wc: wgs/cu=%d G=%d per=%lld\n", wwc, Gc, (long long)perc);
    for (int shift = 0; shift < kbits; shift += kRB) {
      for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL((upsweep_kernel<RecDigits>), dim3(Gc), dim3(kBlock), 0, 0, RecDigits{A}, n, perc, Gc, shift,
                           cnt);
        hipLaunchKernelGGL(scan_chunks_kernel, dim3(kBins), dim3(256), 0, 0, cnt, Gc, dbase);
        hipLaunchKernelGGL(digit_base_kernel, dim3(1), dim3(kBlock), 0, 0, dbase);
        CK(hipEventRecord(e2));
        hipLaunchKernelGGL((downsweep_wc_kernel<1, RecSrc>), dim3(Gc), dim3(kWcBlock), 0, 0, RecSrc{A}, B, nullptr, n,
                           perc, nullptr, Gc, shift, cnt, dbase);
        CK(hipEventRecord(e3));
        CK(hipDeviceSynchronize());
        float dn = 0;
        CK(hipEventElapsedTime(&dn, e2, e3));
        printf("wc record pass shift %d: down %.3f ms (%.0f GB/s)\n", shift, dn, n * 32 / (dn * 1e-3) / 1e9);
        report_stamps("wc record");
      }
      if (shift == 0) {  // check: B is A stably ordered by the digit
        std::vector<uint4> ha(n), hb(n);
        CK(hipMemcpy(ha.data(), A, n * 16, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hb.data(), B, n * 16, hipMemcpyDeviceToHost));
        std::vector<int64_t> pos(kBins + 1, 0);
        for (int64_t i = 0; i < n; ++i) pos[((ha[i].x & kKeyMask) & (kBins - 1)) + 1]++;
        for (int d = 0; d < kBins; ++d) pos[d + 1] += pos[d];
        int64_t bad = 0;
        for (int64_t i = 0; i < n; ++i) {
          const uint4 r = ha[i], q = hb[pos[(r.x & kKeyMask) & (kBins - 1)]++];
          bad += q.x != r.x || q.y != r.y || q.z != r.z || q.w != r.w;
        }
        printf("wc record pass check: %lld mismatches\n", (long long)bad);
      }
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
  {
    int wwc = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&wwc, downsweep_wc_kernel<2, PairSrc>, kWcBlock, 0));
    const int Gc = (int)std::min<int64_t>((n + kTile - 1) / kTile, 2LL * wwc * cus);
    const int64_t perc = round_up((n + Gc - 1) / Gc, kTile);
    for (int rep = 0; rep < 3; ++rep) {
      hipLaunchKernelGGL((upsweep_kernel<PairDigits>), dim3(Gc), dim3(kBlock), 0, 0, PairDigits{P}, n, perc, Gc, 0, cnt);
      hipLaunchKernelGGL(scan_chunks_kernel, dim3(kBins), dim3(256), 0, 0, cnt, Gc, dbase);
      hipLaunchKernelGGL(digit_base_kernel, dim3(1), dim3(kBlock), 0, 0, dbase);
      CK(hipEventRecord(e2));
      hipLaunchKernelGGL((downsweep_wc_kernel<2, PairSrc>), dim3(Gc), dim3(kWcBlock), 0, 0, PairSrc{P}, nullptr, Q, n,
                         perc, nullptr, Gc, 0, cnt, dbase);
      CK(hipEventRecord(e3));
      CK(hipDeviceSynchronize());
      float dn = 0;
      CK(hipEventElapsedTime(&dn, e2, e3));
      printf("wc pair pass: down %.3f ms (%.0f GB/s)\n", dn, n * 16 / (dn * 1e-3) / 1e9);
      report_stamps("wc pair");
    }
    std::vector<uint64_t> hp(n), hq(n);
    CK(hipMemcpy(hp.data(), P, n * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hq.data(), Q, n * 8, hipMemcpyDeviceToHost));
    std::vector<int64_t> pos(kBins + 1, 0);
    for (int64_t i = 0; i < n; ++i) pos[((hp[i] >> 32) & (kBins - 1)) + 1]++;
    for (int d = 0; d < kBins; ++d) pos[d + 1] += pos[d];
    int64_t bad = 0;
    for (int64_t i = 0; i < n; ++i) bad += hq[pos[(hp[i] >> 32) & (kBins - 1)]++] != hp[i];
    printf("wc pair pass check: %lld mismatches\n", (long long)bad);
  }
  // walk over sorted records (keyed, c2 = e2 > e1 on exact codes)
  {
    const int64_t K = 1000000;
    hipLaunchKernelGGL(fill_sorted, dim3((n + 255) / 256), dim3(256), 0, 0, A, n, K);
    int wwpc = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&wwpc, walk_kernel<true, CMP_GT, false>, kWalkBlock, 0));
    const int Gw = (int)std::min<int64_t>((n + kWalkTile - 1) / kWalkTile, (int64_t)wwpc * cus);
    const int64_t perw = round_up((n + Gw - 1) / Gw, kWalkTile);
    uint32_t *mcount, *jcnt;  // per walk chunk (Gw may exceed the sort grid G the count buffer above is sized for)
    CK(hipMalloc(&mcount, 4ull * Gw));
    CK(hipMalloc(&jcnt, 4ull * kBins * Gw));
    NfaStream hs{};
    hs.nattr = 4;
    hs.types[1] = T_LONG;
    hs.cols[1] = A;  // never read: exact codes
    NfaStream* ds;
    CK(hipMalloc(&ds, sizeof(NfaStream)));
    CK(hipMemcpy(ds, &hs, sizeof(hs), hipMemcpyHostToDevice));
    WalkArgs wa{};
    wa.rec = A;
    wa.st = ds;
    wa.vattr = 1;
    wa.vtype = T_LONG;
    wa.within = 1000;
    wa.n = n;
    wa.exact_codes = true;
    gPhase = kWalkPhase;
    printf("walk: G=%d per=%lld wgs/cu=%d\n", Gw, (long long)perw, wwpc);
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(e2));
      if ((int64_t)Gw * perw < n) throw std::runtime_error("walk chunks do not cover the records");
      hipLaunchKernelGGL((walk_kernel<true, CMP_GT, false>), dim3(Gw), dim3(kWalkBlock), 0, 0, wa, perw, Gw, P, mcount,
                         jcnt);
      CK(hipEventRecord(e3));
      CK(hipDeviceSynchronize());
      float dn = 0;
      CK(hipEventElapsedTime(&dn, e2, e3));
      std::vector<uint32_t> hm(Gw);
      CK(hipMemcpy(hm.data(), mcount, 4ull * Gw, hipMemcpyDeviceToHost));
      long long M = 0;
      for (auto x : hm) M += x;
      printf("walk: %.3f ms, %lld matches (%.0f GB/s of 16 B/record + 8 B/match)\n", dn, M,
             (n * 16.0 + M * 8.0) / (dn * 1e-3) / 1e9);
      report_stamps("walk");
    }
  }
  return 0;
}
