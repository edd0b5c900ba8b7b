// Host wave emulator of the bucket-stack ring kernel (siddhi_amd/csrc/kernels/stack_dev.h, stack4_kernel): the SAME
// device source, compiled for the host with SM_HOST_EMU (hd.h): every GPU thread of a workgroup is a fiber of one host
// thread, wave64 operations are barriers of a wave's fibers. Test infrastructure only (tests/test_stack_emu.py): it lets the kernel's
// ranking, ring hand-off, pop log and emission be checked against a plain pending-list model on the CPU, and lets a
// fault be found with AddressSanitizer instead of on the GPU.
#define SM_HOST_EMU 1
#include "../../siddhi_amd/csrc/kernels/stack_dev.h"
#include "../../siddhi_amd/csrc/kernels/order_dev.h"

#include "emu_fibers.h"

extern "C" {

// One launch of stack4_kernel<CMP_GT, FP = true> over bucketed records (pass-0 layout). Carried partials: rows
// [key, ordinal, ts, value bits] (w = 4) sorted by (key, ordinal), or nc = 0. Returns 0.
int sm_stack4_emu(const uint32_t* rec, const uint32_t* dbase, uint32_t n, int H, int32_t within, uint32_t ntiles,
                  int grid, const double* vcol, int64_t kmin, int64_t ts0, int64_t obase, int32_t o0,
                  const uint32_t* cin, const uint32_t* cstart, const uint32_t* cend, const int64_t* crow,
                  const uint32_t* sbase, uint64_t* stage, uint32_t* mstart, uint32_t* mtot, int64_t* cand,
                  uint32_t cand_cap, uint32_t* cand_n, uint32_t* err, uint4* spill) {
  using namespace sm;
  Stack4Cold c4{};
  c4.kmin = kmin;
  c4.ts0 = ts0;
  c4.within = within;
  c4.obase = obase;
  c4.n = n;
  c4.vtype = T_DOUBLE;
  c4.vattr = 0;
  c4.cwidth = 4;
  c4.o0 = o0;
  c4.exact_codes = false;
  c4.vcol = vcol;
  c4.ord = nullptr;
  c4.cin = (const uint4*)cin;
  c4.cstart = cstart;
  c4.cend = cend;
  c4.crow = crow;
  c4.cand = cand;
  c4.cand_n = cand_n;
  c4.cand_cap = cand_cap;
  Stack4Args a{};
  a.rec = (const uint4*)rec;
  a.dbase = dbase;
  a.n = n;
  a.H = H;
  a.within = within;
  a.exact_codes = false;
  a.ntiles = ntiles;
  a.sbase = sbase;
  a.stage = stage;
  a.mstart = mstart;
  a.mtot = mtot;
  a.spill = spill;
  a.err = err;
  a.cold = &c4;
  emu_launch(grid, kT4, [&] { stack4_kernel<CMP_GT, true>(a); });
  return 0;
}

int sm_stack4_emu_consts(int* out) {  // kBins, kKeys, kTB, kQ, kSS, kR, kC
  using namespace sm;
  out[0] = kBins;
  out[1] = kKeys;
  out[2] = kTB;
  out[3] = kQ;
  out[4] = kSS;
  out[5] = kR;
  out[6] = kC;
  return 0;
}

// One launch of order2_kernel (order_dev.h) over staged matches: bucket d's run at stage[sbase[d] ..), mt[t][d] =
// matches of bucket d whose j precedes tile t (ntiles + 1 rows of kBins). Returns the kernel's image capacity.
int sm_order2_emu(const uint64_t* stage, const uint32_t* sbase, const uint32_t* mt, int64_t ntiles, uint64_t* out) {
  using namespace sm;
  OrderArgs a{};
  a.stage = stage;
  a.sbase = sbase;
  a.mt = mt;
  a.ntiles = ntiles;
  a.out = out;
  emu_launch((int)((ntiles + kGT2 - 1) / kGT2), kOB, [&] { order2_kernel(a); });
  return kOC2;
}
}
