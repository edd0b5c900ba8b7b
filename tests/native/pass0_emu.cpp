// Host wave emulator of key pass 0 (siddhi_amd/csrc/kernels/pass0_dev.h, pass0_kernel): the SAME device source,
// compiled for the host with SM_HOST_EMU (hd.h), over precomputed 16-byte records. Test infrastructure only
// (tests/test_pass0_emu.py: the output must be the stable partition of the records by their low key digit).
#define SM_HOST_EMU 1
#include "../../siddhi_amd/csrc/kernels/pass0_dev.h"

#include "emu_fibers.h"

namespace {
struct RecSrcEmu {  // records already built: pass 0 moves them
  const uint4* r;
  typedef uint4 Raw;
  void init() {}
  void flush() {}
  Raw load(int64_t p) const { return r[p]; }
  uint4 record(const Raw& x, int64_t) const { return x; }
};
}  // namespace

extern "C" int sm_pass0_emu(const uint32_t* rec, int64_t n, int64_t per, int G, const uint32_t* cnt,
                            const uint32_t* dbase, uint32_t* out) {
  using namespace sm;
  RecSrcEmu src{(const uint4*)rec};
  emu_launch(G, kP0Block, [&] { pass0_kernel<RecSrcEmu>(src, (uint4*)out, n, per, G, cnt, dbase); });
  return 0;
}
