// Bucket-stack pipeline for `partition with (k of S) begin from every e1=S[c1] -> e2=S[c2] within T end` with
// c2 = `e2.x OP e1.x`, OP one of > >= < <=.
//
// Why a stack. Per key, the reference keeps the e2 pre-processor's pending list in spawn order
// (StreamPreStateProcessor.addState :208-221, updateState :268-271). An arriving event j walks that list
// (processAndReturn :274-327): a partial whose e1 is more than T older than j is dropped (isExpired :102-121),
// one that satisfies c2 emits and leaves (stateChanged), the rest stay; then j's own partial is appended
// (e2 runs before e1: PatternMultiProcessStreamReceiver :39-45). Expired partials are a prefix of the list
// (event time is non-decreasing) and, for an order compare, the partials c2 accepts are a suffix: after j the
// list is monotone in the compared value (non-increasing for >, strictly decreasing for >=, mirrored for < <=),
// so j accepts exactly the run of partials at the young end that it beats. The pending list is therefore a
// monotone stack: pop while c2 holds (emitting in pop order, i.e. youngest e1 first), push j if c1. Expiry
// is applied lazily: a popped candidate that has expired means every older one has too.
//
// Pipeline after key pass 0 (fastpath3.hip) has scattered the records into kBins buckets by the low key
// digit (stable, so each bucket is in arrival order):
//   stack_kernel  one workgroup per bucket (persistent), thread t owns in-bucket key h = t. The bucket is read
//                 once, in slices of kS records: the slice is ranked by key in LDS (wave64 ballot peer masks),
//                 every thread runs its key's events of the slice against its stack (top kC entries in
//                 registers, older ones spilled to a per-thread HBM ring), the matches of the slice are put in
//                 arrival order of j (count per j, block scan, placement) and written to the bucket's staging
//                 run. Per (bucket, pass-0 chunk) the staging offset of the chunk's first j is recorded.
//   order_kernel  per pass-0 chunk, tile by tile in arrival order: each thread owns one bucket and reads that
//                 bucket's staged matches whose j falls in the tile (they are contiguous and in j order); a tile
//                 count / scan / placement interleaves them by j. The output (i, j) pairs are written once,
//                 in reference order (j, then i).
// HBM traffic: records 16 B/event read, staged matches 8 B written + 8 B read, output 8 B per match. No sort by
// j is needed: pass 0's bucket layout is inverted exactly, by ordinal ranges.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "fastpath.h"
#include "stack_dev.h"
#include "order_dev.h"

namespace sm {

namespace {

#ifndef SM_STACK_KPT
#define SM_STACK_KPT 2          // A/B build flag: in-bucket keys per thread (2: 512 threads and a 256-VGPR budget for
#endif                          // both stacks; 1: 1024 threads, 4 waves per SIMD)
constexpr int kKPT = SM_STACK_KPT;
constexpr int kSB = kKeys / kKPT;  // threads per bucket workgroup: thread t owns in-bucket keys t (and t + kSB)
constexpr int kSW = kSB / 64;
#ifndef SM_STACK_KSI
#define SM_STACK_KSI (SM_STACK_KPT == 2 ? 9 : 4)  // A/B build flag (config 4 stack kernel: 8 -> 33.2 ms, 9 -> 32.2 ms)
#endif
constexpr int kSI = SM_STACK_KSI;  // records per thread per slice
constexpr int kS = kSB * kSI;      // slice: 4608 records
constexpr int kLog = 4096;     // match log of a slice: kLog / H entries per key thread ...
constexpr int kOvf = 1024;     // ... and a shared overflow (more: the batch takes the sort / walk kernels)
// matches of a tile staged in LDS before one coalesced write (what the tile counts leave of the LDS; none for tiles of
// 2^15 ordinals, whose direct writes land in a ~190 KB window that the L2 combines)
// (tiles of 2^14 ordinals counted in packed u16 pairs, to keep the image in LDS, were exact and ran 22.9 ms against
// 6.5: adjacent ordinals' atomics then hit one LDS word)
// Round 6, measured and not kept: tiles of 2^14 ordinals (SM_ORDER_TB=14) with u32 counts, placed into the LDS image one
// half (2^13 ordinals) at a time (kSplit passes of the placement), so that a bucket's segment of a tile is twice as long
// (about 11 matches) and the line it shares with the next tile's segment, which comes back from HBM (VERDICT r05 #2:
// the kernel reads 3.8x its staged bytes), is read half as often per match: exact (order tiles, device stream / batch,
// sparse keys, bench-shape tests green), but 9.6 against 6.7 ms on the same box (the second placement pass over the
// segments costs more than the boundary lines it saves; a 64 KB count array leaves one workgroup per CU).
#ifndef SM_ORDER_SPLIT
#define SM_ORDER_SPLIT (SM_ORDER_TB >= 14 ? 2 : 1)
#endif
constexpr int kSplit = SM_ORDER_SPLIT;  // placement passes per tile, each into the image
constexpr int kOHB = kTB - (kSplit == 2 ? 1 : 0);  // log2 of the ordinals per placement pass
static_assert(kSplit == 1 || kSplit == 2, "one or two placement passes");
constexpr int kOCapMax = (160 * 1024 - kOT * 4 - 2 * kBins * 4 - 256) / 8;
constexpr int kOCap = kOCapMax >= 12288 ? 12288 : (kOCapMax >= 8192 ? kOCapMax : 0);
#ifndef SM_ORDER_GT
#define SM_ORDER_GT (SM_ORDER_TB >= 15 ? 4 : SM_ORDER_TB == 14 ? 8 : 16)  // A/B build flag
#endif
constexpr int kGT = SM_ORDER_GT;  // consecutive tiles per order workgroup
#ifndef SM_ORDER_V1
#define SM_ORDER_V1 0  // A/B build flag: 1 = this round-3 order kernel instead of order2_kernel (order_dev.h)
#endif
#ifndef SM_ORDER_XCD
#define SM_ORDER_XCD 0  // A/B build flag: 1 = XCD-contiguous tile groups (blocks b and b + 8 share an XCD and its L2)
#endif

static_assert(kBins == kKeys && kKeys == kKPT * kSB && kBins == kOB && (kKPT == 1 || kKPT == 2),
              "one or two in-bucket keys per thread, one bucket per order thread");
static_assert(kSW * kKeys * 2 <= kLog * 8, "the per-wave key counts of the ranking fit the match log area");

#ifndef SM_STACK_STAMPS_BUILD
#define SM_STACK_STAMPS_BUILD 0  // build flag: phase clock + counters of the stack kernel (env SM_STACK_STAMPS=1 reads them)
#endif
constexpr bool kStamps = SM_STACK_STAMPS_BUILD != 0;

struct StackArgs {
  const uint4* rec;
  const uint32_t* dbase;
  int64_t ntiles;  // order tiles: relative ordinals [0, ntiles << kTB)
  int64_t n;
  int H;
  int64_t kmin;
  int64_t within;
  int64_t ts0;
  // exact comparison of equal inexact codes
  bool exact_codes;
  int vtype;
  const void* vcol;
  const int64_t* ord;
  int64_t obase;
  int32_t o0;  // relative ordinal of the batch's first event; carried partials lie before it
  // carried partials (carry_in_kernel): cin[i] = {ordinal - base, code, ts - ts0}, rows [cstart, cend) of a key
  const uint4* cin;
  const uint32_t* cstart;
  const uint32_t* cend;
  const int64_t* crow;
  int cwidth, vattr;
  // outputs
  const uint32_t* sbase;
  uint64_t* stage;
  uint32_t* mstart;
  uint32_t* mtot;
  uint4* spill;
  int64_t* cand;
  uint32_t* cand_n;
  uint32_t cand_cap;
  uint32_t* err;
  unsigned long long* stamps;  // optional (SM_STACK_STAMPS=1): clock ticks per kernel phase, summed over waves
  int dbg;                     // diagnostic mode (SM_STACK_DEBUG): 1 = skip the stacks (wrong results; timing only)
  unsigned long long* counts;  // with stamps: events, pops, refills, spills, exact compares, log overflows
};

template <int OP, bool FP>
__global__ void __launch_bounds__(kSB) stack_kernel(StackArgs a) {
  __shared__ uint4 rec[kS];         // the slice grouped by key (arrival order within a key); .x = slice position | c1
  __shared__ uint32_t ordt[kS];     // ordinal of each slice position (arrival order)
  __shared__ uint64_t area[kLog];   // ranking: per-wave key counts (u16 [kSW][kKeys]); then the match log
  __shared__ uint64_t ovf[kOvf];    // log entries beyond a thread's slots
  __shared__ uint16_t hst[kKeys], hcn[kKeys];
  __shared__ uint16_t jcnt[kS], joff[kS];
  __shared__ uint32_t lw[kSW];
  __shared__ uint32_t s_ovf, s_slice_tot, s_lastj;

  uint16_t(*wcnt)[kKeys] = (uint16_t(*)[kKeys])area;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // within < 2^30 and event times in [-2^30, 2^30) relative to the batch: differences fit 32 bits
  const int32_t within32 = (int32_t)a.within;
  // phase clock (diagnostic): 0 slice setup, 1 ranking, 2 placement, 3 stacks, 4 scan + tiles, 5 match writes,
  // 6 bucket tail + carry out
  unsigned long long st_acc[7] = {0, 0, 0, 0, 0, 0, 0}, st_last = kStamps && a.stamps ? __builtin_amdgcn_s_memtime() : 0;
#define SM_PHASE(i)                                               \
  do {                                                            \
    if (kStamps && a.stamps) {                                    \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
      st_acc[i] += t_ - st_last;                                  \
      st_last = t_;                                               \
    }                                                             \
  } while (0)
  const uint64_t lt = lanemask_lt();
  // the two keys of this thread: h = tid (A) and h = tid + kSB (B)
  const bool hasA = tid < a.H, hasB = kKPT == 2 && tid + kSB < a.H;
  uint4* spA = a.spill + ((int64_t)blockIdx.x * kKeys + tid) * kQ;
  uint4* spB = spA + (int64_t)kSB * kQ;
  // match log: slot k of thread t at area[k * kLStride + t] (slot-major: the lanes of a wave write consecutive words;
  // thread-major t * kSlots + k put every lane of a wave on the same two banks)
  const uint32_t kLStride = (uint32_t)(a.H < kSB ? a.H : kSB);
  const uint32_t kSlots = kLog / kLStride;
  unsigned long long cn[2] = {0, 0};

  for (int d = blockIdx.x; d < kBins; d += gridDim.x) {
    const int64_t b0 = a.dbase[d];
    const int64_t b1 = d + 1 < kBins ? (int64_t)a.dbase[d + 1] : a.n;
    const int64_t blen = b1 - b0;
    const int64_t sb = a.sbase[d];
    uint32_t* mst = a.mstart + (int64_t)d * (a.ntiles + 1);
    Stack sA, sB;
    sA.n = sA.hb = sA.hn = 0;
    sB.n = sB.hb = sB.hn = 0;
    ExactSrc exA{a.exact_codes, a.vtype, a.vattr, a.cwidth, a.vcol, a.ord, a.obase, a.n, a.crow, a.o0, 0u, 0u};
    ExactSrc exB = exA;
    const uint32_t krA = ((uint32_t)tid << kRB) | (uint32_t)d, krB = ((uint32_t)(tid + kSB) << kRB) | (uint32_t)d;
    // carried partials first (oldest first)
    auto carry_in = [&](Stack& s, ExactSrc& ex, uint4* sp, uint32_t kr) {
      ex.cs = a.cstart[kr];
      ex.ce = a.cend[kr];
      for (uint32_t q = ex.cs; q < ex.ce; ++q) {
        const uint4 e = a.cin[q];
        st_push(s, sp, e.x, e.y, (int32_t)e.z, (int32_t)e.z, a.within, a.err);
      }
    };
    if (a.cin) {
      if (hasA) carry_in(sA, exA, spA, krA);
      if (hasB) carry_in(sB, exB, spB, krB);
    }
    // event time of each key's last event in the batch: partials it did not find expired stay pending
    int32_t tlA = 0, tlB = 0;
    bool seenA = false, seenB = false;
    if (tid == 0) s_lastj = 0xffffffffu;  // ordinal before the bucket's first record (none)
    uint32_t mrun = 0;                    // matches of the bucket so far

    uint4 pre[kSI];
    auto prefetch = [&](int64_t q) {
#pragma unroll
      for (int k = 0; k < kSI; ++k) {
        const int64_t p = q + w * 64 * kSI + k * 64 + lane;
        if (p < blen) {
          typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
          const u32x4 v = __builtin_nontemporal_load((const u32x4*)a.rec + b0 + p);
          pre[k] = make_uint4(v.x, v.y, v.z, v.w);
        }
      }
    };
    prefetch(0);

    for (int64_t q = 0; q < blen; q += kS) {
      const int sn = (int)(blen - q < kS ? blen - q : kS);
      lds_barrier();  // previous slice's readers are done
      for (int k = tid; k < kSW * kKeys / 4; k += kSB) area[k] = 0;
      if (tid == 0) s_ovf = 0;
      lds_barrier();
      SM_PHASE(0);

      // ---- rank by key, stable (arrival order) within a key; the slice lands in LDS grouped by key
      uint32_t hk[kSI], lp[kSI];
#pragma unroll
      for (int k = 0; k < kSI; ++k) {
        const int e = w * 64 * kSI + k * 64 + lane;
        const bool valid = e < sn;
        hk[k] = valid ? (pre[k].x & kKeyMask) >> kRB : 0u;
        const uint64_t peers = peer_mask(hk[k], valid);
        uint32_t old = 0;
        if (valid) old = wcnt[w][hk[k]];
        const uint32_t below = (uint32_t)__popcll(peers & lt);
        if (valid && below == 0) wcnt[w][hk[k]] = (uint16_t)(old + (uint32_t)__popcll(peers));
        lp[k] = old + below;
      }
      lds_barrier();
      {
        // keys kKPT * tid + u: exclusive over waves in place, totals, block scan over keys
        uint32_t r2[kKPT];
#pragma unroll
        for (int u = 0; u < kKPT; ++u) {
          const int h = kKPT * tid + u;
          uint32_t r = 0;
          for (int qq = 0; qq < kSW; ++qq) {
            const uint32_t c = wcnt[qq][h];
            wcnt[qq][h] = (uint16_t)r;
            r += c;
          }
          hcn[h] = (uint16_t)r;
          r2[u] = r;
        }
        uint32_t tot;
        if constexpr (kKPT == 2) {
          const uint32_t st0 = block_excl<kSB>(r2[0] + r2[1], lw, &tot);
          hst[2 * tid] = (uint16_t)st0;
          hst[2 * tid + 1] = (uint16_t)(st0 + r2[0]);
        } else {
          hst[tid] = (uint16_t)block_excl<kSB>(r2[0], lw, &tot);
        }
      }
      lds_barrier();
      SM_PHASE(1);
#pragma unroll
      for (int k = 0; k < kSI; ++k) {
        const int e = w * 64 * kSI + k * 64 + lane;
        if (e < sn) {
          const uint4 r = pre[k];
          rec[hst[hk[k]] + wcnt[w][hk[k]] + lp[k]] = make_uint4((uint32_t)e | (r.x & 0x80000000u), r.y, r.z, r.w);
          ordt[e] = r.y;
        }
      }
      lds_barrier();
      SM_PHASE(2);

      // ---- each key's events of the slice against its stack; matches go to the log (the thread's slots, then
      // the shared overflow)
      // One event j of a key against the key's stack. The register part is evaluated at once: entry k is popped
      // iff entries 0..k all satisfy c2 and none has expired (the stack is monotone, so j accepts a prefix of it);
      // the first entry that stops the run clears the whole stack when it has expired. Only a run through all the
      // register entries with spilled ones behind them goes on entry by entry (rare).
      auto log_put = [&](uint32_t& nlog, uint64_t ent) {
        if (nlog < kSlots) {
          area[nlog * kLStride + tid] = ent;
        } else {
          const uint32_t o = atomicAdd(&s_ovf, 1u);
          if (o < kOvf) ovf[o] = ent;
          else atomicOr(a.err, SE_LOG);
        }
        ++nlog;
      };
      auto step = [&](Stack& s, const ExactSrc& ex, uint4* sp, uint32_t& nlog, const uint4 r) {
        const uint32_t e = r.x & 0xffffu;
        const int32_t jt = (int32_t)r.w;
        const uint32_t cj = r.z, oj = r.y;
        if (FP && cj == kNanCode) atomicOr(a.err, SE_NAN);
        uint32_t hit = 0, exp = 0, tie = 0;
#pragma unroll
        for (int k = 0; k < kC; ++k) {
          const bool live = k < s.n;
          const bool x = within32 >= 0 && jt - s.t[k] > within32;
          const bool t = !a.exact_codes && s.c[k] == cj;
          const bool nan = FP && ((s.c[k] == kNanCode) | (cj == kNanCode));
          hit |= (live && cmp_fixed<OP>(cj, s.c[k])) ? (1u << k) : 0u;
          exp |= (live && x) ? (1u << k) : 0u;
          tie |= (live && (t || nan)) ? (1u << k) : 0u;
        }
        if (tie) {  // equal inexact codes: the exact values decide (out of line)
#pragma unroll
          for (int k = 0; k < kC; ++k)
            if ((tie >> k) & 1u) {
              const bool h = c2_exact<OP, FP>(ex, s.o[k], oj);
              hit = h ? (hit | (1u << k)) : (hit & ~(1u << k));
            }
        }
        const uint32_t ok = hit & ~exp;
        uint32_t npop = (uint32_t)__builtin_ctz(~ok);  // leading entries popped
        if (npop > (uint32_t)s.n) npop = s.n;
#pragma unroll
        for (int k = 0; k < kC; ++k)
          if ((uint32_t)k < npop) log_put(nlog, (uint64_t)s.o[k] | ((uint64_t)(e | ((uint32_t)k << 16)) << 32));
        const bool stop_expired = npop < (uint32_t)s.n && ((exp >> npop) & 1u);
        // shift the register part down by npop (npop < 8)
#pragma unroll
        for (int b = 1; b < kC; b <<= 1)
          if (npop & b) {
#pragma unroll
            for (int k = 0; k < kC; ++k)
              if (k + b < kC) {
                s.o[k] = s.o[k + b];
                s.c[k] = s.c[k + b];
                s.t[k] = s.t[k + b];
              }
          }
        s.n -= (int)npop;
        if (stop_expired) {  // the entry that stopped the run has expired: so has every older one
          s.n = 0;
          s.hn = 0;
        } else if (s.n == 0 && s.hn > 0) {  // ran through the registers: continue into the spill
          for (;;) {
            st_refill(s, sp);
            if (within32 >= 0 && jt - s.t[0] > within32) {
              s.n = 0;
              s.hn = 0;
              break;
            }
            if (!c2_hit<OP, FP>(ex, s.c[0], s.o[0], cj, oj)) break;
            log_put(nlog, (uint64_t)s.o[0] | ((uint64_t)(e | (npop << 16)) << 32));
            ++npop;
            st_pop(s);
            if (s.hn == 0) break;
          }
        }
        jcnt[e] = (uint16_t)npop;
        if (r.x >> 31) st_push(s, sp, oj, cj, jt, jt, a.within, a.err);
        if (kStamps && a.counts) {
          cn[0] += 1;
          cn[1] += npop;
        }
      };
      uint32_t nlog = 0;
      if (a.dbg == 1)
        for (int k = tid; k < sn; k += kSB) jcnt[k] = 0;
      if (a.dbg != 1) {
        const int cA = hasA ? hcn[tid] : 0, cB = hasB ? hcn[(tid + kSB) & (kKeys - 1)] : 0;
        const int sA0 = hst[tid], sB0 = hst[(tid + kSB) & (kKeys - 1)];
        const int cmax = cA > cB ? cA : cB;
        if (cA) {
          tlA = (int32_t)rec[sA0 + cA - 1].w;
          seenA = true;
        }
        if (cB) {
          tlB = (int32_t)rec[sB0 + cB - 1].w;
          seenB = true;
        }
        // the two keys' events interleaved: two independent dependency chains per thread
        for (int x = 0; x < cmax; ++x) {
          if (x < cA) step(sA, exA, spA, nlog, rec[sA0 + x]);
          if (x < cB) step(sB, exB, spB, nlog, rec[sB0 + x]);
        }
      }
      SM_PHASE(3);
      // ---- matches of the slice in arrival order of j: exclusive scan of the per-j counts
      if (q + kS < blen) prefetch(q + kS);  // the next slice's loads overlap the scan and the match writes
      lds_barrier();
      {
        uint32_t v[kSI], sum = 0;
#pragma unroll
        for (int k = 0; k < kSI; ++k) {
          const int e = tid * kSI + k;
          v[k] = e < sn ? jcnt[e] : 0u;
          sum += v[k];
        }
        uint32_t tot;
        uint32_t r = block_excl<kSB>(sum, lw, &tot);
        const uint32_t jprev = tid == 0 ? s_lastj : 0u;
#pragma unroll
        for (int k = 0; k < kSI; ++k) {
          const int e = tid * kSI + k;
          if (e < sn) {
            joff[e] = (uint16_t)r;
            // ordinal tiles whose first ordinal falls in (previous record's ordinal, this record's]: their first
            // match in this bucket is this record's first
            const uint32_t j = ordt[e];
            const uint32_t jp = e == 0 ? jprev : ordt[e - 1];
            const uint32_t t0 = jp == 0xffffffffu ? 0u : (jp >> kTB) + 1u;
            for (uint32_t t = t0; t <= (j >> kTB); ++t) mst[t] = mrun + r;
          }
          r += v[k];
        }
        if (tid == 0) s_slice_tot = tot;
      }
      lds_barrier();
      SM_PHASE(4);
      if (tid == 0) s_lastj = ordt[sn - 1];
      const uint32_t stot = s_slice_tot;
      const uint32_t no = s_ovf < kOvf ? s_ovf : kOvf;
      auto emit = [&](uint64_t ent) {
        const uint32_t io = (uint32_t)ent, pe = (uint32_t)(ent >> 32);
        const uint32_t e = pe & 0xffffu, pop = pe >> 16;
        const uint32_t pos = mrun + joff[e] + (jcnt[e] - 1u - pop);
        a.stage[sb + pos] = ((uint64_t)ordt[e] << 32) | io;
      };
      for (uint32_t k = 0; k < nlog && k < kSlots; ++k) emit(area[k * kLStride + tid]);
      for (uint32_t k = tid; k < no; k += kSB) emit(ovf[k]);
      mrun += stot;
      SM_PHASE(5);
    }
    // tiles after the bucket's last record start at its end
    __syncthreads();
    {
      const uint32_t jl = s_lastj;
      const uint32_t t0 = jl == 0xffffffffu ? 0u : (jl >> kTB) + 1u;
      for (uint32_t t = t0 + tid; t <= (uint32_t)a.ntiles; t += kSB) mst[t] = mrun;
      if (tid == 0) a.mtot[d] = mrun;
    }

    // ---- carry out: the partials still pending in the reference, i.e. those the key's last event found neither
    // matched nor expired (a key without events in this batch keeps all of its carried partials)
    auto keep_of = [&](const Stack& s, const uint4* sp, int32_t tl, bool seen) {
      auto pending = [&](int32_t t) { return !seen || a.within < 0 || (int64_t)tl - t <= a.within; };
      uint32_t keep = 0;
#pragma unroll
      for (int k = 0; k < kC; ++k)
        if (k < s.n && pending(s.t[k])) ++keep;
      for (int k = 0; k < s.hn; ++k)
        if (pending((int32_t)sp[(s.hb + k) & (kQ - 1)].z)) ++keep;
      return keep;
    };
    const uint32_t keepA = hasA ? keep_of(sA, spA, tlA, seenA) : 0u;
    const uint32_t keepB = hasB ? keep_of(sB, spB, tlB, seenB) : 0u;
    const uint32_t keep = keepA + keepB;
    uint32_t inc = keep;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(inc, o, 64);
      if (lane >= o) inc += u;
    }
    uint32_t base = 0;
    if (lane == 63 && inc) base = atomicAdd(a.cand_n, inc);
    base = __shfl(base, 63, 64) + inc - keep;
    auto put_all = [&](const Stack& s, const ExactSrc& ex, const uint4* sp, int32_t tl, bool seen, uint32_t kr) {
      auto pending = [&](int32_t t) { return !seen || a.within < 0 || (int64_t)tl - t <= a.within; };
      const int64_t key = a.kmin + (int64_t)kr;
      auto put = [&](uint32_t o, int32_t t) {
        if (!pending(t)) return;
        if (base < a.cand_cap) {
          int64_t* c = a.cand + 4 * (int64_t)base;
          c[0] = key;
          c[1] = (int64_t)(int32_t)o + a.obase;
          c[2] = (int64_t)t + a.ts0;
          c[3] = ex.carried(o) ? -(int64_t)ex.carry_row(o) - 1 : ex.row_of(o);
        } else {
          atomicOr(a.err, SE_CAND);
        }
        ++base;
      };
      // Invariant the carry-out relies on (build_carry with key_runs_ordered): a key's pending partials are written
      // as ONE contiguous run, oldest first: the spill ring from its head upward, then the registers from the bottom
      // (kC - 1) to the top (0). One stable sort by key then orders the whole carry by (key, ordinal); reordering
      // these loops would silently corrupt the carry order of later batches.
      for (int k = 0; k < s.hn; ++k) {
        const uint4 e = sp[(s.hb + k) & (kQ - 1)];
        put(e.x, (int32_t)e.z);
      }
#pragma unroll
      for (int k = kC - 1; k >= 0; --k)
        if (k < s.n) put(s.o[k], s.t[k]);
    };
    if (keepA) put_all(sA, exA, spA, tlA, seenA, krA);
    if (keepB) put_all(sB, exB, spB, tlB, seenB, krB);
    __syncthreads();  // LDS of this bucket is free for the next one
    SM_PHASE(6);
  }
  if (kStamps && a.stamps && lane == 0)
    for (int i = 0; i < 7; ++i) atomicAdd(&a.stamps[i], st_acc[i]);
  if (kStamps && a.counts) {
    atomicAdd(&a.counts[0], cn[0]);
    atomicAdd(&a.counts[1], cn[1]);
  }
#undef SM_PHASE
}

// mstart [d][t] (written bucket by bucket) → [t][d] (read tile by tile)
__global__ void __launch_bounds__(256) transpose_kernel(const uint32_t* __restrict__ src, int64_t cols,
                                                        uint32_t* __restrict__ dst) {
  __shared__ uint32_t tile[32][33];
  const int64_t c0 = (int64_t)blockIdx.x * 32, r0 = (int64_t)blockIdx.y * 32;  // src rows = buckets
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int k = ty; k < 32; k += 8) {
    const int64_t c = c0 + tx;
    tile[k][tx] = c < cols ? src[(r0 + k) * cols + c] : 0u;
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int64_t c = c0 + k;
    if (c < cols) dst[c * kBins + r0 + tx] = tile[tx][k];
  }
}

// Tiles [blockIdx.x * kGT, +kGT) of kOT ordinals each, in order. Per tile, bucket d's staged matches with j in
// the tile are one contiguous segment in (j, i) order (a j's matches are consecutive in it); 16 lanes read a
// bucket's segment together (one 128-byte line per 16 matches). Pass A counts matches per ordinal (LDS atomics),
// a block scan turns the counts into offsets, pass B re-reads the segments (cache-hot) and places each match at
// offset of its j + its rank among the j's matches in an LDS image of the tile's output, which leaves as one
// contiguous, coalesced run (its base = matches whose j precedes the tile, summed over buckets). A tile whose
// output exceeds the LDS image writes its matches to their places directly.
__global__ void __launch_bounds__(kOB) order_kernel(OrderArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t cnt[kOT];
  __shared__ uint64_t obuf[kOCap > 0 ? kOCap : 1];
  __shared__ uint32_t sst[kBins], slen[kBins];
  __shared__ uint32_t lw[kOB / 64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l16 = lane & 15, g = lane >> 4;
  const uint64_t gmask = 0xffffull << (g * 16);
  // groups of kGT tiles, one per workgroup. XCD-contiguous: the dispatcher deals blocks round-robin over the 8 XCDs
  // (MI355X_MICROARCH.md, dispatch), so block b is remapped to group xcd_rank(b): the ~32 workgroups an XCD runs at
  // once take consecutive groups, and the segment lines two neighbouring tiles share are fetched into that XCD's L2
  // once, by whichever of them reads first (a bucket's segments of consecutive tiles are adjacent in its run)
  int64_t blk = blockIdx.x;
  if (SM_ORDER_XCD) {
    const int64_t G = gridDim.x, q = G >> 3, r = G & 7, x = blk & 7, i = blk >> 3;
    blk = x < r ? x * (q + 1) + i : r * (q + 1) + (x - r) * q + i;
  }
  // SM_ORDER_XCD == 2: a cohort of kCoh XCD-consecutive workgroups (about the 32 an XCD runs at once) takes kCoh * kGT
  // consecutive tiles, member m every kCoh-th of them: at each step the cohort orders kCoh adjacent tiles, whose
  // shared segment lines its L2 fetches once, and each workgroup still orders kGT tiles
  constexpr int64_t kCoh = 32;
  const int64_t coh = blk / kCoh, mem = blk % kCoh;
  // members of this cohort (the last one may be partial; the grid covers ntiles <= gridDim.x * kGT, so its members
  // still reach every tile of its range in kGT steps)
  const int64_t cw = (int64_t)gridDim.x - coh * kCoh < kCoh ? (int64_t)gridDim.x - coh * kCoh : kCoh;
  auto tile_at = [&](int64_t base, int64_t k) {
    return SM_ORDER_XCD == 2 ? coh * kCoh * kGT + mem + cw * k : base + k;
  };
  for (int64_t tb = SM_ORDER_XCD == 2 ? 0 : blk * kGT; tb < a.ntiles; tb += (int64_t)gridDim.x * kGT) {
  const int64_t te = SM_ORDER_XCD == 2 ? kGT : (tb + kGT < a.ntiles ? tb + kGT : a.ntiles) - tb;
  uint32_t ms = 0, tot = 0;
  int64_t out = 0;  // matches whose j precedes the tile
  if (SM_ORDER_XCD != 2) {
    ms = a.mt[tb * kBins + tid];
    (void)block_excl(ms, lw, &tot);
    out = tot;
  }
  for (int64_t k = 0; k < te; ++k) {
    const int64_t t = tile_at(tb, k);
    if (t >= a.ntiles) break;
    if (SM_ORDER_XCD == 2) {  // not the previous tile's successor: this tile's own prefix over the buckets
      lds_barrier();          // lw's previous readers are done
      ms = a.mt[t * kBins + tid];
      (void)block_excl(ms, lw, &tot);
      out = tot;
    }
    const uint32_t me = a.mt[(t + 1) * kBins + tid];
    const uint32_t j0 = (uint32_t)(t << kTB);
    lds_barrier();  // previous tile's readers are done
    sst[tid] = a.sbase[tid] + ms;
    slen[tid] = me - ms;
    for (int e = tid; e < kOT; e += kOB) cnt[e] = 0;
    ms = me;
    lds_barrier();
    auto count = [&](uint32_t j) { atomicAdd(&cnt[j - j0], 1u); };
    // pass A: matches per ordinal. The first 16 matches of each of the wave's 64 buckets are loaded at once (one
    // load per round, all in flight) and kept for pass B; longer segments (rare) are walked chunk by chunk.
    uint64_t v0[16];
    uint32_t s0r[16], lenr[16];
    bool more = false;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int d = w * 64 + r * 4 + g;
      s0r[r] = sst[d];
      lenr[r] = slen[d];
      more |= lenr[r] > 16u;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) v0[r] = (uint32_t)l16 < lenr[r] ? a.stage[s0r[r] + l16] : 0ull;
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if ((uint32_t)l16 < lenr[r]) count((uint32_t)(v0[r] >> 32));
    if (__any(more))
      for (int r = 0; r < 16; ++r)
        for (uint32_t c = 16; __any(c < lenr[r]); c += 16)
          if (c + l16 < lenr[r]) count((uint32_t)(a.stage[s0r[r] + c + l16] >> 32));
    lds_barrier();
    {  // exclusive scan of the counts, kPer ordinals per thread (read again from LDS rather than held in registers:
       // holding them spilled 4 VGPRs; 6.75 -> 6.5 ms)
      constexpr int kPer = kOT / kOB;
      static_assert(kPer % 4 == 0, "16-byte count reads");
      uint4* c4 = (uint4*)(cnt + tid * kPer);
      uint32_t sum = 0;
#pragma unroll
      for (int k = 0; k < kPer / 4; ++k) {
        const uint4 c = c4[k];
        sum += c.x + c.y + c.z + c.w;
      }
      uint32_t r = block_excl(sum, lw, &tot);
#pragma unroll
      for (int k = 0; k < kPer / 4; ++k) {
        const uint4 c = c4[k];
        uint4 o;
        o.x = r;
        o.y = o.x + c.x;
        o.z = o.y + c.y;
        o.w = o.z + c.z;
        r = o.w + c.w;
        c4[k] = o;
      }
    }
    lds_barrier();
    // pass B, once per part of the tile (kSplit): rank of each match among its j's matches = its segment position -
    // the position where its j's run starts (runs may continue from the previous 16-match chunk of the segment); the
    // part's matches go to the LDS image (a j's run lies in one part)
    for (int h = 0; h < kSplit; ++h) {
    const uint32_t hb = h == 0 ? 0u : cnt[h << kOHB];  // the part's first output offset within the tile
    const uint32_t he = h + 1 < kSplit ? cnt[(h + 1) << kOHB] : tot;
    const bool staged = kOCap > 0 && he - hb <= (uint32_t)kOCap;
    auto place = [&](uint64_t v, bool valid, uint32_t c, uint32_t& cj, uint32_t& cstart) {
      const uint32_t j = (uint32_t)(v >> 32);
      uint32_t jp = __shfl_up(j, 1, 16);
      if (l16 == 0) jp = cj;
      const bool start = valid && j != jp;
      const uint32_t sm = (uint32_t)((__ballot(start) & gmask) >> (g * 16));
      const uint32_t upto = sm & ((2u << l16) - 1u);
      const uint32_t rs = upto ? c + 31u - (uint32_t)__clz(upto) : cstart;
      if (valid && (kSplit == 1 || (int)((j - j0) >> kOHB) == h)) {
        const uint32_t pos = cnt[j - j0] + (c + l16 - rs);
        if (staged) obuf[pos - hb] = v;
        else a.out[out + pos] = v;
      }
      const uint32_t vm = (uint32_t)((__ballot(valid) & gmask) >> (g * 16));
      const int last = vm ? 31 - __clz(vm) : 0;
      cj = __shfl(j, last, 16);
      cstart = __shfl(rs, last, 16);
    };
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      uint32_t cj = 0xffffffffu, cstart = 0;
      place(v0[r], (uint32_t)l16 < lenr[r], 0, cj, cstart);
      if (__any(lenr[r] > 16u))
        for (uint32_t c = 16; __any(c < lenr[r]); c += 16) {
          const bool valid = c + l16 < lenr[r];
          place(valid ? a.stage[s0r[r] + c + l16] : 0ull, valid, c, cj, cstart);
        }
    }
    lds_barrier();
    if (staged)
      for (uint32_t k = tid; k < he - hb; k += kOB) a.out[out + hb + k] = obuf[k];
    if (kSplit > 1) lds_barrier();  // the image's readers are done before the next part's placement
    }
    out += tot;
  }
  }
}

template <int OP, bool FP>
void launch_stack4_t(const Stack4Args& a4, int grid, hipStream_t s) {
  hipLaunchKernelGGL((stack4_kernel<OP, FP>), dim3(grid), dim3(kT4), 0, s, a4);
}

// Carried partials for this batch: codes of the compared value and each key's row range. Keys outside the
// batch's key range see no event: their partials go straight to the carry-out candidates.
template <typename VT>
__global__ void carry_in_kernel(const int64_t* __restrict__ rows, int64_t n, int w, int vattr, int vtype, int vmode,
                                int64_t vmin, int64_t kmin, int64_t span, int64_t obase, int64_t o0, int64_t ts0,
                                uint4* __restrict__ cin, uint32_t* __restrict__ cstart, uint32_t* __restrict__ cend,
                                uint32_t* __restrict__ ccnt, int64_t* __restrict__ cand, uint32_t* __restrict__ cand_n,
                                uint32_t* __restrict__ err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t* r = rows + i * w;
  const int64_t key = r[0];
  const int64_t kr = key - kmin;
  if (kr < 0 || kr > span) {
    const uint32_t q = atomicAdd(cand_n, 1u);
    int64_t* c = cand + 4 * (int64_t)q;
    c[0] = key;
    c[1] = r[1];
    c[2] = r[2];
    c[3] = -i - 1;
    return;
  }
  const int64_t o = r[1] - obase;
  if (o >= o0 || o < INT32_MIN) atomicOr(err, SE_ORD);
  int64_t t = r[2] - ts0;  // older than 2^30 ms: dead for any event of this batch (within < 2^30)
  if (t < -(1ll << 30)) t = -(1ll << 30);
  const StackVal v = uncanon((uint64_t)r[3 + vattr], vtype);
  uint32_t code;
  if constexpr (std::is_same<VT, float>::value) code = vcode<float>((float)v.d, vmode, vmin);
  else if constexpr (std::is_same<VT, double>::value) code = vcode<double>(v.d, vmode, vmin);
  else if constexpr (std::is_same<VT, int32_t>::value) code = vcode<int32_t>((int32_t)v.i, vmode, vmin);
  else code = vcode<int64_t>(v.i, vmode, vmin);
  cin[i] = make_uint4((uint32_t)(int32_t)o, code, (uint32_t)(int32_t)t, 0u);
  if (i == 0 || rows[(i - 1) * w] != key) cstart[kr] = (uint32_t)i;
  if (i == n - 1 || rows[(i + 1) * w] != key) cend[kr] = (uint32_t)(i + 1);
  atomicAdd(&ccnt[kr & (kBins - 1)], 1u);
}

// staging run of each bucket: its records plus its carried partials (a bucket's matches cannot exceed them)
__global__ void __launch_bounds__(kOB) stage_base_kernel(const uint32_t* __restrict__ dbase,
                                                         const uint32_t* __restrict__ ccnt, uint32_t* __restrict__ sbase,
                                                         uint32_t* __restrict__ stot) {
  __shared__ uint32_t lw[kOB / 64];
  const int d = threadIdx.x;
  const uint32_t c = ccnt ? ccnt[d] : 0u;
  uint32_t tot;
  const uint32_t r = block_excl(c, lw, &tot);
  sbase[d] = dbase[d] + r;
  if (d == 0) *stot = tot;
}

// ---- carry out
__global__ void carry_rows_kernel(const int64_t* __restrict__ cand, int64_t n, const NfaStream* __restrict__ st,
                                  int nattr, const int64_t* __restrict__ old, int w, int64_t kmin, int key_bits,
                                  int64_t* __restrict__ rows, uint64_t* __restrict__ kord, uint64_t* __restrict__ kkey,
                                  uint32_t* __restrict__ idx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t* c = cand + 4 * i;
  int64_t* r = rows + i * w;
  if (c[3] >= 0) {
    r[0] = c[0];
    r[1] = c[1];
    r[2] = c[2];
    for (int k = 0; k < nattr; ++k) r[3 + k] = (int64_t)canon(col_value(st, k, c[3]), st->types[k]);
  } else {  // a carried partial that stays pending: its row unchanged
    const int64_t* o = old + (-c[3] - 1) * w;
    for (int k = 0; k < w; ++k) r[k] = o[k];
  }
  kord[i] = (uint64_t)c[1] ^ 0x8000000000000000ull;
  kkey[i] = key_bits < 64 ? (uint64_t)(c[0] - kmin) : (uint64_t)c[0] ^ 0x8000000000000000ull;
  idx[i] = (uint32_t)i;
}

__global__ void gather_u64_kernel(const uint64_t* __restrict__ src, const uint32_t* __restrict__ idx, int64_t n,
                                  uint64_t* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[idx[i]];
}

__global__ void gather_rows_kernel(const int64_t* __restrict__ src, const uint32_t* __restrict__ idx, int64_t n, int w,
                                   int64_t* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t* s = src + (int64_t)idx[i] * w;
  for (int k = 0; k < w; ++k) dst[i * w + k] = s[k];
}

inline dim3 grid_of(int64_t n, int t = 256) { return dim3((unsigned)std::max<int64_t>(1, (n + t - 1) / t)); }

template <int OP, bool FP>
void launch_stack_t(const StackArgs& sa, int grid, hipStream_t s) {
  hipLaunchKernelGGL((stack_kernel<OP, FP>), dim3(grid), dim3(kSB), 0, s, sa);
}

}  // namespace

void FastCarry::reserve(int64_t rows_needed, int w) {
  if (rows_needed <= cap && w == width) return;
  int64_t* p = nullptr;
  const int64_t c = std::max<int64_t>(rows_needed, std::max<int64_t>(cap * 2, 1024));
  SM_HIP(hipMalloc(&p, (size_t)c * w * 8));
  if (rows && n && w == width) SM_HIP(hipMemcpy(p, rows, (size_t)n * w * 8, hipMemcpyDeviceToDevice));
  if (rows) SM_HIP(hipFree(rows));
  rows = p;
  cap = c;
  width = w;
}

void FastCarry::release() {
  if (rows) (void)hipFree(rows);
  rows = nullptr;
  cap = n = 0;
}

void build_carry(const int64_t* cand, int64_t ncand, const NfaStream* st, int nattr, FastCarry& carry, Scratch& sc,
                 hipStream_t s, int key_bits, int64_t kmin, bool key_runs_ordered) {
  const int w = 3 + nattr;
  if (ncand == 0) {
    carry.n = 0;
    carry.width = w;
    return;
  }
  const size_t mark = sc.used;
  int64_t* rows = (int64_t*)sc.take((size_t)ncand * w * 8);
  uint64_t* kord = (uint64_t*)sc.take((size_t)ncand * 8);
  uint64_t* kkey = (uint64_t*)sc.take((size_t)ncand * 8);
  uint64_t* k2 = (uint64_t*)sc.take((size_t)ncand * 8);
  uint32_t* idx = (uint32_t*)sc.take((size_t)ncand * 4);
  uint32_t* idx2 = (uint32_t*)sc.take((size_t)ncand * 4);
  hipLaunchKernelGGL(carry_rows_kernel, grid_of(ncand), dim3(256), 0, s, cand, ncand, st, nattr,
                     (const int64_t*)carry.rows, w, kmin, key_bits, rows, kord, kkey, idx);
  const uint32_t* fin;
  if (key_runs_ordered) {
    // every key's candidates are one run already in ordinal order: a stable sort by key (its significant bits) only
    const bool alt = radix_sort_pairs<uint64_t>(kkey, k2, idx, idx2, (size_t)ncand, 0, key_bits, sc, s);
    fin = alt ? idx2 : idx;
  } else {
    // stable sort by ordinal, then by key
    bool alt = radix_sort_pairs<uint64_t>(kord, k2, idx, idx2, (size_t)ncand, 0, 64, sc, s);
    uint32_t* i1 = alt ? idx2 : idx;
    uint32_t* i1b = alt ? idx : idx2;
    hipLaunchKernelGGL(gather_u64_kernel, grid_of(ncand), dim3(256), 0, s, kkey, i1, ncand, k2);
    alt = radix_sort_pairs<uint64_t>(k2, kkey, i1, i1b, (size_t)ncand, 0, key_bits, sc, s);
    fin = alt ? i1b : i1;
  }
  carry.reserve(ncand, w);
  hipLaunchKernelGGL(gather_rows_kernel, grid_of(ncand), dim3(256), 0, s, rows, fin, ncand, w, carry.rows);
  SM_HIP(hipStreamSynchronize(s));
  carry.n = ncand;
  sc.used = mark;
}

int64_t stack_pipeline(const StackPlan& p, const FastArgs& a, const FastHostInfo& hi, FastState& fs, FastCarry& carry,
                       uint32_t* pairs_out, int64_t pairs_cap, Scratch& sc, hipStream_t s, FastTimings* tm) {
  const size_t mark = sc.used;
  auto tmark = [&](const char* l) {
    if (tm) tm->mark(l, s);
  };
  const int64_t n = p.n;
  uint32_t* err = (uint32_t*)sc.take(16);
  uint32_t* cand_n = err + 1;
  uint32_t* stot = err + 2;
  SM_HIP(hipMemsetAsync(err, 0, 16, s));
  StackArgs sa{};
  sa.rec = (const uint4*)p.rec;
  sa.dbase = p.dbase;
  sa.ntiles = (p.omax >> kTB) + 1;
  sa.n = n;
  sa.H = p.H;
  sa.kmin = p.kmin;
  sa.within = p.within;
  sa.ts0 = p.ts0;
  sa.exact_codes = p.exact_codes;
  sa.vtype = p.vtype;
  sa.vcol = p.vcol;
  sa.ord = a.ordinals;
  sa.obase = a.ordinal_base;
  sa.o0 = p.o0;
  sa.vattr = p.vattr;
  sa.err = err;

  // carry-out candidates: every partial still pending at the end (at most the batch's events + the carried ones)
  int64_t nc = carry.n;
  const int64_t cand_cap = std::min<int64_t>(n + nc, (int64_t)8 * p.H * kBins + nc) + 1024;
  sa.cand = (int64_t*)sc.take((size_t)cand_cap * 32);
  sa.cand_n = cand_n;
  sa.cand_cap = (uint32_t)std::min<int64_t>(cand_cap, 0xffffffffll);
  // carried partials of keys in this batch's key range
  uint32_t* ccnt = nullptr;
  if (nc > 0) {
    const int64_t span = (int64_t)p.H << kRB;
    uint4* cin = (uint4*)sc.take((size_t)nc * 16);
    uint32_t* cst = (uint32_t*)sc.take((size_t)span * 4);
    uint32_t* cen = (uint32_t*)sc.take((size_t)span * 4);
    ccnt = (uint32_t*)sc.take(kBins * 4);
    SM_HIP(hipMemsetAsync(cst, 0, (size_t)span * 4, s));
    SM_HIP(hipMemsetAsync(cen, 0, (size_t)span * 4, s));
    SM_HIP(hipMemsetAsync(ccnt, 0, kBins * 4, s));
#define SM_CIN(VT)                                                                                                  \
  hipLaunchKernelGGL((carry_in_kernel<VT>), grid_of(nc), dim3(256), 0, s, (const int64_t*)carry.rows, nc, carry.width, \
                     p.vattr, p.vtype, p.vmode, p.vmin, p.kmin, span - 1, a.ordinal_base, p.o0, p.ts0, cin, cst, cen, ccnt,  \
                     sa.cand, cand_n, err)
    switch (p.vtype) {
      case T_INT: SM_CIN(int32_t); break;
      case T_LONG: SM_CIN(int64_t); break;
      case T_FLOAT: SM_CIN(float); break;
      default: SM_CIN(double); break;
    }
#undef SM_CIN
    sa.cin = cin;
    sa.cstart = cst;
    sa.cend = cen;
    sa.crow = (const int64_t*)carry.rows;
    sa.cwidth = carry.width;
  }
  uint32_t* sbase = (uint32_t*)sc.take(kBins * 4);
  hipLaunchKernelGGL(stage_base_kernel, dim3(1), dim3(kOB), 0, s, p.dbase, ccnt, sbase, stot);
  uint32_t hs[3];
  SM_HIP(hipMemcpyAsync(hs, err, 12, hipMemcpyDeviceToHost, s));
  SM_HIP(hipStreamSynchronize(s));
  if (hs[0] & SE_ORD) {
    sc.used = mark;
    throw std::runtime_error("a carried partial lies more than 2^31 events before the batch's ordinal base (match "
                             "tuples are 32-bit ordinals relative to it), or not before the batch");
  }
  const int64_t extra = hs[2];
  const int64_t ncand_in = hs[1];  // carried partials of keys outside this batch's key range (unordered appends)
  if (fs.cus == 0) {
    int dev = 0;
    SM_HIP(hipGetDevice(&dev));
    SM_HIP(hipDeviceGetAttribute(&fs.cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  // the ring kernel (v4) by default; SM_STACK_V2=1 runs the slice-synchronous kernel (A/B). (A barrier-free v3,
  // whose lanes walked their key's events through an HBM permutation, was exact but slower: its drifting lanes
  // gathered records and scattered pop slots with little locality, 54.6 + 35 ms against 31.7 + 6.7 ms.)
  static const bool v2 = getenv("SM_STACK_V2") && atoi(getenv("SM_STACK_V2")) != 0;
  int64_t M = 0;
  {
    sa.sbase = sbase;
    sa.stage = (uint64_t*)sc.take((size_t)(n + extra) * 8);
    sa.mstart = (uint32_t*)sc.take((size_t)kBins * (sa.ntiles + 1) * 4);
    sa.mtot = (uint32_t*)sc.take(kBins * 4);
    // resident workgroups (LDS bound: one per CU)
    if (fs.cus == 0) {
      int dev = 0;
      SM_HIP(hipGetDevice(&dev));
      SM_HIP(hipDeviceGetAttribute(&fs.cus, hipDeviceAttributeMultiprocessorCount, dev));
    }
    const int grid = std::min(kBins, fs.cus);
    sa.spill = (uint4*)sc.take((size_t)grid * kKeys * kQ * 16);
    static const bool want_stamps = getenv("SM_STACK_STAMPS") != nullptr;
    static const int dbg = getenv("SM_STACK_DEBUG") ? atoi(getenv("SM_STACK_DEBUG")) : 0;
    sa.dbg = dbg;
    if (want_stamps) {
      sa.stamps = (unsigned long long*)sc.take(128);
      sa.counts = sa.stamps + 8;
      SM_HIP(hipMemsetAsync(sa.stamps, 0, 128, s));
    }
    tmark("stack_prep");
    if (v2) {
      switch (p.op * 2 + (p.fp ? 1 : 0)) {
        case CMP_GT * 2: launch_stack_t<CMP_GT, false>(sa, grid, s); break;
        case CMP_GT * 2 + 1: launch_stack_t<CMP_GT, true>(sa, grid, s); break;
        case CMP_GE * 2: launch_stack_t<CMP_GE, false>(sa, grid, s); break;
        case CMP_GE * 2 + 1: launch_stack_t<CMP_GE, true>(sa, grid, s); break;
        case CMP_LT * 2: launch_stack_t<CMP_LT, false>(sa, grid, s); break;
        case CMP_LT * 2 + 1: launch_stack_t<CMP_LT, true>(sa, grid, s); break;
        case CMP_LE * 2: launch_stack_t<CMP_LE, false>(sa, grid, s); break;
        case CMP_LE * 2 + 1: launch_stack_t<CMP_LE, true>(sa, grid, s); break;
        default: sc.used = mark; return -1;
      }
    } else {
      Stack4Cold c4{};
      c4.kmin = sa.kmin;
      c4.ts0 = sa.ts0;
      c4.within = sa.within;
      c4.obase = sa.obase;
      c4.n = n;
      c4.vtype = sa.vtype;
      c4.vattr = sa.vattr;
      c4.cwidth = sa.cwidth;
      c4.o0 = sa.o0;
      c4.exact_codes = sa.exact_codes;
      c4.vcol = sa.vcol;
      c4.ord = sa.ord;
      c4.cin = sa.cin;
      c4.cstart = sa.cstart;
      c4.cend = sa.cend;
      c4.crow = sa.crow;
      c4.cand = sa.cand;
      c4.cand_n = sa.cand_n;
      c4.cand_cap = sa.cand_cap;
      Stack4Cold* c4d = (Stack4Cold*)sc.take(sizeof(Stack4Cold));
      SM_HIP(hipMemcpyAsync(c4d, &c4, sizeof(c4), hipMemcpyHostToDevice, s));
      SM_HIP(hipStreamSynchronize(s));  // c4 is a local of this block
      Stack4Args a4{};
      a4.rec = sa.rec;
      a4.dbase = sa.dbase;
      a4.n = (uint32_t)n;
      a4.H = sa.H;
      a4.within = sa.within < 0 ? -1 : (int32_t)sa.within;
      a4.exact_codes = sa.exact_codes;
      a4.ntiles = (uint32_t)sa.ntiles;
      a4.sbase = sa.sbase;
      a4.stage = sa.stage;
      a4.mstart = sa.mstart;
      a4.mtot = sa.mtot;
      a4.spill = sa.spill;
      a4.err = sa.err;
      a4.cold = c4d;
      a4.stamps = sa.stamps;
      switch (p.op * 2 + (p.fp ? 1 : 0)) {
        case CMP_GT * 2: launch_stack4_t<CMP_GT, false>(a4, grid, s); break;
        case CMP_GT * 2 + 1: launch_stack4_t<CMP_GT, true>(a4, grid, s); break;
        case CMP_GE * 2: launch_stack4_t<CMP_GE, false>(a4, grid, s); break;
        case CMP_GE * 2 + 1: launch_stack4_t<CMP_GE, true>(a4, grid, s); break;
        case CMP_LT * 2: launch_stack4_t<CMP_LT, false>(a4, grid, s); break;
        case CMP_LT * 2 + 1: launch_stack4_t<CMP_LT, true>(a4, grid, s); break;
        case CMP_LE * 2: launch_stack4_t<CMP_LE, false>(a4, grid, s); break;
        case CMP_LE * 2 + 1: launch_stack4_t<CMP_LE, true>(a4, grid, s); break;
        default: sc.used = mark; return -1;
      }
    }
    tmark("stack");
    if (sa.stamps && !v2) {
      unsigned long long hst[5];
      SM_HIP(hipMemcpyAsync(hst, sa.stamps, sizeof(hst), hipMemcpyDeviceToHost, s));
      SM_HIP(hipStreamSynchronize(s));
      double tot = 0;
      for (double v : hst) tot += v;
      if (tot > 0)
        fprintf(stderr, "[stack4 phases] rank %.3f stacks %.3f wait %.3f emit %.3f rest %.3f; wave-clocks %.3g\n",
                hst[0] / tot, hst[1] / tot, hst[2] / tot, hst[3] / tot, hst[4] / tot, tot);
    } else if (sa.stamps) {
      unsigned long long hst[7], hcn[2];
      SM_HIP(hipMemcpyAsync(hst, sa.stamps, sizeof(hst), hipMemcpyDeviceToHost, s));
      SM_HIP(hipMemcpyAsync(hcn, sa.counts, sizeof(hcn), hipMemcpyDeviceToHost, s));
      SM_HIP(hipStreamSynchronize(s));
      double tot = 0;
      for (double v : hst) tot += v;
      fprintf(stderr, "[stack phases] setup %.3f rank %.3f place %.3f stacks %.3f scan %.3f writes %.3f tail %.3f\n",
              hst[0] / tot, hst[1] / tot, hst[2] / tot, hst[3] / tot, hst[4] / tot, hst[5] / tot, hst[6] / tot);
      fprintf(stderr, "[stack counts] events %llu pops %llu; wave-cycles %.3g\n", hcn[0], hcn[1], tot);
    }
    std::vector<uint32_t> mt(kBins);
    SM_HIP(hipMemcpyAsync(mt.data(), sa.mtot, kBins * 4, hipMemcpyDeviceToHost, s));
    SM_HIP(hipMemcpyAsync(hs, err, 12, hipMemcpyDeviceToHost, s));
    SM_HIP(hipStreamSynchronize(s));
    if (hs[0]) {
      sc.used = mark;
      return -1;
    }
      for (uint32_t v : mt) M += v;
    if (M > pairs_cap) {
      sc.used = mark;
      throw std::runtime_error("match buffer too small");
    }
    OrderArgs oa{};
    oa.stage = sa.stage;
    oa.sbase = sbase;
    oa.out = (uint64_t*)pairs_out;
    if (M > 0) {
      uint32_t* mt = (uint32_t*)sc.take((size_t)kBins * (sa.ntiles + 1) * 4);
      hipLaunchKernelGGL(transpose_kernel, dim3((unsigned)((sa.ntiles + 1 + 31) / 32), kBins / 32), dim3(256), 0, s,
                         sa.mstart, sa.ntiles + 1, mt);
      oa.mt = mt;
      oa.ntiles = sa.ntiles;
      // (a variant keeping each bucket's cursor line in registers from tile to tile, so that the line shared by
      // consecutive tiles' segments is fetched once, was exact but slower, 15.5 against 6.6 ms: the held lines
      // spill at 1024 threads x 128 VGPRs, and line B's reads then wait one by one)
      // (a persistent grid of 128 or 64 workgroups, so that fewer tiles' segment lines compete for each XCD's L2,
      // ran 12.2 / 24.2 ms against 6.7: the kernel is bound by its concurrency, one workgroup per CU, not by the
      // boundary lines it fetches again)
      // (also measured: two 512-thread workgroups per CU, 8-lane groups, packed u16 counts and a 7000-match image in
      // 80 KB of LDS: exact, 8.5 against 6.75 ms; the same 16 waves per CU, more passes over longer segments; and the
      // next tile's first matches loaded during this tile's scan and placement: 7.6 ms, 18 VGPRs spilled; and
      // nontemporal stores of the output image: 6.58 against 6.48 ms)
      if (SM_ORDER_V1)
        hipLaunchKernelGGL(order_kernel, dim3((unsigned)((sa.ntiles + kGT - 1) / kGT)), dim3(kOB), 0, s, oa);
      else  // round 6: LDS images, loading and storing waves apart (order_dev.h)
        hipLaunchKernelGGL(order2_kernel, dim3((unsigned)((sa.ntiles + kGT2 - 1) / kGT2)), dim3(kOB), 0, s, oa);
#if SM_ORDER2_STAMPS
      {
        unsigned long long h[8];
        SM_HIP(hipMemcpyFromSymbolAsync(h, HIP_SYMBOL(g_o2_stamps), sizeof(h), 0, hipMemcpyDeviceToHost, s));
        SM_HIP(hipStreamSynchronize(s));
        double tot = 0;
        for (unsigned long long v : h) tot += v;
        fprintf(stderr, "[order2 phases] prologue %.3f issue %.3f count %.3f scan %.3f place %.3f land %.3f writes %.3f "
                "desc %.3f\n", h[0] / tot, h[6] / tot, h[1] / tot, h[2] / tot, h[3] / tot, h[7] / tot, h[4] / tot,
                h[5] / tot);
        const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        SM_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_o2_stamps), z, sizeof(z), 0, hipMemcpyHostToDevice, s));
      }
#endif
    }
  }
  tmark("order");
  // carry out (the stack kernel left each key's open partials as candidates)
  const int64_t ncand = hs[1];
  // the stack kernel writes each key's pending partials as one run, oldest first (put_all): with no out-of-range
  // carried partials appended before it, one key sort of span bits orders the carry
  int kb = 1;
  while (kb < 63 && ((((int64_t)p.H << kRB) - 1) >> kb) != 0) ++kb;
  if (ncand_in == 0) build_carry(sa.cand, ncand, a.st, hi.nattr, carry, sc, s, kb, p.kmin, true);
  else build_carry(sa.cand, ncand, a.st, hi.nattr, carry, sc, s);
  tmark("carry_out");
  SM_HIP(hipStreamSynchronize(s));
  sc.used = mark;
  return M;
}

// ---- on-device projection of the closed form's outputs (QuerySelector.processNoGroupBy :124-167): output k is
// the match (e1, e2) = pairs[k]; its select programs read slot 0 (e1) and slot 1 (e2) of the batch, or for an e1
// carried from an earlier batch (negative relative ordinal) that partial's carry row (canonical attribute words)
namespace {
struct ProjLoader {
  const NfaStream* st;
  int64_t r1, r2;     // batch rows
  const int64_t* c1;  // e1's carry row, or nullptr
  __device__ StackVal var(const Instr& in) const {
    if (in.op == OP_COL) return col_value(st, in.a, r1);  // a single-stream query: column in.a of its row
    if (in.a == 0 && c1) {
      StackVal v = uncanon((uint64_t)c1[3 + in.c], in.t0);
      if (in.t0 == T_STRING) v.null = v.i < 0;
      return v;
    }
    return col_value(st, in.c, in.a == 0 ? r1 : r2);
  }
};

__device__ __forceinline__ int64_t batch_row(const int64_t* ord, int64_t n, int64_t base, uint32_t rel) {
  if (!ord) return (int64_t)rel;
  const int64_t want = base + (int64_t)rel;
  int64_t lo = 0, hi = n - 1;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (ord[mid] < want) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__global__ void carry_ord_keys_kernel(const int64_t* __restrict__ rows, int64_t n, int w, int64_t base,
                                      uint32_t* __restrict__ key, uint32_t* __restrict__ idx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  key[i] = (uint32_t)(rows[i * w + 1] - base + 0x80000000ll);  // carried ordinals lie in [base - 2^31, base)
  idx[i] = (uint32_t)i;
}

__global__ void pair_project_kernel(const uint32_t* __restrict__ pairs, int64_t m, const NfaStream* __restrict__ st,
                                    const int64_t* __restrict__ ord, int64_t n, int64_t base,
                                    const int64_t* __restrict__ ts, const int64_t* __restrict__ crow, int cw,
                                    const uint32_t* __restrict__ ckey, const uint32_t* __restrict__ cidx, int64_t nc,
                                    const char* __restrict__ blob, bool rows, DVal* __restrict__ out,
                                    int64_t* __restrict__ ts_out, int64_t* __restrict__ words,
                                    uint8_t* __restrict__ nulls) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= m) return;
  const DQuery* q = (const DQuery*)blob;
  const Instr* code = (const Instr*)(blob + q->off_code);
  const DVal* consts = (const DVal*)(blob + q->off_const);
  const int32_t* sel = (const int32_t*)(blob + q->off_sel);
  // rows: a filter query's kept rows (one event per output: slot 0 is the row itself)
  const uint32_t e1 = rows ? pairs[k] : pairs[2 * k], e2 = rows ? pairs[k] : pairs[2 * k + 1];
  ProjLoader ld{st, 0, batch_row(ord, n, base, e2), nullptr};
  if (!rows && (int32_t)e1 < 0) {  // carried e1: its row in the previous carry, by ordinal
    const uint32_t want = (uint32_t)((int32_t)e1 + 0x80000000ll);
    int64_t lo = 0, hi = nc - 1;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (ckey[mid] < want) lo = mid + 1;
      else hi = mid;
    }
    ld.c1 = crow + (int64_t)cidx[lo] * cw;
  } else {
    ld.r1 = batch_row(ord, n, base, e1);
  }
  if (words) {  // compact form (nsel <= 8): one 64-bit word per value, the null flags as bits of one byte
    int64_t* o = words + k * q->nsel;
    uint32_t nb = 0;
    for (int a = 0; a < q->nsel; ++a) {
      const StackVal v = eval_prog(code + sel[3 * a], sel[3 * a + 1], consts, ld);
      DVal d;
      if (sel[3 * a + 2] == T_FLOAT || sel[3 * a + 2] == T_DOUBLE) d.d = v.d;
      else d.i = v.i;
      o[a] = d.i;
      nb |= (v.null ? 1u : 0u) << a;
    }
    nulls[k] = (uint8_t)nb;
  } else {
    DVal* o = out + k * q->nsel;
    for (int a = 0; a < q->nsel; ++a) {
      const StackVal v = eval_prog(code + sel[3 * a], sel[3 * a + 1], consts, ld);
      DVal d;
      if (sel[3 * a + 2] == T_FLOAT || sel[3 * a + 2] == T_DOUBLE) d.d = v.d;
      else d.i = v.i;
      d.null = v.null;
      d.pad = 0;
      o[a] = d;
    }
  }
  if (ts_out) ts_out[k] = ts[ld.r2];  // StateEvent.timestamp: the last event's (e2's) event time
}
}  // namespace

void pair_project_carry_order(const int64_t* prev_carry, int64_t nc, int cw, int64_t base, Scratch& sc, hipStream_t s,
                              const uint32_t** carry_keys, const uint32_t** carry_idx) {
  uint32_t* ck = (uint32_t*)sc.take((size_t)nc * 4);
  uint32_t* ci = (uint32_t*)sc.take((size_t)nc * 4);
  uint32_t* ck2 = (uint32_t*)sc.take((size_t)nc * 4);
  uint32_t* ci2 = (uint32_t*)sc.take((size_t)nc * 4);
  hipLaunchKernelGGL(carry_ord_keys_kernel, grid_of(nc), dim3(256), 0, s, prev_carry, nc, cw, base, ck, ci);
  if (radix_sort_pairs<uint32_t>(ck, ck2, ci, ci2, (size_t)nc, 0, 32, sc, s)) {
    ck = ck2;
    ci = ci2;
  }
  *carry_keys = ck;
  *carry_idx = ci;
}

void pair_project(const uint32_t* pairs, int64_t m, const NfaStream* st_dev, const int64_t* ord, int64_t n,
                  int64_t base, const int64_t* ts, const int64_t* prev_carry, int64_t nc, int cw, const char* blob_dev,
                  DVal* out, int64_t* ts_out, Scratch& sc, hipStream_t s, bool rows, int64_t* words,
                  uint8_t* nulls, const uint32_t* carry_keys, const uint32_t* carry_idx, bool sync) {
  if (m <= 0) return;
  const size_t mark = sc.used;
  const uint32_t *ck = carry_keys, *ci = carry_idx;
  if (nc > 0 && !rows && !ck) pair_project_carry_order(prev_carry, nc, cw, base, sc, s, &ck, &ci);
  hipLaunchKernelGGL(pair_project_kernel, grid_of(m), dim3(256), 0, s, pairs, m, st_dev, ord, n, base, ts, prev_carry,
                     cw, ck, ci, nc, blob_dev, rows, out, ts_out, words, nulls);
  SM_HIP(hipGetLastError());
  if (sync) {
    SM_HIP(hipStreamSynchronize(s));
    sc.used = mark;
  }
}

}  // namespace sm

