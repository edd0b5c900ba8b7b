// Device side of the bucket-stack pipeline (stack.hip): the register stack, exact comparison of equal value codes,
// block scan, and the ring kernel (v4). A header of its own so that the same source also builds on the host under
// the wave emulator of tests/native/ (SM_HOST_EMU, hd.h), where tests/test_stack_emu.py checks the kernel against a
// plain per-key pending-list model on the CPU.
#pragma once
#include "fastpath_dev.h"

namespace sm {
namespace {

constexpr int kKeys = 1024;  // in-bucket keys
#ifndef SM_STACK_KC
#define SM_STACK_KC 5         // A/B build flag (v2, config 4, slices of 4608: 3 -> 34.9 ms, 4 -> 32.1, 5 -> 31.7)
#endif
constexpr int kC = SM_STACK_KC;  // stack entries held in registers
constexpr int kQ = 32;           // spilled entries per thread (HBM ring)
constexpr int kOB = 1024;        // order workgroup: thread d owns bucket d
#ifndef SM_ORDER_TB
#define SM_ORDER_TB 13  // A/B build flag (config 4 order kernel: 13 -> 6.65 ms, 15 (direct writes) -> 9.8 ms; round 6:
#endif                  // 14 with two placement passes per tile (stack.hip kSplit) 9.6 against 6.7 ms, same box)
constexpr int kTB = SM_ORDER_TB;  // order tile: 2^kTB consecutive relative ordinals
constexpr int kOT = 1 << kTB;

enum : uint32_t { SE_OVERFLOW = 1, SE_LOG = 2, SE_NAN = 4, SE_CAND = 8, SE_ORD = 16 };

// Exact value of a compared attribute: a batch row's column, or a carried partial's stored value.
struct ExactSrc {
  bool exact_codes;
  int vtype, vattr, cwidth;
  const void* vcol;
  const int64_t* ord;
  int64_t obase, n;
  const int64_t* crow;
  int32_t o0;
  uint32_t cs, ce;  // this key's carried rows
  __device__ bool carried(uint32_t o) const { return (int32_t)o < o0; }
  __device__ int64_t row_of(uint32_t o) const {
    if (!ord) return o;
    const int64_t want = (int64_t)o + obase;
    int64_t lo = 0, hi = n - 1;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (ord[mid] < want) lo = mid + 1;
      else hi = mid;
    }
    return lo;
  }
  __device__ int64_t carry_row(uint32_t o) const {
    const int64_t want = (int64_t)(int32_t)o + obase;
    uint32_t lo = cs, hi = ce;
    while (lo + 1 < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (crow[(int64_t)mid * cwidth + 1] <= want) lo = mid;
      else hi = mid;
    }
    return lo;
  }
  __device__ double fval(uint32_t o) const {
    if (carried(o)) return __longlong_as_double((long long)crow[carry_row(o) * cwidth + 3 + vattr]);
    const int64_t r = row_of(o);
    return vtype == T_FLOAT ? (double)((const float*)vcol)[r] : ((const double*)vcol)[r];
  }
  __device__ int64_t ival(uint32_t o) const {
    if (carried(o)) return crow[carry_row(o) * cwidth + 3 + vattr];
    const int64_t r = row_of(o);
    return vtype == T_INT ? (int64_t)((const int32_t*)vcol)[r] : ((const int64_t*)vcol)[r];
  }
};

// equal inexact codes (or NaN): the exact values decide. Out of line: rare, and its binary searches must not
// hold registers in the event loop; the source is passed by value (a reference would put it in scratch).
#ifndef SM_EXACT_INLINE
#define SM_EXACT_INLINE __noinline__
#endif
template <int OP, bool FP>
__device__ SM_EXACT_INLINE bool c2_exact_v(bool exact_codes, int vtype, int vattr, int cwidth, const void* vcol,
                                        const int64_t* ord, int64_t obase, int64_t n, const int64_t* crow, int32_t o0,
                                        uint32_t cs, uint32_t ce, uint32_t oi, uint32_t oj) {
  const ExactSrc ex{exact_codes, vtype, vattr, cwidth, vcol, ord, obase, n, crow, o0, cs, ce};
  if constexpr (FP) return cmp_fixed<OP>(ex.fval(oj), ex.fval(oi));
  else return cmp_fixed<OP>(ex.ival(oj), ex.ival(oi));
}
template <int OP, bool FP>
__device__ __forceinline__ bool c2_exact(const ExactSrc& ex, uint32_t oi, uint32_t oj) {
  return c2_exact_v<OP, FP>(ex.exact_codes, ex.vtype, ex.vattr, ex.cwidth, ex.vcol, ex.ord, ex.obase, ex.n, ex.crow,
                            ex.o0, ex.cs, ex.ce, oi, oj);
}

// c2 = `e2.x OP e1.x` for partial i (code ci, ordinal oi) and event j
template <int OP, bool FP>
__device__ __forceinline__ bool c2_hit(const ExactSrc& ex, uint32_t ci, uint32_t oi, uint32_t cj, uint32_t oj) {
  const bool nan = FP & ((ci == kNanCode) | (cj == kNanCode));
  if (!nan & (ex.exact_codes | (ci != cj))) return cmp_fixed<OP>(cj, ci);
  return c2_exact<OP, FP>(ex, oi, oj);
}

struct Stack {
  uint32_t o[kC], c[kC];
  int32_t t[kC];
  int n;       // entries in registers
  int hb, hn;  // spill ring: head, count
};

__device__ __forceinline__ void st_pop(Stack& s) {
#pragma unroll
  for (int k = 0; k + 1 < kC; ++k) {
    s.o[k] = s.o[k + 1];
    s.c[k] = s.c[k + 1];
    s.t[k] = s.t[k + 1];
  }
  --s.n;
}

// the registers ran empty: bring back the youngest spilled entry (one at a time; spills are rare)
__device__ __forceinline__ void st_refill(Stack& s, const uint4* sp) {
  const uint4 e = sp[(s.hb + s.hn - 1) & (kQ - 1)];
  s.o[0] = e.x;
  s.c[0] = e.y;
  s.t[0] = (int32_t)e.z;
  s.hn -= 1;
  s.n = 1;
}

// push (o, c, t) on top; `now` = event time of the pushing event (entries older than now - within are dead)
__device__ __forceinline__ void st_push(Stack& s, uint4* sp, uint32_t o, uint32_t c, int32_t t, int32_t now,
                                        int64_t within, uint32_t* err) {
  if (s.n == kC) {
    if (within >= 0 && now - s.t[kC - 1] > (int32_t)within) {  // the register bottom and all spilled are dead
      s.hn = 0;
      s.n = kC - 1;
    } else {
      if (s.hn == kQ) {  // free the ring's dead head first
#pragma unroll 1
        while (s.hn > 0 && within >= 0 && now - (int32_t)sp[s.hb & (kQ - 1)].z > (int32_t)within) {
          s.hb = (s.hb + 1) & (kQ - 1);
          --s.hn;
        }
        if (s.hn == kQ) {  // more than kC + kQ live partials on one key: the walk pipeline takes the batch
          atomicOr(err, SE_OVERFLOW);
          s.hb = (s.hb + 1) & (kQ - 1);
          --s.hn;
        }
      }
      sp[(s.hb + s.hn) & (kQ - 1)] = make_uint4(s.o[kC - 1], s.c[kC - 1], (uint32_t)s.t[kC - 1], 0u);
      ++s.hn;
      s.n = kC - 1;
    }
  }
#pragma unroll
  for (int k = kC - 1; k > 0; --k) {
    s.o[k] = s.o[k - 1];
    s.c[k] = s.c[k - 1];
    s.t[k] = s.t[k - 1];
  }
  s.o[0] = o;
  s.c[0] = c;
  s.t[0] = t;
  ++s.n;
}

// block-wide exclusive scan of one value per thread (NT threads); returns the total through *tot
template <int NT = kOB>
__device__ __forceinline__ uint32_t block_excl(uint32_t v, uint32_t* lw, uint32_t* tot) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(inc, o, 64);
    if (lane >= o) inc += u;
  }
  if (lane == 63) lw[w] = inc;
  lds_barrier();
  uint32_t r = inc - v, t = 0;
  for (int q = 0; q < NT / 64; ++q) {
    const uint32_t x = lw[q];
    if (q < w) r += x;
    t += x;
  }
  *tot = t;
  return r;
}

// ============================================================================================================
// v4 (default): the same closed form with a ring of ranked slices, so that no lane waits for the slowest key chain
// of one slice.
//   One workgroup per bucket (persistent), 1024 threads, thread h = in-bucket key h. The bucket is read once, in
//   slices of kSS records; kR consecutive slices are held in LDS, each ranked by key (wave64 ballot peer masks:
//   stable, arrival order within a key). In epoch e the slots hold slices e .. e+kR-1: every lane runs its key's
//   events against its register stack in one flat loop that must finish its events of slice e and may go on into
//   slices e+1 .. e+kR-1. A wave stops when all of its lanes have finished slice e, so a lane with many events in
//   slice e is mostly covered by lanes doing later slices' work instead of idling (simulated lane efficiency
//   0.58 against 0.35 for one slice at a time). Then slice e's matches are written (count per event, block scan,
//   placement at (offset of j) + (rank among j's pops counted from the oldest)) and slice e + kR is ranked into
//   the freed slot.
//   Per event the lane records its pops in the slot: the youngest popped e1 inline (pk, by arrival position), the
//   count (jc), and further pops in the slot's pool {i, position | k << 16}.
#ifndef SM_STACK_R
#define SM_STACK_R 2
#endif
#ifndef SM_STACK_SS
#define SM_STACK_SS 3072
#endif
constexpr int kR = SM_STACK_R;    // slices held in LDS
constexpr int kSS = SM_STACK_SS;  // records per slice
constexpr int kT4 = kKeys;        // threads: one in-bucket key each
constexpr int kW4 = kT4 / 64;     // waves (16): ranking counts per (key, wave) are 16 bytes per key
constexpr int kI4 = kSS / kT4;    // records per thread per slice
constexpr int kPool = kSS / 2;    // pops beyond the first per slice (more: the batch takes the sort / walk kernels)
static_assert(kSS % kT4 == 0 && kI4 * 64 <= 255 && kW4 == 16, "u8 per-(key, wave) counts, 16 waves");
static_assert(kSS <= 32768, "arrival positions | c1 fit 16 bits");

struct Slot4 {
  uint2 grp[kSS];       // key-grouped records {code, ts - ts0}
  uint32_t ordt[kSS];   // ordinal by arrival position
  uint32_t pk[kSS];     // youngest pop (e1 ordinal) by arrival position    } the ranking's u8 counts [key][wave]
  uint2 pool[kPool];    // further pops {e1 ordinal, position | k << 16}    } alias pk + pool (16 KB)
  uint32_t kst[kKeys];  // run of key h: start | count << 16
  uint16_t epos[kSS];   // key-grouped arrival position | c1 << 15; after the slice's epoch: output offset by position
  uint8_t jc[kSS];      // pops by arrival position
};
static_assert(sizeof(uint32_t) * kSS + sizeof(uint2) * kPool >= kKeys * kW4, "ranking counts fit pk + pool");

// fields the event loop does not read (exact comparisons of equal codes, carried partials, carry-out): one struct in
// device memory, read where needed, so that they hold no registers across the loop
struct Stack4Cold {
  int64_t kmin, ts0, within, obase, n;
  int vtype, vattr, cwidth;
  int32_t o0;
  bool exact_codes;
  const void* vcol;
  const int64_t* ord;
  const uint4* cin;
  const uint32_t* cstart;
  const uint32_t* cend;
  const int64_t* crow;
  int64_t* cand;
  uint32_t* cand_n;
  uint32_t cand_cap;
};

#ifndef SM_EXACT4_INLINE
#define SM_EXACT4_INLINE __noinline__
#endif
struct Stack4Args {
  const uint4* rec;
  const uint32_t* dbase;
  uint32_t n;  // records (< 2^32: ordinals are u32)
  int H;
  int32_t within;  // < 0: no `within`
  bool exact_codes;
  uint32_t ntiles;
  const uint32_t* sbase;
  uint64_t* stage;
  uint32_t* mstart;
  uint32_t* mtot;
  uint4* spill;
  uint32_t* err;
  const Stack4Cold* cold;
  unsigned long long* stamps;  // SM_STACK4_STAMPS builds: shader clocks per phase, summed over waves
};

#ifndef SM_STACK4_SKIP
#define SM_STACK4_SKIP 0  // diagnostic build flag: 1 = no event loop (every pop count 0; wrong results, timing only)
#endif
#ifndef SM_STACK4_STAMPS
#define SM_STACK4_STAMPS 0  // diagnostic build flag: phase clock of stack4_kernel (0 rank, 1 stacks, 2 wait, 3 emit, 4 rest)
#endif
#if SM_STACK4_STAMPS && defined(__HIP_DEVICE_COMPILE__)
#define SM4_CLOCK() __builtin_amdgcn_s_memtime()
#else
#define SM4_CLOCK() 0ull
#endif
#define SM4_PHASE(i)                              \
  do {                                            \
    if (SM_STACK4_STAMPS) {                       \
      const unsigned long long t_ = SM4_CLOCK();  \
      st_acc[i] += t_ - st_last;                  \
      st_last = t_;                               \
    }                                             \
  } while (0)

template <int OP, bool FP>
__device__ SM_EXACT4_INLINE bool c2_exact4(const Stack4Cold* c, uint32_t cs, uint32_t ce, uint32_t oi, uint32_t oj) {
  return c2_exact_v<OP, FP>(c->exact_codes, c->vtype, c->vattr, c->cwidth, c->vcol, c->ord, c->obase, c->n, c->crow,
                            c->o0, cs, ce, oi, oj);
}

#ifndef SM_RANK4_INLINE
#define SM_RANK4_INLINE __forceinline__
#endif
// rank slice [q0, q0 + sn) of the bucket (records in pre[]) into slot S: key runs (kst), key-grouped {code, ts}
// and arrival positions | c1, ordinals by arrival position
__device__ SM_RANK4_INLINE void rank4(Slot4& S, const uint4 (&pre)[kI4], int sn, uint32_t* lw, bool fp,
                                       uint32_t* err) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  uint8_t* cnt = (uint8_t*)S.pk;  // [key][wave]
  *(uint4*)(cnt + 16 * tid) = make_uint4(0, 0, 0, 0);
  lds_barrier();
  const uint64_t lt = lanemask_lt();
  uint32_t hk[kI4], lp[kI4];
  bool nan = false;
#pragma unroll
  for (int k = 0; k < kI4; ++k) {
    const int e = w * 64 * kI4 + k * 64 + lane;
    const bool valid = e < sn;
    nan |= fp && valid && pre[k].z == kNanCode;  // a NaN sends the batch to the sort / walk kernels (SE_NAN)
    hk[k] = valid ? (pre[k].x & kKeyMask) >> kRB : 0u;
    const uint64_t peers = peer_mask(hk[k], valid);
    uint32_t old = 0;
    if (valid) old = cnt[16 * hk[k] + w];
    wave_lockstep();
    const uint32_t below = (uint32_t)__popcll(peers & lt);
    if (valid && below == 0) cnt[16 * hk[k] + w] = (uint8_t)(old + (uint32_t)__popcll(peers));
    wave_lockstep();
    lp[k] = old + below;
  }
  if (__any(nan) && lane == 0) atomicOr(err, SE_NAN);
  lds_barrier();
  {  // key h = tid: its count over the waves, block scan over keys
    const uint4 c = *(const uint4*)(cnt + 16 * tid);
    const uint32_t ones = 0x01010101u;
    const uint32_t tot = sm_udot4(c.x, ones, 0u) + sm_udot4(c.y, ones, 0u) +
                         sm_udot4(c.z, ones, 0u) + sm_udot4(c.w, ones, 0u);
    uint32_t all;
    const uint32_t st = block_excl<kT4>(tot, lw, &all);
    S.kst[tid] = st | (tot << 16);
  }
  lds_barrier();
#pragma unroll
  for (int k = 0; k < kI4; ++k) {
    const int e = w * 64 * kI4 + k * 64 + lane;
    if (e < sn) {
      // same-key records of earlier waves: the bytes of waves 0 .. w-1 in the key's 16-byte row
      const uint4 c = *(const uint4*)(cnt + 16 * hk[k]);
      const uint32_t wb = (uint32_t)w * 8u;  // bits of the row below wave w
      auto part = [&](uint32_t word, uint32_t lo) {
        const uint32_t nb = wb > lo ? (wb - lo >= 32u ? 32u : wb - lo) : 0u;
        const uint32_t m = nb >= 32u ? 0xffffffffu : ((1u << nb) - 1u);
        return sm_udot4(word & m, 0x01010101u, 0u);
      };
      const uint32_t before = part(c.x, 0) + part(c.y, 32) + part(c.z, 64) + part(c.w, 96);
      const uint32_t pos = (S.kst[hk[k]] & 0xffffu) + before + lp[k];
      S.grp[pos] = make_uint2(pre[k].z, pre[k].w);
      S.epos[pos] = (uint16_t)((uint32_t)e | ((pre[k].x >> 31) << 15));
      S.ordt[e] = pre[k].y;
      if (SM_STACK4_SKIP) S.jc[e] = 0;
    }
  }
  lds_barrier();
}

template <int OP, bool FP>
__global__ void __launch_bounds__(kT4) stack4_kernel(Stack4Args a) {
  __shared__ __attribute__((aligned(16))) Slot4 sl[kR];
  __shared__ uint32_t lw[kW4];
  __shared__ uint32_t s_pool[kR];
  __shared__ uint32_t s_lastj, s_tot;
  const int tid = threadIdx.x, lane = tid & 63;
  const int h = tid;
  const bool has = h < a.H;
  const int32_t within32 = a.within;
  uint4* sp = a.spill + ((int64_t)blockIdx.x * kKeys + h) * kQ;
  unsigned long long st_acc[5] = {0, 0, 0, 0, 0}, st_last = SM4_CLOCK();

  for (int d = blockIdx.x; d < kBins; d += gridDim.x) {
    const uint32_t b0 = a.dbase[d];
    const uint32_t blen = (d + 1 < kBins ? a.dbase[d + 1] : a.n) - b0;
    const uint32_t nsl = (blen + kSS - 1) / kSS;
    const uint4* recb = a.rec + b0;
    uint64_t* stb = a.stage + a.sbase[d];
    uint32_t* mst = a.mstart + (int64_t)d * (a.ntiles + 1);
    const uint32_t kr = ((uint32_t)h << kRB) | (uint32_t)d;
    Stack st;
    st.n = st.hb = st.hn = 0;
    uint32_t cs = 0, ce = 0;
    if (has && a.cold->cin) {  // carried partials first (oldest first)
      const Stack4Cold* c4 = a.cold;
      cs = c4->cstart[kr];
      ce = c4->cend[kr];
      for (uint32_t q = cs; q < ce; ++q) {
        const uint4 c = c4->cin[q];
        st_push(st, sp, c.x, c.y, (int32_t)c.z, (int32_t)c.z, within32, a.err);
      }
    }
    int32_t tl = 0;
    bool seen = false;
    uint32_t mrun = 0;
    __syncthreads();  // the previous bucket's readers of the slots are done
    if (tid == 0) s_lastj = 0xffffffffu;
    if (tid < kR) s_pool[tid] = 0;

    uint4 pre[kI4];
    auto load = [&](uint32_t s) {
#pragma unroll
      for (int k = 0; k < kI4; ++k) {
        const uint32_t p = s * kSS + (tid >> 6) * 64 * kI4 + k * 64 + lane;
        if (p < blen) {
          typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
          const u32x4 v = __builtin_nontemporal_load((const u32x4*)recb + p);
          pre[k] = make_uint4(v.x, v.y, v.z, v.w);
        }
      }
    };
    auto slice_n = [&](uint32_t s) { return (int)(blen - s * kSS < (uint32_t)kSS ? blen - s * kSS : (uint32_t)kSS); };
    // the lane's runs in the held slices, relative to the epoch: k = 0 is slice e
    uint32_t off[kR], cnt[kR];
    SM4_PHASE(4);
    for (uint32_t s = 0; s < (uint32_t)kR; ++s) {
      off[s] = cnt[s] = 0;
      if (s < nsl) {
        load(s);
        rank4(sl[s], pre, slice_n(s), lw, FP, a.err);
        const uint32_t v = sl[s].kst[h];
        off[s] = v & 0xffffu;
        cnt[s] = v >> 16;
      }
    }
    if (kR < nsl) load(kR);

    SM4_PHASE(0);
    for (uint32_t e = 0; e < nsl; ++e) {
      const int q0 = (int)(e % kR);
      // ---- stack phase: finish this lane's events of slice e; go on into the later held slices meanwhile
      while (!SM_STACK4_SKIP && __any(cnt[0] != 0)) {
        // the lane's next event: its first held slice with events left
        int k = kR - 1;
#pragma unroll
        for (int u = kR - 2; u >= 0; --u)
          if (cnt[u]) k = u;
        uint32_t o_ = off[kR - 1], c_ = cnt[kR - 1];
#pragma unroll
        for (int u = kR - 2; u >= 0; --u)
          if (u == k) {
            o_ = off[u];
            c_ = cnt[u];
          }
        if (c_ != 0) {  // else nothing is held for this lane: it waits for the wave
#pragma unroll
        for (int u = 0; u < kR; ++u)
          if (u == k) {
            off[u] = o_ + 1;
            cnt[u] = c_ - 1;
          }
        const int q = q0 + k >= kR ? q0 + k - kR : q0 + k;
        Slot4& S = sl[q];
        const uint2 g = S.grp[o_];
        const uint32_t ep = S.epos[o_];
        const uint32_t p = ep & 0x7fffu;
        const uint32_t cj = g.x;
        const int32_t jt = (int32_t)g.y;
        tl = jt;
        seen = true;
        // a NaN anywhere sent the batch to the sort / walk kernels (rank4: SE_NAN), so the codes alone decide here
        uint32_t hit = 0, exp = 0, tie = 0;
#pragma unroll
        for (int u = 0; u < kC; ++u) {
          const bool lv = u < st.n;
          hit |= (lv && cmp_fixed<OP>(cj, st.c[u])) ? (1u << u) : 0u;
          exp |= (lv && within32 >= 0 && jt - st.t[u] > within32) ? (1u << u) : 0u;
          tie |= (lv && !a.exact_codes && st.c[u] == cj) ? (1u << u) : 0u;
        }
        if (tie) {  // equal inexact codes: the exact values decide (out of line, one call site)
          const uint32_t oj = S.ordt[p];
#pragma unroll 1
          for (uint32_t m = tie; m; m &= m - 1u) {
            const int u = __builtin_ctz(m);
            uint32_t oi = st.o[0];
#pragma unroll
            for (int v = 1; v < kC; ++v)
              if (v == u) oi = st.o[v];
            if (c2_exact4<OP, FP>(a.cold, cs, ce, oi, oj)) hit |= 1u << u;
            else hit &= ~(1u << u);
          }
        }
        const uint32_t ok = hit & ~exp;
        uint32_t npop = (uint32_t)__builtin_ctz(~ok);  // leading entries popped
        if (npop > (uint32_t)st.n) npop = st.n;
        const bool stop_expired = npop < (uint32_t)st.n && ((exp >> npop) & 1u);
        const bool cont = !stop_expired && npop == (uint32_t)st.n && st.hn > 0;
        if (npop) S.pk[p] = st.o[0];
        if (npop > 1) {  // further pops go to the slot's pool
          const uint32_t base = atomicAdd(&s_pool[q], npop - 1u);
          if (base + npop - 1u > (uint32_t)kPool) atomicOr(a.err, SE_LOG);
#pragma unroll
          for (int u = 1; u < kC; ++u)
            if ((uint32_t)u < npop && base + u - 1u < (uint32_t)kPool)
              S.pool[base + u - 1u] = make_uint2(st.o[u], p | ((uint32_t)u << 16));
        }
        // shift the register part down by npop
#pragma unroll
        for (int b = 1; b < kC; b <<= 1)
          if (npop & b) {
#pragma unroll
            for (int u = 0; u < kC; ++u)
              if (u + b < kC) {
                st.o[u] = st.o[u + b];
                st.c[u] = st.c[u + b];
                st.t[u] = st.t[u + b];
              }
          }
        st.n -= (int)npop;
        if (stop_expired) {  // the entry that stopped the run has expired: so has every older one
          st.n = 0;
          st.hn = 0;
        } else if (cont) {  // ran through the registers: continue into the spill ring (rare)
#pragma unroll 1
          for (;;) {
            st_refill(st, sp);
            if (within32 >= 0 && jt - st.t[0] > within32) {
              st.n = 0;
              st.hn = 0;
              break;
            }
            const bool hh = (a.exact_codes | (st.c[0] != cj)) ? cmp_fixed<OP>(cj, st.c[0])
                                                               : c2_exact4<OP, FP>(a.cold, cs, ce, st.o[0], S.ordt[p]);
            if (!hh) break;
            if (npop == 0) {
              S.pk[p] = st.o[0];
            } else {  // each spilled pop reserves its own pool entry
              const uint32_t b1 = atomicAdd(&s_pool[q], 1u);
              if (b1 < (uint32_t)kPool) S.pool[b1] = make_uint2(st.o[0], p | (npop << 16));
              else atomicOr(a.err, SE_LOG);
            }
            ++npop;
            st_pop(st);
            if (st.hn == 0) break;
          }
        }
        S.jc[p] = (uint8_t)npop;
        if (ep >> 15) st_push(st, sp, S.ordt[p], cj, jt, jt, within32, a.err);
        }
      }
      SM4_PHASE(1);
      lds_barrier();  // every lane is done with slice e
      SM4_PHASE(2);

      // ---- slice e's matches, in arrival order of j
      {
        Slot4& S = sl[q0];
        const int sn = slice_n(e);
        uint32_t v[kI4], sum = 0;
#pragma unroll
        for (int k = 0; k < kI4; ++k) {
          const int p = tid * kI4 + k;
          v[k] = p < sn ? S.jc[p] : 0u;
          sum += v[k];
        }
        uint32_t tot;
        uint32_t r = block_excl<kT4>(sum, lw, &tot);
        const uint32_t jprev = s_lastj;
#pragma unroll
        for (int k = 0; k < kI4; ++k) {
          const int p = tid * kI4 + k;
          if (p < sn) {
            S.epos[p] = (uint16_t)r;  // the key-grouped positions are dead: output offsets by arrival position
            const uint32_t j = S.ordt[p];
            // ordinal tiles whose first ordinal falls in (previous record's ordinal, this record's]: their first
            // match in this bucket is this record's first
            const uint32_t jp = p == 0 ? jprev : S.ordt[p - 1];
            const uint32_t t0 = jp == 0xffffffffu ? 0u : (jp >> kTB) + 1u;
            for (uint32_t t = t0; t <= (j >> kTB); ++t) mst[t] = mrun + r;
            if (v[k]) stb[mrun + r + v[k] - 1u] = ((uint64_t)j << 32) | S.pk[p];
          }
          r += v[k];
        }
        if (tid == 0) s_tot = tot;
        lds_barrier();
        const uint32_t np = s_pool[q0] < (uint32_t)kPool ? s_pool[q0] : (uint32_t)kPool;
        for (uint32_t k = tid; k < np; k += kT4) {
          const uint2 pe = S.pool[k];
          const uint32_t p = pe.y & 0xffffu, kk = pe.y >> 16;
#ifdef SM_EMU_DEBUG
          if (kk >= S.jc[p] || p >= (uint32_t)sn) {
            printf("bad pool entry k=%u/%u p=%u kk=%u jc=%u epos=%u sn=%d e=%u q0=%d d=%d\n", k, np, p, kk, S.jc[p], S.epos[p], sn, e, q0, d);
            continue;
          }
#endif
          stb[mrun + S.epos[p] + S.jc[p] - 1u - kk] = ((uint64_t)S.ordt[p] << 32) | pe.x;
        }
        mrun += s_tot;
        lds_barrier();
        if (tid == 0) {
          s_lastj = S.ordt[sn - 1];
          s_pool[q0] = 0;
        }
      }
      SM4_PHASE(3);
      // ---- slice e + kR into the freed slot
      off[0] = off[1];
      cnt[0] = cnt[1];
#pragma unroll
      for (int u = 1; u + 1 < kR; ++u) {
        off[u] = off[u + 1];
        cnt[u] = cnt[u + 1];
      }
      off[kR - 1] = cnt[kR - 1] = 0;
      if (e + kR < nsl) {
        rank4(sl[q0], pre, slice_n(e + kR), lw, FP, a.err);
        const uint32_t vv = sl[q0].kst[h];
        off[kR - 1] = vv & 0xffffu;
        cnt[kR - 1] = vv >> 16;
        if (e + kR + 1 < nsl) load(e + kR + 1);  // lands during the next stack phase
      }
      SM4_PHASE(0);
    }
    // tiles after the bucket's last record start at its end
    __syncthreads();
    {
      const uint32_t jl = s_lastj;
      const uint32_t t0 = jl == 0xffffffffu ? 0u : (jl >> kTB) + 1u;
      for (uint32_t t = t0 + tid; t <= (uint32_t)a.ntiles; t += kT4) mst[t] = mrun;
      if (tid == 0) a.mtot[d] = mrun;
    }

    // ---- carry out: the partials still pending in the reference (not matched, not found expired by the key's
    // last event; a key without events in this batch keeps all of its carried partials)
    auto pending = [&](int32_t t) { return !seen || within32 < 0 || (int64_t)tl - t <= within32; };
    uint32_t keep = 0;
    if (has) {
#pragma unroll
      for (int k = 0; k < kC; ++k)
        if (k < st.n && pending(st.t[k])) ++keep;
      for (int k = 0; k < st.hn; ++k)
        if (pending((int32_t)sp[(st.hb + k) & (kQ - 1)].z)) ++keep;
    }
    uint32_t inc = keep;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(inc, o, 64);
      if (lane >= o) inc += u;
    }
    uint32_t base = 0;
    const Stack4Cold* c4 = a.cold;
    if (lane == 63 && inc) base = atomicAdd(c4->cand_n, inc);
    base = __shfl(base, 63, 64) + inc - keep;
    if (keep) {
      const ExactSrc ex{c4->exact_codes, c4->vtype, c4->vattr, c4->cwidth, c4->vcol, c4->ord, c4->obase, c4->n,
                        c4->crow, c4->o0, cs, ce};
      const int64_t key = c4->kmin + (int64_t)kr;
      auto put = [&](uint32_t o, int32_t t) {
        if (!pending(t)) return;
        if (base < c4->cand_cap) {
          int64_t* c = c4->cand + 4 * (int64_t)base;
          c[0] = key;
          c[1] = (int64_t)(int32_t)o + c4->obase;
          c[2] = (int64_t)t + c4->ts0;
          c[3] = ex.carried(o) ? -(int64_t)ex.carry_row(o) - 1 : ex.row_of(o);
        } else {
          atomicOr(a.err, SE_CAND);
        }
        ++base;
      };
      // one run per key, oldest first (build_carry's key_runs_ordered relies on it): spill ring, then registers
      for (int k = 0; k < st.hn; ++k) {
        const uint4 c = sp[(st.hb + k) & (kQ - 1)];
        put(c.x, (int32_t)c.z);
      }
#pragma unroll
      for (int k = kC - 1; k >= 0; --k)
        if (k < st.n) put(st.o[k], st.t[k]);
    }
  }
  SM4_PHASE(4);
  if (SM_STACK4_STAMPS && a.stamps && lane == 0)
    for (int i = 0; i < 5; ++i) atomicAdd(&a.stamps[i], st_acc[i]);
}

}  // namespace
}  // namespace sm
