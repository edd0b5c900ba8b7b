// FilterProcessor over a device-resident batch (config 2 `StockStream[price > 70 and
// volume < 1000]`): `FilterProcessor.process` (core/query/processor/filter/FilterProcessor.java:50-62) keeps the
// events whose condition is true, in arrival order. Output: the uint32 row (ordinal - base) of every kept event.
//
// Two HBM passes, both streaming:
//   count  read the columns the condition references once (the only per-event bytes), evaluate, one ballot
//          word per 64 rows (staged in LDS, written coalesced per block) and one count per block
//   scan   exclusive over the block counts (primitives.hip)
//   write  read the mask words only, write the kept rows (u32) at their block offset + in-block rank
// Conditions that are a conjunction of up to kMaxLeaves leaves `x CMP y` (x, y a column or a constant; And
// tree shapes of any association) take the typed form: every column load of a block's rows is issued before any
// comparison, comparisons use the compare executor's own promotion (do_compare: the CMP instruction's t0/t1/t2,
// CompareConditionExpressionExecutor.java:39-43). Anything else (or, not, math, strings, nulls) is evaluated by
// the bytecode interpreter in the same two-pass frame.
#include "expr.h"
#include "filter.h"

namespace sm {

namespace {

constexpr int kFBlock = 256;
constexpr int kFWaves = kFBlock / 64;
constexpr int kFItems = 16;                     // rows per thread
constexpr int kFTile = kFBlock * kFItems;       // 4096 rows per block
constexpr int kFWords = kFTile / 64;            // mask words per block

struct FLeafDev {  // column CMP constant (the host mirrors `constant CMP column`)
  Instr cmp;        // operator + promotion types (t1 = column side, t2 = constant side)
  int32_t col;
  int32_t ctype;
  StackVal k;
};

struct FSpecDev {
  int32_t nleaf;
  FLeafDev leaf[kFilterMaxLeaves];
  const void* cols[kMaxAttrs];
};

// One leaf over the thread's kFItems rows: column type T, compare domain D (Java binary numeric promotion:
// static_cast is Java's widening / int→float conversion). The operator is applied branch-free from the
// lt / eq / gt flags (NaN: all false, so only != holds, as in Java).
template <typename T, typename D>
__device__ __forceinline__ void leaf_items(const T* __restrict__ col, const FLeafDev& L, int64_t base, int64_t n,
                                           bool (&pass)[kFItems]) {
  T v[kFItems];
#pragma unroll
  for (int k = 0; k < kFItems; ++k)
    if (base + k * 64 < n) v[k] = __builtin_nontemporal_load(col + base + k * 64);
  const D y = is_fp(L.cmp.t2) ? (D)L.k.d : (D)L.k.i;
  const int op = L.cmp.sub;
  const bool ne = op == CMP_NE;
  const bool mlt = op == CMP_LT || op == CMP_LE, meq = op == CMP_EQ || op == CMP_LE || op == CMP_GE,
             mgt = op == CMP_GT || op == CMP_GE;
#pragma unroll
  for (int k = 0; k < kFItems; ++k) {
    const D x = static_cast<D>(v[k]);
    const bool lt = x < y, eq = x == y, gt = x > y;
    const bool r = ne ? !eq : ((lt && mlt) || (eq && meq) || (gt && mgt));
    pass[k] = pass[k] && r;
  }
}

template <typename T>
__device__ __forceinline__ void leaf_col(const T* col, const FLeafDev& L, int64_t base, int64_t n,
                                         bool (&pass)[kFItems]) {
  switch (L.cmp.t0) {  // wave-uniform
    case CT_INT: leaf_items<T, int32_t>(col, L, base, n, pass); break;
    case CT_LONG: leaf_items<T, int64_t>(col, L, base, n, pass); break;
    case CT_FLOAT: leaf_items<T, float>(col, L, base, n, pass); break;
    default: leaf_items<T, double>(col, L, base, n, pass); break;
  }
}

// count pass, typed leaves: NL leaves; per leaf every load of the thread's rows is issued before the first
// comparison
template <int NL>
__global__ void __launch_bounds__(kFBlock) filter_count_leaves_kernel(const FSpecDev* __restrict__ spec, int64_t n,
                                                                      uint64_t* __restrict__ masks,
                                                                      uint32_t* __restrict__ counts) {
  __shared__ uint64_t wmask[kFWords];
  __shared__ uint32_t wsum[kFWaves];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t base = (int64_t)blockIdx.x * kFTile + (int64_t)w * 64 * kFItems + lane;
  bool pass[kFItems];
#pragma unroll
  for (int k = 0; k < kFItems; ++k) pass[k] = base + k * 64 < n;
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    const FLeafDev& L = spec->leaf[l];
    const void* col = spec->cols[L.col];
    switch (L.ctype) {  // wave-uniform
      case T_INT: leaf_col((const int32_t*)col, L, base, n, pass); break;
      case T_LONG: leaf_col((const int64_t*)col, L, base, n, pass); break;
      case T_FLOAT: leaf_col((const float*)col, L, base, n, pass); break;
      default: leaf_col((const double*)col, L, base, n, pass); break;
    }
  }
  uint32_t cnt = 0;
#pragma unroll
  for (int k = 0; k < kFItems; ++k) {
    const uint64_t m = __ballot(pass[k]);
    if (lane == 0) wmask[w * kFItems + k] = m;
    cnt += (uint32_t)__popcll(m);
  }
  if (lane == 0) wsum[w] = cnt;
  __syncthreads();
  const int64_t w0 = (int64_t)blockIdx.x * kFWords, nw = (n + 63) >> 6;
  if (threadIdx.x < kFWords && w0 + threadIdx.x < nw) masks[w0 + threadIdx.x] = wmask[threadIdx.x];
  if (threadIdx.x == 0) {
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < kFWaves; ++k) s += wsum[k];
    counts[blockIdx.x] = s;
  }
}

struct StreamLoader {
  const NfaStream* st;
  int64_t row;
  __device__ StackVal var(const Instr& in) const {
    StackVal v;
    v.i = 0;
    v.d = 0;
    v.null = 0;
    const int a = in.a;
    if (st->nulls[a] && st->nulls[a][row]) {
      v.null = 1;
      return v;
    }
    switch (st->types[a]) {
      case T_INT: v.i = ((const int32_t*)st->cols[a])[row]; break;
      case T_LONG: v.i = ((const int64_t*)st->cols[a])[row]; break;
      case T_FLOAT: v.d = (double)((const float*)st->cols[a])[row]; break;
      case T_DOUBLE: v.d = ((const double*)st->cols[a])[row]; break;
      case T_STRING: v.i = ((const int32_t*)st->cols[a])[row]; v.null = v.i < 0; break;
      default: v.i = ((const uint8_t*)st->cols[a])[row]; break;
    }
    return v;
  }
};

// count pass, any condition: the bytecode interpreter per row (same block / mask layout as the typed form)
__global__ void __launch_bounds__(kFBlock) filter_count_prog_kernel(const NfaStream* __restrict__ st, int64_t n,
                                                                    const Instr* __restrict__ code, int len,
                                                                    const DVal* __restrict__ consts,
                                                                    uint64_t* __restrict__ masks,
                                                                    uint32_t* __restrict__ counts) {
  __shared__ uint64_t wmask[kFWords];
  __shared__ uint32_t wsum[kFWaves];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t base = (int64_t)blockIdx.x * kFTile + (int64_t)w * 64 * kFItems + lane;
  uint32_t cnt = 0;
  for (int k = 0; k < kFItems; ++k) {
    const int64_t row = base + k * 64;
    const bool pass = row < n && (len == 0 || truthy(eval_prog(code, len, consts, StreamLoader{st, row})));
    const uint64_t m = __ballot(pass);
    if (lane == 0) wmask[w * kFItems + k] = m;
    cnt += (uint32_t)__popcll(m);
  }
  if (lane == 0) wsum[w] = cnt;
  __syncthreads();
  const int64_t w0 = (int64_t)blockIdx.x * kFWords, nw = (n + 63) >> 6;
  if (threadIdx.x < kFWords && w0 + threadIdx.x < nw) masks[w0 + threadIdx.x] = wmask[threadIdx.x];
  if (threadIdx.x == 0) {
    uint32_t s = 0;
    for (int k = 0; k < kFWaves; ++k) s += wsum[k];
    counts[blockIdx.x] = s;
  }
}

// write pass: mask words → kept rows (u32, ordinal - base when explicit ordinals are given). One block per
// kWTiles count-pass tiles; wave w handles tiles w, w + kFWaves, ...: lane l loads the tile's mask word l, the
// wave scans the popcounts, each lane expands its word's set bits into the wave's LDS buffer, and the wave
// then stores the tile's kept rows as one contiguous, coalesced run.
constexpr int kWTiles = 16;
constexpr int kWPerWave = kWTiles / kFWaves;
__global__ void __launch_bounds__(kFBlock) filter_write_u32_kernel(const uint64_t* __restrict__ masks, int64_t n,
                                                                   const uint32_t* __restrict__ offsets,
                                                                   int64_t ntiles, const int64_t* __restrict__ ord,
                                                                   int64_t obase, uint32_t* __restrict__ out) {
  __shared__ uint16_t buf[kFWaves][kFTile];  // kept rows of the wave's current tile, relative to the tile
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t nw = (n + 63) >> 6;
  // every mask word and tile offset of the wave's tiles in flight at once
  uint64_t mw[kWPerWave];
  uint32_t ow[kWPerWave];
#pragma unroll
  for (int t = 0; t < kWPerWave; ++t) {
    const int64_t tile = (int64_t)blockIdx.x * kWTiles + t * kFWaves + w;
    const int64_t wi = tile * kFWords + lane;
    mw[t] = tile < ntiles && wi < nw ? masks[wi] : 0ull;
    ow[t] = tile < ntiles ? offsets[tile] : 0u;
  }
#pragma unroll
  for (int t = 0; t < kWPerWave; ++t) {
    const int64_t tile = (int64_t)blockIdx.x * kWTiles + t * kFWaves + w;
    if (tile >= ntiles) break;
    uint64_t m = mw[t];
    const uint32_t c = (uint32_t)__popcll(m);
    uint32_t inc = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t x = __shfl_up(inc, o, 64);
      if (lane >= o) inc += x;
    }
    const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane(inc, 63);
    uint32_t p = inc - c;
    while (m) {
      buf[w][p++] = (uint16_t)(lane * 64 + __ffsll((unsigned long long)m) - 1);
      m &= m - 1;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t row0 = (uint32_t)(tile * kFTile);
    for (uint32_t q = lane; q < tot; q += 64) {
      const uint32_t row = row0 + buf[w][q];
      out[ow[t] + q] = ord ? (uint32_t)(ord[row] - obase) : row;
    }
    __builtin_amdgcn_wave_barrier();  // buffer reads done before the next tile's expansion
  }
}

static_assert(kFWords == 64, "write pass scans one mask word per lane of one wave");

}  // namespace

bool filter_leaves(const Instr* code, int len, const DVal* consts, const int32_t* types, int nattr,
                   FilterLeaves& out) {
  out.n = 0;
  if (len == 0) return false;  // no condition: the interpreter form counts every row
  // postfix: operand, operand, CMP → one leaf; AND of two conjunctions → their union
  std::vector<int> stk;  // number of leaves of each conjunction on the stack (-1 = plain operand)
  std::vector<FilterLeaf> leaves;
  std::vector<Instr> ops;
  for (int pc = 0; pc < len; ++pc) {
    const Instr& in = code[pc];
    if (in.op == OP_CONST || in.op == OP_COL) {
      if (in.op == OP_COL) {
        if (in.a < 0 || in.a >= nattr) return false;
        const int t = types[in.a];
        if (t != T_INT && t != T_LONG && t != T_FLOAT && t != T_DOUBLE) return false;
      } else if (consts[in.a].null) {
        return false;
      }
      ops.push_back(in);
      stk.push_back(-1);
    } else if (in.op == OP_CMP) {
      if (stk.size() < 2 || stk[stk.size() - 1] != -1 || stk[stk.size() - 2] != -1) return false;
      FilterLeaf L;
      L.cmp = in;
      for (int s = 0; s < 2; ++s) {
        const Instr& o = ops[ops.size() - 2 + s];
        L.is_col[s] = o.op == OP_COL;
        L.idx[s] = o.a;
      }
      if (L.is_col[0] == L.is_col[1]) return false;  // column vs column / constant folding: interpreter
      ops.resize(ops.size() - 2);
      stk.resize(stk.size() - 2);
      leaves.push_back(L);
      stk.push_back(1);
    } else if (in.op == OP_AND) {
      if (stk.size() < 2 || stk[stk.size() - 1] < 1 || stk[stk.size() - 2] < 1) return false;
      const int t = stk[stk.size() - 1] + stk[stk.size() - 2];
      stk.resize(stk.size() - 2);
      stk.push_back(t);
    } else {
      return false;
    }
  }
  if (stk.size() != 1 || stk[0] < 1 || (int)leaves.size() > kFilterMaxLeaves) return false;
  out.n = (int)leaves.size();
  for (int l = 0; l < out.n; ++l) out.leaf[l] = leaves[l];
  return true;
}

int64_t filter_device(const NfaStream& st_host, const NfaStream* st_dev, int64_t n, const Instr* code_dev,
                      const Instr* code_host, int len, const DVal* consts_dev, const DVal* consts_host,
                      const int64_t* ordinals, int64_t ordinal_base, uint32_t* out, Scratch& sc, hipStream_t s,
                      FastTimings* tm, bool* typed_out) {
  if (n == 0) return 0;
  if (n > (int64_t)UINT32_MAX) throw std::invalid_argument("device filter batches hold at most 2^32 - 1 rows");
  const size_t mark = sc.used;
  const int64_t nblocks = (n + kFTile - 1) / kFTile;
  uint64_t* masks = (uint64_t*)sc.take(nblocks * kFWords * 8);
  uint32_t* counts = (uint32_t*)sc.take((nblocks + 1) * 4);
  uint32_t* total = (uint32_t*)sc.take(4);
  FilterLeaves fl;
  const bool typed = filter_leaves(code_host, len, consts_host, st_host.types, st_host.nattr, fl);
  bool nulls = false;
  for (int a = 0; a < st_host.nattr; ++a) nulls |= st_host.nulls[a] != nullptr;
  if (tm) {
    tm->nmk = 0;
    tm->mark("start", s);
  }
  if (typed && !nulls) {
    FSpecDev h;
    memset(&h, 0, sizeof(h));
    h.nleaf = fl.n;
    for (int a = 0; a < st_host.nattr; ++a) h.cols[a] = st_host.cols[a];
    for (int l = 0; l < fl.n; ++l) {
      const FilterLeaf& L = fl.leaf[l];
      FLeafDev& D = h.leaf[l];
      D.cmp = L.cmp;
      const int cs = L.is_col[0] ? 0 : 1;  // the column side; `k CMP col` is evaluated as `col CMP' k`
      D.col = L.idx[cs];
      D.ctype = st_host.types[D.col];
      const DVal c = consts_host[L.idx[1 - cs]];
      D.k.i = c.i;
      D.k.d = c.d;
      D.k.null = c.null;
      if (cs == 1) {
        std::swap(D.cmp.t1, D.cmp.t2);
        static const int32_t mirror[6] = {CMP_EQ, CMP_NE, CMP_GT, CMP_GE, CMP_LT, CMP_LE};
        D.cmp.sub = mirror[D.cmp.sub];
      }
    }
    FSpecDev* d = (FSpecDev*)sc.take(sizeof(FSpecDev));
    SM_HIP(hipMemcpyAsync(d, &h, sizeof(h), hipMemcpyHostToDevice, s));
    switch (fl.n) {
      case 1: hipLaunchKernelGGL(filter_count_leaves_kernel<1>, dim3((unsigned)nblocks), dim3(kFBlock), 0, s, d, n, masks, counts); break;
      case 2: hipLaunchKernelGGL(filter_count_leaves_kernel<2>, dim3((unsigned)nblocks), dim3(kFBlock), 0, s, d, n, masks, counts); break;
      case 3: hipLaunchKernelGGL(filter_count_leaves_kernel<3>, dim3((unsigned)nblocks), dim3(kFBlock), 0, s, d, n, masks, counts); break;
      default: hipLaunchKernelGGL(filter_count_leaves_kernel<4>, dim3((unsigned)nblocks), dim3(kFBlock), 0, s, d, n, masks, counts); break;
    }
  } else {
    hipLaunchKernelGGL(filter_count_prog_kernel, dim3((unsigned)nblocks), dim3(kFBlock), 0, s, st_dev, n, code_dev, len,
                       consts_dev, masks, counts);
  }
  if (tm) tm->mark("filter_count", s);
  exclusive_scan_u32(counts, nblocks, sc, s, total);
  if (tm) tm->mark("filter_scan", s);
  hipLaunchKernelGGL(filter_write_u32_kernel, dim3((unsigned)((nblocks + kWTiles - 1) / kWTiles)), dim3(kFBlock), 0, s,
                     masks, n, counts, nblocks, ordinals, ordinal_base, out);
  if (tm) tm->mark("filter_write", s);
  uint32_t h = 0;
  SM_HIP(hipMemcpyAsync(&h, total, 4, hipMemcpyDeviceToHost, s));
  SM_HIP(hipStreamSynchronize(s));
  if (typed_out) *typed_out = typed && !nulls;
  sc.used = mark;
  return h;
}

}  // namespace sm
