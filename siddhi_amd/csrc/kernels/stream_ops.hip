// Column-scan kernels for gfx950:
//   * filter (FilterProcessor.process, core/query/processor/filter/FilterProcessor.java:50-62) as a two-pass
//     ordered stream compaction: pass 1 evaluates the predicate per row and keeps one wave64 ballot word per
//     64 rows plus a per-block count; an exclusive scan of the counts gives each block its output offset;
//     pass 2 expands the ballot words into row indices (popcount prefix within the word).
//   * projection of matched rows (QuerySelector.processNoGroupBy :124-167) into output records
//   * partition-key evaluation (ValuePartitionExecutor.execute :34-40) and the device key table
//     (PartitionRuntime.cloneIfNotExist :256 — key → per-key state slot)
#include "expr.h"
#include "nfa.h"
#include "stream_ops.h"

namespace sm {

namespace {

constexpr int kFThreads = 256;
constexpr int kFIters = 8;  // 64-row groups per wave → tile = 256 threads × 8 = 2048 rows per block

struct ColLoader {
  const NfaStream* st;
  int64_t row;
  __device__ StackVal var(const Instr& in) const {
    StackVal v;
    v.i = 0;
    v.d = 0;
    v.null = 0;
    int a = in.a;
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

__global__ __launch_bounds__(kFThreads) void filter_mask_kernel(const NfaStream* __restrict__ st, int64_t n,
                                                                const Instr* __restrict__ code, int len,
                                                                const DVal* __restrict__ consts,
                                                                uint64_t* __restrict__ masks,
                                                                uint32_t* __restrict__ block_counts) {
  __shared__ uint32_t wsum[kFThreads / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t tile = (int64_t)blockIdx.x * kFThreads * kFIters;
  uint32_t cnt = 0;
  for (int it = 0; it < kFIters; ++it) {
    int64_t group = (tile >> 6) + (int64_t)it * (kFThreads / 64) + w;  // 64-row group index
    int64_t row = group * 64 + lane;
    bool pass = false;
    if (row < n) {
      if (len == 0) pass = true;
      else {
        ColLoader ld{st, row};
        pass = truthy(eval_prog(code, len, consts, ld));
      }
    }
    uint64_t m = __ballot(pass);
    if (lane == 0 && group * 64 < n) masks[group] = m;
    cnt += (uint32_t)__popcll(m);
  }
  if (lane == 0) wsum[w] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t s = 0;
    for (int k = 0; k < kFThreads / 64; ++k) s += wsum[k];
    block_counts[blockIdx.x] = s;
  }
}

__global__ __launch_bounds__(kFThreads) void filter_write_kernel(const uint64_t* __restrict__ masks, int64_t n,
                                                                 const uint32_t* __restrict__ block_offsets,
                                                                 int64_t* __restrict__ out_rows) {
  __shared__ uint32_t wbase[kFThreads / 64][kFIters];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t tile = (int64_t)blockIdx.x * kFThreads * kFIters;
  // per-(iteration, wave) popcounts in group order: group = it * 4 + w
  for (int it = 0; it < kFIters; ++it) {
    int64_t group = (tile >> 6) + (int64_t)it * (kFThreads / 64) + w;
    uint64_t m = (group * 64 < n) ? masks[group] : 0ull;
    if (lane == 0) wbase[w][it] = (uint32_t)__popcll(m);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = block_offsets[blockIdx.x];
    for (int it = 0; it < kFIters; ++it)
      for (int k = 0; k < kFThreads / 64; ++k) {
        uint32_t c = wbase[k][it];
        wbase[k][it] = acc;
        acc += c;
      }
  }
  __syncthreads();
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int it = 0; it < kFIters; ++it) {
    int64_t group = (tile >> 6) + (int64_t)it * (kFThreads / 64) + w;
    if (group * 64 >= n) break;
    uint64_t m = masks[group];
    if ((m >> lane) & 1ull) out_rows[wbase[w][it] + __popcll(m & lt)] = group * 64 + lane;
  }
}

__global__ void project_kernel(const NfaStream* __restrict__ st, const int64_t* __restrict__ rows, int64_t nm,
                               const int64_t* __restrict__ row_pos, const int64_t* __restrict__ ev_ts,
                               const int64_t* __restrict__ ev_ord, const char* __restrict__ blob, int32_t query_order, char* out,
                               uint32_t stride) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nm) return;
  const DQuery* q = (const DQuery*)blob;
  const Instr* code = (const Instr*)(blob + q->off_code);
  const DVal* consts = (const DVal*)(blob + q->off_const);
  const int32_t* sel = (const int32_t*)(blob + q->off_sel);
  int64_t row = rows[i];
  int64_t p = row_pos[row];
  OutRec* o = (OutRec*)(out + (size_t)i * stride);
  o->pos = p;
  o->time = 0;
  o->create = -1;
  o->ts = ev_ts[p];
  o->phase = 1;
  o->query = query_order;
  o->sched = -1;
  o->seq = 0;
  o->key = 0;
  DVal* vals = (DVal*)((char*)o + sizeof(OutRec));
  ColLoader ld{st, row};
  for (int k = 0; k < q->nsel; ++k) {
    StackVal v = eval_prog(code + sel[3 * k], sel[3 * k + 1], consts, ld);
    if (sel[3 * k + 2] == T_FLOAT || sel[3 * k + 2] == T_DOUBLE) vals[k].d = v.d;
    else vals[k].i = v.i;
    vals[k].null = v.null;
    vals[k].pad = 0;
  }
  int64_t* rf = (int64_t*)(vals + q->nsel);
  for (int k = 0; k < q->nrefs; ++k) rf[k] = ev_ord[p];
}

// records of the query's streams (+ START markers when `with_start`), as positions
// The records a query reads, as 64-record ballot masks + per-block counts (the filter's two-pass compaction:
// one byte-free pass instead of flag bytes, a widening pass and a full-length scan)
__global__ __launch_bounds__(kFThreads) void select_mask_kernel(const int32_t* __restrict__ ev_stream, int64_t n,
                                                                uint32_t stream_mask_lo, uint32_t stream_mask_hi,
                                                                int with_start, uint64_t* __restrict__ masks,
                                                                uint32_t* __restrict__ block_counts) {
  __shared__ uint32_t wsum[kFThreads / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t tile = (int64_t)blockIdx.x * kFThreads * kFIters;
  uint32_t cnt = 0;
  for (int it = 0; it < kFIters; ++it) {
    const int64_t group = (tile >> 6) + (int64_t)it * (kFThreads / 64) + w;
    const int64_t i = group * 64 + lane;
    bool f = false;
    if (i < n) {
      const int sid = ev_stream[i];
      if (sid == NFA_START) f = with_start;
      else if (sid >= 0) f = (sid < 32) ? ((stream_mask_lo >> sid) & 1u) : ((stream_mask_hi >> (sid - 32)) & 1u);
    }
    const uint64_t m = __ballot(f);
    if (lane == 0 && group * 64 < n) masks[group] = m;
    cnt += (uint32_t)__popcll(m);
  }
  if (lane == 0) wsum[w] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int k = 0; k < kFThreads / 64; ++k) t += wsum[k];
    block_counts[blockIdx.x] = t;
  }
}

// Run starts of a sorted key array as ballot masks + per-block counts, and the exclusive rank of every element
// among them (= its run's index): two streaming passes instead of a flag array and a full-length scan
template <typename K>
__global__ __launch_bounds__(kFThreads) void run_mask_kernel(const K* __restrict__ sk, int64_t n,
                                                             uint64_t* __restrict__ masks,
                                                             uint32_t* __restrict__ block_counts) {
  __shared__ uint32_t wsum[kFThreads / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t tile = (int64_t)blockIdx.x * kFThreads * kFIters;
  uint32_t cnt = 0;
  for (int it = 0; it < kFIters; ++it) {
    const int64_t group = (tile >> 6) + (int64_t)it * (kFThreads / 64) + w;
    const int64_t i = group * 64 + lane;
    const bool f = i < n && (i == 0 || sk[i] != sk[i - 1]);
    const uint64_t m = __ballot(f);
    if (lane == 0 && group * 64 < n) masks[group] = m;
    cnt += (uint32_t)__popcll(m);
  }
  if (lane == 0) wsum[w] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int k = 0; k < kFThreads / 64; ++k) t += wsum[k];
    block_counts[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(kFThreads) void mask_rank_kernel(const uint64_t* __restrict__ masks, int64_t n,
                                                              const uint32_t* __restrict__ block_offsets,
                                                              uint32_t* __restrict__ excl) {
  __shared__ uint32_t wbase[kFThreads / 64][kFIters];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t tile = (int64_t)blockIdx.x * kFThreads * kFIters;
  for (int it = 0; it < kFIters; ++it) {
    const int64_t group = (tile >> 6) + (int64_t)it * (kFThreads / 64) + w;
    const uint64_t m = (group * 64 < n) ? masks[group] : 0ull;
    if (lane == 0) wbase[w][it] = (uint32_t)__popcll(m);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = block_offsets[blockIdx.x];
    for (int it = 0; it < kFIters; ++it)
      for (int k = 0; k < kFThreads / 64; ++k) {
        const uint32_t c = wbase[k][it];
        wbase[k][it] = acc;
        acc += c;
      }
  }
  __syncthreads();
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int it = 0; it < kFIters; ++it) {
    const int64_t group = (tile >> 6) + (int64_t)it * (kFThreads / 64) + w;
    if (group * 64 >= n) break;
    const int64_t i = group * 64 + lane;
    if (i < n) excl[i] = wbase[w][it] + (uint32_t)__popcll(masks[group] & lt);
  }
}

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

// Key evaluation and key-table lookup in one pass (group_by_key): each record's partition key, then its slot (-1: not in the
// table, -2: null key / other stream). A key that is one column (the common `partition with (symbol of S)`) is
// loaded directly instead of through the expression evaluator's operand stack. Misses are counted per workgroup.
__global__ __launch_bounds__(256) void key_lookup_kernel(const int64_t* __restrict__ pos, int64_t n,
                                                         const int32_t* __restrict__ ev_stream,
                                                         const int64_t* __restrict__ ev_row,
                                                         const NfaStream* __restrict__ streams, int nstreams,
                                                         const KeyProg* __restrict__ progs, int nprogs,
                                                         const int64_t* __restrict__ tkeys,
                                                         const int32_t* __restrict__ tslots, uint64_t mask, bool empty,
                                                         int64_t* __restrict__ keys, int32_t* __restrict__ slot_out,
                                                         uint32_t* __restrict__ nmissing) {
  __shared__ uint32_t wmiss[4];
  __shared__ NfaStream lst[kLdsStreams];  // the stream descriptors, read by every record's key load
  if (nstreams <= kLdsStreams) {
    const int words = nstreams * (int)(sizeof(NfaStream) / 8);
    for (int q = threadIdx.x; q < words; q += blockDim.x) ((uint64_t*)lst)[q] = ((const uint64_t*)streams)[q];
    __syncthreads();
    streams = lst;
  }
  uint32_t miss = 0;
  // grid-stride over a bounded grid: one miss-count atomic per workgroup (all on one address, they serialise in
  // the L2: a workgroup per 256 records made them 3x the kernel's own time on a batch of new keys)
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = pos ? pos[i] : i;  // no pos: the query keeps every batch record
    const int s = ev_stream[p];
    int32_t slot = -2;
    int64_t key = 0;
    for (int k = 0; k < nprogs; ++k) {
      if (progs[k].stream != s) continue;
      ColLoader ld{&streams[s], ev_row ? ev_row[p] : p};
      StackVal v;
      if (progs[k].len == 1 && (progs[k].code[0].op == OP_VAR || progs[k].code[0].op == OP_COL))
        v = ld.var(progs[k].code[0]);
      else
        v = eval_prog(progs[k].code, progs[k].len, progs[k].consts, ld);
      if (v.null) break;
      if (progs[k].type == T_FLOAT || progs[k].type == T_DOUBLE) {
        double d = v.d;
        if (d != d) d = __longlong_as_double(0x7ff8000000000000ll);  // String.valueOf(NaN) == "NaN" for every NaN
        key = __double_as_longlong(d);
      } else {
        key = v.i;
      }
      slot = -1;
      if (!empty) {
        uint64_t h = mix64((uint64_t)key) & mask;
        for (;;) {
          const int32_t t = tslots[h];
          if (t == 0) break;
          if (tkeys[h] == key) {
            slot = t - 1;
            break;
          }
          h = (h + 1) & mask;
        }
      }
      break;
    }
    keys[i] = key;
    slot_out[i] = slot;
    miss += slot == -1;
  }
  for (int o = 32; o > 0; o >>= 1) miss += __shfl_xor(miss, o, 64);
  if ((threadIdx.x & 63) == 0) wmiss[threadIdx.x >> 6] = miss;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t t = wmiss[0] + wmiss[1] + wmiss[2] + wmiss[3];
    if (t) atomicAdd(nmissing, t);
  }
}

__global__ void table_insert_kernel(const int64_t* __restrict__ keys, const int32_t* __restrict__ slots, int64_t n,
                                    int64_t* __restrict__ tkeys, int32_t* __restrict__ tslots, uint64_t mask) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int64_t k = keys[i];
  uint64_t h = mix64((uint64_t)k) & mask;
  for (;;) {
    if (atomicCAS(&tslots[h], 0, slots[i] + 1) == 0) {
      tkeys[h] = k;
      return;
    }
    h = (h + 1) & mask;
  }
}

__global__ void minmax_kernel(const int64_t* __restrict__ keys, int64_t n, unsigned long long* __restrict__ mm) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // order-preserving map int64 → uint64
  uint64_t lo = ~0ull, hi = 0;
  for (; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t u = (uint64_t)keys[i] ^ 0x8000000000000000ull;
    lo = u < lo ? u : lo;
    hi = u > hi ? u : hi;
  }
  atomicMin(&mm[0], (unsigned long long)lo);
  atomicMax(&mm[1], (unsigned long long)hi);
}

// K = uint32_t when the batch's key span fits 32 bits (the sort then moves 8 instead of 12 bytes per item and pass)
template <typename K>
__global__ void rebase_keys_kernel(const int64_t* __restrict__ keys, int64_t n, uint64_t lo, K* __restrict__ out,
                                   uint32_t* __restrict__ idx) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = (K)(((uint64_t)keys[i] ^ 0x8000000000000000ull) - lo);
  idx[i] = (uint32_t)i;
}

// after sorting (rebased key, idx): run starts get a new slot id; every entry learns its run's slot
template <typename K>
__global__ void assign_new_slots_kernel(const K* __restrict__ sk, const uint32_t* __restrict__ sidx,
                                        const uint32_t* __restrict__ run_excl, int64_t n, int32_t base,
                                        const int64_t* __restrict__ keys_of_missing,
                                        const uint32_t* __restrict__ missing_map, int32_t* __restrict__ slot_out,
                                        int64_t* __restrict__ new_keys, int32_t* __restrict__ new_slots,
                                        int64_t* __restrict__ slot_keys) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bool start = (i == 0 || sk[i] != sk[i - 1]);
  uint32_t run = run_excl[i] + (start ? 1u : 0u) - 1u;  // inclusive count - 1
  int32_t slot = base + (int32_t)run;
  uint32_t m = sidx[i];  // index into the missing list
  if (slot_out) slot_out[missing_map ? missing_map[m] : m] = slot;
  if (start) {
    new_keys[run] = keys_of_missing[m];
    new_slots[run] = slot;
    slot_keys[slot] = keys_of_missing[m];
  }
}

// every record of the batch carried a new key: the key-sorted missing list already is the per-slot grouping
// (slots were numbered in key order from `base`), so it becomes key_pos / key_off directly
template <typename K>
__global__ void all_new_csr_kernel(const K* __restrict__ sk, const uint32_t* __restrict__ sidx,
                                   const uint32_t* __restrict__ run_excl, const uint32_t* __restrict__ missing_map,
                                   const int64_t* __restrict__ pos, int64_t n, int32_t base,
                                   int64_t* __restrict__ key_pos, int64_t* __restrict__ key_off) {
  int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint32_t m = sidx[j];
  const uint32_t x = missing_map ? missing_map[m] : m;  // no map: the missing list is the whole batch
  key_pos[j] = pos ? pos[x] : x;                        // no pos: every batch record is the query's
  const bool start = (j == 0 || sk[j] != sk[j - 1]);
  if (start) key_off[base + run_excl[j]] = j;
  if (j == n - 1) key_off[base + run_excl[j] + (start ? 1 : 0)] = n;  // one past the last run
}

template <typename T>
__global__ void compact_flag_kernel(const uint8_t* __restrict__ flag, const uint32_t* __restrict__ excl, int64_t n,
                                    T* __restrict__ out_idx) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (flag[i]) out_idx[excl[i]] = (T)i;
}

__global__ void u8_to_u32_kernel(const uint8_t* __restrict__ f, int64_t n, uint32_t* __restrict__ o) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) o[i] = f[i];
}

__global__ void missing_flags_kernel(const int32_t* __restrict__ slot, int64_t n, uint8_t* __restrict__ f) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) f[i] = slot[i] == -1;
}

__global__ void gather_i64_kernel(const int64_t* __restrict__ src, const uint32_t* __restrict__ idx, int64_t n,
                                  int64_t* __restrict__ dst) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[idx[i]];
}

__global__ void slot_to_u32_kernel(const int32_t* __restrict__ slot, int64_t n, uint32_t nslots,
                                   uint32_t* __restrict__ key, uint32_t* __restrict__ idx) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    key[i] = slot[i] < 0 ? nslots : (uint32_t)slot[i];  // records without a key (null) sort last
    idx[i] = (uint32_t)i;
  }
}

__global__ void count_slots_kernel(const uint32_t* __restrict__ sorted_slot, int64_t n, uint32_t* __restrict__ counts) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) atomicAdd(&counts[sorted_slot[i]], 1u);
}

__global__ void u32_to_i64_kernel(const uint32_t* __restrict__ a, int64_t n, int64_t* __restrict__ o) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) o[i] = a[i];
}

// sk is sorted: equal slots are adjacent, so each run inside a wave adds its length with one atomic
__global__ void count_valid_slots_kernel(const uint32_t* __restrict__ sk, int64_t n, uint32_t nslots,
                                         uint32_t* __restrict__ counts) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const uint32_t key = i < n ? sk[i] : 0xffffffffu;
  const uint32_t prev = __shfl_up(key, 1, 64);
  const bool head = i < n && (lane == 0 || prev != key);
  const uint64_t heads = __ballot(head || i >= n);
  if (head && key < nslots) {
    const uint64_t after = lane == 63 ? 0ull : heads & (~0ull << (lane + 1));
    const int next = after ? __ffsll((unsigned long long)after) - 1 : 64;
    atomicAdd(&counts[key], (uint32_t)(next - lane));
  }
}

__global__ void gather_pos_kernel(const int64_t* __restrict__ pos, const uint32_t* __restrict__ si, int64_t n,
                                  int64_t* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = pos[si[i]];
}

__global__ void rehash_kernel(const int64_t* __restrict__ slot_keys, int64_t nslots, int64_t* __restrict__ tkeys,
                              int32_t* __restrict__ tslots, uint64_t mask) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nslots) return;
  int64_t k = slot_keys[i];
  uint64_t h = mix64((uint64_t)k) & mask;
  for (;;) {
    if (atomicCAS(&tslots[h], 0, (int32_t)i + 1) == 0) {
      tkeys[h] = k;
      return;
    }
    h = (h + 1) & mask;
  }
}

inline dim3 grid_for(int64_t n, int t = 256) { return dim3((unsigned)((n + t - 1) / t)); }

// ---- dense key ids (remap_keys)
constexpr int64_t kDkBusy = -1;
#ifndef SM_DK_LOAD_SHIFT
#define SM_DK_LOAD_SHIFT 1  // A/B build flag: table entries = id capacity << shift
#endif

// Lookup-or-insert of each event's key. An entry is claimed with a CAS from empty to busy, filled, then published
// with its id; a reader meeting a busy entry reads it again (the claiming lane fills it in the same loop iteration,
// so no lane waits on work another lane of its wave has not done yet). An id beyond the id capacity releases the
// entry and flags an overflow: the host grows the table and runs the batch again (found keys are found again).
// One key from entry h on: plain reads while they decide, then the atomic protocol.
__device__ __forceinline__ int32_t dk_lookup(int64_t k, uint64_t h, int64_t* __restrict__ table, uint64_t mask,
                                          int64_t* __restrict__ slot_keys, int64_t limit, uint32_t* __restrict__ counter,
                                          uint32_t* __restrict__ overflow) {
  int32_t res = -1;
  uint64_t probes = 0;
  // found keys (all but the first sighting of each) with plain 16-byte reads: a non-zero key word is final (written
  // once, before its entry is published), so an entry holding another key is passed over and one holding this key
  // with a published id is a hit; an empty or busy entry, an entry whose key word is not visible yet, or the key 0
  // go on at that entry with the atomic protocol
  if (k != 0) {
    while (probes <= mask) {
      const longlong2 e = *(const longlong2*)&table[2 * h];
      if (e.x == k && e.y > 0) return (int32_t)(e.y - 1);
      if (e.x == 0 || e.x == k) break;
      h = (h + 1) & mask;
      ++probes;
    }
  }
  while (probes <= mask) {
    unsigned long long* st = (unsigned long long*)&table[2 * h + 1];
    const int64_t sv = (int64_t)__hip_atomic_load(st, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    if (sv == kDkBusy) continue;
    if (sv == 0) {
      if (atomicCAS(st, 0ull, (unsigned long long)kDkBusy) != 0ull) continue;
      const uint32_t id = atomicAdd(counter, 1u);
      if ((int64_t)id >= limit) {
        __hip_atomic_store(st, 0ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        atomicOr(overflow, 1u);
        break;
      }
      table[2 * h] = k;
      slot_keys[id] = k;
      __hip_atomic_store(st, (unsigned long long)id + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      res = (int32_t)id;
      break;
    }
    if (table[2 * h] == k) {
      res = (int32_t)(sv - 1);
      break;
    }
    h = (h + 1) & mask;
    ++probes;
  }
  return res;
}

template <typename KT>
__global__ void __launch_bounds__(256) remap_kernel(const KT* __restrict__ col, int64_t n, int64_t* __restrict__ table,
                                                    uint64_t mask, int64_t* __restrict__ slot_keys, int64_t limit,
                                                    uint32_t* __restrict__ counter, int32_t* __restrict__ out,
                                                    uint32_t* __restrict__ overflow) {
  // (four lookups in flight per lane, each key's first entry read together, measured slower: 76 against 66 ms per
  // config-4 step of 1e9 events; the kernel is bound by the random line fills of the table, not by latency)
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = dk_lookup((int64_t)col[i], mix64((uint64_t)(int64_t)col[i]) & mask, table, mask, slot_keys, limit,
                       counter, overflow);
}

template <typename KT>
__global__ void __launch_bounds__(256) key_minmax_kernel(const KT* __restrict__ col, int64_t n,
                                                         unsigned long long* __restrict__ mm) {
  uint64_t lo = ~0ull, hi = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t u = (uint64_t)(int64_t)col[i] ^ 0x8000000000000000ull;
    lo = u < lo ? u : lo;
    hi = u > hi ? u : hi;
  }
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t l2 = __shfl_xor(lo, off, 64), h2 = __shfl_xor(hi, off, 64);
    lo = l2 < lo ? l2 : lo;
    hi = h2 > hi ? h2 : hi;
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMin(&mm[0], (unsigned long long)lo);
    atomicMax(&mm[1], (unsigned long long)hi);
  }
}

__global__ void dk_rehash_kernel(const int64_t* __restrict__ slot_keys, int64_t n, int64_t* __restrict__ table,
                                 uint64_t mask) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t k = slot_keys[i];
  uint64_t h = mix64((uint64_t)k) & mask;
  for (;;) {
    unsigned long long* st = (unsigned long long*)&table[2 * h + 1];
    if (atomicCAS(st, 0ull, (unsigned long long)i + 1) == 0ull) {
      table[2 * h] = k;
      return;
    }
    h = (h + 1) & mask;
  }
}



// ---- device-resident interleaved batch (sm_app_process_device_events): the per-event arrays the host path
// builds record by record in stage_record (runtime.cpp) — row, ordinal, playback clock after sendData and the
// clock-advance points (StreamJunction.sendData :232-237: the clock moves, and listeners fire, only if ts >= clock).
constexpr int kIxThreads = 256, kIxItems = 16, kIxTile = kIxThreads * kIxItems;

__device__ __forceinline__ int64_t block_max_i64(int64_t v, int64_t* red) {
  for (int o = 32; o > 0; o >>= 1) {
    int64_t u = __shfl_xor(v, o, 64);
    v = u > v ? u : v;
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  v = red[0];
  for (int k = 1; k < kIxThreads / 64; ++k) v = red[k] > v ? red[k] : v;
  __syncthreads();
  return v;
}

__global__ __launch_bounds__(kIxThreads) void ts_tile_max_kernel(const int64_t* __restrict__ ts, int64_t n,
                                                                 int64_t* __restrict__ tile_max) {
  __shared__ int64_t red[kIxThreads / 64];
  const int64_t base = (int64_t)blockIdx.x * kIxTile;
  int64_t m = INT64_MIN;
  for (int k = 0; k < kIxItems; ++k) {
    int64_t i = base + (int64_t)k * kIxThreads + threadIdx.x;
    if (i < n) m = ts[i] > m ? ts[i] : m;
  }
  m = block_max_i64(m, red);
  if (threadIdx.x == 0) tile_max[blockIdx.x] = m;
}

// exclusive running max over the tiles, seeded with the clock before the batch (one workgroup, sequential chunks)
__global__ __launch_bounds__(kIxThreads) void tile_prefix_max_kernel(int64_t* __restrict__ tile_max, int64_t ntiles,
                                                                     int64_t clock_in, int64_t* __restrict__ clock_out) {
  __shared__ int64_t buf[kIxThreads];
  int64_t carry = clock_in;
  for (int64_t c = 0; c < ntiles; c += kIxThreads) {
    int64_t i = c + threadIdx.x;
    int64_t v = i < ntiles ? tile_max[i] : INT64_MIN;
    buf[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < kIxThreads; o <<= 1) {  // Hillis-Steele inclusive max
      int64_t u = threadIdx.x >= o ? buf[threadIdx.x - o] : INT64_MIN;
      __syncthreads();
      if (u > buf[threadIdx.x]) buf[threadIdx.x] = u;
      __syncthreads();
    }
    int64_t excl = threadIdx.x ? buf[threadIdx.x - 1] : INT64_MIN;
    excl = excl > carry ? excl : carry;
    if (i < ntiles) tile_max[i] = excl;
    int64_t last = buf[kIxThreads - 1];
    __syncthreads();
    carry = last > carry ? last : carry;
  }
  if (threadIdx.x == 0) *clock_out = carry;
}

// per event: row = i, ordinal, clock after sendData, advance flag (playback only)
__global__ __launch_bounds__(kIxThreads) void event_index_kernel(
    const int32_t* __restrict__ sid, int32_t nstreams, const int64_t* __restrict__ ts, int64_t n,
    const int64_t* __restrict__ ord_in, int64_t ord_base, int playback, int64_t clock_in,
    const int64_t* __restrict__ tile_prefix, int64_t* __restrict__ ev_row, int64_t* __restrict__ ev_ord,
    int64_t* __restrict__ ev_clock, uint64_t* __restrict__ adv_mask, uint32_t* __restrict__ adv_cnt,
    int32_t* __restrict__ bad) {
  __shared__ int64_t wmax[kIxThreads / 64];
  __shared__ uint32_t wadv[kIxThreads / 64];
  uint32_t nadv = 0;  // advance points of this wave (lane 0)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t base = (int64_t)blockIdx.x * kIxTile;
  int64_t carry = tile_prefix[blockIdx.x];  // clock before this tile (clock_in folded in)
  // kIxItems rounds of 256 consecutive events (coalesced): block inclusive max-scan per round, carried over
  for (int k = 0; k < kIxItems; ++k) {
    const int64_t i = base + (int64_t)k * kIxThreads + threadIdx.x;
    const bool in = i < n;
    const int64_t t = in ? ts[i] : INT64_MIN;
    int64_t v = t;
    for (int o = 1; o < 64; o <<= 1) {
      int64_t u = __shfl_up(v, o, 64);
      if (lane >= o && u > v) v = u;
    }
    if (lane == 63) wmax[w] = v;
    __syncthreads();
    int64_t before = carry;  // max of everything before this event (exclusive)
    for (int q = 0; q < w; ++q) before = wmax[q] > before ? wmax[q] : before;
    int64_t up = __shfl_up(v, 1, 64);
    if (lane > 0 && up > before) before = up;
    int64_t round_max = carry;
    for (int q = 0; q < kIxThreads / 64; ++q) round_max = wmax[q] > round_max ? wmax[q] : round_max;
    __syncthreads();
    carry = round_max;
    // advance points as one ballot mask per 64 consecutive events (rounds are 64-aligned)
    const bool adv = in && playback && t >= before;
    const uint64_t am = __ballot(adv);
    if (lane == 0 && i < n) adv_mask[i >> 6] = am;
    nadv += (uint32_t)__popcll(am);
    if (!in) continue;
    const int32_t st = sid[i];
    if (st < NFA_TICK || st >= nstreams) *bad = 1;  // plain vector store: any offender sets the flag
    if (ev_row) ev_row[i] = i;  // nullptr: the caller reads rows as positions (ev_row = identity)
    // heartbeats carry no event ordinal; nullptr: the caller reads ord_in itself (its data events' ordinals)
    if (ev_ord) ev_ord[i] = st < 0 ? -1 : ord_in ? ord_in[i] : ord_base + i;
    ev_clock[i] = playback ? (t > before ? t : before) : clock_in;
  }
  if (lane == 0) wadv[w] = nadv;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t c = 0;
    for (int q = 0; q < kIxThreads / 64; ++q) c += wadv[q];
    adv_cnt[blockIdx.x] = c;
  }
}

// Advance-point list and per-position counts from the masks: block offsets (exclusive scan of adv_cnt), then per
// 64-event group its offset within the tile (round-major, wave-minor, as event_index_kernel visits them)
__global__ __launch_bounds__(kIxThreads) void advance_rank_kernel(const uint64_t* __restrict__ adv_mask, int64_t n,
                                                                  const uint32_t* __restrict__ tile_off,
                                                                  const int64_t* __restrict__ ts,
                                                                  int64_t* __restrict__ adv_pos,
                                                                  int64_t* __restrict__ adv_clock,
                                                                  int64_t* __restrict__ adv_wall,
                                                                  int64_t* __restrict__ adv_upto) {
  __shared__ uint32_t gbase[kIxItems][kIxThreads / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t base = (int64_t)blockIdx.x * kIxTile;
  for (int k = 0; k < kIxItems; ++k) {
    const int64_t g0 = base + (int64_t)k * kIxThreads + w * 64;
    if (lane == 0) gbase[k][w] = g0 < n ? (uint32_t)__popcll(adv_mask[g0 >> 6]) : 0u;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = tile_off[blockIdx.x];
    for (int k = 0; k < kIxItems; ++k)
      for (int q = 0; q < kIxThreads / 64; ++q) {
        const uint32_t c = gbase[k][q];
        gbase[k][q] = acc;
        acc += c;
      }
  }
  __syncthreads();
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int k = 0; k < kIxItems; ++k) {
    const int64_t i = base + (int64_t)k * kIxThreads + threadIdx.x;
    if (i >= n) break;
    const uint64_t m = adv_mask[i >> 6];
    const uint32_t o = gbase[k][w] + (uint32_t)__popcll(m & lt);
    const bool f = (m >> lane) & 1ull;
    adv_upto[i] = (int64_t)o + f;
    if (f) {
      adv_pos[o] = i;
      adv_clock[o] = ts[i];
      adv_wall[o] = -1;
    }
  }
}
}  // namespace

void KeyTable::release() {
  if (tkeys) (void)hipFree(tkeys);
  if (tslots) (void)hipFree(tslots);
  if (slot_keys) (void)hipFree(slot_keys);
  tkeys = nullptr;
  tslots = nullptr;
  slot_keys = nullptr;
  cap = 0;
  slot_cap = 0;
  nslots = 0;
}

// Restore: take nslots keys (host array, slot order) and rebuild the hash table from them.
void KeyTable::load(const int64_t* keys_host, int32_t n, hipStream_t s) {
  nslots = 0;
  reserve(n, s);
  if (tslots) SM_HIP(hipMemsetAsync(tslots, 0, (size_t)cap * 4, s));
  if (n > 0) {
    SM_HIP(hipMemcpyAsync(slot_keys, keys_host, (size_t)n * 8, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(rehash_kernel, grid_for(n), dim3(256), 0, s, slot_keys, (int64_t)n, tkeys, tslots, mask);
  }
  nslots = n;
  SM_HIP(hipStreamSynchronize(s));
}

void DenseKeys::reserve(int64_t slots, hipStream_t s) {
  if (slots > INT32_MAX - 1) throw std::runtime_error("too many partition keys");
  if (slots > slot_cap) {
    int64_t nc = std::max<int64_t>(1 << 16, slot_cap);
    while (nc < slots) nc *= 2;
    int64_t* nk = nullptr;
    SM_HIP(hipMalloc(&nk, nc * 8));
    if (slot_keys && nslots) SM_HIP(hipMemcpyAsync(nk, slot_keys, (size_t)nslots * 8, hipMemcpyDeviceToDevice, s));
    SM_HIP(hipStreamSynchronize(s));
    if (slot_keys) SM_HIP(hipFree(slot_keys));
    slot_keys = nk;
    slot_cap = nc;
  }
  if (!counter) {
    SM_HIP(hipMalloc(&counter, 8));
    SM_HIP(hipMemsetAsync(counter, 0, 8, s));
  }
  // load factor at most 2^-SM_DK_LOAD_SHIFT when every id is handed out: a wave's lookup takes as many dependent
  // rounds as its longest probe chain among 64 lanes
  if ((slot_cap << SM_DK_LOAD_SHIFT) > cap) {
    int64_t nc = std::max<int64_t>(1 << 17, cap);
    while (nc < (slot_cap << SM_DK_LOAD_SHIFT)) nc *= 2;
    if (table) SM_HIP(hipFree(table));
    SM_HIP(hipMalloc(&table, (size_t)nc * 16));
    SM_HIP(hipMemsetAsync(table, 0, (size_t)nc * 16, s));
    cap = nc;
    if (nslots > 0)
      hipLaunchKernelGGL(dk_rehash_kernel, grid_for(nslots), dim3(256), 0, s, slot_keys, nslots, table,
                         (uint64_t)cap - 1);
  }
}

void DenseKeys::load(const int64_t* keys_host, int64_t n, hipStream_t s) {
  clear(s);
  reserve(std::max<int64_t>(n, 1), s);
  if (n) SM_HIP(hipMemcpyAsync(slot_keys, keys_host, (size_t)n * 8, hipMemcpyHostToDevice, s));
  nslots = n;
  const uint32_t c = (uint32_t)n;
  SM_HIP(hipMemcpyAsync(counter, &c, 4, hipMemcpyHostToDevice, s));
  if (n) hipLaunchKernelGGL(dk_rehash_kernel, grid_for(n), dim3(256), 0, s, slot_keys, n, table, (uint64_t)cap - 1);
  SM_HIP(hipStreamSynchronize(s));
}

void DenseKeys::clear(hipStream_t s) {
  if (table) SM_HIP(hipMemsetAsync(table, 0, (size_t)cap * 16, s));
  if (counter) SM_HIP(hipMemsetAsync(counter, 0, 8, s));
  nslots = 0;
}

void DenseKeys::release() {
  if (table) (void)hipFree(table);
  if (slot_keys) (void)hipFree(slot_keys);
  if (counter) (void)hipFree(counter);
  table = slot_keys = nullptr;
  counter = nullptr;
  cap = slot_cap = nslots = 0;
}

void key_range(const void* col, int key_type, int64_t n, int64_t* lo, int64_t* hi, Scratch& sc, hipStream_t s) {
  const size_t mark = sc.used;
  unsigned long long* mm = (unsigned long long*)sc.take(16);
  const unsigned long long init[2] = {~0ull, 0ull};
  SM_HIP(hipMemcpyAsync(mm, init, 16, hipMemcpyHostToDevice, s));
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 2048));
  if (key_type == T_LONG)
    hipLaunchKernelGGL(key_minmax_kernel<int64_t>, dim3(g), dim3(256), 0, s, (const int64_t*)col, n, mm);
  else
    hipLaunchKernelGGL(key_minmax_kernel<int32_t>, dim3(g), dim3(256), 0, s, (const int32_t*)col, n, mm);
  unsigned long long h[2];
  SM_HIP(hipMemcpyAsync(h, mm, 16, hipMemcpyDeviceToHost, s));
  SM_HIP(hipStreamSynchronize(s));
  sc.used = mark;
  *lo = (int64_t)(h[0] ^ 0x8000000000000000ull);
  *hi = (int64_t)(h[1] ^ 0x8000000000000000ull);
}

void remap_keys(DenseKeys& D, const void* col, int key_type, int64_t n, int32_t* out, hipStream_t s) {
  if (n <= 0) return;
  // room for the ids seen so far plus up to 2^20 new ones; more new keys overflow and grow the table
  D.reserve(D.nslots + std::min<int64_t>(n, (int64_t)1 << 20), s);
  uint32_t* ovf = nullptr;
  SM_HIP(hipMalloc(&ovf, 4));
  struct Free {
    uint32_t* p;
    ~Free() { (void)hipFree(p); }
  } fr{ovf};
  for (;;) {
    SM_HIP(hipMemsetAsync(ovf, 0, 4, s));
    const unsigned g = (unsigned)std::min<int64_t>((n + 255) / 256, 16384);
    if (key_type == T_LONG)
      hipLaunchKernelGGL(remap_kernel<int64_t>, dim3(g), dim3(256), 0, s, (const int64_t*)col, n, D.table,
                         (uint64_t)D.cap - 1, D.slot_keys, D.slot_cap, D.counter, out, ovf);
    else
      hipLaunchKernelGGL(remap_kernel<int32_t>, dim3(g), dim3(256), 0, s, (const int32_t*)col, n, D.table,
                         (uint64_t)D.cap - 1, D.slot_keys, D.slot_cap, D.counter, out, ovf);
    uint32_t h[2] = {0, 0};
    SM_HIP(hipMemcpyAsync(&h[0], ovf, 4, hipMemcpyDeviceToHost, s));
    SM_HIP(hipMemcpyAsync(&h[1], D.counter, 4, hipMemcpyDeviceToHost, s));
    SM_HIP(hipStreamSynchronize(s));
    D.nslots = std::min<int64_t>(h[1], D.slot_cap);
    if (!h[0]) return;
    // ids ran out: the counter went past the capacity; keep the ids handed out, grow, and run the batch again
    const uint32_t c = (uint32_t)D.nslots;
    SM_HIP(hipMemcpyAsync(D.counter, &c, 4, hipMemcpyHostToDevice, s));
    D.reserve(D.slot_cap * 4, s);
  }
}

void KeyTable::reserve(int64_t total, hipStream_t s) {
  if (total > INT32_MAX - 1) throw std::runtime_error("too many partition keys");
  if (total > slot_cap) {
    int64_t nc = std::max<int64_t>(1024, slot_cap);
    while (nc < total) nc *= 2;
    int64_t* nk = nullptr;
    SM_HIP(hipMalloc(&nk, nc * 8));
    if (slot_keys && nslots) SM_HIP(hipMemcpyAsync(nk, slot_keys, (size_t)nslots * 8, hipMemcpyDeviceToDevice, s));
    SM_HIP(hipStreamSynchronize(s));
    if (slot_keys) SM_HIP(hipFree(slot_keys));
    slot_keys = nk;
    slot_cap = nc;
  }
  if (total * 2 > cap) {
    int64_t nc = std::max<int64_t>(2048, cap);
    while (nc < total * 2) nc *= 2;
    if (tkeys) SM_HIP(hipFree(tkeys));
    if (tslots) SM_HIP(hipFree(tslots));
    SM_HIP(hipMalloc(&tkeys, nc * 8));
    SM_HIP(hipMalloc(&tslots, nc * 4));
    SM_HIP(hipMemsetAsync(tslots, 0, nc * 4, s));
    cap = nc;
    mask = (uint64_t)nc - 1;
    if (nslots > 0)
      hipLaunchKernelGGL(rehash_kernel, grid_for(nslots), dim3(256), 0, s, slot_keys, (int64_t)nslots, tkeys, tslots,
                         mask);
  }
}

int64_t filter_rows(const NfaStream* st_dev, int64_t n, const Instr* code, int len, const DVal* consts,
                    int64_t* out_rows, Scratch& sc, hipStream_t s) {
  if (n == 0) return 0;
  size_t mark = sc.used;
  int64_t ngroups = (n + 63) / 64;
  int64_t tile = (int64_t)kFThreads * kFIters;
  int64_t nblocks = (n + tile - 1) / tile;
  uint64_t* masks = (uint64_t*)sc.take(ngroups * 8);
  uint32_t* counts = (uint32_t*)sc.take((nblocks + 1) * 4);
  uint32_t* total = (uint32_t*)sc.take(4);
  hipLaunchKernelGGL(filter_mask_kernel, dim3((unsigned)nblocks), dim3(kFThreads), 0, s, st_dev, n, code, len, consts,
                     masks, counts);
  exclusive_scan_u32(counts, nblocks, sc, s, total);
  hipLaunchKernelGGL(filter_write_kernel, dim3((unsigned)nblocks), dim3(kFThreads), 0, s, masks, n, counts, out_rows);
  uint32_t h = 0;
  SM_HIP(hipMemcpyAsync(&h, total, 4, hipMemcpyDeviceToHost, s));
  SM_HIP(hipStreamSynchronize(s));
  sc.used = mark;
  return h;
}

void project_rows(const NfaStream* st_dev, const int64_t* rows, int64_t nm, const int64_t* row_pos,
                  const int64_t* ev_ts, const int64_t* ev_ord, const char* blob_dev, int32_t query_order, char* out,
                  uint32_t stride, hipStream_t s) {
  if (nm == 0) return;
  hipLaunchKernelGGL(project_kernel, grid_for(nm), dim3(256), 0, s, st_dev, rows, nm, row_pos, ev_ts, ev_ord,
                     blob_dev, query_order, out, stride);
}

int64_t select_records(const int32_t* ev_stream, int64_t n, uint64_t stream_mask, bool with_start, int64_t* out_pos,
                       Scratch& sc, hipStream_t s) {
  if (n == 0) return 0;
  size_t mark = sc.used;
  const int64_t tile = (int64_t)kFThreads * kFIters;
  const int64_t nblocks = (n + tile - 1) / tile;
  uint64_t* masks = (uint64_t*)sc.take(((n + 63) / 64) * 8);
  uint32_t* counts = (uint32_t*)sc.take((nblocks + 1) * 4);
  uint32_t* total = (uint32_t*)sc.take(4);
  hipLaunchKernelGGL(select_mask_kernel, dim3((unsigned)nblocks), dim3(kFThreads), 0, s, ev_stream, n,
                     (uint32_t)stream_mask, (uint32_t)(stream_mask >> 32), (int)with_start, masks, counts);
  exclusive_scan_u32(counts, nblocks, sc, s, total);
  hipLaunchKernelGGL(filter_write_kernel, dim3((unsigned)nblocks), dim3(kFThreads), 0, s, masks, n, counts, out_pos);
  uint32_t h = 0;
  SM_HIP(hipMemcpyAsync(&h, total, 4, hipMemcpyDeviceToHost, s));
  SM_HIP(hipStreamSynchronize(s));
  sc.used = mark;
  return h;
}

// Group a query's records by partition key. Returns the number of valid records; key_pos / key_off (CSR over
// all `*nslots` slots) are written into buffers from `sc` (valid until the caller releases the scratch).
int64_t group_by_key(KeyTable& T, const int64_t* pos, int64_t n, const int32_t* ev_stream, const int64_t* ev_row, int nstreams,
                     const NfaStream* streams_dev, const KeyProg* progs_dev, int nprogs, int64_t** key_pos_out,
                     int64_t** key_off_out, Scratch& sc, hipStream_t s, bool pos_identity) {
  int64_t* keys = (int64_t*)sc.take(std::max<int64_t>(n, 1) * 8);
  int32_t* slot = (int32_t*)sc.take(std::max<int64_t>(n, 1) * 4);
  uint32_t* nmiss = (uint32_t*)sc.take(4);
  SM_HIP(hipMemsetAsync(nmiss, 0, 4, s));
  if (n > 0)
    hipLaunchKernelGGL(key_lookup_kernel, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 8192)), dim3(256), 0, s,
                       pos_identity ? nullptr : pos, n, ev_stream,
                       ev_row, streams_dev, nstreams, progs_dev, nprogs, T.tkeys, T.tslots, T.mask, T.nslots == 0, keys, slot,
                       nmiss);
  uint32_t hm = 0;
  SM_HIP(hipMemcpyAsync(&hm, nmiss, 4, hipMemcpyDeviceToHost, s));
  SM_HIP(hipStreamSynchronize(s));
  if (hm > 0) {
    // new keys: compact, sort by key (stable → first occurrence first), one new slot per distinct key
    const bool all_new = (int64_t)hm == n;
    const int32_t base = T.nslots;
    int64_t* fast_pos = all_new ? (int64_t*)sc.take((size_t)n * 8) : nullptr;
    int64_t* fast_off = all_new ? (int64_t*)sc.take(((size_t)base + hm + 2) * 8) : nullptr;
    size_t mark = sc.used;
    // the missing list (records whose key is not in the table) and its keys; when every record misses, it is
    // the whole batch in order (miss = identity: no compaction, no gathers)
    uint32_t* miss = nullptr;
    int64_t* mkeys = keys;
    if (!all_new) {
      uint8_t* f = (uint8_t*)sc.take(n);
      uint32_t* ex = (uint32_t*)sc.take(n * 4);
      hipLaunchKernelGGL(missing_flags_kernel, grid_for(n), dim3(256), 0, s, slot, n, f);
      hipLaunchKernelGGL(u8_to_u32_kernel, grid_for(n), dim3(256), 0, s, f, n, ex);
      exclusive_scan_u32(ex, n, sc, s);
      miss = (uint32_t*)sc.take(hm * 4);
      hipLaunchKernelGGL(compact_flag_kernel<uint32_t>, grid_for(n), dim3(256), 0, s, f, ex, n, miss);
      mkeys = (int64_t*)sc.take(hm * 8);
      hipLaunchKernelGGL(gather_i64_kernel, grid_for(hm), dim3(256), 0, s, keys, miss, (int64_t)hm, mkeys);
    }
    unsigned long long* mm = (unsigned long long*)sc.take(16);
    unsigned long long init[2] = {~0ull, 0ull};
    SM_HIP(hipMemcpyAsync(mm, init, 16, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(minmax_kernel, dim3(std::min<int64_t>(1024, (hm + 255) / 256)), dim3(256), 0, s, mkeys,
                       (int64_t)hm, mm);
    unsigned long long hmm[2];
    SM_HIP(hipMemcpyAsync(hmm, mm, 16, hipMemcpyDeviceToHost, s));
    SM_HIP(hipStreamSynchronize(s));
    uint64_t span = hmm[1] - hmm[0];
    int bits = 0;
    while (bits < 64 && (span >> bits) != 0) ++bits;
    auto new_slots = [&](auto key_type) -> bool {
      using K = decltype(key_type);
      K* sk = (K*)sc.take(hm * sizeof(K));
      K* sk2 = (K*)sc.take(hm * sizeof(K));
      uint32_t* si = (uint32_t*)sc.take(hm * 4);
      uint32_t* si2 = (uint32_t*)sc.take(hm * 4);
      hipLaunchKernelGGL(rebase_keys_kernel<K>, grid_for(hm), dim3(256), 0, s, mkeys, (int64_t)hm, (uint64_t)hmm[0], sk, si);
      bool alt = radix_sort_pairs<K>(sk, sk2, si, si2, hm, 0, bits, sc, s);
      if (alt) {
        std::swap(sk, sk2);
        std::swap(si, si2);
      }
      uint32_t* runs = (uint32_t*)sc.take(hm * 4);
      uint32_t* nruns = (uint32_t*)sc.take(4);
      {
        const int64_t tile = (int64_t)kFThreads * kFIters;
        const int64_t nb = ((int64_t)hm + tile - 1) / tile;
        uint64_t* rmask = (uint64_t*)sc.take((((size_t)hm + 63) / 64) * 8);
        uint32_t* rcnt = (uint32_t*)sc.take(((size_t)nb + 1) * 4);
        hipLaunchKernelGGL(run_mask_kernel<K>, dim3((unsigned)nb), dim3(kFThreads), 0, s, sk, (int64_t)hm, rmask, rcnt);
        exclusive_scan_u32(rcnt, nb, sc, s, nruns);
        hipLaunchKernelGGL(mask_rank_kernel, dim3((unsigned)nb), dim3(kFThreads), 0, s, rmask, (int64_t)hm, rcnt, runs);
      }
      uint32_t hr = 0;
      SM_HIP(hipMemcpyAsync(&hr, nruns, 4, hipMemcpyDeviceToHost, s));
      SM_HIP(hipStreamSynchronize(s));
      T.reserve((int64_t)T.nslots + hr, s);
      int64_t* nk = (int64_t*)sc.take(hr * 8);
      int32_t* ns = (int32_t*)sc.take(hr * 4);
      hipLaunchKernelGGL(assign_new_slots_kernel<K>, grid_for(hm), dim3(256), 0, s, sk, si, runs, (int64_t)hm, T.nslots,
                         mkeys, miss, all_new ? nullptr : slot, nk, ns, T.slot_keys);
      hipLaunchKernelGGL(table_insert_kernel, grid_for(hr), dim3(256), 0, s, nk, ns, (int64_t)hr, T.tkeys, T.tslots,
                         T.mask);
      T.nslots += hr;
      if (all_new) {
        SM_HIP(hipMemsetAsync(fast_off, 0, ((size_t)base + 1) * 8, s));
        hipLaunchKernelGGL(all_new_csr_kernel<K>, grid_for(hm), dim3(256), 0, s, sk, si, runs, miss,
                           pos_identity ? nullptr : pos, (int64_t)hm, base,
                           fast_pos, fast_off);
        *key_pos_out = fast_pos;
        *key_off_out = fast_off;
        return true;
      }
      return false;
    };
    const bool done = bits <= 32 ? new_slots(uint32_t{}) : new_slots(uint64_t{});
    if (done) {
      sc.used = mark;
      return hm;
    }
    sc.used = mark;
  }
  // stable group by slot: sort (slot, record index) pairs; invalid records (-2) sort last and are dropped
  uint32_t* sk = (uint32_t*)sc.take(std::max<int64_t>(n, 1) * 4);
  uint32_t* sk2 = (uint32_t*)sc.take(std::max<int64_t>(n, 1) * 4);
  uint32_t* si = (uint32_t*)sc.take(std::max<int64_t>(n, 1) * 4);
  uint32_t* si2 = (uint32_t*)sc.take(std::max<int64_t>(n, 1) * 4);
  if (n > 0) hipLaunchKernelGGL(slot_to_u32_kernel, grid_for(n), dim3(256), 0, s, slot, n, (uint32_t)T.nslots, sk, si);
  int bits = 0;  // sort keys are 0 .. nslots: only their significant bits take radix passes
  while (bits < 32 && ((uint64_t)T.nslots >> bits) != 0) ++bits;
  bool alt = radix_sort_pairs<uint32_t>(sk, sk2, si, si2, n, 0, bits, sc, s);
  if (alt) {
    std::swap(sk, sk2);
    std::swap(si, si2);
  }
  int64_t* key_off = (int64_t*)sc.take(((int64_t)T.nslots + 2) * 8);
  uint32_t* counts = (uint32_t*)sc.take(((int64_t)T.nslots + 2) * 4);
  uint32_t* total = (uint32_t*)sc.take(4);
  SM_HIP(hipMemsetAsync(counts, 0, ((int64_t)T.nslots + 2) * 4, s));
  if (n > 0) hipLaunchKernelGGL(count_valid_slots_kernel, grid_for(n), dim3(256), 0, s, sk, n, (uint32_t)T.nslots, counts);
  exclusive_scan_u32(counts, (int64_t)T.nslots + 1, sc, s, total);
  hipLaunchKernelGGL(u32_to_i64_kernel, grid_for((int64_t)T.nslots + 1), dim3(256), 0, s, counts,
                     (int64_t)T.nslots + 1, key_off);
  uint32_t hv = 0;
  SM_HIP(hipMemcpyAsync(&hv, total, 4, hipMemcpyDeviceToHost, s));
  SM_HIP(hipStreamSynchronize(s));
  int64_t* key_pos = (int64_t*)sc.take(std::max<int64_t>(hv, 1) * 8);
  if (hv > 0) hipLaunchKernelGGL(gather_pos_kernel, grid_for(hv), dim3(256), 0, s, pos, si, (int64_t)hv, key_pos);
  *key_pos_out = key_pos;
  *key_off_out = key_off;
  return hv;
}

namespace {
__global__ void iota_kernel(int64_t* __restrict__ out, int64_t n, int64_t start) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = start + i;
}
}  // namespace

namespace {
__global__ void __launch_bounds__(256) carry_columns_kernel(const int64_t* __restrict__ rows, int64_t n, CarryCols c) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const int64_t* row = rows + r * c.width;
  c.ord[r] = row[1];
  c.ts[r] = row[2];
  for (int k = 0; k < c.nattr; ++k) {
    const int64_t v = row[3 + k];
    const int t = c.types[k];
    if (t == T_INT || t == T_STRING) ((int32_t*)c.cols[k])[r] = (int32_t)v;
    else if (t == T_FLOAT) ((float*)c.cols[k])[r] = (float)__longlong_as_double(v);
    else if (t == T_LONG || t == T_DOUBLE) ((int64_t*)c.cols[k])[r] = v;
    else ((uint8_t*)c.cols[k])[r] = (uint8_t)(v != 0);
  }
}
}  // namespace

namespace {
__global__ void strided_get_kernel(const int64_t* __restrict__ rows, int64_t n, int w, int64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = rows[i * w];
}
__global__ void strided_put_kernel(const int32_t* __restrict__ ids, int64_t n, int w, int64_t* __restrict__ rows) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) rows[i * w] = ids[i];
}
}  // namespace

void remap_carry_keys(DenseKeys& D, int64_t* rows, int64_t n, int width, Scratch& sc, hipStream_t s) {
  if (n <= 0) return;
  const size_t mark = sc.used;
  int64_t* k = (int64_t*)sc.take((size_t)n * 8);
  int32_t* ids = (int32_t*)sc.take((size_t)n * 4);
  hipLaunchKernelGGL(strided_get_kernel, grid_for(n), dim3(256), 0, s, (const int64_t*)rows, n, width, k);
  remap_keys(D, k, T_LONG, n, ids, s);  // an INT key's carried value is its sign extension: the same table entry
  hipLaunchKernelGGL(strided_put_kernel, grid_for(n), dim3(256), 0, s, (const int32_t*)ids, n, width, rows);
  SM_HIP(hipStreamSynchronize(s));
  sc.used = mark;
}

void carry_rows_to_columns(const int64_t* rows, int64_t n, const CarryCols& c, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(carry_columns_kernel, grid_for(n), dim3(256), 0, s, rows, n, c);
}

void iota_i64(int64_t* out, int64_t n, int64_t start, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(iota_kernel, grid_for(n), dim3(256), 0, s, out, n, start);
}

namespace {
// sort keys of each record: key creation ordinal + 1 (0 = non-partitioned listener, first), time (sign-flipped),
// (pos << 1) | phase; flag[0] |= 1 when a timer record's time differs from its position's clock (wall-clock
// emulation: several steps at one advance point), which makes the time pass necessary
__global__ void out_keys_kernel(const char* __restrict__ recs, int64_t n, uint32_t stride,
                                const int64_t* __restrict__ ev_clock, uint64_t* __restrict__ kc,
                                uint64_t* __restrict__ kt, uint64_t* __restrict__ kp, uint32_t* __restrict__ idx,
                                uint32_t* __restrict__ flag) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const OutRec& r = *(const OutRec*)(recs + (size_t)i * stride);
  kc[i] = (uint64_t)(r.create + 1);
  kt[i] = (uint64_t)r.time ^ 0x8000000000000000ull;
  kp[i] = ((uint64_t)r.pos << 1) | (uint64_t)(r.phase & 1);
  idx[i] = (uint32_t)i;
  if (r.phase == 0 && (!ev_clock || r.time != ev_clock[r.pos])) atomicOr(flag, 1u);
}

// pos (a batch position) -> the batch's ordinal there: the trigger's global ordinal (a heartbeat's entry is the
// ordinal of the event that advanced the clock)
__global__ void trigger_ordinals_kernel(char* __restrict__ recs, int64_t n, uint32_t stride,
                                        const int64_t* __restrict__ ev_ord) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  OutRec& r = *(OutRec*)(recs + (size_t)i * stride);
  r.pos = ev_ord[r.pos];
}

__global__ void gather_key_kernel(const uint64_t* __restrict__ src, const uint32_t* __restrict__ idx, int64_t n,
                                  uint64_t* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[idx[i]];
}

// a thread per 8-byte word of the ordered copy
__global__ void gather_records_kernel(const char* __restrict__ recs, const uint32_t* __restrict__ idx, int64_t n,
                                      uint32_t words, char* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * words) return;
  const int64_t i = t / words, w = t - i * words;
  ((uint64_t*)out)[i * words + w] = ((const uint64_t*)recs)[(int64_t)idx[i] * words + w];
}

}  // namespace

void trigger_ordinals(char* recs, int64_t n, uint32_t stride, const int64_t* ev_ord, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(trigger_ordinals_kernel, grid_for(n), dim3(256), 0, s, recs, n, stride, ev_ord);
}

const char* order_outputs(const char* recs, int64_t n, uint32_t stride, const int64_t* ev_clock, Scratch& sc,
                          hipStream_t s, int pos_bits, char* out_to) {
  if (n >= (int64_t)UINT32_MAX) throw std::runtime_error("too many output records to order");
  if (stride % 8) throw std::logic_error("output record stride");
  uint64_t* kc = (uint64_t*)sc.take((size_t)n * 8);
  uint64_t* kt = (uint64_t*)sc.take((size_t)n * 8);
  uint64_t* kp = (uint64_t*)sc.take((size_t)n * 8);
  uint64_t* k2 = (uint64_t*)sc.take((size_t)n * 8);
  uint32_t* idx = (uint32_t*)sc.take((size_t)n * 4);
  uint32_t* idx2 = (uint32_t*)sc.take((size_t)n * 4);
  uint32_t* flag = (uint32_t*)sc.take(4);
  char* out = out_to ? out_to : (char*)sc.take((size_t)n * stride);
  SM_HIP(hipMemsetAsync(flag, 0, 4, s));
  hipLaunchKernelGGL(out_keys_kernel, grid_for(n), dim3(256), 0, s, recs, n, stride, ev_clock, kc, kt, kp, idx, flag);
  uint32_t hflag = 0;
  SM_HIP(hipMemcpyAsync(&hflag, flag, 4, hipMemcpyDeviceToHost, s));
  SM_HIP(hipStreamSynchronize(s));
  // least significant first: creation ordinal (40 bits cover any batch history), time (if it varies), (pos, phase)
  uint32_t* cur = idx;
  uint32_t* alt = idx2;
  auto pass = [&](uint64_t* keys, int bits, bool gathered) {
    uint64_t* k = keys;
    if (gathered) {  // the keys in the current order
      hipLaunchKernelGGL(gather_key_kernel, grid_for(n), dim3(256), 0, s, keys, cur, n, k2);
      k = k2;
    }
    uint64_t* kalt = k == k2 ? keys : k2;
    if (radix_sort_pairs<uint64_t>(k, kalt, cur, alt, (size_t)n, 0, bits, sc, s)) std::swap(cur, alt);
  };
  // creation ordinals: batch-history ordinals within one app fit 41 bits; the multi-GPU merge (no ev_clock) sorts
  // global ordinals, as wide as the trigger ordinals
  pass(kc, ev_clock ? 41 : std::min(64, pos_bits + 1), false);
  if (hflag) pass(kt, 64, true);
  pass(kp, pos_bits + 1, true);  // batch positions < 2^32 (build_event_index); trigger ordinals: 63 bits
  const uint32_t words = stride / 8;
  hipLaunchKernelGGL(gather_records_kernel, grid_for(n * words), dim3(256), 0, s, recs, cur, n, words, out);
  return out;
}

int64_t build_event_index(int64_t n, const int32_t* sid, int32_t nstreams, const int64_t* ts, const int64_t* ord_in,
                          int64_t ord_base, bool playback, int64_t clock_in, int64_t* ev_row, int64_t* ev_ord,
                          int64_t* ev_clock, int64_t* adv_pos, int64_t* adv_clock, int64_t* adv_wall,
                          int64_t* adv_upto, int64_t* clock_out, Scratch& sc, hipStream_t s) {
  *clock_out = clock_in;
  if (n == 0) return 0;
  if (n >= (int64_t)UINT32_MAX) throw std::runtime_error("device event batch too large (>= 2^32 events)");
  size_t mark = sc.used;
  const int64_t ntiles = (n + kIxTile - 1) / kIxTile;
  int64_t* tile_max = (int64_t*)sc.take(ntiles * 8);
  int64_t* dclock = (int64_t*)sc.take(8);
  uint64_t* amask = (uint64_t*)sc.take(((n + 63) / 64) * 8);
  uint32_t* acnt = (uint32_t*)sc.take((ntiles + 1) * 4);
  uint32_t* total = (uint32_t*)sc.take(4);
  int32_t* bad = (int32_t*)sc.take(4);
  SM_HIP(hipMemsetAsync(bad, 0, 4, s));
  hipLaunchKernelGGL(ts_tile_max_kernel, dim3((unsigned)ntiles), dim3(kIxThreads), 0, s, ts, n, tile_max);
  hipLaunchKernelGGL(tile_prefix_max_kernel, dim3(1), dim3(kIxThreads), 0, s, tile_max, ntiles, clock_in, dclock);
  hipLaunchKernelGGL(event_index_kernel, dim3((unsigned)ntiles), dim3(kIxThreads), 0, s, sid, nstreams, ts, n, ord_in,
                     ord_base, (int)playback, clock_in, tile_max, ev_row, ev_ord, ev_clock, amask, acnt, bad);
  int64_t nadv = 0;
  if (!playback) SM_HIP(hipMemsetAsync(adv_upto, 0, (size_t)n * 8, s));
  if (playback) {
    exclusive_scan_u32(acnt, ntiles, sc, s, total);
    hipLaunchKernelGGL(advance_rank_kernel, dim3((unsigned)ntiles), dim3(kIxThreads), 0, s, amask, n, acnt, ts,
                       adv_pos, adv_clock, adv_wall, adv_upto);
    uint32_t h = 0;
    SM_HIP(hipMemcpyAsync(&h, total, 4, hipMemcpyDeviceToHost, s));
    nadv = h;
  }
  int64_t hc = clock_in;
  int32_t hbad = 0;
  SM_HIP(hipMemcpyAsync(&hc, dclock, 8, hipMemcpyDeviceToHost, s));
  SM_HIP(hipMemcpyAsync(&hbad, bad, 4, hipMemcpyDeviceToHost, s));
  SM_HIP(hipStreamSynchronize(s));
  if (hbad) throw std::invalid_argument("stream index out of range in device event batch");
  if (playback) *clock_out = hc > clock_in ? hc : clock_in;
  sc.used = mark;
  return nadv;
}

}  // namespace sm
