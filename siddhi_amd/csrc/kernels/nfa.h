// Device batch descriptors shared by the runtime (host) and the NFA / filter / fast-path kernels.
#pragma once
#include "hd.h"

#include "../plan.h"

namespace sm {

constexpr int kMaxAttrs = 48;
constexpr int NFA_START = -3;  // ev_stream marker: SiddhiAppRuntime.start()
constexpr int NFA_TICK = -1;   // playback heartbeat (clock advance without an event)
constexpr int NFA_WALL = -2;   // wall-clock emulation tick

enum : int32_t { NFA_ERR_ARENA = 1, NFA_ERR_TIMERS = 2, NFA_ERR_OUTPUT = 4, NFA_ERR_NPE = 8 };

struct NfaStream {
  int32_t nattr;
  int32_t types[kMaxAttrs];
  const void* cols[kMaxAttrs];
  const uint8_t* nulls[kMaxAttrs];  // null flags per attribute or nullptr
};

// One event of a query's batch in key order (built by the lane-events pass from key_pos and the batch
// columns): position, stream, clock after sendData, advance points up to it (-1 = unknown), then the chain-node
// image the NFA copies into a partial (word 0 unused, ts, ordinal, null mask, attribute words).
struct LaneEv {
  enum : int { kPos = 0, kStream = 1, kClock = 2, kUpto = 3, kNode = 4 };
  // padded to whole 64-byte halves / 128-byte lines: the lane-events pass scatters records to key order, and a
  // record that fills its lines is written without a partial-line merge in HBM (96 -> 128 B for StockStream)
  static __host__ __device__ constexpr int64_t words(int node_words) {
    return kNode + node_words <= 8 ? 8 : (kNode + node_words + 15) / 16 * 16;
  }
  // Compact form (NfaBatch::lane_compact; node images of at most 8 words = up to 4 attributes): one 64-byte record
  //   w0 = position (u32) | advance points up to it (i32) << 32, w1 = clock, w2 = event time,
  //   w3 = ordinal - lane_ord_base (48 bits, all ones = none) | stream (i8) << 48 | null mask (8 bits) << 56,
  //   w4..w7 = attribute words.
  // Half the bytes of the 128-byte form for the lane-events pass to write and the NFA lanes to read.
  static __host__ __device__ constexpr int64_t words(int node_words, bool compact) {
    return compact ? 8 : words(node_words);
  }
};
constexpr uint64_t kLeOrdMask = (1ull << 48) - 1;

struct NfaBatch {
  // app batch (all records in arrival order)
  const int32_t* ev_stream;  // stream index or NFA_* marker
  const int64_t* ev_row;     // row within the stream's columns (nullptr: the position; device batches)
  const int64_t* ev_ts;
  const int64_t* ev_clock;   // playback clock after the record's sendData
  const int64_t* ev_ord;     // global arrival ordinal of each data event (-1 for markers)
  const NfaStream* streams;
  // advance points (playback listener firings / wall ticks), ascending position
  const int64_t* adv_pos;
  const int64_t* adv_clock;
  const int64_t* adv_wall;   // wall tick target, -1 for playback points
  const int64_t* adv_upto;   // per record position: advance points at positions <= it (nullable)
  int64_t nadv;
  int64_t clock_in;          // clock before the batch
  // clock index of the advance points (round 5; nullable): adv_cidx[c - adv_cmin] = the first advance point whose
  // clock is >= c, for c in [adv_cmin, adv_cmin + adv_cspan), so a timer's due point is one load (timer_fire)
  const int32_t* adv_cidx;
  int64_t adv_cmin, adv_cspan;
  // this query's records grouped by key slot: key_pos[key_off[k] .. key_off[k+1]) ascending
  const int64_t* key_off;
  const int64_t* key_pos;
  const int64_t* lane_ev;    // LaneEv records, one per key_pos entry (filled by launch_lane_events)
  int32_t lane_compact;      // LaneEv records in the compact 64-byte form (LaneEv)
  int64_t lane_ord_base;     // compact form: ordinals are stored relative to it
  int32_t create_all;        // non-partitioned: the single lane exists from app creation
  const uint32_t* lane_perm; // lane -> key slot (launch_lane_balance), nullptr = identity
  // output
  void* out;
  uint32_t* out_count;
  uint32_t out_cap;
  uint32_t out_stride;
  // device-wide overflow pool of per-key arenas: a key whose live partial matches outgrow its own arena moves its
  // heap into a larger region bump-allocated here (Lane::promote). pool_top counts the words handed out; a request
  // that does not fit claims nothing, and pool_top[1] keeps the largest such request, so that the host sizes the pool
  // for it after the batch (without the demand a hot key's failed promotion never grew the pool).
  int64_t* pool;
  unsigned long long* pool_top;
  int64_t pool_cap;
};

// Fields of a LaneEv record in either form (b.lane_compact; a query-specialised kernel is compiled for one form,
// SM_LANE_COMPACT_CONST, so the choice folds away)
#ifdef SM_LANE_COMPACT_CONST
#define SM_LE_C(b) (SM_LANE_COMPACT_CONST != 0)
#else
#define SM_LE_C(b) ((b).lane_compact != 0)
#endif
__host__ __device__ inline int64_t le_pos(const NfaBatch& b, const int64_t* r) {
  return SM_LE_C(b) ? (int64_t)(uint32_t)r[0] : r[LaneEv::kPos];
}
__host__ __device__ inline int64_t le_upto(const NfaBatch& b, const int64_t* r) {
  return SM_LE_C(b) ? (int64_t)(int32_t)((uint64_t)r[0] >> 32) : r[LaneEv::kUpto];
}
__host__ __device__ inline int le_stream(const NfaBatch& b, const int64_t* r) {
  return SM_LE_C(b) ? (int)(int8_t)(uint8_t)((uint64_t)r[3] >> 48) : (int)r[LaneEv::kStream];
}
__host__ __device__ inline int64_t le_clock(const NfaBatch& b, const int64_t* r) {
  return SM_LE_C(b) ? r[1] : r[LaneEv::kClock];
}
// word w (1 .. node_words - 1) of the chain-node image: event time, ordinal, null mask, attribute words
__host__ __device__ inline int64_t le_node(const NfaBatch& b, const int64_t* r, int w) {
  if (!SM_LE_C(b)) return r[LaneEv::kNode + w];
  if (w == 1) return r[2];
  if (w == 2) {
    const uint64_t v = (uint64_t)r[3] & kLeOrdMask;
    return v == kLeOrdMask ? -1 : b.lane_ord_base + (int64_t)v;
  }
  if (w == 3) return (int64_t)(((uint64_t)r[3] >> 56) & 0xFF);
  return r[w];  // attribute a = w - 4 at word 4 + a
}

// LaneEv records for key_pos[0, nq) of a batch of n records: b.lane_ev must point at
// nq * LaneEv::words(node_words, b.lane_compact) words, inv_scratch at n int32
void launch_lane_events(const NfaBatch& b, int64_t n, int64_t nq, int32_t node_words, int32_t* inv_scratch,
                        int nstreams, hipStream_t s);
// stream descriptors a kernel copies into LDS (per-record attribute reads then find column pointers and types there
// instead of in device memory): batches with at most this many streams
constexpr int kLdsStreams = 8;

static_assert(sizeof(NfaStream) % 8 == 0, "stream descriptors are copied as 8-byte words");
// Lane order by descending event count of the batch (stable by slot), so that the 64 lanes of a wave walk about
// as many events each: a wave runs as long as its longest lane. perm must hold nkeys uint32.
struct Scratch;
void launch_lane_balance(const int64_t* key_off, int32_t nkeys, uint32_t* perm, Scratch& sc, hipStream_t s);
// The clock index of a batch's advance points (NfaBatch::adv_cidx): idx[c] = first advance point whose clock is
// >= cmin + c, for c in [0, span). One thread per clock value, a binary search over adv_clock (non-decreasing).
void launch_clock_index(const int64_t* adv_clock, int64_t nadv, int64_t cmin, int64_t span, int32_t* idx, hipStream_t s);
// Whether this batch's LaneEv records can take the compact form: node images of at most 8 words, positions and
// advance points below 2^31, stream indices in int8, and the data events' ordinals within a 2^48 - 1 range (a
// reduction over ev_ord; *ord_base = their minimum).
bool lane_compact_ok(const NfaBatch& b, int64_t n, int32_t node_words, int nstreams, Scratch& sc, hipStream_t s,
                     int64_t* ord_base);
// ks is lane-interleaved: word w of key k at [w * lanes + k] (lanes = allocated key capacity); heap is key-major
void launch_nfa(const NfaBatch& b, const char* blob_dev, int64_t* ks, int64_t* heap, int32_t heap_half, int64_t lanes,
                int32_t nkeys, int32_t* err_dev, hipStream_t s);

// One pass of the overflow-pool compaction over nkeys key slots (nfa_impl.h nfa_pool_lane): pass 0 writes each key's
// new home to new_off (-2 none, -1 its own arena, else an offset claimed from new_top), pass 1 moves the live objects.
void launch_pool_compact(int pass, const char* blob_dev, int64_t* ks, int64_t* heap, int32_t heap_half, int64_t lanes,
                         int32_t nkeys, int64_t* old_pool, int64_t* new_pool, unsigned long long* new_top,
                         int64_t* new_off, hipStream_t s);

}  // namespace sm
