// Stable partition of a columnar batch by owner rank (multi-GPU key exchange); see partition.hip.
#pragma once
#include <vector>

#include "primitives.h"

namespace sm {

constexpr int kMaxOwners = 64;
constexpr int kMaxPartCols = 16;

struct PartCols {
  int32_t n;
  int32_t width[kMaxPartCols];   // bytes per element: 1, 2, 4 or 8
  int32_t stride[kMaxPartCols];  // bytes between consecutive destination elements (= width for a column;
                                 // the record size when several columns are packed into one record buffer)
  const void* src[kMaxPartCols];
  void* dst[kMaxPartCols];
};

// Owner rank of a partition key: the high half of the splitmix64 finalizer of the key's 64-bit two's complement
// image, modulo world (hash-by-key, so keys with structure in their low residues still spread over the ranks).
// siddhi_amd/shard.py owner_of computes the same function with torch.
__host__ __device__ inline uint32_t key_owner(int64_t key, uint32_t world) {
  uint64_t z = (uint64_t)key;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32) % world;
}

// Matches received from the key-owning ranks, ordered back into the reference's global order for the ordinal
// slice [lo, hi) this rank ingested: pairs are (e2 << 32) | e1 (e1 as 32-bit two's complement), the input is the
// concatenation of per-source runs each ordered by (e2, e1), and every e2 appears in one run only.
void order_matches(const uint64_t* pairs, int64_t n, int64_t lo, int64_t hi, uint64_t* out, Scratch& sc,
                   hipStream_t s);

void partition_by_owner(const void* keys, int key_width, int64_t n, uint32_t world, const PartCols& cols,
                        uint64_t* counts_host, Scratch& sc, hipStream_t s);

// Output of merge_heartbeats: the merged sequence's stream index (-1 = heartbeat), event time, global ordinal (-1 for
// a heartbeat) and every column (src[c] of the events -> dst[c]; a heartbeat's attribute words are zero).
struct MergeOut {
  int32_t ncols;
  int32_t width[kMaxPartCols];  // 4 or 8
  const void* src[kMaxPartCols];
  void* dst[kMaxPartCols];
  int32_t* sid;
  int64_t* ts;
  int64_t* ord;
};

// Multi-GPU playback (@app:playback partitioned apps): a rank's received events (n, global ordinals `ord`
// ascending) merged with the global clock-advance points (m, ordinals `tord` ascending, clock `tts`) in ordinal
// order; a point at an ordinal this rank holds is dropped (that event advances the clock itself,
// StreamJunction.sendData :232-237). Returns the merged length (n + points kept); outputs need n + m entries.
int64_t merge_heartbeats(const int64_t* ord, const int32_t* sid, const int64_t* ts, int64_t n, const int64_t* tord,
                         const int64_t* tts, int64_t m, const MergeOut& o, Scratch& sc, hipStream_t s);

// Receive side of the key exchange: the packed records the all-to-all-v delivered (m records of rec_words 8-byte
// words, runs per source rank in rank order) split into contiguous columns in ONE pass, and the field holding each
// record's uint32 offset inside its source's ingest slice turned into the int64 global ordinal
// (src_first[source] + offset). Replaces one strided copy per column plus the ordinal arithmetic.
struct UnpackCols {
  int32_t n;                     // fields
  int32_t rec_words;             // record size in 8-byte words (<= 8)
  int32_t off[kMaxPartCols];     // byte offset of each field in the record
  int32_t width[kMaxPartCols];   // 1, 2, 4 or 8
  void* dst[kMaxPartCols];       // contiguous output column (nullptr: not copied)
  int32_t ord_field;             // field with the in-slice uint32 offset (-1: none)
  int32_t nsrc;                  // source ranks (runs), <= kMaxOwners
  int64_t run_end[kMaxOwners];   // exclusive end of each source's run in the received buffer
  int64_t src_first[kMaxOwners]; // first global ordinal of each source's ingest slice
  int64_t* ord_out;
};

void unpack_records(const uint64_t* rec, int64_t m, const UnpackCols& u, hipStream_t s);

}  // namespace sm
