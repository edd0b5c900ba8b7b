// Host entry points of the column-scan / key-grouping kernels (stream_ops.hip).
#pragma once
#include "nfa.h"
#include "primitives.h"

namespace sm {

struct KeyProg {  // partition key expression of one stream (device copy)
  int32_t stream, len, type, pad;
  const Instr* code;
  const DVal* consts;
};

// Device key → slot table (open addressing) with slot → key inverse; slots are per-key state indices.
struct KeyTable {
  int64_t* tkeys = nullptr;
  int32_t* tslots = nullptr;  // slot + 1, 0 = empty
  uint64_t mask = 0;
  int64_t cap = 0;
  int64_t* slot_keys = nullptr;
  int64_t slot_cap = 0;
  int32_t nslots = 0;
  void reserve(int64_t total_slots, hipStream_t s);
  void load(const int64_t* keys_host, int32_t n, hipStream_t s);
  void release();
};

// Dense ids of a closed-form query's partition keys (remap_keys): any int32 / int64 key domain (sparse 64-bit ids,
// spans of 2^40 ...) becomes ids 0 .. nslots-1, so the keyed pipelines see a key span of the number of distinct keys.
// An open-addressing table of 16-byte entries {key, id + 1 | busy}, filled by the lookup kernel itself (an event whose
// key is missing claims an entry and the next id), persistent across batches: carried partials hold dense ids.
struct DenseKeys {
  int64_t* table = nullptr;      // cap entries of two words: key, state (0 empty, -1 being inserted, else id + 1)
  int64_t* slot_keys = nullptr;  // id -> key
  uint32_t* counter = nullptr;   // device: ids handed out
  int64_t cap = 0, slot_cap = 0;
  int64_t nslots = 0;
  void reserve(int64_t slots, hipStream_t s);
  void load(const int64_t* keys_host, int64_t n, hipStream_t s);  // restore: ids 0 .. n-1 = keys_host
  void clear(hipStream_t s);
  void release();
};
// smallest and largest key of an int32 / int64 key column
void key_range(const void* col, int key_type, int64_t n, int64_t* lo, int64_t* hi, Scratch& sc, hipStream_t s);
// out[i] = dense id of key column col[i] (key_type T_INT or T_LONG), new keys added; n events.
void remap_keys(DenseKeys& D, const void* col, int key_type, int64_t n, int32_t* out, hipStream_t s);
// the key word (word 0) of n carried closed-form rows of `width` words, in place: raw key -> dense id (a query that
// starts giving its keys dense ids after partials were carried under their values)
void remap_carry_keys(DenseKeys& D, int64_t* rows, int64_t n, int width, Scratch& sc, hipStream_t s);

// FilterProcessor over rows [0, n) of one stream; writes matching row indices (ascending), returns the count.
int64_t filter_rows(const NfaStream* st_dev, int64_t n, const Instr* code, int len, const DVal* consts,
                    int64_t* out_rows, Scratch& sc, hipStream_t s);
void project_rows(const NfaStream* st_dev, const int64_t* rows, int64_t nm, const int64_t* row_pos,
                  const int64_t* ev_ts, const int64_t* ev_ord, const char* blob_dev, int32_t query_order, char* out,
                  uint32_t stride, hipStream_t s);
int64_t select_records(const int32_t* ev_stream, int64_t n, uint64_t stream_mask, bool with_start, int64_t* out_pos,
                       Scratch& sc, hipStream_t s);
int64_t group_by_key(KeyTable& T, const int64_t* pos, int64_t n, const int32_t* ev_stream, const int64_t* ev_row, int nstreams,
                     const NfaStream* streams_dev, const KeyProg* progs_dev, int nprogs, int64_t** key_pos_out,
                     int64_t** key_off_out, Scratch& sc, hipStream_t s, bool pos_identity = false);

// Per-event index arrays of a device-resident interleaved batch (the device restatement of stage_record);
// returns the number of clock-advance points written to adv_*.
// sid[i] = stream index, or NFA_TICK (-1) for a playback heartbeat (clock advance without an event).
// out[i] = start + i
void iota_i64(int64_t* out, int64_t n, int64_t start, hipStream_t s);
// Carried closed-form partials (rows of `width` int64: key, ordinal, event time, then the attributes in canonical
// form: integers as int64, FLOAT / DOUBLE as double bits) as the columns of a stream: attribute k (type types[k]) to
// cols[k] in its own width, event time to ts, ordinal to ord (the hand-over of the carry to the NFA kernel).
struct CarryCols {
  int32_t nattr, width;
  int32_t types[kMaxAttrs];
  void* cols[kMaxAttrs];
  int64_t* ts;
  int64_t* ord;
};
void carry_rows_to_columns(const int64_t* rows, int64_t n, const CarryCols& c, hipStream_t s);

// One query's n output records (stride bytes each, OutRec first) in delivery order (runtime.cpp deliver): by
// (pos, phase), then for timer-phase records (time, listener group, key creation ordinal); a lane's own records
// keep their emission order (the sorts are stable and a lane's slots ascend). Returns the ordered copy (scratch, or
// out_to). ev_clock null: the records' time always takes part (the multi-GPU merge: pos holds trigger ordinals of
// pos_bits bits).
const char* order_outputs(const char* recs, int64_t n, uint32_t stride, const int64_t* ev_clock, Scratch& sc,
                          hipStream_t s, int pos_bits = 32, char* out_to = nullptr);

// Output records' pos (batch position) -> ev_ord[pos] (the trigger's global ordinal).
void trigger_ordinals(char* recs, int64_t n, uint32_t stride, const int64_t* ev_ord, hipStream_t s);

int64_t build_event_index(int64_t n, const int32_t* sid, int32_t nstreams, const int64_t* ts, const int64_t* ord_in,
                          int64_t ord_base, bool playback, int64_t clock_in, int64_t* ev_row, int64_t* ev_ord,
                          int64_t* ev_clock, int64_t* adv_pos, int64_t* adv_clock, int64_t* adv_wall,
                          int64_t* adv_upto, int64_t* clock_out, Scratch& sc, hipStream_t s);

}  // namespace sm
