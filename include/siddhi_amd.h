/* siddhi_amd — MI355X-native pattern/sequence matching engine, C ABI (the drop-in boundary).
 *
 * Each entry point replaces one reference API (paths relative to
 * modules/siddhi-core/src/main/java/org/wso2/siddhi/core/):
 *   sm_manager_create / destroy     SiddhiManager()                         SiddhiManager.java:56
 *   sm_app_create                   SiddhiManager.createSiddhiAppRuntime    SiddhiManager.java:73
 *   sm_app_input_handler            SiddhiAppRuntime.getInputHandler        SiddhiAppRuntime.java:337
 *   sm_input_send                   InputHandler.send(long, Object[])       stream/input/InputHandler.java:53
 *   sm_input_send_columns           InputHandler.send(Event[])              stream/input/InputHandler.java:65 (columnar)
 *   sm_app_add_stream_callback      SiddhiAppRuntime.addCallback(String, StreamCallback)  :243
 *   sm_count_events_callback        the counting StreamCallback of the reference's performance samples
 *   sm_app_add_query_callback       SiddhiAppRuntime.addCallback(String, QueryCallback)   :254
 *   sm_app_add_stream_columns_callback  SiddhiAppRuntime.addCallback(String, StreamCallback), Event[] as columns
 *   sm_app_start / sm_app_shutdown  SiddhiAppRuntime.start / shutdown       :353 / :396
 *   sm_app_advance_time             @app:playback heartbeat (EventTimeBasedMillisTimestampGenerator.java:99)
 *   sm_app_process_device_batch     StreamJunction.sendData over a device-resident columnar batch (no Java
 *                                   counterpart: the bulk entry a JNI/Panama receiver would call)
 *   sm_app_snapshot / sm_app_restore  SiddhiAppRuntime.snapshot() / restore(byte[])  :548 / :560
 *   sm_partition_by_owner           multi-GPU form of PartitionStreamReceiver.receive (partition/
 *                                   PartitionStreamReceiver.java:156): route each event to its key's owner rank
 *   sm_merge_heartbeats             multi-GPU playback: the global clock advances (StreamJunction.sendData :232)
 *                                   replayed as heartbeats among a rank's received events
 *   sm_unpack_records               multi-GPU receive side of the key exchange: packed records -> columns + global
 *                                   ordinals (no reference counterpart: one JVM has no exchange)
 *   sm_app_copy_device_outputs      the ordered output records of the last interleaved device batch (multi-GPU merge)
 *   sm_order_outputs                multi-GPU merge of per-rank output records into one JVM's delivery order
 *   sm_order_matches                multi-GPU merge of the per-rank outputs back into the single output order a
 *                                   query callback sees (QueryCallback.receive, query/output/callback/
 *                                   QueryCallback.java:51): no Java counterpart, one JVM has one output queue
 *   sm_app_copy_device_matches      the device tuples of the last batch into a caller buffer (for collectives)
 *   sm_app_device_project           QuerySelector.processNoGroupBy (query/selector/QuerySelector.java:124-167) for
 *                                   those tuples, on the device: Event.data + timestamp of each output
 *   sm_compile_dump                 SiddhiCompiler.parse (siddhi-query-compiler .../SiddhiCompiler.java:56)
 *   sm_nfa_jit_compile              QueryParser.parse (core/util/parser/QueryParser.java:79) for one query, as the
 *                                   query-specialised NFA kernel (no device needed): the build check of the JIT
 *   sm_app_process_device_events    a sequence of InputHandler.send calls over several streams of one
 *                                   schema (InputHandler.java:53 → StreamJunction.sendData :232), device-resident
 *
 * Threading / delivery: an app handle is single-owner (calls are serialised internally). Events are
 * staged on send and processed on the GPU at sm_app_flush (also at shutdown and when the staging buffer
 * fills); callbacks run on the calling thread at that point, in the reference's emission order (per output
 * chunk the query's QueryCallbacks, then its output stream's StreamCallbacks: OutputRateLimiter.sendToCallBacks
 * :61-73). Event
 * arrays passed to callbacks are valid only during the callback. Errors never cross the ABI as exceptions:
 * every call returns a status and sm_last_error() holds the thread-local message.
 */
#ifndef SIDDHI_AMD_H
#define SIDDHI_AMD_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

enum {
  SM_OK = 0,
  SM_E_PARSE = 1,        /* SiddhiParserException */
  SM_E_VALIDATION = 2,   /* SiddhiAppValidationException / SiddhiAppCreationException */
  SM_E_UNSUPPORTED = 3,  /* construct outside the hot-path subset */
  SM_E_TYPE = 4,         /* value type does not match the stream definition (ClassCastException) */
  SM_E_DEVICE = 5,       /* HIP error */
  SM_E_RUNTIME = 6,      /* runtime failure (reference NullPointerException paths, capacity) */
  SM_E_ARG = 7
};

enum { SM_INT = 0, SM_LONG = 1, SM_FLOAT = 2, SM_DOUBLE = 3, SM_STRING = 4, SM_BOOL = 5 };

typedef struct sm_value {
  int32_t type;
  int32_t is_null;
  int64_t i;     /* INT / LONG / BOOL */
  double d;      /* FLOAT / DOUBLE */
  const char* s; /* STRING */
} sm_value;

typedef struct sm_event {
  int64_t timestamp;
  const sm_value* data;
  int32_t n;
} sm_event;

typedef struct sm_manager sm_manager;
typedef struct sm_app sm_app;
typedef struct sm_input sm_input;

typedef void (*sm_stream_callback)(void* user, const sm_event* events, size_t n);
/* A StreamCallback taking its Event[] as columns (round 6): n events, ts[k] the timestamp of event k, values[k * nsel +
 * a] its attribute a as an 8-byte word (INT / LONG / BOOL as the integer, FLOAT / DOUBLE as the double's bits, FLOAT
 * widened), bit a of null_bits[k] set when that attribute is null. The same chunks, in the same order and among the
 * same other callbacks as sm_stream_callback receives them; the arrays are valid during the call only. */
typedef void (*sm_stream_columns_callback)(void* user, size_t n, const int64_t* ts, const int64_t* values,
                                           const uint8_t* null_bits, int32_t nsel);
typedef void (*sm_query_callback)(void* user, int64_t timestamp, const sm_event* in_events, size_t n_in,
                                  const sm_event* removed_events, size_t n_removed);

const char* sm_last_error(void);
const char* sm_version(void);
/* Identity of this build: 16 hex digits of sha256 over the library's sources, headers and build flags. Not a
 * reference API; profiles/pmc_config<C>.json records it so bench.py reports PMC traffic only for the build measured. */
const char* sm_build_id(void);

int sm_manager_create(sm_manager** out);
void sm_manager_destroy(sm_manager* m);

int sm_app_create(sm_manager* m, const char* siddhiql, sm_app** out);
/* Parse only (no device needed): the app's query tree as canonical JSON (shapes in siddhiql/dump.cpp) into buf,
 * NUL-terminated when it fits in cap; *len = its length. Errors as sm_app_create reports them for the same text. */
int sm_compile_dump(const char* siddhiql, char* buf, size_t cap, size_t* len);
/* Compile query number `query` (app order) of the app into its query-specialised NFA kernel (the interpreter with
 * the query's plan fixed at compile time, hiprtc for gfx950; no device needed). *code_size = the code object's
 * size; on failure the compiler log is in log (NUL-terminated, at most cap bytes) and sm_last_error. The app option
 * "nfa_jit" (1 / 0 / -1 = automatic, for batches of 2^20 query records or more) selects this kernel at run time. */
int sm_nfa_jit_compile(const char* siddhiql, int query, char* log, size_t cap, size_t* code_size);
void sm_app_destroy(sm_app* app);
int sm_app_start(sm_app* app);
int sm_app_flush(sm_app* app);
int sm_app_shutdown(sm_app* app);

int sm_app_input_handler(sm_app* app, const char* stream_id, sm_input** out);
int sm_input_send(sm_input* in, int64_t timestamp, const sm_value* row, size_t n);
/* n events of the handler's stream; cols[k] = host column of attribute k (int32 / int64 / float / double /
 * uint8 for BOOL / const char* for STRING); null_flags may be NULL or hold per-attribute uint8 arrays.
 * Events are staged and processed at the next flush, except a batch of at least option "bulk_min" events (default
 * 65536) with no null flags and no STRING attribute sent into an app whose queries are all filters and
 * `every e1 -> e2 within T` patterns: it is processed inside the call, on the device-batch pipelines (closed form,
 * carried partials shared with device batches), uploaded in chunks of option "bulk_chunk" events (default 2^24) with
 * the upload of the next chunk overlapping the processing of the current one, and its outputs reach the callbacks
 * chunk by chunk before the call returns. Staged events of such an app take the same pipelines at flush. */
int sm_input_send_columns(sm_input* in, size_t n, const int64_t* timestamps, const void* const* cols,
                          const uint8_t* const* null_flags);

/* attribute types (SM_INT …) of a stream: writes up to cap entries, returns the count in *n */
int sm_app_stream_schema(sm_app* app, const char* stream_id, int32_t* types, size_t cap, size_t* n);

int sm_app_advance_time(sm_app* app, int64_t timestamp);
/* wall-clock scheduler emulation: fire every due timer at its scheduled time up to `timestamp` */
int sm_app_advance_wallclock(sm_app* app, int64_t timestamp);

int sm_app_add_stream_callback(sm_app* app, const char* stream_id, sm_stream_callback cb, void* user);
/* A ready-made sm_stream_callback that adds each call's event count to the int64 `user` points at (the counting
 * StreamCallback of the reference's performance samples, e.g. PartitionPerformance.java). */
void sm_count_events_callback(void* user, const sm_event* events, size_t n);
int sm_app_add_query_callback(sm_app* app, const char* query_name, sm_query_callback cb, void* user);
/* StreamCallback.receive(Event[]) (stream/output/StreamCallback.java:65-76) in the columns form above, for output streams
 * of at most 8 attributes and none STRING (SM_E_UNSUPPORTED otherwise). When every callback of a query's outputs takes
 * columns, the outputs of the device-batch pipelines reach them as views of the outputs' host copies: no per-Event
 * record is written (8 bytes per value and one null byte per event, against a 24-byte sm_event and a 32-byte sm_value
 * per value). */
int sm_app_add_stream_columns_callback(sm_app* app, const char* stream_id, sm_stream_columns_callback cb, void* user);
/* The counting callback in the columns form: adds n to the int64 `user` points at. */
void sm_count_columns_callback(void* user, size_t n, const int64_t* ts, const int64_t* values, const uint8_t* null_bits,
                               int32_t nsel);

/* Parity/diagnostics: collect every output as JSON
 * {"streams": {"<id>": [[ts, [values], [refs]], ...]}, "queries": {"<name>": [[ts, [[values]...]], ...]}}
 * where refs are the global arrival ordinals of the events at the select list's variable positions. */
int sm_app_set_collect(sm_app* app, int collect);
size_t sm_app_dump_outputs(sm_app* app, char* buf, size_t len);

/* Options (before the first flush): "heap_words" (per-key partial-match arena, words per semispace),
 * "batch_events" (auto-flush threshold), "fast_general" (1 = device batches always take the general
 * closed-form kernels), "fast_timing" (1 = record HIP events around the device-batch phases), "reset" (drop all
 * matching state, keep the device allocations), "lane_balance" (N > 0: order the NFA lanes of a partitioned batch
 * with >= N keys by descending event count, default 2^16; 0 = off; outputs are unchanged either way),
 * "fast_stack" (closed-form pipeline: 0 automatic, 1 bucket stack whenever it applies, 2 sort / walk),
 * "key_remap" (closed-form partition keys as dense device ids: 1 always, 0 never, -1 automatic = when the first
 * batch's key span exceeds 2^20 or a later batch's keys leave the span the closed form can hold),
 * "bulk_min" / "bulk_chunk" (sm_input_send_columns: events from which a send goes to the device directly, events
 * per uploaded chunk), "pool_words" (first size of an NFA query's overflow pool, words), "keep_outputs" (1 = interleaved device batches
 * keep their ordered output records for sm_app_copy_device_outputs), "nfa_jit" (0 = the NFA interpreter instead of
 * the query-specialised kernel), "output_records" (NFA output record capacity; 0 = automatic). */
int sm_app_set_option(sm_app* app, const char* key, int64_t value);

/* Device-resident batch of ONE stream (columns already in HBM, hipStream given as void*): the device form of a
 * sequence of InputHandler.send(ts, row) calls on that stream. Filter queries and `every e1 -> e2 within T` patterns
 * run on the GPU; the pattern is a streaming receiver: each key's open partials are carried into the next batch
 * (StreamPreStateProcessor's pending list across sends), and a batch that leaves the closed form's premise (event
 * time going back, a condition outside its envelope) hands the query to the general NFA kernel for good. The match
 * tuples stay on the device (sm_app_device_matches); when a StreamCallback / QueryCallback is registered for a query
 * (or the collect dump is on), its outputs are also projected on the device and delivered as Events before the
 * call returns, in reference order, one callback call per input event that produced output
 * (OutputRateLimiter.sendToCallBacks :61 → StreamCallback.receive :65). `ordinals` (int64, may be NULL = base +
 * index) gives each event's global arrival ordinal (multi-GPU shards keep the ordinals of the unsharded stream).
 * hip_stream: the stream the batch was produced on (the call's work is ordered after it); NULL = the library waits
 * for all work on the device first. The same holds for sm_app_process_device_events. */
int sm_app_process_device_batch(sm_app* app, const char* stream_id, size_t n, const int64_t* d_timestamps,
                                const void* const* d_cols, const int64_t* d_ordinals, int64_t ordinal_base,
                                void* hip_stream);
/* Interleaved device batch: event i belongs to stream d_stream_idx[i] (the index of sm_app_stream_schema
 * order = define-stream order); every stream a query reads has the schema of d_cols. Pattern / sequence queries
 * run on the GPU (general NFA kernel, playback timers included); outputs go to the callbacks in reference
 * order before the call returns. Ordinals: d_ordinals[i] if given, else ordinal_base + i. d_stream_idx[i] = -1
 * marks a playback heartbeat (sm_app_advance_time at d_timestamps[i]; no event, no ordinal).
 * "output_events:<query>" (sm_app_get_stat) = output events of the last such batch; "nfa_kernel:<query>" = which NFA
 * kernel ran it (1 = query-specialised, 2 = interpreter, 0 = none yet). */
int sm_app_process_device_events(sm_app* app, size_t n, const int32_t* d_stream_idx, const int64_t* d_timestamps,
                                 const void* const* d_cols, const int64_t* d_ordinals, int64_t ordinal_base,
                                 void* hip_stream);
/* Persistence. sm_app_snapshot flushes staged events, then serialises the app's matching state (partition
 * instances, partial matches with their event chains, pending timers, playback clock, arrival ordinal, string
 * dictionary) into buf and stores its size in *len; with buf == NULL it only reports the size (a non-NULL buf
 * smaller than that fails with SM_E_RUNTIME). sm_app_restore loads such a snapshot into an app created from the
 * same SiddhiQL text (SM_E_RUNTIME, the reference's CannotRestoreSiddhiAppStateException, otherwise); staged
 * events are discarded. */
int sm_app_snapshot(sm_app* app, uint8_t* buf, size_t cap, size_t* len);
int sm_app_restore(sm_app* app, const uint8_t* buf, size_t len);
/* Stable partition of a device batch by owner rank (keys: 4- or 8-byte signed integers, world <= 64). The owner of key
 * k is (hi32(splitmix64_finalizer((uint64_t)(int64_t)k))) mod world, hash-by-key so that structured keys spread.
 * Column c (widths[c] bytes per element: 1, 2, 4 or 8) is copied from d_src[c] to d_dst[c] grouped by owner,
 * arrival order kept within each owner; element i of the output lands at d_dst[c] + i * strides[c] (strides
 * NULL = widths: plain columns; a record size: several columns packed into one record buffer, each field aligned
 * to its width); counts[o] = events for owner o (host array of world entries). The send side of the key
 * exchange before the RCCL all-to-all-v (one packed record per event, siddhi_amd/shard.py). */
int sm_partition_by_owner(const void* d_keys, int key_width, size_t n, uint32_t world, int ncols,
                          const int32_t* widths, const int32_t* strides, const void* const* d_src,
                          void* const* d_dst, uint64_t* counts, void* hip_stream);
/* Receive side of the key exchange (siddhi_amd/shard.py exchange_with_ordinals): m packed records of rec_bytes
 * (8..64, a multiple of 8) as the RCCL all-to-all-v delivered them (runs per source rank, in rank order) split into
 * contiguous columns in one pass: field c (offsets[c] bytes into the record, widths[c] = 1, 2, 4 or 8) goes to
 * d_dst[c] (NULL entry or d_dst NULL: not copied). ord_field >= 0 names the 4-byte field holding each record's
 * offset inside its source rank's ingest slice; d_ordinals[i] then = src_first[source of i] + that offset (the
 * global arrival ordinal of the unsharded stream), the source runs given by run_counts (host, nsrc <= 64 entries
 * adding up to m). Replaces the reference's single-JVM junction hand-off (StreamJunction.sendData), which has no
 * exchange; the received columns feed sm_app_process_device_batch / _events with d_ordinals. */
int sm_unpack_records(const void* d_rec, size_t m, int rec_bytes, int ncols, const int32_t* offsets,
                      const int32_t* widths, void* const* d_dst, int ord_field, int nsrc, const uint64_t* run_counts,
                      const int64_t* src_first, int64_t* d_ordinals, void* hip_stream);
/* Receive side of the multi-GPU match return: n match pairs (e2 << 32) | uint32(e1) of global ordinals, every e2
 * in [lo, hi) (this rank's ingest slice), given as the concatenation of per-source runs each in reference order
 * (e2, then e1; one e2's matches all in one run) → d_out (n entries, not aliasing d_pairs) in the reference's
 * global output order for that slice. Concatenating the ranks' outputs in rank order gives the single-process
 * output order. */
int sm_order_matches(const uint64_t* d_pairs, size_t n, int64_t lo, int64_t hi, uint64_t* d_out, void* hip_stream);
/* Multi-GPU playback (@app:playback partitioned apps, siddhi_amd/shard.py merge_heartbeats): a rank's received
 * events (n; global ordinals d_ord ascending; stream index, event time and ncols columns of 4 or 8 bytes) merged
 * in ordinal order with the global clock-advance points (m; ordinals d_tick_ord ascending, clock d_tick_ts), a point
 * at an ordinal this rank holds dropped: the playback clock is global (StreamJunction.sendData :232-237) while a rank
 * holds only its keys' events, so it replays the other ranks' clock advances as heartbeats (stream index -1, zero
 * attributes; its ordinal entry holds the ordinal of the event that advanced the clock, the trigger of the timers the
 * heartbeat fires, see sm_app_copy_device_outputs). Outputs hold n + m entries; *n_out = merged length. */
int sm_merge_heartbeats(size_t n, const int64_t* d_ord, const int32_t* d_sid, const int64_t* d_ts, int ncols,
                        const int32_t* widths, const void* const* d_src, size_t m, const int64_t* d_tick_ord,
                        const int64_t* d_tick_ts, int32_t* d_sid_out, int64_t* d_ts_out, int64_t* d_ord_out,
                        void* const* d_dst, size_t* n_out, void* hip_stream);
/* The output records of the last sm_app_process_device_events batch of a query (needs option "keep_outputs" = 1 set
 * before the batch), in the reference's delivery order: each record is *stride bytes, an sm_out_rec followed by the
 * select values (nsel sm_dval) and the events' ordinals (int64), with pos = the ordinal of the output's trigger: the
 * event whose processing emitted it, or for a timer the event that advanced the playback clock (a heartbeat's ordinal
 * entry). *n = records; with d_dst == NULL only *n and *stride are set. The multi-GPU merge of config 5 sends each
 * record to the rank whose ingest slice holds its trigger and orders the received runs with sm_order_outputs. */
typedef struct sm_out_rec {
  int64_t pos;     /* trigger ordinal */
  int64_t time;    /* timer phase: the clock step; data phase: 0 (or a broadcast copy's rank + 1) */
  int64_t create;  /* ordinal of the event that created the output's partition instance, -1 outside partitions */
  int64_t ts;      /* output event timestamp */
  int32_t phase;   /* 0 = fired by the clock advance before the trigger's own processing, 1 = the trigger's */
  int32_t query;   /* query order in the app */
  int32_t sched;
  int32_t seq;     /* emission order within the instance */
  int32_t key;     /* key slot (diagnostic, differs between apps) */
  int32_t pad;
} sm_out_rec;
int sm_app_copy_device_outputs(sm_app* app, const char* query_name, void* d_dst, size_t cap_bytes, size_t* n,
                               size_t* stride, void* hip_stream);
/* Multi-GPU merge of output records (sm_app_copy_device_outputs layout, n of stride bytes): a concatenation of runs,
 * each in delivery order, into the reference's delivery order (QueryCallback / StreamCallback order of one JVM):
 * by trigger ordinal and phase, then for timer outputs by clock step and instance creation ordinal (the scheduler
 * listeners' registration order, core/util/timestamp/EventTimeBasedMillisTimestampGenerator.java:99-116,
 * core/partition/PartitionRuntime.java:256-309), records equal in all of these keeping their run order. d_out must
 * not alias d_recs. */
int sm_order_outputs(const void* d_recs, size_t n, size_t stride, void* d_out, void* hip_stream);
/* Match tuples of the last device batch for a query: n pairs (e1, e2) of ordinals relative to the batch's
 * ordinal_base, uint32[2*n] in device memory, in reference output order (e2 ordinal, then e1 ordinal). */
int sm_app_device_matches(sm_app* app, const char* query_name, const uint32_t** d_pairs, size_t* n);
/* The same tuples (or a filter query's kept rows, uint32 each) copied into a caller-owned device buffer of
 * cap_bytes on hip_stream (asynchronous); *n = tuples. Lets a caller hand them to its own collectives. */
int sm_app_copy_device_matches(sm_app* app, const char* query_name, void* d_dst, size_t cap_bytes, size_t* n,
                               void* hip_stream);
/* One value of a device-side output event: INT / LONG / BOOL / STRING (dictionary id) in i, FLOAT / DOUBLE (FLOAT
 * widened) in d. */
typedef struct sm_dval {
  union {
    int64_t i;
    double d;
  };
  int32_t is_null;
  int32_t pad;
} sm_dval;
/* QuerySelector.processNoGroupBy (query/selector/QuerySelector.java:124-167) on the device for the outputs of the
 * last device batch of a query: output k (the k-th tuple of sm_app_device_matches, or a filter query's k-th kept
 * row) gets its select list in d_values[k * nsel .. k * nsel + nsel) and its timestamp (the last event's time,
 * StateEvent.timestamp) in d_ts[k] (d_ts may be NULL). An e1 carried from an earlier batch is read from the carried
 * partial; a batch the NFA kernel took returns the values the kernel evaluated. With d_values == NULL only *n and
 * *nsel are set. The batch's columns, event times and ordinals are read again: call it before freeing them.
 * SM_E_UNSUPPORTED when the query's last outputs came from host-API events (they reach the callbacks). */
int sm_app_device_project(sm_app* app, const char* query_name, sm_dval* d_values, size_t cap_values, int64_t* d_ts,
                          size_t* n, int32_t* nsel, void* hip_stream);
/* Diagnostics of the last device batch: "fast_path:<query>" = the device path it took: patterns 3 = bucket-stack
 * kernels, 2 = sort / walk kernels, 1 = general closed form (option fast_general), 5 = general NFA kernel (hand-over);
 * filter queries 3 = filter interpreter, 4 = typed conjunction. "output_events:<query>" = its output count.
 * "kernel_ms:<label>" / "kernel_calls:<label>" and "fast_ms:group" / "fast_ms:walk" / "fast_ms:order" (per-kernel
 * and phase times in ms; need the "fast_timing" option). "nfa_state:<query>" = 1 once a closed-form pattern's matching
 * state is held by the general NFA kernel for good: host events it could not take on the closed form (a null value,
 * a chained or broadcast app) or a device batch outside its premise (event time decreasing) handed its carried
 * partials over, and every later batch of that query runs on the NFA kernel (same results, the NFA's speed).
 * NFA overflow pool of a pattern query: "pool_words:<query>", "pool_used:<query>", "pool_compactions:<query>",
 * "pool_refused:<query>" (batches in which a key's promotion did not fit; the pool is grown for it after the batch). */
int sm_app_get_stat(sm_app* app, const char* key, double* out);

#ifdef __cplusplus
}
#endif
#endif
