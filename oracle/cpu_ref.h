/* CPU oracle for the Siddhi pattern/sequence hot path — TEST INFRASTRUCTURE ONLY.
 *
 * A literal C++ restatement of the reference's Java object graph (StreamPreStateProcessor & siblings,
 * receivers, FilterProcessor, typed compare executors, partition cloning, playback timers). Used by
 * tests/ (parity checker), __graft_entry__.smoke() and bench.py's cpu_baseline leg ONLY. The product
 * (libsiddhi_amd.so) never links or calls this library.
 *
 * Pinned by the reference's own known-answer tests, transcribed to explicit timestamps in
 * tests/golden/kat_*.json (see tests/test_oracle_kat.py). The Java engine itself cannot run here
 * (no JVM).
 */
#ifndef SIDDHI_CPU_REF_H
#define SIDDHI_CPU_REF_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct cr_app cr_app;

/* same layout as sm_value in include/siddhi_amd.h */
typedef struct cr_value {
  int32_t type; /* 0 INT 1 LONG 2 FLOAT 3 DOUBLE 4 STRING 5 BOOL */
  int32_t is_null;
  int64_t i;    /* INT / LONG / BOOL */
  double d;     /* FLOAT / DOUBLE */
  const char* s;/* STRING (borrowed for the call) */
} cr_value;

/* status codes: 0 ok, 1 parse, 2 validation, 3 unsupported, 4 type, 6 runtime */
int cr_app_create(const char* siddhiql, cr_app** out, char* err, size_t errlen);
void cr_app_destroy(cr_app* app);
int cr_app_start(cr_app* app);
int cr_stream_index(cr_app* app, const char* stream_id);
int cr_send(cr_app* app, int stream_index, int64_t ts, const cr_value* row, char* err, size_t errlen);
/* Fast columnar path for the CPU baseline: n events of one stream; cols[k] points to the k-th
 * attribute column (int32_t*, int64_t*, float*, double*; strings unsupported here). */
int cr_send_columns(cr_app* app, int stream_index, size_t n, const int64_t* ts, const void* const* cols,
                    char* err, size_t errlen);
/* interleaved batch over streams sharing one schema: event i -> stream stream_idx[i];
 * stream_idx[i] == -1 is a playback heartbeat at ts[i] (as cr_advance_time; its columns are not read) */
int cr_send_interleaved(cr_app* app, size_t n, const int32_t* stream_idx, const int64_t* ts, const void* const* cols,
                        char* err, size_t errlen);
/* cr_send_interleaved with given arrival ordinals: event i gets ordinal ord[i] (a key-sharded rank's events keep the
 * ordinals of the unsharded stream); a heartbeat's ord[i] is the ordinal of the event that advanced the global clock
 * there (the trigger of the timers it fires, see cr_output_order). */
int cr_send_interleaved_ord(cr_app* app, size_t n, const int32_t* stream_idx, const int64_t* ts, const int64_t* ord,
                            const void* const* cols, char* err, size_t errlen);
/* The place of each collected output of a stream in the reference's emission order, 4 int64 per output: the ordinal
 * of its trigger (the input event whose processing emitted it; for a timer, the event whose arrival advanced the
 * playback clock), its phase (0 = a timer fired by that clock advance, before the event itself is processed; 1 = the
 * event's own processing), the clock value of the advance (phase 0; else 0) and the ordinal of the event that created
 * its partition instance (-1 outside partitions). Test infrastructure for the multi-GPU output merge. Returns the
 * output count; writes min(count, cap) entries. */
size_t cr_output_order(cr_app* app, const char* stream_id, int64_t* out, size_t cap);
/* Outputs collected since creation, as JSON text:
 * {"streams": {"<id>": [[ts, [values...], [refs...]], ...]},
 *  "queries": {"<name>": [[ts, [[values...], ...]], ...]}}
 * refs = global arrival ordinals of the events at the select list's variable positions (-1 = null).
 * Returns required size (excluding NUL); writes when buf large enough. */
size_t cr_dump_outputs(cr_app* app, char* buf, size_t len);
/* Playback heartbeat: advance the event-time clock without an event (the reference's
 * @app:playback(idle.time, increment) TimeInjector path, EventTimeBasedMillisTimestampGenerator.java:99). */
int cr_advance_time(cr_app* app, int64_t ts, char* err, size_t errlen);
/* Wall-clock emulation for absent tests written against the wall-clock scheduler: advances the clock
 * through every due timer time (in time order) up to ts. */
int cr_advance_wallclock(cr_app* app, int64_t ts, char* err, size_t errlen);
/* number of output events emitted on a stream (cheap, for benchmarks) */
int64_t cr_output_count(cr_app* app, const char* stream_id);
void cr_clear_outputs(cr_app* app);
/* When 0, outputs are counted but not materialised (baseline timing). Default 1. */
void cr_set_collect(cr_app* app, int collect);

#ifdef __cplusplus
}
#endif
#endif
