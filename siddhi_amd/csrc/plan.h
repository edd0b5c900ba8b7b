// Device-visible query plan: compact POD tables the host compiler (compiler.cpp) lowers a SiddhiQL query
// into, and the HIP kernels (kernels.hip) interpret. Layout rules: plain structs of int32/int64, no
// pointers inside (tables are packed into one device buffer per query and addressed by offsets).
//
//   Predicate / projection bytecode  ← ExpressionParser (core/util/parser/ExpressionParser.java:231-1371)
//   DPre / DPost                     ← *PreStateProcessor / *PostStateProcessor (core/query/input/stream/state)
//   DInner                           ← runtime/*InnerStateRuntime.java (reset/update recursion of sequences)
//   DReceiver                        ← Pattern/Sequence{Single,Multi}ProcessStreamReceiver
#pragma once
#include <stdint.h>

namespace sm {

// ---- value types (same numbering as sql::AttrType / sm_value.type)
enum : int32_t { T_INT = 0, T_LONG = 1, T_FLOAT = 2, T_DOUBLE = 3, T_STRING = 4, T_BOOL = 5 };

// A device value: integral kinds (INT/LONG/BOOL/STRING dictionary id) in i, FLOAT/DOUBLE in d.
struct DVal {
  union {
    int64_t i;
    double d;
  };
  int32_t null;
  int32_t pad;
};

// ---- bytecode
enum : int32_t {
  OP_CONST = 0,  // push consts[a]
  OP_COL = 1,    // stream context: push column a (type t0)
  OP_VAR = 2,    // state context: push attribute c of the event at (slot a, chain index b) (type t0)
  OP_CMP = 3,    // pop r, l; push l <sub> r compared as type t0 (CT_*); null → false (NE: null → true)
  OP_MATH = 4,   // pop r, l; push l <sub> r computed in result type t0
  OP_AND = 5,
  OP_OR = 6,
  OP_NOT = 7,
  OP_ISNULL = 8,
  OP_TS = 9,     // push the event/state timestamp (internal)
};
enum : int32_t { CMP_EQ = 0, CMP_NE = 1, CMP_LT = 2, CMP_LE = 3, CMP_GT = 4, CMP_GE = 5 };
enum : int32_t { M_ADD = 0, M_SUB = 1, M_MUL = 2, M_DIV = 3, M_MOD = 4 };
// comparison domains (Java binary numeric promotion, plus the double-domain Equal/NotEqual Float×Long
// executors: compare/equal/EqualCompareConditionExpressionExecutorFloatLong.java)
enum : int32_t { CT_INT = 0, CT_LONG = 1, CT_FLOAT = 2, CT_DOUBLE = 3, CT_ID = 4 };

struct Instr {
  int32_t op;
  int32_t sub;  // CMP / MATH operator
  int32_t t0;   // result / compare type
  int32_t t1;   // OP_CMP: left operand type; OP_MATH: left type
  int32_t t2;   // OP_CMP / OP_MATH: right operand type
  int32_t a, b, c;
};

constexpr int kMaxStack = 8;  // device operand stack (per lane, scratch): compiler rejects deeper expressions
constexpr int kMaxSlots = 16;
constexpr int kMaxProcs = 8;

// ---- NFA tables
enum : int32_t { PK_STREAM = 0, PK_COUNT = 1, PK_LOGICAL = 2, PK_ABSENT_STREAM = 3, PK_ABSENT_LOGICAL = 4 };
enum : int32_t { IK_STREAM = 0, IK_NEXT = 1, IK_EVERY = 2, IK_LOGICAL = 3, IK_COUNT = 4 };
enum : int32_t { LT_AND = 0, LT_OR = 1 };

struct DWithin {
  int64_t t;
  int32_t ids[2];  // state ids; -1 = ANY (StateEvent.timestamp)
  int32_t n;
  int32_t pad;
};

struct DPre {
  int32_t kind, stateId, sequence, isStart;
  int32_t withinOff, withinCnt;
  int32_t progOff, progLen;  // filter program (AND of the state's filters); progLen 0 = pass
  int32_t post, thisLast, partner;
  int32_t minCount, maxCount, ltype;
  int32_t sched;             // scheduler index or -1
  int32_t ksOff;             // first of its per-key state words (kPreWords, or kPreWordsAbsent for an absent pre)
  int32_t trialCur;          // 1: the filter reads its own state's chain only at CURRENT (the incoming event), so a
                             // partial can be tried against the incoming event without adding it to the chain
  // operand cache of the pending / newAndEvery list nodes (round 5): the filter's loads of other states (at most 2
  // distinct (state, index, attribute) operands, each of an earlier single-event stream state, whose chain no longer
  // changes once the partial reaches this state) are evaluated when a partial joins the list and kept in its node, so
  // a trial reads the node only. cacheIns[k] = index into the code of a load of operand k; ncache 0 = none.
  int32_t ncache;
  int32_t cacheIns[2];
  int64_t waitingTime;       // absent: 'for' time, -1 when absent (logical 'and not X' without for)
};

struct DPost {
  int32_t kind, stateId, nextPre, nextEveryPre, thisPre, hasNext, callbackPre, ltype, partnerPre, partnerPost;
  int32_t minCount, maxCount;
};

struct DInner {
  int32_t kind, first, last, a, b;
};

struct DReceiver {
  int32_t stream;  // app stream index
  int32_t multi;
  int32_t nproc;   // processors in processing order (eventSequence applied)
  int32_t procs[kMaxProcs];
  int32_t nstate;  // addStatefulProcessor order
  int32_t stateProcs[kMaxProcs];
  int32_t hasQuerySelector;
};

// Per-query device plan header; all arrays follow in one blob at the given word offsets.
struct DQuery {
  int32_t kind;         // 0 = single-stream filter query, 1 = pattern, 2 = sequence
  int32_t query_order;  // position in the app (output interleaving)
  int32_t partitioned;
  int32_t nslots;       // state slots (meta stream events)
  int32_t npre, npost, ninner, nrecv, nsched, nwithin;
  int32_t root_inner;
  // StateStreamRuntime.resetAndUpdate (sequences, StateStreamRuntime.java:90-93) flattened at compile time:
  // the pre processors inner reset() then update() visit, in the order the inner-runtime tree visits them
  int32_t nreset, nupdate;
  int32_t reset_seq[2 * kMaxSlots], update_seq[2 * kMaxSlots];
  int32_t nsel;         // output attributes
  int32_t nrefs;        // variable references written per output: the select's (parity tuples), then for a
                        // closed-form query two hidden ones, (e1, e2), read by the NFA fallback of device batches
  int32_t nrefs_vis;    // the select's references (the first nrefs_vis)
  int32_t nconst;
  int32_t slot_nattr[kMaxSlots];   // attributes stored per chain node of each slot (its stream's width)
  int32_t slot_stream[kMaxSlots];  // app stream index of each slot
  int32_t node_words;              // words of a chain node (3 + max attrs)
  int32_t rec_words;               // words of a run record (2 + ceil(nslots/2))
  // offsets (in bytes from the blob start)
  int32_t off_pre, off_post, off_inner, off_recv, off_within, off_code, off_const;
  int32_t off_sel;      // nsel x (progOff, progLen, type)
  int32_t off_refs;     // nrefs x (slot, idx)
  // single-stream query
  int32_t stream;       // input stream (kind 0)
  int32_t filt_off, filt_len;
  // per-key state layout (words of int64 per key)
  int32_t ks_words;
  int32_t ks_pre;       // per pre (DPre.ksOff): pendHead|pendTail, newHead|newTail, flags, the returned list of
                        // processAndReturn; an absent pre also lastArrival (only absent processors read it)
  int32_t ks_post;      // one word: bit o = isEventReturned of post processor o
  int32_t ks_sched;     // per scheduler: 2 + kSchedCap words (head, count, ring)
  int32_t ks_misc;      // create position, heap bump, semispace, state-id counter
  // state query: having condition (QuerySelector.java:138-139) over the run record, output attributes
  // substituted by their select programs; having_len 0 = none. A single-stream query ANDs it into filt.
  int32_t having_off, having_len;
};
constexpr int kSchedCap = 32;
constexpr int kPreWords = 4;
constexpr int kPreWordsAbsent = 5;

// pre flags (bit set in the flags word)
enum : int64_t { F_STATE_CHANGED = 1, F_INITIALIZED = 2, F_SUCCESS = 4, F_START_RESET = 8, F_ACTIVE = 16 };

// ---- output record emitted by the NFA interpreter (host orders by (pos, phase, time, group, create,
// query, sched, seq) = the reference's callback order)
struct OutRec {
  int64_t pos;       // batch position of the triggering event / clock-advance point
  int64_t time;      // timer phase: step time; data phase: 0
  int64_t create;    // partition key creation position (global ordinal), -1 non-partitioned
  int64_t ts;        // output event timestamp (StateEvent.timestamp)
  int32_t phase;     // 0 = timer (before the data event), 1 = data
  int32_t query;     // query order
  int32_t sched;     // scheduler index (timer phase)
  int32_t seq;       // emission counter within the lane
  int32_t key;       // key slot (diagnostics)
  int32_t pad;
  // followed by nsel DVal values and nrefs int64 ordinals (record stride set by the host)
};

}  // namespace sm
