// NFA interpreter implementation shared by the HIP kernel (nfa.hip) and the CPU debug build of the same
// device code (tests/native/nfa_host_harness.cpp, compiled with g++ and the shims in hd_shim.h).
#pragma once
// General pattern/sequence NFA interpreter for gfx950: one lane per partition key (one lane in total for a
// non-partitioned query), stepping that key's events in arrival order against the key's persistent
// partial-match state in HBM.
//
// The per-key state is a small copying-collected heap of
//   run records  (StateEvent, core/event/state/StateEvent.java:53)      — shared by reference
//   chain nodes  (StreamEvent copies, StreamEventCloner.java:46-63)       — shared by shallow copies
//   list nodes   (pending / newAndEvery LinkedLists of each pre-state processor)
// plus per-processor flags and FIFO timer queues (util/Scheduler.java:44). Every function below restates
// the reference method named in its comment; the CPU oracle (oracle/cpu_ref.cpp) restates the same methods
// independently over an object graph.
#include "nfa.h"
#include "expr.h"

namespace sm {
namespace {

constexpr int K_REC = 1, K_NODE = 2, K_LNODE = 3, K_LNODE4 = 4, K_FWD = 0xFF;
// words of a heap object of kind k (K_LNODE4: a list node with its operand cache, DPre.ncache)
#define SM_OBJ_WORDS(k) ((k) == K_REC ? PQ->rec_words : (k) == K_NODE ? PQ->node_words : (k) == K_LNODE4 ? 4 : 2)

struct Lane;

// Inlining of the interpreter's large member functions. Each non-inlined call saves the callee's registers to
// per-lane scratch around the call, and at 4 waves per SIMD that scratch outgrows L2 and MALL. deliver and
// pre_process are inlined (scratch 1216 -> 880 B per lane, config-5 NFA kernel 81.2 -> 75.8 ms); also inlining
// fire_all (1040 B, 79.5 ms) or addState (1608 B, 335 VGPR spills) was worse. SM_NFA_CALL_DELIVER /
// SM_NFA_CALL_PRE restore the calls, SM_NFA_INLINE_FIRE / SM_NFA_INLINE_ADD inline the others (A/B builds).
// SM_NFA_INLINE_SMALL forces the small list / slot helpers inline: 992 B scratch, 293 VGPR spills, 76.2 -> 82.1 ms.
#if defined(__HIPCC__) || defined(__HIP__)
#define SM_NFA_ALWAYS_INLINE __attribute__((always_inline))
#else
#define SM_NFA_ALWAYS_INLINE
#endif
#ifndef SM_NFA_CALL_DELIVER
#define SM_INL_DELIVER SM_NFA_ALWAYS_INLINE
#else
#define SM_INL_DELIVER
#endif
#ifndef SM_NFA_CALL_PRE
#define SM_INL_PRE SM_NFA_ALWAYS_INLINE
#else
#define SM_INL_PRE
#endif
#ifdef SM_NFA_INLINE_PAR
#define SM_INL_PAR SM_NFA_ALWAYS_INLINE
#else
#define SM_INL_PAR
#endif
#ifdef SM_NFA_INLINE_SMALL
#define SM_INL_SMALL SM_NFA_ALWAYS_INLINE
#else
#define SM_INL_SMALL
#endif
#ifdef SM_NFA_INLINE_ADD
#define SM_INL_ADD SM_NFA_ALWAYS_INLINE
#else
#define SM_INL_ADD
#endif
#ifdef SM_NFA_INLINE_FIRE
#define SM_INL_FIRE SM_NFA_ALWAYS_INLINE
#else
#define SM_INL_FIRE
#endif

// Plan tables. The interpreter reads the plan from a device buffer (one build serves every query). A JIT build
// (SM_NFA_JIT, nfa_jit.cpp) compiles this file once per query plan with the plan as a constant array
// (sm::kPlanBlob): every PQ->field and table entry is then a compile-time constant, the plan's loops and kind
// switches fold away and the filter / projection programs become straight-line code.
#ifdef SM_NFA_JIT
#define PQ ((const DQuery*)::sm::kPlanBlob)
#define PPRE ((const DPre*)(::sm::kPlanBlob + PQ->off_pre))
#define PPOST ((const DPost*)(::sm::kPlanBlob + PQ->off_post))
#define PRECV ((const DReceiver*)(::sm::kPlanBlob + PQ->off_recv))
#define PWITHIN ((const DWithin*)(::sm::kPlanBlob + PQ->off_within))
#define PCODE ((const Instr*)(::sm::kPlanBlob + PQ->off_code))
#define PCONSTS ((const DVal*)(::sm::kPlanBlob + PQ->off_const))
#define PSEL ((const int32_t*)(::sm::kPlanBlob + PQ->off_sel))
#define PREFS ((const int32_t*)(::sm::kPlanBlob + PQ->off_refs))
#endif

// SM_NFA_JIT_INLINE_ALL (JIT A/B): every member function on the event path inline into the kernel
#ifdef SM_NFA_JIT_INLINE_ALL
#define SM_JIT_INL SM_NFA_ALWAYS_INLINE
#else
#define SM_JIT_INL
#endif

constexpr int kNfaLdsMisc = 3;  // misc words staged: 1..3 (bump, space, id counter); create (0, read per output) and
                                // initialised (4, read once) stay in HBM

struct StateLoader {  // OP_VAR loads for a run record
  const Lane* L;
  int rec;
  __device__ StackVal var(const Instr& in) const;
};
// A state's filter tried before the incoming event joins the partial (DPre.trialCur): loads of the state's own slot
// (always at CURRENT, which the incoming event would become) read the event's LaneEv record; other slots as above.
struct TrialLoader {
  const Lane* L;
  int rec;
  int sid;
  const int64_t* evr;
  __device__ StackVal var(const Instr& in) const;
};
// A trial whose other-state operands come from the list node's cache (DPre.ncache, K_LNODE4): the partial's run record
// and chain nodes are not read at all (one read of the node per rejected partial)
struct CachedTrialLoader {
  const Lane* L;
  int32_t ln;
  int sid;
  int pre;
  const int64_t* evr;
  __device__ StackVal var(const Instr& in) const;
};

// The words of one lane inside a lane-interleaved allocation (structure of arrays across lanes): word w of lane k
// lives at base[w * lanes + k]. The 64 lanes of a wave that touch the same per-key state word (list heads,
// flags, timer queues: fixed offsets) then share cache lines instead of each pulling its own line.
// stride 1 = the plain key-major layout (the heap).
#ifdef SM_COUNT_ACCESS
// [0] key-state word accesses, [1] heap word accesses, [2] words allocated, [3] words copied by collections
// (gc + promote), [4] collections, [5] events delivered, [6] run records allocated, [7] chain nodes allocated
extern int64_t g_access[8];
// per phase of the lane's work (SM_PHASE): key-state / heap word accesses ([0][ph] / [1][ph])
extern int g_phase;
extern int64_t g_phase_acc[2][16];
struct PhaseScope {
  int prev;
  explicit PhaseScope(int ph) : prev(g_phase) { g_phase = ph; }
  ~PhaseScope() { g_phase = prev; }
};
#define SM_COUNT(i, v) (::sm::g_access[i] += (v))
#define SM_PHASE(ph) ::sm::PhaseScope sm_phase_scope_(ph)
#else
#define SM_COUNT(i, v) ((void)0)
#define SM_PHASE(ph) ((void)0)
#endif
struct LaneWords {
  int64_t* p;      // &base[lane]
  int64_t stride;  // lanes per word row
#ifdef SM_COUNT_ACCESS  // CPU debug build only (tests/native): per-event access mix of key-state words vs heap words
  int64_t& operator[](int64_t w) const {
    ++g_access[stride == 1 ? 1 : 0];
    ++g_phase_acc[stride == 1 ? 1 : 0][g_phase];
    return p[w * stride];
  }
#else
  __device__ __forceinline__ int64_t& operator[](int64_t w) const { return p[w * stride]; }
#endif
  __device__ __forceinline__ LaneWords at(int64_t w) const { return {p + w * stride, stride}; }
};

struct Lane {
  // plan
#ifndef SM_NFA_JIT
  const DQuery* PQ;
  const DPre* PPRE;
  const DPost* PPOST;
  const DReceiver* PRECV;
  const DWithin* PWITHIN;
  const Instr* PCODE;
  const DVal* PCONSTS;
  const int32_t* PSEL;
  const int32_t* PREFS;
#endif
  // state
  LaneWords ks;   // per-key state words: list heads, flags, post words, misc (LDS-staged under SM_NFA_LDS)
  LaneWords ksh;  // the same key's words in HBM (timer queues always live there)
  LaneWords heap;
  int32_t half;  // words per semispace
  // batch
  const NfaBatch* b;
  // output
  int32_t key;
  int64_t pos, time;
  int32_t phase, sched;
  int32_t seq;
  mutable int32_t err;  // (mutable: the const loaders of a filter report a broken plan invariant too)
  int64_t clock;  // EventTimeBasedMillisTimestampGenerator.currentTime() as seen by this lane
  // the earliest head of the lane's timer queues (min_head), INT64_MAX when all are empty: kept in a register, so the
  // per-event "is a timer due" check reads no timer-queue word (they live in HBM); set at lane start, lowered by
  // notifyAt when it gives an empty queue its head, recomputed after timers fire (round 5)
  int64_t due;

  // ------------------------------------------------------------ heap
  // misc words: create position, heap bump, semispace, state-id counter, initialised. Staged (SM_NFA_LDS), they sit
  // right after the post words.
#ifdef SM_NFA_LDS
  __device__ __forceinline__ int64_t& misc(int k) const {
    return (k >= 1 && k <= kNfaLdsMisc) ? ks[PQ->ks_sched + k - 1] : ksh[PQ->ks_misc + k];
  }
#else
  __device__ int64_t& misc(int k) const { return ks[PQ->ks_misc + k]; }
#endif
  __device__ int32_t alloc(int words) {
    int64_t space = misc(2);
    int64_t end = (space + 1) * half;
    int64_t bump = misc(1);
    if (bump + words > end) {
      err |= NFA_ERR_ARENA;
      return 2 * half;  // dummy region (writes harmless; lane aborts at the next safe point)
    }
    misc(1) = bump + words;
    SM_COUNT(2, words);
    return (int32_t)bump;
  }
  __device__ int kind_of(int32_t o) const { return (int)(heap[o] & 0xFF); }
  __device__ int32_t hi(int32_t o) const { return (int32_t)(heap[o] >> 32); }
  __device__ void set_hi(int32_t o, int32_t v) const {
    heap[o] = (heap[o] & 0xFFFFFFFFll) | ((int64_t)(uint32_t)v << 32);
  }
  // run record
  __device__ int64_t& rts(int32_t r) const { return heap[r + 1]; }
  __device__ int32_t slot(int32_t r, int s) const {
    int64_t w = heap[r + 2 + (s >> 1)];
    return (s & 1) ? (int32_t)(w >> 32) : (int32_t)w;
  }
  SM_INL_SMALL __device__ void set_slot(int32_t r, int s, int32_t v) const {
    int64_t& w = heap[r + 2 + (s >> 1)];
    if (s & 1) w = (w & 0xFFFFFFFFll) | ((int64_t)(uint32_t)v << 32);
    else w = (w & ~0xFFFFFFFFll) | (int64_t)(uint32_t)v;
  }
  SM_JIT_INL __device__ int32_t new_rec() {
    int32_t r = alloc(PQ->rec_words);
    SM_COUNT(6, 1);
    heap[r] = K_REC;
    heap[r + 1] = -1;  // StateEvent.timestamp = -1
    for (int k = 2; k < PQ->rec_words; ++k) heap[r + k] = -1;  // all slots null (two -1 halves)
    return r;
  }
  // StateEventCloner.copyStateEvent :46-57 (shallow)
  SM_JIT_INL __device__ int32_t copy_rec(int32_t src) {
    int32_t r = alloc(PQ->rec_words);
    SM_COUNT(6, 1);
    for (int k = 0; k < PQ->rec_words; ++k) heap[r + k] = heap[src + k];
    return r;
  }
  // chain node
  __device__ int32_t nnext(int32_t n) const { return hi(n); }
  __device__ void set_nnext(int32_t n, int32_t v) const { set_hi(n, v); }
  __device__ int64_t nts(int32_t n) const { return heap[n + 1]; }
  __device__ int64_t nord(int32_t n) const { return heap[n + 2]; }
  SM_INL_SMALL __device__ int32_t copy_node(int32_t src) {  // StreamEventCloner.copyStreamEvent: next = null
    int32_t n = alloc(PQ->node_words);
    SM_COUNT(7, 1);
    for (int k = 1; k < PQ->node_words; ++k) heap[n + k] = heap[src + k];
    heap[n] = K_NODE | ((int64_t)(uint32_t)-1 << 32);
    return n;
  }
  SM_JIT_INL __device__ int32_t empty_node() {  // streamEventPool.borrowEvent(): ts -1, null data
    int32_t n = alloc(PQ->node_words);
    SM_COUNT(7, 1);
    heap[n] = K_NODE | ((int64_t)(uint32_t)-1 << 32);
    heap[n + 1] = -1;
    heap[n + 2] = -1;
    heap[n + 3] = -1;  // every attribute null
    for (int k = 4; k < PQ->node_words; ++k) heap[n + k] = 0;
    return n;
  }
  // StreamEventCloner.copyStreamEvent of the incoming event: the copy is made straight from the node image the
  // lane-events pass built (LaneEv, nfa.h). The event itself is never materialised in the heap: every use of it
  // in processAndReturn is such a copy, so an event no pending partial takes allocates nothing.
  SM_INL_SMALL __device__ int32_t copy_event(const int64_t* __restrict__ r) {
    int32_t n = alloc(PQ->node_words);
    SM_COUNT(7, 1);
    heap[n] = K_NODE | ((int64_t)(uint32_t)-1 << 32);
    for (int w = 1; w < PQ->node_words; ++w) heap[n + w] = le_node(*b, r, w);
    return n;
  }
  // StateEvent.addEvent :212-222; returns the chain's length afterwards (its last node is n), which the count post
  // processor that runs right after it would otherwise walk the chain again for (post_process: chain_n)
  SM_INL_SMALL __device__ int add_event(int32_t r, int s, int32_t n) {
    int32_t a = slot(r, s);
    if (a < 0) {
      set_slot(r, s, n);
      return 1;
    }
    int len = 2;
    while (nnext(a) >= 0) {
      a = nnext(a);
      ++len;
    }
    set_nnext(a, n);
    return len;
  }
  // StateEvent.removeLastEvent :224-235
  SM_INL_SMALL __device__ void remove_last_event(int32_t r, int s) {
    int32_t a = slot(r, s);
    if (a >= 0) {
      while (nnext(a) >= 0) {
        if (nnext(nnext(a)) < 0) { set_nnext(a, -1); return; }
        a = nnext(a);
      }
      set_slot(r, s, -1);
    }
  }
  // StateEvent.getStreamEvent(int[] position) :138-182
  SM_JIT_INL __device__ int32_t at(int32_t r, int chain, int idx) const {
    int32_t e = slot(r, chain);
    if (e < 0) return -1;
    if (idx >= 0) {
      for (int k = 1; k <= idx; ++k) {
        e = nnext(e);
        if (e < 0) return -1;
      }
    } else if (idx == -1) {
      while (nnext(e) >= 0) e = nnext(e);
    } else if (idx == -2) {
      if (nnext(e) < 0) return -1;
      while (nnext(nnext(e)) >= 0) e = nnext(e);
    } else {
      int len = 0;
      for (int32_t x = e; x >= 0; x = nnext(x)) ++len;
      int index = len + idx;
      if (index < 0) return -1;
      for (int k = 0; k < index; ++k) e = nnext(e);
    }
    return e;
  }

  // ------------------------------------------------------------ lists (LinkedList<StateEvent>)
  // which: 0 pending list, 1 newAndEvery list, 2 flags, 3 the list processAndReturn returns; absent pres only:
  // 4 lastArrival
  __device__ int64_t& lw(int p, int which) const { return ks[PPRE[p].ksOff + which]; }
  __device__ int32_t lhead(int p, int w) const { return (int32_t)lw(p, w); }
  __device__ int32_t ltail(int p, int w) const { return (int32_t)(lw(p, w) >> 32); }
  __device__ void lset(int p, int w, int32_t h, int32_t t) const {
    lw(p, w) = (int64_t)(uint32_t)h | ((int64_t)(uint32_t)t << 32);
  }
  __device__ int32_t ln_rec(int32_t ln) const { return hi(ln); }
  __device__ int32_t ln_next(int32_t ln) const { return (int32_t)heap[ln + 1]; }
  __device__ void ln_set_next(int32_t ln, int32_t v) const { heap[ln + 1] = v; }
  __device__ bool lempty(int p, int w) const { return lhead(p, w) < 0; }
  // the trial operands of pre q's filter for run record `rec`, read once when the partial joins q's list (DPre.ncache)
  // into the K_LNODE4 node ln {hdr | nulls << 8, next, v0, v1}; returns the null bits for the header
  __device__ int64_t cache_fill(int q, int32_t ln, int32_t rec) {
    int64_t nb = 0;
    StateLoader ld{this, rec};
    for (int k = 0; k < PPRE[q].ncache; ++k) {
      const StackVal v = ld.var(PCODE[PPRE[q].cacheIns[k]]);
      heap[ln + 2 + k] = v.null ? 0 : v.i;
      if (v.null) nb |= (int64_t)1 << (8 + k);
    }
    return nb;
  }
  // A node of a pre with a cache is K_LNODE4 from the start; its cache is filled when the node moves from the
  // newAndEvery list to the pending list (lsplice, the only way a node reaches the list processAndReturn walks), so
  // the fill has one call site instead of one per inlined append. Between the append and the splice nothing changes
  // the cached states' chains (DPre.ncache).
  SM_INL_SMALL __device__ void lappend(int p, int w, int32_t rec) {
    const bool c4 = w < 2 && PPRE[p].ncache > 0;
    int32_t ln = alloc(c4 ? 4 : 2);
    heap[ln] = (c4 ? K_LNODE4 : K_LNODE) | ((int64_t)(uint32_t)rec << 32);
    heap[ln + 1] = -1;
    int32_t t = ltail(p, w);
    if (t < 0) lset(p, w, ln, ln);
    else {
      ln_set_next(t, ln);
      lset(p, w, lhead(p, w), ln);
    }
  }
  __device__ void lclear(int p, int w) const { lset(p, w, -1, -1); }
  __device__ int lsize(int p, int w) const {
    int n = 0;
    for (int32_t x = lhead(p, w); x >= 0; x = ln_next(x)) ++n;
    return n;
  }
  __device__ void lsplice(int p, int dst, int src) {  // dst.addAll(src); src.clear()
    int32_t sh = lhead(p, src);
    if (sh < 0) return;
    if (dst == 0) {  // newAndEvery -> pending: fill the operand caches of the arriving nodes (lappend)
#ifdef SM_NFA_JIT_INLINE_ALL
#pragma unroll
      for (int q = 0; q < PQ->npre; ++q)
        if (q == p && PPRE[q].ncache > 0)
          for (int32_t x = sh; x >= 0; x = ln_next(x)) heap[x] |= cache_fill(q, x, ln_rec(x));
#else
      if (PPRE[p].ncache > 0)
        for (int32_t x = sh; x >= 0; x = ln_next(x)) heap[x] |= cache_fill(p, x, ln_rec(x));
#endif
    }
    int32_t dt = ltail(p, dst);
    if (dt < 0) lset(p, dst, sh, ltail(p, src));
    else {
      ln_set_next(dt, sh);
      lset(p, dst, lhead(p, dst), ltail(p, src));
    }
    lclear(p, src);
  }
  // iterator.remove(): unlink `cur` whose predecessor is `prev` (-1 = head); returns the successor
  SM_INL_SMALL __device__ int32_t lerase(int p, int w, int32_t prev, int32_t cur) {
    int32_t nx = ln_next(cur);
    int32_t h = lhead(p, w), t = ltail(p, w);
    if (prev < 0) h = nx;
    else ln_set_next(prev, nx);
    if (t == cur) t = prev;
    lset(p, w, h, t);
    return nx;
  }
  SM_INL_SMALL __device__ void lremove_rec(int p, int w, int32_t rec) {  // LinkedList.remove(Object): first occurrence
    int32_t prev = -1;
    for (int32_t x = lhead(p, w); x >= 0; prev = x, x = ln_next(x))
      if (ln_rec(x) == rec) {
        lerase(p, w, prev, x);
        return;
      }
  }

  // ------------------------------------------------------------ flags
  __device__ int64_t& flags(int p) const { return lw(p, 2); }
  __device__ bool fl(int p, int64_t f) const { return (flags(p) & f) != 0; }
  SM_INL_SMALL __device__ void setfl(int p, int64_t f, bool v) const {
    if (v) flags(p) |= f;
    else flags(p) &= ~f;
  }
  __device__ int64_t& lastArrival(int p) const { return lw(p, 4); }
  // isEventReturned of every post processor (StreamPostStateProcessor :74-78): one bit each in one word
  __device__ bool returned(int o) const { return (ks[PQ->ks_post] >> o) & 1; }
  __device__ void set_returned(int o, bool v) const {
    int64_t& w = ks[PQ->ks_post];
    w = v ? (w | (1ll << o)) : (w & ~(1ll << o));
  }

  // ------------------------------------------------------------ timers (Scheduler FIFO)
  __device__ LaneWords sq(int s) const { return ksh.at(PQ->ks_sched + s * (2 + kSchedCap)); }
  SM_JIT_INL __device__ void notifyAt(int s, int64_t t) {  // Scheduler.notifyAt :66-74
    LaneWords S = sq(s);
    const int64_t n = S[1];
    if (n >= kSchedCap) {
      err |= NFA_ERR_TIMERS;
      return;
    }
    S[2 + (S[0] + n) % kSchedCap] = t;
    S[1] = n + 1;
    if (n == 0 && t < due) due = t;  // a new head (FIFO: a later entry never is one)
  }
  __device__ bool qempty(int s) const { return sq(s)[1] == 0; }
  __device__ int64_t qhead(int s) const {
    const LaneWords S = sq(s);
    return S[2 + S[0]];
  }
  __device__ void qpop(int s) const {
    LaneWords S = sq(s);
    S[0] = (S[0] + 1) % kSchedCap;
    S[1]--;
  }

  // ------------------------------------------------------------ evaluation
  SM_JIT_INL __device__ bool filter_pass(int p, int32_t rec) const {
#ifdef SM_NFA_JIT_INLINE_ALL
    // plan-constant dispatch: each pre processor's program is evaluated with a constant length, so it unrolls and
    // its operand stack lives in registers (a dynamic-length evaluation keeps the stack in scratch)
    bool pass = true;
#pragma unroll
    for (int q = 0; q < PQ->npre; ++q)
      if (q == p && PPRE[q].progLen != 0) {
        StateLoader ld{this, rec};
        pass = truthy(eval_prog(PCODE + PPRE[q].progOff, PPRE[q].progLen, PCONSTS, ld));
      }
    return pass;
#else
    const DPre& P = PPRE[p];
    if (P.progLen == 0) return true;
    StateLoader ld{this, rec};
    return truthy(eval_prog(PCODE + P.progOff, P.progLen, PCONSTS, ld));
#endif
  }
  // trial_pass with the other states' operands from the list node's cache (DPre.ncache > 0)
  SM_JIT_INL __device__ bool trial_cached(int p, int32_t ln, const int64_t* evr) const {
#ifdef SM_NFA_JIT_INLINE_ALL
    bool pass = true;
#pragma unroll
    for (int q = 0; q < PQ->npre; ++q)
      if (q == p && PPRE[q].progLen != 0 && PPRE[q].ncache > 0) {  // the only pres that call it
        CachedTrialLoader ld{this, ln, PPRE[q].stateId, q, evr};
        pass = truthy(eval_prog(PCODE + PPRE[q].progOff, PPRE[q].progLen, PCONSTS, ld));
      }
    return pass;
#else
    const DPre& P = PPRE[p];
    if (P.progLen == 0) return true;
    CachedTrialLoader ld{this, ln, P.stateId, p, evr};
    return truthy(eval_prog(PCODE + P.progOff, P.progLen, PCONSTS, ld));
#endif
  }
  // filter_pass for a trialCur state with the incoming event in place of its own slot's CURRENT: nothing is added to
  // the partial, so a partial that fails costs only the loads of the other slots' values
  SM_JIT_INL __device__ bool trial_pass(int p, int32_t rec, const int64_t* evr) const {
#ifdef SM_NFA_JIT_INLINE_ALL
    bool pass = true;
#pragma unroll
    for (int q = 0; q < PQ->npre; ++q)
      if (q == p && PPRE[q].progLen != 0 && PPRE[q].ncache == 0) {  // pres with a cache use trial_cached
        TrialLoader ld{this, rec, PPRE[q].stateId, evr};
        pass = truthy(eval_prog(PCODE + PPRE[q].progOff, PPRE[q].progLen, PCONSTS, ld));
      }
    return pass;
#else
    const DPre& P = PPRE[p];
    if (P.progLen == 0) return true;
    TrialLoader ld{this, rec, P.stateId, evr};
    return truthy(eval_prog(PCODE + P.progOff, P.progLen, PCONSTS, ld));
#endif
  }
  __device__ bool is_absent(int p) const { return PPRE[p].kind == PK_ABSENT_STREAM || PPRE[p].kind == PK_ABSENT_LOGICAL; }

  // StreamPreStateProcessor.isExpired :102-121
  SM_INL_SMALL __device__ bool expired(int p, int32_t rec, int64_t now) {
    const DPre& P = PPRE[p];
    for (int w = 0; w < P.withinCnt; ++w) {
      const DWithin& W = PWITHIN[P.withinOff + w];
      for (int k = 0; k < W.n; ++k) {
        int id = W.ids[k];
        int64_t ref;
        if (id < 0) ref = rts(rec);
        else {
          int32_t se = slot(rec, id);
          if (se < 0) {
            err |= NFA_ERR_NPE;
            return false;
          }
          ref = nts(se);
        }
        int64_t d = ref - now;
        if (d < 0) d = -d;
        if (d > W.t) return true;
      }
    }
    return false;
  }

  // ------------------------------------------------------------ selector (QuerySelector.processNoGroupBy)
  SM_JIT_INL __device__ void emit(int32_t rec) {
    SM_PHASE(12);
    if (PQ->having_len > 0) {  // QuerySelector.processNoGroupBy :138-139: the having condition drops the output
      StateLoader hl{this, rec};
      if (!truthy(eval_prog(PCODE + PQ->having_off, PQ->having_len, PCONSTS, hl))) return;
    }
#if defined(__HIP_DEVICE_COMPILE__)
    // one output-slot claim per wave: the lanes emitting together take consecutive slots (ballot + rank); the
    // records are put in delivery order afterwards (order_outputs), so slot order carries no meaning
    const uint64_t m = __ballot(1);
    const int leader = __ffsll((unsigned long long)m) - 1;
    const uint32_t rank = (uint32_t)__popcll(m & ((1ull << __lane_id()) - 1ull));
    uint32_t first = 0;
    if ((int)__lane_id() == leader) first = atomicAdd(b->out_count, (uint32_t)__popcll(m));
    const uint32_t idx = (uint32_t)__shfl((int)first, leader, 64) + rank;
#else
    uint32_t idx = atomicAdd(b->out_count, 1u);
#endif
    if (idx >= b->out_cap) {
      err |= NFA_ERR_OUTPUT;
      return;
    }
    char* base = (char*)b->out + (size_t)idx * b->out_stride;
    OutRec* o = (OutRec*)base;
    o->pos = pos;
    o->time = time;
    o->create = PQ->partitioned ? misc(0) : -1;
    o->ts = rts(rec);
    o->phase = phase;
    o->query = PQ->query_order;
    o->sched = sched;
    o->seq = seq++;
    o->key = key;
    DVal* vals = (DVal*)(base + sizeof(OutRec));
    StateLoader ld{this, rec};
    SM_EXPR_UNROLL
    for (int k = 0; k < PQ->nsel; ++k) {
      StackVal v = eval_prog(PCODE + PSEL[3 * k], PSEL[3 * k + 1], PCONSTS, ld);
      if (PSEL[3 * k + 2] == T_FLOAT || PSEL[3 * k + 2] == T_DOUBLE) vals[k].d = v.d;
      else vals[k].i = v.i;
      vals[k].null = v.null;
      vals[k].pad = 0;
    }
    int64_t* rf = (int64_t*)(vals + PQ->nsel);
    for (int k = 0; k < PQ->nrefs; ++k) {
      int32_t n = at(rec, PREFS[2 * k], PREFS[2 * k + 1]);
      rf[k] = n >= 0 ? nord(n) : -1;
    }
  }

  // ------------------------------------------------------------ pre-state processors
  // StreamPreStateProcessor.init :165-174
  SM_JIT_INL __device__ void pre_init(int p) {
    const DPre& P = PPRE[p];
    const DPost& TP = PPOST[P.post];
    if (P.isStart && (!fl(p, F_INITIALIZED) || TP.nextEveryPre >= 0 ||
                      (P.sequence && TP.nextPre >= 0 && is_absent(TP.nextPre)))) {
      int32_t r = new_rec();
      misc(3)++;
      addState(p, r);
      setfl(p, F_INITIALIZED, true);
    }
  }

  // addState → (count min 0) processMinCountReached → next.addState / nextEvery.addEveryState is recursive
  // in the reference; here it runs over an explicit LIFO work list (same depth-first order) so the kernel has
  // a static stack.
  SM_INL_ADD __device__ void addState(int p0, int32_t r) {
    enum { ACT_ADD = 0, ACT_MIN = 1, ACT_EVERY = 2 };
    uint16_t work[3 * kMaxSlots + 4];  // (processor index << 2) | action: a small per-lane (scratch) stack
    int sp = 0;
    work[sp++] = (uint16_t)(p0 << 2 | ACT_ADD);
    while (sp > 0) {
      --sp;
      const int a = work[sp] & 3, p = work[sp] >> 2;
      if (a == ACT_EVERY) {
        addEveryState(p, r);
        continue;
      }
      if (a == ACT_MIN) {  // CountPostStateProcessor.processMinCountReached :73-85 (p = post index)
        const DPost& O = PPOST[p];
        if (O.hasNext) {
          setfl(O.thisPre, F_STATE_CHANGED, true);
          set_returned(p, 1);
        }
        if (sp + 2 > 3 * kMaxSlots + 4) {
          err |= NFA_ERR_NPE;
          return;
        }
        if (O.nextEveryPre >= 0) work[sp++] = (uint16_t)(O.nextEveryPre << 2 | ACT_EVERY);
        if (O.nextPre >= 0) work[sp++] = (uint16_t)(O.nextPre << 2 | ACT_ADD);
        continue;
      }
      const DPre& P = PPRE[p];
      switch (P.kind) {
        case PK_STREAM:  // StreamPreStateProcessor.addState :208-221
          if (P.sequence) {
            if (lempty(p, 1)) lappend(p, 1, r);
          } else {
            lappend(p, 1, r);
          }
          break;
        case PK_COUNT:  // CountPreStateProcessor.addState :109-127
          if (P.sequence) {
            if (lempty(p, 1)) lappend(p, 1, r);
          } else {
            lappend(p, 1, r);
          }
          if (P.minCount == 0 && slot(r, P.stateId) < 0) {
            work[sp++] = (uint16_t)(P.post << 2 | ACT_MIN);
          }
          break;
        case PK_LOGICAL:
        case PK_ABSENT_LOGICAL: {  // LogicalPreStateProcessor.addState :62-77 (+ AbsentLogical override)
          if (P.kind == PK_ABSENT_LOGICAL && !fl(p, F_ACTIVE)) break;
          int pt = P.partner;
          if (P.isStart || P.sequence) {
            if (lempty(p, 1)) lappend(p, 1, r);
            if (pt >= 0 && lempty(pt, 1)) lappend(pt, 1, r);
          } else {
            lappend(p, 1, r);
            if (pt >= 0) lappend(pt, 1, r);
          }
          if (P.kind == PK_ABSENT_LOGICAL && !P.isStart && P.waitingTime != -1) {
            notifyAt(P.sched, rts(r) + P.waitingTime);
            if (PPRE[pt].kind == PK_ABSENT_LOGICAL) notifyAt(PPRE[pt].sched, rts(r) + PPRE[pt].waitingTime);
          }
          break;
        }
        default:  // PK_ABSENT_STREAM: AbsentStreamPreStateProcessor.addState :89-108
          if (!fl(p, F_ACTIVE)) break;
          if (P.sequence) {
            lclear(p, 1);
            lappend(p, 1, r);
          } else {
            lappend(p, 1, r);
          }
          if (!P.isStart) notifyAt(P.sched, rts(r) + P.waitingTime);
          break;
      }
    }
  }

  SM_JIT_INL __device__ void addEveryState(int p, int32_t r) {
    const DPre& P = PPRE[p];
    switch (P.kind) {
      case PK_LOGICAL: {  // LogicalPreStateProcessor.addEveryState :80-88
        int32_t c = copy_rec(r);
        set_slot(c, P.stateId, -1);
        lappend(p, 1, c);
        if (P.partner >= 0) {
          set_slot(c, PPRE[P.partner].stateId, -1);
          lappend(P.partner, 1, c);
        }
        break;
      }
      case PK_ABSENT_LOGICAL: {  // AbsentLogicalPreStateProcessor.addEveryState
        int32_t c = copy_rec(r);
        int32_t own = slot(c, P.stateId);
        if (own >= 0) rts(c) = nts(own);
        set_slot(c, P.stateId, -1);
        set_slot(c, PPRE[P.partner].stateId, -1);
        lappend(p, 1, c);
        lappend(P.partner, 1, c);
        break;
      }
      default:  // StreamPreStateProcessor.addEveryState :224-226
        lappend(p, 1, copy_rec(r));
        break;
    }
  }

  SM_JIT_INL __device__ void updateState(int p) {
    SM_PHASE(14);
    const DPre& P = PPRE[p];
    if (P.kind == PK_COUNT && fl(p, F_START_RESET)) {  // CountPreStateProcessor.updateState :145-151
      setfl(p, F_START_RESET, false);
      pre_init(p);
    }
    lsplice(p, 0, 1);  // StreamPreStateProcessor.updateState :268-271
    if (P.kind == PK_LOGICAL || P.kind == PK_ABSENT_LOGICAL) lsplice(P.partner, 0, 1);
  }

  __device__ bool seq_guard(int p) const {
    const DPre& P = PPRE[p];
    const DPost& TP = PPOST[P.post];
    return P.sequence && TP.nextEveryPre < 0 && TP.nextPre >= 0 && !lempty(TP.nextPre, 0);
  }

  SM_JIT_INL __device__ void resetState(int p) {
    const DPre& P = PPRE[p];
    switch (P.kind) {
      case PK_STREAM:
      case PK_COUNT:  // StreamPreStateProcessor.resetState :253-265
        lclear(p, 0);
        if (P.isStart && lempty(p, 1)) {
          if (P.sequence && PPOST[P.post].nextEveryPre < 0 && PPOST[P.post].nextPre < 0) {
            err |= NFA_ERR_NPE;
            return;
          }
          if (seq_guard(p)) return;
          pre_init(p);
        }
        break;
      case PK_LOGICAL:
      case PK_ABSENT_LOGICAL:  // LogicalPreStateProcessor.resetState :98-113
        if (P.ltype == LT_OR || lsize(p, 0) == lsize(P.partner, 0)) {
          lclear(p, 0);
          lclear(P.partner, 0);
          if (P.isStart && lempty(p, 1)) {
            if (seq_guard(p)) return;
            pre_init(p);
          }
        }
        break;
      default:  // AbsentStreamPreStateProcessor.resetState :111-126
        lclear(p, 0);
        if (P.isStart) {
          if (seq_guard(p)) return;
          pre_init(p);
        }
        break;
    }
  }

  // CountPreStateProcessor.startStateReset :137-142
  // (the callback branch re-enters the same processor; callbackPreStateProcessor is only ever set from
  //  CountPostStateProcessor.setNextStatePreProcessor before setStartState runs, so it is never taken)
  __device__ void count_startStateReset(int p) { setfl(p, F_START_RESET, true); }

  // StreamPreStateProcessor.process(StateEvent) :123-129 → FilterProcessor → post
  SM_INL_PRE __device__ void pre_process(int p, int32_t r, int chain_n = 0, int32_t chain_last = -1) {
    setfl(p, F_STATE_CHANGED, false);
    if (!filter_pass(p, r)) return;
    post_process(PPRE[p].post, r, chain_n, chain_last);
  }

  // processAndReturn of every pre kind; returned records are appended to the temporary list `ret`
  // (the pre's list word 3: the selector runs after the loop, as in the receivers).
  SM_INL_PAR __device__ void processAndReturn(int p, const int64_t* __restrict__ evr, int64_t now) {
    SM_PHASE(1 + p);
    const DPre& P = PPRE[p];
    const int sid = P.stateId;
    lclear(p, 3);
    switch (P.kind) {
      case PK_STREAM:
      case PK_ABSENT_STREAM: {
        if (P.kind == PK_ABSENT_STREAM && !fl(p, F_ACTIVE)) return;
        int32_t prev = -1;
        // A partial whose filter fails keeps nothing of this event (its copy is garbage): the filter is tried
        // against one copy of the event shared by the failing partials; the first partial that passes keeps that
        // copy as its own (StreamEventCloner.copyStreamEvent: one clone per partial) and the next trial makes a
        // fresh one.
        const bool trial = P.kind == PK_STREAM && P.progLen != 0;
        int32_t shared = -1;
        for (int32_t ln = lhead(p, 0); ln >= 0;) {
          if (err) return;
          int32_t s = ln_rec(ln);
          if (P.withinCnt > 0 && expired(p, s, now)) {
            ln = lerase(p, 0, prev, ln);
            continue;
          }
          if (trial) {
            bool pass;
            if (P.trialCur) {
              pass = P.ncache > 0 ? trial_cached(p, ln, evr) : trial_pass(p, s, evr);
              // the reference sets the slot to the event and back to null on a rejection: an every-copy that
              // arrived with the slot filled leaves it null
              if (!pass) set_slot(s, sid, -1);
            } else {
              if (shared < 0) shared = copy_event(evr);
              set_slot(s, sid, shared);
              pass = filter_pass(p, s);
              if (!pass) set_slot(s, sid, -1);
            }
            setfl(p, F_STATE_CHANGED, false);
            if (!pass) {  // what the loop below does for a partial the filter rejects
              if (!P.sequence) {
                prev = ln;
                ln = ln_next(ln);
              } else {
                ln = lerase(p, 0, prev, ln);
                int cb = PPOST[P.post].callbackPre;
                if (cb >= 0) count_startStateReset(cb);
              }
              continue;
            }
            if (shared < 0) shared = copy_event(evr);
            set_slot(s, sid, shared);
            shared = -1;
            post_process(P.post, s);  // pre_process after its filter
          } else {
            set_slot(s, sid, copy_event(evr));
            pre_process(p, s);
          }
          int tl = P.thisLast;
          if (returned(tl)) {
            set_returned(tl, 0);
            lappend(p, 3, s);
          }
          if (fl(p, F_STATE_CHANGED)) {
            ln = lerase(p, 0, prev, ln);
          } else if (!P.sequence) {
            set_slot(s, sid, -1);
            prev = ln;
            ln = ln_next(ln);
          } else {
            set_slot(s, sid, -1);
            ln = lerase(p, 0, prev, ln);
            int cb = PPOST[P.post].callbackPre;
            if (cb >= 0) count_startStateReset(cb);
          }
        }
        if (P.kind == PK_ABSENT_STREAM) lclear(p, 3);  // AbsentStreamPreStateProcessor.processAndReturn :218-231
        return;
      }
      case PK_COUNT: {  // CountPreStateProcessor.processAndReturn :58-93
        int32_t prev = -1;
        const bool trial = P.progLen != 0;  // as for PK_STREAM: a failing partial keeps nothing of the event
        int32_t shared = -1;
        // with an operand cache the trial comes first and the run record is read only for a partial that passes
        // (lazy removal): a partial whose next state is already filled is removed by the first event that would
        // otherwise act on it, and until then nothing reads it, so every output and list order is the reference's
        const bool lazy = lazy_count(P);  // trial && P.trialCur && P.ncache > 0
        for (int32_t ln = lhead(p, 0); ln >= 0;) {
          if (err) return;
          int32_t s = ln_rec(ln);
          auto next_filled = [&]() {
            return (PQ->nslots > sid + 1 && slot(s, sid + 1) >= 0) || (PQ->nslots > sid + 2 && slot(s, sid + 2) >= 0);
          };
          if (!lazy && next_filled()) {
            ln = lerase(p, 0, prev, ln);
            continue;
          }
          if (trial) {
            bool pass;
            if (lazy) {
              pass = trial_cached(p, ln, evr);
              if (pass && next_filled()) {
                ln = lerase(p, 0, prev, ln);
                continue;
              }
            } else if (P.trialCur) {
              pass = trial_pass(p, s, evr);
            } else {
              if (shared < 0) shared = copy_event(evr);
              add_event(s, sid, shared);
              pass = filter_pass(p, s);
              if (!pass) remove_last_event(s, sid);
            }
            setfl(p, F_SUCCESS, false);
            setfl(p, F_STATE_CHANGED, false);
            if (!pass) {  // what the loop below does for a partial the filter rejects
              if (!P.sequence) {
                prev = ln;
                ln = ln_next(ln);
              } else {
                ln = lerase(p, 0, prev, ln);
              }
              continue;
            }
            int cn = 0;
            int32_t cl = -1;
            if (P.trialCur) {
              if (shared < 0) shared = copy_event(evr);
              cn = add_event(s, sid, shared);
              cl = shared;
            }
            shared = -1;  // the partial keeps the copy
            post_process(P.post, s, cn, cl);  // pre_process after its filter
          } else {
            const int32_t ev = copy_event(evr);
            const int cn = add_event(s, sid, ev);
            setfl(p, F_SUCCESS, false);
            pre_process(p, s, cn, ev);
          }
          int tl = P.thisLast;
          if (returned(tl)) {
            set_returned(tl, 0);
            lappend(p, 3, s);
          }
          bool removed = false;
          if (fl(p, F_STATE_CHANGED)) {
            ln = lerase(p, 0, prev, ln);
            removed = true;
          }
          if (!fl(p, F_SUCCESS)) {
            remove_last_event(s, sid);
            if (P.sequence) {
              if (removed) {
                err |= NFA_ERR_NPE;
                return;
              }
              ln = lerase(p, 0, prev, ln);
              removed = true;
            }
          }
          if (!removed) {
            prev = ln;
            ln = ln_next(ln);
          }
        }
        return;
      }
      case PK_LOGICAL: {  // LogicalPreStateProcessor.processAndReturn :125-163
        int32_t prev = -1;
        const int psid = PPRE[P.partner].stateId;
        for (int32_t ln = lhead(p, 0); ln >= 0;) {
          if (err) return;
          int32_t s = ln_rec(ln);
          if (P.withinCnt > 0 && expired(p, s, now)) {
            ln = lerase(p, 0, prev, ln);
            continue;
          }
          if (P.ltype == LT_OR && slot(s, psid) >= 0) {
            ln = lerase(p, 0, prev, ln);
            continue;
          }
          set_slot(s, sid, copy_event(evr));
          pre_process(p, s);
          int tl = P.thisLast;
          if (returned(tl)) {
            set_returned(tl, 0);
            lappend(p, 3, s);
          }
          if (fl(p, F_STATE_CHANGED)) {
            ln = lerase(p, 0, prev, ln);
          } else if (!P.sequence) {
            set_slot(s, sid, -1);
            prev = ln;
            ln = ln_next(ln);
          } else {
            set_slot(s, sid, -1);
            ln = lerase(p, 0, prev, ln);
          }
        }
        return;
      }
      default: {  // PK_ABSENT_LOGICAL: AbsentLogicalPreStateProcessor.processAndReturn (always returns empty)
        if (!fl(p, F_ACTIVE)) return;
        int32_t prev = -1;
        const int psid = PPRE[P.partner].stateId;
        for (int32_t ln = lhead(p, 0); ln >= 0;) {
          if (err) return;
          int32_t s = ln_rec(ln);
          if (P.withinCnt > 0 && expired(p, s, now)) {
            ln = lerase(p, 0, prev, ln);
            continue;
          }
          if (P.ltype == LT_OR && slot(s, psid) >= 0) {
            ln = lerase(p, 0, prev, ln);
            continue;
          }
          int32_t current = slot(s, sid);
          set_slot(s, sid, copy_event(evr));
          pre_process(p, s);
          if (P.waitingTime != -1 || (P.sequence && P.ltype == LT_AND && PPOST[P.post].nextEveryPre >= 0))
            set_slot(s, sid, current);
          bool removed = false;
          int tl = P.thisLast;
          if (returned(tl)) {
            set_returned(tl, 0);
            int32_t nx = lerase(p, 0, prev, ln);
            removed = true;
            if (P.sequence) lremove_rec(P.partner, 0, s);
            ln = nx;
          }
          if (!fl(p, F_STATE_CHANGED)) {
            set_slot(s, sid, current);
            if (P.sequence) {
              if (removed) {
                err |= NFA_ERR_NPE;
                return;
              }
              ln = lerase(p, 0, prev, ln);
              removed = true;
            }
          }
          if (!removed) {
            prev = ln;
            ln = ln_next(ln);
          }
        }
        return;
      }
    }
  }

  // ------------------------------------------------------------ post-state processors
  SM_JIT_INL __device__ void stream_post(int o, int32_t r) {  // StreamPostStateProcessor.process :53-72
    const DPost& O = PPOST[o];
    setfl(O.thisPre, F_STATE_CHANGED, true);
    rts(r) = nts(slot(r, O.stateId));
    if (O.hasNext) set_returned(o, 1);
    if (O.nextPre >= 0) addState(O.nextPre, r);
    if (O.nextEveryPre >= 0) addEveryState(O.nextEveryPre, r);
    if (O.callbackPre >= 0) count_startStateReset(O.callbackPre);
  }
  // CountPostStateProcessor.processMinCountReached :73-85 (non-recursive: nested addState via the work list)
  SM_JIT_INL __device__ void count_minReached(int o, int32_t r) {
    const DPost& O = PPOST[o];
    if (O.hasNext) {
      setfl(O.thisPre, F_STATE_CHANGED, true);
      set_returned(o, 1);
    }
    if (O.nextPre >= 0) addState(O.nextPre, r);
    if (O.nextEveryPre >= 0) addEveryState(O.nextEveryPre, r);
  }
  // AbsentLogicalPreStateProcessor.partnerCanProceed
  SM_JIT_INL __device__ bool partnerCanProceed(int p, int32_t r) {
    const DPre& P = PPRE[p];
    const DPost& TP = PPOST[P.post];
    if (P.sequence && TP.nextEveryPre < 0 && lastArrival(p) > 0) return false;
    if (P.waitingTime == -1) {
      if (TP.nextEveryPre < 0) return slot(r, P.stateId) < 0;
      if (lastArrival(p) > 0) {
        lastArrival(p) = 0;
        pre_init(p);
        return false;
      }
      return true;
    }
    return slot(r, P.stateId) >= 0;
  }
  // chain_n > 0: a count state's chain has just been appended to (add_event), its length and last node known
  SM_JIT_INL __device__ void post_process(int o, int32_t r, int chain_n = 0, int32_t chain_last = -1) {
    const DPost& O = PPOST[o];
    switch (O.kind) {
      case PK_STREAM: stream_post(o, r); break;
      case PK_COUNT: {  // CountPostStateProcessor.process :45-71
        int32_t e;
        int n;
        if (chain_n > 0) {
          e = chain_last;
          n = chain_n;
        } else {
          e = slot(r, O.stateId);
          n = 1;
          while (nnext(e) >= 0) {
            ++n;
            e = nnext(e);
          }
        }
        setfl(O.thisPre, F_SUCCESS, true);
        rts(r) = nts(e);
        if (n >= O.minCount) {
          if (PPRE[O.thisPre].sequence) {
            if (O.nextPre >= 0) addState(O.nextPre, r);
            if (n != O.maxCount) addState(O.thisPre, r);
          } else if (n == O.minCount) {
            count_minReached(o, r);
          }
          if (n == O.maxCount) setfl(O.thisPre, F_STATE_CHANGED, true);
        }
        break;
      }
      case PK_LOGICAL: {  // LogicalPostStateProcessor.process :59-87
        if (O.ltype == LT_AND) {
          bool proceed;
          if (PPRE[O.partnerPre].kind == PK_ABSENT_LOGICAL) proceed = partnerCanProceed(O.partnerPre, r);
          else proceed = slot(r, PPRE[O.partnerPre].stateId) >= 0;
          if (proceed) stream_post(o, r);
          else setfl(O.thisPre, F_STATE_CHANGED, true);
        } else {
          stream_post(o, r);
          if (PPOST[O.partnerPost].hasNext && PPRE[O.thisPre].thisLast == O.partnerPost) set_returned(O.partnerPost, 1);
        }
        break;
      }
      case PK_ABSENT_STREAM: {  // AbsentStreamPostStateProcessor.process :36-55
        setfl(O.thisPre, F_STATE_CHANGED, true);
        int32_t se = slot(r, O.stateId);
        rts(r) = nts(se);
        set_returned(o, 1);
        if (PPRE[O.thisPre].isStart && O.nextEveryPre >= 0 && O.nextEveryPre == O.thisPre)
          addEveryState(O.nextEveryPre, r);
        lastArrival(O.thisPre) = nts(se);
        break;
      }
      default: {  // AbsentLogicalPostStateProcessor.process :37-50
        setfl(O.thisPre, F_STATE_CHANGED, true);
        set_returned(o, 1);
        lastArrival(O.thisPre) = nts(slot(r, O.stateId));
        break;
      }
    }
  }

  // ------------------------------------------------------------ absent timers
  SM_JIT_INL __device__ void absent_sendEvent(int p, int32_t r) {  // AbsentStreamPreStateProcessor.sendEvent :200-215
    const DPre& P = PPRE[p];
    const DPost& TP = PPOST[P.post];
    if (TP.hasNext) emit(r);
    if (TP.nextPre >= 0) addState(TP.nextPre, r);
    if (TP.nextEveryPre >= 0) {
      addEveryState(TP.nextEveryPre, r);
    } else if (P.isStart) {
      setfl(p, F_ACTIVE, false);
      if (P.kind == PK_ABSENT_LOGICAL && P.ltype == LT_OR && PPRE[P.partner].kind == PK_ABSENT_LOGICAL)
        setfl(P.partner, F_ACTIVE, false);
    }
    if (TP.callbackPre >= 0) count_startStateReset(TP.callbackPre);
  }

  // AbsentStreamPreStateProcessor.process(ComplexEventChunk) :129-198 /
  // AbsentLogicalPreStateProcessor.process(ComplexEventChunk)
  SM_JIT_INL __device__ void absent_timer(int p, int64_t now) {
    const DPre& P = PPRE[p];
    if (!fl(p, F_ACTIVE)) return;
    bool notProcessed = true;
    const int sid = P.stateId;
    lclear(p, 3);
    if (now >= lastArrival(p) + P.waitingTime) {
      if (P.kind == PK_ABSENT_STREAM) {
        bool initialize = P.isStart && lempty(p, 1) && lempty(p, 0);
        if (initialize && P.sequence && PPOST[P.post].nextEveryPre < 0 && lastArrival(p) > 0) initialize = false;
        if (initialize) {
          addState(p, new_rec());
        } else if (P.sequence && !lempty(p, 1)) {
          resetState(p);
        }
      } else {
        if (P.isStart && P.sequence && lempty(p, 1) && lempty(p, 0)) addState(p, new_rec());
        else if (P.sequence && !lempty(p, 1)) resetState(p);
      }
      updateState(p);
      int32_t prev = -1;
      for (int32_t ln = lhead(p, 0); ln >= 0;) {
        if (err) return;
        int32_t s = ln_rec(ln);
        if (P.withinCnt > 0 && expired(p, s, now)) {
          ln = lerase(p, 0, prev, ln);
          continue;
        }
        if (P.kind == PK_ABSENT_STREAM) {
          if (now >= rts(s) + P.waitingTime) {
            ln = lerase(p, 0, prev, ln);
            rts(s) = now;
            lappend(p, 3, s);
            continue;
          }
        } else {
          int32_t own = slot(s, sid);
          bool passed = own >= 0 ? now >= nts(own) + P.waitingTime : now >= rts(s) + P.waitingTime;
          if (passed) {
            ln = lerase(p, 0, prev, ln);
            bool partner_has = slot(s, PPRE[P.partner].stateId) >= 0;
            if (P.ltype == LT_OR && !partner_has) {
              add_event(s, sid, empty_node());
              lappend(p, 3, s);
            } else if (P.ltype == LT_AND && partner_has) {
              lappend(p, 3, s);
            } else if (P.ltype == LT_AND && !partner_has) {
              add_event(s, sid, empty_node());
            }
            continue;
          }
        }
        prev = ln;
        ln = ln_next(ln);
      }
      notProcessed = lempty(p, 3);
      for (int32_t ln = lhead(p, 3); ln >= 0; ln = ln_next(ln)) absent_sendEvent(p, ln_rec(ln));
      lclear(p, 3);
      lastArrival(p) = 0;
    }
    const DPost& TP = PPOST[P.post];
    bool rearm = (P.kind == PK_ABSENT_STREAM) ? (TP.nextEveryPre == p || (notProcessed && P.isStart))
                                              : (TP.nextEveryPre >= 0 || (notProcessed && P.isStart));
    if (rearm) {
      int64_t base = (P.kind == PK_ABSENT_STREAM) ? now : clock;
      int64_t nb = (lastArrival(p) == 0) ? base + P.waitingTime : lastArrival(p) + P.waitingTime;
      notifyAt(P.sched, nb);
    }
  }

  // ------------------------------------------------------------ garbage collection (Cheney, safe points only)
  __device__ int32_t fwd(int32_t o, int64_t& top) {
    if (o < 0) return o;
    int k = kind_of(o);
    if (k == K_FWD) return hi(o);
    int words = SM_OBJ_WORDS(k);
    int32_t n = (int32_t)top;
    SM_COUNT(3, words);
    for (int w = 0; w < words; ++w) heap[n + w] = heap[o + w];
    top += words;
    heap[o] = K_FWD | ((int64_t)(uint32_t)n << 32);
    return n;
  }
  // A key's heap in the overflow pool (misc(5) = pool offset + 1, misc(6) = its words per semispace) once its live
  // partial matches no longer fit its own arena: the reference's pending lists are unbounded LinkedLists
  // (StreamPreStateProcessor :58-59), so a hot key keeps growing while the other keys keep their small arenas.
  // After a collection that leaves a semispace more than a quarter full, the live objects are copied (the same
  // Cheney copy as gc, into a region of the pool) to a region with >= 8x their size per semispace.
  __device__ int32_t fwd_to(int32_t o, int64_t& top, const LaneWords& dst) {
    if (o < 0) return o;
    const int64_t h0 = heap[o];
    const int k = (int)(h0 & 0xFF);
    if (k == K_FWD) return (int32_t)(h0 >> 32);
    const int words = SM_OBJ_WORDS(k);
    const int32_t n = (int32_t)top;
    SM_COUNT(3, words);
    for (int w = 0; w < words; ++w) dst[n + w] = heap[o + w];
    top += words;
    heap[o] = K_FWD | ((int64_t)(uint32_t)n << 32);
    return n;
  }
  // Cheney copy of the live objects (reachable from the pending / newAndEvery lists, the collector's roots) into
  // semispace 0 of dst; returns the words copied. The source is left holding forwarding words.
  __device__ int64_t copy_live(const LaneWords& dst) {
    auto hi_of = [&](int64_t w) { return (int32_t)(w >> 32); };
    auto with_hi = [&](int64_t w, int32_t v) { return (w & 0xFFFFFFFFll) | ((int64_t)(uint32_t)v << 32); };
    int64_t top = 0, scan = 0;
    prune_stale();
    for (int p = 0; p < PQ->npre; ++p)
      for (int w = 0; w < 2; ++w) {
        const int32_t h = fwd_to(lhead(p, w), top, dst);
        const int32_t t = ltail(p, w) >= 0 ? fwd_to(ltail(p, w), top, dst) : -1;
        lset(p, w, h, t);
      }
    while (scan < top) {
      const int32_t o = (int32_t)scan;
      const int64_t h0 = dst[o];
      const int k = (int)(h0 & 0xFF);
      if (k == K_LNODE || k == K_LNODE4) {
        dst[o] = with_hi(h0, fwd_to(hi_of(h0), top, dst));
        dst[o + 1] = fwd_to((int32_t)dst[o + 1], top, dst);
        scan += k == K_LNODE4 ? 4 : 2;
      } else if (k == K_REC) {
        for (int s = 0; s < PQ->nslots; ++s) {
          int64_t& w = dst[o + 2 + (s >> 1)];
          const int32_t v = (s & 1) ? (int32_t)(w >> 32) : (int32_t)w;
          const int32_t nv = fwd_to(v, top, dst);
          w = (s & 1) ? with_hi(w, nv) : ((w & ~0xFFFFFFFFll) | (int64_t)(uint32_t)nv);
        }
        scan += PQ->rec_words;
      } else {
        dst[o] = with_hi(h0, fwd_to(hi_of(h0), top, dst));
        scan += PQ->node_words;
      }
    }
    return top;
  }
  // words per semispace of a pool region for `live` live words: at least twice the own arena, 8x the live data
  __device__ static int64_t pool_half(int64_t live, int32_t own_half) {
    int64_t nh = 2 * (int64_t)own_half;
    if (nh < 8 * live) nh = 8 * live;
    return (nh + 63) & ~(int64_t)63;
  }
  // `words` of the overflow pool, or -1 when it is full (a failed request claims nothing; it leaves its size in
  // pool_top[1], from which the host sizes the pool after the batch)
  __device__ int64_t pool_claim(int64_t words) {
    unsigned long long cur = *(volatile unsigned long long*)b->pool_top;
    for (;;) {
      if ((int64_t)cur + words > b->pool_cap) {
        atomicMax(b->pool_top + 1, (unsigned long long)words);
        return -1;
      }
      const unsigned long long prev = atomicCAS(b->pool_top, cur, cur + (unsigned long long)words);
      if (prev == cur) return (int64_t)cur;
      cur = prev;
    }
  }
  __device__ void promote(int64_t live) {
    const int64_t nh = pool_half(live, half);
    if (nh > ((int64_t)1 << 30)) return;  // heap offsets are 32-bit: stay (alloc reports an arena overflow)
    const int64_t words = 2 * nh + 64;
    if (!b->pool) return;
    const int64_t off = pool_claim(words);
    if (off < 0) return;  // pool full: the host grows it after the batch
    const LaneWords dst{b->pool + off, 1};
    const int64_t top = copy_live(dst);
    heap = dst;
    half = (int32_t)nh;
    misc(2) = 0;
    misc(1) = top;
    misc(5) = off + 1;
    misc(6) = nh;
  }
  // Stale partials of a lazily removed count state: with an operand cache a count partial is tried before
  // its run record is read, so one whose next state is already filled stays in the pending list until an event passes
  // its trial (processAndReturn, PK_COUNT). The reference drops it at the next event whatever the filter says
  // (CountPreStateProcessor.processAndReturn :58-93, removeIfNextStateProcessed), and until then nothing reads it, so
  // the collector may drop it first: the lists are pruned before they are forwarded, and a key whose count partials
  // keep failing their trials holds only its live partials (outputs and list order are unchanged).
  __device__ static bool lazy_count(const DPre& P) {
    return P.kind == PK_COUNT && P.progLen != 0 && P.trialCur && P.ncache > 0;
  }
  __device__ void prune_stale() {
    for (int p = 0; p < PQ->npre; ++p) {
      if (!lazy_count(PPRE[p])) continue;
      const int sid = PPRE[p].stateId;
      int32_t prev = -1;
      for (int32_t ln = lhead(p, 0); ln >= 0;) {
        const int32_t s = ln_rec(ln);
        if ((PQ->nslots > sid + 1 && slot(s, sid + 1) >= 0) || (PQ->nslots > sid + 2 && slot(s, sid + 2) >= 0)) {
          ln = lerase(p, 0, prev, ln);
        } else {
          prev = ln;
          ln = ln_next(ln);
        }
      }
    }
  }
  __device__ void gc() {
    int64_t space = misc(2);
    SM_COUNT(4, 1);
    prune_stale();
    int64_t to = (1 - space) * half;
    int64_t top = to, scan = to;
    for (int p = 0; p < PQ->npre; ++p)
      for (int w = 0; w < 2; ++w) {
        int32_t h = fwd(lhead(p, w), top);
        int32_t t = ltail(p, w) >= 0 ? fwd(ltail(p, w), top) : -1;
        lset(p, w, h, t);
      }
    while (scan < top) {
      int32_t o = (int32_t)scan;
      int k = kind_of(o);
      if (k == K_LNODE || k == K_LNODE4) {
        set_hi(o, fwd(hi(o), top));
        int32_t nx = (int32_t)heap[o + 1];
        heap[o + 1] = fwd(nx, top);
        scan += k == K_LNODE4 ? 4 : 2;
      } else if (k == K_REC) {
        for (int s = 0; s < PQ->nslots; ++s) set_slot(o, s, fwd(slot(o, s), top));
        scan += PQ->rec_words;
      } else {
        set_hi(o, fwd(hi(o), top));
        scan += PQ->node_words;
      }
    }
    misc(2) = 1 - space;
    misc(1) = top;
  }
  SM_JIT_INL __device__ void safe_point() {
    SM_PHASE(15);
    int64_t used = misc(1) - misc(2) * half;
    if (used * 2 > half) {
      gc();
      used = misc(1) - misc(2) * half;
      if (used * 4 > half) promote(used);
    }
  }

  // ------------------------------------------------------------ event delivery
  // MultiProcessStreamReceiver.receive / SingleProcessStreamReceiver.processAndClear + selector dispatch
  SM_INL_DELIVER __device__ void deliver(const int64_t* __restrict__ r) {
    const int64_t p = le_pos(*b, r);
    const int s = le_stream(*b, r);
    const DReceiver* R = nullptr;
    for (int k = 0; k < PQ->nrecv; ++k)
      if (PRECV[k].stream == s) R = &PRECV[k];
    if (!R) return;
    SM_COUNT(5, 1);
    pos = p;
    time = 0;
    phase = 1;
    sched = -1;
    int64_t now = le_node(*b, r, 1);
    // stabilizeStates
    if (PQ->kind == 2) {
      for (int k = 0; k < PQ->nreset; ++k) resetState(PQ->reset_seq[k]);  // inner reset(), flattened (plan.h)
      for (int k = 0; k < PQ->nupdate; ++k) updateState(PQ->update_seq[k]);
    } else if (R->multi) {
      for (int k = 0; k < R->nstate; ++k) updateState(R->stateProcs[k]);
    } else if (R->nstate > 0) {
      updateState(R->stateProcs[0]);
    }
    for (int k = 0; k < R->nproc && !err; ++k) {
      int pp = R->procs[k];
      processAndReturn(pp, r, now);
      if (err) return;
      if (!lempty(pp, 3)) {
        if (!R->hasQuerySelector && !R->multi) {
          err |= NFA_ERR_NPE;
          return;
        }
        if (R->hasQuerySelector)
          for (int32_t ln = lhead(pp, 3); ln >= 0; ln = ln_next(ln)) emit(ln_rec(ln));
      }
      lclear(pp, 3);
    }
  }

  // Playback listeners: every scheduler of this key drains its FIFO while head <= now (Scheduler.sendTimerEvents)
  SM_INL_FIRE __device__ void fire_all(int64_t now, int64_t at_pos, int64_t step_time) {
    SM_PHASE(13);
    clock = now;
    for (int p = 0; p < PQ->npre; ++p) {
      if (!is_absent(p)) continue;
      int s = PPRE[p].sched;
      while (!qempty(s) && qhead(s) - now <= 0 && !err) {
        int64_t t = qhead(s);
        qpop(s);
        pos = at_pos;
        time = step_time;
        phase = 0;
        sched = s;
        absent_timer(p, t);
      }
    }
    int64_t h;
    due = min_head(h) ? h : INT64_MAX;
  }
  SM_JIT_INL __device__ bool min_head(int64_t& t) const {
    bool any = false;
    for (int p = 0; p < PQ->npre; ++p) {
      if (!is_absent(p)) continue;
      int s = PPRE[p].sched;
      if (!qempty(s)) {
        int64_t h = qhead(s);
        if (!any || h < t) t = h;
        any = true;
      }
    }
    return any;
  }
};

__device__ StackVal StateLoader::var(const Instr& in) const {
  StackVal v;
  v.i = 0;
  v.d = 0;
  v.null = 1;
  int32_t n = L->at(rec, in.a, in.b);
  if (n < 0) return v;
  if ((L->heap[n + 3] >> in.c) & 1) return v;
  int64_t w = L->heap[n + 4 + in.c];
  v.null = 0;
  if (in.t0 == T_FLOAT || in.t0 == T_DOUBLE) v.d = __longlong_as_double(w);
  else v.i = w;
  return v;
}

__device__ StackVal TrialLoader::var(const Instr& in) const {
  if (in.a != sid) return StateLoader{L, rec}.var(in);
  StackVal v;
  v.i = 0;
  v.d = 0;
  v.null = 1;
  if ((le_node(*L->b, evr, 3) >> in.c) & 1) return v;
  const int64_t w = le_node(*L->b, evr, 4 + in.c);
  v.null = 0;
  if (in.t0 == T_FLOAT || in.t0 == T_DOUBLE) v.d = __longlong_as_double(w);
  else v.i = w;
  return v;
}

__device__ StackVal CachedTrialLoader::var(const Instr& in) const {
  if (in.a == sid) return TrialLoader{L, -1, sid, evr}.var(in);
#ifdef SM_NFA_JIT
  const DPre* PP = PPRE;
  const Instr* PC = PCODE;
#else
  const DPre* PP = L->PPRE;
  const Instr* PC = L->PCODE;
#endif
  // operand k of this pre's cache (DPre.cacheIns; plan constants in the query-specialised build). A load that is none
  // of them breaks the compiler's invariant (every other-state load of a cached filter is a cached operand): error,
  // never a silent read of the other slot
  const DPre& P = PP[pre];
  int k = -1;
  for (int c = 0; c < P.ncache && c < 2; ++c) {
    const Instr& ci = PC[P.cacheIns[c]];
    if (k < 0 && ci.op == in.op && ci.a == in.a && ci.b == in.b && ci.c == in.c) k = c;
  }
  StackVal v;
  if (k < 0) {
    L->err |= NFA_ERR_NPE;
    v.i = 0;
    v.null = 1;
    return v;
  }
  v.i = L->heap[ln + 2 + k];
  v.null = (int)((L->heap[ln] >> (8 + k)) & 1);
  return v;
}

// First index a in [from, n) with v[a] >= x (or, with strict, v[a] > x) over a non-decreasing array; n if none.
// Galloping from `from`: a key lane's successive searches land close to the previous answer, and a batch of N
// playback events has N advance points, so a linear step per key would make the whole launch O(keys x N).
template <bool strict>
__device__ int64_t gallop(const int64_t* __restrict__ v, int64_t from, int64_t n, int64_t x) {
  auto before = [&](int64_t a) { return strict ? v[a] <= x : v[a] < x; };
  if (from >= n || !before(from)) return from;
  int64_t lo = from, step = 1;  // invariant: before(lo)
  int64_t hi = from + 1;
  while (hi < n && before(hi)) {
    lo = hi;
    step <<= 1;
    hi = lo + step;
  }
  if (hi > n) hi = n;  // answer in (lo, hi]
  while (hi - lo > 1) {
    int64_t mid = lo + ((hi - lo) >> 1);
    if (before(mid)) lo = mid;
    else hi = mid;
  }
  return hi;
}

#ifndef SM_LE_NT
#define SM_LE_NT 1  // A/B build flag: nontemporal column loads in the lane-events pass (config 5 step 33.5 -> 33.0 ms)
#endif
// Record k of the query's batch, in key order, as its LaneEv record (nfa.h): a lane then reads one contiguous
// record per event instead of chasing key_pos -> stream / row / ts / clock / ordinal / columns.
__device__ __forceinline__ int64_t lane_attr(const NfaStream& st, int a, int64_t row, int64_t& nulls) {
  int64_t v = 0;
  bool isnull = st.nulls[a] && st.nulls[a][row];
#if SM_LE_NT && defined(__HIP_DEVICE_COMPILE__)
#define SM_LE_LD(T, p) __builtin_nontemporal_load((const T*)(p))
#else
#define SM_LE_LD(T, p) (*(const T*)(p))
#endif
  switch (st.types[a]) {
    case T_INT: v = SM_LE_LD(int32_t, (const int32_t*)st.cols[a] + row); break;
    case T_LONG: v = SM_LE_LD(int64_t, (const int64_t*)st.cols[a] + row); break;
    case T_FLOAT: { double d = (double)SM_LE_LD(float, (const float*)st.cols[a] + row); v = __double_as_longlong(d); break; }
    case T_DOUBLE: v = __double_as_longlong(SM_LE_LD(double, (const double*)st.cols[a] + row)); break;
    case T_STRING: v = SM_LE_LD(int32_t, (const int32_t*)st.cols[a] + row); isnull = isnull || v < 0; break;
    default: v = ((const uint8_t*)st.cols[a])[row]; break;
  }
#undef SM_LE_LD
  if (isnull) nulls |= (1ll << a);
  return v;
}

__device__ __forceinline__ void lane_event_record(const NfaBatch& b, int64_t p, int64_t k, int32_t node_words,
                                                  int64_t* __restrict__ out) {
  const int64_t W = LaneEv::words(node_words, SM_LE_C(b));
  int64_t* r = out + k * W;
  const int s = b.ev_stream[p];
  const NfaStream* st = s >= 0 ? &b.streams[s] : nullptr;
  const int na = st ? st->nattr : 0;
  const int64_t row = st ? (b.ev_row ? b.ev_row[p] : p) : 0;  // no ev_row: rows are positions (device batches)
  if (SM_LE_C(b)) {
    // the compact 64-byte form (nfa.h LaneEv): at most 4 attributes
    int64_t v[8];
    int64_t nulls = 0;
    const int64_t upto = b.adv_upto ? b.adv_upto[p] : -1;
    v[0] = (int64_t)(((uint64_t)(uint32_t)p) | ((uint64_t)(uint32_t)(int32_t)upto << 32));
    v[1] = b.ev_clock[p];
    v[2] = b.ev_ts[p];
#pragma unroll
    for (int a = 0; a < 4; ++a) v[4 + a] = (a < na) ? lane_attr(*st, a, row, nulls) : 0;
    const int64_t o = b.ev_ord[p];
    const uint64_t ov = o < 0 ? kLeOrdMask : ((uint64_t)(o - b.lane_ord_base) & kLeOrdMask);
    v[3] = (int64_t)(ov | ((uint64_t)(uint8_t)(int8_t)s << 48) | ((uint64_t)(nulls & 0xFF) << 56));
    longlong2* r2 = (longlong2*)r;
#pragma unroll
    for (int w = 0; w < 4; ++w) r2[w] = make_longlong2(v[2 * w], v[2 * w + 1]);
    return;
  }
  if (W == 16) {
    // the common shape (<= 8 attributes): the record in registers, one full 128-byte line in 16-byte stores
    int64_t v[16];
    int64_t nulls = 0;
    v[LaneEv::kPos] = p;
    v[LaneEv::kStream] = s;
    v[LaneEv::kClock] = b.ev_clock[p];
    v[LaneEv::kUpto] = b.adv_upto ? b.adv_upto[p] : -1;
    v[LaneEv::kNode] = 0;
    v[LaneEv::kNode + 1] = b.ev_ts[p];
    v[LaneEv::kNode + 2] = b.ev_ord[p];
#pragma unroll
    for (int a = 0; a < 8; ++a) v[LaneEv::kNode + 4 + a] = (a < na) ? lane_attr(*st, a, row, nulls) : 0;
    v[LaneEv::kNode + 3] = nulls;
    longlong2* r2 = (longlong2*)r;
#pragma unroll
    for (int w = 0; w < 8; ++w) r2[w] = make_longlong2(v[2 * w], v[2 * w + 1]);
    return;
  }
  r[LaneEv::kPos] = p;
  r[LaneEv::kStream] = s;
  r[LaneEv::kClock] = b.ev_clock[p];
  r[LaneEv::kUpto] = b.adv_upto ? b.adv_upto[p] : -1;
  int64_t* node = r + LaneEv::kNode;
  node[0] = 0;
  node[1] = b.ev_ts[p];
  node[2] = b.ev_ord[p];
  int64_t nulls = 0;
  for (int a = 0; a < na; ++a) node[4 + a] = lane_attr(*st, a, row, nulls);
  node[3] = nulls;
  for (int64_t w = LaneEv::kNode + 4 + na; w < W; ++w) r[w] = 0;  // padding too: whole lines are written
}

// First advance point after position x, at or after index `from`: O(1) through the per-position count of
// advance points (upto = advance points at positions <= x, carried in the event's LaneEv record), galloping when
// the batch has none.
__device__ __forceinline__ int64_t adv_after(const NfaBatch& b, int64_t from, int64_t x, int64_t upto) {
  if (x == INT64_MAX) return b.nadv > from ? b.nadv : from;
  if (upto < 0) return gallop<true>(b.adv_pos, from, b.nadv, x);
  return upto > from ? upto : from;
}

// The rare part of a lane's timer loop: find the advance point where the earliest timer falls due and fire the
// timers there. Out of line (SM_TIMER_INLINE undoes it, A/B), so that its registers stay off the per-event path.
#if defined(SM_NFA_JIT_INLINE_ALL)
#define SM_TIMER_ATTR SM_NFA_ALWAYS_INLINE  // JIT: the Lane must not escape into a call (it would live in scratch)
#elif defined(SM_TIMER_INLINE)
#define SM_TIMER_ATTR
#else
#define SM_TIMER_ATTR __attribute__((noinline))
#endif
SM_TIMER_ATTR __device__ bool timer_fire(Lane& L, const NfaBatch& b, int64_t a1, int64_t t, int64_t next_pos,
                                         int64_t& search_from) {
  // the first advance point at or after search_from whose clock reaches t: one load of the clock index (the clock
  // only moves forward, so it is the later of search_from and the first point overall); a gallop without the index.
  // (The gallop was a chain of about 26 dependent loads per firing, which the lane's whole wave waits for: the
  // emitting config-5 variant fires about 13 timers per key)
  int64_t a2;
  if (b.adv_cidx) {
    const int64_t c = t - b.adv_cmin;
    const int64_t g = c <= 0 ? 0 : (c >= b.adv_cspan ? b.nadv : (int64_t)b.adv_cidx[c]);
    a2 = g > search_from ? g : search_from;
  } else {
    a2 = gallop<false>(b.adv_clock, search_from, b.nadv, t);
  }
  const int64_t a = a1 < a2 ? a1 : a2;
  if (a >= b.nadv || b.adv_pos[a] > next_pos) {
    search_from = a;
    return false;
  }
  if (b.adv_wall[a] >= 0) {
    // wall-clock emulation: step through due timer times up to the tick target
    int64_t target = b.adv_wall[a];
    int64_t h;
    while (L.min_head(h) && h <= target && h >= L.clock && !L.err) L.fire_all(h, b.adv_pos[a], h);
    L.fire_all(target, b.adv_pos[a], target);
  } else {
    L.fire_all(b.adv_clock[a], b.adv_pos[a], b.adv_clock[a]);
  }
  search_from = a + 1;
  L.safe_point();
  return true;
}

struct Lane;
SM_JIT_INL __device__ void nfa_lane_run(Lane& L, const NfaBatch& b, int32_t key, int32_t* err_out);

SM_JIT_INL __device__ void nfa_lane(const NfaBatch& b, const char* __restrict__ blob, int64_t* ks_all, int64_t* heap_all,
                         int32_t heap_half, int64_t lanes, int32_t key, int32_t* err_out) {
  Lane L;
#ifdef SM_NFA_JIT
  blob = (const char*)::sm::kPlanBlob;  // the kernel passes no plan buffer
#else
  L.PQ = (const DQuery*)blob;
  L.PPRE = (const DPre*)(blob + L.PQ->off_pre);
  L.PPOST = (const DPost*)(blob + L.PQ->off_post);
  L.PRECV = (const DReceiver*)(blob + L.PQ->off_recv);
  L.PWITHIN = (const DWithin*)(blob + L.PQ->off_within);
  L.PCODE = (const Instr*)(blob + L.PQ->off_code);
  L.PCONSTS = (const DVal*)(blob + L.PQ->off_const);
  L.PSEL = (const int32_t*)(blob + L.PQ->off_sel);
  L.PREFS = (const int32_t*)(blob + L.PQ->off_refs);
  const DQuery* PQ = L.PQ;
  const DPre* PPRE = L.PPRE;
#endif
  L.ks = LaneWords{ks_all + key, lanes};
  L.ksh = L.ks;
  L.half = heap_half;
  // the heap stays key-major: a lane's run records and chain nodes are private, pointer-chased objects, so
  // keeping each object's words in one line beats sharing lines with other lanes' (unrelated) offsets
  L.heap = LaneWords{heap_all + (int64_t)key * (2 * (int64_t)heap_half + 64), 1};
  L.b = &b;
  {  // a key promoted to the overflow pool by an earlier batch (Lane::promote)
    const int64_t po = L.ksh[PQ->ks_misc + 5];
    if (po > 0) {
      L.heap = LaneWords{b.pool + (po - 1), 1};
      L.half = (int32_t)L.ksh[PQ->ks_misc + 6];
    }
  }
  L.key = key;
  L.err = 0;
  L.seq = 0;
  L.clock = b.clock_in;
  L.due = INT64_MAX;

#ifdef SM_NFA_LDS
  // LDS staging of the lane's per-key state words (north_star: "LDS staging of active partial matches per
  // workgroup"): the pre / post / misc words every event reads and writes (about 40 accesses per event on
  // config 5) live in the workgroup's LDS, lane-interleaved (word w of thread t at [w * 64 + t]), for the lane's
  // whole event run, and go back to HBM once at its end. Timer queues stay in HBM (touched only when a timer is
  // scheduled or fires). Needs blockDim.x == 64 and (ks_sched + kNfaLdsMisc) words x 64 x 8 B of dynamic LDS.
  extern __shared__ int64_t sm_nfa_lds[];
  const int nst = PQ->ks_sched;
  LaneWords st{sm_nfa_lds + threadIdx.x, 64};
  for (int w = 0; w < nst; ++w) st[w] = L.ksh[w];
  for (int k = 0; k < kNfaLdsMisc; ++k) st[nst + k] = L.ksh[PQ->ks_misc + 1 + k];
  L.ks = st;
#endif
  nfa_lane_run(L, b, key, err_out);
#ifdef SM_NFA_LDS
  for (int w = 0; w < nst; ++w) L.ksh[w] = st[w];
  for (int k = 0; k < kNfaLdsMisc; ++k) L.ksh[PQ->ks_misc + 1 + k] = st[nst + k];
#endif
}

// A lane's event run (after its Lane is set up): lane creation, then its events in arrival order with the timers
// due before each.
SM_JIT_INL __device__ void nfa_lane_run(Lane& L, const NfaBatch& b, int32_t key, int32_t* err_out) {
#ifndef SM_NFA_JIT
  const DQuery* PQ = L.PQ;
  const DPre* PPRE = L.PPRE;
  const DReceiver* PRECV = L.PRECV;
#endif
  const char* blob = (const char*)PQ;
  const int64_t ebeg = b.key_off[key], eend = b.key_off[key + 1];
  const int64_t W = LaneEv::words(PQ->node_words, SM_LE_C(b));
  const bool has_timers = PQ->nsched > 0;
  // lane creation: QueryRuntime constructor → init() seeds the start state (PartitionRuntime.clonePartition)
  if (L.misc(4) == 0) {
    if (ebeg == eend && !(b.create_all)) return;
    const int32_t* init = (const int32_t*)(blob + PQ->filt_off);
    for (int p = 0; p < PQ->npre; ++p) {
      L.lset(p, 0, -1, -1);
      L.lset(p, 1, -1, -1);
      L.flags(p) = F_ACTIVE;
      L.lset(p, 3, -1, -1);
      if (L.is_absent(p)) L.lastArrival(p) = 0;
    }
    L.ks[PQ->ks_post] = 0;  // no post processor has returned an event
    for (int s = 0; s < PQ->nsched; ++s) {
      L.sq(s)[0] = 0;
      L.sq(s)[1] = 0;
    }
    L.misc(0) = (ebeg < eend) ? le_node(b, b.lane_ev + ebeg * W, 2) : -1;  // creation ordinal
    L.misc(1) = 0;
    L.misc(2) = 0;
    L.misc(3) = 0;
    L.misc(4) = 1;
    for (int k = 0; k < init[0]; ++k) L.pre_init(init[1 + k]);
  }
  if (ebeg == eend && !has_timers) {
    return;
  }
  if (has_timers) {  // timers left by earlier batches (a lane created just now has only what pre_init scheduled)
    int64_t h;
    L.due = L.min_head(h) ? h : INT64_MAX;
  }
  // Walk this key's events; before each, fire timers due at clock-advance points (playback) in order.
  // (Measured and not kept, round 5: greedy stream rounds, where per round a wave ran only the lanes whose next event
  // came from its most common receiver stream, to cut divergent path runs: emitting variant NFA 108.4 -> 120.8 ms,
  // literal 17.8 -> 24.4 ms; each round pays the event-record and timer checks again, which cost more than the
  // path runs it saves.)
  int64_t k = ebeg;
  int64_t search_from = 0;  // advance-point index
  for (;;) {
    // this key's events are consecutive LaneEv records (key order): one contiguous read per event
    const int64_t* __restrict__ r = b.lane_ev + k * W;
    const int64_t next_pos = (k < eend) ? le_pos(b, r) : INT64_MAX;
    if (has_timers) {
      for (;;) {
        if (L.err) break;
        const int64_t t = L.due;  // the earliest timer (Lane::due, kept up to date by notifyAt / fire_all)
        if (t == INT64_MAX) break;
        // first advance point at or after search_from whose position <= next_pos and (clock >= t or wall tick)
        // (both arrays are non-decreasing: positions ascend and the playback clock only moves forward)
        const int64_t a1 = adv_after(b, search_from, next_pos, k < eend ? le_upto(b, r) : -1);
        // quick reject: every advance point up to next_pos has clock <= the clock after next_pos's sendData
        if (next_pos != INT64_MAX && le_clock(b, r) < t) {
          search_from = a1;
          break;
        }
        if (!timer_fire(L, b, a1, t, next_pos, search_from)) break;
      }
    }
    if (L.err || k >= eend) break;
    const int64_t p = next_pos;
    // clock as of this event (sendData advanced it before delivery)
    L.clock = le_clock(b, r);
    if (le_stream(b, r) == NFA_START) {
      // SiddhiAppRuntime.start → AbsentStreamPreStateProcessor.start :261-269 (non-partitioned queries)
      for (int pp = 0; pp < PQ->npre; ++pp)
        if (L.is_absent(pp) && PPRE[pp].isStart && PPRE[pp].waitingTime != -1 && L.fl(pp, F_ACTIVE))
          L.notifyAt(PPRE[pp].sched, L.clock + PPRE[pp].waitingTime);
    } else {
      L.deliver(r);
    }
    // timers scheduled by this event may only fire at later advance points
    search_from = adv_after(b, search_from, p, le_upto(b, r));
    ++k;
    if (L.err) break;
    L.safe_point();
  }
  if (L.err) atomicOr(err_out, L.err);
}

#if !defined(SM_NFA_JIT) && !defined(SM_NFA_LDS)
// Batch-boundary compaction of a query's overflow pool (runtime.cpp compact_pool): pass 0 sizes each promoted key's
// new home, pass 1 moves its live objects there (the collector's copy). A key whose live data fits a quarter of its own
// arena goes back to it (misc(5) = 0); every other promoted key gets a pool region sized for its live data in the new
// pool. Nothing of the old pool stays reachable afterwards: regions abandoned by keys promoted again, and regions of
// keys whose hot phase is over, are reclaimed, so the pool holds what the live partial matches need.
__device__ void nfa_pool_lane(const char* __restrict__ blob, int64_t* ks_all, int64_t* heap_all, int32_t heap_half,
                              int64_t lanes, int32_t key, int pass, int64_t* old_pool, int64_t* new_pool,
                              unsigned long long* new_top, int64_t* new_off) {
  Lane L;
  L.PQ = (const DQuery*)blob;
  L.PPRE = (const DPre*)(blob + L.PQ->off_pre);
  L.PPOST = (const DPost*)(blob + L.PQ->off_post);
  L.PRECV = (const DReceiver*)(blob + L.PQ->off_recv);
  L.PWITHIN = (const DWithin*)(blob + L.PQ->off_within);
  L.PCODE = (const Instr*)(blob + L.PQ->off_code);
  L.PCONSTS = (const DVal*)(blob + L.PQ->off_const);
  L.PSEL = (const int32_t*)(blob + L.PQ->off_sel);
  L.PREFS = (const int32_t*)(blob + L.PQ->off_refs);
  L.ks = LaneWords{ks_all + key, lanes};
  L.ksh = L.ks;
  L.b = nullptr;
  L.err = 0;
  if (L.misc(4) == 0 || L.misc(5) <= 0) {  // no lane yet, or its heap is its own arena
    if (pass == 0) new_off[key] = -2;
    return;
  }
  L.heap = LaneWords{old_pool + (L.misc(5) - 1), 1};
  L.half = (int32_t)L.misc(6);
  if (pass == 0) L.gc();  // in place: what is in use afterwards is exactly the live data
  const int64_t live = L.misc(1) - L.misc(2) * L.half;
  if (pass == 0) {
    new_off[key] = live * 4 <= heap_half ? -1
                                         : (int64_t)atomicAdd(new_top, (unsigned long long)(2 * Lane::pool_half(live, heap_half) + 64));
    return;
  }
  const int64_t o = new_off[key];
  if (o == -2) return;
  const LaneWords dst = o == -1 ? LaneWords{heap_all + (int64_t)key * (2 * (int64_t)heap_half + 64), 1}
                                : LaneWords{new_pool + o, 1};
  const int64_t top = L.copy_live(dst);
  L.misc(2) = 0;
  L.misc(1) = top;
  L.misc(5) = o == -1 ? 0 : o + 1;
  L.misc(6) = o == -1 ? 0 : Lane::pool_half(live, heap_half);
}
#endif

}  // namespace
}  // namespace sm
