// replay.hip — MI355X (gfx950) kernels of the batched workflow-history replay engine.
//
// Reference hot path: stateBuilderImpl.applyEvents (service/history/stateBuilder.go:
// 112-611) driving mutableStateBuilder.Replicate*Event, one goroutine per workflow.
//
// MI355X design (DESIGN.md has the full argument):
//   * One wavefront = one 64-thread workgroup = one slice of the sliced layout (cdr.h):
//     64 workflows of similar length, one per lane, walked in lockstep.  Column loads
//     are buffer loads through per-slice descriptors built once from wave-uniform
//     values, so each load of a step is one fully coalesced 256/512-B wave access.
//   * Type-directed loads.  The type column runs two steps ahead of the operand
//     columns; a column the lane's event type never reads gets an out-of-range buffer
//     offset, which returns 0 without touching memory.  The load is still issued, so
//     every step issues a fixed number of vector-memory ops and the compiler's
//     s_waitcnt vmcnt(N) counts stay exact: the operands of event k are waited for only
//     when event k is processed, CDR_DEPTH steps after they were issued.
//   * Per-workflow scalar state (ExecutionInfo, decision FSM, version-history head,
//     replication state, call bookkeeping) lives in VGPRs for the whole history.
//   * Live activities and user timers, which the order-dependent timer picks
//     (timerBuilder.go:171-312) scan after every activity/timer event, live in LDS
//     working slots, lane-interleaved (plane p of slot j of lane L at word
//     (j*P+p)*64+L: conflict-free ds_read_b64).  Slices whose live sets exceed the LDS
//     budget replay in a second launch whose slots live in global scratch.  The tiers
//     are never mixed behind one pointer: a generic pointer compiles to flat_*, whose
//     out-of-order return forces vmcnt(0) on every use and serialises the prefetch.
//   * Children / request-cancels / signals write straight into their output slot
//     ranges (rare, never scanned by a pick).
//   * Errors: the first error/panic of a workflow stops it (the caller discards the
//     mutable state); its code and event are reported per workflow.
//   * Continue-as-new runs are separate lanes; k_finalize stitches their status into
//     the parent afterwards (stateBuilder.go:537-595).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "cdr/cdr.h"
#include "ctx.h"

#ifndef CDR_DEPTH
#define CDR_DEPTH 1 /* events whose operand loads are in flight beyond the one processed */
#endif
#ifndef CDR_TYPED
#define CDR_TYPED 1 /* 1: read only the operand columns the event's type needs */
#endif
#ifndef CDR_WPE
#define CDR_WPE 3 /* waves per SIMD the register allocator must leave room for */
#endif
#ifndef CDR_LDS_ACT_MAX
#define CDR_LDS_ACT_MAX 1 /* activity working slots per lane kept in LDS */
#endif
#ifndef CDR_LDS_TIM_MAX
#define CDR_LDS_TIM_MAX 4 /* user-timer working slots per lane kept in LDS */
#endif

#define GAS __attribute__((address_space(1)))
#define DEAD_KEY ((int64_t)0x8000000000000000ll)
#define NS_PER_S 1000000000ll
#define T_NONE ((int64_t)0x7FFFFFFFFFFFFFFFll)
#define OOB 0x80000000u /* buffer offset beyond every slice: load returns 0, no memory access */

namespace {

// workflowExecutionInfo.go:45-147 — true if the transition is accepted
__device__ __forceinline__ bool transition_ok(int cur, int cur_close, int st, int cs) {
  switch (cur) {
    case CDR_STATE_VOID:
      return true;
    case CDR_STATE_CREATED:
      if (st == CDR_STATE_COMPLETED) return cs == CDR_CLOSE_TERMINATED || cs == CDR_CLOSE_TIMED_OUT;
      if (st == CDR_STATE_CREATED || st == CDR_STATE_RUNNING || st == CDR_STATE_ZOMBIE) return cs == CDR_CLOSE_NONE;
      return false;
    case CDR_STATE_RUNNING:
      if (st == CDR_STATE_CREATED) return false;
      if (st == CDR_STATE_RUNNING || st == CDR_STATE_ZOMBIE) return cs == CDR_CLOSE_NONE;
      if (st == CDR_STATE_COMPLETED) return cs != CDR_CLOSE_NONE;
      return false;
    case CDR_STATE_COMPLETED:
      return st == CDR_STATE_COMPLETED && cs == cur_close;
    case CDR_STATE_ZOMBIE:
      if (st == CDR_STATE_CREATED || st == CDR_STATE_RUNNING) return cs == CDR_CLOSE_NONE;
      if (st == CDR_STATE_COMPLETED || st == CDR_STATE_ZOMBIE) return cs != CDR_CLOSE_NONE;
      return false;
  }
  return false;
}

// ClusterNameForFailoverVersion (common/cluster/metadata.go:187-203): -1 = no owner
template <class M>  // cdr_cluster_meta in any address space
__device__ __forceinline__ int cluster_for_version(const M& m, int64_t v) {
  if (v == CDR_EMPTY_VERSION) return m.current_cluster;
  int64_t init = v % m.failover_version_increment;
  int r = -1;
#pragma unroll
  for (int i = 0; i < CDR_MAX_CLUSTERS; i++)
    if (i < m.n_clusters && m.initial_version[i] == init && r < 0) r = i;
  return r;
}

// Move live rows (key != DEAD) to the front, ascending by key (selection sort; live
// sets are small).  Returns the live count.
template <class Row, class KeyF>
__device__ uint32_t compact_sorted(Row* rows, uint32_t hw, KeyF keyf) {
  uint32_t n = 0;
  for (uint32_t i = 0; i < hw; i++) {
    int best = -1;
    int64_t bk = 0;
    for (uint32_t j = i; j < hw; j++) {
      if (!keyf.live(rows[j])) continue;
      int64_t k = keyf.key(rows[j]);
      if (best < 0 || k < bk) {
        best = (int)j;
        bk = k;
      }
    }
    if (best < 0) break;
    if ((uint32_t)best != i) {
      Row tmp = rows[i];
      rows[i] = rows[best];
      rows[best] = tmp;
    }
    n++;
  }
  return n;
}
struct ActKey {
  __device__ bool live(const cdr_activity_info& r) const { return r.schedule_id != DEAD_KEY; }
  __device__ int64_t key(const cdr_activity_info& r) const { return r.schedule_id; }
};
struct TimerKey {
  __device__ bool live(const cdr_timer_info& r) const { return r.started_id != DEAD_KEY; }
  __device__ int64_t key(const cdr_timer_info& r) const { return (int64_t)r.timer_id; }
};
struct ChildKey {
  __device__ bool live(const cdr_child_info& r) const { return r.initiated_id != DEAD_KEY; }
  __device__ int64_t key(const cdr_child_info& r) const { return r.initiated_id; }
};
struct CancelKey {
  __device__ bool live(const cdr_cancel_info& r) const { return r.initiated_id != DEAD_KEY; }
  __device__ int64_t key(const cdr_cancel_info& r) const { return r.initiated_id; }
};
struct SignalKey {
  __device__ bool live(const cdr_signal_info& r) const { return r.initiated_id != DEAD_KEY; }
  __device__ int64_t key(const cdr_signal_info& r) const { return r.initiated_id; }
};

// whole-record copies to / from global memory (C++ copy operators do not cross
// address spaces); every record is a multiple of 8 bytes
template <class T>
__device__ __forceinline__ void gput(GAS T* p, const T& v) {
  static_assert(sizeof(T) % 8 == 0, "record size");
  const uint64_t* s = reinterpret_cast<const uint64_t*>(&v);
  GAS uint64_t* d = (GAS uint64_t*)p;
#pragma unroll
  for (uint32_t i = 0; i < sizeof(T) / 8; i++) d[i] = s[i];
}
template <class T>
__device__ __forceinline__ T gget(const GAS T* p) {
  static_assert(sizeof(T) % 8 == 0, "record size");
  T v;
  uint64_t* d = reinterpret_cast<uint64_t*>(&v);
  const GAS uint64_t* s = (const GAS uint64_t*)p;
#pragma unroll
  for (uint32_t i = 0; i < sizeof(T) / 8; i++) d[i] = s[i];
  return v;
}

// ---- lastDecision of the entry's last applyEvents call (stateBuilder.go:126,200,213,
// 238,256,610).  Per lane, ld = CDR_LD_* source | LD_CAPTURED | event index << 3.  A
// source event's decisionInfo equals the ExecutionInfo decision fields right after it
// (UpdateDecision, mutableStateDecisionTaskManager.go:677-702) and those change again
// only at a DecisionTaskCompleted / Failed / TimedOut or the next source event, so the
// record is written just before such a clearing event (rare: both in one call) or once
// after the loop; the call's first event resets it (lastDecision is a local of each call).
#define LD_CAPTURED 4u
__device__ __forceinline__ bool ld_pending(uint32_t ld) { return (ld & 3u) != 0u && !(ld & LD_CAPTURED); }
__device__ __forceinline__ uint32_t ld_make(uint32_t src, uint32_t k) { return src | (k << 3); }
__device__ __forceinline__ cdr_last_decision ld_rec(uint32_t ld, int64_t dv, int64_t dsched, int64_t dstart,
                                                    uint32_t dreq, int32_t dto, int64_t datt, int64_t dsc_ts,
                                                    int64_t dst_ts, int64_t dorig_ts) {
  cdr_last_decision r;
  const bool any = (ld & 3u) != 0u;
  r.source = ld & 3u;
  r.request_id = any ? dreq : 0u;
  r.event_index = any ? (int64_t)(ld >> 3) : 0;
  r.version = any ? dv : 0;
  r.schedule_id = any ? dsched : 0;
  r.started_id = any ? dstart : 0;
  r.attempt = any ? datt : 0;
  r.scheduled_ts = any ? dsc_ts : 0;
  r.started_ts = any ? dst_ts : 0;
  r.original_scheduled_ts = any ? dorig_ts : 0;
  r.decision_timeout = any ? dto : 0;
  r._pad = 0;
  return r;
}
__device__ __forceinline__ void ld_write(GAS cdr_last_decision* o, uint32_t ld, int64_t dv, int64_t dsched,
                                         int64_t dstart, uint32_t dreq, int32_t dto, int64_t datt, int64_t dsc_ts,
                                         int64_t dst_ts, int64_t dorig_ts) {
  gput(o, ld_rec(ld, dv, dsched, dstart, dreq, dto, datt, dsc_ts, dst_ts, dorig_ts));
}

// Opaque copy of a wave-uniform base pointer: loads through it cannot be hoisted out
// of the replay loop, so per-workflow descriptors and table bases are re-read in the
// (rare) event types that need them instead of occupying VGPRs for the whole history.
template <class T>
__device__ __forceinline__ GAS T* late(T* base) {
  GAS T* p = (GAS T*)base;
  asm volatile("" : "+s"(p));
  return p;
}
template <class T>
__device__ __forceinline__ const GAS T* late(const T* base) {
  const GAS T* p = (const GAS T*)base;
  asm volatile("" : "+s"(p));
  return p;
}

template <class Row>
__device__ __forceinline__ int find_initiated(const GAS Row* rows, uint32_t hw, int64_t id) {
  for (uint32_t j = 0; j < hw; j++)
    if (rows[j].initiated_id == id) return (int)j;
  return -1;
}
template <class Row>
__device__ __forceinline__ int alloc_initiated(const GAS Row* rows, uint32_t& hw, uint32_t cap) {
  for (uint32_t j = 0; j < hw; j++)
    if (rows[j].initiated_id == DEAD_KEY) return (int)j;
  if (hw < cap) return (int)(hw++);
  return -1;
}

// ---------------------------------------------------------------- event columns
// One buffer descriptor per slice (the slice's block of the slab, cdr.h); a column
// is selected by its uniform start offset (soffset), an element by the lane's byte
// offset (voffset).  Columns an event's type does not read get bit 31 set in the
// voffset: past the block, the load returns 0 without touching memory.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
#define OOB_BIT 0x80000000u
// cache policy of a slab load (the buffer instruction's aux bits; gfx950: 2 = nt, a streaming
// load whose lines the L2 may drop first).  The fast kernel reads each slab line once: its
// loads stream (C2 -1.7%); the class kernels re-read rows of the original block at emission,
// so theirs stay cached (nt on the class-block loads: C3 -3.2%, C4 +6.7%, C5 +7.2%; the fast
// kernel's: C2 -1.5%, interleaved A/B in one process, profiles/r6_nt)
#ifndef CDR_NT_FAST
#define CDR_NT_FAST 2
#endif
#ifndef CDR_NT_CLS
#define CDR_NT_CLS 0
#endif
template <int AUX = 0>
__device__ __forceinline__ int64_t bld64(rsrc_t r, uint32_t voff, uint32_t soff) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, AUX);
  return (int64_t)(((uint64_t)v[1] << 32) | (uint64_t)v[0]);
}
template <int AUX = 0>
__device__ __forceinline__ uint32_t bld32(rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, AUX);
}
struct Slice {
  rsrc_t r;
  uint32_t elems;  // slice_len * 64
  uint32_t l4;     // lane * 4: an element of a 4-byte column sits l4 below its 8-byte twin
  __device__ __forceinline__ uint32_t col(int c) const { return cdr_col_off(c); }
};
// voffset of element (k, lane) of an 8-byte column relative to the column's start in
// row 0 (OOB_BIT set when k is past the lane's history); 4-byte columns: minus l4
__device__ __forceinline__ uint32_t el8(uint32_t k, uint32_t len, uint32_t lane) {
  return (k < len ? k * CDR_ROW_BYTES : OOB_BIT) + lane * 8u;
}

// one event's operands (cdr.h "operand columns per type"); task_id is read once,
// for the last event, after the loop (only the last applied event's value survives)
struct Ev {
  uint32_t tf, h;
  int32_t n;
  int64_t id, ver, ts, key, aux;
};
template <int AUX = 0>
__device__ __forceinline__ uint32_t load_tf(const Slice& S, uint32_t o8) {
  return bld32<AUX>(S.r, o8 - S.l4, S.col(CDR_COL_TYPE_FLAGS));
}
// need bit b of tf (CDR_SEF_NEED_*) clear -> OOB_BIT
__device__ __forceinline__ uint32_t gate(uint32_t off, uint32_t tf, uint32_t bit) {
  return off | ((tf & bit) ? 0u : OOB_BIT);
}
// DELTA: skip the event_id / version loads the packer's CDR_SEF_ID_NEXT / VER_SAME bits
// make redundant (the consumer rebuilds them, ev_delta)
template <bool DELTA = false, int AUX = 0>
__device__ __forceinline__ Ev load_ops(const Slice& S, uint32_t o8, uint32_t tf) {
  const uint32_t o4 = o8 - S.l4;
  Ev e;
  e.tf = tf;
  e.id = bld64<AUX>(S.r, DELTA ? o8 | ((tf & CDR_SEF_ID_NEXT) ? OOB_BIT : 0u) : o8, S.col(CDR_COL_EVENT_ID));
  e.ver = bld64<AUX>(S.r, DELTA ? o8 | ((tf & CDR_SEF_VER_SAME) ? OOB_BIT : 0u) : o8, S.col(CDR_COL_VERSION));
#if CDR_TYPED
  e.ts = bld64<AUX>(S.r, gate(o8, tf, CDR_SEF_NEED_TS), S.col(CDR_COL_TIMESTAMP));
  e.key = bld64<AUX>(S.r, gate(o8, tf, CDR_SEF_NEED_KEY), S.col(CDR_COL_KEY));
  e.aux = bld64<AUX>(S.r, gate(o8, tf, CDR_SEF_NEED_AUX), S.col(CDR_COL_AUX));
  e.h = bld32<AUX>(S.r, gate(o4, tf, CDR_SEF_NEED_H), S.col(CDR_COL_H));
  e.n = (int32_t)bld32<AUX>(S.r, gate(o4, tf, CDR_SEF_NEED_N), S.col(CDR_COL_N));
#else
  e.ts = bld64<AUX>(S.r, o8, S.col(CDR_COL_TIMESTAMP));
  e.key = bld64<AUX>(S.r, o8, S.col(CDR_COL_KEY));
  e.aux = bld64<AUX>(S.r, o8, S.col(CDR_COL_AUX));
  e.h = bld32<AUX>(S.r, o4, S.col(CDR_COL_H));
  e.n = (int32_t)bld32<AUX>(S.r, o4, S.col(CDR_COL_N));
#endif
  return e;
}

// ---------------------------------------------------------------- working slots
// activity working-slot planes (8-byte words)
enum : uint32_t {
  AP_SID = 0,          // scheduleID (DEAD_KEY = free slot)
  AP_TS2C = 1,         // ScheduleToClose candidate: sched + s2c (ExpirationTime is never earlier)
  AP_TALT = 2,         // ScheduleToStart candidate before start, StartToClose after
  AP_THB = 3,          // Heartbeat candidate (started and hb > 0) else T_NONE
  AP_META = 4,         // activityID handle | AF_* << 32 | TimerTaskStatus << 40
  AP_VER = 5,
  AP_STARTED_ID = 6,
  AP_STARTED_TIME = 7,
  AP_CANCEL_ID = 8,
  AP_ROWS = 9,         // row of the ActivityTaskScheduled event | row of its call's first event << 32
  AP_STC_HB = 10,      // StartToClose | HeartbeatTimeout << 32 (seconds)
  AP_REQ = 11,         // RequestID handle
};
static_assert(AP_REQ + 1 == CDR_ACT_PLANES, "activity planes");
enum : uint32_t { TP_SID = 0, TP_TID_TASK = 1, TP_EXPIRY = 2, TP_VER = 3 };
static_assert(TP_VER + 1 == CDR_TIM_PLANES, "timer planes");
#define AF_AIDMAP 0x1ull /* this slot holds byActivityID[aid] */
#define AF_STARTED 0x2ull
#define AF_CANCEL 0x4ull
#define META_FLAG(f) ((f) << 32)
#define META_TTS_SHIFT 40
// event types whose replay only updates registers (one shared dispatch pass)
#define SIMPLE_TYPES                                                                                         \
  (CDR_TB(CDR_EV_WF_SIGNALED) | CDR_TB(CDR_EV_DT_SCHEDULED) | CDR_TB(CDR_EV_DT_STARTED) |                    \
   CDR_TB(CDR_EV_MARKER_RECORDED) | CDR_TB(CDR_EV_CANCEL_TIMER_FAILED) | CDR_TB(CDR_EV_AT_REQ_CANCEL_FAILED) | \
   CDR_TB(CDR_EV_WF_CANCEL_REQUESTED))
#define AP_CARRIED ((int64_t)1 << 62) /* AP_ROWS: row j of the loaded activity table (cdr_carry) */

extern __shared__ uint64_t cdr_lds[];

// LDS tier: this lane's plane 0 of slot 0 at word l
template <uint32_t P>
struct LdsSlots {
  uint32_t l;
  __device__ __forceinline__ int64_t ld(uint32_t j, uint32_t p) const {
    return (int64_t)cdr_lds[l + (j * P + p) * CDR_SLICE_WIDTH];
  }
  __device__ __forceinline__ void st(uint32_t j, uint32_t p, int64_t v) const {
    cdr_lds[l + (j * P + p) * CDR_SLICE_WIDTH] = (uint64_t)v;
  }
};
// One record per active lane (`on` lanes only), written by the whole wave together through an
// LDS transpose at cdr_lds[lw ..] (8-B words; (CW + 1) * 65 of them): in each pass of up to CW
// words, work item i is word i % cw of the record of the lane ranked i / cw, so that
// consecutive lanes store consecutive words of one record in one instruction — whole segments
// instead of one write request per field store from lanes whose records lie apart
// (tools/calib.hip k_cal_wrec: 8 B per store from lanes 256 B apart cost a 64-B request each).
// Every active lane of the wave calls it (wave-uniform control flow); the LDS words are free
// for the caller again when it returns.
template <uint32_t CW, class T>
__device__ __forceinline__ void coop_put(GAS T* dst, const T& v, bool on, uint32_t lw) {
  static_assert(sizeof(T) % 8 == 0, "record size");
  constexpr uint32_t NW = sizeof(T) / 8, RS = 65;
  const uint64_t* src = reinterpret_cast<const uint64_t*>(&v);
  const uint64_t em = __builtin_amdgcn_read_exec();
  const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(em >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)em, 0u));
  const uint32_t na = (uint32_t)__builtin_popcountll(em);
  uint64_t* const L = cdr_lds + lw;
#pragma unroll
  for (uint32_t w0 = 0; w0 < NW; w0 += CW) {
    constexpr uint32_t one = 1;
    const uint32_t cw = NW - w0 < CW ? NW - w0 : CW;
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): earlier LDS traffic has landed
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (uint32_t j = 0; j < CW; j++)
      if (j < cw) L[j * RS + rank] = src[w0 + j];
    L[CW * RS + rank] = on ? (uint64_t)(uintptr_t)((GAS uint64_t*)dst + w0) : 0ull;
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
    for (uint32_t i = rank; i < cw * na; i += na) {
      const uint32_t rr = i / cw, j = i - rr * cw;
      const uint64_t p = L[CW * RS + rr];
      if (p) ((GAS uint64_t*)(uintptr_t)p)[j] = L[j * RS + rr];
    }
    (void)one;
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_wave_barrier();
}

// one 128-B half of a cdr_exec_info record (schema.h: the Started half, then the replay half)
struct exec_half {
  uint64_t w[16];
};
static_assert(sizeof(cdr_exec_info) == 2 * sizeof(exec_half), "ExecutionInfo halves");

// global tier: the slice's lane-interleaved scratch (same plane layout)
template <uint32_t P>
struct GlbSlots {
  GAS uint64_t* g;
  __device__ __forceinline__ int64_t ld(uint32_t j, uint32_t p) const {
    return (int64_t)g[((uint64_t)j * P + p) * CDR_SLICE_WIDTH];
  }
  __device__ __forceinline__ void st(uint32_t j, uint32_t p, int64_t v) const {
    g[((uint64_t)j * P + p) * CDR_SLICE_WIDTH] = (uint64_t)v;
  }
};

// activity timer pick (timerBuilder.go:211-312) over the live working slots
template <class A>
__device__ __forceinline__ void act_pick(const A& S, uint32_t hw) {
  int best = -1;
  int64_t bt = 0, bs = 0;
  int bo = 0;
  uint32_t bbit = 0;
  for (uint32_t j = 0; j < hw; j++) {
    const int64_t sid = S.ld(j, AP_SID);
    if (sid == DEAD_KEY) continue;
    const uint64_t meta = (uint64_t)S.ld(j, AP_META);
    int64_t t = S.ld(j, AP_TS2C);
    int o = 0;
    uint32_t bit = CDR_TTS_SCHEDULE_TO_CLOSE;
    const int64_t ta = S.ld(j, AP_TALT), th = S.ld(j, AP_THB);
    if (ta < t) {  // append order breaks ties: S2C, then STC/S2S, then HB
      t = ta;
      o = 1;
      bit = (meta & META_FLAG(AF_STARTED)) ? CDR_TTS_START_TO_CLOSE : CDR_TTS_SCHEDULE_TO_START;
    }
    if (th < t) {
      t = th;
      o = 2;
      bit = CDR_TTS_HEARTBEAT;
    }
    if (best < 0 || t < bt || (t == bt && (sid < bs || (sid == bs && o < bo)))) {
      best = (int)j;
      bt = t;
      bs = sid;
      bo = o;
      bbit = bit;
    }
  }
  if (best >= 0) {
    const uint64_t m = (uint64_t)S.ld((uint32_t)best, AP_META);
    const uint64_t b = (uint64_t)bbit << META_TTS_SHIFT;
    if (!(m & b)) S.st((uint32_t)best, AP_META, (int64_t)(m | b));
  }
}

// user timer pick (timerBuilder.go:171-184,233-247): head by (ExpiryTime, StartedID)
template <class T>
__device__ __forceinline__ void tim_pick(const T& S, uint32_t hw) {
  int best = -1;
  int64_t be = 0, bs = 0;
  for (uint32_t j = 0; j < hw; j++) {
    const int64_t sid = S.ld(j, TP_SID);
    if (sid == DEAD_KEY) continue;
    const int64_t ex = S.ld(j, TP_EXPIRY);
    if (best < 0 || ex < be || (ex == be && sid < bs)) {
      best = (int)j;
      be = ex;
      bs = sid;
    }
  }
  if (best >= 0) {
    const uint64_t v = (uint64_t)S.ld((uint32_t)best, TP_TID_TASK);
    if ((v >> 32) != CDR_TIMER_TASK_STATUS_CREATED)
      S.st((uint32_t)best, TP_TID_TASK,
           (int64_t)((v & 0xFFFFFFFFull) | ((uint64_t)CDR_TIMER_TASK_STATUS_CREATED << 32)));
  }
}

// Predicated forms of the picks for the replay loop: the slot scan runs to the
// slice's uniform slot count `cap` (slots past the lane's high-water mark `hw` are
// ignored), state is carried in selects, and only the final status-bit store is
// lane-masked.  `on` = the lane's event asked for a pick.
// what a pick created (the timer task createNewTask returns, timerBuilder.go:391-408)
struct Pick {
  bool made;
  int32_t timeout_type, slot;
  int64_t vis, event_id;
};
template <class A>
__device__ __forceinline__ Pick act_pick_p(const A& S, uint32_t hw, uint32_t cap, bool on) {
  int best = -1;
  int64_t bt = 0, bs = 0;
  int bo = 0;
  uint32_t bbit = 0;
  uint64_t bm = 0;
  for (uint32_t j = 0; j < cap; j++) {
    const int64_t sid = S.ld(j, AP_SID);
    const uint64_t meta = (uint64_t)S.ld(j, AP_META);
    const int64_t t0 = S.ld(j, AP_TS2C), ta = S.ld(j, AP_TALT), th = S.ld(j, AP_THB);
    // append order breaks ties within an activity: S2C, then STC/S2S, then HB
    const bool pa = ta < t0;
    const int64_t t1 = pa ? ta : t0;
    const bool ph = th < t1;
    const int64_t t = ph ? th : t1;
    const int o = ph ? 2 : (pa ? 1 : 0);
    const uint32_t bit = ph ? CDR_TTS_HEARTBEAT
                            : (pa ? ((meta & META_FLAG(AF_STARTED)) ? CDR_TTS_START_TO_CLOSE : CDR_TTS_SCHEDULE_TO_START)
                                  : CDR_TTS_SCHEDULE_TO_CLOSE);
    const bool better = on && j < hw && sid != DEAD_KEY &&
                        (best < 0 || t < bt || (t == bt && (sid < bs || (sid == bs && o < bo))));
    best = better ? (int)j : best;
    bt = better ? t : bt;
    bs = better ? sid : bs;
    bo = better ? o : bo;
    bbit = better ? bit : bbit;
    bm = better ? meta : bm;
  }
  const uint64_t b = (uint64_t)bbit << META_TTS_SHIFT;
  const bool made = best >= 0 && !(bm & b);
  if (made) S.st((uint32_t)best, AP_META, (int64_t)(bm | b));
  // TimerTaskStatus bit -> shared.TimeoutType (StartToClose 0 ... Heartbeat 3)
  return Pick{made, (int32_t)__builtin_ctz(bbit | 16u), best, bt, bs};
}
template <class T>
__device__ __forceinline__ Pick tim_pick_p(const T& S, uint32_t hw, uint32_t cap, bool on) {
  int best = -1;
  int64_t be = 0, bs = 0;
  uint64_t bv = 0;
  for (uint32_t j = 0; j < cap; j++) {
    const int64_t sid = S.ld(j, TP_SID);
    const int64_t ex = S.ld(j, TP_EXPIRY);
    const uint64_t v = (uint64_t)S.ld(j, TP_TID_TASK);
    const bool better = on && j < hw && sid != DEAD_KEY && (best < 0 || ex < be || (ex == be && sid < bs));
    best = better ? (int)j : best;
    be = better ? ex : be;
    bs = better ? sid : bs;
    bv = better ? v : bv;
  }
  const bool made = best >= 0 && (bv >> 32) != CDR_TIMER_TASK_STATUS_CREATED;
  if (made)
    S.st((uint32_t)best, TP_TID_TASK, (int64_t)((bv & 0xFFFFFFFFull) | ((uint64_t)CDR_TIMER_TASK_STATUS_CREATED << 32)));
  return Pick{made, 0, best, be, bs};
}

}  // namespace

// ============================================================== replay kernel
// Launch parameters.  The kernel reads them through the kernarg segment pointer made
// opaque at each use (KA()): every field is a fresh scalar load where it is needed,
// so rarely used parameters (table bases, cluster map, uuid seed ...) do not occupy
// SGPRs across the replay loop.
struct cdr_launch {
  cdr_dev_batch B;
  cdr_out O;
  uint32_t la, lt;  // activity / user-timer working slots per lane held in LDS
  uint32_t fast;    // CDR_SLICE_FAST slices go to k_replay_fast (else every slice here)
  uint32_t reg;     // CDR_SLICE_REG slices go to k_replay_reg (else here)
  uint32_t s0;      // slice of block 0 (the launch covers its kernel class's slice range)
  uint32_t retry;   // k_replay_reg: only the entries k_replay_cls left CLS_RETRY
  // k_replay_cls lists each slice where it left an entry CLS_RETRY (rlist[*rcount++]); the
  // retry pass of k_replay_reg walks that list (null: every slice of its range)
  uint32_t* rlist;
  uint32_t* rcount;
  // carry-in launches: the list k_replay_reg appends the slices it hands on to (the next
  // tier's rlist)
  uint32_t* olist;
  uint32_t* ocount;
  // PAR k_replay_cls: workgroups started (the other classes' streams wait until every PAR
  // workgroup holds its CU, so that the bulk classes' small workgroups cannot starve them)
  uint32_t* pstart;
  // k_replay_cls<TASKS>: the per-class staging lists of the task records and the per-entry
  // headers k_tasks_merge reads (replay_cls.inc)
  uint64_t* tstage;
  uint32_t* thead;
  uint64_t trows;  // records tstage holds (a staging index at or past it: the entry is handed on)
};
// result code k_replay_cls (or a carry-in k_replay_reg below the 12-activity variant) leaves
// on an entry it hands to k_replay_reg (never returned)
#define CLS_RETRY 0x7FFF
// result code the carry-in 12-activity k_replay_reg leaves on an entry it hands to the
// general kernel's retry pass (never returned)
#define CLS_RETRY2 0x7FFE
// result flag k_replay_cls sets when its pending rows are already dense and in key
// order (k_tables skips their sort and clears it; never returned)
#define RF_ROWS_SORTED 0x80000000u
#define AS4 __attribute__((address_space(4)))
__device__ __forceinline__ const AS4 cdr_launch* KA() {
  const AS4 cdr_launch* p = (const AS4 cdr_launch*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return p;
}
template <class T>
__device__ __forceinline__ GAS T* gp(T* p) {
  return (GAS T*)p;
}
template <class T>
__device__ __forceinline__ const GAS T* gp(const T* p) {
  return (const GAS T*)p;
}

// LDS = true: slices whose working slots fit (act_slots <= la, tim_slots <= lt);
// LDS = false: the rest, with working slots in the global scratch.
// loaded-state tables whose field names the kernel below uses as macros
__device__ __forceinline__ const GAS cdr_reset_point* carry_rp(const GAS cdr_carry* c) { return gp(c->state.rp); }
__device__ __forceinline__ const GAS cdr_kv* carry_sa(const GAS cdr_carry* c) { return gp(c->state.sa); }
__device__ __forceinline__ const GAS cdr_vh_item* carry_vh(const GAS cdr_carry* c) { return gp(c->state.vh); }

template <bool LDS, bool TASKS>
__global__ __launch_bounds__(CDR_SLICE_WIDTH) __attribute__((amdgpu_waves_per_eu(CDR_WPE, 8))) void k_replay(
    cdr_launch L) {
  (void)L;  // read through KA()
  // retry: the slices a carry-in k_replay_reg listed (block b: list entry b), their
  // CLS_RETRY2 entries only
  const bool retry = KA()->retry != 0u;
  if (retry && blockIdx.x >= __builtin_amdgcn_readfirstlane(*KA()->rcount)) return;
  const uint32_t s = retry ? __builtin_amdgcn_readfirstlane(KA()->rlist[blockIdx.x]) : blockIdx.x + KA()->s0;
  const uint32_t lane = threadIdx.x;
  if (s >= KA()->B.ev.n_slices) return;
  // slice scalars (readfirstlane makes their uniformity visible, so the descriptor
  // lives in SGPRs and no buffer load needs a waterfall loop)
  const uint32_t act_cap = __builtin_amdgcn_readfirstlane(KA()->B.ev.slice_act_slots[s]);
  const uint32_t tim_cap = __builtin_amdgcn_readfirstlane(KA()->B.ev.slice_tim_slots[s]);
  const uint32_t la = KA()->la, lt = KA()->lt;
  if ((act_cap <= la && tim_cap <= lt) != LDS) return;
  if (!retry) {
    const uint32_t sf = __builtin_amdgcn_readfirstlane(KA()->B.ev.slice_flags[s]);
    if (sf & CDR_SLICE_WAVE) return;  // k_replay_wave
    if (KA()->fast && (sf & CDR_SLICE_FAST)) return;
    if (KA()->reg && (sf & (CDR_SLICE_REG | CDR_SLICE_REG2 | CDR_SLICE_REG0 | CDR_SLICE_PAR))) return;  // k_replay_reg / cls
  }
  const uint64_t row0_ = KA()->B.ev.slice_row0[s];
  const uint64_t row0 = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(row0_ >> 32)) << 32) |
                        __builtin_amdgcn_readfirstlane((uint32_t)row0_);
  Slice S;
  S.elems = __builtin_amdgcn_readfirstlane(KA()->B.ev.slice_len[s]) * CDR_SLICE_WIDTH;
  S.r = __builtin_amdgcn_make_buffer_rsrc((void*)(KA()->B.ev.slab + row0 * CDR_ROW_BYTES), (short)0,
                                          (int)(S.elems * CDR_EL_BYTES), 0x00020000);
  S.l4 = lane * 4u;
  const int32_t w = KA()->B.ev.lane_wf[(uint64_t)s * CDR_SLICE_WIDTH + lane];
  if (w < 0 || (KA()->B.skip && KA()->B.skip[w])) return;  // empty lane / masked entry
  if (retry && gp(KA()->O.result)[w].code != CLS_RETRY2) return;

  // per-workflow descriptor, capacities and output records, re-read where used
#define B_ (KA()->B)
#define O_ (KA()->O)
#define D (gp(B_.wfs)[w])
#define CP (gp(B_.caps)[w])
#define X (gp(O_.exec) + w)
#define RS (gp(O_.repl) + w)
#define chi (gp(O_.child) + CP.child_off)
#define can (gp(O_.cancel) + CP.cancel_off)
#define sig (gp(O_.signal) + CP.signal_off)
#define vh (gp(O_.vh) + CP.vh_off)
#define rp (gp(O_.rp) + CP.rp_off)
#define sa (gp(O_.sa) + CP.sa_off)
  const uint32_t len = (uint32_t)D.ev_len;
  const uint32_t builder = D.builder;
  const uint32_t EU = B_.empty_uuid;
  const bool isRS = builder == CDR_BUILDER_2DC;
  const bool isVH = builder == CDR_BUILDER_NDC;

  // working slots of pending activities / user timers
  typedef typename std::conditional<LDS, LdsSlots<CDR_ACT_PLANES>, GlbSlots<CDR_ACT_PLANES>>::type ASlots;
  typedef typename std::conditional<LDS, LdsSlots<CDR_TIM_PLANES>, GlbSlots<CDR_TIM_PLANES>>::type TSlots;
  ASlots A;
  TSlots T;
  if constexpr (LDS) {
    A.l = lane;
    T.l = la * CDR_ACT_PLANES * CDR_SLICE_WIDTH + lane;
  } else {
    GAS uint64_t* g = gp(B_.scratch + B_.ev.slice_scratch_off[s] + lane);
    A.g = g;
    T.g = g + (uint64_t)act_cap * CDR_ACT_PLANES * CDR_SLICE_WIDTH;
  }
  uint32_t cks_ok = 0;  // a binary checksum known to be in AutoResetPoints

  // ---- ExecutionInfo fields that later events change (registers); the fields only
  // WorkflowExecutionStarted writes go straight to the output record.
  uint32_t x_flags = 0;
  int64_t x_completion_batch = 0, x_next_event = CDR_FIRST_EVENT_ID, x_last_processed = CDR_EMPTY_EVENT_ID;
  int32_t x_dt_timeout_value = 0, x_state = CDR_STATE_CREATED, x_close = CDR_CLOSE_NONE, x_signals = 0;
  // decision (decisionInfo, mutableStateDecisionTaskManager.go:677-690)
  int64_t dv = CDR_EMPTY_VERSION, dsched = CDR_EMPTY_EVENT_ID, dstart = CDR_EMPTY_EVENT_ID, datt = 0, dst_ts = 0,
          dsc_ts = 0, dorig_ts = 0;
  uint32_t dreq = EU;
  uint32_t ld = 0;  // lastDecision bookkeeping (ld_write)
  const bool want_ld = O_.last_decision != nullptr;
  int32_t dto = 0;
  // versions
  int64_t curv = D.failover_version;  // NDC currentVersion
  // 2DC ReplicationState: CurrentVersion and LastWrite{Version,EventID} always end as
  // the last applied event's (prev_ver / prev_id); StartVersion is written through at
  // WorkflowExecutionStarted; only the LastReplicationInfo mask stays in a register
  uint32_t rs_mask = 0;
  int64_t vh_last_id = 0, vh_last_ver = 0;  // the last VH item lives in registers
  uint32_t n_vh = 0;
  // tables
  uint32_t hw_act = 0, hw_tim = 0, hw_chi = 0, hw_can = 0, hw_sig = 0;
  uint32_t live_chi = 0, live_can = 0, live_sig = 0, n_rp = 0, n_sa = 0;
  // calls / errors
  int64_t call_first_id = 0, prev_id = 0, prev_ver = 0;
  uint32_t call_first_k = 0, call_idx = 0;
  bool newrun_applied = false, stop_at_call_end = false;
  uint32_t nr_call = 0xFFFFFFFFu;  // the call that applied the new run (a cluster panic there: never attempted)
  int32_t err = len == 0 ? CDR_E_HISTORY_EMPTY : CDR_OK;
  int64_t err_id = 0;
  uint32_t err_k = 0;

#define FAIL(code)           \
  do {                       \
    err = (code);            \
    err_id = e.id;           \
    err_k = k;               \
    stop_at_call_end = true; \
  } while (0)

  // ---- carry-in (cdr_carry): start from a loaded state instead of the fresh builder
  // (mutableStateBuilder.Load, mutableStateBuilder.go:272-295): the persisted records
  // become the registers, working slots and output rows the replay continues from
  const int32_t csrc = B_.carry ? gp(B_.carry)->src[w] : -1;
  if (csrc >= 0) {
    const GAS cdr_carry* CY = gp(B_.carry);
    const cdr_wf_caps cc = gget(gp(CY->caps) + csrc);
    const cdr_wf_result cr = gget(gp(CY->state.result) + csrc);
    const cdr_exec_info x = gget(gp(CY->state.exec) + csrc);
    gput(X, x);  // the Started half stays as loaded; the replay half is rewritten at the end
    x_flags = x.flags;
    x_completion_batch = x.completion_event_batch_id;
    x_next_event = x.next_event_id;
    x_last_processed = x.last_processed_event;
    x_dt_timeout_value = x.decision_timeout_value;
    x_state = x.state;
    x_close = x.close_status;
    x_signals = x.signal_count;
    dv = x.decision_version;
    dsched = x.decision_schedule_id;
    dstart = x.decision_started_id;
    datt = x.decision_attempt;
    dst_ts = x.decision_started_ts;
    dsc_ts = x.decision_scheduled_ts;
    dorig_ts = x.decision_original_scheduled_ts;
    dreq = x.decision_request_id;
    dto = x.decision_timeout;
    curv = CDR_EMPTY_VERSION;  // :291 (an in-memory builder keeps its own: after the VH load below)
    if (isRS) {
      const cdr_repl_state rs0 = gget(gp(CY->state.repl) + csrc);
      gput(RS, rs0);
      rs_mask = rs0.lri_mask;
    }
    n_rp = cr.n_reset_points;
    for (uint32_t j = 0; j < n_rp; j++) gput(rp + j, gget(carry_rp(CY) + cc.rp_off + j));
    n_sa = cr.n_search_attr;
    for (uint32_t j = 0; j < n_sa; j++) gput(sa + j, gget(carry_sa(CY) + cc.sa_off + j));
    if (isVH && cr.n_vh > 0) {
      for (uint32_t j = 0; j + 1 < cr.n_vh; j++) gput(vh + j, gget(carry_vh(CY) + cc.vh_off + j));
      const cdr_vh_item it = gget(carry_vh(CY) + cc.vh_off + cr.n_vh - 1);
      n_vh = cr.n_vh;
      vh_last_id = it.event_id;
      vh_last_ver = it.version;
      // cdr_carry.in_memory: the rebuilt builder nDCConflictResolver.rebuild returns
      // (nDCConflictResolver.go:117-184) never went through Load — its currentVersion is
      // what the rebuild's replay left, its last version-history item's version
      if (CY->in_memory && CY->in_memory[w]) curv = vh_last_ver;
    }
    hw_chi = live_chi = cr.n_child;
    for (uint32_t j = 0; j < hw_chi; j++) gput(chi + j, gget(gp(CY->state.child) + cc.child_off + j));
    hw_can = live_can = cr.n_cancel;
    for (uint32_t j = 0; j < hw_can; j++) gput(can + j, gget(gp(CY->state.cancel) + cc.cancel_off + j));
    hw_sig = live_sig = cr.n_signal;
    for (uint32_t j = 0; j < hw_sig; j++) gput(sig + j, gget(gp(CY->state.signal) + cc.signal_off + j));
    // user timers: every field lives in the working slot
    hw_tim = cr.n_timer;
    for (uint32_t j = 0; j < hw_tim; j++) {
      const cdr_timer_info t = gget(gp(CY->state.timer) + cc.timer_off + j);
      T.st(j, TP_SID, t.started_id);
      T.st(j, TP_TID_TASK, (int64_t)(t.timer_id | ((uint64_t)t.task_id << 32)));
      T.st(j, TP_EXPIRY, t.expiry_time);
      T.st(j, TP_VER, t.version);
    }
    // activities: the slot carries what the replay reads or changes; AP_ROWS names the
    // loaded row (AP_CARRIED) for the rest, read again at emission.  The timer
    // candidates follow loadActivityTimers (timerBuilder.go:249-312) on loaded values.
    hw_act = cr.n_activity;
    for (uint32_t j = 0; j < hw_act; j++) {
      const cdr_activity_info a = gget(gp(CY->state.act) + cc.act_off + j);
      const bool started = a.started_id != CDR_EMPTY_EVENT_ID;
      const int64_t s2c = a.scheduled_time + (int64_t)a.s2c * NS_PER_S;
      // StartedTime / LastHeartBeatUpdatedTime are Go zero times unless the flag is set
      const bool tset = (a.flags & CDR_AI_STARTED_TIME_SET) != 0;
      const int64_t st = tset ? a.started_time : 0, hb0 = tset ? a.last_heartbeat_time : 0;
      const int64_t lhb = hb0 > st ? hb0 : st;
      bool map = true;  // byActivityID: the largest scheduleID of an activityID holds it (Load's map order)
      for (uint32_t i = 0; i < hw_act; i++) {
        const cdr_activity_info b = gget(gp(CY->state.act) + cc.act_off + i);
        map = map && !(i != j && b.activity_id == a.activity_id && b.schedule_id > a.schedule_id);
      }
      A.st(j, AP_SID, a.schedule_id);
      A.st(j, AP_TS2C, a.expiration_time < s2c ? a.expiration_time : s2c);
      A.st(j, AP_TALT, started ? st + (int64_t)a.stc * NS_PER_S
                               : a.scheduled_time + (int64_t)a.s2s * NS_PER_S);
      A.st(j, AP_THB, started && a.hb > 0 ? lhb + (int64_t)a.hb * NS_PER_S : T_NONE);
      A.st(j, AP_META, (int64_t)(a.activity_id | (map ? META_FLAG(AF_AIDMAP) : 0ull) |
                                 (started ? META_FLAG(AF_STARTED) : 0ull) |
                                 ((a.flags & CDR_AI_CANCEL_REQUESTED) ? META_FLAG(AF_CANCEL) : 0ull) |
                                 ((uint64_t)(a.timer_task_status & 0xFF) << META_TTS_SHIFT)));
      A.st(j, AP_VER, a.version);
      A.st(j, AP_STARTED_ID, a.started_id);
      A.st(j, AP_STARTED_TIME, st);
      A.st(j, AP_CANCEL_ID, a.cancel_request_id);
      A.st(j, AP_ROWS, (int64_t)(AP_CARRIED | j));
      A.st(j, AP_STC_HB, (int64_t)((uint32_t)a.stc | ((uint64_t)(uint32_t)a.hb << 32)));
      A.st(j, AP_REQ, (int64_t)a.request_id);
    }
  }

  // ---- transfer / timer tasks (stateBuilder.go:613-804), when the caller asks for
  // them (cdr_out.transfer != NULL): appended in generation order to the entry's slices
  constexpr bool TK = TASKS;  // instantiated without task code for the common case
  uint32_t n_xt = 0, n_tt = 0, xt_cap = 0, tt_cap = 0;
  if (TK) {
    xt_cap = CP.xfer_cap;
    tt_cap = CP.ttask_cap;
  }
  auto task_x = [&](bool c, uint32_t type, int64_t eid, uint32_t dom, uint32_t tl, uint32_t twf, uint32_t trun,
                    uint32_t fl) {
    c = c && n_xt < xt_cap;
    if (c) {
      cdr_task t;
      t.type = type;
      t.timeout_type = 0;
      t.event_id = eid;
      t.visibility_ts = 0;
      t.attempt = 0;
      t.domain_id = dom;
      t.task_list = tl;
      t.target_workflow_id = twf;
      t.target_run_id = trun;
      t.flags = fl;
      t._pad = 0;
      t.version = 0;  // stateBuilder's tasks leave Version to the caller (schema.h cdr_task)
      gput(gp(O_.transfer) + CP.xfer_off + n_xt, t);
    }
    n_xt += c ? 1u : 0u;
  };
  auto task_t = [&](bool c, uint32_t type, int32_t tt, int64_t eid, int64_t vis, int64_t att) {
    c = c && n_tt < tt_cap;
    if (c) {
      cdr_task t;
      t.type = type;
      t.timeout_type = tt;
      t.event_id = eid;
      t.visibility_ts = vis;
      t.attempt = att;
      t.domain_id = t.task_list = t.target_workflow_id = t.target_run_id = t.flags = t._pad = 0;
      t.version = 0;
      gput(gp(O_.timer_tasks) + CP.ttask_off + n_tt, t);
    }
    n_tt += c ? 1u : 0u;
  };
  // ExecutionInfo.TaskList as of now (getTaskList, stateBuilder.go:789-794)
  auto task_list_now = [&]() -> uint32_t { return ((x_flags & CDR_XI_STARTED) || csrc >= 0) ? X->task_list : 0u; };
  // ActivityTimeoutTask: the activity timer pick's task (Attempt: 0 unless loaded)
  auto act_task = [&](const Pick& p) {
    if (!(TK && p.made)) return;
    int64_t att = 0;
    const uint64_t rows = (uint64_t)A.ld((uint32_t)p.slot, AP_ROWS);
    if (rows & AP_CARRIED) {
      const GAS cdr_carry* CY = gp(B_.carry);
      att = gget(gp(CY->state.act) + gget(gp(CY->caps) + csrc).act_off + (uint32_t)rows).attempt;
    }
    task_t(true, CDR_TT_ACTIVITY_TIMEOUT, p.timeout_type, p.event_id, p.vis, att);
  };
  auto tim_task = [&](const Pick& p) { task_t(TK && p.made, CDR_TT_USER_TIMER, 0, p.event_id, p.vis, 0); };
  // appendTasksForFinishedExecutions (:775-787)
  auto close_tasks = [&](bool c, int64_t ts) {
    task_x(TK && c, CDR_TT_CLOSE_EXECUTION, 0, 0, 0, 0, 0, 0);
    task_t(TK && c, CDR_TT_DELETE_HISTORY, 0, 0, ts + (int64_t)D.retention_days * 86400ll * NS_PER_S, 0);
  };

  // ---- software pipeline: operands of event k+CDR_DEPTH and the type of event
  // k+CDR_DEPTH+2 are issued while event k is processed
#if CDR_DEPTH == 2
  Ev q0 = load_ops(S, el8(0, len, lane), load_tf(S, el8(0, len, lane)));
  Ev q1 = load_ops(S, el8(1, len, lane), load_tf(S, el8(1, len, lane)));
  uint32_t t2 = load_tf(S, el8(2, len, lane)), t3 = load_tf(S, el8(3, len, lane));
#else
  Ev q0 = load_ops(S, el8(0, len, lane), load_tf(S, el8(0, len, lane)));
  uint32_t t1 = load_tf(S, el8(1, len, lane)), t2 = load_tf(S, el8(2, len, lane));
#endif
  const uint32_t vh_cap = CP.vh_cap;
  bool done = len == 0;  // the lane stopped (end of a failed call) or ran out of events

  // Control flow below is wave-uniform (the step loop runs to the slice length, the
  // dispatch loop over the event types present in the wave); per-lane effects on the
  // register state are selects and only memory side effects are lane-masked.  This
  // keeps the compiler from structurising a divergent CFG around ~80 live registers.
#define SEL(c, a, b) ((c) ? (a) : (b))
#define PFAIL(cond, code)               \
  do {                                  \
    const bool f_ = (cond);             \
    err = SEL(f_, (int32_t)(code), err); \
    err_id = SEL(f_, e.id, err_id);     \
    err_k = SEL(f_, k, err_k);          \
    stop_at_call_end |= f_;             \
  } while (0)
  // lastDecision: the record of a pending source event, before a clearing event
#define GLD_CAPTURE(mine_)                                                                                 \
  do {                                                                                                     \
    const bool c_ = (mine_) && ld_pending(ld);                                                             \
    if (c_ && want_ld)                                                                                     \
      ld_write(gp(O_.last_decision) + w, ld, dv, dsched, dstart, dreq, dto, datt, dsc_ts, dst_ts, dorig_ts); \
    ld |= c_ ? LD_CAPTURED : 0u;                                                                           \
  } while (0)
  const uint32_t srows = S.elems / CDR_SLICE_WIDTH;
  for (uint32_t k = 0; k < srows; k++) {
    if (__builtin_amdgcn_ballot_w64(!done) == 0) break;  // every lane finished
    const Ev e = q0;
#if CDR_DEPTH == 2
    q0 = q1;
    const uint32_t t4 = load_tf(S, el8(k + 4, len, lane));
    q1 = load_ops(S, el8(k + 2, len, lane), t2);
    t2 = t3;
    t3 = t4;
#else
    const uint32_t t3 = load_tf(S, el8(k + 3, len, lane));
    q0 = load_ops(S, el8(k + 1, len, lane), t1);
    t1 = t2;
    t2 = t3;
#endif
    done |= k >= len;
    const uint32_t type = e.tf & 0xFFu;
    // ---- call boundary: end of the previous call (stateBuilder.go:603-604), plus the
    // replication state whose source is the call's last event (mutableStateBuilder.go:561-581)
    const bool bf = !done && ((e.tf & CDR_SEF_BATCH_FIRST) || k == 0);
    const bool end_call = bf && k > 0;
    if (isRS && end_call) {  // 2DC only; lane-masked block (rare)
      const int src = cluster_for_version(B_.cluster, prev_ver);
      if (src < 0) {  // the panic fires at the call's first event, before anything else
        err = CDR_P_UNKNOWN_CLUSTER;
        err_id = call_first_id;
        err_k = call_first_k;
        newrun_applied = newrun_applied && nr_call != call_idx;
      } else if (src != B_.cluster.current_cluster) {
        RS->lri_version[src] = prev_ver;
        RS->lri_last_event_id[src] = prev_id;
        rs_mask |= 1u << src;
      }
    }
    done |= end_call && err != CDR_OK;  // a failed call ends the replay (the Go caller returns)
    const bool nxt_call = end_call && !done;
    x_next_event = SEL(nxt_call, prev_id + 1, x_next_event);
    call_idx += nxt_call ? 1u : 0u;
    const bool start_call = bf && !done;
    call_first_id = SEL(start_call, e.id, call_first_id);
    call_first_k = SEL(start_call, k, call_first_k);
    ld = SEL(start_call, 0u, ld);
    prev_id = SEL(done, prev_id, e.id);
    prev_ver = SEL(done, prev_ver, e.ver);
    bool go = !done && !stop_at_call_end;  // rest of a failed call: only its last event matters (2DC)

    // ---- version prelude (stateBuilder.go:134-154); 2DC: UpdateReplicationStateVersion
    // (v, true) leaves CurrentVersion = e.ver, read back from prev_ver at the end
    if (isVH) {
      const bool gv = go;
      curv = SEL(gv && (x_state == CDR_STATE_CREATED || x_state == CDR_STATE_RUNNING), e.ver, curv);
      // NewVersionHistoryItem + AddOrUpdateItem (versionHistory.go:31-42,203-236)
      const bool newitem = n_vh == 0 || e.ver > vh_last_ver;
      const int32_t code = (e.id < 0 || (e.ver < 0 && e.ver != CDR_EMPTY_VERSION)) ? CDR_P_VH_ITEM_INVALID
                           : (n_vh != 0 && e.ver < vh_last_ver)                     ? CDR_E_VH_LOWER_VERSION
                           : (n_vh != 0 && e.id <= vh_last_id)                      ? CDR_E_VH_LOWER_EVENT_ID
                           : (newitem && n_vh >= vh_cap)                            ? CDR_E_BAD_INPUT
                                                                                    : CDR_OK;
      const bool f = gv && code != CDR_OK;
      PFAIL(f, code);
      go = go && !f;
      const bool add = go && newitem;
      if (add && n_vh != 0) gput(vh + (n_vh - 1), cdr_vh_item{vh_last_id, vh_last_ver});  // close the previous item
      n_vh += add ? 1u : 0u;
      vh_last_ver = SEL(add, e.ver, vh_last_ver);
      vh_last_id = SEL(go, e.id, vh_last_id);
    }
    // LastEventTaskID (:155) is read once after the loop (last applied event)

    // ---- dispatch (stateBuilder.go:157-600): one pass per distinct event type among
    // the lanes that apply an event; the type of each pass is wave-uniform, so the
    // switch is a scalar branch tree and a pass executes only its own case
    for (uint64_t pend = __builtin_amdgcn_ballot_w64(go); pend;) {
      uint32_t ut = __builtin_amdgcn_readlane(type, __builtin_ctzll(pend));
      asm volatile("" : "+s"(ut));  // keep the switch on the SGPR copy
      // register-only types (signals, the decision schedule/start, no-ops, cancel
      // request) share one pass: each lane applies its own type's selects
      const bool simple = ((SIMPLE_TYPES >> ut) & 1ull) != 0;
      const bool mine = go && (simple ? ((SIMPLE_TYPES >> type) & 1ull) != 0 : type == ut);
      pend &= ~__builtin_amdgcn_ballot_w64(mine);
      if (simple) {
        const bool ms = mine && type == CDR_EV_DT_SCHEDULED;  // :186-200 -> :143-167
        dv = SEL(ms, e.ver, dv);
        dsched = SEL(ms, e.id, dsched);
        dstart = SEL(ms, CDR_EMPTY_EVENT_ID, dstart);
        dreq = SEL(ms, EU, dreq);
        dto = SEL(ms, e.n, dto);
        datt = SEL(ms, e.aux, datt);
        dsc_ts = SEL(ms, e.ts, dsc_ts);
        dst_ts = SEL(ms, (int64_t)0, dst_ts);
        dorig_ts = SEL(ms, e.ts, dorig_ts);
        ld = SEL(ms, ld_make(CDR_LD_SCHEDULED, k), ld);
        task_x(TK && ms, CDR_TT_DECISION, e.id, D.domain_id, task_list_now(), 0, 0, 0);  // :196-197
        const bool mt = mine && type == CDR_EV_DT_STARTED;  // :202-213 -> :200-253
        const bool f = mt && e.key != dsched;
        PFAIL(f, CDR_E_DECISION_NOT_FOUND);
        const bool ok = mt && !f;
        x_state = SEL(ok && x_state == CDR_STATE_CREATED, (int32_t)CDR_STATE_RUNNING, x_state);  // (:56-60)
        dv = SEL(ok, e.ver, dv);
        dstart = SEL(ok, e.id, dstart);
        dreq = SEL(ok, e.h, dreq);
        datt = SEL(ok, (int64_t)0, datt);
        dst_ts = SEL(ok, e.ts, dst_ts);
        ld = SEL(ok, ld_make(CDR_LD_STARTED, k), ld);
        task_t(TK && ok, CDR_TT_DECISION_TIMEOUT, CDR_TIMEOUT_START_TO_CLOSE, e.key, e.ts + (int64_t)dto * NS_PER_S, 0);
        x_signals += (mine && type == CDR_EV_WF_SIGNALED) ? 1 : 0;                           // :473-476
        x_flags |= (mine && type == CDR_EV_WF_CANCEL_REQUESTED) ? CDR_XI_CANCEL_REQUESTED : 0u;  // :478-481
        continue;  // MarkerRecorded, CancelTimerFailed, RequestCancelActivityTaskFailed: no-ops
      }
      switch (ut) {
        case CDR_EV_WF_STARTED: {  // stateBuilder.go:158-184 -> mutableStateBuilder.go:1639-1716
          GLD_CAPTURE(mine);  // a later Started resets the decision fields
          // every lane reads a valid record (the first one for lanes of other types)
          const GAS cdr_attr_wf_started* a =
              gp((const cdr_attr_wf_started*)(B_.ev.arena + (uint64_t)(mine ? e.aux : 0)));
          const uint32_t af = a->flags;
          const bool f1 = mine && (af & CDR_SF_HAS_PARENT_DOMAIN) && (af & CDR_SF_PARENT_DOMAIN_MISSING);
          const bool f2 = mine && !f1 && !transition_ok(x_state, x_close, CDR_STATE_CREATED, CDR_CLOSE_NONE);
          PFAIL(f1, CDR_E_DOMAIN_NOT_FOUND);
          PFAIL(f2, CDR_E_INVALID_STATE_TRANSITION);
          const bool ok = mine && !f1 && !f2;
          const bool first = !(x_flags & CDR_XI_STARTED);  // fields absent from a first Started stay zero
          uint32_t nrp = n_rp, nsa = n_sa, xf = x_flags;
          if (ok) {  // output-record side effects (lane-masked)
            X->domain_id = D.domain_id;
            X->workflow_id = D.workflow_id;
            X->run_id = D.run_id;
            X->create_request_id = D.request_id;
            X->task_list = a->task_list;
            X->workflow_type = a->workflow_type;
            X->workflow_timeout = a->exec_timeout_s;
            X->cron_schedule = a->cron_schedule;
            X->attempt = a->attempt;
            X->initiated_id = (af & CDR_SF_HAS_PARENT_INITIATED) ? a->parent_initiated_id : CDR_EMPTY_EVENT_ID;
            if (af & CDR_SF_HAS_PARENT_DOMAIN) X->parent_domain_id = a->parent_domain_id;
            else if (first) X->parent_domain_id = 0;
            if (af & CDR_SF_HAS_PARENT_EXEC) {
              X->parent_workflow_id = a->parent_workflow_id;
              X->parent_run_id = a->parent_run_id;
            } else if (first) {
              X->parent_workflow_id = 0;
              X->parent_run_id = 0;
            }
            if (a->expiration_ts != 0) {
              X->expiration_time = a->expiration_ts;
              xf |= CDR_XI_HAS_EXPIRATION;
            } else if (first) {
              X->expiration_time = 0;
            }
            if (af & CDR_SF_HAS_RETRY) {
              xf |= CDR_XI_HAS_RETRY;
              X->backoff_coefficient = a->backoff_coefficient;
              X->expiration_seconds = a->retry_expiration_s;
              X->initial_interval = a->retry_initial_s;
              X->maximum_attempts = a->retry_max_attempts;
              X->maximum_interval = a->retry_max_interval_s;
              X->nonretriable = a->nonretriable;
            } else if (first) {
              X->backoff_coefficient = 0.0;
              X->expiration_seconds = 0;
              X->initial_interval = 0;
              X->maximum_attempts = 0;
              X->maximum_interval = 0;
              X->nonretriable = 0;
            }
            // rolloverAutoResetPointsWithExpiringTime (:3184-3205)
            nrp = 0;
            xf &= ~CDR_XI_HAS_RESET_POINTS;
            if (af & CDR_SF_HAS_RESET_POINTS) {
              xf |= CDR_XI_HAS_RESET_POINTS;
              const int64_t expiring = e.ts + (int64_t)D.retention_days * 24ll * 3600ll * NS_PER_S;
              const uint32_t crun = a->continued_run_id, off = a->reset_points_off, cnt = a->reset_points_len;
              const uint32_t cap = CP.rp_cap;
              for (uint32_t q = 0; q < cnt && q < cap; q++) {
                cdr_reset_point p = gget(gp(B_.rps) + (off + q));
                const uint32_t run = (p.flags & CDR_RP_HAS_RUN_ID) ? p.run_id : 0u;
                if (run == crun) {
                  p.flags |= CDR_RP_HAS_EXPIRING;
                  p.expiring_time_nano = expiring;
                }
                gput(rp + nrp++, p);
              }
            }
            if (af & CDR_SF_HAS_MEMO) {
              xf |= CDR_XI_HAS_MEMO;
              X->memo = a->memo;
            } else if (first) {
              X->memo = 0;
            }
            if (af & CDR_SF_HAS_SEARCH_ATTR) {
              nsa = 0;
              const uint32_t off = a->search_attr_off, cnt = a->search_attr_len, cap = CP.sa_cap;
              for (uint32_t q = 0; q < cnt && q < cap; q++) gput(sa + nsa++, gget(gp(B_.kvs) + (off + q)));
              if (nsa) xf |= CDR_XI_HAS_SEARCH_ATTR;
              else xf &= ~CDR_XI_HAS_SEARCH_ATTR;
            }
            xf |= CDR_XI_STARTED | (isVH ? CDR_XI_VH_BRANCH : CDR_XI_HAS_BRANCH);
            // SetHistoryTree (:313-339): branch token on ExecutionInfo, or on the VH for NDC
            uint64_t lo, hi;
            cdr_uuid(B_.uuid_seed, D.wf_key, CDR_UUID_BRANCH, e.id, &lo, &hi);
            X->branch_tree_id = D.run_id;
            X->branch_id_lo = lo;
            X->branch_id_hi = hi;
            if (isRS) RS->start_version = e.ver;  // :182-184
          }
          n_rp = SEL(ok, nrp, n_rp);
          n_sa = SEL(ok, nsa, n_sa);
          x_flags = SEL(ok, xf, x_flags);
          if (TK && ok) {  // scheduleWorkflowTimerTask (:706-735) + RecordWorkflowStartedTask (:614-616)
            const int64_t backoff = (int64_t)a->first_decision_backoff_s * NS_PER_S;
            task_t(backoff != 0, CDR_TT_WORKFLOW_BACKOFF, (af & CDR_SF_CRON_INITIATOR) ? 1 : 0, 0, e.ts + backoff, 0);
            task_t(true, CDR_TT_WORKFLOW_TIMEOUT, 0, 0, e.ts + (int64_t)a->exec_timeout_s * NS_PER_S + backoff, 0);
            task_x(true, CDR_TT_RECORD_STARTED, 0, 0, 0, 0, 0, 0);
          }
          cks_ok = SEL(ok, 0u, cks_ok);
          x_dt_timeout_value = SEL(ok, a->task_timeout_s, x_dt_timeout_value);
          x_state = SEL(ok, (int32_t)CDR_STATE_CREATED, x_state);
          x_close = SEL(ok, (int32_t)CDR_CLOSE_NONE, x_close);
          x_last_processed = SEL(ok, CDR_EMPTY_EVENT_ID, x_last_processed);
          dv = SEL(ok, CDR_EMPTY_VERSION, dv);
          dsched = SEL(ok, CDR_EMPTY_EVENT_ID, dsched);
          dstart = SEL(ok, CDR_EMPTY_EVENT_ID, dstart);
          dreq = SEL(ok, EU, dreq);
          dto = SEL(ok, 0, dto);
          break;
        }
        case CDR_EV_DT_SCHEDULED:  // :186-200 -> mutableStateDecisionTaskManager.go:143-167
          dv = SEL(mine, e.ver, dv);
          dsched = SEL(mine, e.id, dsched);
          dstart = SEL(mine, CDR_EMPTY_EVENT_ID, dstart);
          dreq = SEL(mine, EU, dreq);
          dto = SEL(mine, e.n, dto);
          datt = SEL(mine, e.aux, datt);
          dsc_ts = SEL(mine, e.ts, dsc_ts);
          dst_ts = SEL(mine, (int64_t)0, dst_ts);
          dorig_ts = SEL(mine, e.ts, dorig_ts);
          ld = SEL(mine, ld_make(CDR_LD_SCHEDULED, k), ld);
          task_x(TK && mine, CDR_TT_DECISION, e.id, D.domain_id, task_list_now(), 0, 0, 0);  // :196-197
          break;
        case CDR_EV_DT_STARTED: {  // :202-213 -> :200-253
          const bool f = mine && e.key != dsched;
          PFAIL(f, CDR_E_DECISION_NOT_FOUND);
          const bool ok = mine && !f;
          x_state = SEL(ok && x_state == CDR_STATE_CREATED, (int32_t)CDR_STATE_RUNNING, x_state);  // (:56-60)
          dv = SEL(ok, e.ver, dv);
          dstart = SEL(ok, e.id, dstart);
          dreq = SEL(ok, e.h, dreq);
          datt = SEL(ok, (int64_t)0, datt);
          dst_ts = SEL(ok, e.ts, dst_ts);
          ld = SEL(ok, ld_make(CDR_LD_STARTED, k), ld);
          // scheduleDecisionTimerTask (:210-211; timerBuilder.go:322-331)
          task_t(TK && ok, CDR_TT_DECISION_TIMEOUT, CDR_TIMEOUT_START_TO_CLOSE, e.key, e.ts + (int64_t)dto * NS_PER_S, 0);
          break;
        }
        case CDR_EV_DT_COMPLETED: {  // :215-219 -> :255-262,659-674,789-800
          GLD_CAPTURE(mine);
          dv = SEL(mine, CDR_EMPTY_VERSION, dv);
          dsched = SEL(mine, CDR_EMPTY_EVENT_ID, dsched);
          dstart = SEL(mine, CDR_EMPTY_EVENT_ID, dstart);
          dreq = SEL(mine, EU, dreq);
          dto = SEL(mine, 0, dto);
          datt = SEL(mine, (int64_t)0, datt);
          dst_ts = SEL(mine, (int64_t)0, dst_ts);
          dsc_ts = SEL(mine, (int64_t)0, dsc_ts);  // OriginalScheduledTimestamp kept
          x_last_processed = SEL(mine, e.aux, x_last_processed);
          const uint32_t cks = e.h;
          const bool chk = mine && cks != 0 && cks != cks_ok;
          if (__builtin_amdgcn_ballot_w64(chk)) {  // addBinaryCheckSumIfNotExists (mutableStateBuilder.go:1798-1842)
            bool exists = false;
            for (uint32_t q = 0; chk && q < n_rp; q++) {
              const cdr_reset_point p = gget(rp + q);
              exists |= ((p.flags & CDR_RP_HAS_CHECKSUM) ? p.binary_checksum : 0u) == cks;
            }
            const bool app = chk && !exists;
            const bool f = app && n_rp >= CP.rp_cap;
            PFAIL(f, CDR_E_BAD_INPUT);
            const bool put = app && !f;
            if (put) {
              const bool resettable = live_chi == 0 && live_can == 0 && live_sig == 0;
              cdr_reset_point p;
              p.binary_checksum = cks;
              p.run_id = D.run_id;
              p.first_decision_completed_id = e.id;
              p.created_time_nano = B_.now_ns;
              p.expiring_time_nano = 0;
              p.flags = CDR_RP_HAS_CHECKSUM | CDR_RP_HAS_RUN_ID | CDR_RP_HAS_FIRST_DC_ID | CDR_RP_HAS_CREATED |
                        CDR_RP_HAS_RESETTABLE | (resettable ? CDR_RP_RESETTABLE : 0u);
              p._pad = 0;
              gput(rp + n_rp, p);
            }
            n_rp += put ? 1u : 0u;
            x_flags |= put ? CDR_XI_HAS_RESET_POINTS : 0u;
            cks_ok = SEL(chk && !f, cks, cks_ok);  // the list only grows until the next Started
          }
          break;
        }
        case CDR_EV_DT_TIMED_OUT:  // :221-239 -> FailDecision :635-656 + transient :169-198
        case CDR_EV_DT_FAILED: {   // :241-257
          GLD_CAPTURE(mine);
          const bool inc = ut == CDR_EV_DT_FAILED || e.n != CDR_TIMEOUT_SCHEDULE_TO_START;
          const int64_t now = B_.now_ns;
          const int64_t na = inc ? datt + 1 : 0;
          const bool tr = na != 0;  // transient decision: no decision is pending here by construction
          dv = SEL(mine, tr ? (isRS ? e.ver : (isVH ? curv : CDR_EMPTY_VERSION)) : CDR_EMPTY_VERSION, dv);
          dsched = SEL(mine, tr ? x_next_event : CDR_EMPTY_EVENT_ID, dsched);  // NextEventID as of the call's start
          dstart = SEL(mine, CDR_EMPTY_EVENT_ID, dstart);
          dreq = SEL(mine, EU, dreq);
          dto = SEL(mine, tr ? x_dt_timeout_value : 0, dto);
          dst_ts = SEL(mine, (int64_t)0, dst_ts);
          dorig_ts = SEL(mine, (int64_t)0, dorig_ts);
          dsc_ts = SEL(mine, (tr || inc) ? now : (int64_t)0, dsc_ts);
          datt = SEL(mine, na, datt);
          ld = SEL(mine && tr, ld_make(CDR_LD_TRANSIENT, k), ld);
          task_x(TK && mine && tr, CDR_TT_DECISION, x_next_event, D.domain_id, task_list_now(), 0, 0, 0);  // :235,253
          break;
        }
        case CDR_EV_AT_SCHEDULED: {  // :259-269 -> mutableStateBuilder.go:1982-2028
          const uint32_t aid = (uint32_t)e.key;
          int slot = -1;
          for (uint32_t j = 0; j < act_cap; j++) {
            const bool in = mine && j < hw_act;
            const int64_t sid = A.ld(j, AP_SID);
            const uint64_t m = (uint64_t)A.ld(j, AP_META);
            slot = SEL(in && sid == DEAD_KEY && slot < 0, (int)j, slot);
            // byActivityID[aid] is overwritten: drop the mapping flag of the old holder
            const bool clr = in && sid != DEAD_KEY && (uint32_t)m == aid && (m & META_FLAG(AF_AIDMAP));
            if (clr) A.st(j, AP_META, (int64_t)(m & ~META_FLAG(AF_AIDMAP)));
          }
          const bool grow = mine && slot < 0;
          const bool f = grow && hw_act >= act_cap;
          PFAIL(f, CDR_E_BAD_INPUT);
          const bool ok = mine && !f;
          slot = SEL(grow, (int)hw_act, slot);
          hw_act += (grow && !f) ? 1u : 0u;
          if (ok) {
            const uint32_t j = (uint32_t)slot;
            const int32_t s2c = (int32_t)e.h, s2s = e.n;
            A.st(j, AP_SID, e.id);
            A.st(j, AP_TS2C, e.ts + (int64_t)s2c * NS_PER_S);
            A.st(j, AP_TALT, e.ts + (int64_t)s2s * NS_PER_S);
            A.st(j, AP_THB, T_NONE);
            A.st(j, AP_META, (int64_t)(aid | META_FLAG(AF_AIDMAP)));
            A.st(j, AP_VER, e.ver);
            A.st(j, AP_STARTED_ID, CDR_EMPTY_EVENT_ID);
            A.st(j, AP_STARTED_TIME, 0);
            A.st(j, AP_CANCEL_ID, CDR_EMPTY_EVENT_ID);
            A.st(j, AP_ROWS, (int64_t)(k | ((uint64_t)call_first_k << 32)));
            A.st(j, AP_STC_HB, (int64_t)(((uint64_t)e.key >> 32) | ((uint64_t)e.aux & 0xFFFFFFFF00000000ull)));
            A.st(j, AP_REQ, 0);
          }
          task_x(TK && ok, CDR_TT_ACTIVITY, e.id, D.domain_id, task_list_now(), 0, 0, 0);  // :265-266
          act_task(act_pick_p(A, hw_act, act_cap, ok));
          break;
        }
        case CDR_EV_AT_STARTED: {  // :271-278 -> :2083-2098
          int slot = -1;
          for (uint32_t j = 0; j < act_cap; j++) slot = SEL(mine && j < hw_act && A.ld(j, AP_SID) == e.key, (int)j, slot);
          const bool f = mine && slot < 0;
          PFAIL(f, CDR_P_ACTIVITY_STARTED_NIL);  // nil deref in Go
          const bool ok = mine && !f;
          if (ok) {
            const uint32_t j = (uint32_t)slot;
            const uint64_t th = (uint64_t)A.ld(j, AP_STC_HB);
            const int32_t stc = (int32_t)(uint32_t)th, hb = (int32_t)(uint32_t)(th >> 32);
            A.st(j, AP_VER, e.ver);
            A.st(j, AP_STARTED_ID, e.id);
            A.st(j, AP_REQ, (int64_t)e.h);
            A.st(j, AP_STARTED_TIME, e.ts);  // LastHeartBeatUpdatedTime = StartedTime
            A.st(j, AP_META, (int64_t)((uint64_t)A.ld(j, AP_META) | META_FLAG(AF_STARTED)));
            A.st(j, AP_TALT, e.ts + (int64_t)stc * NS_PER_S);
            A.st(j, AP_THB, hb > 0 ? e.ts + (int64_t)hb * NS_PER_S : T_NONE);
          }
          act_task(act_pick_p(A, hw_act, act_cap, ok));
          break;
        }
        case CDR_EV_AT_COMPLETED:  // :280-305,312-319 -> DeleteActivity :1247-1269
        case CDR_EV_AT_FAILED:
        case CDR_EV_AT_TIMED_OUT:
        case CDR_EV_AT_CANCELED: {
          int slot = -1;
          for (uint32_t j = 0; j < act_cap; j++) slot = SEL(mine && j < hw_act && A.ld(j, AP_SID) == e.key, (int)j, slot);
          const bool f = mine && slot < 0;
          PFAIL(f, CDR_E_ACTIVITY_NOT_FOUND);
          bool ok = mine && !f;
          bool found = false;
          if (ok) {
            const uint64_t m = (uint64_t)A.ld((uint32_t)slot, AP_META);
            const uint32_t aid = (uint32_t)m;
            A.st((uint32_t)slot, AP_SID, DEAD_KEY);
            A.st((uint32_t)slot, AP_META, (int64_t)(m & ~META_FLAG(AF_AIDMAP)));
            found = (m & META_FLAG(AF_AIDMAP)) != 0;
            if (!found)
              for (uint32_t j = 0; j < hw_act; j++) {
                if (A.ld(j, AP_SID) == DEAD_KEY) continue;
                const uint64_t mj = (uint64_t)A.ld(j, AP_META);
                if ((uint32_t)mj == aid && (mj & META_FLAG(AF_AIDMAP))) {
                  A.st(j, AP_META, (int64_t)(mj & ~META_FLAG(AF_AIDMAP)));
                  found = true;
                }
              }
          }
          const bool f2 = ok && !found;
          PFAIL(f2, CDR_E_ACTIVITY_ID_NOT_FOUND);
          ok = ok && !f2;
          act_task(act_pick_p(A, hw_act, act_cap, ok));
          break;
        }
        case CDR_EV_AT_CANCEL_REQUESTED: {  // :307-310 -> :2264-2285
          const uint32_t aid = (uint32_t)e.key;
          int slot = -1;
          for (uint32_t j = 0; j < act_cap; j++) {
            const int64_t sid = A.ld(j, AP_SID);
            const uint64_t mj = (uint64_t)A.ld(j, AP_META);
            slot = SEL(mine && j < hw_act && sid != DEAD_KEY && (uint32_t)mj == aid && (mj & META_FLAG(AF_AIDMAP)),
                       (int)j, slot);
          }
          const bool f = mine && slot < 0;
          PFAIL(f, CDR_E_MISSING_ACTIVITY_INFO);
          if (mine && !f) {
            const uint32_t j = (uint32_t)slot;
            A.st(j, AP_VER, e.ver);
            A.st(j, AP_META, (int64_t)((uint64_t)A.ld(j, AP_META) | META_FLAG(AF_CANCEL)));
            A.st(j, AP_CANCEL_ID, e.id);
          }
          break;
        }
        case CDR_EV_TIMER_STARTED: {  // :324-332 -> :2877-2900
          const uint32_t tid = (uint32_t)e.key;
          int slot = -1, free_slot = -1;
          for (uint32_t j = 0; j < tim_cap; j++) {
            const bool in = mine && j < hw_tim;
            const int64_t sid = T.ld(j, TP_SID);
            const uint32_t tj = (uint32_t)T.ld(j, TP_TID_TASK);
            free_slot = SEL(in && sid == DEAD_KEY && free_slot < 0, (int)j, free_slot);
            slot = SEL(in && sid != DEAD_KEY && tj == tid, (int)j, slot);
          }
          slot = slot < 0 ? free_slot : slot;
          const bool grow = mine && slot < 0;
          const bool f = grow && hw_tim >= tim_cap;
          PFAIL(f, CDR_E_BAD_INPUT);
          const bool ok = mine && !f;
          slot = SEL(grow, (int)hw_tim, slot);
          hw_tim += (grow && !f) ? 1u : 0u;
          if (ok) {
            const uint32_t j = (uint32_t)slot;
            T.st(j, TP_SID, e.id);
            T.st(j, TP_TID_TASK, (int64_t)tid);  // TaskID = TimerTaskStatusNone
            T.st(j, TP_EXPIRY, e.ts + e.aux * NS_PER_S);
            T.st(j, TP_VER, e.ver);
          }
          tim_task(tim_pick_p(T, hw_tim, tim_cap, ok));
          break;
        }
        case CDR_EV_TIMER_FIRED:       // :334-341
        case CDR_EV_TIMER_CANCELED: {  // :343-350
          const uint32_t tid = (uint32_t)e.key;
          for (uint32_t j = 0; j < tim_cap; j++) {
            const bool hit = mine && j < hw_tim && T.ld(j, TP_SID) != DEAD_KEY && (uint32_t)T.ld(j, TP_TID_TASK) == tid;
            if (hit) T.st(j, TP_SID, DEAD_KEY);
          }
          tim_task(tim_pick_p(T, hw_tim, tim_cap, mine));
          break;
        }
        case CDR_EV_CHILD_INITIATED: {  // :355-371 -> :3256-3280
          int slot = -1;
          if (mine) slot = alloc_initiated(chi, hw_chi, CP.child_cap);
          const bool f = mine && slot < 0;
          PFAIL(f, CDR_E_BAD_INPUT);
          const bool ok = mine && !f;
          if (ok) {
            cdr_child_info c;
            c.version = e.ver;
            c.initiated_id = e.id;
            c.initiated_event_batch_id = call_first_id;
            c.started_id = CDR_EMPTY_EVENT_ID;
            uint64_t lo, hi;
            cdr_uuid(B_.uuid_seed, D.wf_key, CDR_UUID_CHILD_REQ, e.id, &lo, &hi);
            c.create_request_lo = lo;
            c.create_request_hi = hi;
            c.started_workflow_id = e.h;
            c.started_run_id = 0;
            c.domain_name = (uint32_t)e.key;
            c.workflow_type = (uint32_t)e.aux;
            c.parent_close_policy = e.n;
            c._pad = 0;
            gput(chi + slot, c);
          }
          live_chi += ok ? 1u : 0u;
          PFAIL(ok && (e.tf & CDR_SEF_DOMAIN_MISSING), CDR_E_DOMAIN_NOT_FOUND);
          if (TK && ok && !(e.tf & CDR_SEF_DOMAIN_MISSING)) {  // scheduleStartChildWorkflowTransferTask (:370-371)
            const cdr_attr_external xa = gget(gp((const cdr_attr_external*)(B_.ev.arena + ((uint64_t)e.key >> 32))));
            task_x(true, CDR_TT_START_CHILD, e.id, xa.target_domain_id, 0, xa.workflow_id, 0, 0);
          }
          break;
        }
        case CDR_EV_CHILD_STARTED: {  // :378-381 -> :3312-3325
          int slot = -1;
          if (mine) slot = find_initiated(chi, hw_chi, e.key);
          const bool f = mine && slot < 0;
          PFAIL(f, CDR_P_CHILD_STARTED_NIL);
          if (mine && !f) {
            chi[slot].started_id = e.id;
            chi[slot].started_run_id = e.h;
          }
          break;
        }
        case CDR_EV_CHILD_START_FAILED:
        case CDR_EV_CHILD_COMPLETED:
        case CDR_EV_CHILD_FAILED:
        case CDR_EV_CHILD_CANCELED:
        case CDR_EV_CHILD_TIMED_OUT:
        case CDR_EV_CHILD_TERMINATED: {  // DeletePendingChildExecution :1138-1144
          int slot = -1;
          if (mine) slot = find_initiated(chi, hw_chi, e.key);
          if (slot >= 0) chi[slot].initiated_id = DEAD_KEY;
          live_chi -= slot >= 0 ? 1u : 0u;
          break;
        }
        case CDR_EV_RCE_INITIATED: {  // :408-427 -> :2577-2596
          int slot = -1;
          if (mine) slot = alloc_initiated(can, hw_can, CP.cancel_cap);
          const bool f = mine && slot < 0;
          PFAIL(f, CDR_E_BAD_INPUT);
          const bool ok = mine && !f;
          if (ok) {
            cdr_cancel_info c;
            c.version = e.ver;
            c.initiated_event_batch_id = call_first_id;
            c.initiated_id = e.id;
            uint64_t lo, hi;
            cdr_uuid(B_.uuid_seed, D.wf_key, CDR_UUID_CANCEL_REQ, e.id, &lo, &hi);
            c.cancel_request_lo = lo;
            c.cancel_request_hi = hi;
            gput(can + slot, c);
          }
          live_can += ok ? 1u : 0u;
          PFAIL(ok && (e.tf & CDR_SEF_DOMAIN_MISSING), CDR_E_DOMAIN_NOT_FOUND);
          if (TK && ok && !(e.tf & CDR_SEF_DOMAIN_MISSING)) {  // scheduleCancelExternalWorkflowTransferTask (:421-427)
            const cdr_attr_external xa = gget(gp((const cdr_attr_external*)(B_.ev.arena + ((uint64_t)e.key >> 32))));
            task_x(true, CDR_TT_CANCEL_EXECUTION, e.id, xa.target_domain_id, 0, xa.workflow_id, xa.run_id,
                   (xa.flags & CDR_XF_CHILD_ONLY) ? CDR_TF_CHILD_ONLY : 0u);
          }
          break;
        }
        case CDR_EV_RCE_FAILED:
        case CDR_EV_EXT_CANCEL_REQUESTED: {  // DeletePendingRequestCancel :1147-1153
          int slot = -1;
          if (mine) slot = find_initiated(can, hw_can, e.key);
          if (slot >= 0) can[slot].initiated_id = DEAD_KEY;
          live_can -= slot >= 0 ? 1u : 0u;
          break;
        }
        case CDR_EV_SE_INITIATED: {  // :439-458 -> :2701-2723
          int slot = -1;
          if (mine) slot = alloc_initiated(sig, hw_sig, CP.signal_cap);
          const bool f = mine && slot < 0;
          PFAIL(f, CDR_E_BAD_INPUT);
          const bool ok = mine && !f;
          if (ok) {
            cdr_signal_info c;
            c.version = e.ver;
            c.initiated_event_batch_id = call_first_id;
            c.initiated_id = e.id;
            uint64_t lo, hi;
            cdr_uuid(B_.uuid_seed, D.wf_key, CDR_UUID_SIGNAL_REQ, e.id, &lo, &hi);
            c.signal_request_lo = lo;
            c.signal_request_hi = hi;
            c.signal_name = e.h;
            c.input = (uint32_t)((uint64_t)e.aux >> 32);
            c.control = (uint32_t)e.aux;
            c._pad = 0;
            gput(sig + slot, c);
          }
          live_sig += ok ? 1u : 0u;
          PFAIL(ok && (e.tf & CDR_SEF_DOMAIN_MISSING), CDR_E_DOMAIN_NOT_FOUND);
          if (TK && ok && !(e.tf & CDR_SEF_DOMAIN_MISSING)) {  // scheduleSignalWorkflowTransferTask (:452-458)
            const cdr_attr_external xa = gget(gp((const cdr_attr_external*)(B_.ev.arena + ((uint64_t)e.key >> 32))));
            task_x(true, CDR_TT_SIGNAL_EXECUTION, e.id, xa.target_domain_id, 0, xa.workflow_id, xa.run_id,
                   (xa.flags & CDR_XF_CHILD_ONLY) ? CDR_TF_CHILD_ONLY : 0u);
          }
          break;
        }
        case CDR_EV_SE_FAILED:
        case CDR_EV_EXT_SIGNALED: {  // DeletePendingSignal :1156-1162
          int slot = -1;
          if (mine) slot = find_initiated(sig, hw_sig, e.key);
          if (slot >= 0) sig[slot].initiated_id = DEAD_KEY;
          live_sig -= slot >= 0 ? 1u : 0u;
          break;
        }
        case CDR_EV_AT_REQ_CANCEL_FAILED:
        case CDR_EV_CANCEL_TIMER_FAILED:
        case CDR_EV_MARKER_RECORDED:
          break;
        case CDR_EV_WF_SIGNALED:  // :473-476
          x_signals += mine ? 1 : 0;
          break;
        case CDR_EV_WF_CANCEL_REQUESTED:  // :478-481
          x_flags |= mine ? CDR_XI_CANCEL_REQUESTED : 0u;
          break;
        case CDR_EV_WF_COMPLETED:
        case CDR_EV_WF_FAILED:
        case CDR_EV_WF_TIMED_OUT:
        case CDR_EV_WF_CANCELED:
        case CDR_EV_WF_TERMINATED: {  // :483-531
          const int cs = ut == CDR_EV_WF_COMPLETED   ? CDR_CLOSE_COMPLETED
                         : ut == CDR_EV_WF_FAILED    ? CDR_CLOSE_FAILED
                         : ut == CDR_EV_WF_TIMED_OUT ? CDR_CLOSE_TIMED_OUT
                         : ut == CDR_EV_WF_CANCELED  ? CDR_CLOSE_CANCELED
                                                     : CDR_CLOSE_TERMINATED;
          const bool f = mine && !transition_ok(x_state, x_close, CDR_STATE_COMPLETED, cs);
          PFAIL(f, CDR_E_INVALID_STATE_TRANSITION);
          const bool ok = mine && !f;
          x_state = SEL(ok, (int32_t)CDR_STATE_COMPLETED, x_state);
          x_close = SEL(ok, (int32_t)cs, x_close);
          x_completion_batch = SEL(ok, call_first_id, x_completion_batch);
          close_tasks(ok, e.ts);
          break;
        }
        case CDR_EV_UPSERT_SA: {  // :533-535 -> :2746-2768
          uint32_t nsa = n_sa;
          if (mine) {
            const uint64_t off = (uint64_t)e.aux;
            const uint32_t cnt = e.h, cap = CP.sa_cap;
            for (uint32_t q = 0; q < cnt; q++) {
              const cdr_kv kv = gget(gp(B_.kvs) + (off + q));
              bool found = false;
              for (uint32_t j = 0; j < nsa; j++)
                if (sa[j].key == kv.key) {
                  sa[j].value = kv.value;
                  found = true;
                }
              if (!found && nsa < cap) gput(sa + nsa++, kv);
            }
          }
          n_sa = SEL(mine, nsa, n_sa);
          x_flags |= mine ? CDR_XI_HAS_SEARCH_ATTR : 0u;
          task_x(TK && mine, CDR_TT_UPSERT_SA, 0, 0, 0, 0, 0, 0);  // :535
          break;
        }
        case CDR_EV_WF_CONTINUED_AS_NEW: {  // :537-595
          bool empty = true;
          if (mine) {
            const int32_t nr = D.newrun;
            empty = nr < 0 || call_idx != D.newrun_call || gp(B_.wfs)[nr].ev_len == 0;
          }
          const bool f = mine && empty;
          PFAIL(f, CDR_E_NEWRUN_HISTORY_EMPTY);
          const bool ap = mine && !f;
          newrun_applied |= ap;  // the new run replays in its own lane; k_finalize joins
          nr_call = ap ? call_idx : nr_call;
          const bool f2 = ap && !transition_ok(x_state, x_close, CDR_STATE_COMPLETED, CDR_CLOSE_CONTINUED_AS_NEW);
          PFAIL(f2, CDR_E_INVALID_STATE_TRANSITION);
          const bool ok = ap && !f2;
          x_state = SEL(ok, (int32_t)CDR_STATE_COMPLETED, x_state);
          x_close = SEL(ok, (int32_t)CDR_CLOSE_CONTINUED_AS_NEW, x_close);
          x_completion_batch = SEL(ok, call_first_id, x_completion_batch);
          close_tasks(ok, e.ts);  // :592
          break;
        }
        default:
          PFAIL(mine, CDR_E_UNKNOWN_EVENT_TYPE);  // :597-599
          break;
      }
    }
  }
#undef PFAIL
#undef SEL
#undef GLD_CAPTURE
  // ---- end of the last call
  if (len > 0 && (err == CDR_OK || stop_at_call_end)) {
    if (isRS) {
      const int src = cluster_for_version(B_.cluster, prev_ver);
      if (src < 0) {
        err = CDR_P_UNKNOWN_CLUSTER;
        err_id = call_first_id;
        err_k = call_first_k;
        newrun_applied = newrun_applied && nr_call != call_idx;
      } else if (src != B_.cluster.current_cluster && err == CDR_OK) {
        RS->lri_version[src] = prev_ver;
        RS->lri_last_event_id[src] = prev_id;
        rs_mask |= 1u << src;
      }
    }
    if (err == CDR_OK) x_next_event = prev_id + 1;
  }
  if (err == CDR_OK && D.parent < 0 && D.expected_next_event_id != 0 && x_next_event != D.expected_next_event_id) {
    err = CDR_E_REBUILD_NEXT_EVENT_ID;  // nDCStateRebuilder.go:139-143
    err_id = prev_id;
    err_k = len;
  }

  cdr_wf_result r;
  r.code = err;
  r.flags = (newrun_applied ? CDR_RF_NEWRUN_APPLIED : 0u) | (D.parent >= 0 ? CDR_RF_IS_NEWRUN : 0u);
  r.fail_event_id = err_id;
  r.fail_index = err_k;
  // table high-water marks; k_tables compacts them to live counts (a failed
  // workflow reports no state)
  if (err != CDR_OK) hw_act = hw_tim = hw_chi = hw_can = hw_sig = n_vh = n_rp = n_sa = n_xt = n_tt = 0;
  if (TK) {
    gp(O_.n_tasks)[2 * (uint64_t)w] = n_xt;
    gp(O_.n_tasks)[2 * (uint64_t)w + 1] = n_tt;
  }
  r.n_activity = 0;  // set by the emission below
  r.n_timer = 0;
  r.n_child = hw_chi;
  r.n_cancel = hw_can;
  r.n_signal = hw_sig;
  r.n_vh = n_vh;
  r.n_reset_points = n_rp;
  r.n_search_attr = n_sa;
  if (err == CDR_OK) {
    // emit the live working slots as persisted rows (k_tables orders them by key);
    // fields the loop did not carry are re-read from the scheduling event's row
    GAS cdr_activity_info* act = gp(O_.act) + CP.act_off;
    GAS cdr_timer_info* tim = gp(O_.timer) + CP.timer_off;
    uint32_t n = 0;
    for (uint32_t j = 0; j < hw_act; j++) {
      const int64_t sid = A.ld(j, AP_SID);
      if (sid == DEAD_KEY) continue;
      const uint64_t rows = (uint64_t)A.ld(j, AP_ROWS);
      if (rows & AP_CARRIED) {  // a loaded activity: its row, with what the replay changed
        const GAS cdr_carry* CY = gp(B_.carry);
        const uint32_t ci = (uint32_t)rows;
        cdr_activity_info o = gget(gp(CY->state.act) + gget(gp(CY->caps) + csrc).act_off + ci);
        const uint64_t m = (uint64_t)A.ld(j, AP_META);
        const int64_t st_id = A.ld(j, AP_STARTED_ID);
        if (st_id != o.started_id) {  // ActivityTaskStarted replayed onto it (:2083-2098)
          o.started_time = A.ld(j, AP_STARTED_TIME);
          o.last_heartbeat_time = o.started_time;
          o.flags |= CDR_AI_STARTED_TIME_SET;
        }
        o.version = A.ld(j, AP_VER);
        o.started_id = st_id;
        o.cancel_request_id = A.ld(j, AP_CANCEL_ID);
        o.request_id = (uint32_t)A.ld(j, AP_REQ);
        o.timer_task_status = (int32_t)((m >> META_TTS_SHIFT) & 0xFFu);
        o.flags = (o.flags & ~CDR_AI_CANCEL_REQUESTED) | ((m & META_FLAG(AF_CANCEL)) ? CDR_AI_CANCEL_REQUESTED : 0u);
        gput(act + n++, o);
        continue;
      }
      const uint32_t o_s = el8((uint32_t)rows, len, lane), o_b = el8((uint32_t)(rows >> 32), len, lane);
      const int64_t sched_ts = bld64(S.r, o_s, S.col(CDR_COL_TIMESTAMP));
      const uint32_t arec = (uint32_t)bld64(S.r, o_s, S.col(CDR_COL_AUX));
      const GAS cdr_attr_at_scheduled* a = gp((const cdr_attr_at_scheduled*)(B_.ev.arena + arec));
      const uint64_t m = (uint64_t)A.ld(j, AP_META);
      const bool retry = (a->flags & CDR_AF_HAS_RETRY) != 0;
      const int32_t s2c = a->s2c_s, xs = a->retry_expiration_s;
      cdr_activity_info o;
      o.version = A.ld(j, AP_VER);
      o.schedule_id = sid;
      o.scheduled_event_batch_id = bld64(S.r, o_b, S.col(CDR_COL_EVENT_ID));
      o.scheduled_time = sched_ts;
      o.started_id = A.ld(j, AP_STARTED_ID);
      o.started_time = A.ld(j, AP_STARTED_TIME);
      o.last_heartbeat_time = o.started_time;
      o.expiration_time = sched_ts + (int64_t)((retry && xs > s2c) ? xs : s2c) * NS_PER_S;
      o.cancel_request_id = A.ld(j, AP_CANCEL_ID);
      o.activity_id = (uint32_t)m;
      o.request_id = (uint32_t)A.ld(j, AP_REQ);
      o.task_list = a->task_list;
      o.nonretriable = retry ? a->nonretriable : 0u;
      o.s2s = a->s2s_s;
      o.s2c = s2c;
      o.stc = a->stc_s;
      o.hb = a->hb_s;
      o.timer_task_status = (int32_t)((m >> META_TTS_SHIFT) & 0xFFu);
      o.attempt = 0;
      o.initial_interval = retry ? a->retry_initial_s : 0;
      o.maximum_interval = retry ? a->retry_max_interval_s : 0;
      o.maximum_attempts = retry ? a->retry_max_attempts : 0;
      o.flags = (retry ? CDR_AI_HAS_RETRY : 0u) | ((m & META_FLAG(AF_CANCEL)) ? CDR_AI_CANCEL_REQUESTED : 0u) |
                ((m & META_FLAG(AF_STARTED)) ? CDR_AI_STARTED_TIME_SET : 0u);
      o.backoff_coefficient = retry ? a->backoff_coefficient : 0.0;
      gput(act + n++, o);
    }
    r.n_activity = n;
    n = 0;
    for (uint32_t j = 0; j < hw_tim; j++) {
      const int64_t sid = T.ld(j, TP_SID);
      if (sid == DEAD_KEY) continue;
      const uint64_t tt = (uint64_t)T.ld(j, TP_TID_TASK);
      cdr_timer_info o;
      o.version = T.ld(j, TP_VER);
      o.started_id = sid;
      o.expiry_time = T.ld(j, TP_EXPIRY);
      o.task_id = (int64_t)(tt >> 32);
      o.timer_id = (uint32_t)tt;
      o._pad = 0;
      gput(tim + n++, o);
    }
    r.n_timer = n;
  }
  gput(gp(O_.result) + w, r);
  if (err != CDR_OK) return;
  if (want_ld && !(ld & LD_CAPTURED))
    ld_write(gp(O_.last_decision) + w, ld, dv, dsched, dstart, dreq, dto, datt, dsc_ts, dst_ts, dorig_ts);
  if (n_vh) gput(vh + (n_vh - 1), cdr_vh_item{vh_last_id, vh_last_ver});
  if (!(x_flags & CDR_XI_STARTED) && csrc < 0) {  // no WorkflowExecutionStarted: its fields keep their zero values
    X->domain_id = X->workflow_id = X->run_id = X->create_request_id = 0;
    X->parent_domain_id = X->parent_workflow_id = X->parent_run_id = X->task_list = 0;
    X->workflow_type = X->cron_schedule = X->memo = X->nonretriable = X->branch_tree_id = 0;
    X->initiated_id = 0;
    X->workflow_timeout = X->attempt = X->initial_interval = X->maximum_interval = X->maximum_attempts = 0;
    X->expiration_seconds = 0;
    X->backoff_coefficient = 0.0;
    X->expiration_time = 0;
    X->branch_id_lo = X->branch_id_hi = 0;
  }
  X->decision_request_id = dreq;
  X->flags = x_flags;
  X->_pad0 = 0;
  X->completion_event_batch_id = x_completion_batch;
  X->decision_timeout_value = x_dt_timeout_value;
  X->state = x_state;
  X->close_status = x_close;
  X->last_first_event_id = call_first_id;  // stateBuilder.go:603 of the last call
  // LastEventTaskID (stateBuilder.go:155): every applied event sets it, so an OK
  // workflow ends with its last event's task id
  X->last_event_task_id = bld64(S.r, el8(len - 1, len, lane), S.col(CDR_COL_TASK_ID));
  X->next_event_id = x_next_event;
  X->last_processed_event = x_last_processed;
  X->signal_count = x_signals;
  X->decision_timeout = dto;
  X->decision_version = dv;
  X->decision_schedule_id = dsched;
  X->decision_started_id = dstart;
  X->decision_attempt = datt;
  X->decision_started_ts = dst_ts;
  X->decision_scheduled_ts = dsc_ts;
  X->decision_original_scheduled_ts = dorig_ts;
  X->_pad1 = 0;
  X->reset_points_len = n_rp;
  X->search_attr_len = n_sa;
  if (isRS) {
    RS->current_version = prev_ver;
    if (!(x_flags & CDR_XI_STARTED) && csrc < 0) RS->start_version = D.failover_version;
    RS->last_write_version = prev_ver;
    RS->last_write_event_id = prev_id;
    for (int c = 0; c < CDR_MAX_CLUSTERS; c++)
      if (!(rs_mask & (1u << c))) {
        RS->lri_version[c] = 0;
        RS->lri_last_event_id[c] = 0;
      }
    RS->lri_mask = rs_mask;
    RS->present = 1;
  }  // other builders: ReplicationState is nil and the record is left untouched (schema.h)
#undef D
#undef CP
#undef X
#undef RS
#undef chi
#undef can
#undef sig
#undef vh
#undef rp
#undef sa
#undef B_
#undef O_
}

#include "replay_fast.inc"
#include "replay_wave.inc"
#include "replay_reg.inc"
#include "replay_cls.inc"

// Per-workflow table epilogue: move live rows to the front in key order (the
// canonical order of the Go maps' keys), sort the SearchAttributes map by key, and
// turn high-water marks into live counts.
__global__ __launch_bounds__(256) void k_tables(cdr_dev_batch B, cdr_out O) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= B.n_wfs || (B.skip && B.skip[w])) return;
  cdr_wf_result& r = O.result[w];
  if (r.code != CDR_OK) return;
  const cdr_wf_caps& cp = B.caps[w];
  if (r.flags & RF_ROWS_SORTED) {  // k_replay_cls wrote its rows dense and in key order
    r.flags &= ~RF_ROWS_SORTED;
  } else {
    r.n_activity = compact_sorted(O.act + cp.act_off, r.n_activity, ActKey{});
    r.n_timer = compact_sorted(O.timer + cp.timer_off, r.n_timer, TimerKey{});
    r.n_child = compact_sorted(O.child + cp.child_off, r.n_child, ChildKey{});
    r.n_cancel = compact_sorted(O.cancel + cp.cancel_off, r.n_cancel, CancelKey{});
    r.n_signal = compact_sorted(O.signal + cp.signal_off, r.n_signal, SignalKey{});
  }
  cdr_kv* sa = O.sa + cp.sa_off;
  const uint32_t n = r.n_search_attr;
  for (uint32_t a = 1; a < n; a++) {
    const cdr_kv v = sa[a];
    uint32_t b = a;
    while (b > 0 && sa[b - 1].key > v.key) {
      sa[b] = sa[b - 1];
      b--;
    }
    sa[b] = v;
  }
}

// The class kernels' staged tasks into the entries' task slices (k_replay_cls<TASKS>): one
// workgroup per class slice (launched on the class's stream after its kernel, so that it
// overlaps the other classes' replay), one lane per entry, merging its four class lists (W,
// activity, timer, external — each in history order) by history index, which is the order
// stateBuilder appends them in (getTransferTasks / getTimerTasks, stateBuilder.go:38-52,
// 613-804).  It fills what the class loops left to it (DomainID and TaskList of decision /
// activity tasks, the external initiations' targets from their attributes, the
// DeleteHistoryEvent retention) and writes the records by the wave together (coop_put: 8 whole
// records per store instruction).  Each list keeps its head and the two records after it in
// registers, so a step waits for a load only when one list is taken three times running.  Entries
// without a complete header (handed on to k_replay_reg) are left alone.
struct task_words {
  uint64_t w[8];
};
static_assert(sizeof(cdr_task) == sizeof(task_words), "cdr_task words");
template <uint32_t SFLAG>
__global__ __launch_bounds__(CDR_SLICE_WIDTH) CDR_MERGE_ATTR void k_tasks_merge(cdr_launch L) {
  (void)L;  // read through KA()
  const uint32_t s = blockIdx.x + KA()->s0;
  const uint32_t lane = threadIdx.x;
  if (s >= KA()->B.ev.n_slices) return;
  if (!(__builtin_amdgcn_readfirstlane(KA()->B.ev.slice_flags[s]) & SFLAG)) return;
  const int32_t w = KA()->B.ev.lane_wf[(uint64_t)s * CDR_SLICE_WIDTH + lane];
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  u32x4 h = {0u, 0u, 0u, 0u};
  if (w >= 0) h = *(const u32x4*)(KA()->thead + 8ull * (uint64_t)w);
  const bool valid = (h.x >> 31) != 0;
  if (__builtin_amdgcn_ballot_w64(valid) == 0) return;  // wave-uniform: coop_put needs the wave
  const uint32_t n[4] = {h.x & 0x7FFFFFFFu, h.y, h.z, h.w};
  cdr_wf_caps cp{};
  uint32_t dom = 0, tl = 0;
  int64_t ret = 0;
  if (valid) {
    cp = KA()->B.caps[w];
    dom = KA()->B.wfs[w].domain_id;
    ret = (int64_t)KA()->B.wfs[w].retention_days * 86400ll * NS_PER_S;
    tl = KA()->thead[8ull * (uint64_t)w + 4];
  }
  typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
  const GAS u64x2* const st = (const GAS u64x2*)KA()->tstage;
  const uint64_t sb = 4ull * (cp.xfer_off + cp.ttask_off), sc = (uint64_t)cp.xfer_cap + cp.ttask_cap;
  // record i of list c (w0 with the history index in its high word, event id, value); past
  // the list: key ~0
  struct Rec {
    uint64_t w0;
    int64_t eid, v;
  };
  auto ld = [&](uint32_t c, uint32_t i) -> Rec {
    Rec r{~0ull, 0, 0};
    if (i < n[c]) {
      const uint64_t q = 2ull * (sb + c * sc + i);
      const u64x2 a = st[q], b = st[q + 1];
      r.w0 = a.x;
      r.eid = (int64_t)a.y;
      r.v = (int64_t)b.x;
    }
    return r;
  };
  Rec hd[4], nx[4], n2[4];  // each list's head and the two records after it
  uint32_t cur[4];
#pragma unroll
  for (uint32_t c = 0; c < 4; c++) {
    hd[c] = ld(c, 0);
    nx[c] = ld(c, 1);
    if (!CDR_MERGE_D2) n2[c] = ld(c, 2);
    cur[c] = 0;
  }
  uint32_t n_xt = 0, n_tt = 0;
  bool lost = false;  // a record past the entry's task slice (capacities too small)
  auto key = [](const Rec& r) { return (uint32_t)(r.w0 >> 32); };
  while (__builtin_amdgcn_ballot_w64(valid && (key(hd[0]) & key(hd[1]) & key(hd[2]) & key(hd[3])) != 0xFFFFFFFFu)) {
    // the head with the lowest history index (two lists never tie: an event is in one class)
    uint32_t c = 0, km = key(hd[0]);
#pragma unroll
    for (uint32_t j = 1; j < 4; j++) {
      const bool lt = key(hd[j]) < km;
      c = lt ? j : c;
      km = lt ? key(hd[j]) : km;
    }
    const bool on = valid && km != 0xFFFFFFFFu;
    // the taken head by selects (an indexed pick would put the heads in scratch)
    Rec r;
    r.w0 = c == 0 ? hd[0].w0 : c == 1 ? hd[1].w0 : c == 2 ? hd[2].w0 : hd[3].w0;
    r.eid = c == 0 ? hd[0].eid : c == 1 ? hd[1].eid : c == 2 ? hd[2].eid : hd[3].eid;
    r.v = c == 0 ? hd[0].v : c == 1 ? hd[1].v : c == 2 ? hd[2].v : hd[3].v;
    const uint32_t type = (uint32_t)r.w0 & 0xFFu;
    const bool tim = (r.w0 >> 12) & 1u;
    // the cdr_task record as its eight 8-B words (schema.h layout), kept in registers
    uint32_t t_dom = 0, t_tl = 0, t_wf = 0, t_run = 0, t_fl = 0;
    if (!tim && (type == CDR_TT_DECISION || type == CDR_TT_ACTIVITY)) {  // stateBuilder.go:196-197,265-266
      t_dom = dom;
      t_tl = tl;
    }
    const bool ext = on && !tim &&
                     (type == CDR_TT_START_CHILD || type == CDR_TT_CANCEL_EXECUTION || type == CDR_TT_SIGNAL_EXECUTION);
    if (ext) {  // :370-371, :421-427, :452-458
      const GAS cdr_attr_external* xa = gp((const cdr_attr_external*)(KA()->B.ev.arena + (uint64_t)r.v));
      t_dom = xa->target_domain_id;
      t_wf = xa->workflow_id;
      if (type != CDR_TT_START_CHILD) {
        t_run = xa->run_id;
        t_fl = (xa->flags & CDR_XF_CHILD_ONLY) ? CDR_TF_CHILD_ONLY : 0u;
      }
    }
    task_words t;
    t.w[0] = type | (((r.w0 >> 8) & 0xFull) << 32);                       // type, timeout_type
    t.w[1] = (uint64_t)r.eid;                                               // event_id
    t.w[2] = tim ? (uint64_t)(r.v + (type == CDR_TT_DELETE_HISTORY ? ret : 0)) : 0ull;  // visibility_ts
    t.w[3] = 0;                                                             // attempt
    t.w[4] = t_dom | ((uint64_t)t_tl << 32);                                // domain_id, task_list
    t.w[5] = t_wf | ((uint64_t)t_run << 32);                                // target workflow / run
    t.w[6] = t_fl;                                                          // flags, _pad
    t.w[7] = 0;                                                             // version
    const bool fits = tim ? n_tt < cp.ttask_cap : n_xt < cp.xfer_cap;
    GAS task_words* dst = (GAS task_words*)(tim ? gp(KA()->O.timer_tasks) + cp.ttask_off + n_tt
                                                : gp(KA()->O.transfer) + cp.xfer_off + n_xt);
    // the taken list advances: its next record becomes the head, the one after is loaded
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
      const bool tk = on && c == j;
      if (tk) {
        hd[j] = nx[j];
        nx[j] = CDR_MERGE_D2 ? ld(j, cur[j] + 2) : n2[j];
        cur[j]++;
        if (!CDR_MERGE_D2) n2[j] = ld(j, cur[j] + 2);
      }
    }
    coop_put<8>(dst, t, on && fits, 0);
    lost |= on && !fits;
    n_tt += (on && fits && tim) ? 1u : 0u;
    n_xt += (on && fits && !tim) ? 1u : 0u;
  }
  if (valid) {  // (a truncated list is not returned: the entry reports the bad capacities)
    KA()->O.n_tasks[2ull * (uint64_t)w] = lost ? 0u : n_xt;
    KA()->O.n_tasks[2ull * (uint64_t)w + 1] = lost ? 0u : n_tt;
    if (lost) KA()->O.result[w].code = CDR_E_BAD_INPUT;
  }
}

// continue-as-new stitching (stateBuilder.go:557-574): a parent that applied its new
// run inherits the new run's error; a new run its parent never reached is NOT_APPLIED.
__global__ void k_finalize(cdr_dev_batch B, cdr_out O) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= B.n_wfs || (B.skip && B.skip[w])) return;
  const int32_t c = B.wfs[w].newrun;
  if (c < 0) return;
  cdr_wf_result& P = O.result[w];
  cdr_wf_result& C = O.result[c];
  if (P.flags & CDR_RF_NEWRUN_APPLIED) {
    if (C.code != CDR_OK) {
      P.code = C.code;
      P.flags |= CDR_RF_IN_NEWRUN;
      P.fail_event_id = C.fail_event_id;
      P.fail_index = C.fail_index;
      P.n_activity = P.n_timer = P.n_child = P.n_cancel = P.n_signal = 0;
      P.n_vh = P.n_reset_points = P.n_search_attr = 0;
    }
  } else {
    C.code = CDR_NOT_APPLIED;
    C.fail_event_id = 0;
    C.fail_index = 0;
    C.n_activity = C.n_timer = C.n_child = C.n_cancel = C.n_signal = 0;
    C.n_vh = C.n_reset_points = C.n_search_attr = 0;
  }
  C.flags = CDR_RF_IS_NEWRUN;
}

// ============================================================ host API
// struct cdr_ctx: ctx.h


#define HIPCHK(x)                                                                      \
  do {                                                                                 \
    hipError_t _e = (x);                                                               \
    if (_e != hipSuccess) {                                                            \
      fprintf(stderr, "cdr: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(_e), __FILE__, __LINE__); \
      return CDR_API_EDEVICE;                                                          \
    }                                                                                  \
  } while (0)

void* cdr_ws_get(cdr_ctx* c, int slot, uint64_t bytes) {
  if (!c || slot < 0 || slot >= WS_NUM) return nullptr;
  if (bytes == 0) bytes = 8;
  if (c->ws[slot] && c->ws_bytes[slot] >= bytes) return c->ws[slot];
  if (c->ws[slot]) (void)hipFree(c->ws[slot]);
  c->ws[slot] = nullptr;
  c->ws_bytes[slot] = 0;
  const uint64_t want = bytes + bytes / 8;  // headroom: a slowly growing caller reallocates rarely
  void* p = nullptr;
  if (hipMalloc(&p, want) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  c->ws[slot] = p;
  c->ws_bytes[slot] = want;
  return p;
}

void* cdr_hs_get(cdr_ctx* c, int slot, uint64_t bytes) {
  const uint64_t want = bytes ? bytes : 8;
  if (c->hs[slot] && c->hs_bytes[slot] >= want) return c->hs[slot];
  if (c->hs[slot]) (void)hipHostFree(c->hs[slot]);
  c->hs[slot] = nullptr;
  c->hs_bytes[slot] = 0;
  void* p = nullptr;
  if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  c->hs[slot] = p;
  c->hs_bytes[slot] = want;
  return p;
}

// a register-table launch with or without the task lists (the TASKS instantiation, compiled
// for CDR_WPE_REG waves per SIMD: its emission code spills at the smaller variant's 3)
template <int NA, int NT, int NX, uint32_t SF, int WPE, bool CARRY>
static void launch_reg(bool tasks, dim3 g, hipStream_t sq, const cdr_launch& x) {
  typedef RegLds<NA, NT, NX> LY;
  if (tasks)
    hipLaunchKernelGGL((k_replay_reg<NA, NT, NX, SF, CDR_WPE_REG, CARRY, true>), g, dim3(CDR_SLICE_WIDTH), LY::bytes, sq,
                       x);
  else
    hipLaunchKernelGGL((k_replay_reg<NA, NT, NX, SF, WPE, CARRY, false>), g, dim3(CDR_SLICE_WIDTH), LY::bytes, sq, x);
}

extern "C" {

void cdr_opts_default(cdr_opts* o) {
  if (!o) return;
  *o = cdr_opts{};
  o->plan_mode = CDR_PLAN_WAVE | CDR_PLAN_PAR;
  o->fast_path = 1;
  o->reg_path = 1;
  o->concurrent = 1;
}

cdr_ctx* cdr_create(int device, const cdr_opts* opts) {
  cdr_opts o;
  cdr_opts_default(&o);
  if (opts) o = *opts;
  if (o.plan_mode & ~(uint32_t)(CDR_PLAN_WAVE | CDR_PLAN_WAVE_ALL | CDR_PLAN_NO_LONG | CDR_PLAN_PAR)) return nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= device || device < 0) return nullptr;
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  cdr_ctx* c = new cdr_ctx();
  c->device = device;
  c->fast = o.fast_path ? 1 : 0;
  c->reg = o.reg_path ? 1 : 0;
  c->plan_mode = o.plan_mode;
  for (int i = 0; i < 4; i++)
    if (hipEventCreate(&c->ev[i]) != hipSuccess) {
      delete c;
      return nullptr;
    }
  c->timed = false;
  // the PAR slices' stream gets high priority: their workgroups are dispatched before the
  // bulk classes fill the CUs (CDR_STREAM_PRIO overrides, a bit mask of side streams)
  int prio_lo = 0, prio_hi = 0;
  if (hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess) prio_lo = prio_hi = 0;
  bool sides_ok = hipEventCreateWithFlags(&c->fork, hipEventDisableTiming) == hipSuccess;
  // experiment (CDR_WAVE_CUS=k): the wave class on every k-th CU alone, the others elsewhere
  int wave_cus = 0;
  if (const char* e = std::getenv("CDR_WAVE_CUS")) wave_cus = std::atoi(e);
  hipDeviceProp_t prop{};
  const int n_cu = (wave_cus > 1 && hipGetDeviceProperties(&prop, device) == hipSuccess) ? prop.multiProcessorCount : 0;
  // side streams at high priority (bit i: stream i): the PAR slices only — their long
  // histories set the critical path; every other mask measured was slower on C4/C5
  // (tools/gpu_prio_streams.sh: C5 7.7 ms vs 9.0 with wave / 12-activity / general / PAR
  // high, 10.3-10.7 with PAR plus any one other class high)
  uint32_t hi_mask = 0x40u;
  if (const char* e = std::getenv("CDR_STREAM_PRIO")) hi_mask = (uint32_t)std::strtoul(e, nullptr, 0);
  // hardware queues of this process's HIP runtime (it reads GPU_MAX_HW_QUEUES once, at
  // start; default 4): group the classes onto three side streams unless every class can
  // have a queue (CDR_SIDE_STREAMS=3|7 overrides)
  int hwq = 4;
  if (const char* e = std::getenv("GPU_MAX_HW_QUEUES")) hwq = std::atoi(e) > 0 ? std::atoi(e) : 4;
  int n_side = hwq >= cdr_ctx::N_SIDE + 1 ? cdr_ctx::N_SIDE : 3;
  if (const char* e = std::getenv("CDR_SIDE_STREAMS")) n_side = std::atoi(e) == 3 ? 3 : cdr_ctx::N_SIDE;
  if (n_side == 3) {
    // four streams, one per queue: the wave and 12-activity classes (few slices, long
    // histories) | the small-table class | the general, fast and 6-activity classes on the
    // caller's stream | PAR.  Measured at 4 queues (tools/gpu_groups.sh, 1M workflows,
    // ms/step C3 / C4 / C5): 5.32 / 14.0 / 8.72 against 6.40 / 19.0 / 11.7 with every lane
    // class on one side stream and 5.98 / 16.3 / 10.1 with a stream per class
    // (CDR_SIDE_GROUPS=<7 digits> overrides: class i's stream, 7 = the caller's stream)
    int grouped[cdr_ctx::N_SIDE] = {0, 0, 7, 5, 7, 7, 6};
    if (const char* e = std::getenv("CDR_SIDE_GROUPS"))
      if (std::strlen(e) == (size_t)cdr_ctx::N_SIDE)
        for (int i = 0; i < cdr_ctx::N_SIDE; i++)
          if (e[i] >= '0' && e[i] <= '0' + cdr_ctx::N_SIDE) grouped[i] = e[i] - '0';
    for (int i = 0; i < cdr_ctx::N_SIDE; i++) c->side_of[i] = grouped[i];
  }
  bool need[cdr_ctx::N_SIDE] = {};  // only the streams some class launches on (each takes a queue)
  for (int i = 0; i < cdr_ctx::N_SIDE; i++)
    if (c->side_of[i] < cdr_ctx::N_SIDE) need[c->side_of[i]] = true;
  for (int i = 0; i < cdr_ctx::N_SIDE; i++) {
    if (!need[i]) continue;
    if (n_cu > 0) {
      std::vector<uint32_t> m((n_cu + 31) / 32, 0u);
      for (int cu = 0; cu < n_cu; cu++)
        if ((cu % wave_cus == 0) == (i == 0)) m[cu / 32] |= 1u << (cu % 32);
      sides_ok = sides_ok && hipExtStreamCreateWithCUMask(&c->side[i], (uint32_t)m.size(), m.data()) == hipSuccess;
    } else {
      sides_ok = sides_ok &&
                 hipStreamCreateWithPriority(&c->side[i], hipStreamNonBlocking, ((hi_mask >> i) & 1u) ? prio_hi : prio_lo) ==
                     hipSuccess;
    }
    sides_ok = sides_ok && hipEventCreateWithFlags(&c->join[i], hipEventDisableTiming) == hipSuccess;
  }
  if (!sides_ok)
    c->concurrent = 0;
  if (const char* e = std::getenv("CDR_SERIAL_KERNELS")) c->concurrent = c->concurrent && e[0] == '0';
  c->concurrent = c->concurrent && o.concurrent;
  if (o.workspace_bytes && !cdr_ws_get(c, WS_SLAB, o.workspace_bytes)) {
    cdr_destroy(c);
    return nullptr;
  }
  return c;
}

int cdr_set_fast_path(cdr_ctx* c, int enable) {
  if (!c) return CDR_API_EINVAL;
  const int old = c->fast;
  c->fast = enable ? 1 : 0;
  return old;
}

int cdr_set_cls_path(cdr_ctx* c, int mode) {
  if (!c || mode < CDR_CLS_OFF || mode > CDR_CLS_BUILD) return CDR_API_EINVAL;
  const int old = c->cls;
  c->cls = mode;
  return old;
}

int cdr_cls_plan_async(cdr_ctx* c, const cdr_dev_batch* in, uint32_t* cls_rows, uint64_t* cls_row0, void* stream) {
  if (!c || !in || !cls_rows || !cls_row0) return CDR_API_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  HIPCHK(hipSetDevice(c->device));
  const uint32_t ns = in->ev.n_slices;
  // the per-event map k_cls_gather transposes with (16 B per slab element); without the room for
  // it, cdr_cls_pack_async scatters lane by lane (k_cls_fill)
  void* map = ns ? cdr_ws_get(c, WS_CLS_MAP, in->ev.n_rows * CDR_SLICE_WIDTH * 16ull) : nullptr;
  c->cls_map_slab = map ? (const void*)in->ev.slab : nullptr;
  c->cls_map_rows = map ? in->ev.n_rows : 0;
  if (ns) hipLaunchKernelGGL(k_cls_count, dim3(ns), dim3(CDR_SLICE_WIDTH), 0, st, *in, cls_rows, cls_row0, map);
  HIPCHK(hipGetLastError());
  hipLaunchKernelGGL(k_cls_scan, dim3(1), dim3(1024), 0, st, cls_row0, ns);
  HIPCHK(hipGetLastError());
  return CDR_API_OK;
}

int cdr_cls_pack_async(cdr_ctx* c, const cdr_dev_batch* in, void* stream) {
  if (!c || !in || !in->cls_slab || !in->cls_row0 || !in->cls_rows) return CDR_API_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  HIPCHK(hipSetDevice(c->device));
  const bool map = c->ws[WS_CLS_MAP] && c->cls_map_slab == (const void*)in->ev.slab &&
                   c->cls_map_rows == in->ev.n_rows && in->ev.n_rows;
  if (map && in->ev.n_slices) {  // the LDS transposition, then the slices too long for it
    static const bool attr = hipFuncSetAttribute((const void*)k_cls_gather, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 (int)CLS_G_LDS) == hipSuccess;
    (void)attr;
    hipLaunchKernelGGL(k_cls_gather, dim3(in->ev.n_slices), dim3(CLS_G_THREADS), CLS_G_LDS, st, *in,
                       (const void*)c->ws[WS_CLS_MAP]);
    HIPCHK(hipGetLastError());
  }
  if (in->ev.n_slices)
    hipLaunchKernelGGL(k_cls_fill, dim3(in->ev.n_slices), dim3(CDR_SLICE_WIDTH), 0, st, *in, map ? 0 : 1);
  HIPCHK(hipGetLastError());
  return CDR_API_OK;
}

int cdr_set_reg_path(cdr_ctx* c, int enable) {
  if (!c) return CDR_API_EINVAL;
  const int old = c->reg;
  c->reg = enable ? 1 : 0;
  return old;
}

int cdr_set_plan_mode(cdr_ctx* c, uint32_t mode) {
  if (!c || (mode & ~(uint32_t)(CDR_PLAN_WAVE | CDR_PLAN_WAVE_ALL | CDR_PLAN_NO_LONG | CDR_PLAN_PAR))) return CDR_API_EINVAL;
  const uint32_t old = c->plan_mode;
  c->plan_mode = mode;
  return (int)old;
}
uint32_t cdr_get_plan_mode(const cdr_ctx* c) { return c ? c->plan_mode : 0u; }
int cdr_ctx_device(const cdr_ctx* c) { return c ? c->device : 0; }

void cdr_destroy(cdr_ctx* c) {
  if (!c) return;
  for (int i = 0; i < 4; i++) (void)hipEventDestroy(c->ev[i]);
  for (hipEvent_t e : c->ring) (void)hipEventDestroy(e);
  for (int i = 0; i < cdr_ctx::N_SIDE; i++) {
    if (c->side[i]) (void)hipStreamDestroy(c->side[i]);
    if (c->join[i]) (void)hipEventDestroy(c->join[i]);
  }
  if (c->fork) (void)hipEventDestroy(c->fork);
  if (hipSetDevice(c->device) == hipSuccess)
    for (void* p : c->ws) (void)hipFree(p);
  for (void* p : c->hs)
    if (p) (void)hipHostFree(p);
  delete c;
}

int cdr_replay_sliced_async(cdr_ctx* c, const cdr_dev_batch* in, const cdr_out* out, void* stream) {
  if (!c || !in || !out) return CDR_API_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  HIPCHK(hipSetDevice(c->device));
  // LDS budget: up to CDR_LDS_ACT_MAX activity and CDR_LDS_TIM_MAX timer slots per
  // lane; slices that need more replay in the scratch-slot launch
  const uint32_t la = in->max_act_slots < CDR_LDS_ACT_MAX ? in->max_act_slots : CDR_LDS_ACT_MAX;
  const uint32_t lt = in->max_tim_slots < CDR_LDS_TIM_MAX ? in->max_tim_slots : CDR_LDS_TIM_MAX;
  const size_t lds = (size_t)(la * CDR_ACT_PLANES + lt * CDR_TIM_PLANES) * CDR_SLICE_WIDTH * sizeof(uint64_t);
  const bool spill = in->max_act_slots > la || in->max_tim_slots > lt;
  const uint32_t blocks = in->ev.n_slices;
  // task emission: the general kernel, the fast kernel's and the register-table kernels'
  // TASKS instantiations (a plan without wave slices is required; no class blocks, no
  // loaded state on the register-table kernels)
  const bool tasks = out->transfer != nullptr;
  if (tasks && (in->n_wave_slices > 0 || !out->timer_tasks || !out->n_tasks)) return CDR_API_EINVAL;
  // (the fast kernel's TASKS instantiation emits them for its slices)
  const bool fast = c->fast && in->n_fast_slices > 0;
  // register-table kernel: LastReplicationInfo kept for clusters < CDR_REG_NCL only (a loaded
  // state with tasks: the CARRY + TASKS instantiations, nDCHistoryReplicator.go:341-348 then
  // stateBuilder.go:606-608)
  const bool reg = c->fast && c->reg &&
                   in->n_reg_slices + in->n_reg2_slices + in->n_reg0_slices + in->n_par_slices > 0 &&
                   in->cluster.n_clusters <= (int)CDR_REG_NCL;
  // carry-in batches (cdr_dev_batch.carry): the register-table slices replay in the carry-in
  // instantiations of k_replay_reg, each class followed by its hand-on chain (below)
  const bool carry = in->carry != nullptr;
  // class-decomposed replay of the register-table slices (their class-sorted blocks)
  // (with tasks: k_replay_cls<TASKS> on the lane slices, k_tasks_merge after; the PAR slices'
  // tasks from k_replay_reg<TASKS>)
  const bool cls = reg && !carry && c->cls && in->cls_slab && in->cls_row0 && in->cls_rows;
  const bool cls_fb = c->cls != 2;  // 2 (tests): no k_replay_reg pass for the CLS_RETRY entries
  auto retry_of = [](cdr_launch x) {
    x.retry = 1u;
    return x;
  };
  // the retry passes walk k_replay_cls's lists with this many workgroups at most
  constexpr uint32_t RETRY_WGS = 256;
  auto retry_grid = [&](dim3 g) { return dim3(g.x < RETRY_WGS ? g.x : RETRY_WGS); };
  const bool wave = in->n_wave_slices > 0;
  const bool general = (fast ? in->n_fast_slices : 0u) +
                           (reg ? in->n_reg_slices + in->n_reg2_slices + in->n_reg0_slices + in->n_par_slices : 0u) +
                           in->n_wave_slices <
                       in->ev.n_slices;
  const bool ring = c->ring_used + 2 <= c->ring.size();
  HIPCHK(hipEventRecord(ring ? c->ring[c->ring_used] : c->ev[0], st));
  cdr_launch L{*in, *out, la, lt, fast ? 1u : 0u, reg ? 1u : 0u, 0u, 0u, nullptr, nullptr, nullptr, nullptr, nullptr,
               nullptr, nullptr, 0ull};
  // k_replay_cls<TASKS>: per-class staging lists (4 x the entry's task rows, 32 B per record) and
  // per-entry headers (zeroed: no header = not a class-kernel entry)
  const bool cls_tasks = cls && tasks && in->n_wfs > 0;
  if (cls_tasks) {
    // the task-slice rows: the caller's (cdr_dev_batch.task_rows), else the last entry's
    // offsets + capacities read on the launch stream (every launch: the same caps buffer may
    // hold another batch's capacities next time)
    uint64_t rows = in->task_rows;
    if (rows == 0) {
      cdr_wf_caps last;
      HIPCHK(hipMemcpyAsync(&last, in->caps + (in->n_wfs - 1), sizeof(last), hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      rows = (uint64_t)last.xfer_off + last.xfer_cap + last.ttask_off + last.ttask_cap;
    }
    L.tstage = (uint64_t*)cdr_ws_get(c, WS_TSTAGE, 4ull * rows * 32ull + 32ull);
    L.trows = 4ull * rows;
    L.thead = (uint32_t*)cdr_ws_get(c, WS_THEAD, 32ull * in->n_wfs);
    if (!L.tstage || !L.thead) return CDR_API_ENOMEM;
    HIPCHK(hipMemsetAsync(L.thead, 0, 32ull * in->n_wfs, st));
  }
  // retry lists (k_replay_cls -> k_replay_reg): counters zeroed on the launch stream
  // (carry-in: a second level of lists, k_replay_reg<12-activity> -> the general kernel,
  // counters 8 + class)
  uint32_t* rws = nullptr;
  if ((cls && cls_fb) || (carry && reg)) {
    rws = (uint32_t*)cdr_ws_get(c, WS_RETRY, (16ull + 2ull * cdr_ctx::N_SIDE * blocks) * 4ull);
    if (!rws) return CDR_API_ENOMEM;
    HIPCHK(hipMemsetAsync(rws, 0, 16 * 4, st));
  }
  auto with_list = [&](cdr_launch x, int cls_id) {
    if (rws) {
      x.rcount = rws + cls_id;
      x.rlist = rws + 16 + (uint64_t)cls_id * blocks;
    }
    return x;
  };
  // carry-in hand-on lists of class cls_id: level 1 (-> the 12-activity variant), level 2
  // (-> the general kernel)
  auto out_list = [&](cdr_launch x, int cls_id, int level) {
    x.ocount = rws + (level == 1 ? 0 : 8) + cls_id;
    x.olist = rws + 16 + (uint64_t)((level == 1 ? 0 : cdr_ctx::N_SIDE) + cls_id) * blocks;
    return x;
  };
  auto in_list = [&](int cls_id, int level) {
    cdr_launch x = L;
    x.retry = 1u;
    x.rcount = rws + (level == 1 ? 0 : 8) + cls_id;
    x.rlist = rws + 16 + (uint64_t)((level == 1 ? 0 : cdr_ctx::N_SIDE) + cls_id) * blocks;
    return x;
  };
  // after a carry-in register-table launch of class cls_id over grid g on stream sq: the
  // 12-activity variant over its level-1 list (below12: the class's tables are smaller),
  // then the general kernel over the level-2 list
  auto carry_tail = [&](int cls_id, dim3 g, hipStream_t sq, bool below12) {
    if (below12)  // a whole grid: unlike k_replay_cls's few leftovers, a loaded state outgrowing the
                  // smaller tables is common, and this variant runs one wave per SIMD
      launch_reg<CDR_REG2_NA, CDR_REG_NT, CDR_REG_NX, CDR_CLS_SLICES, CDR_WPE_REG, true>(
          tasks, g, sq, out_list(in_list(cls_id, 1), cls_id, 2));
    if (tasks) {
      hipLaunchKernelGGL((k_replay<true, true>), g, dim3(CDR_SLICE_WIDTH), lds, sq, in_list(cls_id, 2));
      if (spill) hipLaunchKernelGGL((k_replay<false, true>), g, dim3(CDR_SLICE_WIDTH), 0, sq, in_list(cls_id, 2));
    } else {
      hipLaunchKernelGGL((k_replay<true, false>), g, dim3(CDR_SLICE_WIDTH), lds, sq, in_list(cls_id, 2));
      if (spill) hipLaunchKernelGGL((k_replay<false, false>), g, dim3(CDR_SLICE_WIDTH), 0, sq, in_list(cls_id, 2));
    }
  };
  // each kernel over its class's slice range (cdr_plan_class_ranges), or every slice
  bool ranged = false;
  for (int c = 0; c < 6; c++) ranged |= in->class_hi[c] > 0;
  auto grid_of = [&](int cls, cdr_launch& Lc) {
    Lc = L;
    if (!ranged) return dim3(blocks);
    const uint32_t lo = in->class_lo[cls], hi = in->class_hi[cls] < blocks ? in->class_hi[cls] : blocks;
    Lc.s0 = lo < hi ? lo : 0u;
    return dim3(lo < hi ? hi - lo : 0u);
  };
  cdr_launch Lw, Lr2, Lg, Lr0, Lf, Lr1;
  const dim3 gw = grid_of(CDR_CLASS_WAVE, Lw), gr2 = grid_of(CDR_CLASS_REG2, Lr2), gg = grid_of(CDR_CLASS_GENERAL, Lg),
             gr0 = grid_of(CDR_CLASS_REG0, Lr0), gf = grid_of(CDR_CLASS_FAST, Lf), gr1 = grid_of(CDR_CLASS_REG, Lr1);
  // kernel streams: each replay kernel class present gets a side stream of its own
  // (all forked from the caller's stream, so none is dispatched ahead of the others but
  // by priority), launched longest-first: the wave kernel (the batch's longest histories, one wave each, scalar-unit-
  // bound), the 12-activity register kernel (one wave per SIMD), the general kernel (the
  // few histories no specialised kernel takes), the small-table register kernel, the
  // fast kernel — so that no class's slices wait for another's kernel to finish
  const bool reg1 = blocks && reg && in->n_reg_slices && gr1.x;
  const bool reg0 = blocks && reg && in->n_reg0_slices && gr0.x;
  const bool reg2 = blocks && reg && in->n_reg2_slices && gr2.x;
  const bool wv = blocks && wave && gw.x, fst = blocks && fast && gf.x;
  // the PAR slices (the batch's long register-table histories): slices 0 .. n_par_slices - 1
  const uint32_t npar = in->n_par_slices < blocks ? in->n_par_slices : blocks;
  const bool par = blocks && reg && npar > 0;
  // the general kernel also takes the fast / register slices whose kernels are off
  const dim3 gg_all = (ranged && (!fast || !reg)) ? dim3(blocks) : gg;
  if (ranged && (!fast || !reg)) Lg.s0 = 0;
  const bool gen = blocks && general && gg_all.x;
  const bool on[cdr_ctx::N_SIDE] = {wv, reg2, gen, reg0, fst, reg1, par};
  int kinds = 0;
  for (bool o : on) kinds += o ? 1 : 0;
  // this launch's class -> stream map: a class sharing a stream with another takes the PAR
  // stream instead when the batch has no PAR slices (that stream's queue would sit idle)
  int so[cdr_ctx::N_SIDE];
  for (int i = 0; i < cdr_ctx::N_SIDE; i++) so[i] = c->side_of[i];
  if (!on[6] && so[6] < cdr_ctx::N_SIDE)
    for (int i = 0; i < 6; i++)
      if (on[i] && so[i] < cdr_ctx::N_SIDE && so[i] != so[6]) {
        bool shared = false;
        for (int j = 0; j < i; j++) shared |= on[j] && so[j] == so[i];
        if (shared) {
          so[i] = so[6];
          break;
        }
      }
  bool fk[cdr_ctx::N_SIDE];  // class i forks onto side[so[i]]
  bool used[cdr_ctx::N_SIDE] = {};  // side stream j carries a forked class
  bool any_fork = false;
  for (int i = 0; i < cdr_ctx::N_SIDE; i++) {
    any_fork |= (fk[i] = c->concurrent && on[i] && kinds > 1 && so[i] < cdr_ctx::N_SIDE);
    if (fk[i]) used[so[i]] = true;
  }
  if (any_fork) HIPCHK(hipEventRecord(c->fork, st));
  for (int j = 0; j < cdr_ctx::N_SIDE; j++)
    if (used[j]) HIPCHK(hipStreamWaitEvent(c->side[j], c->fork, 0));
  auto sx = [&](int i) { return fk[i] ? c->side[so[i]] : st; };
  static const char* order = [] {
    const char* e = std::getenv("CDR_LAUNCH_ORDER");
    uint32_t seen = 0;  // a permutation of the side-stream indices, or the default
    for (size_t j = 0; e && j < std::strlen(e); j++)
      if (e[j] >= '0' && e[j] < '0' + cdr_ctx::N_SIDE) seen |= 1u << (e[j] - '0');
    return (e && std::strlen(e) == (size_t)cdr_ctx::N_SIDE && seen == (1u << cdr_ctx::N_SIDE) - 1u) ? e : "6012345";
  }();
  // big workgroups first: a PAR workgroup takes a whole CU (four 256-VGPR waves), a 12-activity
  // class workgroup one 193-VGPR wave, and once the bulk classes' small workgroups hold the
  // CUs they find no room until those drain (measured: C4 + long histories, the PAR kernel
  // started ~7 ms late).  Their workgroups count themselves in (rws word 15, zeroed above);
  // the other classes' streams wait until the PAR workgroups (or, without them, up to
  // CDR_GATE_REG2 of the 12-activity ones) have started (CDR_NO_PAR_GATE: no gate;
  // CDR_GATE_REG2=0: PAR only)
  if (c->wait_value < 0) {
    int v = 0;
    c->wait_value = hipDeviceGetAttribute(&v, hipDeviceAttributeCanUseStreamWaitValue, c->device) == hipSuccess && v;
  }
  static const uint32_t gate_reg2_max = [] {
    const char* e = std::getenv("CDR_GATE_REG2");
    return e ? (uint32_t)std::strtoul(e, nullptr, 0) : 1024u;
  }();
  // (not under a counter-collecting profiler, which serializes dispatches: a stream waiting
  // on a value another queue's kernel writes would wait on a kernel it holds back)
  static const bool gate_env = !std::getenv("CDR_NO_PAR_GATE") && !std::getenv("ROCPROF_COUNTER_COLLECTION");
  const bool gate_ok = cls && !carry && rws && c->wait_value && c->concurrent && gate_env &&
                       order[0] == '6' && std::strchr(order, '1') < std::strchr(order, '2') &&
                       std::strchr(order, '1') < std::strchr(order, '3') && std::strchr(order, '1') < std::strchr(order, '4') &&
                       std::strchr(order, '1') < std::strchr(order, '5');
  const bool gate = gate_ok && par && fk[6] && !tasks;  // (with tasks the PAR slices run k_replay_reg: nothing counts in)
  // (the 12-activity class only in a batch without PAR slices: with them, holding the other
  // classes back for it too cost C4 / C5 0.2-0.4 ms; without, it is C3's longest class and
  // gains 5%: 5.07 -> 4.84 ms)
  const bool gate2 = gate_ok && !par && reg2 && gate_reg2_max > 0 && fk[1] && so[1] != so[6] && !(wv && so[0] == so[1]);
  const uint32_t gate_n = (gate ? (npar < 256u ? npar : 256u) : 0u) + (gate2 ? (gr2.x < gate_reg2_max ? gr2.x : gate_reg2_max) : 0u);
  const bool gating = gate || gate2;
  // each class's launches (its stream sx(i)); the order they are issued in decides which
  // class's workgroups take the CUs first (CDR_LAUNCH_ORDER overrides: a digit string of
  // side-stream indices, default \"6012345\": PAR, wave, 12-activity, general, small-table,
  // fast, 6-activity)
  auto launch_class = [&](int i) {
    switch (i) {
      case 6:
    if (par && carry) {
      cdr_launch Lp = L;
      Lp.s0 = 0;
      launch_reg<CDR_REG2_NA, CDR_REG_NT, CDR_REG_NX, CDR_SLICE_PAR, CDR_WPE_REG, true>(tasks, dim3(npar), sx(6),
                                                                                        out_list(Lp, 6, 2));
      carry_tail(6, dim3(npar), sx(6), false);
    } else if (par) {  // first: the longest critical paths of the batch
      cdr_launch Lp = L;
      Lp.s0 = 0;
      typedef RegLds<CDR_REG2_NA, CDR_REG_NT, CDR_REG_NX> LY;
      if (cls && !tasks) {
        typedef ClsLds<CDR_REG2_NA, CDR_REG_NT, CDR_REG_NX, true> LC;
        cdr_launch Lpg = with_list(Lp, 6);
        if (rws && gate) Lpg.pstart = rws + 15;
        hipLaunchKernelGGL((k_replay_cls<CDR_REG2_NA, CDR_REG_NT, CDR_REG_NX, CDR_SLICE_PAR, CDR_WPE_CLS2, true>),
                           dim3(npar), dim3(4 * CDR_SLICE_WIDTH), LC::bytes, sx(6), Lpg);
      }
      if (tasks)
        hipLaunchKernelGGL((k_replay_reg<CDR_REG2_NA, CDR_REG_NT, CDR_REG_NX, CDR_SLICE_PAR, CDR_WPE_REG, false, true>),
                           dim3(npar), dim3(CDR_SLICE_WIDTH), LY::bytes, sx(6), Lp);
      else if (!cls)  // (with class blocks: its retry pass after the join, launch_retry)
        hipLaunchKernelGGL((k_replay_reg<CDR_REG2_NA, CDR_REG_NT, CDR_REG_NX, CDR_SLICE_PAR>), dim3(npar),
                           dim3(CDR_SLICE_WIDTH), LY::bytes, sx(6), Lp);
    }
        break;
      case 0:
    if (wv) hipLaunchKernelGGL(k_replay_wave, gw, dim3(CDR_SLICE_WIDTH), 0, sx(0), Lw);
        break;
      case 1:
    if (reg2 && carry) {
      launch_reg<CDR_REG2_NA, CDR_REG_NT, CDR_REG_NX, CDR_SLICE_REG2, CDR_WPE_REG, true>(tasks, gr2, sx(1),
                                                                                         out_list(Lr2, 1, 2));
      carry_tail(1, gr2, sx(1), false);
    } else if (reg2) {
      typedef RegLds<CDR_REG2_NA, CDR_REG_NT, CDR_REG_NX> LY;
      if (cls) {
        typedef ClsLds<CDR_REG2_NA, CDR_REG_NT, CDR_REG_NX> LC;
        cdr_launch Lg2 = with_list(Lr2, 1);
        if (rws && gate2) Lg2.pstart = rws + 15;
        if (tasks)
          hipLaunchKernelGGL((k_replay_cls<CDR_REG2_NA, CDR_REG_NT, CDR_REG_NX, CDR_SLICE_REG2, CDR_WPE_CLS2, false, true>),
                             gr2, dim3(CDR_SLICE_WIDTH), LC::bytes + CLS_TQ_BYTES, sx(1), Lg2);
        else
          hipLaunchKernelGGL((k_replay_cls<CDR_REG2_NA, CDR_REG_NT, CDR_REG_NX, CDR_SLICE_REG2, CDR_WPE_CLS2>), gr2,
                             dim3(CDR_SLICE_WIDTH), LC::bytes, sx(1), Lg2);
      }
      if (cls && tasks)  // the class kernel's staged tasks into the task slices (the handed-on
                         // entries have no header: their tasks come from the retry pass)
        hipLaunchKernelGGL(k_tasks_merge<CDR_SLICE_REG2>, gr2, dim3(CDR_SLICE_WIDTH), 9 * 65 * 8, sx(1), Lr2);
      if (tasks && !cls)
        hipLaunchKernelGGL((k_replay_reg<CDR_REG2_NA, CDR_REG_NT, CDR_REG_NX, CDR_SLICE_REG2, CDR_WPE_REG, false, true>), gr2,
                           dim3(CDR_SLICE_WIDTH), LY::bytes, sx(1), Lr2);
      else if (!cls)  // (with class blocks: its retry pass after the join, launch_retry)
        hipLaunchKernelGGL((k_replay_reg<CDR_REG2_NA, CDR_REG_NT, CDR_REG_NX, CDR_SLICE_REG2>), gr2, dim3(CDR_SLICE_WIDTH), LY::bytes, sx(1),
                           Lr2);
    }
        break;
      case 2:
    if (gen) {
      if (tasks)
        hipLaunchKernelGGL((k_replay<true, true>), gg_all, dim3(CDR_SLICE_WIDTH), lds, sx(2), Lg);
      else
        hipLaunchKernelGGL((k_replay<true, false>), gg_all, dim3(CDR_SLICE_WIDTH), lds, sx(2), Lg);
    }
    if (gen && spill) {
      if (tasks)
        hipLaunchKernelGGL((k_replay<false, true>), gg_all, dim3(CDR_SLICE_WIDTH), 0, sx(2), Lg);
      else
        hipLaunchKernelGGL((k_replay<false, false>), gg_all, dim3(CDR_SLICE_WIDTH), 0, sx(2), Lg);
    }
        break;
      case 3:
    if (reg0 && carry) {
      launch_reg<CDR_REG0_NA, CDR_REG0_NT, CDR_REG0_NX, CDR_SLICE_REG0, 3, true>(tasks, gr0, sx(3), out_list(Lr0, 3, 1));
      carry_tail(3, gr0, sx(3), true);
    } else if (reg0) {  // the small-table variant, at 3 waves per SIMD
      typedef RegLds<CDR_REG0_NA, CDR_REG0_NT, CDR_REG0_NX> LY;
      if (cls) {
        typedef ClsLds<CDR_REG0_NA, CDR_REG0_NT, CDR_REG0_NX> LC;
        if (tasks)
          hipLaunchKernelGGL((k_replay_cls<CDR_REG0_NA, CDR_REG0_NT, CDR_REG0_NX, CDR_SLICE_REG0, CDR_WPE_CLS_T, false, true>),
                             gr0, dim3(CDR_SLICE_WIDTH), LC::bytes + CLS_TQ_BYTES, sx(3), with_list(Lr0, 3));
        else
          hipLaunchKernelGGL((k_replay_cls<CDR_REG0_NA, CDR_REG0_NT, CDR_REG0_NX, CDR_SLICE_REG0, CDR_WPE_CLS0>), gr0,
                             dim3(CDR_SLICE_WIDTH), LC::bytes, sx(3), with_list(Lr0, 3));
      }
      if (cls && tasks)  // the class kernel's staged tasks into the task slices (the handed-on
                         // entries have no header: their tasks come from the retry pass)
        hipLaunchKernelGGL(k_tasks_merge<CDR_SLICE_REG0>, gr0, dim3(CDR_SLICE_WIDTH), 9 * 65 * 8, sx(3), Lr0);
      if (tasks && !cls)
        hipLaunchKernelGGL((k_replay_reg<CDR_REG0_NA, CDR_REG0_NT, CDR_REG0_NX, CDR_SLICE_REG0, CDR_WPE_REG, false, true>), gr0,
                           dim3(CDR_SLICE_WIDTH), LY::bytes, sx(3), Lr0);
      else if (!cls)  // (with class blocks: its retry pass after the join, launch_retry)
        hipLaunchKernelGGL((k_replay_reg<CDR_REG0_NA, CDR_REG0_NT, CDR_REG0_NX, CDR_SLICE_REG0, 3>), gr0, dim3(CDR_SLICE_WIDTH), LY::bytes, sx(3),
                           Lr0);
    }
        break;
      case 4:
    if (fst && tasks) hipLaunchKernelGGL(k_replay_fast<true>, gf, dim3(CDR_SLICE_WIDTH), FAST_LDS_BYTES + FAST_TBUF_BYTES, sx(4), Lf);
    else if (fst) hipLaunchKernelGGL(k_replay_fast<false>, gf, dim3(CDR_SLICE_WIDTH), FAST_LDS_BYTES, sx(4), Lf);
        break;
      case 5:
    if (reg1 && carry) {
      launch_reg<CDR_REG_NA, CDR_REG_NT, CDR_REG_NX, CDR_SLICE_REG, CDR_WPE_REG, true>(tasks, gr1, sx(5), out_list(Lr1, 5, 1));
      carry_tail(5, gr1, sx(5), true);
    } else if (reg1) {
      typedef RegLds<CDR_REG_NA, CDR_REG_NT, CDR_REG_NX> LY;
      if (cls) {
        typedef ClsLds<CDR_REG_NA, CDR_REG_NT, CDR_REG_NX> LC;
        if (tasks)
          hipLaunchKernelGGL((k_replay_cls<CDR_REG_NA, CDR_REG_NT, CDR_REG_NX, CDR_SLICE_REG, CDR_WPE_CLS_T, false, true>),
                             gr1, dim3(CDR_SLICE_WIDTH), LC::bytes + CLS_TQ_BYTES, sx(5), with_list(Lr1, 5));
        else
          hipLaunchKernelGGL((k_replay_cls<CDR_REG_NA, CDR_REG_NT, CDR_REG_NX, CDR_SLICE_REG, CDR_WPE_CLS>), gr1,
                             dim3(CDR_SLICE_WIDTH), LC::bytes, sx(5), with_list(Lr1, 5));
      }
      if (cls && tasks)  // the class kernel's staged tasks into the task slices (the handed-on
                         // entries have no header: their tasks come from the retry pass)
        hipLaunchKernelGGL(k_tasks_merge<CDR_SLICE_REG>, gr1, dim3(CDR_SLICE_WIDTH), 9 * 65 * 8, sx(5), Lr1);
      if (tasks && !cls)
        hipLaunchKernelGGL((k_replay_reg<CDR_REG_NA, CDR_REG_NT, CDR_REG_NX, CDR_SLICE_REG, CDR_WPE_REG, false, true>), gr1,
                           dim3(CDR_SLICE_WIDTH), LY::bytes, sx(5), Lr1);
      else if (!cls)  // (with class blocks: its retry pass after the join, launch_retry)
        hipLaunchKernelGGL((k_replay_reg<CDR_REG_NA, CDR_REG_NT, CDR_REG_NX, CDR_SLICE_REG>), gr1, dim3(CDR_SLICE_WIDTH), LY::bytes, sx(5),
                           Lr1);
    }
        break;
    }
  };
  // the class kernels' retry passes (k_replay_reg over the slices where k_replay_cls handed an
  // entry on), on the caller's stream after the join: a pass has nothing to do in a clean batch,
  // yet its 256-VGPR workgroups, dispatched beside the class kernels, each wait for a whole
  // SIMD's registers to free and hold back the other kernels' dispatch meanwhile (measured:
  // the empty 12-activity pass "ran" 2.7-7 ms and slowed the small-table class kernel)
  auto launch_retry = [&](int i) {
    if (!cls || !cls_fb || carry) return;
    switch (i) {
      case 6:
        if (par && !tasks) {
          typedef RegLds<CDR_REG2_NA, CDR_REG_NT, CDR_REG_NX> LY;
          cdr_launch Lp = L;
          Lp.s0 = 0;
          hipLaunchKernelGGL((k_replay_reg<CDR_REG2_NA, CDR_REG_NT, CDR_REG_NX, CDR_SLICE_PAR>), retry_grid(dim3(npar)),
                             dim3(CDR_SLICE_WIDTH), LY::bytes, st, retry_of(with_list(Lp, 6)));
        }
        break;
      case 1:
        if (reg2) {
          typedef RegLds<CDR_REG2_NA, CDR_REG_NT, CDR_REG_NX> LY;
          if (tasks)
            hipLaunchKernelGGL((k_replay_reg<CDR_REG2_NA, CDR_REG_NT, CDR_REG_NX, CDR_SLICE_REG2, CDR_WPE_REG, false, true>),
                               retry_grid(gr2), dim3(CDR_SLICE_WIDTH), LY::bytes, st, retry_of(with_list(Lr2, 1)));
          else
            hipLaunchKernelGGL((k_replay_reg<CDR_REG2_NA, CDR_REG_NT, CDR_REG_NX, CDR_SLICE_REG2>), retry_grid(gr2),
                               dim3(CDR_SLICE_WIDTH), LY::bytes, st, retry_of(with_list(Lr2, 1)));
        }
        break;
      case 3:
        if (reg0) {
          typedef RegLds<CDR_REG0_NA, CDR_REG0_NT, CDR_REG0_NX> LY;
          if (tasks)
            hipLaunchKernelGGL((k_replay_reg<CDR_REG0_NA, CDR_REG0_NT, CDR_REG0_NX, CDR_SLICE_REG0, CDR_WPE_REG, false, true>),
                               retry_grid(gr0), dim3(CDR_SLICE_WIDTH), LY::bytes, st, retry_of(with_list(Lr0, 3)));
          else
            hipLaunchKernelGGL((k_replay_reg<CDR_REG0_NA, CDR_REG0_NT, CDR_REG0_NX, CDR_SLICE_REG0, 3>), retry_grid(gr0),
                               dim3(CDR_SLICE_WIDTH), LY::bytes, st, retry_of(with_list(Lr0, 3)));
        }
        break;
      case 5:
        if (reg1) {
          typedef RegLds<CDR_REG_NA, CDR_REG_NT, CDR_REG_NX> LY;
          if (tasks)
            hipLaunchKernelGGL((k_replay_reg<CDR_REG_NA, CDR_REG_NT, CDR_REG_NX, CDR_SLICE_REG, CDR_WPE_REG, false, true>),
                               retry_grid(gr1), dim3(CDR_SLICE_WIDTH), LY::bytes, st, retry_of(with_list(Lr1, 5)));
          else
            hipLaunchKernelGGL((k_replay_reg<CDR_REG_NA, CDR_REG_NT, CDR_REG_NX, CDR_SLICE_REG>), retry_grid(gr1),
                               dim3(CDR_SLICE_WIDTH), LY::bytes, st, retry_of(with_list(Lr1, 5)));
        }
        break;
    }
  };
  // The gated kernels are issued before any wait: a wait-value packet blocks its whole
  // hardware queue, so a wait issued ahead of the kernel whose workgroups it counts could
  // block that kernel's own queue (streams share the 4 hardware queues) and never be met.
  // Issued after it, every wait is met once the gated kernel's workgroups have started,
  // whatever the stream -> queue mapping or a profiler's dispatch serialisation.
  bool issued[cdr_ctx::N_SIDE] = {};
  if (gating) {
    for (int j = 0; j < cdr_ctx::N_SIDE; j++) {
      const int i = order[j] - '0';
      if ((gate && i == 6) || (gate2 && i == 1)) {
        launch_class(i);
        HIPCHK(hipGetLastError());
        issued[i] = true;
      }
    }
    // every other class's stream waits for the gated workgroups
    hipStream_t waited[cdr_ctx::N_SIDE + 1];
    int nw = 0;
    for (int q = 0; q < 6; q++) {
      if (!on[q] || q == 1 || (gate && sx(q) == sx(6)) || (gate2 && sx(q) == sx(1))) continue;
      bool dup = false;
      for (int r = 0; r < nw; r++) dup |= waited[r] == sx(q);
      if (dup) continue;
      waited[nw++] = sx(q);
      HIPCHK(hipStreamWaitValue32(sx(q), rws + 15, gate_n, hipStreamWaitValueGte, 0xFFFFFFFFu));
    }
  }
  for (int j = 0; j < cdr_ctx::N_SIDE; j++) {
    const int i = order[j] - '0';
    if (issued[i]) continue;
    launch_class(i);
    HIPCHK(hipGetLastError());
  }
  for (int j = 0; j < cdr_ctx::N_SIDE; j++)
    if (used[j]) {
      HIPCHK(hipEventRecord(c->join[j], c->side[j]));
      HIPCHK(hipStreamWaitEvent(st, c->join[j], 0));
    }
  for (int i : {6, 1, 3, 5}) launch_retry(i);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(ring ? c->ring[c->ring_used + 1] : c->ev[1], st));
  if (ring) {
    // keep ev[0..1] meaningful for cdr_last_kernel_ms as well
    c->ring_used += 2;
    HIPCHK(hipEventRecord(c->ev[0], st));
    HIPCHK(hipEventRecord(c->ev[1], st));
  }
  const uint32_t fb = (in->n_wfs + 255) / 256;
  if (fb) hipLaunchKernelGGL(k_tables, dim3(fb), dim3(256), 0, st, *in, *out);
  HIPCHK(hipGetLastError());
  if (fb) hipLaunchKernelGGL(k_finalize, dim3(fb), dim3(256), 0, st, *in, *out);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(c->ev[2], st));
  c->timed = true;
  return CDR_API_OK;
}

uint32_t cdr_build_flags(void) {
  uint32_t f = 0;
#ifdef CDR_PAR_PROF
  f |= 1u;
#endif
  if (CDR_PAR_PRIO != 0 || CDR_FDEPTH != 2 || CDR_DEPTH != 1 || CDR_TYPED != 1 || CDR_FAST_DELTA != 1 ||
      CDR_VHBF != 1 || CDR_VHQUICK != 1 || CDR_CLS_DEPTH != 1 || CDR_CLS_PDEPTH != 4 || CDR_CLS_DEPTH_PAR != 4 ||
      CDR_CLS_PDEPTH_PAR != 16 || CDR_WPE_FAST != 3 || CDR_WPE != 3 || CDR_WPE_CLS != 4 || CDR_WPE_CLS0 != 4 ||
      CDR_WPE_CLS2 != 2 || FAST_CK != 8u || CDR_FAST_TBUF != 5 || CDR_WPE_FAST_TBUF != 2)
    f |= 2u;
  return f;
}

int cdr_last_kernel_ms(cdr_ctx* c, float* replay_ms, float* finalize_ms) {
  if (!c || !c->timed) return CDR_API_EINVAL;
  HIPCHK(hipEventSynchronize(c->ev[2]));
  float a = 0, b = 0;
  HIPCHK(hipEventElapsedTime(&a, c->ev[0], c->ev[1]));
  HIPCHK(hipEventElapsedTime(&b, c->ev[1], c->ev[2]));
  if (replay_ms) *replay_ms = a;
  if (finalize_ms) *finalize_ms = b;
  return CDR_API_OK;
}

// Start recording the replay kernel of the next `max_launches` launches with HIP
// events on their launch stream (bench.py's in-process kernel timing).
int cdr_timing_begin(cdr_ctx* c, uint32_t max_launches) {
  if (!c) return CDR_API_EINVAL;
  HIPCHK(hipSetDevice(c->device));
  while (c->ring.size() < 2ull * max_launches) {
    hipEvent_t e;
    HIPCHK(hipEventCreate(&e));
    c->ring.push_back(e);
  }
  c->ring_used = 0;
  return CDR_API_OK;
}

// Synchronise and return the recorded replay-kernel durations (ms); *n in = capacity,
// out = launches recorded.  Stops recording.
int cdr_timing_read(cdr_ctx* c, float* ms, uint32_t* n) {
  if (!c || !n) return CDR_API_EINVAL;
  const uint32_t k = c->ring_used / 2;
  for (uint32_t i = 0; i < k && i < *n; i++) {
    HIPCHK(hipEventSynchronize(c->ring[2 * i + 1]));
    HIPCHK(hipEventElapsedTime(&ms[i], c->ring[2 * i], c->ring[2 * i + 1]));
  }
  *n = k < *n ? k : *n;
  c->ring_used = (uint32_t)c->ring.size();  // full: later launches are not recorded
  return CDR_API_OK;
}

}  // extern "C"
