/*
 * cdr/cdr.h — C ABI of the MI355X workflow-history replay engine (libcdr.so).
 *
 * Drop-in boundary for the reference's replay hot path.  Each entry point names
 * the reference interface it replaces (paths relative to /root/reference):
 *
 *   stateBuilder.applyEvents            service/history/stateBuilder.go:38-52,112-611
 *     -> cdr_replay_batch (many workflows, each a sequence of applyEvents calls on a
 *        fresh mutable state) and cdr_replay_sliced (same, device-resident input)
 *   stateBuilderProvider / newStateBuilder
 *                                       service/history/historyReplicator.go:54,144
 *                                       service/history/nDCHistoryReplicator.go:136-141
 *     -> cdr_create / cdr_destroy (one context per goroutine-equivalent / stream)
 *   nDCStateRebuilder.rebuild batch loop service/history/nDCStateRebuilder.go:92-160
 *     -> cdr_replay_batch with cdr_wf_desc.expected_next_event_id set
 *   mutableStateTaskRefresher.refreshTasks (after nDCStateRebuilder.rebuild's replay)
 *                                       service/history/mutableStateTaskRefresher.go:66-160
 *                                       service/history/nDCStateRebuilder.go:154-157
 *     -> cdr_refresh_tasks_async (device-resident) / cdr_rebuild_batch (host buffers)
 *   sql row blobs (timerInfoToBlob, requestCancelInfoToBlob)
 *                                       common/persistence/sql/workflowStateMaps.go:239-260,504-521
 *     -> cdr_encode_rows_async
 *   common.WorkflowIDToHistoryShard     common/util.go:249-252
 *     -> cdr_workflow_id_to_shard (farmhash Fingerprint32 % numShards)
 *
 * Conventions: plain C, caller-owned buffers, no exceptions across the boundary.
 * Every call is synchronous on the stream it is given unless named *_async.
 * Return value: 0 on success, a negative CDR_API_* code on API misuse / device
 * failure.  Per-workflow replay outcomes (the Go `error` of applyEvents) are in
 * cdr_wf_result.code, never in the return value.
 */
#ifndef CDR_CDR_H
#define CDR_CDR_H

#include <stddef.h>
#include <stdint.h>

#include "cdr/schema.h"

#ifdef __cplusplus
extern "C" {
#endif

#define CDR_API_OK 0
#define CDR_API_EINVAL (-1)   /* bad arguments / inconsistent batch */
#define CDR_API_ENODEV (-2)   /* no HIP device or kernel image not loadable */
#define CDR_API_EDEVICE (-3)  /* HIP runtime error */
#define CDR_API_ENOMEM (-4)

#define CDR_SLICE_WIDTH 64 /* workflows per slice = one wavefront */

/* Sliced event layout ("SELL-64" rows in a slab): workflows are grouped 64 to a
 * slice (one lane each, slices sorted by length).  Slice s owns slice_len[s]
 * consecutive rows of the slab starting at row slice_row0[s]; row k of a slice holds
 * event k of its 64 lanes, column after column (cdr_col_off below), in
 * CDR_ROW_BYTES.  A wavefront that walks its 64 histories in lockstep therefore reads
 * each column of a step as one coalesced 256/512-B access and a whole step from one
 * contiguous 3.75 KB row (DRAM-page friendly), and one buffer descriptor per slice
 * addresses every column with an immediate column offset.  The kernel reads only the
 * operand columns an event's type needs (CDR_SEF_NEED_* bits of type_flags).
 *
 * Operand columns per type (all others 0):
 *   WorkflowExecutionStarted  aux = arena word offset of cdr_attr_wf_started
 *   DecisionTaskScheduled     aux = attempt, n = StartToCloseTimeoutSeconds
 *   DecisionTaskStarted       key = scheduledEventId, h = requestId
 *   DecisionTaskCompleted     key = scheduledEventId, aux = startedEventId, h = binaryChecksum
 *   DecisionTaskTimedOut      n = timeoutType
 *   ActivityTaskScheduled     key = activityId | (u32)StartToClose << 32, h = (u32)ScheduleToClose,
 *                             n = ScheduleToStart, aux = arena word offset (< 2^32) of
 *                             cdr_attr_at_scheduled | (u32)Heartbeat << 32
 *   ActivityTask{Started,Completed,Failed,TimedOut,Canceled}  key = scheduledEventId
 *                             (Started: h = requestId)
 *   ActivityTaskCancelRequested / RequestCancelActivityTaskFailed  key = activityId
 *   Timer{Started,Fired,Canceled}, CancelTimerFailed  key = timerId (Started: aux = startToFireSeconds)
 *   StartChildWorkflowExecutionInitiated  key = domain, aux = workflowType, h = workflowId,
 *                             n = parentClosePolicy
 *   SignalExternalWorkflowExecutionInitiated  key = domain, aux = input << 32 | control, h = signalName
 *   RequestCancelExternalWorkflowExecutionInitiated  key = domain
 *                             (these three: key |= arena word offset (< 2^32) of their
 *                             cdr_attr_external << 32, read only when tasks are emitted)
 *   ChildWorkflowExecutionStarted  key = initiatedEventId, h = runId
 *   other child / external closes  key = initiatedEventId
 *   UpsertWorkflowSearchAttributes  aux = kv offset, h = kv count
 *   WorkflowExecutionContinuedAsNew  h = newExecutionRunId */
enum cdr_col {
  CDR_COL_EVENT_ID = 0, /* i64 */
  CDR_COL_VERSION,      /* i64 */
  CDR_COL_TIMESTAMP,    /* i64 */
  CDR_COL_TASK_ID,      /* i64 */
  CDR_COL_KEY,          /* i64 entity key: scheduled/initiated event id, activity/timer handle ... */
  CDR_COL_AUX,          /* i64 second operand or arena word offset (type-dependent) */
  CDR_COL_TYPE_FLAGS,   /* u32 bits 0-7 cdr_event_type, 8+ CDR_SEF_* */
  CDR_COL_H,            /* u32 string handle operand (type-dependent) */
  CDR_COL_N,            /* i32 small integer operand (type-dependent) */
  CDR_NUM_COLS
};
#define CDR_EL_BYTES 60u /* bytes of one (row, lane) element over all columns */
#define CDR_ROW_BYTES (CDR_EL_BYTES * CDR_SLICE_WIDTH) /* 3840: one event of 64 lanes */
/* element size of a column and its byte offset within a row; element (k, L) of
 * column c of a slice is at k * CDR_ROW_BYTES + cdr_col_off(c) + L * cdr_col_size(c)
 * from the slice's first row */
CDR_HD uint32_t cdr_col_size(int c) { return c < CDR_COL_TYPE_FLAGS ? 8u : 4u; }
CDR_HD uint32_t cdr_col_off(int c) {
  return CDR_SLICE_WIDTH * (c <= CDR_COL_TYPE_FLAGS ? 8u * (uint32_t)c : 48u + 4u * (uint32_t)(c - CDR_COL_TYPE_FLAGS));
}

typedef struct cdr_slices {
  uint32_t n_slices, _pad;
  uint64_t n_rows;        /* sum of slice_len */
  uint64_t arena_words;   /* 8-byte words of attribute records */
  const uint64_t* slice_row0; /* [n_slices] prefix sum of slice_len */
  const uint32_t* slice_len;  /* [n_slices] */
  const int32_t* lane_wf;     /* [n_slices*64] workflow index, -1 = empty lane */
  const uint8_t* slab;        /* n_rows * CDR_ROW_BYTES bytes of event rows */
  const uint64_t* arena; /* WorkflowExecutionStarted / ActivityTaskScheduled attribute records */
  /* working-state scratch of each slice (cdr_plan_scratch): pending activities and
   * user timers are kept lane-interleaved ("plane j*P+p, lane L") while they are live */
  const uint64_t* slice_scratch_off; /* [n_slices] 8-byte-word offset into the scratch buffer */
  const uint32_t* slice_act_slots;   /* [n_slices] activity working slots per lane */
  const uint32_t* slice_tim_slots;   /* [n_slices] user-timer working slots per lane */
  const uint32_t* slice_flags;       /* [n_slices] CDR_SLICE_* */
} cdr_slices;
#define CDR_SLICE_FAST 0x1u /* every lane's history has CDR_CAP_FAST */
/* a wave slice: ONE workflow (lane_wf[64 s]; the other lanes -1) replayed by a whole
 * wavefront (replay_wave.inc); its slice_len rows hold the workflow's events 64 at a
 * time, event k in row k/64, lane k%64 (cdr_plan_slices_ex with CDR_PLAN_WAVE) */
#define CDR_SLICE_WAVE 0x2u
/* every lane's history has CDR_CAP_REG: the slice replays in k_replay_reg
 * (replay_reg.inc: entity tables in registers, no global memory traffic in the step
 * loop beyond the event stream) */
#define CDR_SLICE_REG 0x4u
/* every lane's history has CDR_CAP_REG2 or CDR_CAP_REG: the register-table kernel's
 * variant with CDR_REG2_NA activity slots */
#define CDR_SLICE_REG2 0x8u
/* every lane's history has CDR_CAP_REG0: the register-table variant with the small tables
 * (CDR_REG0_*) at 3 waves per SIMD */
#define CDR_SLICE_REG0 0x10u
/* a lane slice of the batch's long register-table histories (cdr_plan_slices_ex with
 * CDR_PLAN_PAR; the first n_par_slices slices): replayed by k_replay_cls's four-wave
 * variant, its loops at once (replay_cls.inc), or by k_replay_reg <CDR_REG2_NA, ...> */
#define CDR_SLICE_PAR 0x20u
/* event types the fast-path kernel replays (bit = cdr_event_type) */
#define CDR_FAST_TYPES                                                                                       \
  (CDR_TB(CDR_EV_WF_STARTED) | CDR_TB(CDR_EV_WF_COMPLETED) | CDR_TB(CDR_EV_WF_FAILED) |                      \
   CDR_TB(CDR_EV_WF_TIMED_OUT) | CDR_TB(CDR_EV_DT_SCHEDULED) | CDR_TB(CDR_EV_DT_STARTED) |                   \
   CDR_TB(CDR_EV_DT_COMPLETED) | CDR_TB(CDR_EV_DT_TIMED_OUT) | CDR_TB(CDR_EV_DT_FAILED) |                    \
   CDR_TB(CDR_EV_AT_SCHEDULED) | CDR_TB(CDR_EV_AT_STARTED) | CDR_TB(CDR_EV_AT_COMPLETED) |                   \
   CDR_TB(CDR_EV_AT_FAILED) | CDR_TB(CDR_EV_AT_TIMED_OUT) | CDR_TB(CDR_EV_AT_CANCEL_REQUESTED) |             \
   CDR_TB(CDR_EV_AT_REQ_CANCEL_FAILED) | CDR_TB(CDR_EV_AT_CANCELED) | CDR_TB(CDR_EV_CANCEL_TIMER_FAILED) |   \
   CDR_TB(CDR_EV_WF_CANCEL_REQUESTED) | CDR_TB(CDR_EV_WF_CANCELED) | CDR_TB(CDR_EV_MARKER_RECORDED) |        \
   CDR_TB(CDR_EV_WF_SIGNALED) | CDR_TB(CDR_EV_WF_TERMINATED))

#define CDR_ACT_PLANES 12 /* words per activity working slot (replay.hip) */
#define CDR_TIM_PLANES 4  /* words per user-timer working slot */

#define CDR_SEF_BATCH_FIRST (1u << 8)
#define CDR_SEF_DOMAIN_MISSING (1u << 9)
/* delta bits (set by the packer for every event after an entry's first): the event's
 * event_id is the previous event's + 1 / its version equals the previous event's.  The
 * columns still hold the full values; the fast-path kernel skips loading them when
 * the bit is set (16 of the ~46 bytes a C2 event costs it) and rebuilds them from its
 * registers */
#define CDR_SEF_ID_NEXT (1u << 21)
#define CDR_SEF_VER_SAME (1u << 22)
/* operand columns the event's type reads (set by the packer from CDR_NEED_*) */
#define CDR_SEF_NEED_TS (1u << 16)
#define CDR_SEF_NEED_KEY (1u << 17)
#define CDR_SEF_NEED_AUX (1u << 18)
#define CDR_SEF_NEED_H (1u << 19)
#define CDR_SEF_NEED_N (1u << 20)
/* per-column sets of event types (bit = cdr_event_type) that read it; every type
 * reads type_flags, event_id and version (stateBuilder.go:134-155) */
#define CDR_TB(t) (1ull << (t))
#define CDR_NEED_TS                                                                                  \
  (CDR_TB(CDR_EV_WF_STARTED) | CDR_TB(CDR_EV_DT_SCHEDULED) | CDR_TB(CDR_EV_DT_STARTED) |              \
   CDR_TB(CDR_EV_AT_SCHEDULED) | CDR_TB(CDR_EV_AT_STARTED) | CDR_TB(CDR_EV_TIMER_STARTED) |            \
   CDR_TB(CDR_EV_WF_COMPLETED) | CDR_TB(CDR_EV_WF_FAILED) | CDR_TB(CDR_EV_WF_TIMED_OUT) |              \
   CDR_TB(CDR_EV_WF_CANCELED) | CDR_TB(CDR_EV_WF_TERMINATED) | CDR_TB(CDR_EV_WF_CONTINUED_AS_NEW))
#define CDR_NEED_KEY                                                                                 \
  (CDR_TB(CDR_EV_DT_STARTED) | CDR_TB(CDR_EV_AT_SCHEDULED) | CDR_TB(CDR_EV_AT_STARTED) |              \
   CDR_TB(CDR_EV_AT_COMPLETED) | CDR_TB(CDR_EV_AT_FAILED) | CDR_TB(CDR_EV_AT_TIMED_OUT) |              \
   CDR_TB(CDR_EV_AT_CANCELED) | CDR_TB(CDR_EV_AT_CANCEL_REQUESTED) | CDR_TB(CDR_EV_TIMER_STARTED) |    \
   CDR_TB(CDR_EV_TIMER_FIRED) | CDR_TB(CDR_EV_TIMER_CANCELED) | CDR_TB(CDR_EV_CHILD_INITIATED) |       \
   CDR_TB(CDR_EV_CHILD_STARTED) | CDR_TB(CDR_EV_CHILD_START_FAILED) | CDR_TB(CDR_EV_CHILD_COMPLETED) | \
   CDR_TB(CDR_EV_CHILD_FAILED) | CDR_TB(CDR_EV_CHILD_CANCELED) | CDR_TB(CDR_EV_CHILD_TIMED_OUT) |      \
   CDR_TB(CDR_EV_CHILD_TERMINATED) | CDR_TB(CDR_EV_RCE_FAILED) | CDR_TB(CDR_EV_EXT_CANCEL_REQUESTED) | \
   CDR_TB(CDR_EV_SE_FAILED) | CDR_TB(CDR_EV_EXT_SIGNALED) | CDR_TB(CDR_EV_RCE_INITIATED) |                 \
   CDR_TB(CDR_EV_SE_INITIATED))
#define CDR_NEED_AUX                                                                                 \
  (CDR_TB(CDR_EV_WF_STARTED) | CDR_TB(CDR_EV_DT_SCHEDULED) | CDR_TB(CDR_EV_DT_COMPLETED) |            \
   CDR_TB(CDR_EV_AT_SCHEDULED) | CDR_TB(CDR_EV_TIMER_STARTED) | CDR_TB(CDR_EV_CHILD_INITIATED) |       \
   CDR_TB(CDR_EV_SE_INITIATED) | CDR_TB(CDR_EV_UPSERT_SA))
#define CDR_NEED_H                                                                                   \
  (CDR_TB(CDR_EV_DT_STARTED) | CDR_TB(CDR_EV_DT_COMPLETED) | CDR_TB(CDR_EV_AT_SCHEDULED) |            \
   CDR_TB(CDR_EV_AT_STARTED) | CDR_TB(CDR_EV_CHILD_INITIATED) | CDR_TB(CDR_EV_CHILD_STARTED) |        \
   CDR_TB(CDR_EV_SE_INITIATED) | CDR_TB(CDR_EV_UPSERT_SA))
#define CDR_NEED_N \
  (CDR_TB(CDR_EV_DT_SCHEDULED) | CDR_TB(CDR_EV_DT_TIMED_OUT) | CDR_TB(CDR_EV_AT_SCHEDULED) | CDR_TB(CDR_EV_CHILD_INITIATED))
/* type_flags word of an event: type, flags and its column-need bits */
CDR_HD uint32_t cdr_type_flags(uint32_t type, uint32_t flags) {
  uint32_t tf = (type & 0xFFu) | flags;
  if (type < 64) {
    const uint64_t b = 1ull << type;
    tf |= ((CDR_NEED_TS & b) ? CDR_SEF_NEED_TS : 0u) | ((CDR_NEED_KEY & b) ? CDR_SEF_NEED_KEY : 0u) |
          ((CDR_NEED_AUX & b) ? CDR_SEF_NEED_AUX : 0u) | ((CDR_NEED_H & b) ? CDR_SEF_NEED_H : 0u) |
          ((CDR_NEED_N & b) ? CDR_SEF_NEED_N : 0u);
  }
  return tf;
}

/* everything the device needs for one replay launch (all pointers device memory) */
typedef struct cdr_dev_batch {
  cdr_slices ev;
  uint64_t* scratch; /* working-state buffer, cdr_plan_scratch words (device) */
  const cdr_wf_desc* wfs; /* [n_wfs] */
  const cdr_wf_caps* caps; /* [n_wfs] */
  const cdr_kv* kvs;
  const cdr_reset_point* rps;
  uint32_t n_wfs;
  uint32_t empty_uuid; /* handle of "emptyUuid" (mutableStateBuilder.go:42) */
  /* max over slices of slice_act_slots / slice_tim_slots (cdr_plan_scratch): the
   * launcher keeps up to this many working slots per lane in LDS (0 = all in scratch) */
  uint32_t max_act_slots, max_tim_slots;
  uint32_t n_fast_slices; /* slices with CDR_SLICE_FAST (cdr_plan_scratch) */
  uint32_t n_wave_slices; /* slices with CDR_SLICE_WAVE (cdr_plan_slices_ex) */
  uint32_t n_reg_slices;  /* slices with CDR_SLICE_REG (cdr_plan_scratch) */
  uint32_t n_reg2_slices; /* slices with CDR_SLICE_REG2 (cdr_plan_scratch) */
  uint32_t n_reg0_slices; /* slices with CDR_SLICE_REG0 (cdr_plan_scratch) */
  uint32_t n_par_slices;  /* slices with CDR_SLICE_PAR: slices 0 .. n_par_slices - 1 (cdr_plan_slices_ex) */
  /* slice index range [class_lo[c], class_hi[c]) holding every slice of kernel class c
   * (CDR_CLASS_*, cdr_plan_class_ranges): each replay kernel is launched over its range
   * only; all zero = unknown, every kernel is launched over every slice */
  uint32_t class_lo[6], class_hi[6];
  cdr_cluster_meta cluster;
  int64_t now_ns;
  uint64_t uuid_seed;
  /* device copy of the batch's cdr_carry (pointers into device memory), or NULL; its
   * entries replay with the general kernel (cdr_plan_caps clears CDR_CAP_FAST/WAVE) */
  const cdr_carry* carry;
  /* class-sorted copy of the register-table slices (cdr_cls_plan_async +
   * cdr_cls_pack_async), or NULL: slice s's block starts at row cls_row0[s] of cls_slab
   * (standard CDR_ROW_BYTES rows) and holds its lanes' W, activity, timer and external
   * events in four regions of cls_rows[4 s + 0..3] rows (CDR_CLS_*) */
  const uint8_t* cls_slab;
  const uint64_t* cls_row0; /* [n_slices + 1], exclusive scan of the blocks' rows */
  const uint32_t* cls_rows; /* [n_slices * 4] */
  /* [n_wfs] device, nullable: entries with skip[w] != 0 are not replayed by this launch —
   * their lanes stay idle and their output records untouched (the caller marks them,
   * e.g. result.code = CDR_NOT_RUN).  A masked launch replays without class-sorted blocks. */
  const uint8_t* skip;
  /* task-slice rows of the batch (cdr_totals.xfer + cdr_totals.ttask), used to size the class
   * kernels' task staging when the output asks for task lists; 0 = unknown: the launcher
   * reads the last entry's capacities from caps (a copy and a stream synchronisation) */
  uint64_t task_rows;
} cdr_dev_batch;

/* Class-sorted blocks (replay_cls.inc).  Every register-table slice (CDR_SLICE_REG /
 * REG2 / REG0) can carry a second copy of its events, permuted per lane into four
 * class regions aligned across the slice's 64 lanes: W (decision and workflow events),
 * activity events, user-timer events, external (child / request-cancel / signal)
 * events, each region in history order; MarkerRecorded, CancelTimerFailed and
 * RequestCancelActivityTaskFailed (no state of their own) are left out, and a lane with
 * fewer events of a class than the slice's maximum gets CDR_EV_PAD rows there.  Columns
 * are the standard ones except: the task_id column holds the annotation
 * CDR_CLS_ANN(k, k - k0, d) — k the event's index in its history, k0 the index of its
 * call's first event, d = event_id - NextEventID at its call (0xFFFFFFFF when that does
 * not fit) — and type_flags' bits 21 / 22 mean "event_id not needed" / "version not
 * needed or equal to the previous W event's".  The replay reads them instead of the
 * original rows for the entity FSMs (one class per step), and the original rows for the
 * call structure and the version bookkeeping. */
#define CDR_CLS_W 0
#define CDR_CLS_A 1
#define CDR_CLS_T 2
#define CDR_CLS_X 3
#define CDR_SEF_CLS_NO_ID (1u << 21)
#define CDR_SEF_CLS_VER_SAME (1u << 22)
#define CDR_CLS_ANN(k, dk, d) ((uint64_t)(k) | ((uint64_t)(dk) << 20) | ((uint64_t)(d) << 32))
#define CDR_CLS_DROP 4 /* cdr_cls_of: a type with no state of its own (only the P loop sees it) */
#define CDR_CLS_SLICES (CDR_SLICE_REG | CDR_SLICE_REG2 | CDR_SLICE_REG0 | CDR_SLICE_PAR) /* slices with a block */
#define CDR_CLS_A_TYPES                                                                                       \
  (CDR_TB(CDR_EV_AT_SCHEDULED) | CDR_TB(CDR_EV_AT_STARTED) | CDR_TB(CDR_EV_AT_COMPLETED) |                    \
   CDR_TB(CDR_EV_AT_FAILED) | CDR_TB(CDR_EV_AT_TIMED_OUT) | CDR_TB(CDR_EV_AT_CANCELED) |                      \
   CDR_TB(CDR_EV_AT_CANCEL_REQUESTED))
#define CDR_CLS_T_TYPES (CDR_TB(CDR_EV_TIMER_STARTED) | CDR_TB(CDR_EV_TIMER_FIRED) | CDR_TB(CDR_EV_TIMER_CANCELED))
#define CDR_CLS_X_TYPES                                                                                         \
  (CDR_TB(CDR_EV_CHILD_INITIATED) | CDR_TB(CDR_EV_CHILD_STARTED) | CDR_TB(CDR_EV_CHILD_START_FAILED) |         \
   CDR_TB(CDR_EV_CHILD_COMPLETED) | CDR_TB(CDR_EV_CHILD_FAILED) | CDR_TB(CDR_EV_CHILD_CANCELED) |              \
   CDR_TB(CDR_EV_CHILD_TIMED_OUT) | CDR_TB(CDR_EV_CHILD_TERMINATED) | CDR_TB(CDR_EV_RCE_INITIATED) |           \
   CDR_TB(CDR_EV_RCE_FAILED) | CDR_TB(CDR_EV_EXT_CANCEL_REQUESTED) | CDR_TB(CDR_EV_SE_INITIATED) |             \
   CDR_TB(CDR_EV_SE_FAILED) | CDR_TB(CDR_EV_EXT_SIGNALED))
#define CDR_CLS_DROP_TYPES \
  (CDR_TB(CDR_EV_MARKER_RECORDED) | CDR_TB(CDR_EV_CANCEL_TIMER_FAILED) | CDR_TB(CDR_EV_AT_REQ_CANCEL_FAILED))
/* class-sorted events whose event_id a class loop reads (the others get CDR_SEF_CLS_NO_ID) */
#define CDR_CLS_NEED_ID                                                                                          \
  (CDR_TB(CDR_EV_WF_STARTED) | CDR_TB(CDR_EV_DT_SCHEDULED) | CDR_TB(CDR_EV_DT_STARTED) |                         \
   CDR_TB(CDR_EV_DT_TIMED_OUT) | CDR_TB(CDR_EV_DT_FAILED) | CDR_TB(CDR_EV_AT_SCHEDULED) |                        \
   CDR_TB(CDR_EV_TIMER_STARTED) | CDR_TB(CDR_EV_CHILD_INITIATED) | CDR_TB(CDR_EV_RCE_INITIATED) |                 \
   CDR_TB(CDR_EV_SE_INITIATED))
/* class region of an event type (CDR_CLS_W / A / T / X, or CDR_CLS_DROP); unknown types
 * go to W, whose loop reports them */
CDR_HD uint32_t cdr_cls_of(uint32_t type) {
  if (type >= 64) return CDR_CLS_W;
  const uint64_t b = 1ull << type;
  return (b & CDR_CLS_A_TYPES)      ? (uint32_t)CDR_CLS_A
         : (b & CDR_CLS_T_TYPES)    ? (uint32_t)CDR_CLS_T
         : (b & CDR_CLS_X_TYPES)    ? (uint32_t)CDR_CLS_X
         : (b & CDR_CLS_DROP_TYPES) ? (uint32_t)CDR_CLS_DROP
                                    : (uint32_t)CDR_CLS_W;
}

/* ------------------------------------------------------------ host planning */

/* Per-workflow output capacities (upper bounds derived from the input: counts of
 * entity-creating events, version runs, reset points, search-attribute pairs)
 * and their prefix offsets. */
int cdr_plan_caps(const cdr_batch* b, cdr_wf_caps* caps, cdr_totals* totals);

/* Slice assignment: workflows sorted by event count (descending, stable) and
 * dealt 64 to a slice.  Outputs lane_wf[n_slices*64], slice_len[n_slices],
 * slice_row0[n_slices]; returns n_slices via *n_slices and rows via *n_rows.
 * Call with lane_wf == NULL to query sizes only. */
int cdr_plan_slices(const cdr_wf_desc* wfs, uint32_t n_wfs, int32_t* lane_wf, uint32_t* slice_len,
                    uint64_t* slice_row0, uint32_t* n_slices, uint64_t* n_rows);

/* As cdr_plan_slices, with a mode: CDR_PLAN_WAVE gives every entry whose caps carry
 * CDR_CAP_WAVE and neither register-table cap (CDR_CAP_REG / REG2) a wave slice of its
 * own (after the lane slices, longest first) and
 * marks it in slice_flags (nullable; the other slices get 0).  `caps` may be NULL
 * when mode is 0.  Returns the number of wave slices via *n_wave (nullable). */
#define CDR_PLAN_WAVE 0x1u
/* with CDR_PLAN_WAVE: also the register-table entries get wave slices (by default they
 * stay in lane slices, where they replay cheaper) */
#define CDR_PLAN_WAVE_ALL 0x2u
/* with CDR_PLAN_WAVE the planner also gives a wave slice to every CDR_CAP_WAVE entry
 * whose history is longer than T = max(CDR_LONG_MIN, CDR_LONG_FACTOR x the lane events
 * per resident lane slot, i.e. lane events / (64 x CDR_LANE_RESIDENT)) — T /
 * CDR_LONG_REG2_DIV (at least CDR_LONG_MIN / 2) for CDR_CAP_REG2 entries: such a history
 * alone would set the lane kernels' critical path.  This bit turns that rule off. */
#define CDR_PLAN_NO_LONG 0x4u
/* with CDR_PLAN_WAVE (default on): the long register-table histories the rule above would
 * give wave slices go instead to CDR_SLICE_PAR lane slices (longest first, CDR_PAR_LANES to
 * a slice, the first slices of the plan), where the class-decomposed kernel runs their
 * loops on four waves at once */
#define CDR_PLAN_PAR 0x8u
/* with CDR_PLAN_PAR: every PAR history alone in its slice, the CDR_PAR_SOLO_MAX longest at most —
 * the plan of batches with task lists, whose PAR slices replay on k_replay_reg<TASKS>: a row there
 * costs the union of the handler groups its lanes hit, so one history per slice steps one group
 * (C5 --tasks 23.6 -> 16.0 ms; the PAR class kernel emits no tasks) */
#define CDR_PLAN_PAR_SOLO 0x10u
#define CDR_PAR_SOLO_MAX 512u
#define CDR_PAR_LANES 16u /* histories per CDR_SLICE_PAR slice (lanes 0 .. 15; the rest empty) */
#define CDR_PAR_SOLO 0u   /* ... except the longest CDR_PAR_SOLO, one per slice */
#define CDR_PAR_SOLO_LEN 16384u /* ... and every PAR history at least this long, one per slice
                                   (k_replay_cls: its class loops in wave form) */
#define CDR_PAR_MAX_SLICES 128u /* at most this many PAR slices (the longest histories); the rest stay lane slices */
#define CDR_LONG_MIN 1024u
#define CDR_LONG_FACTOR 2u
#define CDR_LONG_REG2_DIV 2u
#define CDR_PAR_FACTOR 1u /* CDR_PLAN_PAR: the long threshold's factor for PAR slices */
#define CDR_LANE_RESIDENT 2048u
int cdr_plan_slices_ex(const cdr_wf_desc* wfs, const cdr_wf_caps* caps, uint32_t n_wfs, uint32_t mode,
                       int32_t* lane_wf, uint32_t* slice_len, uint64_t* slice_row0, uint32_t* slice_flags,
                       uint32_t* n_slices, uint64_t* n_rows, uint32_t* n_wave);

/* Working-state scratch layout: per slice, slots = max over its lanes of the live
 * bounds in caps, and the slice's CDR_SLICE_* flags (CDR_SLICE_WAVE, when set on input by
 * cdr_plan_slices_ex, is kept and such slices get no scratch); returns the total words via
 * *total_words and the number of CDR_SLICE_FAST slices via *n_fast (nullable).
 * Outputs sized [n_slices]; pass NULL outputs to query the totals only. */
/* Kernel classes of the slices (by their CDR_SLICE_* flags) and the index range each
 * class's slices span: lo[c] = first, hi[c] = last + 1 (0, 0 for an absent class).  The
 * planner above puts a class's slices next to each other, so a range holds only its
 * class's slices; the kernels check the flags, so any order stays correct. */
enum cdr_kernel_class {
  CDR_CLASS_FAST = 0, CDR_CLASS_REG0 = 1, CDR_CLASS_REG = 2, CDR_CLASS_REG2 = 3, CDR_CLASS_WAVE = 4,
  CDR_CLASS_GENERAL = 5
};
int cdr_plan_class_ranges(const uint32_t* slice_flags, uint32_t n_slices, uint32_t* lo, uint32_t* hi);
int cdr_plan_scratch(const cdr_wf_caps* caps, const int32_t* lane_wf, uint32_t n_slices, uint64_t* scratch_off,
                     uint32_t* act_slots, uint32_t* tim_slots, uint32_t* slice_flags, uint64_t* total_words,
                     uint32_t* n_fast);

/* Arena words needed by the batch's attribute records. */
uint64_t cdr_plan_arena_words(const cdr_batch* b);

/* Pack the natural-order batch into the sliced columns (host memory, sized by the
 * planners above).  Columns are passed through a cdr_slices whose pointers are
 * cast away from const by the packer.  `threads` host threads (<=0: hardware). */
int cdr_pack_slices(const cdr_batch* b, cdr_slices* out, int threads);

/* ------------------------------------------------------------- device entry */

typedef struct cdr_ctx cdr_ctx;
/* Context options (cdr_opts_default fills the defaults). */
typedef struct cdr_opts {
  uint32_t plan_mode;       /* CDR_PLAN_* of the host-buffer calls' planning (CDR_PLAN_WAVE) */
  int32_t fast_path;        /* CDR_SLICE_FAST / REG / REG2 slices on their kernels (1) */
  int32_t reg_path;         /* CDR_SLICE_REG / REG2 slices on k_replay_reg (1) */
  int32_t concurrent;       /* wave-kernel slices on a side stream, concurrent with the lane kernels (1) */
  uint64_t workspace_bytes; /* device bytes reserved at creation for the host-buffer calls' event slab
                             * (0: on demand; the workspace only grows) */
} cdr_opts;
void cdr_opts_default(cdr_opts* opts);
/* A context on HIP device `device` (opts NULL: defaults); NULL when the device is absent
 * or its kernel image cannot load — there is no CPU fallback. */
cdr_ctx* cdr_create(int device, const cdr_opts* opts);
void cdr_destroy(cdr_ctx* ctx);

/* Route CDR_SLICE_FAST slices to the fast-path kernel and CDR_SLICE_REG slices to the
 * register-table kernel (default 1) or replay every lane slice with the general kernel
 * (0; parity tests run both).  Returns the old value. */
int cdr_set_fast_path(cdr_ctx* ctx, int enable);
/* Route CDR_SLICE_REG slices to k_replay_reg (default 1) or to the general kernel (0);
 * returns the old value. */
int cdr_set_reg_path(cdr_ctx* ctx, int enable);
/* Replay register-table slices that carry a class-sorted block (cdr_dev_batch.cls_slab)
 * with the class-decomposed kernel k_replay_cls (entries it leaves CLS_RETRY go through
 * k_replay_reg) or with k_replay_reg alone (CDR_CLS_OFF).  Modes:
 *   CDR_CLS_OFF      k_replay_reg alone
 *   CDR_CLS_ON       (default) k_replay_cls for device-resident batches that carry blocks
 *                    (the packer emitted them: cdr_pack_cls); the host-buffer calls
 *                    (cdr_replay_batch / cdr_rebuild_batch / cdr_replay_one) build none —
 *                    a batch replayed once pays more for its block (packing + H2D of a
 *                    second copy of the slab) than k_replay_cls saves over k_replay_reg
 *   CDR_CLS_ALONE    (tests) as CDR_CLS_BUILD, with no k_replay_reg pass, so an entry it
 *                    hands on keeps the internal result code 0x7FFF
 *   CDR_CLS_BUILD    as CDR_CLS_ON, and the host-buffer calls pack blocks too (host packer)
 * Returns the old mode. */
#define CDR_CLS_OFF 0
#define CDR_CLS_ON 1
#define CDR_CLS_ALONE 2
#define CDR_CLS_BUILD 3
int cdr_set_cls_path(cdr_ctx* ctx, int mode);

/* Host packer of the class-sorted blocks (the layout above), from a packed host slab
 * (cdr_pack_slices / the synthetic generator) and the entries' descriptors (ev_len):
 * cdr_plan_cls writes cls_rows[4 s + c] (n_slices * 4: the rows of each class region of
 * every CDR_CLS_SLICES slice, 0 for the others) and cls_row0[0..n_slices] (their
 * exclusive scan; cls_row0[n_slices] = total rows); cdr_pack_cls then writes the blocks
 * into cls_slab (total * CDR_ROW_BYTES bytes; padding elements carry type_flags
 * CDR_EV_PAD | CDR_SEF_CLS_NO_ID | CDR_SEF_CLS_VER_SAME and zero columns).  Byte for byte
 * the blocks cdr_cls_plan_async / cdr_cls_pack_async build on the device (padding
 * elements' other columns aside).  `threads` host threads (<= 0: hardware). */
int cdr_plan_cls(const cdr_slices* s, const cdr_wf_desc* wfs, uint32_t* cls_rows, uint64_t* cls_row0);
int cdr_pack_cls(const cdr_slices* s, const cdr_wf_desc* wfs, const uint32_t* cls_rows, const uint64_t* cls_row0,
                 uint8_t* cls_slab, int threads);

/* Size pass of the class-sorted blocks (see cdr_dev_batch.cls_slab): cls_rows[4 s + c]
 * (device, n_slices * 4) = the rows of each class region of every register-table slice
 * (0 for the others) and cls_row0[0..n_slices] (device, n_slices + 1) their exclusive
 * scan; the caller reads the total, cls_row0[n_slices], and allocates cls_slab at
 * total * CDR_ROW_BYTES bytes.  It also keeps, in the context's workspace (16 B per slab
 * element), each event's class position, block type word and annotation for the write pass.
 * Asynchronous. */
int cdr_cls_plan_async(cdr_ctx* ctx, const cdr_dev_batch* in, uint32_t* cls_rows, uint64_t* cls_row0,
                       void* stream);
/* Write pass: the class-sorted blocks into in->cls_slab at in->cls_row0 / cls_rows (from
 * cdr_cls_plan_async on the same batch, the last plan on this context): a transposition
 * through LDS, column by column, one workgroup per slice (slices longer than its LDS budget,
 * and every slice when the plan's map is not this batch's: a per-lane scatter).
 * Asynchronous. */
int cdr_cls_pack_async(cdr_ctx* ctx, const cdr_dev_batch* in, void* stream);

/* Slicing mode of cdr_replay_batch's planning (CDR_PLAN_*; default CDR_PLAN_WAVE).
 * Returns the previous mode. */
int cdr_set_plan_mode(cdr_ctx* ctx, uint32_t mode);

/* Replay a device-resident sliced batch into device-resident outputs on `stream`
 * (a hipStream_t; NULL = default stream).  Asynchronous: enqueues the replay
 * kernel and the continue-as-new finalize kernel and returns.
 * A context's asynchronous calls all go on ONE stream, in order: the retry lists and the
 * side streams the kernel classes fork onto are the context's (per-context workspace), so
 * two calls in flight on one context from different streams would share them.  Use one
 * context per stream (per goroutine in the cgo shim).
 * Carry-in (in->carry): loaded entries replay in the register-table kernels' carry-in
 * instantiations (their slices) or the general kernel; an entry whose loaded state
 * outgrows its variant is handed on, on the device, to the 12-activity variant and then to
 * the general kernel (replay_reg.inc).  Never plan a loaded entry onto a fast or wave slice
 * (cdr_plan_caps / cdr_plan_ndc_apply never do: CDR_CAP_LOADED).
 * Task lists (out->transfer set) with class-sorted blocks (in->cls_slab): the class kernels
 * stage each entry's tasks per class in the context's workspace and merge them on the device
 * (replay_cls.inc, k_tasks_merge); the workspace is sized from the batch's task-slice total,
 * which the first launch over a batch (a new in->caps pointer or entry count) reads back with
 * one blocking 40-byte copy of in->caps[n_wfs - 1] — later launches over the same batch stay
 * fully asynchronous.  A plan with task lists must have no wave slices (CDR_API_EINVAL). */
int cdr_replay_sliced_async(cdr_ctx* ctx, const cdr_dev_batch* in, const cdr_out* out, void* stream);

/* Whole pipeline for host-resident data: plan + pack + H2D + replay + D2H on `stream`
 * (a hipStream_t; NULL = the default stream).  `caps` must come from cdr_plan_caps on the
 * same batch; `out` points at host buffers sized by its totals (out->last_decision, if
 * set, at n_wfs records).  Device buffers come from the context's grow-only workspace:
 * a warmed-up context allocates nothing.  Synchronous on `stream`; one call at a time
 * per context. */
int cdr_replay_batch(cdr_ctx* ctx, const cdr_batch* b, const cdr_wf_caps* caps, const cdr_totals* totals,
                     cdr_out* out, void* stream);

/* The drop-in applyEvents shim's call: the sequence of applyEvents calls
 * of ONE workflow — `b` holds its entry (0) and, when its history continues as new, the
 * new run's entry (b->n_wfs 1 or 2).  The context plans the capacities itself and
 * replays into its own host buffers: *view receives the outputs (tables at the
 * offsets in *caps, last_decision set), valid until the next call on `ctx`.  Synchronous
 * on `stream`. */
int cdr_replay_one(cdr_ctx* ctx, const cdr_batch* b, const cdr_out** view, const cdr_wf_caps** caps, void* stream);

/* refreshTasks (mutableStateTaskRefresher.go:66-160) over the rebuilt states of a
 * replay: run after cdr_replay_sliced_async on the same `in` / `out` (same stream).
 * For every entry whose result is CDR_OK it regenerates the transfer and timer tasks
 * of the rebuilt state at time `now_ns` into out->transfer / out->timer_tasks (the
 * entry's caps.xfer_off / ttask_off slices, counts in out->n_tasks — the stateBuilder
 * lists, if any, are replaced), clears every pending activity's TimerTaskStatus and
 * every user timer's TaskID and sets the ones the activity / user-timer picks created
 * (:264-342).  Events the refresher reads (WorkflowExecutionStarted, the scheduled /
 * initiated events of pending entities — the reference's events cache) are looked up
 * among the entry's own events in `in`; a miss, a Decider initiator with a first-decision
 * backoff, an unknown target domain or an overflowing task slice set the entry's
 * result.code (CDR_E_REFRESH_*, CDR_E_DOMAIN_NOT_FOUND) and leave its tables unchanged
 * with no tasks.  `flags`: CDR_REFRESH_ADVANCED_VISIBILITY adds the
 * UpsertWorkflowSearchAttributes task (:148-156); CDR_REFRESH_SNAPSHOT_PASSIVE below.
 * Asynchronous. */
#define CDR_REFRESH_ADVANCED_VISIBILITY 0x1u
/* then CloseTransactionAsSnapshot(now, transactionPolicyPassive)
 * (mutableStateBuilder.go:3787-3855): with the passive policy and no new events its only
 * effect on the outputs is setTaskInfo (historyEngine.go:2383-2397) — every task's Version
 * becomes GetCurrentVersion() (LastUpdatedTimestamp = now is the caller's: the record
 * omits it) */
#define CDR_REFRESH_SNAPSHOT_PASSIVE 0x2u
int cdr_refresh_tasks_async(cdr_ctx* ctx, const cdr_dev_batch* in, const cdr_out* out, int64_t now_ns,
                            uint32_t flags, void* stream);

/* nDCStateRebuilder.rebuild's replay + refreshTasks for host-resident data: as
 * cdr_replay_batch, then cdr_refresh_tasks_async at b->now_ns.  out->transfer,
 * timer_tasks and n_tasks are required (sized by `totals`).  Synchronous on `stream`. */
int cdr_rebuild_batch(cdr_ctx* ctx, const cdr_batch* b, const cdr_wf_caps* caps, const cdr_totals* totals,
                      cdr_out* out, uint32_t flags, void* stream);

/* Persisted-format row encoders: the SQL persistence's per-row blobs,
 * thriftrw binary protocol (common/persistence/sql/blob.go:61-73, protocol.Binary) of
 * the sqlblobs structs the row writers build (common/persistence/sql/workflowStateMaps.go):
 *   table 1  TimerInfo{Version, StartedID, ExpiryTimeNanos, TaskID}
 *            (sqlblobs.thrift:201-206, workflowStateMaps.go:242-247): CDR_BLOB_TIMER_BYTES
 *   table 3  RequestCancelInfo{Version, InitiatedEventBatchID, CancelRequestID}
 *            (sqlblobs.thrift:195-199, workflowStateMaps.go:507-511): CDR_BLOB_CANCEL_BYTES;
 *            CancelRequestID is the row's UUID in RFC 4122 text form (hi then lo, 8-4-4-4-12
 *            lowercase hex)
 * Every field is set (the row writers pass pointers), so each blob has a fixed size
 * (CDR_BLOB_*_BYTES); row r of the table (caps.*_off + j) is written to the 16-B aligned
 * slot blobs + r * CDR_BLOB_*_STRIDE (its first *_BYTES bytes are the blob, the rest
 * zero), for the rows j < result.n_* of every CDR_OK entry (other slots untouched);
 * `blobs` must be 16-B aligned.  Asynchronous. */
#define CDR_BLOB_TIMER_BYTES 45u
#define CDR_BLOB_TIMER_STRIDE 48u
#define CDR_BLOB_CANCEL_BYTES 66u
#define CDR_BLOB_CANCEL_STRIDE 80u
int cdr_encode_rows_async(cdr_ctx* ctx, int table, const cdr_dev_batch* in, const cdr_out* out, uint8_t* blobs,
                          void* stream);

/* The variable-size row blobs (encode_var.hip):
 *   table 0  ActivityInfo        (sqlblobs.thrift:136-168, workflowStateMaps.go:48-83)
 *   table 2  ChildExecutionInfo  (sqlblobs.thrift:170-184, workflowStateMaps.go:371-385)
 *   table 4  SignalInfo          (sqlblobs.thrift:186-193, workflowStateMaps.go:632-639)
 *   table 5  WorkflowExecutionInfo of the execution row (sqlblobs.thrift:73-134,
 *            buildExecutionRow sqlExecutionManagerUtil.go:1197-1308), one row per entry
 * Strings come from a device string table (handle h's bytes are bytes[off[h], off[h+1]),
 * handle 0 = "" / nil).  Its conventions: a plain string or binary field is its bytes; a
 * NonRetriableErrors handle holds the wire body of the list<string> (element type, i32
 * count, elements) and a Memo handle the wire body of the Memo struct — what
 * cdr_ingest_decode interns.  UUID-typed binaries (ParentDomainID, ParentRunID,
 * StartedRunID) are MustParseUUID of their strings; ID strings the replay generates
 * (CreateRequestID, SignalRequestID, the branch ID) are RFC 4122 text of their 128 bits.
 * Go's map iteration order is random, so the reference has no fixed byte order for the
 * map fields (LastReplicationInfo, SearchAttributes, Memo): they are written in cluster-
 * index, row and input order.  Not carried by the replay projection, and so written as a
 * fresh replay leaves them: ScheduledEvent / StartedEvent / InitiatedEvent (nil),
 * CompletionEvent (nil), the branch's ancestors ([]); the execution row's fields outside
 * the projection come from cdr_exec_persist.
 * Two calls: with blobs == NULL, a size pass and an exclusive scan write row_off[0..n_rows]
 * (device, n_rows + 1: row r's blob is bytes [row_off[r], row_off[r+1]) — zero-length for
 * rows past an entry's count and for entries that did not replay OK) and per-row
 * CDR_BLOB_* status codes into row_status (device, nullable); the caller reads
 * row_off[n_rows] (the total), allocates `blobs` and calls again to write them.  Rows are
 * the table's capacity rows (caps.*_off + j; n_rows = the table's total capacity), for
 * table 5 the entries (n_rows = n_wfs); cluster_names[i] (device) is the handle of cluster
 * i's name, the LastReplicationInfo key of 2DC entries.  Asynchronous on `stream`. */
typedef struct cdr_strtab {
  const uint8_t* bytes; /* device */
  const uint64_t* off;  /* device, n + 1 */
  uint32_t n, _pad;
} cdr_strtab;
/* per-entry inputs of buildExecutionRow outside the replay projection */
typedef struct cdr_exec_persist {
  int64_t start_version, current_version; /* buildExecutionRow's startVersion / currentVersion */
  int64_t start_time, last_updated_time;  /* UnixNano (CDR_ZERO_TIME_NANOS: Go's zero time) */
  int64_t history_size, sticky_s2s_timeout;
  uint32_t execution_context, sticky_task_list; /* handles */
  uint32_t client_library_version, client_feature_version, client_impl, _pad;
} cdr_exec_persist;
#define CDR_ZERO_TIME_NANOS (-6795364578871345152ll) /* time.Time{}.UnixNano() */
#define CDR_BLOB_OK 0
#define CDR_BLOB_E_UUID 1   /* MustParseUUID would panic on the string */
#define CDR_BLOB_E_HANDLE 2 /* a handle past the string table */
#define CDR_BLOB_E_MEMO 3   /* the Memo handle does not hold a Memo struct body */
int cdr_encode_blobs_async(cdr_ctx* ctx, int table, const cdr_dev_batch* in, const cdr_out* out,
                           const cdr_strtab* strs, const cdr_exec_persist* persist, const uint32_t* cluster_names,
                           uint64_t n_rows, uint64_t* row_off, uint8_t* blobs, int32_t* row_status, void* stream);

/* The Cassandra persistence's form of the same rows (common/persistence/cassandra/
 * cassandraPersistenceUtil.go; CQL templates cassandraPersistence.go:114-306,439-520): per row
 * the values the statement that writes it binds, in order, each a CQL native-protocol [bytes]
 * value — big-endian int32 length (-1 = null), then the value as gocql (v0.0.0-20171220143535-
 * 56a164ee9f31, go.mod:22) marshals it for the column's CQL type: bigint / int big-endian,
 * boolean one byte, double IEEE big-endian, timestamp milliseconds since the epoch (the zero
 * time.Time: zero bytes), text / blob the bytes (a nil []byte: null), uuid the 16 bytes gocql's
 * ParseUUID reads from the string (CDR_BLOB_E_UUID where it fails), list<text> / map<text, blob>
 * an int32 count and the [bytes] elements, a UDT its fields' [bytes] in declaration order.
 *   table 0  activity_map[schedule_id] = activity_info (updateActivityInfos :1264-1337): the
 *            key, then the UDT's 33 fields
 *   table 1  timer_map[timer_id] = timer_info (updateTimerInfos :1384-1422)
 *   table 2  child_executions_map[initiated_id] = child_execution_info (:1444-1503; "" started
 *            run -> emptyRunID)
 *   table 3  request_cancel_map[initiated_id] = request_cancel_info (:1530-1568)
 *   table 4  signal_map[initiated_id] = signal_info (:1590-1631)
 *   table 5  the execution row's SET values of updateExecution (:625-890): the
 *            workflow_execution UDT's 58 fields (no parent -> emptyDomainID / "" / emptyRunID /
 *            emptyInitiatedID), then the 2DC replication_state's 5 (last_replication_info
 *            a map<text, frozen<replication_info>> keyed by cluster_names) and next_event_id,
 *            or next_event_id, version_histories and its encoding (NDC), or next_event_id
 *            (local); what the projection does not carry comes from `persist`, as for table 5
 *            of cdr_encode_blobs_async
 * The statements' WHERE / IF values (shard, row type, the execution's keys, the condition) are
 * the caller's.  Map iteration order is Go's random order in the reference; maps are written
 * in input / cluster-index order.  Two calls (sizes, then values) as cdr_encode_blobs_async. */
int cdr_encode_cql_async(cdr_ctx* ctx, int table, const cdr_dev_batch* in, const cdr_out* out,
                         const cdr_strtab* strs, const cdr_exec_persist* persist, const uint32_t* cluster_names,
                         uint64_t n_rows, uint64_t* row_off, uint8_t* values, int32_t* row_status, void* stream);

/* Stream compaction of the per-workflow pending tables into dense tables
 * (device pointers): for each table, rows [caps.off, caps.off + result.n) of every
 * workflow are copied to dense[row_base[w] ...]; row_base is an exclusive scan of
 * the counts (written to `row_base` [n_wfs+1]).  Tables: 0 activity, 1 timer,
 * 2 child, 3 cancel, 4 signal. */
int cdr_compact_async(cdr_ctx* ctx, int table, const cdr_dev_batch* in, const cdr_out* out, void* dense,
                      uint64_t* row_base, void* stream);

/* Order-independent 64-bit checksum of every OK workflow's outputs (sum over
 * workflows of a per-workflow hash) — reduced across GPUs with RCCL by the
 * multi-GPU driver.  Writes one u64 to `*dev_sum` (device memory). */
int cdr_checksum_async(cdr_ctx* ctx, const cdr_dev_batch* in, const cdr_out* out, uint64_t* dev_sum,
                       void* stream);
/* The same, plus each entry's hash in per_entry[n_wfs] (device memory, nullable): the
 * full-size parity check compares these entry by entry with the CPU restatement's
 * (oracle/digest_ref.cpp restates the hash).  Hash of entry w: a fold of cdr_mix64 over
 * (code | flags << 32), fail_event_id and, when OK, the 8-byte words of its ExecutionInfo,
 * ReplicationState (2DC builder), version-history items, pending rows, reset points and
 * search attributes — the CopyToPersistence projection (mutableStateBuilder.go:257-270). */
int cdr_entry_digests_async(cdr_ctx* ctx, const cdr_dev_batch* in, const cdr_out* out, uint64_t* per_entry,
                            uint64_t* dev_sum, void* stream);

/* ------------------------------------------------ NDC branches (ndc.hip) */
/* Conflict resolution around the replay when replication tasks fork a history
 * (SURVEY §8(d) C5).  Per workflow w (all pointers device memory):
 *
 *   cdr_ndc_branch_async: task[w] against the workflow's persisted VersionHistories
 *     vhs[w] (items in `pool`): nDCBranchMgr.prepareVersionHistory
 *     (service/history/nDCBranchMgr.go:80-249: FindLCAVersionHistoryIndexAndItem,
 *     IsLCAAppendable, verifyEventsOrder, DuplicateUntilLCAItem + createNewBranch's
 *     AddVersionHistory) then nDCConflictResolver.prepareMutableState
 *     (nDCConflictResolver.go:73-114), and for a lower-version task on a non-current
 *     branch the backfill's AddOrUpdateItem (nDCHistoryReplicator.go:437-447).  vhs[w]
 *     is updated only when dec[w].code is CDR_OK; dec[w].action says what the caller
 *     replays next (CDR_NDC_*).
 *   cdr_ndc_rebuild_verify_async: after the rebuild replay of every CDR_NDC_REBUILD
 *     workflow (entry w of `out`, NDC builder, expected_next_event_id =
 *     dec[w].rebuild_next_event_id — nDCStateRebuilder.rebuild, nDCStateRebuilder.go:92-160):
 *     SetCurrentBranchToken(dec[w].rebuild_token), the rebuilt VersionHistory must equal
 *     the branch's (else result.code = CDR_E_REBUILD_VH_MISMATCH, nDCConflictResolver.go:
 *     154-165), then vhs[w].current = the branch (SetCurrentVersionHistoryIndex, :172-174).
 *   cdr_vhs_sync_async: after a replay applied to the current branch, its VersionHistory
 *     (the replay output's items and token) becomes branch vhs[w].current (a workflow
 *     with no branch gets its first, NewVersionHistories).  Needs items_cap >= the
 *     entry's caps.vh_cap.
 * Asynchronous on `stream`. */
int cdr_ndc_branch_async(cdr_ctx* ctx, const cdr_ndc_task* tasks, const cdr_vh_item* task_items, uint32_t n,
                         cdr_vhs* vhs, cdr_vh_item* pool, cdr_ndc_decision* dec, void* stream);
int cdr_ndc_rebuild_verify_async(cdr_ctx* ctx, uint32_t n, const cdr_ndc_decision* dec, cdr_vhs* vhs,
                                 const cdr_vh_item* pool, const cdr_wf_caps* caps, const cdr_out* out, void* stream);
int cdr_vhs_sync_async(cdr_ctx* ctx, uint32_t n, cdr_vhs* vhs, cdr_vh_item* pool, const cdr_wf_caps* caps,
                       const cdr_out* out, void* stream);

/* One round of NDC replication tasks over n workflows, device-resident end to end — the
 * batch form of nDCHistoryReplicator.applyNonStartEvents (service/history/
 * nDCHistoryReplicator.go:246-470) for task w of workflow w:
 *   1. nDCBranchMgr.prepareVersionHistory + nDCConflictResolver.prepareMutableState
 *      (k_ndc_branch, as cdr_ndc_branch_async) -> dec[w];
 *   2. CDR_NDC_REBUILD: nDCStateRebuilder.rebuild (nDCStateRebuilder.go:92-160) — entry w of
 *      `rebuild` replayed on a fresh NDC builder (the other entries masked), the
 *      next-event check, SetCurrentBranchToken, refreshTasks at refresh_now (its tasks in
 *      rebuild_out) — then nDCConflictResolver.rebuild's verification and branch switch
 *      (nDCConflictResolver.go:117-184, as cdr_ndc_rebuild_verify_async);
 *   3. applyNonStartEventsToCurrentBranch (:330-398): entry w of `apply` replayed onto the
 *      REBUILT state kept in memory (cdr_carry.in_memory: no Load) or, for
 *      CDR_NDC_APPLY_CURRENT, onto the loaded current state; its VersionHistory becomes the
 *      current branch's (as cdr_vhs_sync_async);
 *   4. `state` (device records with per-entry capacities state_caps) := the applied state;
 *      a task that fails leaves its error in state->result[w] (that workflow is skipped by
 *      later rounds); skipped / backfilled tasks leave the state as it was.
 * `rebuild` / `apply` are device-resident batches (host structs holding device pointers)
 * with entry w = workflow w and no continue-as-new entries; `apply` is planned with
 * cdr_plan_ndc_apply(state_caps) and both without class-sorted blocks.  rebuild_out needs
 * transfer / timer_tasks / n_tasks (the refresher's task lists).  Entries a step does not
 * run have result.code CDR_NOT_RUN in that step's output.  No device allocation once the
 * context's workspace is warm; asynchronous on `stream`. */
typedef struct cdr_ndc_round {
  const cdr_ndc_task* tasks;     /* [n] device */
  const cdr_vh_item* task_items; /* device */
  cdr_dev_batch rebuild;
  cdr_out rebuild_out;
  cdr_dev_batch apply;
  cdr_out apply_out;
  cdr_ndc_decision* dec; /* [n] device, out */
  int64_t refresh_now;   /* nDCStateRebuilder.rebuild's `now` */
  uint32_t refresh_flags, _pad; /* CDR_REFRESH_* of the rebuild's refreshTasks */
} cdr_ndc_round;
int cdr_ndc_replicate_async(cdr_ctx* ctx, uint32_t n, const cdr_ndc_round* round, cdr_vhs* vhs, cdr_vh_item* pool,
                            const cdr_wf_caps* state_caps, const cdr_out* state, void* stream);
/* Capacities of a round's `apply` batch (cdr_plan_caps restated for carry-in entries whose
 * loaded state has at most state_caps[w] rows; every entry replays in the general kernel). */
int cdr_plan_ndc_apply(const cdr_batch* b, const cdr_wf_caps* state_caps, cdr_wf_caps* caps, cdr_totals* totals);

/* ------------------------------------------------------------------ misc */

/* farmhash Fingerprint32(workflowID) % numShards (common/util.go:249-252) */
uint32_t cdr_fingerprint32(const char* s, size_t len);
int32_t cdr_workflow_id_to_shard(const char* workflow_id, size_t len, int32_t num_shards);

/* Kernel statistics of the last replay launch on ctx: average duration (ms) of
 * the replay kernel measured with HIP events on the launch stream. */
int cdr_last_kernel_ms(cdr_ctx* ctx, float* replay_ms, float* finalize_ms);

/* Per-launch timing ring: record the replay kernel of the next max_launches launches
 * with HIP events on their stream; read back durations (ms) after the fact. */
int cdr_timing_begin(cdr_ctx* ctx, uint32_t max_launches);
int cdr_timing_read(cdr_ctx* ctx, float* ms, uint32_t* n);

const char* cdr_version(void);

/* The measurement's bandwidth ceiling: copy `bytes` (a multiple of 64) from src to dst on
 * `stream` with 16-B vector loads and stores, one per lane, one-shot grid (the MI355X guide's
 * float4 copy, ~6.3 TB/s of read + write).  bench.py times it beside the replay kernel. */
int cdr_stream_copy_async(void* dst, const void* src, uint64_t bytes, void* stream);

/* Compile-time variant flags of this build (0 = the product build): bit 0 the PAR
 * profiling variant (CDR_PAR_PROF: writes per-wave times into result fields), bit 1 any
 * tuning knob off its default (prefetch depths, wave priority, kernel variants).  bench.py
 * refuses to report a line from a library that is not 0. */
uint32_t cdr_build_flags(void);

#ifdef __cplusplus
}
#endif
#endif /* CDR_CDR_H */
