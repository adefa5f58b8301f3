"""ctypes mirrors of include/cdr/schema.h, include/cdr/cdr.h and include/cdr/synth.h.

The C headers are the source of truth; ``check_layouts()`` compares every mirror's
size with ``cdr_struct_size`` exported by libcdr so a drift fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

u8, u32, i32, u64, i64, f64 = C.c_uint8, C.c_uint32, C.c_int32, C.c_uint64, C.c_int64, C.c_double

# ------------------------------------------------------------------ constants
FIRST_EVENT_ID = 1
EMPTY_EVENT_ID = -23
EMPTY_VERSION = -24

(STATE_CREATED, STATE_RUNNING, STATE_COMPLETED, STATE_ZOMBIE, STATE_VOID) = range(5)
(CLOSE_NONE, CLOSE_COMPLETED, CLOSE_FAILED, CLOSE_CANCELED, CLOSE_TERMINATED,
 CLOSE_CONTINUED_AS_NEW, CLOSE_TIMED_OUT) = range(7)
TIMEOUT_START_TO_CLOSE, TIMEOUT_SCHEDULE_TO_START, TIMEOUT_SCHEDULE_TO_CLOSE, TIMEOUT_HEARTBEAT = range(4)
TTS_START_TO_CLOSE, TTS_SCHEDULE_TO_START, TTS_SCHEDULE_TO_CLOSE, TTS_HEARTBEAT = 1, 2, 4, 8
BUILDER_LOCAL, BUILDER_2DC, BUILDER_NDC = 0, 1, 2

EVENT_TYPES = [
    "WorkflowExecutionStarted", "WorkflowExecutionCompleted", "WorkflowExecutionFailed",
    "WorkflowExecutionTimedOut", "DecisionTaskScheduled", "DecisionTaskStarted",
    "DecisionTaskCompleted", "DecisionTaskTimedOut", "DecisionTaskFailed", "ActivityTaskScheduled",
    "ActivityTaskStarted", "ActivityTaskCompleted", "ActivityTaskFailed", "ActivityTaskTimedOut",
    "ActivityTaskCancelRequested", "RequestCancelActivityTaskFailed", "ActivityTaskCanceled",
    "TimerStarted", "TimerFired", "CancelTimerFailed", "TimerCanceled",
    "WorkflowExecutionCancelRequested", "WorkflowExecutionCanceled",
    "RequestCancelExternalWorkflowExecutionInitiated", "RequestCancelExternalWorkflowExecutionFailed",
    "ExternalWorkflowExecutionCancelRequested", "MarkerRecorded", "WorkflowExecutionSignaled",
    "WorkflowExecutionTerminated", "WorkflowExecutionContinuedAsNew",
    "StartChildWorkflowExecutionInitiated", "StartChildWorkflowExecutionFailed",
    "ChildWorkflowExecutionStarted", "ChildWorkflowExecutionCompleted", "ChildWorkflowExecutionFailed",
    "ChildWorkflowExecutionCanceled", "ChildWorkflowExecutionTimedOut",
    "ChildWorkflowExecutionTerminated", "SignalExternalWorkflowExecutionInitiated",
    "SignalExternalWorkflowExecutionFailed", "ExternalWorkflowExecutionSignaled",
    "UpsertWorkflowSearchAttributes",
]
EV = {name: i for i, name in enumerate(EVENT_TYPES)}
EVF_BATCH_FIRST = 0x1

STATUS = {
    0: "OK", 1: "E_HISTORY_EMPTY", 2: "E_NEWRUN_HISTORY_EMPTY", 3: "E_UNKNOWN_EVENT_TYPE",
    4: "E_INVALID_STATE_TRANSITION", 5: "E_VH_LOWER_VERSION", 6: "E_VH_LOWER_EVENT_ID",
    7: "E_DECISION_NOT_FOUND", 8: "E_ACTIVITY_NOT_FOUND", 9: "E_ACTIVITY_ID_NOT_FOUND",
    10: "E_MISSING_ACTIVITY_INFO", 11: "E_DOMAIN_NOT_FOUND", 12: "E_REBUILD_NEXT_EVENT_ID",
    13: "E_BAD_INPUT", 14: "E_REFRESH_EVENT_NOT_FOUND", 15: "E_REFRESH_BACKOFF_INITIATOR",
    16: "E_REFRESH_CAPACITY", 17: "E_VH_NO_LCA", 18: "E_VH_LCA_NOT_CONTAINED", 19: "E_VH_FIRST_ITEM_MISMATCH",
    20: "E_NDC_RETRY_TASK", 21: "E_NDC_BRANCH_CHANGED", 22: "E_NDC_SAME_VERSION", 23: "E_REBUILD_VH_MISMATCH",
    24: "E_VHS_CAPACITY", 25: "E_VH_EMPTY", 32: "P_ACTIVITY_STARTED_NIL", 33: "P_CHILD_STARTED_NIL",
    34: "P_VH_ITEM_INVALID", 35: "P_UNKNOWN_CLUSTER", 64: "NOT_APPLIED", 65: "NOT_RUN",
}
OK = 0
E_HISTORY_EMPTY = 1
RF_IN_NEWRUN, RF_IS_NEWRUN, RF_NEWRUN_APPLIED = 1, 2, 4

SF_HAS_PARENT_DOMAIN, SF_PARENT_DOMAIN_MISSING, SF_HAS_PARENT_EXEC = 0x1, 0x2, 0x4
SF_HAS_PARENT_INITIATED, SF_HAS_RETRY, SF_HAS_MEMO, SF_HAS_SEARCH_ATTR = 0x8, 0x10, 0x20, 0x40
SF_HAS_RESET_POINTS, SF_CRON_INITIATOR = 0x80, 0x100
SF_HAS_INITIATOR, SF_RETRY_INITIATOR, SF_DECIDER_INITIATOR = 0x200, 0x400, 0x800
REFRESH_ADVANCED_VISIBILITY, REFRESH_SNAPSHOT_PASSIVE = 0x1, 0x2
AF_HAS_RETRY = 0x1
XF_DOMAIN_MISSING, XF_CHILD_ONLY = 0x1, 0x2
RP_HAS_CHECKSUM, RP_HAS_RUN_ID, RP_HAS_FIRST_DC_ID, RP_HAS_CREATED = 0x1, 0x2, 0x4, 0x8
RP_HAS_EXPIRING, RP_HAS_RESETTABLE, RP_RESETTABLE = 0x10, 0x20, 0x40
XI_CANCEL_REQUESTED, XI_HAS_RETRY, XI_HAS_EXPIRATION, XI_HAS_BRANCH = 0x1, 0x2, 0x4, 0x8
XI_HAS_MEMO, XI_HAS_SEARCH_ATTR, XI_HAS_RESET_POINTS, XI_STARTED, XI_VH_BRANCH = 0x10, 0x20, 0x40, 0x80, 0x100
AI_CANCEL_REQUESTED, AI_HAS_RETRY, AI_STARTED_TIME_SET = 0x1, 0x2, 0x4
MAX_CLUSTERS = 8
SLICE_WIDTH = 64


def _S(name, fields):
    return type(name, (C.Structure,), {"_fields_": fields})


# ------------------------------------------------------------------ input
CdrKV = _S("cdr_kv", [("key", u32), ("value", u32)])
CdrResetPoint = _S("cdr_reset_point", [
    ("binary_checksum", u32), ("run_id", u32), ("first_decision_completed_id", i64),
    ("created_time_nano", i64), ("expiring_time_nano", i64), ("flags", u32), ("_pad", u32)])
AttrStarted = _S("cdr_attr_wf_started", [
    ("workflow_type", u32), ("task_list", u32), ("cron_schedule", u32), ("flags", u32),
    ("parent_domain_id", u32), ("parent_workflow_id", u32), ("parent_run_id", u32), ("continued_run_id", u32),
    ("parent_initiated_id", i64), ("expiration_ts", i64),
    ("exec_timeout_s", i32), ("task_timeout_s", i32), ("attempt", i32), ("first_decision_backoff_s", i32),
    ("backoff_coefficient", f64),
    ("retry_initial_s", i32), ("retry_max_interval_s", i32), ("retry_max_attempts", i32),
    ("retry_expiration_s", i32), ("nonretriable", u32), ("memo", u32),
    ("search_attr_off", u32), ("search_attr_len", u32), ("reset_points_off", u32), ("reset_points_len", u32)])
AttrDTSched = _S("cdr_attr_dt_scheduled", [("attempt", i64), ("start_to_close_s", i32), ("task_list", u32)])
AttrDT = _S("cdr_attr_dt", [("scheduled_event_id", i64), ("started_event_id", i64), ("request_id", u32),
                            ("binary_checksum", u32), ("timeout_type", i32), ("_pad", i32)])
AttrATSched = _S("cdr_attr_at_scheduled", [
    ("activity_id", u32), ("task_list", u32), ("s2s_s", i32), ("s2c_s", i32), ("stc_s", i32), ("hb_s", i32),
    ("flags", u32), ("nonretriable", u32), ("retry_initial_s", i32), ("retry_max_interval_s", i32),
    ("retry_max_attempts", i32), ("retry_expiration_s", i32), ("backoff_coefficient", f64),
    ("domain", u32), ("target_domain_id", u32)])
AF_HAS_RETRY, AF_DOMAIN_MISSING = 0x1, 0x2
AttrAT = _S("cdr_attr_at", [("scheduled_event_id", i64), ("started_event_id", i64), ("request_id", u32),
                            ("activity_id", u32), ("timeout_type", i32), ("attempt", i32)])
AttrTimer = _S("cdr_attr_timer", [("timer_id", u32), ("_pad", u32), ("start_to_fire_s", i64),
                                  ("started_event_id", i64)])
AttrExternal = _S("cdr_attr_external", [
    ("domain", u32), ("workflow_id", u32), ("run_id", u32), ("workflow_type", u32), ("signal_name", u32),
    ("input", u32), ("control", u32), ("flags", u32), ("parent_close_policy", i32),
    ("target_domain_id", u32)])
AttrRef = _S("cdr_attr_initiated_ref", [("initiated_event_id", i64), ("run_id", u32), ("_pad", u32)])
AttrCAN = _S("cdr_attr_can", [("new_execution_run_id", u32), ("_pad", u32)])
AttrUpsert = _S("cdr_attr_upsert", [("search_attr_off", u32), ("search_attr_len", u32)])


class AttrUnion(C.Union):
    _fields_ = [("started", AttrStarted), ("dt_sched", AttrDTSched), ("dt", AttrDT), ("at_sched", AttrATSched),
                ("at", AttrAT), ("timer", AttrTimer), ("ext", AttrExternal), ("ref", AttrRef), ("can", AttrCAN),
                ("upsert", AttrUpsert), ("raw", u8 * 112)]


CdrEvent = _S("cdr_event", [("event_id", i64), ("version", i64), ("timestamp", i64), ("task_id", i64),
                            ("type", u32), ("flags", u32), ("a", AttrUnion)])
CdrWfDesc = _S("cdr_wf_desc", [
    ("wf_key", u64), ("ev_off", u64), ("ev_len", u64), ("domain_id", u32), ("workflow_id", u32), ("run_id", u32),
    ("request_id", u32), ("builder", u32), ("retention_days", i32), ("failover_version", i64),
    ("expected_next_event_id", i64), ("parent", i32), ("newrun", i32), ("newrun_call", u32), ("newrun_ndc", u32)])
CdrClusterMeta = _S("cdr_cluster_meta", [("failover_version_increment", i64), ("current_cluster", i32),
                                         ("n_clusters", i32), ("initial_version", i64 * MAX_CLUSTERS)])
CdrBatch = _S("cdr_batch", [
    ("events", C.POINTER(CdrEvent)), ("n_events", u64), ("wfs", C.POINTER(CdrWfDesc)), ("n_wfs", u32),
    ("empty_uuid", u32), ("kvs", C.POINTER(CdrKV)), ("n_kvs", u64), ("rps", C.POINTER(CdrResetPoint)),
    ("n_rps", u64), ("cluster", CdrClusterMeta), ("now_ns", i64), ("uuid_seed", u64), ("carry", C.c_void_p)])

# ------------------------------------------------------------------ output
CdrExecInfo = _S("cdr_exec_info", [
    # first 128 B: set by WorkflowExecutionStarted
    ("domain_id", u32), ("workflow_id", u32), ("run_id", u32), ("create_request_id", u32),
    ("parent_domain_id", u32), ("parent_workflow_id", u32), ("parent_run_id", u32), ("task_list", u32),
    ("workflow_type", u32), ("cron_schedule", u32), ("memo", u32), ("nonretriable", u32),
    ("branch_tree_id", u32), ("workflow_timeout", i32), ("decision_timeout_value", i32), ("attempt", i32),
    ("initiated_id", i64), ("initial_interval", i32), ("maximum_interval", i32), ("backoff_coefficient", f64),
    ("maximum_attempts", i32), ("expiration_seconds", i32), ("expiration_time", i64), ("branch_id_lo", u64),
    ("branch_id_hi", u64), ("_pad0", u32), ("_pad1", u32),
    # second 128 B: updated by the replay
    ("decision_request_id", u32), ("flags", u32), ("completion_event_batch_id", i64), ("state", i32),
    ("close_status", i32), ("last_first_event_id", i64), ("last_event_task_id", i64), ("next_event_id", i64),
    ("last_processed_event", i64), ("signal_count", i32), ("decision_timeout", i32), ("decision_version", i64),
    ("decision_schedule_id", i64), ("decision_started_id", i64), ("decision_attempt", i64),
    ("decision_started_ts", i64), ("decision_scheduled_ts", i64), ("decision_original_scheduled_ts", i64),
    ("reset_points_len", u32), ("search_attr_len", u32)])
CdrReplState = _S("cdr_repl_state", [
    ("current_version", i64), ("start_version", i64), ("last_write_version", i64), ("last_write_event_id", i64),
    ("lri_version", i64 * MAX_CLUSTERS), ("lri_last_event_id", i64 * MAX_CLUSTERS), ("lri_mask", u32),
    ("present", u32)])
CdrVHItem = _S("cdr_vh_item", [("event_id", i64), ("version", i64)])
CdrActivityInfo = _S("cdr_activity_info", [
    ("version", i64), ("schedule_id", i64), ("scheduled_event_batch_id", i64), ("scheduled_time", i64),
    ("started_id", i64), ("started_time", i64), ("last_heartbeat_time", i64), ("expiration_time", i64),
    ("cancel_request_id", i64), ("activity_id", u32), ("request_id", u32), ("task_list", u32), ("nonretriable", u32),
    ("s2s", i32), ("s2c", i32), ("stc", i32), ("hb", i32), ("timer_task_status", i32), ("attempt", i32),
    ("initial_interval", i32), ("maximum_interval", i32), ("maximum_attempts", i32), ("flags", u32),
    ("backoff_coefficient", f64)])
CdrTimerInfo = _S("cdr_timer_info", [("version", i64), ("started_id", i64), ("expiry_time", i64), ("task_id", i64),
                                     ("timer_id", u32), ("_pad", u32)])
CdrChildInfo = _S("cdr_child_info", [
    ("version", i64), ("initiated_id", i64), ("initiated_event_batch_id", i64), ("started_id", i64),
    ("create_request_lo", u64), ("create_request_hi", u64), ("started_workflow_id", u32), ("started_run_id", u32),
    ("domain_name", u32), ("workflow_type", u32), ("parent_close_policy", i32), ("_pad", i32)])
CdrCancelInfo = _S("cdr_cancel_info", [("version", i64), ("initiated_event_batch_id", i64), ("initiated_id", i64),
                                       ("cancel_request_lo", u64), ("cancel_request_hi", u64)])
CdrSignalInfo = _S("cdr_signal_info", [
    ("version", i64), ("initiated_event_batch_id", i64), ("initiated_id", i64), ("signal_request_lo", u64),
    ("signal_request_hi", u64), ("signal_name", u32), ("input", u32), ("control", u32), ("_pad", u32)])
CdrWfResult = _S("cdr_wf_result", [
    ("code", i32), ("flags", u32), ("fail_event_id", i64), ("fail_index", i64), ("n_activity", u32),
    ("n_timer", u32), ("n_child", u32), ("n_cancel", u32), ("n_signal", u32), ("n_vh", u32),
    ("n_reset_points", u32), ("n_search_attr", u32)])
CdrWfCaps = _S("cdr_wf_caps", [
    ("act_off", u64), ("timer_off", u64), ("child_off", u64), ("cancel_off", u64), ("signal_off", u64),
    ("vh_off", u64), ("rp_off", u64), ("sa_off", u64), ("act_cap", u32), ("timer_cap", u32), ("child_cap", u32),
    ("cancel_cap", u32), ("signal_cap", u32), ("vh_cap", u32), ("rp_cap", u32), ("sa_cap", u32),
    ("act_live", u32), ("timer_live", u32), ("flags", u32), ("order_key", u32), ("xfer_off", u64), ("ttask_off", u64),
    ("xfer_cap", u32), ("ttask_cap", u32)])
CdrTotals = _S("cdr_totals", [(n, u64) for n in ("act", "timer", "child", "cancel", "signal", "vh", "rp", "sa",
                                                 "xfer", "ttask")])
CdrOut = _S("cdr_out", [(n, C.c_void_p) for n in (
    "result", "exec", "repl", "vh", "act", "timer", "child", "cancel", "signal", "rp", "sa", "transfer",
    "timer_tasks", "n_tasks", "last_decision")])
CdrLastDecision = _S("cdr_last_decision", [
    ("source", u32), ("request_id", u32), ("event_index", i64), ("version", i64), ("schedule_id", i64),
    ("started_id", i64), ("attempt", i64), ("scheduled_ts", i64), ("started_ts", i64),
    ("original_scheduled_ts", i64), ("decision_timeout", i32), ("_pad", i32)])
LD_NONE, LD_SCHEDULED, LD_STARTED, LD_TRANSIENT = range(4)
CdrIngestIn = _S("cdr_ingest_in", [(n, C.c_void_p) for n in (
    "blob_bytes", "blob_off", "entry_blob0", "seed_bytes", "seed_off", "domain_map")] + [
    ("n_blobs", u32), ("n_entries", u32), ("n_seeds", u32), ("n_domains", u32)])
CdrIngestOut = _S("cdr_ingest_out", [(n, C.c_void_p) for n in (
    "events", "kvs", "rps", "ev_off", "blob_status", "entry_status", "str_ref", "str_len")] + [
    ("n_events", u64), ("n_kvs", u64), ("n_rps", u64), ("n_strings", u32), ("n_bad_blobs", u32)])
DEC_STATUS = {0: "OK", 1: "MISSING_VERSION", 2: "INVALID_VERSION", 3: "TRUNCATED", 4: "DEPTH", 5: "NO_EVENTS",
              6: "BAD_SIZE", 7: "BAD_TYPE"}
CdrOpts = _S("cdr_opts", [("plan_mode", u32), ("fast_path", i32), ("reg_path", i32), ("concurrent", i32),
                          ("workspace_bytes", u64)])
CdrVHToken = _S("cdr_vh_token", [("tree", u32), ("_pad", u32), ("branch_lo", u64), ("branch_hi", u64)])
CdrVHBranch = _S("cdr_vh_branch", [("token", CdrVHToken), ("n_items", u32), ("_pad", u32)])
VHS_MAX_BRANCHES = 8
CdrVHS = _S("cdr_vhs", [("current", u32), ("n_branches", u32), ("items_cap", u32), ("_pad", u32),
                        ("items_off", u64), ("branch", CdrVHBranch * VHS_MAX_BRANCHES)])
CdrNdcTask = _S("cdr_ndc_task", [("items_off", u64), ("n_items", u32), ("_pad", u32), ("first_event_id", i64),
                                 ("last_event_id", i64), ("last_version", i64), ("version", i64),
                                 ("new_token", CdrVHToken)])
CdrNdcDecision = _S("cdr_ndc_decision", [("code", i32), ("action", i32), ("branch_index", u32), ("created", u32),
                                         ("rebuild_next_event_id", i64), ("lca", CdrVHItem),
                                         ("rebuild_token", CdrVHToken)])
NDC_SKIP, NDC_APPLY_CURRENT, NDC_REBUILD, NDC_BACKFILL = range(4)
NDC_ACTIONS = {0: "SKIP", 1: "APPLY_CURRENT", 2: "REBUILD", 3: "BACKFILL"}
CdrTask = _S("cdr_task", [("type", u32), ("timeout_type", i32), ("event_id", i64), ("visibility_ts", i64),
                          ("attempt", i64), ("domain_id", u32), ("task_list", u32), ("target_workflow_id", u32),
                          ("target_run_id", u32), ("flags", u32), ("_pad", u32),
                          ("version", i64)])
TASK_TYPES = {0: "DecisionTask", 1: "ActivityTask", 2: "CloseExecution", 3: "CancelExecution",
              4: "StartChildExecution", 5: "SignalExecution", 6: "RecordWorkflowStarted",
              8: "UpsertWorkflowSearchAttributes", 16: "DecisionTimeout", 17: "ActivityTimeout", 18: "UserTimer",
              19: "WorkflowTimeout", 20: "DeleteHistoryEvent", 22: "WorkflowBackoffTimer"}
CdrCarry = _S("cdr_carry", [("src", C.c_void_p), ("caps", C.c_void_p), ("n_src", u32), ("_pad", u32),
                            ("totals", CdrTotals), ("state", CdrOut), ("in_memory", C.c_void_p)])
CdrSlices = _S("cdr_slices", [
    ("n_slices", u32), ("_pad", u32), ("n_rows", u64), ("arena_words", u64)] + [(n, C.c_void_p) for n in (
        "slice_row0", "slice_len", "lane_wf", "slab", "arena", "slice_scratch_off", "slice_act_slots",
        "slice_tim_slots", "slice_flags")])
SLICE_FAST = 0x1
SLICE_WAVE = 0x2
SLICE_REG = 0x4
SLICE_REG2 = 0x8
SLICE_PAR = 0x20
SLICE_REG0 = 0x10
CAP_FAST = 0x1
CAP_WAVE = 0x2
PLAN_WAVE = 0x1
PLAN_WAVE_ALL = 0x2  # with PLAN_WAVE: lane-friendly (CAP_LANE) entries on the wave kernel too
PLAN_PAR = 0x8  # with PLAN_WAVE: long register-table histories to CDR_SLICE_PAR lane slices (CDR_PLAN_PAR)
PLAN_PAR_SOLO = 0x10  # with PLAN_PAR: every PAR history alone in its slice, the 512 longest at most (task batches)
PLAN_NO_LONG = 0x4  # with PLAN_WAVE: keep long lane-capable histories in lane slices (CDR_PLAN_NO_LONG)
CAP_LANE = 0x4
CAP_REG = 0x8
CAP_REG2 = 0x10
CAP_REG0 = 0x20
CAP_LOADED = 0x40

# variable-size row blobs (cdr.h cdr_encode_blobs_async)
CdrStrtab = _S("cdr_strtab", [("bytes", C.c_void_p), ("off", C.c_void_p), ("n", u32), ("_pad", u32)])
CdrExecPersist = _S("cdr_exec_persist", [
    ("start_version", i64), ("current_version", i64), ("start_time", i64), ("last_updated_time", i64),
    ("history_size", i64), ("sticky_s2s_timeout", i64), ("execution_context", u32), ("sticky_task_list", u32),
    ("client_library_version", u32), ("client_feature_version", u32), ("client_impl", u32), ("_pad", u32)])
ZERO_TIME_NANOS = -6795364578871345152
BLOB_STATUS = {0: "OK", 1: "E_UUID", 2: "E_HANDLE", 3: "E_MEMO"}

# slice-major slab of event columns (cdr.h enum cdr_col): name, dtype, in order
SLAB_COLS = (("event_id", np.int64), ("version", np.int64), ("timestamp", np.int64), ("task_id", np.int64),
             ("key", np.int64), ("aux", np.int64), ("type_flags", np.uint32), ("h", np.uint32), ("n", np.int32))
EL_BYTES = sum(np.dtype(t).itemsize for _, t in SLAB_COLS)  # CDR_EL_BYTES
SEF_BATCH_FIRST, SEF_DOMAIN_MISSING = 1 << 8, 1 << 9
SEF_ID_NEXT, SEF_VER_SAME = 1 << 21, 1 << 22  # delta bits (cdr.h)


ROW_BYTES = EL_BYTES * SLICE_WIDTH  # CDR_ROW_BYTES


def slab_columns(slab, row0=None, slen=None, cols=None):
    """Columns of a slab (uint8 array of rows, cdr.h) in global element order: element
    row * 64 + lane of the result is the event in that slab row for that lane."""
    rows = np.asarray(slab).view(np.uint8).reshape(-1, ROW_BYTES)
    out, off = {}, 0
    for name, dt in SLAB_COLS:
        size = np.dtype(dt).itemsize
        if cols is None or name in cols:
            out[name] = np.ascontiguousarray(rows[:, off * SLICE_WIDTH:(off + size) * SLICE_WIDTH]).view(dt).reshape(-1)
        off += size
    return out
CdrDevBatch = _S("cdr_dev_batch", [
    ("ev", CdrSlices), ("scratch", C.c_void_p), ("wfs", C.c_void_p), ("caps", C.c_void_p), ("kvs", C.c_void_p), ("rps", C.c_void_p),
    ("n_wfs", u32), ("empty_uuid", u32), ("max_act_slots", u32), ("max_tim_slots", u32),
    ("n_fast_slices", u32), ("n_wave_slices", u32), ("n_reg_slices", u32), ("n_reg2_slices", u32),
    ("n_reg0_slices", u32), ("n_par_slices", u32), ("class_lo", u32 * 6), ("class_hi", u32 * 6),
    ("cluster", CdrClusterMeta), ("now_ns", i64), ("uuid_seed", u64), ("carry", C.c_void_p),
    ("cls_slab", C.c_void_p), ("cls_row0", C.c_void_p), ("cls_rows", C.c_void_p), ("skip", C.c_void_p),
    ("task_rows", u64)])
CdrNdcRound = _S("cdr_ndc_round", [("tasks", C.c_void_p), ("task_items", C.c_void_p), ("rebuild", CdrDevBatch),
                                   ("rebuild_out", CdrOut), ("apply", CdrDevBatch), ("apply_out", CdrOut),
                                   ("dec", C.c_void_p), ("refresh_now", i64), ("refresh_flags", u32), ("_pad", u32)])

# ------------------------------------------------------------------ synth
CdrSynthParams = _S("cdr_synth_params", [
    ("config", i32), ("n_wfs", u32), ("seed", u64), ("target_len", u32), ("max_len", u32), ("error_rate", f64),
    ("builder", i32), ("rebuild", i32), ("fault_kinds", u32), ("plan_mode", u32), ("index_map", C.c_void_p),
    ("ndc_part", u32), ("long_stride", u32)])
SYNTH_PART_BASE, SYNTH_PART_REBUILD, SYNTH_PART_FORK_A, SYNTH_PART_FORK_B = range(4)
# synth fault kinds that keep a sequential-activity history on the fast path (synth.cpp inject_fault)
FAULTS_FAST = (1 << 1) | (1 << 2) | (1 << 3) | (1 << 5) | (1 << 6)
CdrSynthSizes = _S("cdr_synth_sizes", [("n_events", u64), ("n_entries", u32), ("_pad", u32), ("n_kvs", u64),
                                       ("n_rps", u64), ("arena_words", u64)])
CdrSynthPlanInfo = _S("cdr_synth_plan_info", [
    ("n_events", u64), ("n_entries", u32), ("n_slices", u32), ("n_rows", u64), ("arena_words", u64),
    ("n_kvs", u64), ("n_rps", u64), ("totals", CdrTotals)])

CLS_RETRY = 0x7FFF  # k_replay_cls's hand-on code (cdr_set_cls_path CLS_ALONE only)
CLS_OFF, CLS_ON, CLS_ALONE, CLS_BUILD = range(4)  # cdr_set_cls_path modes (cdr.h CDR_CLS_*)
CLS_SLICES = 0x4 | 0x8 | 0x10 | 0x20  # CDR_CLS_SLICES: slices that carry a class-sorted block

MIRRORS = {
    "cdr_event": CdrEvent, "cdr_wf_desc": CdrWfDesc, "cdr_cluster_meta": CdrClusterMeta, "cdr_batch": CdrBatch,
    "cdr_kv": CdrKV, "cdr_reset_point": CdrResetPoint, "cdr_attr_wf_started": AttrStarted,
    "cdr_attr_at_scheduled": AttrATSched, "cdr_exec_info": CdrExecInfo, "cdr_repl_state": CdrReplState,
    "cdr_vh_item": CdrVHItem, "cdr_activity_info": CdrActivityInfo, "cdr_timer_info": CdrTimerInfo,
    "cdr_child_info": CdrChildInfo, "cdr_cancel_info": CdrCancelInfo, "cdr_signal_info": CdrSignalInfo,
    "cdr_wf_result": CdrWfResult, "cdr_wf_caps": CdrWfCaps, "cdr_totals": CdrTotals, "cdr_out": CdrOut,
    "cdr_slices": CdrSlices, "cdr_dev_batch": CdrDevBatch, "cdr_carry": CdrCarry,
    "cdr_task": CdrTask, "cdr_vh_token": CdrVHToken, "cdr_vh_branch": CdrVHBranch, "cdr_vhs": CdrVHS,
    "cdr_ndc_task": CdrNdcTask, "cdr_ndc_decision": CdrNdcDecision, "cdr_ndc_round": CdrNdcRound, "cdr_last_decision": CdrLastDecision,
    "cdr_opts": CdrOpts, "cdr_ingest_in": CdrIngestIn, "cdr_ingest_out": CdrIngestOut,
}

# C ABI entry points declared in include/cdr/cdr.h and include/cdr/synth.h
EXPORTS = {
    "cdr_plan_caps": (i32, [C.POINTER(CdrBatch), C.POINTER(CdrWfCaps), C.POINTER(CdrTotals)]),
    "cdr_plan_slices": (i32, [C.POINTER(CdrWfDesc), u32, C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(u32),
                              C.POINTER(u64)]),
    "cdr_plan_slices_ex": (i32, [C.POINTER(CdrWfDesc), C.c_void_p, u32, u32, C.c_void_p, C.c_void_p, C.c_void_p,
                                 C.c_void_p, C.POINTER(u32), C.POINTER(u64), C.POINTER(u32)]),
    "cdr_plan_arena_words": (u64, [C.POINTER(CdrBatch)]),
    "cdr_plan_scratch": (i32, [C.c_void_p, C.c_void_p, u32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                               C.POINTER(u64), C.c_void_p]),
    "cdr_set_fast_path": (i32, [C.c_void_p, i32]),
    "cdr_set_reg_path": (i32, [C.c_void_p, i32]),
    "cdr_set_cls_path": (i32, [C.c_void_p, i32]),
    "cdr_cls_plan_async": (i32, [C.c_void_p, C.POINTER(CdrDevBatch), C.c_void_p, C.c_void_p, C.c_void_p]),
    "cdr_cls_pack_async": (i32, [C.c_void_p, C.POINTER(CdrDevBatch), C.c_void_p]),
    "cdr_plan_cls": (i32, [C.POINTER(CdrSlices), C.c_void_p, C.c_void_p, C.c_void_p]),
    "cdr_pack_cls": (i32, [C.POINTER(CdrSlices), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, i32]),
    "cdr_set_plan_mode": (i32, [C.c_void_p, u32]),
    "cdr_pack_slices": (i32, [C.POINTER(CdrBatch), C.POINTER(CdrSlices), i32]),
    "cdr_create": (C.c_void_p, [i32, C.c_void_p]),
    "cdr_opts_default": (None, [C.c_void_p]),
    "cdr_destroy": (None, [C.c_void_p]),
    "cdr_replay_sliced_async": (i32, [C.c_void_p, C.POINTER(CdrDevBatch), C.POINTER(CdrOut), C.c_void_p]),
    "cdr_replay_batch": (i32, [C.c_void_p, C.POINTER(CdrBatch), C.POINTER(CdrWfCaps), C.POINTER(CdrTotals),
                               C.POINTER(CdrOut), C.c_void_p]),
    "cdr_replay_one": (i32, [C.c_void_p, C.POINTER(CdrBatch), C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                             C.c_void_p]),
    "cdr_refresh_tasks_async": (i32, [C.c_void_p, C.POINTER(CdrDevBatch), C.POINTER(CdrOut), i64, u32,
                                      C.c_void_p]),
    "cdr_rebuild_batch": (i32, [C.c_void_p, C.POINTER(CdrBatch), C.POINTER(CdrWfCaps), C.POINTER(CdrTotals),
                                C.POINTER(CdrOut), u32, C.c_void_p]),
    "cdr_encode_rows_async": (i32, [C.c_void_p, i32, C.POINTER(CdrDevBatch), C.POINTER(CdrOut), C.c_void_p,
                                    C.c_void_p]),
    "cdr_encode_blobs_async": (i32, [C.c_void_p, i32, C.POINTER(CdrDevBatch), C.POINTER(CdrOut),
                                     C.POINTER(CdrStrtab), C.c_void_p, C.c_void_p, u64, C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_void_p]),
    "cdr_encode_cql_async": (i32, [C.c_void_p, i32, C.POINTER(CdrDevBatch), C.POINTER(CdrOut),
                                     C.POINTER(CdrStrtab), C.c_void_p, C.c_void_p, u64, C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_void_p]),
    "cdr_plan_class_ranges": (i32, [C.c_void_p, u32, C.c_void_p, C.c_void_p]),
    "cdr_compact_async": (i32, [C.c_void_p, i32, C.POINTER(CdrDevBatch), C.POINTER(CdrOut), C.c_void_p,
                                C.c_void_p, C.c_void_p]),
    "cdr_checksum_async": (i32, [C.c_void_p, C.POINTER(CdrDevBatch), C.POINTER(CdrOut), C.c_void_p, C.c_void_p]),
    "cdr_entry_digests_async": (i32, [C.c_void_p, C.POINTER(CdrDevBatch), C.POINTER(CdrOut), C.c_void_p,
                                      C.c_void_p, C.c_void_p]),
    "cdr_ndc_branch_async": (i32, [C.c_void_p, C.c_void_p, C.c_void_p, u32, C.c_void_p, C.c_void_p, C.c_void_p,
                                   C.c_void_p]),
    "cdr_ndc_rebuild_verify_async": (i32, [C.c_void_p, u32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                           C.POINTER(CdrOut), C.c_void_p]),
    "cdr_vhs_sync_async": (i32, [C.c_void_p, u32, C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(CdrOut),
                                 C.c_void_p]),
    "cdr_ndc_replicate_async": (i32, [C.c_void_p, u32, C.POINTER(CdrNdcRound), C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.POINTER(CdrOut), C.c_void_p]),
    "cdr_plan_ndc_apply": (i32, [C.POINTER(CdrBatch), C.c_void_p, C.c_void_p, C.POINTER(CdrTotals)]),
    "cdr_fingerprint32": (u32, [C.c_char_p, C.c_size_t]),
    "cdr_workflow_id_to_shard": (i32, [C.c_char_p, C.c_size_t, i32]),
    "cdr_last_kernel_ms": (i32, [C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_float)]),
    "cdr_version": (C.c_char_p, []),
    "cdr_build_flags": (u32, []),
    "cdr_timing_begin": (i32, [C.c_void_p, u32]),
    "cdr_timing_read": (i32, [C.c_void_p, C.POINTER(C.c_float), C.POINTER(u32)]),
    "cdr_stream_copy_async": (i32, [C.c_void_p, C.c_void_p, u64, C.c_void_p]),
    "cdr_synth_shards": (i32, [u64, i32, C.c_void_p]),
    "cdr_synth_weights": (i32, [C.POINTER(CdrSynthParams), u64, C.c_void_p]),
    "cdr_synth_ndc_tasks": (i32, [C.POINTER(CdrSynthParams), i32, C.c_void_p, C.c_void_p, u32]),
    "cdr_struct_size": (u64, [C.c_char_p]),
    "cdr_ingest_decode": (i32, [C.c_void_p, C.POINTER(CdrIngestIn), C.POINTER(CdrIngestOut), C.c_void_p]),
    "cdr_ingest_plan": (i32, [C.c_void_p, C.POINTER(CdrIngestOut), C.POINTER(CdrBatch), u32, C.POINTER(CdrDevBatch),
                              C.c_void_p, C.POINTER(CdrTotals), C.c_void_p]),
    "cdr_synth_encode_history": (i32, [C.POINTER(CdrBatch), C.c_void_p, C.c_void_p, u32, C.c_void_p, C.c_void_p,
                                       C.c_void_p, C.POINTER(u64), C.POINTER(u32), i32]),
    "cdr_synth_size": (i32, [C.POINTER(CdrSynthParams), C.POINTER(CdrSynthSizes)]),
    "cdr_synth_fill": (i32, [C.POINTER(CdrSynthParams), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                             C.POINTER(CdrBatch)]),
    "cdr_synth_sliced_plan": (i32, [C.POINTER(CdrSynthParams), C.POINTER(CdrSynthPlanInfo)]),
    "cdr_synth_sliced_fill": (i32, [C.POINTER(CdrSynthParams), C.POINTER(CdrSlices), C.c_void_p, C.c_void_p,
                                    C.c_void_p, C.c_void_p, C.POINTER(CdrBatch), i32]),
}

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CDR_LIB") or os.path.join(PKG_DIR, "libcdr.so")
_lib = None


class NativeLibraryMissing(RuntimeError):
    pass


def load(path: str):
    """Load a libcdr build and declare its C ABI (``lib()`` caches the default one)."""
    if not os.path.exists(path):
        raise NativeLibraryMissing(
            f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    L = C.CDLL(path)
    for name, (res, args) in EXPORTS.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


def lib():
    """Load the in-tree libcdr.so (fails loudly: there is no fallback path)."""
    global _lib
    if _lib is None:
        _lib = load(LIB_PATH)
    return _lib


def check_layouts():
    """Raise if any ctypes mirror disagrees with the C struct size."""
    L = lib()
    bad = []
    for name, ty in MIRRORS.items():
        n = L.cdr_struct_size(name.encode())
        if n != C.sizeof(ty):
            bad.append((name, n, C.sizeof(ty)))
    if bad:
        raise RuntimeError(f"ABI mirror mismatch (name, C, ctypes): {bad}")


def np_view(arr, ty):
    """numpy structured view (no copy) of a ctypes array of `ty`."""
    return np.frombuffer(arr, dtype=np.dtype((np.void, C.sizeof(ty))))
