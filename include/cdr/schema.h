/*
 * cdr/schema.h — data model of the batched workflow-history replay engine.
 *
 * This header restates the reference's persisted-state vocabulary (Uber Cadence,
 * mounted read-only at /root/reference) as plain C types that are shared by the
 * host packer, the HIP kernels and the test oracle.  Every constant cites the
 * reference definition it mirrors.
 *
 *   event types        .gen/go/shared/shared.go:16404-16445   (EventType 0..41)
 *   sentinels          common/constants.go:28-41
 *   states/close stat. common/persistence/dataInterfaces.go:87-105
 *   timer-task status  service/history/timerBuilder.go:36-47
 *   timeout types      .gen/go/shared/shared.go:47934-47937
 *   persisted records  common/persistence/dataInterfaces.go:259-331,610-706
 *
 * Strings and byte blobs never cross into the kernels: the host interns them into
 * u32 handles (0 == "" / nil) and every string-valued field below is a handle.
 * Nondeterministic values of the reference (uuid.New(), timeSource.Now()) are
 * injected: a per-call `now_ns` and a seeded UUID function (cdr_uuid below).
 */
#ifndef CDR_SCHEMA_H
#define CDR_SCHEMA_H

#include <stddef.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define CDR_HD __host__ __device__ __forceinline__
#else
#define CDR_HD static inline
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- constants */

/* common/constants.go:28-41 */
#define CDR_FIRST_EVENT_ID ((int64_t)1)
#define CDR_EMPTY_EVENT_ID ((int64_t)-23)
#define CDR_EMPTY_VERSION ((int64_t)-24)
#define CDR_BUFFERED_EVENT_ID ((int64_t)-123)
#define CDR_TRANSIENT_EVENT_ID ((int64_t)-124)

/* common/persistence/dataInterfaces.go:87-94 */
enum cdr_wf_state {
  CDR_STATE_CREATED = 0,
  CDR_STATE_RUNNING = 1,
  CDR_STATE_COMPLETED = 2,
  CDR_STATE_ZOMBIE = 3,
  CDR_STATE_VOID = 4
};

/* common/persistence/dataInterfaces.go:97-105 */
enum cdr_close_status {
  CDR_CLOSE_NONE = 0,
  CDR_CLOSE_COMPLETED = 1,
  CDR_CLOSE_FAILED = 2,
  CDR_CLOSE_CANCELED = 3,
  CDR_CLOSE_TERMINATED = 4,
  CDR_CLOSE_CONTINUED_AS_NEW = 5,
  CDR_CLOSE_TIMED_OUT = 6
};

/* service/history/timerBuilder.go:36-47 */
#define CDR_TIMER_TASK_STATUS_NONE 0
#define CDR_TIMER_TASK_STATUS_CREATED 1
#define CDR_TTS_START_TO_CLOSE 1
#define CDR_TTS_SCHEDULE_TO_START 2
#define CDR_TTS_SCHEDULE_TO_CLOSE 4
#define CDR_TTS_HEARTBEAT 8

/* .gen/go/shared/shared.go:47934-47937 */
enum cdr_timeout_type {
  CDR_TIMEOUT_START_TO_CLOSE = 0,
  CDR_TIMEOUT_SCHEDULE_TO_START = 1,
  CDR_TIMEOUT_SCHEDULE_TO_CLOSE = 2,
  CDR_TIMEOUT_HEARTBEAT = 3
};

/* .gen/go/shared/shared.go:16404-16445 */
enum cdr_event_type {
  CDR_EV_WF_STARTED = 0,
  CDR_EV_WF_COMPLETED = 1,
  CDR_EV_WF_FAILED = 2,
  CDR_EV_WF_TIMED_OUT = 3,
  CDR_EV_DT_SCHEDULED = 4,
  CDR_EV_DT_STARTED = 5,
  CDR_EV_DT_COMPLETED = 6,
  CDR_EV_DT_TIMED_OUT = 7,
  CDR_EV_DT_FAILED = 8,
  CDR_EV_AT_SCHEDULED = 9,
  CDR_EV_AT_STARTED = 10,
  CDR_EV_AT_COMPLETED = 11,
  CDR_EV_AT_FAILED = 12,
  CDR_EV_AT_TIMED_OUT = 13,
  CDR_EV_AT_CANCEL_REQUESTED = 14,
  CDR_EV_AT_REQ_CANCEL_FAILED = 15,
  CDR_EV_AT_CANCELED = 16,
  CDR_EV_TIMER_STARTED = 17,
  CDR_EV_TIMER_FIRED = 18,
  CDR_EV_CANCEL_TIMER_FAILED = 19,
  CDR_EV_TIMER_CANCELED = 20,
  CDR_EV_WF_CANCEL_REQUESTED = 21,
  CDR_EV_WF_CANCELED = 22,
  CDR_EV_RCE_INITIATED = 23, /* RequestCancelExternalWorkflowExecutionInitiated */
  CDR_EV_RCE_FAILED = 24,    /* RequestCancelExternalWorkflowExecutionFailed */
  CDR_EV_EXT_CANCEL_REQUESTED = 25,
  CDR_EV_MARKER_RECORDED = 26,
  CDR_EV_WF_SIGNALED = 27,
  CDR_EV_WF_TERMINATED = 28,
  CDR_EV_WF_CONTINUED_AS_NEW = 29,
  CDR_EV_CHILD_INITIATED = 30, /* StartChildWorkflowExecutionInitiated */
  CDR_EV_CHILD_START_FAILED = 31,
  CDR_EV_CHILD_STARTED = 32,
  CDR_EV_CHILD_COMPLETED = 33,
  CDR_EV_CHILD_FAILED = 34,
  CDR_EV_CHILD_CANCELED = 35,
  CDR_EV_CHILD_TIMED_OUT = 36,
  CDR_EV_CHILD_TERMINATED = 37,
  CDR_EV_SE_INITIATED = 38, /* SignalExternalWorkflowExecutionInitiated */
  CDR_EV_SE_FAILED = 39,
  CDR_EV_EXT_SIGNALED = 40,
  CDR_EV_UPSERT_SA = 41,
  CDR_EV_NUM_TYPES = 42,
  CDR_EV_PAD = 0xFF /* padding slot of the sliced layout; never a real event */
};

/* event flags (cdr_event.flags and the high bits of the sliced type column) */
#define CDR_EVF_BATCH_FIRST 0x1u /* first event of an applyEvents call (stateBuilder.go:124) */

/* builder kinds: which replication structure the mutable state carries
 * (mutableStateBuilder.go:137-231) */
enum cdr_builder {
  CDR_BUILDER_LOCAL = 0, /* newMutableStateBuilder */
  CDR_BUILDER_2DC = 1,   /* ...WithReplicationState */
  CDR_BUILDER_NDC = 2    /* ...WithVersionHistories */
};

/* ------------------------------------------------------------- status codes */
/* One code per Go error / panic site on the replay path.  Order of sites inside
 * one event follows stateBuilder.go:132-600 exactly. */
enum cdr_status {
  CDR_OK = 0,
  CDR_E_HISTORY_EMPTY = 1,          /* stateBuilder.go:121-123 */
  CDR_E_NEWRUN_HISTORY_EMPTY = 2,   /* stateBuilder.go:538-540 */
  CDR_E_UNKNOWN_EVENT_TYPE = 3,     /* stateBuilder.go:597-599 BadRequestError */
  CDR_E_INVALID_STATE_TRANSITION = 4, /* workflowExecutionInfo.go:45-147 */
  CDR_E_VH_LOWER_VERSION = 5,       /* versionHistory.go:215-220 */
  CDR_E_VH_LOWER_EVENT_ID = 6,      /* versionHistory.go:222-227 */
  CDR_E_DECISION_NOT_FOUND = 7,     /* mutableStateDecisionTaskManager.go:212-215 */
  CDR_E_ACTIVITY_NOT_FOUND = 8,     /* DeleteActivity mutableStateBuilder.go:1251-1256 */
  CDR_E_ACTIVITY_ID_NOT_FOUND = 9,  /* DeleteActivity mutableStateBuilder.go:1259-1264 */
  CDR_E_MISSING_ACTIVITY_INFO = 10, /* ReplicateActivityTaskCancelRequested :2270-2273 */
  CDR_E_DOMAIN_NOT_FOUND = 11,      /* domain cache lookups stateBuilder.go:162,365,417,448 */
  CDR_E_REBUILD_NEXT_EVENT_ID = 12, /* nDCStateRebuilder.go:139-143 */
  CDR_E_BAD_INPUT = 13,             /* malformed batch (host validation) */
  /* refreshTasks (cdr_refresh_tasks_async; mutableStateTaskRefresher.go:66-160) */
  CDR_E_REFRESH_EVENT_NOT_FOUND = 14, /* GetStartEvent / eventsCache.getEvent miss: the event is not
                                         among the entry's own events (e.g. a carried-in entry) */
  CDR_E_REFRESH_BACKOFF_INITIATOR = 15, /* generateDelayedDecisionTasks InternalServiceError
                                           mutableStateTaskGenerator.go:197-205 */
  CDR_E_REFRESH_CAPACITY = 16,      /* task slice of the entry too small (caller sized it) */
  /* NDC branch management / conflict-resolution rebuild (cdr_ndc_branch_async, ndc.hip) */
  CDR_E_VH_NO_LCA = 17,             /* FindLCAItem "No joint point found" versionHistory.go:285-288 */
  CDR_E_VH_LCA_NOT_CONTAINED = 18,  /* DuplicateUntilLCAItem versionHistory.go:158-186 */
  CDR_E_VH_FIRST_ITEM_MISMATCH = 19, /* AddVersionHistory versionHistory.go:463-465 */
  CDR_E_NDC_RETRY_TASK = 20,        /* verifyEventsOrder gap nDCBranchMgr.go:188-190 */
  CDR_E_NDC_BRANCH_CHANGED = 21,    /* createNewBranch nDCBranchMgr.go:242-246 */
  CDR_E_NDC_SAME_VERSION = 22,      /* prepareMutableState nDCConflictResolver.go:100-105 */
  CDR_E_REBUILD_VH_MISMATCH = 23,   /* rebuilt VH != branch VH nDCConflictResolver.go:154-165 */
  CDR_E_VHS_CAPACITY = 24,          /* branch / item slots exhausted (caller-planned) */
  CDR_E_VH_EMPTY = 25,              /* GetFirstItem / GetLastItem on an empty history :399-420 */
  CDR_P_ACTIVITY_STARTED_NIL = 32,  /* nil deref mutableStateBuilder.go:2089-2091 */
  CDR_P_CHILD_STARTED_NIL = 33,     /* nil deref mutableStateBuilder.go:3319-3320 */
  CDR_P_VH_ITEM_INVALID = 34,       /* NewVersionHistoryItem panic versionHistory.go:36-42 */
  CDR_P_UNKNOWN_CLUSTER = 35,       /* ClusterNameForFailoverVersion panic metadata.go:193-200 */
  CDR_NOT_APPLIED = 64,             /* new-run history never applied (parent stopped first) */
  CDR_NOT_RUN = 65                  /* skipped entry of a masked launch (cdr_dev_batch.skip): the
                                       record was not replayed this time (cdr_ndc_replicate_async) */
};
/* cdr_wf_result.flags */
#define CDR_RF_IN_NEWRUN 0x1u      /* error raised while replaying newRunHistory */
#define CDR_RF_IS_NEWRUN 0x2u      /* this entry is a continue-as-new run */
#define CDR_RF_NEWRUN_APPLIED 0x4u /* parent applied its newRunHistory */

/* --------------------------------------------------------- injected values */
/* Deterministic stand-in for pborman/uuid.New(): 128 bits from (seed, workflow key,
 * call site, event id).  Sites: */
enum cdr_uuid_site {
  CDR_UUID_BRANCH = 1,     /* NewHistoryBranchToken BranchID dataInterfaces.go:2429 */
  CDR_UUID_CHILD_REQ = 2,  /* stateBuilder.go:357 createRequestID */
  CDR_UUID_CANCEL_REQ = 3, /* stateBuilder.go:410 cancelRequestID */
  CDR_UUID_SIGNAL_REQ = 4, /* stateBuilder.go:441 signalRequestID */
  CDR_UUID_NEWRUN_REQ = 5, /* stateBuilder.go:566 requestID of the new run */
  CDR_UUID_NEWRUN_KEY = 6, /* derives the new run's workflow key from its parent's */
  CDR_UUID_FORK = 7        /* ForkHistoryBranch NewBranchToken's BranchID (nDCBranchMgr.go:205-211) */
};

CDR_HD uint64_t cdr_mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
CDR_HD void cdr_uuid(uint64_t seed, uint64_t wf_key, uint32_t site, int64_t event_id,
                     uint64_t* lo, uint64_t* hi) {
  uint64_t a = cdr_mix64(seed ^ cdr_mix64(wf_key));
  uint64_t b = cdr_mix64(a ^ ((uint64_t)site << 56) ^ (uint64_t)event_id);
  *lo = b;
  *hi = cdr_mix64(b ^ 0xD6E8FEB86659FD93ull);
}

/* ============================================================ HOST INPUT ===
 * The decoded history a caller hands over: one record per HistoryEvent, workflows
 * contiguous, events in eventId order, call (batch) boundaries flagged.  Attribute
 * union members mirror the thrift attribute structs (shared.thrift:492-700) and
 * carry only the fields the replay path reads.                                */

/* list element types (auxiliary tables addressed by off/len pairs) */
typedef struct cdr_kv {      /* map<string, binary> entry (SearchAttributes.IndexedFields) */
  uint32_t key, value;
} cdr_kv;

#define CDR_RP_HAS_CHECKSUM 0x01u
#define CDR_RP_HAS_RUN_ID 0x02u
#define CDR_RP_HAS_FIRST_DC_ID 0x04u
#define CDR_RP_HAS_CREATED 0x08u
#define CDR_RP_HAS_EXPIRING 0x10u
#define CDR_RP_HAS_RESETTABLE 0x20u
#define CDR_RP_RESETTABLE 0x40u
typedef struct cdr_reset_point { /* shared.ResetPointInfo */
  uint32_t binary_checksum, run_id;
  int64_t first_decision_completed_id;
  int64_t created_time_nano;
  int64_t expiring_time_nano;
  uint32_t flags, _pad;
} cdr_reset_point;

/* WorkflowExecutionStartedEventAttributes */
#define CDR_SF_HAS_PARENT_DOMAIN 0x001u    /* ParentWorkflowDomain != nil */
#define CDR_SF_PARENT_DOMAIN_MISSING 0x002u /* domain-cache lookup failed (host-resolved) */
#define CDR_SF_HAS_PARENT_EXEC 0x004u      /* ParentWorkflowExecution != nil */
#define CDR_SF_HAS_PARENT_INITIATED 0x008u /* ParentInitiatedEventId != nil */
#define CDR_SF_HAS_RETRY 0x010u            /* RetryPolicy != nil */
#define CDR_SF_HAS_MEMO 0x020u             /* Memo != nil */
#define CDR_SF_HAS_SEARCH_ATTR 0x040u      /* SearchAttributes != nil */
#define CDR_SF_HAS_RESET_POINTS 0x080u     /* PrevAutoResetPoints != nil && Points != nil */
#define CDR_SF_CRON_INITIATOR 0x100u       /* Initiator == CronSchedule (tasks only) */
#define CDR_SF_HAS_INITIATOR 0x200u        /* Initiator != nil (refreshTasks only) */
#define CDR_SF_RETRY_INITIATOR 0x400u      /* Initiator == RetryPolicy (refreshTasks only) */
#define CDR_SF_DECIDER_INITIATOR 0x800u    /* Initiator == Decider (refreshTasks only) */
typedef struct cdr_attr_wf_started {
  uint32_t workflow_type, task_list, cron_schedule, flags;
  uint32_t parent_domain_id, parent_workflow_id, parent_run_id, continued_run_id;
  int64_t parent_initiated_id;
  int64_t expiration_ts; /* ExpirationTimestamp, 0 = unset */
  int32_t exec_timeout_s, task_timeout_s, attempt, first_decision_backoff_s;
  double backoff_coefficient;
  int32_t retry_initial_s, retry_max_interval_s, retry_max_attempts, retry_expiration_s;
  uint32_t nonretriable, memo;
  uint32_t search_attr_off, search_attr_len;   /* -> cdr_kv table */
  uint32_t reset_points_off, reset_points_len; /* -> cdr_reset_point table */
} cdr_attr_wf_started;

typedef struct cdr_attr_dt_scheduled { /* DecisionTaskScheduledEventAttributes */
  int64_t attempt;
  int32_t start_to_close_s;
  uint32_t task_list;
} cdr_attr_dt_scheduled;

typedef struct cdr_attr_dt { /* DecisionTask{Started,Completed,TimedOut,Failed} */
  int64_t scheduled_event_id;
  int64_t started_event_id;
  uint32_t request_id;      /* Started */
  uint32_t binary_checksum; /* Completed */
  int32_t timeout_type;     /* TimedOut */
  int32_t _pad;
} cdr_attr_dt;

#define CDR_AF_HAS_RETRY 0x1u
#define CDR_AF_DOMAIN_MISSING 0x2u /* the domain cache has no entry for `domain` */
typedef struct cdr_attr_at_scheduled { /* ActivityTaskScheduledEventAttributes */
  uint32_t activity_id, task_list;
  int32_t s2s_s, s2c_s, stc_s, hb_s;
  uint32_t flags, nonretriable;
  int32_t retry_initial_s, retry_max_interval_s, retry_max_attempts, retry_expiration_s;
  double backoff_coefficient;
  /* the activity's target domain (attributes.Domain, 0 = ""), and the domain cache's ID
   * for it, resolved by the caller: read only by refreshTasks' ActivityTask
   * (getTargetDomainID, mutableStateTaskGenerator.go:309-326,531-545) */
  uint32_t domain, target_domain_id;
} cdr_attr_at_scheduled;

typedef struct cdr_attr_at { /* ActivityTask{Started,Completed,Failed,TimedOut,Canceled,CancelRequested} */
  int64_t scheduled_event_id;
  int64_t started_event_id;
  uint32_t request_id;  /* Started */
  uint32_t activity_id; /* CancelRequested / RequestCancelActivityTaskFailed */
  int32_t timeout_type; /* TimedOut */
  int32_t attempt;      /* Started (not read by replay) */
} cdr_attr_at;

typedef struct cdr_attr_timer { /* Timer{Started,Fired,Canceled}, CancelTimerFailed */
  uint32_t timer_id, _pad;
  int64_t start_to_fire_s; /* Started */
  int64_t started_event_id;
} cdr_attr_timer;

#define CDR_XF_DOMAIN_MISSING 0x1u /* target/child domain-cache lookup failed */
#define CDR_XF_CHILD_ONLY 0x2u
typedef struct cdr_attr_external { /* StartChild/SignalExternal/RequestCancelExternal ...Initiated */
  uint32_t domain, workflow_id, run_id, workflow_type;
  uint32_t signal_name, input, control, flags;
  int32_t parent_close_policy;
  uint32_t target_domain_id; /* the domain cache's ID for `domain` (transfer tasks only) */
} cdr_attr_external;

typedef struct cdr_attr_initiated_ref { /* every event that closes an external/child entity */
  int64_t initiated_event_id;
  uint32_t run_id; /* ChildWorkflowExecutionStarted.WorkflowExecution.RunId */
  uint32_t _pad;
} cdr_attr_initiated_ref;

typedef struct cdr_attr_can { /* WorkflowExecutionContinuedAsNewEventAttributes */
  uint32_t new_execution_run_id, _pad;
} cdr_attr_can;

typedef struct cdr_attr_upsert { /* UpsertWorkflowSearchAttributesEventAttributes */
  uint32_t search_attr_off, search_attr_len;
} cdr_attr_upsert;

typedef struct cdr_event {
  int64_t event_id;
  int64_t version;
  int64_t timestamp;
  int64_t task_id;
  uint32_t type;  /* cdr_event_type */
  uint32_t flags; /* CDR_EVF_* */
  union {
    cdr_attr_wf_started started;
    cdr_attr_dt_scheduled dt_sched;
    cdr_attr_dt dt;
    cdr_attr_at_scheduled at_sched;
    cdr_attr_at at;
    cdr_attr_timer timer;
    cdr_attr_external ext;
    cdr_attr_initiated_ref ref;
    cdr_attr_can can;
    cdr_attr_upsert upsert;
    uint8_t raw[112];
  } a;
} cdr_event;

/* Per-workflow replay request: the arguments of one stateBuilder.applyEvents
 * sequence on a fresh mutable state (stateBuilder.go:112-119, builders
 * mutableStateBuilder.go:137-231).  A continue-as-new run is its own entry
 * (parent >= 0) so that it replays in parallel with its parent. */
typedef struct cdr_wf_desc {
  uint64_t wf_key;         /* stable key for cdr_uuid (host-assigned) */
  uint64_t ev_off, ev_len; /* events in cdr_batch.events */
  uint32_t domain_id, workflow_id, run_id, request_id; /* handles */
  uint32_t builder;        /* cdr_builder */
  int32_t retention_days;  /* domainEntry.GetRetentionDays(workflowID) */
  int64_t failover_version; /* domainEntry.GetFailoverVersion() */
  int64_t expected_next_event_id; /* nDCStateRebuilder check, 0 = none */
  int32_t parent;          /* index of the parent entry, -1 = none */
  int32_t newrun;          /* index of the new-run entry, -1 = none */
  uint32_t newrun_call;    /* call ordinal (0-based) whose newRunHistory is `newrun` */
  uint32_t newrun_ndc;     /* newRunNDC argument of that call */
} cdr_wf_desc;

#define CDR_MAX_CLUSTERS 8
/* cluster.Metadata restated (common/cluster/metadata.go:187-203) */
typedef struct cdr_cluster_meta {
  int64_t failover_version_increment;
  int32_t current_cluster;   /* index of the current cluster */
  int32_t n_clusters;
  int64_t initial_version[CDR_MAX_CLUSTERS]; /* cluster i owns versions with v % inc == initial_version[i] */
} cdr_cluster_meta;

typedef struct cdr_batch {
  const cdr_event* events;
  uint64_t n_events;
  const cdr_wf_desc* wfs;
  uint32_t n_wfs;
  uint32_t empty_uuid; /* handle the host interned for "emptyUuid" (mutableStateBuilder.go:42) */
  const cdr_kv* kvs;
  uint64_t n_kvs;
  const cdr_reset_point* rps;
  uint64_t n_rps;
  cdr_cluster_meta cluster;
  int64_t now_ns;     /* injected timeSource.Now() */
  uint64_t uuid_seed; /* injected uuid.New() */
  /* loaded mutable states (nullable): entries it names replay onto a loaded state
   * instead of a fresh builder (cdr_carry below) */
  const struct cdr_carry* carry;
} cdr_batch;

/* =========================================================== OUTPUT =======
 * The persisted WorkflowMutableState (dataInterfaces.go:610-622) as fixed-stride
 * records.  Fields that the replay path never writes (StartTimestamp,
 * LastUpdatedTimestamp, ExecutionContext, CompletionEvent, CancelRequestID,
 * Sticky*, Client*, SignalRequestedIDs, BufferedEvents) are omitted: they stay
 * at their zero value on a fresh builder. */

#define CDR_XI_CANCEL_REQUESTED 0x001u
#define CDR_XI_HAS_RETRY 0x002u
#define CDR_XI_HAS_EXPIRATION 0x004u   /* ExpirationTime is not the Go zero time */
#define CDR_XI_HAS_BRANCH 0x008u       /* ExecutionInfo.BranchToken set (non-NDC builders) */
#define CDR_XI_HAS_MEMO 0x010u
#define CDR_XI_HAS_SEARCH_ATTR 0x020u  /* SearchAttributes map non-nil */
#define CDR_XI_HAS_RESET_POINTS 0x040u /* AutoResetPoints non-nil */
#define CDR_XI_STARTED 0x080u          /* a WorkflowExecutionStarted event was applied */
#define CDR_XI_VH_BRANCH 0x100u        /* branch_* fields hold the NDC VersionHistory token */
/* Two 128-B halves (records are 256-B aligned in cdr_out): the first holds what
 * WorkflowExecutionStarted fixes (written once, when it is applied), the second what
 * the rest of the replay updates (written once, at the end) — so that each 128-B line
 * of the record reaches HBM once. */
typedef struct cdr_exec_info {
  /* -- set by WorkflowExecutionStarted (ReplicateWorkflowExecutionStartedEvent) */
  uint32_t domain_id, workflow_id, run_id, create_request_id;
  uint32_t parent_domain_id, parent_workflow_id, parent_run_id, task_list;
  uint32_t workflow_type, cron_schedule, memo, nonretriable;
  uint32_t branch_tree_id;
  int32_t workflow_timeout, decision_timeout_value, attempt;
  int64_t initiated_id;
  int32_t initial_interval, maximum_interval;
  double backoff_coefficient;
  int32_t maximum_attempts, expiration_seconds;
  int64_t expiration_time;
  uint64_t branch_id_lo, branch_id_hi;
  uint32_t _pad0, _pad1;
  /* -- updated by the replay */
  uint32_t decision_request_id, flags;
  int64_t completion_event_batch_id;
  int32_t state, close_status;
  int64_t last_first_event_id, last_event_task_id, next_event_id, last_processed_event;
  int32_t signal_count, decision_timeout;
  int64_t decision_version, decision_schedule_id, decision_started_id, decision_attempt;
  int64_t decision_started_ts, decision_scheduled_ts, decision_original_scheduled_ts;
  uint32_t reset_points_len, search_attr_len;
} cdr_exec_info;
#ifdef __cplusplus
static_assert(sizeof(cdr_exec_info) == 256 && offsetof(cdr_exec_info, decision_request_id) == 128, "cdr_exec_info");
#endif

/* ReplicationState (dataInterfaces.go:325-331) + LastReplicationInfo map keyed by
 * cluster index (bit i of lri_mask = entry present).  Written only for entries replayed
 * with the 2DC builder (present = 1); for other builders Go's ReplicationState is nil
 * and the record is left untouched. */
typedef struct cdr_repl_state {
  int64_t current_version, start_version, last_write_version, last_write_event_id;
  int64_t lri_version[CDR_MAX_CLUSTERS];
  int64_t lri_last_event_id[CDR_MAX_CLUSTERS];
  uint32_t lri_mask, present;
} cdr_repl_state;

typedef struct cdr_vh_item { int64_t event_id, version; } cdr_vh_item;

#define CDR_AI_CANCEL_REQUESTED 0x1u
#define CDR_AI_HAS_RETRY 0x2u
#define CDR_AI_STARTED_TIME_SET 0x4u /* StartedTime / LastHeartBeatUpdatedTime non-zero */
typedef struct cdr_activity_info { /* ActivityInfo dataInterfaces.go:625-662 */
  int64_t version, schedule_id, scheduled_event_batch_id, scheduled_time;
  int64_t started_id, started_time, last_heartbeat_time, expiration_time;
  int64_t cancel_request_id;
  uint32_t activity_id, request_id, task_list, nonretriable;
  int32_t s2s, s2c, stc, hb;
  int32_t timer_task_status, attempt;
  int32_t initial_interval, maximum_interval;
  int32_t maximum_attempts;
  uint32_t flags;
  double backoff_coefficient;
} cdr_activity_info;

typedef struct cdr_timer_info { /* TimerInfo dataInterfaces.go:665-671 */
  int64_t version, started_id, expiry_time, task_id;
  uint32_t timer_id, _pad;
} cdr_timer_info;

typedef struct cdr_child_info { /* ChildExecutionInfo dataInterfaces.go:674-687 */
  int64_t version, initiated_id, initiated_event_batch_id, started_id;
  uint64_t create_request_lo, create_request_hi;
  uint32_t started_workflow_id, started_run_id, domain_name, workflow_type;
  int32_t parent_close_policy, _pad;
} cdr_child_info;

typedef struct cdr_cancel_info { /* RequestCancelInfo dataInterfaces.go:690-695 */
  int64_t version, initiated_event_batch_id, initiated_id;
  uint64_t cancel_request_lo, cancel_request_hi;
} cdr_cancel_info;

typedef struct cdr_signal_info { /* SignalInfo dataInterfaces.go:698-706 */
  int64_t version, initiated_event_batch_id, initiated_id;
  uint64_t signal_request_lo, signal_request_hi;
  uint32_t signal_name, input, control, _pad;
} cdr_signal_info;

/* Transfer and timer tasks applyEvents appends (stateBuilder.go:613-804; the
 * persistence.Task types of dataInterfaces.go:121-155).  Emitted only when the caller
 * asks for them (cdr_out.transfer != NULL): in emission order, per entry, at the
 * caps.xfer_off / ttask_off slices, counts in cdr_out.n_tasks. */
enum cdr_task_type {
  /* transfer tasks (TransferTaskType*) */
  CDR_TT_DECISION = 0,        /* DomainID, TaskList, ScheduleID (event_id) */
  CDR_TT_ACTIVITY = 1,        /* DomainID, TaskList, ScheduleID */
  CDR_TT_CLOSE_EXECUTION = 2,
  CDR_TT_CANCEL_EXECUTION = 3, /* TargetDomainID, TargetWorkflowID, TargetRunID, child-only, InitiatedID */
  CDR_TT_START_CHILD = 4,      /* TargetDomainID, TargetWorkflowID, InitiatedID */
  CDR_TT_SIGNAL_EXECUTION = 5, /* as CANCEL_EXECUTION */
  CDR_TT_RECORD_STARTED = 6,
  CDR_TT_UPSERT_SA = 8,
  /* timer tasks (TaskType*) */
  CDR_TT_DECISION_TIMEOUT = 16 + 0, /* visibility, TimeoutType, EventID = ScheduleID, ScheduleAttempt */
  CDR_TT_ACTIVITY_TIMEOUT = 16 + 1, /* visibility, TimeoutType, EventID = ScheduleID, Attempt */
  CDR_TT_USER_TIMER = 16 + 2,       /* visibility, EventID = StartedID */
  CDR_TT_WORKFLOW_TIMEOUT = 16 + 3, /* visibility */
  CDR_TT_DELETE_HISTORY = 16 + 4,   /* visibility */
  CDR_TT_WORKFLOW_BACKOFF = 16 + 6  /* visibility, TimeoutType = WorkflowBackoffTimeoutType */
};
#define CDR_TF_CHILD_ONLY 0x1u /* TargetChildWorkflowOnly */
typedef struct cdr_task {
  uint32_t type; /* cdr_task_type */
  int32_t timeout_type;
  int64_t event_id;      /* ScheduleID / InitiatedID / EventID, 0 when the type has none */
  int64_t visibility_ts; /* timer tasks (ns); 0 for transfer tasks */
  int64_t attempt;
  uint32_t domain_id, task_list; /* handles: DomainID or TargetDomainID; TaskList */
  uint32_t target_workflow_id, target_run_id;
  uint32_t flags, _pad; /* CDR_TF_* */
  /* Version: set by refreshTasks (mutableStateTaskGenerator.go); stateBuilder's tasks
   * leave it to the caller (0) */
  int64_t version;
} cdr_task;
#ifdef __cplusplus
static_assert(sizeof(cdr_task) == 64, "cdr_task");
#endif

/* applyEvents' second return value, lastDecision *decisionInfo (stateBuilder.go:126,
 * 200,213,238,256,610), for the entry's last call: the decision the call's last
 * DecisionTaskScheduled, DecisionTaskStarted or transient decision (after a
 * DecisionTaskFailed / TimedOut) produced, or none (nil).  Its fields are the decision
 * manager's decisionInfo (mutableStateDecisionTaskManager.go:143-253).  TaskList is not
 * stored: for CDR_LD_SCHEDULED it is the DecisionTaskScheduled event's TaskList (event
 * event_index of the entry), otherwise ExecutionInfo.TaskList (applyEvents clears
 * stickiness, :116).  Written for CDR_OK entries when cdr_out.last_decision is set. */
enum cdr_ld_source { CDR_LD_NONE = 0, CDR_LD_SCHEDULED = 1, CDR_LD_STARTED = 2, CDR_LD_TRANSIENT = 3 };
typedef struct cdr_last_decision {
  uint32_t source;     /* cdr_ld_source */
  uint32_t request_id; /* handle (EmptyUUID until started) */
  int64_t event_index; /* index of the producing event within the entry's events */
  int64_t version, schedule_id, started_id, attempt;
  int64_t scheduled_ts, started_ts, original_scheduled_ts;
  int32_t decision_timeout, _pad;
} cdr_last_decision;
#ifdef __cplusplus
static_assert(sizeof(cdr_last_decision) == 80, "cdr_last_decision");
#endif

/* per-workflow result: status + where each variable-length table lives */
typedef struct cdr_wf_result {
  int32_t code;   /* cdr_status */
  uint32_t flags; /* CDR_RF_* */
  int64_t fail_event_id; /* eventId of the event that raised `code` */
  int64_t fail_index;    /* index of that event within the entry's events */
  uint32_t n_activity, n_timer, n_child, n_cancel, n_signal, n_vh;
  uint32_t n_reset_points, n_search_attr;
} cdr_wf_result;

/* Output capacities: one slot range per workflow and table; filled by
 * cdr_plan() from the input (counts of creating events, version runs, ...). */
typedef struct cdr_wf_caps {
  uint64_t act_off, timer_off, child_off, cancel_off, signal_off, vh_off, rp_off, sa_off;
  /* row capacities of the entry's table slices.  The five pending tables (activities, user
   * timers, children, request-cancels, signals) persist the rows still pending at the end,
   * so their capacity is the simulated peak live set (cdr_plan_caps; a loaded state's rows
   * counted in), or the number of creating events when a live set passes
   * CDR_WAVE_SLOTS + 1 (the device planner tracks no more); version-history items, reset
   * points and search attributes: every row the history can add */
  uint32_t act_cap, timer_cap, child_cap, cancel_cap, signal_cap, vh_cap, rp_cap, sa_cap;
  /* upper bounds of the live set (working slots): activities = max over prefixes of
   * (#scheduled - #closed), timers = peak live user timers */
  uint32_t act_live, timer_live;
  /* flags: CDR_CAP_*; order_key: the lane planner's ordering of register-table entries by
   * entity counts (cdr_plan_slices_ex), scheduled activities << 22 | started user timers << 11
   * | initiated children + request-cancels + signals, each saturating (10 / 11 / 11 bits) */
  uint32_t flags, order_key;
  /* task slices (bounds from the event types; used only when tasks are emitted) */
  uint64_t xfer_off, ttask_off;
  uint32_t xfer_cap, ttask_cap;
} cdr_wf_caps;
/* the history fits the fast-path replay kernel (replay_fast.inc): Started first and
 * only there, event types in CDR_FAST_TYPES, at most one pending activity, builder
 * NDC or local */
#define CDR_CAP_FAST 0x1u
/* the history fits the wave-per-workflow kernel (replay_wave.inc): at most 64 live
 * activities, user timers, children, request-cancels and signals at any time; not
 * CDR_CAP_FAST */
#define CDR_CAP_WAVE 0x2u
/* a CDR_CAP_WAVE history small enough that a lane slice replays it cheaper
 * (cdr_plan_slices_ex keeps it in the lane slices): peak live activities, user timers,
 * children + request-cancels + signals and the event count within these bounds */
#define CDR_CAP_LANE 0x4u
/* the history fits the register-table lane kernel (replay_reg.inc): not CDR_CAP_FAST; at
 * most CDR_REG_NA live activities, CDR_REG_NT live user timers, CDR_REG_NX live children,
 * request-cancels and signals each, CDR_REG_NRP reset points, CDR_REG_NSA search-attribute
 * keys; event ids strictly increasing in [1, 2^31); fewer than 2^20 events and calls
 * shorter than 4096 events (event indices are packed in 20 + 12 bits) */
#define CDR_CAP_REG 0x8u
#define CDR_REG_NA 6u
#define CDR_REG_NT 10u
#define CDR_REG_NX 4u
#define CDR_REG_NRP 6u
#define CDR_REG_NSA 8u
#define CDR_REG_NCL 4u /* 2DC: LastReplicationInfo kept for clusters < 4 (batch with more: general kernel) */
/* the same envelope with up to CDR_REG2_NA live activities (long activity-heavy
 * histories, C4/C5 tails): the kernel's second variant, at lower occupancy */
#define CDR_CAP_REG2 0x10u
#define CDR_REG2_NA 12u
#define CDR_REG2_NRP 12u /* ... and up to 12 reset points (Started's rolled-over ones + new checksums) */
/* the reset-point capacity of the register-table variant with na activity slots */
#define CDR_REG_NRP_OF(na) ((na) >= CDR_REG2_NA ? CDR_REG2_NRP : CDR_REG_NRP)
/* the envelope's small corner (at most CDR_REG0_NA live activities, CDR_REG0_NT live user
 * timers, CDR_REG0_NX live children / request-cancels / signals each): the variant whose
 * tables leave room for 3 waves per SIMD (168 VGPRs); such entries carry CDR_CAP_REG too */
#define CDR_CAP_REG0 0x20u
#define CDR_REG0_NA 3u
#define CDR_REG0_NT 5u
#define CDR_REG0_NX 3u
/* the entry replays onto a loaded state (cdr_carry; cdr_plan_caps / cdr_plan_ndc_apply set
 * it): never planned onto a PAR slice — only the register-table kernels' lane form and the
 * general kernel take a loaded state */
#define CDR_CAP_LOADED 0x40u
#define CDR_LANE_MAX_ACT 6u
#define CDR_LANE_MAX_TIMERS 10u
#define CDR_LANE_MAX_EXT 8u
#define CDR_LANE_MAX_LEN 512u
#define CDR_WAVE_SLOTS 64u

typedef struct cdr_totals {
  uint64_t act, timer, child, cancel, signal, vh, rp, sa;
  uint64_t xfer, ttask; /* task rows (cdr_task) */
} cdr_totals;

/* Caller-allocated output buffers (host or device memory, per the entry point). */
typedef struct cdr_out {
  cdr_wf_result* result;   /* [n_wfs] */
  cdr_exec_info* exec;     /* [n_wfs] */
  cdr_repl_state* repl;    /* [n_wfs] */
  cdr_vh_item* vh;         /* [totals.vh]  (per-wf slice at caps.vh_off) */
  cdr_activity_info* act;  /* [totals.act] */
  cdr_timer_info* timer;   /* [totals.timer] */
  cdr_child_info* child;   /* [totals.child] */
  cdr_cancel_info* cancel; /* [totals.cancel] */
  cdr_signal_info* signal; /* [totals.signal] */
  cdr_reset_point* rp;     /* [totals.rp] */
  cdr_kv* sa;              /* [totals.sa] */
  /* tasks (nullable: NULL = not emitted, the default; rebuild discards them) */
  cdr_task* transfer;      /* [totals.xfer] */
  cdr_task* timer_tasks;   /* [totals.ttask] */
  uint32_t* n_tasks;       /* [2 * n_wfs]: transfer, timer count of entry w */
  cdr_last_decision* last_decision; /* [n_wfs] nullable: applyEvents' lastDecision */
} cdr_out;

/* Carry-in: replay onto a LOADED mutable state, the analogue of
 * mutableStateBuilder.Load (mutableStateBuilder.go:272-295) followed by applyEvents —
 * the NDC replicator's apply-to-current-branch path (nDCHistoryReplicator.go:330-398)
 * and the 2DC historyReplicator.  The loaded states are the persisted records of an
 * earlier replay in cdr_out form (per-entry slices at `caps`' offsets, counts in
 * state.result).  Entry w of the batch loads record src[w] (-1: fresh builder, as
 * without carry).  A loaded entry must have state.result[src].code == CDR_OK.
 * Load's non-persisted effects are restated: currentVersion = EmptyVersion,
 * pendingActivityInfoByActivityID rebuilt from the activity rows (ascending
 * scheduleID, the last duplicate activityID wins).  The caller keeps the fields the
 * records omit (schema.h OUTPUT); applyEvents clears stickiness, so a drop-in shim
 * zeroes Sticky* / Client* after the call.  SignalRequestedIDs and BufferedEvents pass
 * through applyEvents unchanged — no Replicate* method reads or writes them (their only
 * writers are AddSignalRequested / DeleteSignalRequested, mutableStateBuilder.go:
 * 1455-1474, the active-side AddTimerCanceledEvent's checkAndClearTimerFiredEvent,
 * :2959, and CloseTransaction*, :3925) — so the shim carries a loaded state's sets into
 * the result as they are, and a fresh builder's are empty. */
typedef struct cdr_carry {
  const int32_t* src;      /* [n_wfs of the batch] */
  const cdr_wf_caps* caps; /* [n_src] row offsets of the loaded states' tables */
  uint32_t n_src, _pad;    /* entries in `state` */
  cdr_totals totals;       /* rows in each table of `state` */
  cdr_out state;           /* read only */
  /* [n_wfs of the batch], nullable: entry w continues an IN-MEMORY builder rather than a
   * loaded one — the state nDCConflictResolver.rebuild hands to applyEvents
   * (nDCConflictResolver.go:117-184, nDCHistoryReplicator.go:330-398) never went through
   * Load, so its NDC currentVersion is the one the rebuild's replay left: the version of its
   * last event applied while running, which for a history that ends at (or before) its close
   * event is its last version-history item's version.  0 = Load (EmptyVersion). */
  const uint8_t* in_memory;
} cdr_carry;

/* ==================================================== NDC VERSION HISTORIES ===
 * The persisted VersionHistories of an NDC workflow (common/persistence/versionHistory.go:
 * VersionHistories{currentVersionHistoryIndex, histories []*VersionHistory}), one branch
 * per fork of the history tree.  A branch token is the history tree's branch token
 * (TreeID = run handle, BranchID = 128-bit UUID; dataInterfaces.go:2428-2440), compared
 * by value.  The items of branch b of a workflow live at
 * items[vhs.items_off + b * vhs.items_cap ...] (caller-planned capacity). */
#define CDR_VHS_MAX_BRANCHES 8
typedef struct cdr_vh_token {
  uint32_t tree, _pad;
  uint64_t branch_lo, branch_hi;
} cdr_vh_token;
typedef struct cdr_vh_branch { /* one VersionHistory */
  cdr_vh_token token;
  uint32_t n_items, _pad;
} cdr_vh_branch;
typedef struct cdr_vhs { /* VersionHistories */
  uint32_t current, n_branches;
  uint32_t items_cap, _pad;
  uint64_t items_off;
  cdr_vh_branch branch[CDR_VHS_MAX_BRANCHES];
} cdr_vhs;

/* One NDC replication task as nDCBranchMgr.prepareVersionHistory and
 * nDCConflictResolver.prepareMutableState see it (nDCBranchMgr.go:80-125,
 * nDCConflictResolver.go:73-114): the incoming VersionHistory (task.getVersionHistory(),
 * its items in the task item pool), the first / last event and the task's version, and
 * the token ForkHistoryBranch would return if a branch has to be created
 * (nDCBranchMgr.go:205-240, host-supplied). */
typedef struct cdr_ndc_task {
  uint64_t items_off;
  uint32_t n_items, _pad;
  int64_t first_event_id;
  int64_t last_event_id, last_version;
  int64_t version;
  cdr_vh_token new_token;
} cdr_ndc_task;

/* What the replicator does with the task (nDCHistoryReplicator.go:295-470) */
enum cdr_ndc_action {
  CDR_NDC_SKIP = 0,          /* duplicate task: verifyEventsOrder returned doContinue = false */
  CDR_NDC_APPLY_CURRENT = 1, /* branch is the current one: applyEvents onto the mutable state */
  CDR_NDC_REBUILD = 2,       /* rebuild the branch (nDCStateRebuilder, events 1 .. rebuild_next-1),
                                then applyEvents onto the rebuilt state */
  CDR_NDC_BACKFILL = 3       /* non-current branch, lower version: branch VH AddOrUpdateItem(last
                                event) only, mutable state unchanged */
};
typedef struct cdr_ndc_decision {
  int32_t code;   /* cdr_status (CDR_OK or the Go error site) */
  int32_t action; /* cdr_ndc_action */
  uint32_t branch_index, created; /* target branch; 1 if createNewBranch ran */
  int64_t rebuild_next_event_id;  /* REBUILD: baseNextEventID = branch lastItem.EventID + 1 */
  cdr_vh_item lca;                /* FindLCAVersionHistoryIndexAndItem's item */
  cdr_vh_token rebuild_token;     /* REBUILD: the branch's token (SetCurrentBranchToken target) */
} cdr_ndc_decision;

#ifdef __cplusplus
}
#endif
#endif /* CDR_SCHEMA_H */
