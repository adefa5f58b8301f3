// oracle/replay_ref.cpp — TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
//
// A scalar, per-workflow, literal restatement of the reference's replay path
// (Uber Cadence at /root/reference).  It walks each history exactly the way the Go
// code does — one event at a time, mutating map-based mutable state — so that the
// HIP engine in cadence_amd/ can be checked against it field by field.  Nothing in
// the product links or calls this file; tests/, __graft_entry__.smoke() and the
// bench's cpu_baseline leg are its only users.
//
// Followed, function by function (all paths relative to /root/reference):
//   stateBuilderImpl.applyEvents            service/history/stateBuilder.go:112-611
//   timer picks                              service/history/stateBuilder.go:706-729,796-804
//                                            service/history/timerBuilder.go:171-312,410-432
//   mutableStateBuilder ctors                service/history/mutableStateBuilder.go:137-231
//   UpdateCurrentVersion / replication state service/history/mutableStateBuilder.go:445-581
//   Replicate*Event                          service/history/mutableStateBuilder.go:1639-3603
//   DeleteActivity/UserTimer/Pending*        service/history/mutableStateBuilder.go:1138-1297
//   ClearStickyness / IsRunning              service/history/mutableStateBuilder.go:1398-1435
//   binary checksum reset points             service/history/mutableStateBuilder.go:1798-1862
//   rolloverAutoResetPoints                  service/history/mutableStateBuilder.go:3184-3205
//   decision FSM                             service/history/mutableStateDecisionTaskManager.go:143-279,635-800
//   state/close-status validation            common/persistence/workflowExecutionInfo.go:45-147
//   version history                          common/persistence/versionHistory.go:31-236
//   ClusterNameForFailoverVersion            common/cluster/metadata.go:187-203
//   nDCStateRebuilder next-event check       service/history/nDCStateRebuilder.go:139-143
//
// Reference nondeterminism and how it is pinned here:
//   * uuid.New() / timeSource.Now() are injected (cdr_uuid, batch.now_ns).
//   * Go map iteration order decides cross-entity ties in the timer picks; this
//     restatement breaks them by (time, scheduleID, candidate order) for activities
//     and (expiry, startedID) for user timers.  Within one activity the append order
//     wins, as Go's insertion sort does for short slices.
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <map>
#include <system_error>
#include <thread>
#include <vector>

#include "cdr/schema.h"

namespace {

struct GoErr {
  int32_t code = CDR_OK;
  int64_t event_id = 0;
  int64_t index = 0;
  uint32_t flags = 0;
  bool ok() const { return code == CDR_OK; }
};

// ------------------------------------------------------------------ VH
// common/persistence/versionHistory.go
struct VHItem {
  int64_t eventID, version;
};
struct VersionHistory {
  std::vector<VHItem> items;
  bool has_token = false;
  uint32_t tree = 0;
  uint64_t br_lo = 0, br_hi = 0;
  // NewVersionHistoryItem panics (versionHistory.go:36-42) -> CDR_P_VH_ITEM_INVALID
  // AddOrUpdateItem versionHistory.go:203-236
  int32_t AddOrUpdateItem(int64_t eventID, int64_t version) {
    if (eventID < 0 || (version < 0 && version != CDR_EMPTY_VERSION)) return CDR_P_VH_ITEM_INVALID;
    if (items.empty()) {
      items.push_back({eventID, version});
      return CDR_OK;
    }
    VHItem& last = items.back();
    if (version < last.version) return CDR_E_VH_LOWER_VERSION;
    if (eventID <= last.eventID) return CDR_E_VH_LOWER_EVENT_ID;
    if (version > last.version)
      items.push_back({eventID, version});
    else
      last.eventID = eventID;
    return CDR_OK;
  }
};

// ------------------------------------------------------------------ infos
struct ActivityInfo {  // dataInterfaces.go:625-662
  int64_t Version, ScheduleID, ScheduledEventBatchID, ScheduledTime;
  int64_t StartedID;
  bool StartedTimeSet = false;
  int64_t StartedTime = 0;
  uint32_t ActivityID, RequestID = 0;
  int32_t ScheduleToStartTimeout, ScheduleToCloseTimeout, StartToCloseTimeout, HeartbeatTimeout;
  bool CancelRequested = false;
  int64_t CancelRequestID;
  bool LastHeartBeatSet = false;
  int64_t LastHeartBeatUpdatedTime = 0;
  int32_t TimerTaskStatus = 0;
  int32_t Attempt = 0;
  uint32_t TaskList;
  bool HasRetryPolicy;
  int32_t InitialInterval = 0;
  double BackoffCoefficient = 0;
  int32_t MaximumInterval = 0;
  bool ExpirationSet = false;
  int64_t ExpirationTime = 0;
  int32_t MaximumAttempts = 0;
  uint32_t NonRetriableErrors = 0;
  int64_t LastHeartbeatTimeoutVisibility = 0;  // not persisted
};
struct TimerInfo {  // dataInterfaces.go:665-671
  int64_t Version;
  uint32_t TimerID;
  int64_t StartedID, ExpiryTime, TaskID;
};
struct ChildInfo {  // dataInterfaces.go:674-687
  int64_t Version, InitiatedID, InitiatedEventBatchID, StartedID;
  uint32_t StartedWorkflowID, StartedRunID = 0;
  uint64_t CreateReqLo, CreateReqHi;
  uint32_t DomainName, WorkflowTypeName;
  int32_t ParentClosePolicy;
};
struct CancelInfo {  // dataInterfaces.go:690-695
  int64_t Version, InitiatedEventBatchID, InitiatedID;
  uint64_t ReqLo, ReqHi;
};
struct SignalInfo {  // dataInterfaces.go:698-706
  int64_t Version, InitiatedEventBatchID, InitiatedID;
  uint64_t ReqLo, ReqHi;
  uint32_t SignalName, Input, Control;
};

struct ExecutionInfo {  // dataInterfaces.go:259-316 (replay-written subset)
  uint32_t DomainID = 0, WorkflowID = 0, RunID = 0, ParentDomainID = 0, ParentWorkflowID = 0,
           ParentRunID = 0;
  int64_t InitiatedID = 0, CompletionEventBatchID = 0;
  uint32_t TaskList = 0, WorkflowTypeName = 0;
  int32_t WorkflowTimeout = 0, DecisionTimeoutValue = 0;
  int32_t State = CDR_STATE_CREATED, CloseStatus = CDR_CLOSE_NONE;
  int64_t LastFirstEventID = 0, LastEventTaskID = 0, NextEventID = CDR_FIRST_EVENT_ID,
          LastProcessedEvent = CDR_EMPTY_EVENT_ID;
  uint32_t CreateRequestID = 0;
  int32_t SignalCount = 0;
  int64_t DecisionVersion = CDR_EMPTY_VERSION, DecisionScheduleID = CDR_EMPTY_EVENT_ID,
          DecisionStartedID = CDR_EMPTY_EVENT_ID;
  uint32_t DecisionRequestID = 0;  // "emptyUuid" is interned by the host; see kEmptyUUID
  int32_t DecisionTimeout = 0;
  int64_t DecisionAttempt = 0, DecisionStartedTimestamp = 0, DecisionScheduledTimestamp = 0,
          DecisionOriginalScheduledTimestamp = 0;
  bool CancelRequested = false;
  bool HasResetPoints = false;
  std::vector<cdr_reset_point> ResetPoints;
  bool HasMemo = false;
  uint32_t Memo = 0;
  bool HasSearchAttr = false;
  std::vector<cdr_kv> SearchAttributes;  // Go map; kept in insertion order, sorted on output
  int32_t Attempt = 0;
  bool HasRetryPolicy = false;
  int32_t InitialInterval = 0;
  double BackoffCoefficient = 0;
  int32_t MaximumInterval = 0;
  bool ExpirationSet = false;
  int64_t ExpirationTime = 0;
  int32_t MaximumAttempts = 0;
  uint32_t NonRetriableErrors = 0;
  bool HasBranchToken = false;
  uint32_t BranchTree = 0;
  uint64_t BranchLo = 0, BranchHi = 0;
  uint32_t CronSchedule = 0;
  int32_t ExpirationSeconds = 0;
  bool Started = false;
};

struct ReplicationState {  // dataInterfaces.go:325-331
  int64_t CurrentVersion, StartVersion, LastWriteVersion, LastWriteEventID;
  std::map<int, std::pair<int64_t, int64_t>> LastReplicationInfo;  // cluster -> (version, lastEventID)
};

// workflowExecutionInfo.go:45-147 — returns false on an invalid transition
bool UpdateWorkflowStateCloseStatus(ExecutionInfo& e, int state, int closeStatus) {
  auto bad = [] { return false; };
  switch (e.State) {
    case CDR_STATE_VOID:
      break;
    case CDR_STATE_CREATED:
      switch (state) {
        case CDR_STATE_CREATED:
        case CDR_STATE_RUNNING:
        case CDR_STATE_ZOMBIE:
          if (closeStatus != CDR_CLOSE_NONE) return bad();
          break;
        case CDR_STATE_COMPLETED:
          if (closeStatus != CDR_CLOSE_TERMINATED && closeStatus != CDR_CLOSE_TIMED_OUT) return bad();
          break;
        default:
          return bad();
      }
      break;
    case CDR_STATE_RUNNING:
      switch (state) {
        case CDR_STATE_CREATED:
          return bad();
        case CDR_STATE_RUNNING:
        case CDR_STATE_ZOMBIE:
          if (closeStatus != CDR_CLOSE_NONE) return bad();
          break;
        case CDR_STATE_COMPLETED:
          if (closeStatus == CDR_CLOSE_NONE) return bad();
          break;
        default:
          return bad();
      }
      break;
    case CDR_STATE_COMPLETED:
      switch (state) {
        case CDR_STATE_COMPLETED:
          if (closeStatus != e.CloseStatus) return bad();
          break;
        default:
          return bad();
      }
      break;
    case CDR_STATE_ZOMBIE:
      switch (state) {
        case CDR_STATE_CREATED:
        case CDR_STATE_RUNNING:
          if (closeStatus != CDR_CLOSE_NONE) return bad();
          break;
        case CDR_STATE_COMPLETED:
        case CDR_STATE_ZOMBIE:
          if (closeStatus == CDR_CLOSE_NONE) return bad();
          break;
        default:
          return bad();
      }
      break;
    default:
      return bad();
  }
  e.State = state;
  e.CloseStatus = closeStatus;
  return true;
}

struct Ctx {
  const cdr_batch* b;
  uint32_t empty_uuid;  // handle of the "emptyUuid" sentinel (mutableStateBuilder.go:42)
};

struct MutableState {
  const Ctx* ctx;
  int builder;
  uint64_t wf_key;
  int32_t retention_days;
  ExecutionInfo ei;
  // applyEvents' lastDecision of the latest call (stateBuilder.go:126,200,213,238,256,610)
  cdr_last_decision lastDecision{};
  bool hasRS = false;
  ReplicationState rs{};
  bool hasVH = false;
  VersionHistory vh;
  int64_t currentVersion;
  int64_t failover_at_ctor;  // domainEntry.GetFailoverVersion(), reused for the new run's builder
  std::map<int64_t, ActivityInfo> pendingActivityInfoIDs;
  std::map<uint32_t, int64_t> pendingActivityInfoByActivityID;
  std::map<uint32_t, TimerInfo> pendingTimerInfoIDs;
  std::map<int64_t, ChildInfo> pendingChildExecutionInfoIDs;
  std::map<int64_t, CancelInfo> pendingRequestCancelInfoIDs;
  std::map<int64_t, SignalInfo> pendingSignalInfoIDs;
  // stateBuilder.transferTasks / timerTasks (stateBuilder.go:613-804), each task once
  // in generation order (getTransferTasks / getTimerTasks)
  std::vector<cdr_task> transferTasks, timerTasks;
  void AddXfer(uint32_t type, int64_t eventID, uint32_t domain, uint32_t taskList) {
    cdr_task t{};
    t.type = type;
    t.event_id = eventID;
    t.domain_id = domain;
    t.task_list = taskList;
    transferTasks.push_back(t);
  }
  void AddTimer(uint32_t type, int32_t timeoutType, int64_t eventID, int64_t vis, int64_t attempt) {
    cdr_task t{};
    t.type = type;
    t.timeout_type = timeoutType;
    t.event_id = eventID;
    t.visibility_ts = vis;
    t.attempt = attempt;
    timerTasks.push_back(t);
  }

  // newMutableStateBuilder (mutableStateBuilder.go:137-231)
  MutableState(const Ctx* c, int kind, int64_t failover, uint64_t key, int32_t retention)
      : ctx(c), builder(kind), wf_key(key), retention_days(retention), currentVersion(failover),
        failover_at_ctor(failover) {
    ei.DecisionRequestID = c->empty_uuid;
    if (kind == CDR_BUILDER_2DC) {
      hasRS = true;
      rs.StartVersion = currentVersion;
      rs.CurrentVersion = currentVersion;
      rs.LastWriteVersion = CDR_EMPTY_VERSION;
      rs.LastWriteEventID = CDR_EMPTY_EVENT_ID;
    } else if (kind == CDR_BUILDER_NDC) {
      hasVH = true;
    }
  }

  // appendTasksForFinishedExecutions (stateBuilder.go:775-787): CloseExecutionTask +
  // DeleteHistoryEventTask at the event time + the domain's retention
  void AppendTasksForFinishedExecution(int64_t ts) {
    AddXfer(CDR_TT_CLOSE_EXECUTION, 0, 0, 0);
    AddTimer(CDR_TT_DELETE_HISTORY, 0, 0, ts + (int64_t)retention_days * 24LL * 3600LL * 1000000000LL, 0);
  }
  bool IsWorkflowExecutionRunning() const {  // :1422-1435
    return ei.State == CDR_STATE_CREATED || ei.State == CDR_STATE_RUNNING;
  }
  int64_t GetCurrentVersion() const {  // :491-502
    if (hasRS) return rs.CurrentVersion;
    if (hasVH) return currentVersion;
    return CDR_EMPTY_VERSION;
  }
  // :445-489 (NDC branch; the 2DC branch is reached through the prelude instead)
  void UpdateCurrentVersion(int64_t version, bool force) {
    if (!IsWorkflowExecutionRunning()) return;
    if (hasRS) {
      if (version > rs.CurrentVersion || force) rs.CurrentVersion = version;
      return;
    }
    if (hasVH) {
      if (!vh.items.empty()) currentVersion = vh.items.back().version;
      if (version > currentVersion || force) currentVersion = version;
    }
  }
  // cluster.Metadata.ClusterNameForFailoverVersion (metadata.go:187-203); -1 = panic
  int ClusterForVersion(int64_t v) const {
    const cdr_cluster_meta& m = ctx->b->cluster;
    if (v == CDR_EMPTY_VERSION) return m.current_cluster;
    int64_t init = v % m.failover_version_increment;
    for (int i = 0; i < m.n_clusters; i++)
      if (m.initial_version[i] == init) return i;
    return -1;
  }
  void ClearStickyness() {}  // sticky/client fields are not part of the output (always "")

  // decision manager UpdateDecision (:677-702)
  struct DecisionInfo {
    int64_t Version, ScheduleID, StartedID;
    uint32_t RequestID;
    int32_t DecisionTimeout;
    int64_t Attempt, StartedTimestamp, ScheduledTimestamp, OriginalScheduledTimestamp;
  };
  DecisionInfo getDecisionInfo() const {
    return {ei.DecisionVersion,  ei.DecisionScheduleID,        ei.DecisionStartedID,
            ei.DecisionRequestID, ei.DecisionTimeout,          ei.DecisionAttempt,
            ei.DecisionStartedTimestamp, ei.DecisionScheduledTimestamp,
            ei.DecisionOriginalScheduledTimestamp};
  }
  void UpdateDecision(const DecisionInfo& d) {
    ei.DecisionVersion = d.Version;
    ei.DecisionScheduleID = d.ScheduleID;
    ei.DecisionStartedID = d.StartedID;
    ei.DecisionRequestID = d.RequestID;
    ei.DecisionTimeout = d.DecisionTimeout;
    ei.DecisionAttempt = d.Attempt;
    ei.DecisionStartedTimestamp = d.StartedTimestamp;
    ei.DecisionScheduledTimestamp = d.ScheduledTimestamp;
    ei.DecisionOriginalScheduledTimestamp = d.OriginalScheduledTimestamp;
  }
  bool HasPendingDecision() const { return ei.DecisionScheduleID != CDR_EMPTY_EVENT_ID; }
  // the *decisionInfo a decision event returned: the decision fields it just set
  // (TaskList is the event's or ExecutionInfo.TaskList: not recorded, schema.h)
  cdr_last_decision snapDecision(uint32_t source, int64_t index) const {
    cdr_last_decision d{};
    d.source = source;
    d.request_id = ei.DecisionRequestID;
    d.event_index = index;
    d.version = ei.DecisionVersion;
    d.schedule_id = ei.DecisionScheduleID;
    d.started_id = ei.DecisionStartedID;
    d.attempt = ei.DecisionAttempt;
    d.scheduled_ts = ei.DecisionScheduledTimestamp;
    d.started_ts = ei.DecisionStartedTimestamp;
    d.original_scheduled_ts = ei.DecisionOriginalScheduledTimestamp;
    d.decision_timeout = ei.DecisionTimeout;
    return d;
  }
  // FailDecision (:635-656)
  void FailDecision(bool incrementAttempt) {
    ClearStickyness();
    DecisionInfo f{CDR_EMPTY_VERSION, CDR_EMPTY_EVENT_ID, CDR_EMPTY_EVENT_ID, ctx->empty_uuid, 0, 0, 0, 0, 0};
    if (incrementAttempt) {
      f.Attempt = ei.DecisionAttempt + 1;
      f.ScheduledTimestamp = ctx->b->now_ns;
    }
    UpdateDecision(f);
  }
  // DeleteDecision (:659-674)
  void DeleteDecision() {
    DecisionInfo r{CDR_EMPTY_VERSION, CDR_EMPTY_EVENT_ID, CDR_EMPTY_EVENT_ID, ctx->empty_uuid, 0, 0, 0, 0,
                   getDecisionInfo().OriginalScheduledTimestamp};
    UpdateDecision(r);
  }
  // ReplicateTransientDecisionTaskScheduled (:169-198)
  bool ReplicateTransientDecisionTaskScheduled() {
    if (HasPendingDecision() || ei.DecisionAttempt == 0) return false;
    DecisionInfo d{GetCurrentVersion(), ei.NextEventID, CDR_EMPTY_EVENT_ID, ctx->empty_uuid,
                   ei.DecisionTimeoutValue, ei.DecisionAttempt, 0, ctx->b->now_ns, 0};
    UpdateDecision(d);
    return true;
  }

  // DeleteActivity (:1247-1269)
  int32_t DeleteActivity(int64_t scheduleEventID) {
    auto it = pendingActivityInfoIDs.find(scheduleEventID);
    if (it == pendingActivityInfoIDs.end()) return CDR_E_ACTIVITY_NOT_FOUND;
    uint32_t aid = it->second.ActivityID;
    pendingActivityInfoIDs.erase(it);
    auto jt = pendingActivityInfoByActivityID.find(aid);
    if (jt == pendingActivityInfoByActivityID.end()) return CDR_E_ACTIVITY_ID_NOT_FOUND;
    pendingActivityInfoByActivityID.erase(jt);
    return CDR_OK;
  }

  // timerBuilder.GetActivityTimerTaskIfNeeded (:211-230) + loadActivityTimers (:249-312)
  void ActivityTimerPick() {
    struct Cand {
      int64_t t;
      int64_t sched;
      int order;
      int32_t type;
      bool created;
    };
    std::vector<Cand> c;
    for (auto& kv : pendingActivityInfoIDs) {
      const ActivityInfo& v = kv.second;
      if (v.ScheduleID == CDR_EMPTY_EVENT_ID) continue;
      int64_t s2c = v.ScheduledTime + (int64_t)v.ScheduleToCloseTimeout * 1000000000LL;
      if (v.ExpirationSet && v.ExpirationTime < s2c) s2c = v.ExpirationTime;
      c.push_back({s2c, v.ScheduleID, 0, CDR_TIMEOUT_SCHEDULE_TO_CLOSE,
                   (v.TimerTaskStatus & CDR_TTS_SCHEDULE_TO_CLOSE) != 0});
      if (v.StartedID != CDR_EMPTY_EVENT_ID) {
        int64_t st = v.StartedTimeSet ? v.StartedTime : 0;
        c.push_back({st + (int64_t)v.StartToCloseTimeout * 1000000000LL, v.ScheduleID, 1,
                     CDR_TIMEOUT_START_TO_CLOSE, (v.TimerTaskStatus & CDR_TTS_START_TO_CLOSE) != 0});
        if (v.HeartbeatTimeout > 0) {
          int64_t lhb = v.LastHeartBeatSet ? v.LastHeartBeatUpdatedTime : 0;
          if (lhb < st) lhb = st;
          c.push_back({lhb + (int64_t)v.HeartbeatTimeout * 1000000000LL, v.ScheduleID, 2,
                       CDR_TIMEOUT_HEARTBEAT, (v.TimerTaskStatus & CDR_TTS_HEARTBEAT) != 0});
        }
      } else {
        c.push_back({v.ScheduledTime + (int64_t)v.ScheduleToStartTimeout * 1000000000LL, v.ScheduleID, 1,
                     CDR_TIMEOUT_SCHEDULE_TO_START, (v.TimerTaskStatus & CDR_TTS_SCHEDULE_TO_START) != 0});
      }
    }
    if (c.empty()) return;
    std::stable_sort(c.begin(), c.end(), [](const Cand& x, const Cand& y) {
      if (x.t != y.t) return x.t < y.t;
      if (x.sched != y.sched) return x.sched < y.sched;
      return x.order < y.order;
    });
    const Cand& h = c[0];
    if (h.created) return;  // firstActivityTimerTask (:384-389)
    ActivityInfo& ai = pendingActivityInfoIDs[h.sched];
    // createNewTask (timerBuilder.go:391-408): ActivityTimeoutTask
    AddTimer(CDR_TT_ACTIVITY_TIMEOUT, h.type, h.sched, h.t, ai.Attempt);
    int32_t bit = h.type == CDR_TIMEOUT_HEARTBEAT        ? CDR_TTS_HEARTBEAT
                  : h.type == CDR_TIMEOUT_SCHEDULE_TO_START ? CDR_TTS_SCHEDULE_TO_START
                  : h.type == CDR_TIMEOUT_SCHEDULE_TO_CLOSE ? CDR_TTS_SCHEDULE_TO_CLOSE
                                                             : CDR_TTS_START_TO_CLOSE;
    ai.TimerTaskStatus |= bit;
    if (h.type == CDR_TIMEOUT_HEARTBEAT) {
      // .Unix() seconds (timerBuilder.go:224); floor division like Go's time.Unix()
      int64_t t = h.t;
      ai.LastHeartbeatTimeoutVisibility = t >= 0 ? t / 1000000000LL : -((-t + 999999999LL) / 1000000000LL);
    }
  }

  // timerBuilder.GetUserTimerTaskIfNeeded (:171-184) + loadUserTimers (:233-247)
  void UserTimerPick() {
    const TimerInfo* head = nullptr;
    for (auto& kv : pendingTimerInfoIDs) {
      const TimerInfo& t = kv.second;
      if (!head || t.ExpiryTime < head->ExpiryTime ||
          (t.ExpiryTime == head->ExpiryTime && t.StartedID < head->StartedID))
        head = &t;
    }
    if (!head) return;
    if (head->TaskID == CDR_TIMER_TASK_STATUS_CREATED) return;  // firstTimerTask (:370-375)
    AddTimer(CDR_TT_USER_TIMER, 0, head->StartedID, head->ExpiryTime, 0);  // createNewTask: UserTimerTask
    pendingTimerInfoIDs[head->TimerID].TaskID = CDR_TIMER_TASK_STATUS_CREATED;
  }
};

struct StateBuilder {
  const Ctx* ctx;
  const cdr_batch* b;
  MutableState* ms;

  // applyEvents (stateBuilder.go:112-611).  `history` is one call's events.
  // On success *newRun holds the continue-as-new mutable state (or null).
  GoErr applyEvents(uint32_t requestID, uint32_t workflowID, uint32_t runID, uint32_t domainID,
                    const cdr_event* history, size_t n, int64_t index_base,
                    const cdr_event* newRunHistory, size_t n_newrun, bool newRunNDC, uint64_t newrun_key,
                    uint32_t newrun_request, MutableState** newRun, GoErr* newRunErr) {
    GoErr err;
    if (n == 0) {
      err.code = CDR_E_HISTORY_EMPTY;
      return err;
    }
    const cdr_event& first = history[0];
    const cdr_event& last = history[n - 1];
    ms->ClearStickyness();
    ms->lastDecision = cdr_last_decision{};  // var lastDecision *decisionInfo (:126)
    auto fail = [&](int32_t code, size_t i) {
      GoErr e;
      e.code = code;
      e.event_id = history[i].event_id;
      e.index = index_base + (int64_t)i;
      return e;
    };
    for (size_t i = 0; i < n; i++) {
      const cdr_event& ev = history[i];
      // version prelude (:134-154)
      if (ms->hasRS) {
        // UpdateReplicationStateVersion(event.Version, true) (:548-556)
        ms->rs.CurrentVersion = ev.version;
        // UpdateReplicationStateLastEventID(last.Version, last.EventId) (:561-581)
        ms->rs.LastWriteVersion = last.version;
        ms->rs.LastWriteEventID = last.event_id;
        int src = ms->ClusterForVersion(last.version);
        if (src < 0) return fail(CDR_P_UNKNOWN_CLUSTER, i);
        if (src != b->cluster.current_cluster) ms->rs.LastReplicationInfo[src] = {last.version, last.event_id};
      } else if (ms->hasVH) {
        ms->UpdateCurrentVersion(ev.version, true);
        int32_t c = ms->vh.AddOrUpdateItem(ev.event_id, ev.version);
        if (c != CDR_OK) return fail(c, i);
      }
      ms->ei.LastEventTaskID = ev.task_id;  // :155

      ExecutionInfo& ei = ms->ei;
      switch (ev.type) {
        case CDR_EV_WF_STARTED: {  // :158-184
          const cdr_attr_wf_started& a = ev.a.started;
          uint32_t parentDomainID = 0;
          bool hasParentDomain = false;
          if (a.flags & CDR_SF_HAS_PARENT_DOMAIN) {
            if (a.flags & CDR_SF_PARENT_DOMAIN_MISSING) return fail(CDR_E_DOMAIN_NOT_FOUND, i);
            parentDomainID = a.parent_domain_id;
            hasParentDomain = true;
          }
          // ReplicateWorkflowExecutionStartedEvent (mutableStateBuilder.go:1639-1716)
          ei.CreateRequestID = requestID;
          ei.DomainID = domainID;
          ei.WorkflowID = workflowID;
          ei.RunID = runID;
          ei.TaskList = a.task_list;
          ei.WorkflowTypeName = a.workflow_type;
          ei.WorkflowTimeout = a.exec_timeout_s;
          ei.DecisionTimeoutValue = a.task_timeout_s;
          if (!UpdateWorkflowStateCloseStatus(ei, CDR_STATE_CREATED, CDR_CLOSE_NONE))
            return fail(CDR_E_INVALID_STATE_TRANSITION, i);
          ei.LastProcessedEvent = CDR_EMPTY_EVENT_ID;
          ei.LastFirstEventID = ev.event_id;
          ei.DecisionVersion = CDR_EMPTY_VERSION;
          ei.DecisionScheduleID = CDR_EMPTY_EVENT_ID;
          ei.DecisionStartedID = CDR_EMPTY_EVENT_ID;
          ei.DecisionRequestID = ctx->empty_uuid;
          ei.DecisionTimeout = 0;
          ei.CronSchedule = a.cron_schedule;
          if (hasParentDomain) ei.ParentDomainID = parentDomainID;
          if (a.flags & CDR_SF_HAS_PARENT_EXEC) {
            ei.ParentWorkflowID = a.parent_workflow_id;
            ei.ParentRunID = a.parent_run_id;
          }
          ei.InitiatedID = (a.flags & CDR_SF_HAS_PARENT_INITIATED) ? a.parent_initiated_id : CDR_EMPTY_EVENT_ID;
          ei.Attempt = a.attempt;
          if (a.expiration_ts != 0) {
            ei.ExpirationSet = true;
            ei.ExpirationTime = a.expiration_ts;
          }
          if (a.flags & CDR_SF_HAS_RETRY) {
            ei.HasRetryPolicy = true;
            ei.BackoffCoefficient = a.backoff_coefficient;
            ei.ExpirationSeconds = a.retry_expiration_s;
            ei.InitialInterval = a.retry_initial_s;
            ei.MaximumAttempts = a.retry_max_attempts;
            ei.MaximumInterval = a.retry_max_interval_s;
            ei.NonRetriableErrors = a.nonretriable;
          }
          // rolloverAutoResetPointsWithExpiringTime (:3184-3205)
          if (a.flags & CDR_SF_HAS_RESET_POINTS) {
            ei.HasResetPoints = true;
            ei.ResetPoints.clear();
            int64_t expiring = ev.timestamp + (int64_t)ms->retention_days * 24LL * 3600LL * 1000000000LL;
            for (uint32_t k = 0; k < a.reset_points_len; k++) {
              cdr_reset_point rp = b->rps[a.reset_points_off + k];
              uint32_t rpRun = (rp.flags & CDR_RP_HAS_RUN_ID) ? rp.run_id : 0;
              if (rpRun == a.continued_run_id) {
                rp.flags |= CDR_RP_HAS_EXPIRING;
                rp.expiring_time_nano = expiring;
              }
              ei.ResetPoints.push_back(rp);
            }
          } else {
            ei.HasResetPoints = false;
            ei.ResetPoints.clear();
          }
          if (a.flags & CDR_SF_HAS_MEMO) {
            ei.HasMemo = true;
            ei.Memo = a.memo;
          }
          if (a.flags & CDR_SF_HAS_SEARCH_ATTR) {
            ei.HasSearchAttr = a.search_attr_len > 0;  // GetIndexedFields() of an empty map
            ei.SearchAttributes.assign(b->kvs + a.search_attr_off, b->kvs + a.search_attr_off + a.search_attr_len);
          }
          ei.Started = true;
          // SetHistoryTree(execution.RunId) (:313-339)
          {
            uint64_t lo, hi;
            cdr_uuid(b->uuid_seed, ms->wf_key, CDR_UUID_BRANCH, ev.event_id, &lo, &hi);
            if (!ms->hasVH) {
              ei.HasBranchToken = true;
              ei.BranchTree = runID;
              ei.BranchLo = lo;
              ei.BranchHi = hi;
            } else {
              ms->vh.has_token = true;
              ms->vh.tree = runID;
              ms->vh.br_lo = lo;
              ms->vh.br_hi = hi;
            }
          }
          if (ms->hasRS) ms->rs.StartVersion = ev.version;  // :182-184
          {  // scheduleWorkflowTimerTask (:706-735) + RecordWorkflowStartedTask (:614-616)
            const int64_t backoff = (int64_t)a.first_decision_backoff_s * 1000000000LL;
            int64_t timeout = ev.timestamp + (int64_t)ei.WorkflowTimeout * 1000000000LL;
            if (backoff != 0) {
              timeout += backoff;
              ms->AddTimer(CDR_TT_WORKFLOW_BACKOFF, (a.flags & CDR_SF_CRON_INITIATOR) ? 1 : 0, 0,
                           ev.timestamp + backoff, 0);
            }
            ms->AddTimer(CDR_TT_WORKFLOW_TIMEOUT, 0, 0, timeout, 0);
            ms->AddXfer(CDR_TT_RECORD_STARTED, 0, 0, 0);
          }
          break;
        }
        case CDR_EV_DT_SCHEDULED: {  // :186-200 -> decision manager :143-167
          MutableState::DecisionInfo d{ev.version, ev.event_id, CDR_EMPTY_EVENT_ID, ctx->empty_uuid,
                                       ev.a.dt_sched.start_to_close_s, ev.a.dt_sched.attempt, 0,
                                       ev.timestamp, ev.timestamp};
          ms->UpdateDecision(d);
          ms->AddXfer(CDR_TT_DECISION, ev.event_id, domainID, ei.TaskList);  // :196-197
          ms->lastDecision = ms->snapDecision(CDR_LD_SCHEDULED, index_base + (int64_t)i);  // :200
          break;
        }
        case CDR_EV_DT_STARTED: {  // :202-213 -> :200-253
          int64_t scheduleID = ev.a.dt.scheduled_event_id;
          MutableState::DecisionInfo d = ms->getDecisionInfo();
          if (d.ScheduleID != scheduleID) return fail(CDR_E_DECISION_NOT_FOUND, i);
          d.Attempt = 0;
          if (ei.State == CDR_STATE_CREATED) {
            if (!UpdateWorkflowStateCloseStatus(ei, CDR_STATE_RUNNING, CDR_CLOSE_NONE))
              return fail(CDR_E_INVALID_STATE_TRANSITION, i);
          }
          MutableState::DecisionInfo nd{ev.version, scheduleID,   ev.event_id,          ev.a.dt.request_id,
                                        d.DecisionTimeout, d.Attempt, ev.timestamp, d.ScheduledTimestamp,
                                        d.OriginalScheduledTimestamp};
          ms->UpdateDecision(nd);
          // scheduleDecisionTimerTask (:210-211, timerBuilder.go:322-331)
          ms->AddTimer(CDR_TT_DECISION_TIMEOUT, CDR_TIMEOUT_START_TO_CLOSE, scheduleID,
                       ev.timestamp + (int64_t)nd.DecisionTimeout * 1000000000LL, nd.Attempt);
          ms->lastDecision = ms->snapDecision(CDR_LD_STARTED, index_base + (int64_t)i);  // :213
          break;
        }
        case CDR_EV_DT_COMPLETED: {  // :215-219 -> :255-262, :789-800
          ms->DeleteDecision();
          ei.LastProcessedEvent = ev.a.dt.started_event_id;
          // addBinaryCheckSumIfNotExists (mutableStateBuilder.go:1798-1842), maxResetPoints = MaxInt32
          uint32_t cks = ev.a.dt.binary_checksum;
          if (cks != 0) {
            bool exists = false;
            for (auto& rp : ei.ResetPoints) {
              uint32_t c = (rp.flags & CDR_RP_HAS_CHECKSUM) ? rp.binary_checksum : 0;
              if (c == cks) exists = true;
            }
            if (!exists) {
              bool resettable = ms->pendingChildExecutionInfoIDs.empty() &&
                                ms->pendingRequestCancelInfoIDs.empty() && ms->pendingSignalInfoIDs.empty();
              cdr_reset_point rp{};
              rp.binary_checksum = cks;
              rp.run_id = ei.RunID;
              rp.first_decision_completed_id = ev.event_id;
              rp.created_time_nano = b->now_ns;
              rp.flags = CDR_RP_HAS_CHECKSUM | CDR_RP_HAS_RUN_ID | CDR_RP_HAS_FIRST_DC_ID | CDR_RP_HAS_CREATED |
                         CDR_RP_HAS_RESETTABLE | (resettable ? CDR_RP_RESETTABLE : 0);
              ei.ResetPoints.push_back(rp);
              ei.HasResetPoints = true;
            }
          }
          break;
        }
        case CDR_EV_DT_TIMED_OUT:  // :221-239
          ms->FailDecision(ev.a.dt.timeout_type != CDR_TIMEOUT_SCHEDULE_TO_START);
          if (ms->ReplicateTransientDecisionTaskScheduled()) {
            ms->AddXfer(CDR_TT_DECISION, ei.DecisionScheduleID, domainID, ei.TaskList);  // :235-236
            ms->lastDecision = ms->snapDecision(CDR_LD_TRANSIENT, index_base + (int64_t)i);  // :238
          }
          break;
        case CDR_EV_DT_FAILED:  // :241-257
          ms->FailDecision(true);
          if (ms->ReplicateTransientDecisionTaskScheduled()) {
            ms->AddXfer(CDR_TT_DECISION, ei.DecisionScheduleID, domainID, ei.TaskList);  // :253-254
            ms->lastDecision = ms->snapDecision(CDR_LD_TRANSIENT, index_base + (int64_t)i);  // :256
          }
          break;
        case CDR_EV_AT_SCHEDULED: {  // :259-269 -> mutableStateBuilder.go:1982-2028
          const cdr_attr_at_scheduled& a = ev.a.at_sched;
          ActivityInfo ai{};
          ai.Version = ev.version;
          ai.ScheduleID = ev.event_id;
          ai.ScheduledEventBatchID = first.event_id;
          ai.ScheduledTime = ev.timestamp;
          ai.StartedID = CDR_EMPTY_EVENT_ID;
          ai.ActivityID = a.activity_id;
          ai.ScheduleToStartTimeout = a.s2s_s;
          ai.ScheduleToCloseTimeout = a.s2c_s;
          ai.StartToCloseTimeout = a.stc_s;
          ai.HeartbeatTimeout = a.hb_s;
          ai.CancelRequestID = CDR_EMPTY_EVENT_ID;
          ai.TimerTaskStatus = CDR_TIMER_TASK_STATUS_NONE;
          ai.TaskList = a.task_list;
          ai.HasRetryPolicy = (a.flags & CDR_AF_HAS_RETRY) != 0;
          ai.ExpirationSet = true;
          ai.ExpirationTime = ai.ScheduledTime + (int64_t)a.s2c_s * 1000000000LL;
          if (ai.HasRetryPolicy) {
            ai.InitialInterval = a.retry_initial_s;
            ai.BackoffCoefficient = a.backoff_coefficient;
            ai.MaximumInterval = a.retry_max_interval_s;
            ai.MaximumAttempts = a.retry_max_attempts;
            ai.NonRetriableErrors = a.nonretriable;
            if (a.retry_expiration_s > a.s2c_s)
              ai.ExpirationTime = ai.ScheduledTime + (int64_t)a.retry_expiration_s * 1000000000LL;
          }
          ms->pendingActivityInfoIDs[ai.ScheduleID] = ai;
          ms->pendingActivityInfoByActivityID[ai.ActivityID] = ai.ScheduleID;
          ms->AddXfer(CDR_TT_ACTIVITY, ai.ScheduleID, domainID, ei.TaskList);  // :265-266
          ms->ActivityTimerPick();
          break;
        }
        case CDR_EV_AT_STARTED: {  // :271-278 -> :2083-2098
          auto it = ms->pendingActivityInfoIDs.find(ev.a.at.scheduled_event_id);
          if (it == ms->pendingActivityInfoIDs.end()) return fail(CDR_P_ACTIVITY_STARTED_NIL, i);
          ActivityInfo& ai = it->second;
          ai.Version = ev.version;
          ai.StartedID = ev.event_id;
          ai.RequestID = ev.a.at.request_id;
          ai.StartedTimeSet = true;
          ai.StartedTime = ev.timestamp;
          ai.LastHeartBeatSet = true;
          ai.LastHeartBeatUpdatedTime = ev.timestamp;
          ms->ActivityTimerPick();
          break;
        }
        case CDR_EV_AT_COMPLETED:  // :280-305, :312-319
        case CDR_EV_AT_FAILED:
        case CDR_EV_AT_TIMED_OUT:
        case CDR_EV_AT_CANCELED: {
          int32_t c = ms->DeleteActivity(ev.a.at.scheduled_event_id);
          if (c != CDR_OK) return fail(c, i);
          ms->ActivityTimerPick();
          break;
        }
        case CDR_EV_AT_CANCEL_REQUESTED: {  // :307-310 -> :2264-2285
          auto jt = ms->pendingActivityInfoByActivityID.find(ev.a.at.activity_id);
          if (jt == ms->pendingActivityInfoByActivityID.end()) return fail(CDR_E_MISSING_ACTIVITY_INFO, i);
          auto it = ms->pendingActivityInfoIDs.find(jt->second);
          if (it == ms->pendingActivityInfoIDs.end()) return fail(CDR_E_MISSING_ACTIVITY_INFO, i);
          it->second.Version = ev.version;
          it->second.CancelRequested = true;
          it->second.CancelRequestID = ev.event_id;
          break;
        }
        case CDR_EV_AT_REQ_CANCEL_FAILED:  // :321-322
          break;
        case CDR_EV_TIMER_STARTED: {  // :324-332 -> :2877-2900
          TimerInfo ti{ev.version, ev.a.timer.timer_id, ev.event_id,
                       ev.timestamp + ev.a.timer.start_to_fire_s * 1000000000LL, CDR_TIMER_TASK_STATUS_NONE};
          ms->pendingTimerInfoIDs[ti.TimerID] = ti;
          ms->UserTimerPick();
          break;
        }
        case CDR_EV_TIMER_FIRED:     // :334-341 -> :2930-2939
        case CDR_EV_TIMER_CANCELED:  // :343-350 -> :2982-2991
          ms->pendingTimerInfoIDs.erase(ev.a.timer.timer_id);
          ms->UserTimerPick();
          break;
        case CDR_EV_CANCEL_TIMER_FAILED:  // :352-353
          break;
        case CDR_EV_CHILD_INITIATED: {  // :355-371 -> :3256-3280
          const cdr_attr_external& a = ev.a.ext;
          ChildInfo ci{};
          ci.Version = ev.version;
          ci.InitiatedID = ev.event_id;
          ci.InitiatedEventBatchID = first.event_id;
          ci.StartedID = CDR_EMPTY_EVENT_ID;
          ci.StartedWorkflowID = a.workflow_id;
          cdr_uuid(b->uuid_seed, ms->wf_key, CDR_UUID_CHILD_REQ, ev.event_id, &ci.CreateReqLo, &ci.CreateReqHi);
          ci.DomainName = a.domain;
          ci.WorkflowTypeName = a.workflow_type;
          ci.ParentClosePolicy = a.parent_close_policy;
          ms->pendingChildExecutionInfoIDs[ci.InitiatedID] = ci;
          if (a.flags & CDR_XF_DOMAIN_MISSING) return fail(CDR_E_DOMAIN_NOT_FOUND, i);  // :365-368
          {  // scheduleStartChildWorkflowTransferTask (:370-371)
            cdr_task t{};
            t.type = CDR_TT_START_CHILD;
            t.event_id = ci.InitiatedID;
            t.domain_id = a.target_domain_id;
            t.target_workflow_id = a.workflow_id;
            ms->transferTasks.push_back(t);
          }
          break;
        }
        case CDR_EV_CHILD_START_FAILED:  // :373-376
        case CDR_EV_CHILD_COMPLETED:     // :383-406
        case CDR_EV_CHILD_FAILED:
        case CDR_EV_CHILD_CANCELED:
        case CDR_EV_CHILD_TIMED_OUT:
        case CDR_EV_CHILD_TERMINATED:
          ms->pendingChildExecutionInfoIDs.erase(ev.a.ref.initiated_event_id);  // DeletePendingChildExecution
          break;
        case CDR_EV_CHILD_STARTED: {  // :378-381 -> :3312-3325
          auto it = ms->pendingChildExecutionInfoIDs.find(ev.a.ref.initiated_event_id);
          if (it == ms->pendingChildExecutionInfoIDs.end()) return fail(CDR_P_CHILD_STARTED_NIL, i);
          it->second.StartedID = ev.event_id;
          it->second.StartedRunID = ev.a.ref.run_id;
          break;
        }
        case CDR_EV_RCE_INITIATED: {  // :408-427 -> :2577-2596
          CancelInfo rci{};
          rci.Version = ev.version;
          rci.InitiatedEventBatchID = first.event_id;
          rci.InitiatedID = ev.event_id;
          cdr_uuid(b->uuid_seed, ms->wf_key, CDR_UUID_CANCEL_REQ, ev.event_id, &rci.ReqLo, &rci.ReqHi);
          ms->pendingRequestCancelInfoIDs[rci.InitiatedID] = rci;
          if (ev.a.ext.flags & CDR_XF_DOMAIN_MISSING) return fail(CDR_E_DOMAIN_NOT_FOUND, i);
          {  // scheduleCancelExternalWorkflowTransferTask (:421-427)
            cdr_task t{};
            t.type = CDR_TT_CANCEL_EXECUTION;
            t.event_id = rci.InitiatedID;
            t.domain_id = ev.a.ext.target_domain_id;
            t.target_workflow_id = ev.a.ext.workflow_id;
            t.target_run_id = ev.a.ext.run_id;
            t.flags = (ev.a.ext.flags & CDR_XF_CHILD_ONLY) ? CDR_TF_CHILD_ONLY : 0u;
            ms->transferTasks.push_back(t);
          }
          break;
        }
        case CDR_EV_RCE_FAILED:            // :429-432
        case CDR_EV_EXT_CANCEL_REQUESTED:  // :434-437
          ms->pendingRequestCancelInfoIDs.erase(ev.a.ref.initiated_event_id);
          break;
        case CDR_EV_SE_INITIATED: {  // :439-458 -> :2701-2723
          const cdr_attr_external& a = ev.a.ext;
          SignalInfo si{};
          si.Version = ev.version;
          si.InitiatedEventBatchID = first.event_id;
          si.InitiatedID = ev.event_id;
          cdr_uuid(b->uuid_seed, ms->wf_key, CDR_UUID_SIGNAL_REQ, ev.event_id, &si.ReqLo, &si.ReqHi);
          si.SignalName = a.signal_name;
          si.Input = a.input;
          si.Control = a.control;
          ms->pendingSignalInfoIDs[si.InitiatedID] = si;
          if (a.flags & CDR_XF_DOMAIN_MISSING) return fail(CDR_E_DOMAIN_NOT_FOUND, i);
          {  // scheduleSignalWorkflowTransferTask (:452-458)
            cdr_task t{};
            t.type = CDR_TT_SIGNAL_EXECUTION;
            t.event_id = si.InitiatedID;
            t.domain_id = a.target_domain_id;
            t.target_workflow_id = a.workflow_id;
            t.target_run_id = a.run_id;
            t.flags = (a.flags & CDR_XF_CHILD_ONLY) ? CDR_TF_CHILD_ONLY : 0u;
            ms->transferTasks.push_back(t);
          }
          break;
        }
        case CDR_EV_SE_FAILED:    // :460-463
        case CDR_EV_EXT_SIGNALED:  // :465-468
          ms->pendingSignalInfoIDs.erase(ev.a.ref.initiated_event_id);
          break;
        case CDR_EV_MARKER_RECORDED:  // :470-471
          break;
        case CDR_EV_WF_SIGNALED:  // :473-476 -> :3082-3089
          ei.SignalCount++;
          break;
        case CDR_EV_WF_CANCEL_REQUESTED:  // :478-481 -> :2504-2510
          ei.CancelRequested = true;
          break;
        case CDR_EV_WF_COMPLETED:   // :483-491 -> :2379-2394
        case CDR_EV_WF_FAILED:      // :493-501 -> :2419-2434
        case CDR_EV_WF_TIMED_OUT:   // :503-511 -> :2456-2471
        case CDR_EV_WF_CANCELED:    // :513-521 -> :2535-2549
        case CDR_EV_WF_TERMINATED: {  // :523-531 -> :3047-3062
          int cs = ev.type == CDR_EV_WF_COMPLETED   ? CDR_CLOSE_COMPLETED
                   : ev.type == CDR_EV_WF_FAILED    ? CDR_CLOSE_FAILED
                   : ev.type == CDR_EV_WF_TIMED_OUT ? CDR_CLOSE_TIMED_OUT
                   : ev.type == CDR_EV_WF_CANCELED  ? CDR_CLOSE_CANCELED
                                                    : CDR_CLOSE_TERMINATED;
          if (!UpdateWorkflowStateCloseStatus(ei, CDR_STATE_COMPLETED, cs))
            return fail(CDR_E_INVALID_STATE_TRANSITION, i);
          ei.CompletionEventBatchID = first.event_id;
          ms->ClearStickyness();
          ms->AppendTasksForFinishedExecution(ev.timestamp);  // :757-787
          break;
        }
        case CDR_EV_UPSERT_SA: {  // :533-535 -> :2746-2768
          const cdr_attr_upsert& a = ev.a.upsert;
          for (uint32_t k = 0; k < a.search_attr_len; k++) {
            cdr_kv kv = b->kvs[a.search_attr_off + k];
            bool found = false;
            for (auto& cur : ei.SearchAttributes)
              if (cur.key == kv.key) {
                cur.value = kv.value;
                found = true;
              }
            if (!found) ei.SearchAttributes.push_back(kv);
          }
          ei.HasSearchAttr = true;  // mergeMapOfByteArray makes a map if nil
          ms->AddXfer(CDR_TT_UPSERT_SA, 0, 0, 0);  // :535
          break;
        }
        case CDR_EV_WF_CONTINUED_AS_NEW: {  // :537-595
          if (n_newrun == 0) return fail(CDR_E_NEWRUN_HISTORY_EMPTY, i);
          MutableState* nms = new MutableState(ctx, newRunNDC ? CDR_BUILDER_NDC : CDR_BUILDER_2DC,
                                               ms->failover_at_ctor, newrun_key, ms->retention_days);
          StateBuilder nsb{ctx, b, nms};
          uint32_t newRunID = ev.a.can.new_execution_run_id;
          GoErr ne = nsb.applyEvents(newrun_request, workflowID, newRunID, domainID, newRunHistory, n_newrun, 0,
                                     nullptr, 0, false, 0, 0, nullptr, nullptr);
          if (!ne.ok()) {
            if (newRunErr) *newRunErr = ne;
            delete nms;
            GoErr pe = ne;
            pe.flags |= CDR_RF_IN_NEWRUN;
            return pe;
          }
          if (newRunErr) *newRunErr = ne;
          if (newRun) {
            delete *newRun;
            *newRun = nms;
          } else {
            delete nms;
          }
          // ReplicateWorkflowExecutionContinuedAsNewEvent (:3207-3224)
          if (!UpdateWorkflowStateCloseStatus(ei, CDR_STATE_COMPLETED, CDR_CLOSE_CONTINUED_AS_NEW))
            return fail(CDR_E_INVALID_STATE_TRANSITION, i);
          ei.CompletionEventBatchID = first.event_id;
          ms->ClearStickyness();
          ms->AppendTasksForFinishedExecution(ev.timestamp);  // :592
          break;
        }
        default:
          return fail(CDR_E_UNKNOWN_EVENT_TYPE, i);  // :597-599
      }
    }
    ms->ei.LastFirstEventID = first.event_id;  // :603
    ms->ei.NextEventID = last.event_id + 1;    // :604
    return err;
  }
};

}  // namespace


// ------------------------------------------------------------------ writer
namespace {

template <class T, class K>
static void sorted_values(const std::map<K, T>& m, std::vector<T>& out) {
  out.clear();
  for (auto& kv : m) out.push_back(kv.second);
}

bool write_state(const MutableState& ms, const cdr_batch* b, uint32_t w, const cdr_wf_caps* caps, cdr_out* out) {
  (void)b;
  if (out->last_decision) out->last_decision[w] = ms.lastDecision;
  const ExecutionInfo& ei = ms.ei;
  const cdr_wf_caps& cp = caps[w];
  cdr_wf_result& r = out->result[w];
  cdr_exec_info x{};
  x.domain_id = ei.DomainID;
  x.workflow_id = ei.WorkflowID;
  x.run_id = ei.RunID;
  x.create_request_id = ei.CreateRequestID;
  x.parent_domain_id = ei.ParentDomainID;
  x.parent_workflow_id = ei.ParentWorkflowID;
  x.parent_run_id = ei.ParentRunID;
  x.task_list = ei.TaskList;
  x.workflow_type = ei.WorkflowTypeName;
  x.decision_request_id = ei.DecisionRequestID;
  x.cron_schedule = ei.CronSchedule;
  x.memo = ei.HasMemo ? ei.Memo : 0;
  x.nonretriable = ei.NonRetriableErrors;
  x.initiated_id = ei.InitiatedID;
  x.completion_event_batch_id = ei.CompletionEventBatchID;
  x.workflow_timeout = ei.WorkflowTimeout;
  x.decision_timeout_value = ei.DecisionTimeoutValue;
  x.state = ei.State;
  x.close_status = ei.CloseStatus;
  x.last_first_event_id = ei.LastFirstEventID;
  x.last_event_task_id = ei.LastEventTaskID;
  x.next_event_id = ei.NextEventID;
  x.last_processed_event = ei.LastProcessedEvent;
  x.signal_count = ei.SignalCount;
  x.decision_timeout = ei.DecisionTimeout;
  x.decision_version = ei.DecisionVersion;
  x.decision_schedule_id = ei.DecisionScheduleID;
  x.decision_started_id = ei.DecisionStartedID;
  x.decision_attempt = ei.DecisionAttempt;
  x.decision_started_ts = ei.DecisionStartedTimestamp;
  x.decision_scheduled_ts = ei.DecisionScheduledTimestamp;
  x.decision_original_scheduled_ts = ei.DecisionOriginalScheduledTimestamp;
  x.attempt = ei.Attempt;
  x.initial_interval = ei.InitialInterval;
  x.backoff_coefficient = ei.BackoffCoefficient;
  x.maximum_interval = ei.MaximumInterval;
  x.maximum_attempts = ei.MaximumAttempts;
  x.expiration_time = ei.ExpirationSet ? ei.ExpirationTime : 0;
  x.expiration_seconds = ei.ExpirationSeconds;
  uint32_t f = 0;
  if (ei.CancelRequested) f |= CDR_XI_CANCEL_REQUESTED;
  if (ei.HasRetryPolicy) f |= CDR_XI_HAS_RETRY;
  if (ei.ExpirationSet) f |= CDR_XI_HAS_EXPIRATION;
  if (ei.HasMemo) f |= CDR_XI_HAS_MEMO;
  if (ei.HasSearchAttr) f |= CDR_XI_HAS_SEARCH_ATTR;
  if (ei.HasResetPoints) f |= CDR_XI_HAS_RESET_POINTS;
  if (ei.Started) f |= CDR_XI_STARTED;
  if (ei.HasBranchToken) {
    f |= CDR_XI_HAS_BRANCH;
    x.branch_tree_id = ei.BranchTree;
    x.branch_id_lo = ei.BranchLo;
    x.branch_id_hi = ei.BranchHi;
  } else if (ms.hasVH && ms.vh.has_token) {
    f |= CDR_XI_VH_BRANCH;
    x.branch_tree_id = ms.vh.tree;
    x.branch_id_lo = ms.vh.br_lo;
    x.branch_id_hi = ms.vh.br_hi;
  }
  x.flags = f;

  // tables (pending maps in ascending key order; SearchAttributes sorted by key)
  std::vector<cdr_kv> sa = ei.SearchAttributes;
  std::stable_sort(sa.begin(), sa.end(), [](const cdr_kv& a, const cdr_kv& c) { return a.key < c.key; });
  x.reset_points_len = (uint32_t)ei.ResetPoints.size();
  x.search_attr_len = (uint32_t)sa.size();
  out->exec[w] = x;

  cdr_repl_state rs{};
  if (ms.hasRS) {
    rs.present = 1;
    rs.current_version = ms.rs.CurrentVersion;
    rs.start_version = ms.rs.StartVersion;
    rs.last_write_version = ms.rs.LastWriteVersion;
    rs.last_write_event_id = ms.rs.LastWriteEventID;
    for (auto& kv : ms.rs.LastReplicationInfo) {
      rs.lri_mask |= 1u << kv.first;
      rs.lri_version[kv.first] = kv.second.first;
      rs.lri_last_event_id[kv.first] = kv.second.second;
    }
  }
  out->repl[w] = rs;

  if (ms.vh.items.size() > cp.vh_cap || ms.pendingActivityInfoIDs.size() > cp.act_cap ||
      ms.pendingTimerInfoIDs.size() > cp.timer_cap || ms.pendingChildExecutionInfoIDs.size() > cp.child_cap ||
      ms.pendingRequestCancelInfoIDs.size() > cp.cancel_cap || ms.pendingSignalInfoIDs.size() > cp.signal_cap ||
      ei.ResetPoints.size() > cp.rp_cap || sa.size() > cp.sa_cap)
    return false;

  r.n_vh = (uint32_t)ms.vh.items.size();
  for (size_t k = 0; k < ms.vh.items.size(); k++)
    out->vh[cp.vh_off + k] = cdr_vh_item{ms.vh.items[k].eventID, ms.vh.items[k].version};

  uint32_t k = 0;
  for (auto& kv : ms.pendingActivityInfoIDs) {
    const ActivityInfo& a = kv.second;
    cdr_activity_info o{};
    o.version = a.Version;
    o.schedule_id = a.ScheduleID;
    o.scheduled_event_batch_id = a.ScheduledEventBatchID;
    o.scheduled_time = a.ScheduledTime;
    o.started_id = a.StartedID;
    o.started_time = a.StartedTimeSet ? a.StartedTime : 0;
    o.last_heartbeat_time = a.LastHeartBeatSet ? a.LastHeartBeatUpdatedTime : 0;
    o.expiration_time = a.ExpirationTime;
    o.cancel_request_id = a.CancelRequestID;
    o.activity_id = a.ActivityID;
    o.request_id = a.RequestID;
    o.task_list = a.TaskList;
    o.nonretriable = a.NonRetriableErrors;
    o.s2s = a.ScheduleToStartTimeout;
    o.s2c = a.ScheduleToCloseTimeout;
    o.stc = a.StartToCloseTimeout;
    o.hb = a.HeartbeatTimeout;
    o.timer_task_status = a.TimerTaskStatus;
    o.attempt = a.Attempt;
    o.initial_interval = a.InitialInterval;
    o.maximum_interval = a.MaximumInterval;
    o.maximum_attempts = a.MaximumAttempts;
    o.backoff_coefficient = a.BackoffCoefficient;
    o.flags = (a.CancelRequested ? CDR_AI_CANCEL_REQUESTED : 0) | (a.HasRetryPolicy ? CDR_AI_HAS_RETRY : 0) |
              (a.StartedTimeSet ? CDR_AI_STARTED_TIME_SET : 0);
    out->act[cp.act_off + k++] = o;
  }
  r.n_activity = k;
  k = 0;
  for (auto& kv : ms.pendingTimerInfoIDs) {
    const TimerInfo& t = kv.second;
    out->timer[cp.timer_off + k++] = cdr_timer_info{t.Version, t.StartedID, t.ExpiryTime, t.TaskID, t.TimerID, 0};
  }
  r.n_timer = k;
  k = 0;
  for (auto& kv : ms.pendingChildExecutionInfoIDs) {
    const ChildInfo& c = kv.second;
    cdr_child_info o{};
    o.version = c.Version;
    o.initiated_id = c.InitiatedID;
    o.initiated_event_batch_id = c.InitiatedEventBatchID;
    o.started_id = c.StartedID;
    o.create_request_lo = c.CreateReqLo;
    o.create_request_hi = c.CreateReqHi;
    o.started_workflow_id = c.StartedWorkflowID;
    o.started_run_id = c.StartedRunID;
    o.domain_name = c.DomainName;
    o.workflow_type = c.WorkflowTypeName;
    o.parent_close_policy = c.ParentClosePolicy;
    out->child[cp.child_off + k++] = o;
  }
  r.n_child = k;
  k = 0;
  for (auto& kv : ms.pendingRequestCancelInfoIDs) {
    const CancelInfo& c = kv.second;
    out->cancel[cp.cancel_off + k++] = cdr_cancel_info{c.Version, c.InitiatedEventBatchID, c.InitiatedID, c.ReqLo, c.ReqHi};
  }
  r.n_cancel = k;
  k = 0;
  for (auto& kv : ms.pendingSignalInfoIDs) {
    const SignalInfo& s = kv.second;
    cdr_signal_info o{};
    o.version = s.Version;
    o.initiated_event_batch_id = s.InitiatedEventBatchID;
    o.initiated_id = s.InitiatedID;
    o.signal_request_lo = s.ReqLo;
    o.signal_request_hi = s.ReqHi;
    o.signal_name = s.SignalName;
    o.input = s.Input;
    o.control = s.Control;
    out->signal[cp.signal_off + k++] = o;
  }
  r.n_signal = k;
  for (size_t j = 0; j < ei.ResetPoints.size(); j++) out->rp[cp.rp_off + j] = ei.ResetPoints[j];
  r.n_reset_points = (uint32_t)ei.ResetPoints.size();
  for (size_t j = 0; j < sa.size(); j++) out->sa[cp.sa_off + j] = sa[j];
  r.n_search_attr = (uint32_t)sa.size();
  if (out->transfer) {
    if (ms.transferTasks.size() > cp.xfer_cap || ms.timerTasks.size() > cp.ttask_cap) return false;
    for (size_t j = 0; j < ms.transferTasks.size(); j++) out->transfer[cp.xfer_off + j] = ms.transferTasks[j];
    for (size_t j = 0; j < ms.timerTasks.size(); j++) out->timer_tasks[cp.ttask_off + j] = ms.timerTasks[j];
    out->n_tasks[2 * w] = (uint32_t)ms.transferTasks.size();
    out->n_tasks[2 * w + 1] = (uint32_t)ms.timerTasks.size();
  }
  return true;
}

// mutableStateBuilder.Load (mutableStateBuilder.go:272-295) from the persisted records
// of an earlier replay (cdr_carry): the inverse of write_state, plus Load's own
// effects — byActivityID rebuilt from the activity rows (ascending scheduleID, so the
// last duplicate activityID wins) and currentVersion = EmptyVersion
void load_state(MutableState& ms, const cdr_carry& cy, uint32_t src) {
  const cdr_exec_info& x = cy.state.exec[src];
  const cdr_wf_result& r = cy.state.result[src];
  const cdr_wf_caps& cp = cy.caps[src];
  ExecutionInfo& ei = ms.ei;
  ei.DomainID = x.domain_id;
  ei.WorkflowID = x.workflow_id;
  ei.RunID = x.run_id;
  ei.CreateRequestID = x.create_request_id;
  ei.ParentDomainID = x.parent_domain_id;
  ei.ParentWorkflowID = x.parent_workflow_id;
  ei.ParentRunID = x.parent_run_id;
  ei.TaskList = x.task_list;
  ei.WorkflowTypeName = x.workflow_type;
  ei.DecisionRequestID = x.decision_request_id;
  ei.CronSchedule = x.cron_schedule;
  ei.HasMemo = (x.flags & CDR_XI_HAS_MEMO) != 0;
  ei.Memo = x.memo;
  ei.NonRetriableErrors = x.nonretriable;
  ei.InitiatedID = x.initiated_id;
  ei.CompletionEventBatchID = x.completion_event_batch_id;
  ei.WorkflowTimeout = x.workflow_timeout;
  ei.DecisionTimeoutValue = x.decision_timeout_value;
  ei.State = x.state;
  ei.CloseStatus = x.close_status;
  ei.LastFirstEventID = x.last_first_event_id;
  ei.LastEventTaskID = x.last_event_task_id;
  ei.NextEventID = x.next_event_id;
  ei.LastProcessedEvent = x.last_processed_event;
  ei.SignalCount = x.signal_count;
  ei.DecisionTimeout = x.decision_timeout;
  ei.DecisionVersion = x.decision_version;
  ei.DecisionScheduleID = x.decision_schedule_id;
  ei.DecisionStartedID = x.decision_started_id;
  ei.DecisionAttempt = x.decision_attempt;
  ei.DecisionStartedTimestamp = x.decision_started_ts;
  ei.DecisionScheduledTimestamp = x.decision_scheduled_ts;
  ei.DecisionOriginalScheduledTimestamp = x.decision_original_scheduled_ts;
  ei.Attempt = x.attempt;
  ei.InitialInterval = x.initial_interval;
  ei.BackoffCoefficient = x.backoff_coefficient;
  ei.MaximumInterval = x.maximum_interval;
  ei.MaximumAttempts = x.maximum_attempts;
  ei.ExpirationSet = (x.flags & CDR_XI_HAS_EXPIRATION) != 0;
  ei.ExpirationTime = x.expiration_time;
  ei.ExpirationSeconds = x.expiration_seconds;
  ei.CancelRequested = (x.flags & CDR_XI_CANCEL_REQUESTED) != 0;
  ei.HasRetryPolicy = (x.flags & CDR_XI_HAS_RETRY) != 0;
  ei.HasSearchAttr = (x.flags & CDR_XI_HAS_SEARCH_ATTR) != 0;
  ei.HasResetPoints = (x.flags & CDR_XI_HAS_RESET_POINTS) != 0;
  ei.Started = (x.flags & CDR_XI_STARTED) != 0;
  ei.HasBranchToken = (x.flags & CDR_XI_HAS_BRANCH) != 0;
  if (ei.HasBranchToken) {
    ei.BranchTree = x.branch_tree_id;
    ei.BranchLo = x.branch_id_lo;
    ei.BranchHi = x.branch_id_hi;
  }
  ei.ResetPoints.assign(cy.state.rp + cp.rp_off, cy.state.rp + cp.rp_off + r.n_reset_points);
  ei.SearchAttributes.assign(cy.state.sa + cp.sa_off, cy.state.sa + cp.sa_off + r.n_search_attr);
  if (ms.hasRS) {
    const cdr_repl_state& rs = cy.state.repl[src];
    ms.rs.CurrentVersion = rs.current_version;
    ms.rs.StartVersion = rs.start_version;
    ms.rs.LastWriteVersion = rs.last_write_version;
    ms.rs.LastWriteEventID = rs.last_write_event_id;
    ms.rs.LastReplicationInfo.clear();
    for (int c = 0; c < CDR_MAX_CLUSTERS; c++)
      if (rs.lri_mask & (1u << c)) ms.rs.LastReplicationInfo[c] = {rs.lri_version[c], rs.lri_last_event_id[c]};
  }
  if (ms.hasVH) {
    ms.vh.items.clear();
    for (uint32_t k = 0; k < r.n_vh; k++) {
      const cdr_vh_item& it = cy.state.vh[cp.vh_off + k];
      ms.vh.items.push_back({it.event_id, it.version});
    }
    ms.vh.has_token = (x.flags & CDR_XI_VH_BRANCH) != 0;
    if (ms.vh.has_token) {
      ms.vh.tree = x.branch_tree_id;
      ms.vh.br_lo = x.branch_id_lo;
      ms.vh.br_hi = x.branch_id_hi;
    }
  }
  ms.currentVersion = CDR_EMPTY_VERSION;  // :291
  for (uint32_t k = 0; k < r.n_activity; k++) {
    const cdr_activity_info& o = cy.state.act[cp.act_off + k];
    ActivityInfo a{};
    a.Version = o.version;
    a.ScheduleID = o.schedule_id;
    a.ScheduledEventBatchID = o.scheduled_event_batch_id;
    a.ScheduledTime = o.scheduled_time;
    a.StartedID = o.started_id;
    a.StartedTimeSet = (o.flags & CDR_AI_STARTED_TIME_SET) != 0;
    a.StartedTime = o.started_time;
    a.LastHeartBeatSet = (o.flags & CDR_AI_STARTED_TIME_SET) != 0;
    a.LastHeartBeatUpdatedTime = o.last_heartbeat_time;
    a.ExpirationSet = true;
    a.ExpirationTime = o.expiration_time;
    a.CancelRequestID = o.cancel_request_id;
    a.CancelRequested = (o.flags & CDR_AI_CANCEL_REQUESTED) != 0;
    a.ActivityID = o.activity_id;
    a.RequestID = o.request_id;
    a.TaskList = o.task_list;
    a.NonRetriableErrors = o.nonretriable;
    a.ScheduleToStartTimeout = o.s2s;
    a.ScheduleToCloseTimeout = o.s2c;
    a.StartToCloseTimeout = o.stc;
    a.HeartbeatTimeout = o.hb;
    a.TimerTaskStatus = o.timer_task_status;
    a.Attempt = o.attempt;
    a.HasRetryPolicy = (o.flags & CDR_AI_HAS_RETRY) != 0;
    a.InitialInterval = o.initial_interval;
    a.MaximumInterval = o.maximum_interval;
    a.MaximumAttempts = o.maximum_attempts;
    a.BackoffCoefficient = o.backoff_coefficient;
    ms.pendingActivityInfoIDs[a.ScheduleID] = a;
  }
  for (auto& kv : ms.pendingActivityInfoIDs) ms.pendingActivityInfoByActivityID[kv.second.ActivityID] = kv.first;
  for (uint32_t k = 0; k < r.n_timer; k++) {
    const cdr_timer_info& o = cy.state.timer[cp.timer_off + k];
    ms.pendingTimerInfoIDs[o.timer_id] = TimerInfo{o.version, o.timer_id, o.started_id, o.expiry_time, o.task_id};
  }
  for (uint32_t k = 0; k < r.n_child; k++) {
    const cdr_child_info& o = cy.state.child[cp.child_off + k];
    ChildInfo c{};
    c.Version = o.version;
    c.InitiatedID = o.initiated_id;
    c.InitiatedEventBatchID = o.initiated_event_batch_id;
    c.StartedID = o.started_id;
    c.StartedWorkflowID = o.started_workflow_id;
    c.StartedRunID = o.started_run_id;
    c.CreateReqLo = o.create_request_lo;
    c.CreateReqHi = o.create_request_hi;
    c.DomainName = o.domain_name;
    c.WorkflowTypeName = o.workflow_type;
    c.ParentClosePolicy = o.parent_close_policy;
    ms.pendingChildExecutionInfoIDs[c.InitiatedID] = c;
  }
  for (uint32_t k = 0; k < r.n_cancel; k++) {
    const cdr_cancel_info& o = cy.state.cancel[cp.cancel_off + k];
    ms.pendingRequestCancelInfoIDs[o.initiated_id] =
        CancelInfo{o.version, o.initiated_event_batch_id, o.initiated_id, o.cancel_request_lo, o.cancel_request_hi};
  }
  for (uint32_t k = 0; k < r.n_signal; k++) {
    const cdr_signal_info& o = cy.state.signal[cp.signal_off + k];
    ms.pendingSignalInfoIDs[o.initiated_id] =
        SignalInfo{o.version,         o.initiated_event_batch_id, o.initiated_id, o.signal_request_lo,
                   o.signal_request_hi, o.signal_name,             o.input,        o.control};
  }
}

void replay_one(const cdr_batch* b, const Ctx* ctx, uint32_t w, const cdr_wf_caps* caps, cdr_out* out) {
  const cdr_wf_desc& d = b->wfs[w];
  cdr_wf_result& r = out->result[w];
  r = cdr_wf_result{};
  MutableState ms(ctx, (int)d.builder, d.failover_version, d.wf_key, d.retention_days);
  if (b->carry && b->carry->src && b->carry->src[w] >= 0) {
    load_state(ms, *b->carry, (uint32_t)b->carry->src[w]);
    // cdr_carry.in_memory: the builder was never Loaded (nDCConflictResolver.rebuild's
    // result): its currentVersion is what its replay left — see cdro_ndc_replicate_round,
    // which keeps the rebuilt MutableState itself and checks this shortcut against it
    if (b->carry->in_memory && b->carry->in_memory[w] && ms.hasVH && !ms.vh.items.empty())
      ms.currentVersion = ms.vh.items.back().version;
  }
  StateBuilder sb{ctx, b, &ms};
  const cdr_event* ev = b->events + d.ev_off;
  const cdr_event* nr = nullptr;
  size_t n_nr = 0;
  const cdr_wf_desc* nd = nullptr;
  if (d.newrun >= 0) {
    nd = &b->wfs[d.newrun];
    nr = b->events + nd->ev_off;
    n_nr = nd->ev_len;
  }
  MutableState* newRun = nullptr;
  GoErr newRunErr;
  bool newRunAttempted = false;
  GoErr err;
  if (d.ev_len == 0) {
    err.code = CDR_E_HISTORY_EMPTY;
  }
  uint32_t call = 0;
  for (uint64_t s = 0; s < d.ev_len && err.ok();) {
    uint64_t e = s + 1;
    while (e < d.ev_len && !(ev[e].flags & CDR_EVF_BATCH_FIRST)) e++;
    bool thisCall = nd && call == d.newrun_call;
    GoErr ne;
    ne.code = -1;
    err = sb.applyEvents(d.request_id, d.workflow_id, d.run_id, d.domain_id, ev + s, (size_t)(e - s), (int64_t)s,
                         thisCall ? nr : nullptr, thisCall ? n_nr : 0, thisCall && d.newrun_ndc,
                         nd ? nd->wf_key : 0, nd ? nd->request_id : 0, &newRun, &ne);
    if (ne.code != -1) {
      newRunAttempted = true;
      newRunErr = ne;
    }
    s = e;
    call++;
  }
  if (err.ok() && d.expected_next_event_id != 0 && ms.ei.NextEventID != d.expected_next_event_id) {
    err.code = CDR_E_REBUILD_NEXT_EVENT_ID;  // nDCStateRebuilder.go:139-143
    err.event_id = d.ev_len ? ev[d.ev_len - 1].event_id : 0;
    err.index = (int64_t)d.ev_len;
  }
  r.code = err.code;
  r.flags = err.flags | (newRunAttempted ? CDR_RF_NEWRUN_APPLIED : 0);
  r.fail_event_id = err.event_id;
  r.fail_index = err.index;
  if (err.ok()) {
    if (!write_state(ms, b, w, caps, out)) {
      r.code = CDR_E_BAD_INPUT;
    }
  }
  if (nd) {
    cdr_wf_result& nrr = out->result[d.newrun];
    nrr = cdr_wf_result{};
    nrr.flags = CDR_RF_IS_NEWRUN;
    if (!newRunAttempted) {
      nrr.code = CDR_NOT_APPLIED;
    } else if (!newRunErr.ok()) {
      nrr.code = newRunErr.code;
      nrr.fail_event_id = newRunErr.event_id;
      nrr.fail_index = newRunErr.index;
    } else if (newRun) {
      if (!write_state(*newRun, b, (uint32_t)d.newrun, caps, out)) nrr.code = CDR_E_BAD_INPUT;
      nrr.flags = CDR_RF_IS_NEWRUN;
    }
  }
  delete newRun;
}

}  // namespace

extern "C" {

// Replays every top-level entry of `b` (new-run entries are reached through their
// parent's continue-as-new event, as in stateBuilder.go:557-571).
// threads <= 1: single-threaded; otherwise one task per workflow on a pool
// (the analogue of the reference's goroutine-per-workflow).
int cdro_replay_batch(const cdr_batch* b, const cdr_wf_caps* caps, cdr_out* out, int threads) {
  Ctx ctx{b, b->empty_uuid};
  if (threads <= 1) {
    for (uint32_t w = 0; w < b->n_wfs; w++)
      if (b->wfs[w].parent < 0) replay_one(b, &ctx, w, caps, out);
    return 0;
  }
  std::atomic<uint32_t> next{0};
  std::vector<std::thread> pool;
  auto work = [&] {
    for (;;) {
      uint32_t w0 = next.fetch_add(64);
      if (w0 >= b->n_wfs) break;
      uint32_t w1 = std::min(b->n_wfs, w0 + 64);
      for (uint32_t w = w0; w < w1; w++)
        if (b->wfs[w].parent < 0) replay_one(b, &ctx, w, caps, out);
    }
  };
  for (int t = 1; t < threads; t++) {
    try {
      pool.emplace_back(work);
    } catch (const std::system_error&) {
      break;
    }
  }
  work();
  for (auto& th : pool) th.join();
  return 0;
}

// --- unit-test entry points restating the reference's own known-answer tests ---

// versionHistory.AddOrUpdateItem on a list of items (in/out), returns status.
int cdro_vh_add_or_update(cdr_vh_item* items, uint32_t* n, uint32_t cap, int64_t event_id, int64_t version) {
  VersionHistory v;
  for (uint32_t k = 0; k < *n; k++) v.items.push_back({items[k].event_id, items[k].version});
  int32_t c = v.AddOrUpdateItem(event_id, version);
  if (c != CDR_OK) return c;
  if (v.items.size() > cap) return CDR_E_BAD_INPUT;
  *n = (uint32_t)v.items.size();
  for (uint32_t k = 0; k < *n; k++) items[k] = cdr_vh_item{v.items[k].eventID, v.items[k].version};
  return CDR_OK;
}

// WorkflowExecutionInfo.UpdateWorkflowStateCloseStatus: 1 = accepted, 0 = rejected.
// ---- NDC replication round (nDCHistoryReplicator.applyNonStartEvents,
// nDCHistoryReplicator.go:246-470), restated per workflow with the rebuilt mutable state
// KEPT IN MEMORY between nDCStateRebuilder.rebuild (nDCStateRebuilder.go:92-160) and
// applyNonStartEventsToCurrentBranch (:330-398), as nDCConflictResolver.rebuild
// (nDCConflictResolver.go:117-184) hands it over — the parity checker of
// cdr_ndc_replicate_async, which continues from the rebuilt records instead.
int cdro_ndc_branch(const cdr_ndc_task* tasks, const cdr_vh_item* task_items, uint32_t n, cdr_vhs* vhs,
                    cdr_vh_item* pool, cdr_ndc_decision* dec);  // ndc_ref.cpp
int cdro_refresh_one(const cdr_batch* b, const cdr_wf_caps* caps, cdr_out* out, int64_t now_ns, uint32_t flags,
                     uint32_t w);  // refresh_ref.cpp

static void copy_state(const cdr_out& src, const cdr_wf_caps& sc, cdr_out& dst, const cdr_wf_caps& dc, uint32_t w) {
  const cdr_wf_result r = src.result[w];
  dst.exec[w] = src.exec[w];
  dst.repl[w] = src.repl[w];
  dst.result[w] = r;
  if (r.code != CDR_OK) return;
  auto cp = [&](auto* s, auto* d, uint64_t so, uint64_t doff, uint32_t n, uint32_t cap) {
    if (n > cap) {
      dst.result[w].code = CDR_E_BAD_INPUT;
      return;
    }
    for (uint32_t i = 0; i < n; i++) d[doff + i] = s[so + i];
  };
  cp(src.act, dst.act, sc.act_off, dc.act_off, r.n_activity, dc.act_cap);
  cp(src.timer, dst.timer, sc.timer_off, dc.timer_off, r.n_timer, dc.timer_cap);
  cp(src.child, dst.child, sc.child_off, dc.child_off, r.n_child, dc.child_cap);
  cp(src.cancel, dst.cancel, sc.cancel_off, dc.cancel_off, r.n_cancel, dc.cancel_cap);
  cp(src.signal, dst.signal, sc.signal_off, dc.signal_off, r.n_signal, dc.signal_cap);
  cp(src.vh, dst.vh, sc.vh_off, dc.vh_off, r.n_vh, dc.vh_cap);
  cp(src.rp, dst.rp, sc.rp_off, dc.rp_off, r.n_reset_points, dc.rp_cap);
  cp(src.sa, dst.sa, sc.sa_off, dc.sa_off, r.n_search_attr, dc.sa_cap);
}

static void fail_result(cdr_wf_result& r, int32_t code) {
  r = cdr_wf_result{};
  r.code = code;
}

// applyEvents over every call of entry w of b onto ms (no continue-as-new runs)
static GoErr apply_calls(const cdr_batch* b, const Ctx* ctx, uint32_t w, MutableState& ms) {
  const cdr_wf_desc& d = b->wfs[w];
  const cdr_event* ev = b->events + d.ev_off;
  StateBuilder sb{ctx, b, &ms};
  GoErr err;
  if (d.ev_len == 0) err.code = CDR_E_HISTORY_EMPTY;
  for (uint64_t s = 0; s < d.ev_len && err.ok();) {
    uint64_t e = s + 1;
    while (e < d.ev_len && !(ev[e].flags & CDR_EVF_BATCH_FIRST)) e++;
    MutableState* nr = nullptr;
    GoErr ne;
    err = sb.applyEvents(d.request_id, d.workflow_id, d.run_id, d.domain_id, ev + s, (size_t)(e - s), (int64_t)s,
                         nullptr, 0, false, 0, 0, &nr, &ne);
    delete nr;
    s = e;
  }
  if (err.ok() && d.expected_next_event_id != 0 && ms.ei.NextEventID != d.expected_next_event_id) {
    err.code = CDR_E_REBUILD_NEXT_EVENT_ID;  // nDCStateRebuilder.go:139-143
    err.event_id = d.ev_len ? ev[d.ev_len - 1].event_id : 0;
    err.index = (int64_t)d.ev_len;
  }
  return err;
}

// replay_one's epilogue: the result record, and the state when OK; true = OK
static bool finish(const GoErr& e, const MutableState& ms, const cdr_batch* b, uint32_t w, const cdr_wf_caps* caps,
                   cdr_out* out) {
  cdr_wf_result& r = out->result[w];
  r = cdr_wf_result{};
  r.code = e.code;
  r.flags = e.flags;
  r.fail_event_id = e.event_id;
  r.fail_index = e.index;
  if (e.ok() && !write_state(ms, b, w, caps, out)) r.code = CDR_E_BAD_INPUT;
  return r.code == CDR_OK;
}

// the current branch's VersionHistory := the applied state's (cdr_vhs_sync's restatement)
static void sync_vhs(cdr_vhs& s, cdr_vh_item* pool, const cdr_out& o, const cdr_wf_caps& c, uint32_t w) {
  const cdr_wf_result& r = o.result[w];
  if (r.code != CDR_OK) return;
  if (r.n_vh > s.items_cap) {  // the caller's item slots are too few: the workflow fails visibly
    fail_result(o.result[w], CDR_E_VHS_CAPACITY);
    return;
  }
  if (s.n_branches == 0) {
    s.n_branches = 1;
    s.current = 0;
  }
  cdr_vh_branch& b = s.branch[s.current];
  const cdr_exec_info& x = o.exec[w];
  b.token = cdr_vh_token{x.branch_tree_id, 0, x.branch_id_lo, x.branch_id_hi};
  b.n_items = r.n_vh;
  b._pad = 0;
  for (uint32_t i = 0; i < r.n_vh; i++) pool[s.items_off + (uint64_t)s.current * s.items_cap + i] = o.vh[c.vh_off + i];
}

int cdro_ndc_replicate_round(uint32_t n, const cdr_ndc_task* tasks, const cdr_vh_item* task_items,
                             const cdr_batch* rebuild, const cdr_wf_caps* rebuild_caps, cdr_out* rebuild_out,
                             const cdr_batch* apply, const cdr_wf_caps* apply_caps, cdr_out* apply_out,
                             cdr_vhs* vhs, cdr_vh_item* pool, cdr_ndc_decision* dec, const cdr_wf_caps* state_caps,
                             cdr_out* state, int64_t refresh_now, uint32_t refresh_flags, int threads) {
  if (rebuild->n_wfs < n || apply->n_wfs < n) return -1;
  Ctx rctx{rebuild, rebuild->empty_uuid}, actx{apply, apply->empty_uuid};
  auto one = [&](uint32_t w) {
    cdro_ndc_branch(tasks + w, task_items, 1, vhs + w, pool, dec + w);  // nDCBranchMgr + prepareMutableState
    fail_result(rebuild_out->result[w], CDR_NOT_RUN);
    fail_result(apply_out->result[w], CDR_NOT_RUN);
    const cdr_ndc_decision d = dec[w];
    if (state->result[w].code != CDR_OK) return;  // a failed workflow stays failed
    if (d.code != CDR_OK) {
      fail_result(state->result[w], d.code);
      return;
    }
    if (d.action != CDR_NDC_REBUILD && d.action != CDR_NDC_APPLY_CURRENT) return;  // skip / backfill (VH only)
    const cdr_wf_desc& ad = apply->wfs[w];
    MutableState* ms = nullptr;
    if (d.action == CDR_NDC_REBUILD) {
      // nDCStateRebuilder.rebuild: a fresh NDC builder (initializeBuilders :165-176), every
      // event 1 .. lastItem, the next-event check, SetCurrentBranchToken, refreshTasks
      const cdr_wf_desc& rd = rebuild->wfs[w];
      ms = new MutableState(&rctx, (int)rd.builder, rd.failover_version, rd.wf_key, rd.retention_days);
      GoErr e = apply_calls(rebuild, &rctx, w, *ms);
      ms->vh.has_token = true;  // SetCurrentBranchToken(targetBranchToken) (:144-146)
      ms->vh.tree = d.rebuild_token.tree;
      ms->vh.br_lo = d.rebuild_token.branch_lo;
      ms->vh.br_hi = d.rebuild_token.branch_hi;
      if (!finish(e, *ms, rebuild, w, rebuild_caps, rebuild_out)) {
        state->result[w] = rebuild_out->result[w];
        delete ms;
        return;
      }
      const int32_t rc = cdro_refresh_one(rebuild, rebuild_caps, rebuild_out, refresh_now, refresh_flags, w);
      if (rc != CDR_OK) {
        state->result[w] = rebuild_out->result[w];
        delete ms;
        return;
      }
      // the refreshed timer-task marks belong to the in-memory state too
      const cdr_wf_caps& rc0 = rebuild_caps[w];
      for (uint32_t k = 0; k < rebuild_out->result[w].n_activity; k++) {
        const cdr_activity_info& a = rebuild_out->act[rc0.act_off + k];
        ms->pendingActivityInfoIDs[a.schedule_id].TimerTaskStatus = a.timer_task_status;
      }
      for (uint32_t k = 0; k < rebuild_out->result[w].n_timer; k++) {
        const cdr_timer_info& t = rebuild_out->timer[rc0.timer_off + k];
        ms->pendingTimerInfoIDs[t.timer_id].TaskID = t.task_id;
      }
      // nDCConflictResolver.rebuild: the rebuilt VersionHistory must Equal the branch's
      cdr_vhs& s = vhs[w];
      const cdr_vh_branch& br = s.branch[d.branch_index];
      bool eq = br.n_items == ms->vh.items.size() && br.token.tree == d.rebuild_token.tree &&
                br.token.branch_lo == d.rebuild_token.branch_lo && br.token.branch_hi == d.rebuild_token.branch_hi;
      const cdr_vh_item* want = pool + s.items_off + (uint64_t)d.branch_index * s.items_cap;
      for (size_t i = 0; eq && i < ms->vh.items.size(); i++)
        eq = ms->vh.items[i].eventID == want[i].event_id && ms->vh.items[i].version == want[i].version;
      if (!eq) {  // :161-165 (the failed record keeps its flags, as cdr_ndc_rebuild_verify_async)
        cdr_wf_result& r = rebuild_out->result[w];
        const uint32_t fl = r.flags;
        fail_result(r, CDR_E_REBUILD_VH_MISMATCH);
        r.flags = fl;
        state->result[w] = r;
        delete ms;
        return;
      }
      s.current = d.branch_index;  // SetCurrentVersionHistoryIndex (:172-174)
      ms->ctx = &actx;             // the rebuilt builder continues with the task's events
    } else {
      // the persisted state, loaded (mutableStateBuilder.Load)
      ms = new MutableState(&actx, (int)ad.builder, ad.failover_version, ad.wf_key, ad.retention_days);
      cdr_carry cy{};
      cy.caps = state_caps;
      cy.state = *state;
      load_state(*ms, cy, w);
    }
    // applyNonStartEventsToCurrentBranch: stateBuilder.applyEvents onto that state
    GoErr e = apply_calls(apply, &actx, w, *ms);
    if (!finish(e, *ms, apply, w, apply_caps, apply_out)) {
      state->result[w] = apply_out->result[w];
    } else {
      sync_vhs(vhs[w], pool, *apply_out, apply_caps[w], w);
      if (apply_out->result[w].code != CDR_OK)
        state->result[w] = apply_out->result[w];
      else
        copy_state(*apply_out, apply_caps[w], *state, state_caps[w], w);
    }
    delete ms;
  };
  if (threads <= 1) {
    for (uint32_t w = 0; w < n; w++) one(w);
    return 0;
  }
  std::atomic<uint32_t> next{0};
  std::vector<std::thread> th;
  auto work = [&] {
    for (uint32_t w0; (w0 = next.fetch_add(64)) < n;)
      for (uint32_t w = w0; w < std::min(n, w0 + 64); w++) one(w);
  };
  for (int t = 1; t < threads; t++) {
    try {
      th.emplace_back(work);
    } catch (const std::system_error&) {
      break;
    }
  }
  work();
  for (auto& t : th) t.join();
  return 0;
}

int cdro_state_transition(int from_state, int from_close, int to_state, int to_close) {
  ExecutionInfo e;
  e.State = from_state;
  e.CloseStatus = from_close;
  return UpdateWorkflowStateCloseStatus(e, to_state, to_close) ? 1 : 0;
}

}  // extern "C"
