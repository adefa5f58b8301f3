// refresh_ref.cpp — TEST INFRASTRUCTURE ONLY: CPU restatement of the post-rebuild task
// refresher, the parity checker for cadence_amd/csrc/refresh.hip.  Nothing under
// cadence_amd/ links or calls this.
//
// Restates (paths relative to the reference root):
//   mutableStateTaskRefresher.refreshTasks   service/history/mutableStateTaskRefresher.go:66-160
//     ForWorkflowStart :162-191, ForWorkflowClose :193-208, ForRecordWorkflowStarted :210-231,
//     ForDecision :233-262, ForActivity :264-317, ForTimer :319-342, ForChildWorkflow :344-385,
//     ForRequestCancelExternalWorkflow :387-423, ForSignalExternalWorkflow :425-461,
//     ForWorkflowSearchAttr :463-472
//   the task generator                       service/history/mutableStateTaskGenerator.go:122-545
//   timerBuilder picks                       service/history/timerBuilder.go:171-230,233-312
//   nDCStateRebuilder.rebuild's call         service/history/nDCStateRebuilder.go:154-157
//   CloseTransactionAsSnapshot(passive)     service/history/mutableStateBuilder.go:3787-3855: with
//     the passive policy every close-transaction step is a no-op (:4240-4355), a replayed
//     state has no new events, so what remains is setTaskInfo (historyEngine.go:2383-2397):
//     every task's Version = GetCurrentVersion() (flag 2)
//
// It runs on the replay's outputs (cdr_out, the rebuilt mutable state) plus the entry's
// own events (the events cache).  Parity pinning: the reference has no unit test for
// the refresher (nDCStateRebuilder_test.go:321 mocks it), so the expectations in
// tests/test_refresh.py are hand-derived from the code cited above — "parity unpinned"
// by reference vectors; the same restated timer picks are pinned through the
// stateBuilder KATs (tests/test_tasks.py).
//
// Choices the reference leaves open, fixed here and in the kernel alike:
//  - pending activities / children / request-cancels / signals are visited in ascending
//    key order (Go ranges over a map: unspecified order);
//  - an entry whose refresh fails keeps its replayed tables unchanged and gets no tasks
//    (the reference returns the error and the rebuild discards the state);
//  - an activity's target domain is getTargetDomainID(ActivityTaskScheduled.Domain)
//    (mutableStateTaskGenerator.go:309-326,531-545): "" -> the execution's domain; else the
//    domain cache's ID the caller resolved into the event's attributes (cdr_attr_at_scheduled
//    target_domain_id), a failed lookup the domain-not-found error.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "cdr/schema.h"

namespace {

constexpr int64_t kSec = 1000000000LL;

bool is_close_type(uint32_t t) {
  return t == CDR_EV_WF_COMPLETED || t == CDR_EV_WF_FAILED || t == CDR_EV_WF_TIMED_OUT ||
         t == CDR_EV_WF_CANCELED || t == CDR_EV_WF_TERMINATED || t == CDR_EV_WF_CONTINUED_AS_NEW;
}

struct Refresh {
  const cdr_batch* b;
  const cdr_wf_caps* caps;
  cdr_out* out;
  int64_t now;
  uint32_t flags;

  // eventsCache.getEvent restated over the entry's own events (nullptr = miss)
  const cdr_event* find(uint32_t w, int64_t id) const {
    const cdr_wf_desc& d = b->wfs[w];
    for (uint64_t k = 0; k < d.ev_len; k++)
      if (b->events[d.ev_off + k].event_id == id) return &b->events[d.ev_off + k];
    return nullptr;
  }

  // mutableStateBuilder.GetCurrentVersion (:491-502) of the rebuilt in-memory state: the
  // 2DC ReplicationState's; the NDC builder's currentVersion, which the prelude
  // (stateBuilder.go:139-143, UpdateCurrentVersion :445-489) sets to each event's
  // version while the execution runs — i.e. the closing event's version once closed,
  // else the last event's; EmptyVersion for the local builder
  int64_t current_version(uint32_t w) const {
    const cdr_wf_desc& d = b->wfs[w];
    if (d.builder == CDR_BUILDER_2DC) return out->repl[w].current_version;
    if (d.builder != CDR_BUILDER_NDC) return CDR_EMPTY_VERSION;
    const bool closed = out->exec[w].close_status != CDR_CLOSE_NONE;
    int64_t v = CDR_EMPTY_VERSION;
    for (uint64_t k = 0; k < d.ev_len; k++) {
      const cdr_event& e = b->events[d.ev_off + k];
      v = e.version;
      if (closed && is_close_type(e.type)) break;
    }
    return v;
  }

  int32_t one(uint32_t w) {
    const cdr_wf_caps& cp = caps[w];
    cdr_wf_result& r = out->result[w];
    const cdr_exec_info& x = out->exec[w];
    std::vector<cdr_task> xt, tt;
    auto X = [&](uint32_t type, int64_t eid, int64_t ver) -> cdr_task& {
      cdr_task t{};
      t.type = type;
      t.event_id = eid;
      t.visibility_ts = now;  // VisibilityTimestamp: now (every transfer task)
      t.version = ver;
      xt.push_back(t);
      return xt.back();
    };
    auto T = [&](uint32_t type, int32_t tot, int64_t eid, int64_t vis, int64_t att, int64_t ver) {
      cdr_task t{};
      t.type = type;
      t.timeout_type = tot;
      t.event_id = eid;
      t.visibility_ts = vis;
      t.attempt = att;
      t.version = ver;
      tt.push_back(t);
    };
    const int64_t curVer = current_version(w);

    // ---- ForWorkflowStart (:162-191): GetStartEvent, generateWorkflowStartTasks (:122-146)
    const cdr_event* se = find(w, CDR_FIRST_EVENT_ID);
    if (!se || se->type != CDR_EV_WF_STARTED) return CDR_E_REFRESH_EVENT_NOT_FOUND;
    const cdr_attr_wf_started& sa = se->a.started;
    const int64_t backoff = (int64_t)sa.first_decision_backoff_s * kSec;
    {
      int64_t vis = now + (int64_t)x.workflow_timeout * kSec + backoff;
      if ((x.flags & CDR_XI_HAS_EXPIRATION) && vis > x.expiration_time) vis = x.expiration_time;
      T(CDR_TT_WORKFLOW_TIMEOUT, 0, 0, vis, 0, se->version);
    }
    // HasProcessedOrPendingDecision (mutableStateDecisionTaskManager.go:731-733)
    const bool processedOrPending =
        x.decision_schedule_id != CDR_EMPTY_EVENT_ID || x.last_processed_event != CDR_EMPTY_EVENT_ID;
    if (!processedOrPending && sa.first_decision_backoff_s > 0) {  // generateDelayedDecisionTasks :182-222
      int32_t type = 1;  // WorkflowBackoffTimeoutTypeCron (no initiator)
      if (sa.flags & CDR_SF_HAS_INITIATOR) {
        if (sa.flags & CDR_SF_RETRY_INITIATOR)
          type = 0;  // WorkflowBackoffTimeoutTypeRetry
        else if (sa.flags & CDR_SF_CRON_INITIATOR)
          type = 1;
        else
          return CDR_E_REFRESH_BACKOFF_INITIATOR;  // Decider or unknown
      }
      T(CDR_TT_WORKFLOW_BACKOFF, type, 0, now + backoff, 0, se->version);
    }
    // ---- ForWorkflowClose (:193-208) -> generateWorkflowCloseTasks (:148-180)
    if (x.close_status != CDR_CLOSE_NONE) {
      X(CDR_TT_CLOSE_EXECUTION, 0, curVer);
      T(CDR_TT_DELETE_HISTORY, 0, 0, now + (int64_t)b->wfs[w].retention_days * 24LL * 3600LL * kSec, 0, curVer);
    }
    // ---- ForRecordWorkflowStarted (:210-231) -> generateRecordWorkflowStartedTasks (:224-238)
    if (x.close_status == CDR_CLOSE_NONE) X(CDR_TT_RECORD_STARTED, 0, se->version);
    // ---- ForDecision (:233-262)
    if (x.decision_schedule_id != CDR_EMPTY_EVENT_ID) {
      if (x.decision_started_id != CDR_EMPTY_EVENT_ID) {  // generateDecisionStartTasks :277-300
        T(CDR_TT_DECISION_TIMEOUT, CDR_TIMEOUT_START_TO_CLOSE, x.decision_schedule_id,
          now + (int64_t)x.decision_timeout * kSec, x.decision_attempt, x.decision_version);
      } else {  // generateDecisionScheduleTasks :240-275 (stickiness is cleared by replay)
        cdr_task& t = X(CDR_TT_DECISION, x.decision_schedule_id, x.decision_version);
        t.domain_id = x.domain_id;
        t.task_list = x.task_list;
      }
    }
    // ---- ForActivity (:264-317)
    cdr_activity_info* act = out->act + cp.act_off;
    std::vector<int32_t> tts(r.n_activity, 0);  // TimerTaskStatus cleared for every activity
    for (uint32_t j = 0; j < r.n_activity; j++) {
      const cdr_activity_info& a = act[j];
      if (a.started_id != CDR_EMPTY_EVENT_ID) continue;
      const cdr_event* ev = find(w, a.schedule_id);
      if (!ev) return CDR_E_REFRESH_EVENT_NOT_FOUND;
      // generateActivityTransferTasks :302-333: getTargetDomainID(attr.GetDomain()); another
      // event type's nil attributes read as the empty domain
      uint32_t dom = x.domain_id;
      if (ev->type == CDR_EV_AT_SCHEDULED && ev->a.at_sched.domain != 0) {
        if (ev->a.at_sched.flags & CDR_AF_DOMAIN_MISSING) return CDR_E_DOMAIN_NOT_FOUND;
        dom = ev->a.at_sched.target_domain_id;
      }
      cdr_task& t = X(CDR_TT_ACTIVITY, a.schedule_id, a.version);
      t.domain_id = dom;
      t.task_list = a.task_list;
    }
    {  // GetActivityTimerTaskIfNeeded (timerBuilder.go:211-230) over loadActivityTimers (:249-312)
      int best = -1;
      int64_t bt = 0, bs = 0;
      int bo = 0, btype = 0;
      auto cand = [&](int j, int64_t t, int order, int type) {
        const int64_t s = act[j].schedule_id;
        if (best < 0 || t < bt || (t == bt && (s < bs || (s == bs && order < bo)))) {
          best = j;
          bt = t;
          bs = s;
          bo = order;
          btype = type;
        }
      };
      for (uint32_t j = 0; j < r.n_activity; j++) {
        const cdr_activity_info& v = act[j];
        if (v.schedule_id == CDR_EMPTY_EVENT_ID) continue;
        int64_t s2c = v.scheduled_time + (int64_t)v.s2c * kSec;
        if (v.expiration_time < s2c) s2c = v.expiration_time;  // ExpirationTime set at scheduling
        cand((int)j, s2c, 0, CDR_TIMEOUT_SCHEDULE_TO_CLOSE);
        if (v.started_id != CDR_EMPTY_EVENT_ID) {
          const bool set = (v.flags & CDR_AI_STARTED_TIME_SET) != 0;
          const int64_t st = set ? v.started_time : 0;
          cand((int)j, st + (int64_t)v.stc * kSec, 1, CDR_TIMEOUT_START_TO_CLOSE);
          if (v.hb > 0) {
            int64_t lhb = set ? v.last_heartbeat_time : 0;
            if (lhb < st) lhb = st;
            cand((int)j, lhb + (int64_t)v.hb * kSec, 2, CDR_TIMEOUT_HEARTBEAT);
          }
        } else {
          cand((int)j, v.scheduled_time + (int64_t)v.s2s * kSec, 1, CDR_TIMEOUT_SCHEDULE_TO_START);
        }
      }
      if (best >= 0) {  // every status was cleared: the head is never "created"
        T(CDR_TT_ACTIVITY_TIMEOUT, btype, bs, bt, act[best].attempt, 0);
        tts[best] = btype == CDR_TIMEOUT_HEARTBEAT        ? CDR_TTS_HEARTBEAT
                    : btype == CDR_TIMEOUT_SCHEDULE_TO_START ? CDR_TTS_SCHEDULE_TO_START
                    : btype == CDR_TIMEOUT_SCHEDULE_TO_CLOSE ? CDR_TTS_SCHEDULE_TO_CLOSE
                                                             : CDR_TTS_START_TO_CLOSE;
      }
    }
    // ---- ForTimer (:319-342): TaskID cleared, GetUserTimerTaskIfNeeded (timerBuilder.go:171-184)
    cdr_timer_info* tim = out->timer + cp.timer_off;
    int head = -1;
    for (uint32_t j = 0; j < r.n_timer; j++)
      if (head < 0 || tim[j].expiry_time < tim[head].expiry_time ||
          (tim[j].expiry_time == tim[head].expiry_time && tim[j].started_id < tim[head].started_id))
        head = (int)j;
    if (head >= 0) T(CDR_TT_USER_TIMER, 0, tim[head].started_id, tim[head].expiry_time, 0, 0);
    // target domain (getTargetDomainID :531-545)
    auto target = [&](const cdr_attr_external* e, uint32_t* dom) -> int32_t {
      if (e->domain == 0) {  // "" -> the execution's domain
        *dom = x.domain_id;
        return CDR_OK;
      }
      if (e->flags & CDR_XF_DOMAIN_MISSING) return CDR_E_DOMAIN_NOT_FOUND;
      *dom = e->target_domain_id;
      return CDR_OK;
    };
    // ---- ForChildWorkflow (:344-385) -> generateChildWorkflowTasks (:356-387)
    const cdr_child_info* ch = out->child + cp.child_off;
    for (uint32_t j = 0; j < r.n_child; j++) {
      if (ch[j].started_id != CDR_EMPTY_EVENT_ID) continue;
      const cdr_event* ev = find(w, ch[j].initiated_id);
      if (!ev) return CDR_E_REFRESH_EVENT_NOT_FOUND;
      const cdr_attr_external* e = &ev->a.ext;
      const cdr_attr_external zero{};
      if (ev->type != CDR_EV_CHILD_INITIATED) e = &zero;  // nil attributes read as zero values
      uint32_t dom;
      if (int32_t c = target(e, &dom)) return c;
      cdr_task& t = X(CDR_TT_START_CHILD, ch[j].initiated_id, ch[j].version);
      t.domain_id = dom;
      t.target_workflow_id = ch[j].started_workflow_id;
    }
    // ---- ForRequestCancelExternalWorkflow (:387-423) / ForSignalExternalWorkflow (:425-461)
    const cdr_attr_external zero_ext{};  // a nil attribute struct reads as zero values
    auto attrs = [&](const cdr_event* e, uint32_t type) -> const cdr_attr_external* {
      return e->type == type ? &e->a.ext : &zero_ext;
    };
    auto external = [&](uint32_t type, uint32_t evtype, int64_t initiated, int64_t ver) -> int32_t {
      const cdr_event* ev = find(w, initiated);
      if (!ev) return CDR_E_REFRESH_EVENT_NOT_FOUND;
      const cdr_attr_external* e = attrs(ev, evtype);
      uint32_t dom;
      if (int32_t c = target(e, &dom)) return c;
      cdr_task& t = X(type, initiated, ver);
      t.domain_id = dom;
      t.target_workflow_id = e->workflow_id;
      t.target_run_id = e->run_id;
      t.flags = (e->flags & CDR_XF_CHILD_ONLY) ? CDR_TF_CHILD_ONLY : 0u;
      return CDR_OK;
    };
    const cdr_cancel_info* rc = out->cancel + cp.cancel_off;
    for (uint32_t j = 0; j < r.n_cancel; j++)
      if (int32_t c = external(CDR_TT_CANCEL_EXECUTION, CDR_EV_RCE_INITIATED, rc[j].initiated_id, rc[j].version)) return c;
    const cdr_signal_info* sg = out->signal + cp.signal_off;
    for (uint32_t j = 0; j < r.n_signal; j++)
      if (int32_t c = external(CDR_TT_SIGNAL_EXECUTION, CDR_EV_SE_INITIATED, sg[j].initiated_id, sg[j].version)) return c;
    // ---- ForWorkflowSearchAttr (:463-472), when advanced visibility is on (:148-156)
    if (flags & 1u) X(CDR_TT_UPSERT_SA, 0, curVer);

    if (xt.size() > cp.xfer_cap || tt.size() > cp.ttask_cap) return CDR_E_REFRESH_CAPACITY;
    // commit: task lists and the refreshed timer-task masks
    if (flags & 2u) {  // CloseTransactionAsSnapshot(passive): setTaskInfo (historyEngine.go:2383-2397)
      for (auto& t : xt) t.version = curVer;
      for (auto& t : tt) t.version = curVer;
    }
    for (size_t j = 0; j < xt.size(); j++) out->transfer[cp.xfer_off + j] = xt[j];
    for (size_t j = 0; j < tt.size(); j++) out->timer_tasks[cp.ttask_off + j] = tt[j];
    out->n_tasks[2 * w] = (uint32_t)xt.size();
    out->n_tasks[2 * w + 1] = (uint32_t)tt.size();
    for (uint32_t j = 0; j < r.n_activity; j++) act[j].timer_task_status = tts[j];
    for (uint32_t j = 0; j < r.n_timer; j++)
      tim[j].task_id = (int)j == head ? CDR_TIMER_TASK_STATUS_CREATED : CDR_TIMER_TASK_STATUS_NONE;
    return CDR_OK;
  }
};

}  // namespace

// refreshTasks of entry w alone (cdro_ndc_replicate_round's rebuild step); returns the code
extern "C" int cdro_refresh_one(const cdr_batch* b, const cdr_wf_caps* caps, cdr_out* out, int64_t now_ns,
                                uint32_t flags, uint32_t w) {
  if (!b || !caps || !out || w >= b->n_wfs || !out->transfer || !out->timer_tasks || !out->n_tasks) return -1;
  Refresh R{b, caps, out, now_ns, flags};
  out->n_tasks[2 * w] = out->n_tasks[2 * w + 1] = 0;
  if (out->result[w].code != CDR_OK) return out->result[w].code;
  const int32_t c = R.one(w);
  if (c != CDR_OK) {
    cdr_wf_result& r = out->result[w];
    r.code = c;
    r.fail_event_id = 0;
    r.fail_index = 0;
  }
  return c;
}

extern "C" int cdro_refresh_tasks(const cdr_batch* b, const cdr_wf_caps* caps, cdr_out* out, int64_t now_ns,
                                  uint32_t flags) {
  if (!b || !caps || !out || !out->transfer || !out->timer_tasks || !out->n_tasks) return -1;
  Refresh R{b, caps, out, now_ns, flags};
  for (uint32_t w = 0; w < b->n_wfs; w++) {
    out->n_tasks[2 * w] = out->n_tasks[2 * w + 1] = 0;
    if (out->result[w].code != CDR_OK) continue;
    const int32_t c = R.one(w);
    if (c != CDR_OK) {
      cdr_wf_result& r = out->result[w];
      r.code = c;
      r.fail_event_id = 0;
      r.fail_index = 0;
    }
  }
  return 0;
}
