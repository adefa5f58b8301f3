// refresh.hip — refreshTasks over the rebuilt mutable states of a replay
// (mutableStateTaskRefresher.go:66-160, called by nDCStateRebuilder.rebuild
// nDCStateRebuilder.go:154-157; task generator mutableStateTaskGenerator.go:122-545).
//
// One thread per replayed entry, launched over the slice plan's (slice, lane) pairs so
// that a lane slice's 64 entries sit in one wavefront and their event lookups read
// neighbouring slab elements.  The work is a short pass over the entry's output record
// and pending tables (the activity / user-timer picks scan the rows once) plus a few
// binary searches over the entry's own slab rows for the events the reference reads
// from its events cache (WorkflowExecutionStarted, the scheduled / initiated events of
// pending activities, children, request-cancels and signals).  It is HBM-bound and
// small next to the replay: per entry ~0.5 KB of records, 64 B per task written.
//
// Same conventions as the oracle (oracle/refresh_ref.cpp): pending rows in ascending
// key order (the output tables are sorted), an entry whose refresh fails keeps its
// tables and gets no tasks; an activity's target domain comes from its scheduled event's
// attributes (cdr_attr_at_scheduled.domain / target_domain_id, getTargetDomainID).
#include <hip/hip_runtime.h>

#include <cstdio>

#include "cdr/cdr.h"

#define HIPCHK(x)                                                                                     \
  do {                                                                                                \
    hipError_t _e = (x);                                                                              \
    if (_e != hipSuccess) {                                                                           \
      fprintf(stderr, "cdr: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(_e), __FILE__, __LINE__); \
      return CDR_API_EDEVICE;                                                                         \
    }                                                                                                 \
  } while (0)

namespace {

constexpr int64_t kSec = 1000000000LL;

__device__ __forceinline__ bool is_close_type(uint32_t t) {
  return t == CDR_EV_WF_COMPLETED || t == CDR_EV_WF_FAILED || t == CDR_EV_WF_TIMED_OUT || t == CDR_EV_WF_CANCELED ||
         t == CDR_EV_WF_TERMINATED || t == CDR_EV_WF_CONTINUED_AS_NEW;
}

// the entry's events in the slab: event k is element (row0 + k, lane) of a lane slice,
// element (row0 + k / 64, k % 64) of a wave slice
struct Events {
  const uint8_t* slab;
  uint64_t row0;
  uint32_t lane;
  bool wave;
  uint64_t n;
  __device__ const uint8_t* el(uint64_t k, int col) const {
    const uint64_t row = wave ? row0 + k / CDR_SLICE_WIDTH : row0 + k;
    const uint32_t e = wave ? (uint32_t)(k % CDR_SLICE_WIDTH) : lane;
    return slab + row * CDR_ROW_BYTES + cdr_col_off(col) + (uint64_t)e * cdr_col_size(col);
  }
  __device__ int64_t i64(uint64_t k, int col) const { return *(const int64_t*)el(k, col); }
  __device__ uint32_t type(uint64_t k) const { return *(const uint32_t*)el(k, CDR_COL_TYPE_FLAGS) & 0xFFu; }
  // eventsCache.getEvent by event ID: lower bound over the (ascending) event IDs
  __device__ int64_t find(int64_t id) const {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) / 2;
      if (i64(mid, CDR_COL_EVENT_ID) < id)
        lo = mid + 1;
      else
        hi = mid;
    }
    return lo < n && i64(lo, CDR_COL_EVENT_ID) == id ? (int64_t)lo : -1;
  }
};

__global__ __launch_bounds__(256) void k_refresh(cdr_dev_batch B, cdr_out O, int64_t now, uint32_t flags) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (uint64_t)B.ev.n_slices * CDR_SLICE_WIDTH) return;
  const int32_t wi = B.ev.lane_wf[i];
  if (wi < 0) return;
  const uint32_t w = (uint32_t)wi;
  const uint32_t s = (uint32_t)(i / CDR_SLICE_WIDTH);
  // Everything that depends only on (w, s) is loaded before the first branch on any of
  // it, so the chain of dependent global loads is lane_wf -> {records, slice row} -> slab
  // (-> arena) instead of one link per record.
  const uint64_t row0 = B.ev.slice_row0[s];
  const bool wave = (B.ev.slice_flags[s] & CDR_SLICE_WAVE) != 0;
  const cdr_wf_result r = O.result[w];
  const cdr_wf_caps cp = B.caps[w];
  const cdr_wf_desc d = B.wfs[w];
  const cdr_exec_info x = O.exec[w];
  const Events E{B.ev.slab, row0, (uint32_t)(i % CDR_SLICE_WIDTH), wave, d.ev_len};
  const bool any = d.ev_len > 0;
  const int64_t id0 = any ? E.i64(0, CDR_COL_EVENT_ID) : 0;
  const uint32_t ty0 = any ? E.type(0) : (uint32_t)CDR_EV_PAD;
  const int64_t ver0 = any ? E.i64(0, CDR_COL_VERSION) : 0;
  const int64_t aux0 = any ? E.i64(0, CDR_COL_AUX) : 0;
  // the last event: the NDC current version's usual source (a closed history ends with
  // its closing event)
  const uint32_t tyL = any ? E.type(d.ev_len - 1) : (uint32_t)CDR_EV_PAD;
  const int64_t verL = any ? E.i64(d.ev_len - 1, CDR_COL_VERSION) : 0;
  if (r.code != CDR_OK) return;

  uint32_t nx = 0, nt = 0;
  const uint32_t xcap = cp.xfer_cap, tcap = cp.ttask_cap;
  cdr_task* XT = O.transfer + cp.xfer_off;
  cdr_task* TT = O.timer_tasks + cp.ttask_off;
  auto X = [&](uint32_t type, int64_t eid, int64_t ver, uint32_t dom, uint32_t tl, uint32_t twf, uint32_t trun,
               uint32_t fl) {
    if (nx < xcap) {
      cdr_task t;
      t.type = type;
      t.timeout_type = 0;
      t.event_id = eid;
      t.visibility_ts = now;
      t.attempt = 0;
      t.domain_id = dom;
      t.task_list = tl;
      t.target_workflow_id = twf;
      t.target_run_id = trun;
      t.flags = fl;
      t._pad = 0;
      t.version = ver;
      XT[nx] = t;
    }
    nx++;
  };
  auto T = [&](uint32_t type, int32_t tot, int64_t eid, int64_t vis, int64_t att, int64_t ver) {
    if (nt < tcap) {
      cdr_task t;
      t.type = type;
      t.timeout_type = tot;
      t.event_id = eid;
      t.visibility_ts = vis;
      t.attempt = att;
      t.domain_id = t.task_list = t.target_workflow_id = t.target_run_id = t.flags = t._pad = 0;
      t.version = ver;
      TT[nt] = t;
    }
    nt++;
  };

  int32_t code = CDR_OK;
  int best = -1, head = -1;
  int32_t best_bit = 0;
  // GetCurrentVersion (mutableStateBuilder.go:491-502) of the rebuilt in-memory state
  int64_t curVer = CDR_EMPTY_VERSION;
  do {
    if (d.builder == CDR_BUILDER_2DC) {
      curVer = O.repl[w].current_version;
    } else if (d.builder == CDR_BUILDER_NDC && E.n > 0) {
      // the prelude's last version while running: the (only) closing event's, or the last
      curVer = verL;
      if (x.close_status != CDR_CLOSE_NONE && !is_close_type(tyL)) {
        uint64_t k = E.n - 1;
        while (k > 0 && !is_close_type(E.type(k))) k--;
        curVer = E.i64(k, CDR_COL_VERSION);
      }
    }
    // ---- ForWorkflowStart (:162-191): the start event is event 1
    int64_t startVer = ver0, saux = aux0;
    if (id0 != CDR_FIRST_EVENT_ID || ty0 != CDR_EV_WF_STARTED) {  // not the entry's first event
      const int64_t ks = E.find(CDR_FIRST_EVENT_ID);
      if (ks < 0 || E.type(ks) != CDR_EV_WF_STARTED) {
        code = CDR_E_REFRESH_EVENT_NOT_FOUND;
        break;
      }
      startVer = E.i64(ks, CDR_COL_VERSION);
      saux = E.i64(ks, CDR_COL_AUX);
    }
    constexpr uint64_t kStartWords = (sizeof(cdr_attr_wf_started) + 7) / 8;
    if (saux < 0 || B.ev.arena_words < kStartWords ||
        (uint64_t)saux > B.ev.arena_words - kStartWords) {  // malformed input: no attribute record (no wrap)
      code = CDR_E_BAD_INPUT;
      break;
    }
    const cdr_attr_wf_started* sa = (const cdr_attr_wf_started*)(B.ev.arena + (uint64_t)saux);
    const int32_t backoff_s = sa->first_decision_backoff_s;
    const uint32_t sflags = sa->flags;
    const int64_t backoff = (int64_t)backoff_s * kSec;
    {  // generateWorkflowStartTasks (:122-146)
      int64_t vis = now + (int64_t)x.workflow_timeout * kSec + backoff;
      if ((x.flags & CDR_XI_HAS_EXPIRATION) && vis > x.expiration_time) vis = x.expiration_time;
      T(CDR_TT_WORKFLOW_TIMEOUT, 0, 0, vis, 0, startVer);
    }
    const bool processedOrPending =
        x.decision_schedule_id != CDR_EMPTY_EVENT_ID || x.last_processed_event != CDR_EMPTY_EVENT_ID;
    if (!processedOrPending && backoff_s > 0) {  // generateDelayedDecisionTasks (:182-222)
      int32_t type = 1;
      if (sflags & CDR_SF_HAS_INITIATOR) {
        if (sflags & CDR_SF_RETRY_INITIATOR)
          type = 0;
        else if (!(sflags & CDR_SF_CRON_INITIATOR)) {
          code = CDR_E_REFRESH_BACKOFF_INITIATOR;
          break;
        }
      }
      T(CDR_TT_WORKFLOW_BACKOFF, type, 0, now + backoff, 0, startVer);
    }
    // ---- ForWorkflowClose (:193-208) / ForRecordWorkflowStarted (:210-231)
    if (x.close_status != CDR_CLOSE_NONE) {
      X(CDR_TT_CLOSE_EXECUTION, 0, curVer, 0, 0, 0, 0, 0);
      T(CDR_TT_DELETE_HISTORY, 0, 0, now + (int64_t)d.retention_days * 24LL * 3600LL * kSec, 0, curVer);
    } else {
      X(CDR_TT_RECORD_STARTED, 0, startVer, 0, 0, 0, 0, 0);
    }
    // ---- ForDecision (:233-262)
    if (x.decision_schedule_id != CDR_EMPTY_EVENT_ID) {
      if (x.decision_started_id != CDR_EMPTY_EVENT_ID)
        T(CDR_TT_DECISION_TIMEOUT, CDR_TIMEOUT_START_TO_CLOSE, x.decision_schedule_id,
          now + (int64_t)x.decision_timeout * kSec, x.decision_attempt, x.decision_version);
      else
        X(CDR_TT_DECISION, x.decision_schedule_id, x.decision_version, x.domain_id, x.task_list, 0, 0, 0);
    }
    // ---- ForActivity (:264-317): transfer tasks, then the activity timer pick
    const cdr_activity_info* act = O.act + cp.act_off;
    int64_t bt = 0, bs = 0;
    int bo = 0, btype = 0;
    for (uint32_t j = 0; j < r.n_activity; j++) {
      const int64_t sched = act[j].schedule_id, started = act[j].started_id;
      if (started == CDR_EMPTY_EVENT_ID) {
        const int64_t k = E.find(sched);
        if (k < 0) {
          code = CDR_E_REFRESH_EVENT_NOT_FOUND;
          break;
        }
        // generateActivityTransferTasks (mutableStateTaskGenerator.go:302-333): the target
        // domain is getTargetDomainID(attr.GetDomain()) (:531-545) — "" the execution's; a
        // scheduled event of another type has nil attributes (the empty domain)
        uint32_t dom = x.domain_id;
        constexpr uint64_t kAtWords = (sizeof(cdr_attr_at_scheduled) + 7) / 8;
        const uint64_t off = (uint64_t)E.i64(k, CDR_COL_AUX) & 0xFFFFFFFFull;
        if (E.type(k) == CDR_EV_AT_SCHEDULED && off + kAtWords <= B.ev.arena_words) {
          const cdr_attr_at_scheduled* a = (const cdr_attr_at_scheduled*)(B.ev.arena + off);
          if (a->domain != 0) {
            if (a->flags & CDR_AF_DOMAIN_MISSING) {
              code = CDR_E_DOMAIN_NOT_FOUND;
              break;
            }
            dom = a->target_domain_id;
          }
        }
        X(CDR_TT_ACTIVITY, sched, act[j].version, dom, act[j].task_list, 0, 0, 0);
      }
      if (sched == CDR_EMPTY_EVENT_ID) continue;
      // loadActivityTimers (timerBuilder.go:249-312), first by (time, scheduleID, order)
      auto cand = [&](int64_t t, int order, int type) {
        if (best < 0 || t < bt || (t == bt && (sched < bs || (sched == bs && order < bo)))) {
          best = (int)j;
          bt = t;
          bs = sched;
          bo = order;
          btype = type;
        }
      };
      int64_t s2c = act[j].scheduled_time + (int64_t)act[j].s2c * kSec;
      if (act[j].expiration_time < s2c) s2c = act[j].expiration_time;
      cand(s2c, 0, CDR_TIMEOUT_SCHEDULE_TO_CLOSE);
      if (started != CDR_EMPTY_EVENT_ID) {
        const bool set = (act[j].flags & CDR_AI_STARTED_TIME_SET) != 0;
        const int64_t st = set ? act[j].started_time : 0;
        cand(st + (int64_t)act[j].stc * kSec, 1, CDR_TIMEOUT_START_TO_CLOSE);
        if (act[j].hb > 0) {
          int64_t lhb = set ? act[j].last_heartbeat_time : 0;
          if (lhb < st) lhb = st;
          cand(lhb + (int64_t)act[j].hb * kSec, 2, CDR_TIMEOUT_HEARTBEAT);
        }
      } else {
        cand(act[j].scheduled_time + (int64_t)act[j].s2s * kSec, 1, CDR_TIMEOUT_SCHEDULE_TO_START);
      }
    }
    if (code != CDR_OK) break;
    if (best >= 0) {  // GetActivityTimerTaskIfNeeded (timerBuilder.go:211-230), statuses cleared
      T(CDR_TT_ACTIVITY_TIMEOUT, btype, bs, bt, act[best].attempt, 0);
      best_bit = btype == CDR_TIMEOUT_HEARTBEAT          ? CDR_TTS_HEARTBEAT
                 : btype == CDR_TIMEOUT_SCHEDULE_TO_START ? CDR_TTS_SCHEDULE_TO_START
                 : btype == CDR_TIMEOUT_SCHEDULE_TO_CLOSE ? CDR_TTS_SCHEDULE_TO_CLOSE
                                                           : CDR_TTS_START_TO_CLOSE;
    }
    // ---- ForTimer (:319-342): GetUserTimerTaskIfNeeded (timerBuilder.go:171-184)
    const cdr_timer_info* tim = O.timer + cp.timer_off;
    int64_t he = 0, hs = 0;
    for (uint32_t j = 0; j < r.n_timer; j++) {
      const int64_t e = tim[j].expiry_time, st = tim[j].started_id;
      if (head < 0 || e < he || (e == he && st < hs)) {
        head = (int)j;
        he = e;
        hs = st;
      }
    }
    if (head >= 0) T(CDR_TT_USER_TIMER, 0, hs, he, 0, 0);
    // ---- ForChildWorkflow (:344-385), ForRequestCancelExternalWorkflow (:387-423),
    // ForSignalExternalWorkflow (:425-461); target domain per getTargetDomainID (:531-545)
    // the initiated event's attributes; an event of another type has none (Go's nil
    // attribute struct reads as zero values: empty domain, workflow, run)
    const cdr_attr_external zero_ext{};
    constexpr uint64_t kExtWords = (sizeof(cdr_attr_external) + 7) / 8;
    auto ext = [&](int64_t id, uint32_t type) -> const cdr_attr_external* {
      const int64_t k = E.find(id);
      if (k < 0) return nullptr;
      const uint64_t off = (uint64_t)E.i64(k, CDR_COL_KEY) >> 32;
      if (E.type(k) != type || off + kExtWords > B.ev.arena_words) return &zero_ext;
      return (const cdr_attr_external*)(B.ev.arena + off);
    };
    auto target = [&](const cdr_attr_external* a, uint32_t* dom) -> int32_t {
      if (a->domain == 0) {
        *dom = x.domain_id;
        return CDR_OK;
      }
      if (a->flags & CDR_XF_DOMAIN_MISSING) return CDR_E_DOMAIN_NOT_FOUND;
      *dom = a->target_domain_id;
      return CDR_OK;
    };
    const cdr_child_info* ch = O.child + cp.child_off;
    for (uint32_t j = 0; j < r.n_child && code == CDR_OK; j++) {
      if (ch[j].started_id != CDR_EMPTY_EVENT_ID) continue;
      const cdr_attr_external* a = ext(ch[j].initiated_id, CDR_EV_CHILD_INITIATED);
      uint32_t dom = 0;
      code = a ? target(a, &dom) : CDR_E_REFRESH_EVENT_NOT_FOUND;
      if (code == CDR_OK)
        X(CDR_TT_START_CHILD, ch[j].initiated_id, ch[j].version, dom, 0, ch[j].started_workflow_id, 0, 0);
    }
    const cdr_cancel_info* rc = O.cancel + cp.cancel_off;
    for (uint32_t j = 0; j < r.n_cancel && code == CDR_OK; j++) {
      const cdr_attr_external* a = ext(rc[j].initiated_id, CDR_EV_RCE_INITIATED);
      uint32_t dom = 0;
      code = a ? target(a, &dom) : CDR_E_REFRESH_EVENT_NOT_FOUND;
      if (code == CDR_OK)
        X(CDR_TT_CANCEL_EXECUTION, rc[j].initiated_id, rc[j].version, dom, 0, a->workflow_id, a->run_id,
          (a->flags & CDR_XF_CHILD_ONLY) ? CDR_TF_CHILD_ONLY : 0u);
    }
    const cdr_signal_info* sg = O.signal + cp.signal_off;
    for (uint32_t j = 0; j < r.n_signal && code == CDR_OK; j++) {
      const cdr_attr_external* a = ext(sg[j].initiated_id, CDR_EV_SE_INITIATED);
      uint32_t dom = 0;
      code = a ? target(a, &dom) : CDR_E_REFRESH_EVENT_NOT_FOUND;
      if (code == CDR_OK)
        X(CDR_TT_SIGNAL_EXECUTION, sg[j].initiated_id, sg[j].version, dom, 0, a->workflow_id, a->run_id,
          (a->flags & CDR_XF_CHILD_ONLY) ? CDR_TF_CHILD_ONLY : 0u);
    }
    if (code != CDR_OK) break;
    // ---- ForWorkflowSearchAttr (:463-472) under advanced visibility (:148-156)
    if (flags & CDR_REFRESH_ADVANCED_VISIBILITY) X(CDR_TT_UPSERT_SA, 0, curVer, 0, 0, 0, 0, 0);
    if (nx > xcap || nt > tcap) code = CDR_E_REFRESH_CAPACITY;
  } while (false);

  if (code != CDR_OK) {
    cdr_wf_result& R = O.result[w];
    R.code = code;
    R.fail_event_id = 0;
    R.fail_index = 0;
    O.n_tasks[2 * (uint64_t)w] = 0;
    O.n_tasks[2 * (uint64_t)w + 1] = 0;
    return;
  }
  O.n_tasks[2 * (uint64_t)w] = nx;
  O.n_tasks[2 * (uint64_t)w + 1] = nt;
  if (flags & CDR_REFRESH_SNAPSHOT_PASSIVE) {  // setTaskInfo (historyEngine.go:2383-2397)
    for (uint32_t j = 0; j < nx; j++) XT[j].version = curVer;
    for (uint32_t j = 0; j < nt; j++) TT[j].version = curVer;
  }
  // the refreshed masks: every status / TaskID cleared, the picks' set
  cdr_activity_info* act = O.act + cp.act_off;
  for (uint32_t j = 0; j < r.n_activity; j++) act[j].timer_task_status = (int)j == best ? best_bit : 0;
  cdr_timer_info* tim = O.timer + cp.timer_off;
  for (uint32_t j = 0; j < r.n_timer; j++)
    tim[j].task_id = (int)j == head ? CDR_TIMER_TASK_STATUS_CREATED : CDR_TIMER_TASK_STATUS_NONE;
}

// entries without a lane (none in a cdr_plan_slices_ex plan) must still read "no tasks"
__global__ void k_refresh_clear(uint32_t* n_tasks, uint32_t n_wfs) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w < n_wfs) {
    n_tasks[2 * (uint64_t)w] = 0;
    n_tasks[2 * (uint64_t)w + 1] = 0;
  }
}

}  // namespace

extern "C" int cdr_refresh_tasks_async(cdr_ctx* ctx, const cdr_dev_batch* in, const cdr_out* out, int64_t now_ns,
                                       uint32_t flags, void* stream) {
  if (!ctx || !in || !out || !out->transfer || !out->timer_tasks || !out->n_tasks || !out->result || !out->exec)
    return CDR_API_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  if (in->n_wfs) {
    hipLaunchKernelGGL(k_refresh_clear, dim3((in->n_wfs + 255) / 256), dim3(256), 0, st, out->n_tasks, in->n_wfs);
    HIPCHK(hipGetLastError());
  }
  const uint64_t threads = (uint64_t)in->ev.n_slices * CDR_SLICE_WIDTH;
  if (threads) {
    hipLaunchKernelGGL(k_refresh, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, st, *in, *out, now_ns,
                       flags);
    HIPCHK(hipGetLastError());
  }
  return CDR_API_OK;
}
