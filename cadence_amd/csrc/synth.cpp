// synth.cpp — deterministic synthetic workflow histories (test + benchmark input).
//
// Shapes follow the reference's own history generator and canary workflow:
//   * the random walk of common/testing/history_event_util.go:51-960 (decision ->
//     commands -> external events -> decision, batches as in :99-125),
//   * the echo workflow of canary/echo.go:55-79 (config 1),
//   * the per-config shapes of SURVEY §8(d) (configs 1-5).
// Every workflow is a pure function of (seed, index), so a batch can be generated in
// parallel, twice (size pass, fill pass), with no shared state.
//
// Handles are fabricated (no real strings): 0 = "", 1 = "emptyUuid", small constants
// for shared names (task lists, types, activity/timer ids, checksums, SA keys) and
// per-workflow ranges for unique strings (workflow/run/request ids).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <system_error>
#include <thread>
#include <vector>

#include "cdr/cdr.h"
#include "internal.h"

#include "cdr/synth.h"

namespace {

// ---- fabricated handle space
enum : uint32_t {
  H_EMPTY = 0,
  H_EMPTY_UUID = 1,
  H_TASKLIST = 2,
  H_WFTYPE = 3,
  H_ACT_TASKLIST = 4,
  H_CRON = 5,
  H_MEMO = 6,
  H_NONRETRY = 7,
  H_DOMAIN0 = 16,      // +k target domains
  H_DOMAINID0 = 24,    // +k their domain IDs
  H_CHECKSUM0 = 32,    // +k binary checksums
  H_SIGNAME0 = 48,
  H_CHILDTYPE0 = 64,
  H_ACTID0 = 128,      // +k activity ids ("0","1",...)
  H_TIMERID0 = 4096,   // +k timer ids
  H_SAKEY0 = 8192,     // +k search attribute keys
  H_SAVAL0 = 9000,     // +k values
  H_BLOB0 = 10000,     // +k signal inputs / controls
  H_WF0 = 1u << 20     // per-workflow unique strings: H_WF0 + wf*32 + j
};
inline uint32_t wf_handle(uint32_t wf, uint32_t j) { return H_WF0 + wf * 32u + (j & 31u); }

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(cdr_mix64(seed)) {}
  uint64_t next() {
    s += 0x9E3779B97F4A7C15ull;
    return cdr_mix64(s);
  }
  uint32_t below(uint32_t n) { return n ? (uint32_t)(next() % n) : 0; }
  double uni() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
  bool p(double x) { return uni() < x; }
};

struct Pend {
  int64_t id;   // schedule / initiated / started event id
  uint32_t h;   // activity / timer handle
  int state;    // activity: 0 scheduled, 1 started, 2 cancel requested (started or not)
};

struct WfOut {
  std::vector<cdr_event> ev;      // top-level events
  std::vector<cdr_event> newrun;  // newRunHistory (continue-as-new)
  std::vector<cdr_kv> kvs;        // offsets in events are local; rebased on fill
  std::vector<cdr_reset_point> rps;
  cdr_wf_desc d{};
  bool has_newrun = false;
  uint32_t newrun_call = 0;
  bool newrun_ndc = true;
  // config-5 forks: events F+1.. of the two continuations, fork point and versions
  std::vector<cdr_event> fork[2];
  int64_t fork_F = 0, fork_vF = 0, fork_ver[2] = {0, 0};
  bool forked = false;
};

struct Gen {
  const cdr_synth_params& P;
  uint32_t wf;
  Rng r;
  WfOut& o;
  std::vector<cdr_event>* cur;
  int64_t id = 1, t, version, task = 1000;
  uint32_t calls = 0;
  bool batch_open = false;
  std::vector<Pend> acts, timers, children, cancels, signals;
  uint32_t next_act = 0, next_timer = 0;
  int64_t ver_inc = 10;
  bool cancel_requested = false;
  int64_t dsched = 0, dstart = 0;
  bool no_failover = false;  // fork continuations keep one version (a replication task has one)
  uint32_t fork_at = 0;      // config 5: take the fork snapshot once the history reaches this length
  std::vector<Gen>* fork_snap = nullptr;

  Gen(const cdr_synth_params& p, uint32_t w, WfOut& out)
      : P(p), wf(w), r(p.seed ^ cdr_mix64(0x5EED0000ull + (uint64_t)w)), o(out), cur(&out.ev) {
    t = 1600000000000000000ll + (int64_t)(r.next() % 1000000000000ull);
    version = 1;
  }

  cdr_event& emit(uint32_t type, bool new_batch) {
    cdr_event e;
    std::memset(&e, 0, sizeof(e));
    e.event_id = id++;
    t += 1000 + (int64_t)(r.next() % 50000000ull);  // 1 us .. 50 ms apart, ns jitter
    e.timestamp = t;
    e.version = version;
    e.task_id = task++;
    e.type = type;
    if (new_batch || cur->empty()) {
      e.flags = CDR_EVF_BATCH_FIRST;
      calls++;
    }
    cur->push_back(e);
    return cur->back();
  }

  void started(bool first_run) {
    cdr_event& e = emit(CDR_EV_WF_STARTED, true);
    cdr_attr_wf_started& a = e.a.started;
    a.workflow_type = H_WFTYPE;
    a.task_list = H_TASKLIST;
    a.exec_timeout_s = 3600 + (int32_t)r.below(7200);
    a.task_timeout_s = 10 + (int32_t)r.below(50);
    a.attempt = (int32_t)r.below(3);
    if (r.p(0.2)) {
      a.flags |= CDR_SF_HAS_RETRY;
      a.backoff_coefficient = 1.5 + r.below(4) * 0.25;
      a.retry_initial_s = 1 + (int32_t)r.below(5);
      a.retry_max_interval_s = 60 + (int32_t)r.below(100);
      a.retry_max_attempts = (int32_t)r.below(10);
      a.retry_expiration_s = (int32_t)r.below(1000);
      a.nonretriable = H_NONRETRY;
    }
    if (r.p(0.2)) a.expiration_ts = t + 3600ll * 1000000000ll;
    if (r.p(0.15)) {
      a.flags |= CDR_SF_HAS_PARENT_DOMAIN | CDR_SF_HAS_PARENT_EXEC | CDR_SF_HAS_PARENT_INITIATED;
      a.parent_domain_id = H_DOMAIN0 + r.below(4);
      a.parent_workflow_id = wf_handle(wf, 20);
      a.parent_run_id = wf_handle(wf, 21);
      a.parent_initiated_id = 5 + r.below(100);
    }
    if (r.p(0.3)) a.cron_schedule = H_CRON;
    if (r.p(0.3)) {
      a.flags |= CDR_SF_HAS_MEMO;
      a.memo = H_MEMO;
    }
    if (r.p(0.3)) {
      a.flags |= CDR_SF_HAS_SEARCH_ATTR;
      uint32_t n = r.below(3);
      a.search_attr_off = (uint32_t)o.kvs.size();
      a.search_attr_len = n;
      for (uint32_t k = 0; k < n; k++) o.kvs.push_back(cdr_kv{H_SAKEY0 + r.below(6), H_SAVAL0 + r.below(50)});
    }
    if (!first_run || r.p(0.2)) {
      a.flags |= CDR_SF_HAS_RESET_POINTS;
      a.continued_run_id = wf_handle(wf, 22);
      uint32_t n = 1 + r.below(3);
      a.reset_points_off = (uint32_t)o.rps.size();
      a.reset_points_len = n;
      for (uint32_t k = 0; k < n; k++) {
        cdr_reset_point p{};
        p.binary_checksum = H_CHECKSUM0 + r.below(8);
        p.run_id = r.p(0.5) ? a.continued_run_id : wf_handle(wf, 23);
        p.first_decision_completed_id = 4 + r.below(50);
        p.created_time_nano = t - 1000000000ll * (1 + r.below(100));
        p.flags = CDR_RP_HAS_CHECKSUM | CDR_RP_HAS_RUN_ID | CDR_RP_HAS_FIRST_DC_ID | CDR_RP_HAS_CREATED |
                  CDR_RP_HAS_RESETTABLE | (r.p(0.7) ? CDR_RP_RESETTABLE : 0u);
        o.rps.push_back(p);
      }
    }
  }

  void dt_sched(bool new_batch, int64_t attempt = 0) {
    cdr_event& e = emit(CDR_EV_DT_SCHEDULED, new_batch);
    e.a.dt_sched.start_to_close_s = 10 + (int32_t)r.below(20);
    e.a.dt_sched.attempt = attempt;
    e.a.dt_sched.task_list = H_TASKLIST;
    dsched = e.event_id;
  }
  void dt_started() {
    cdr_event& e = emit(CDR_EV_DT_STARTED, true);
    e.a.dt.scheduled_event_id = dsched;
    e.a.dt.request_id = wf_handle(wf, 1 + r.below(8));
    dstart = e.event_id;
  }
  void dt_completed(bool with_checksum) {
    cdr_event& e = emit(CDR_EV_DT_COMPLETED, true);
    e.a.dt.scheduled_event_id = dsched;
    e.a.dt.started_event_id = dstart;
    e.a.dt.binary_checksum = with_checksum ? H_CHECKSUM0 + r.below(4) : 0u;
  }
  void act_sched(int32_t s2s, int32_t s2c, int32_t stc, int32_t hb, bool retry) {
    cdr_event& e = emit(CDR_EV_AT_SCHEDULED, false);
    cdr_attr_at_scheduled& a = e.a.at_sched;
    a.activity_id = H_ACTID0 + (next_act++ % 3000);
    a.task_list = H_ACT_TASKLIST;
    a.s2s_s = s2s;
    a.s2c_s = s2c;
    a.stc_s = stc;
    a.hb_s = hb;
    if (retry) {
      a.flags = CDR_AF_HAS_RETRY;
      a.retry_initial_s = 1;
      a.retry_max_interval_s = 100;
      a.retry_max_attempts = 5;
      a.retry_expiration_s = r.p(0.5) ? s2c * 2 : s2c / 2;
      a.backoff_coefficient = 2.0;
      a.nonretriable = H_NONRETRY;
    }
    acts.push_back(Pend{e.event_id, a.activity_id, 0});
  }
  void act_started(size_t k, bool new_batch) {
    cdr_event& e = emit(CDR_EV_AT_STARTED, new_batch);
    e.a.at.scheduled_event_id = acts[k].id;
    e.a.at.request_id = wf_handle(wf, 9 + r.below(8));
    if (acts[k].state == 0) acts[k].state = 1;
  }
  void act_close(size_t k, uint32_t type, bool new_batch) {
    cdr_event& e = emit(type, new_batch);
    e.a.at.scheduled_event_id = acts[k].id;
    e.a.at.timeout_type = (int32_t)r.below(4);
    acts.erase(acts.begin() + (long)k);
  }
  void timer_started() {
    cdr_event& e = emit(CDR_EV_TIMER_STARTED, false);
    // ids are occasionally reused after fire/cancel (mutableStateBuilder.go:2877-2900)
    uint32_t tid = H_TIMERID0 + (r.p(0.2) && next_timer ? r.below(next_timer) : next_timer++);
    for (auto& p : timers)
      if (p.h == tid) tid = H_TIMERID0 + next_timer++;
    e.a.timer.timer_id = tid;
    e.a.timer.start_to_fire_s = 1 + (int64_t)r.below(3600);
    timers.push_back(Pend{e.event_id, tid, 0});
  }

  // one decision task's commands (after DTCompleted), history_event_util.go:203-420
  void commands(double w_act, double w_timer, double w_ext) {
    uint32_t n = r.below(4);
    for (uint32_t c = 0; c < n; c++) {
      double x = r.uni() * (w_act + w_timer + w_ext + 0.3);
      if (x < w_act) {
        if (acts.size() < 12)
          act_sched(5 + (int32_t)r.below(60), 30 + (int32_t)r.below(600), 10 + (int32_t)r.below(300),
                    r.p(0.3) ? 1 + (int32_t)r.below(60) : 0, r.p(0.3));
      } else if (x < w_act + w_timer) {
        if (!timers.empty() && r.p(0.25)) {
          size_t k = r.below((uint32_t)timers.size());
          cdr_event& e = emit(CDR_EV_TIMER_CANCELED, false);
          e.a.timer.timer_id = timers[k].h;
          e.a.timer.started_event_id = timers[k].id;
          timers.erase(timers.begin() + (long)k);
        } else if (timers.size() < 10) {
          timer_started();
        }
      } else if (x < w_act + w_timer + w_ext) {
        uint32_t kind = r.below(4);
        if (kind == 0 && children.size() < 4) {
          cdr_event& e = emit(CDR_EV_CHILD_INITIATED, false);
          e.a.ext.domain = H_DOMAIN0 + r.below(4);
          e.a.ext.workflow_id = wf_handle(wf, 24 + r.below(4));
          e.a.ext.workflow_type = H_CHILDTYPE0 + r.below(4);
          e.a.ext.parent_close_policy = (int32_t)r.below(3);
          e.a.ext.target_domain_id = H_DOMAINID0 + (e.a.ext.domain - H_DOMAIN0);
          children.push_back(Pend{e.event_id, 0, 0});
        } else if (kind == 1 && signals.size() < 4) {
          cdr_event& e = emit(CDR_EV_SE_INITIATED, false);
          e.a.ext.domain = H_DOMAIN0 + r.below(4);
          e.a.ext.signal_name = H_SIGNAME0 + r.below(4);
          e.a.ext.input = H_BLOB0 + r.below(100);
          e.a.ext.control = r.p(0.5) ? H_BLOB0 + r.below(100) : 0u;
          // target execution / domain ID / child-only: derived, so the generator's random
          // stream (and every committed digest) is unchanged
          e.a.ext.target_domain_id = H_DOMAINID0 + (e.a.ext.domain - H_DOMAIN0);
          e.a.ext.workflow_id = wf_handle(wf, 28 + (uint32_t)(e.event_id & 1));
          e.a.ext.run_id = (e.event_id & 2) ? wf_handle(wf, 30) : 0u;
          e.a.ext.flags |= (e.event_id & 4) ? CDR_XF_CHILD_ONLY : 0u;
          signals.push_back(Pend{e.event_id, 0, 0});
        } else if (kind == 2 && cancels.size() < 4) {
          cdr_event& e = emit(CDR_EV_RCE_INITIATED, false);
          e.a.ext.domain = H_DOMAIN0 + r.below(4);
          e.a.ext.target_domain_id = H_DOMAINID0 + (e.a.ext.domain - H_DOMAIN0);
          e.a.ext.workflow_id = wf_handle(wf, 28 + (uint32_t)(e.event_id & 1));
          e.a.ext.run_id = (e.event_id & 2) ? wf_handle(wf, 30) : 0u;
          e.a.ext.flags |= (e.event_id & 4) ? CDR_XF_CHILD_ONLY : 0u;
          cancels.push_back(Pend{e.event_id, 0, 0});
        } else if (!acts.empty()) {
          size_t k = r.below((uint32_t)acts.size());
          if (acts[k].state != 2) {
            cdr_event& e = emit(CDR_EV_AT_CANCEL_REQUESTED, false);
            e.a.at.activity_id = acts[k].h;
            acts[k].state = 2;
          } else {
            cdr_event& e = emit(CDR_EV_AT_REQ_CANCEL_FAILED, false);
            e.a.at.activity_id = H_ACTID0 + 2999;
          }
        }
      } else {
        uint32_t kind = r.below(3);
        if (kind == 0) {
          emit(CDR_EV_MARKER_RECORDED, false);
        } else if (kind == 1) {
          cdr_event& e = emit(CDR_EV_UPSERT_SA, false);
          uint32_t m = 1 + r.below(2);
          e.a.upsert.search_attr_off = (uint32_t)o.kvs.size();
          e.a.upsert.search_attr_len = m;
          for (uint32_t k = 0; k < m; k++) o.kvs.push_back(cdr_kv{H_SAKEY0 + r.below(6), H_SAVAL0 + r.below(50)});
        } else if (!timers.empty()) {
          cdr_event& e = emit(CDR_EV_CANCEL_TIMER_FAILED, false);
          e.a.timer.timer_id = H_TIMERID0 + 4000;
        }
      }
    }
  }

  // external events that arrive while no decision is in flight, then DTScheduled
  void externals() {
    uint32_t nb = 1 + r.below(2);
    for (uint32_t b = 0; b < nb; b++) {
      uint32_t m = 1 + r.below(3);
      bool first = true;
      for (uint32_t j = 0; j < m; j++) {
        uint32_t kind = r.below(8);
        if (kind <= 2 && !acts.empty()) {
          size_t k = r.below((uint32_t)acts.size());
          if (acts[k].state == 0) {
            act_started(k, first);
          } else if (acts[k].state == 2) {
            act_close(k, CDR_EV_AT_CANCELED, first);
          } else {
            uint32_t ty = r.p(0.7) ? CDR_EV_AT_COMPLETED : (r.p(0.5) ? CDR_EV_AT_FAILED : CDR_EV_AT_TIMED_OUT);
            act_close(k, ty, first);
          }
        } else if (kind == 3 && !timers.empty()) {
          // fire the earliest pending timer
          size_t k = 0;
          cdr_event& e = emit(CDR_EV_TIMER_FIRED, first);
          e.a.timer.timer_id = timers[k].h;
          e.a.timer.started_event_id = timers[k].id;
          timers.erase(timers.begin());
        } else if (kind == 4) {
          emit(CDR_EV_WF_SIGNALED, first);
        } else if (kind == 5 && !children.empty()) {
          size_t k = r.below((uint32_t)children.size());
          if (children[k].state == 0 && r.p(0.8)) {
            cdr_event& e = emit(CDR_EV_CHILD_STARTED, first);
            e.a.ref.initiated_event_id = children[k].id;
            e.a.ref.run_id = wf_handle(wf, 28 + r.below(4));
            children[k].state = 1;
          } else {
            uint32_t ty = children[k].state == 0 ? CDR_EV_CHILD_START_FAILED : CDR_EV_CHILD_COMPLETED + r.below(5);
            cdr_event& e = emit(ty, first);
            e.a.ref.initiated_event_id = children[k].id;
            children.erase(children.begin() + (long)k);
          }
        } else if (kind == 6 && !signals.empty()) {
          cdr_event& e = emit(r.p(0.8) ? CDR_EV_EXT_SIGNALED : CDR_EV_SE_FAILED, first);
          e.a.ref.initiated_event_id = signals[0].id;
          signals.erase(signals.begin());
        } else if (kind == 7 && !cancels.empty()) {
          cdr_event& e = emit(r.p(0.8) ? CDR_EV_EXT_CANCEL_REQUESTED : CDR_EV_RCE_FAILED, first);
          e.a.ref.initiated_event_id = cancels[0].id;
          cancels.erase(cancels.begin());
        } else {
          emit(CDR_EV_WF_SIGNALED, first);
        }
        first = false;
      }
    }
  }

  void maybe_failover() {
    if (P.builder == CDR_BUILDER_LOCAL || no_failover) return;
    if (r.p(0.08)) {
      // next failover version owned by one of the 3 clusters (initial versions 1, 2, 3)
      int64_t next = (version / ver_inc + 1) * ver_inc + 1 + r.below(3);
      version = next;
    }
  }

  // the general random walk (configs 0, 3, 4, 5)
  void random_walk(uint32_t target, bool end_with_can, double w_act, double w_timer, double w_ext) {
    started(true);
    dt_sched(false);
    walk_body(target, w_act, w_timer, w_ext);
    if (fork_snap && fork_snap->empty()) fork_snap->push_back(*this);  // short walks fork here
    walk_end(end_with_can);
  }
  // decision rounds until the history (of the current event vector) reaches `target`; a
  // round starts with DTStarted and ends with the next DTScheduled, so a round boundary
  // is a batch boundary (the fork point of config 5)
  void walk_body(uint32_t target, double w_act, double w_timer, double w_ext) {
    while ((uint32_t)cur->size() + 6 < target) {
      if (fork_snap && fork_snap->empty() && (uint32_t)cur->size() >= fork_at) fork_snap->push_back(*this);
      dt_started();
      if (r.p(0.06)) {
        // decision timeout / failure: FailDecision + transient decision (stateBuilder.go:221-257)
        if (r.p(0.5)) {
          cdr_event& e = emit(CDR_EV_DT_TIMED_OUT, true);
          e.a.dt.scheduled_event_id = dsched;
          e.a.dt.started_event_id = dstart;
          e.a.dt.timeout_type = r.p(0.8) ? CDR_TIMEOUT_START_TO_CLOSE : CDR_TIMEOUT_SCHEDULE_TO_START;
        } else {
          cdr_event& e = emit(CDR_EV_DT_FAILED, true);
          e.a.dt.scheduled_event_id = dsched;
          e.a.dt.started_event_id = dstart;
        }
        maybe_failover();
        dt_sched(true, 1 + r.below(3));
        continue;
      }
      dt_completed(r.p(0.5));
      commands(w_act, w_timer, w_ext);
      if (r.p(0.03) && !cancel_requested) {
        emit(CDR_EV_WF_CANCEL_REQUESTED, true);
        cancel_requested = true;
      }
      maybe_failover();
      externals();
      dt_sched(false);
    }
  }
  void walk_end(bool end_with_can) {
    dt_started();
    dt_completed(r.p(0.5));
    if (end_with_can) {
      cdr_event& e = emit(CDR_EV_WF_CONTINUED_AS_NEW, false);
      e.a.can.new_execution_run_id = wf_handle(wf, 30);
      o.has_newrun = true;
      o.newrun_call = calls - 1;
      o.newrun_ndc = r.p(0.5);
      // newRunHistory: [Started, DTScheduled] of the next run (stateBuilder.go:564-571)
      cur = &o.newrun;
      int64_t saved_id = id;
      id = 1;
      started(false);
      dt_sched(false);
      id = saved_id;
      cur = &o.ev;
    } else {
      uint32_t ty = cancel_requested ? CDR_EV_WF_CANCELED : (r.p(0.85) ? CDR_EV_WF_COMPLETED : CDR_EV_WF_FAILED);
      emit(ty, false);
    }
  }

  // config 1: canary echo, 11 events in 7 batches (canary/echo.go:55-79)
  void echo() {
    started(true);
    dt_sched(false);
    dt_started();
    dt_completed(false);
    act_sched(10, 60, 30, 0, false);
    act_started(0, true);
    act_close(0, CDR_EV_AT_COMPLETED, true);
    dt_sched(false);
    dt_started();
    dt_completed(false);
    emit(CDR_EV_WF_COMPLETED, false);
  }

  // config 2: 1 + 1 + 33 x 6 + 2 = 203 events, sequential activities
  void activity_heavy(uint32_t n_act) {
    started(true);
    dt_sched(false);
    dt_started();
    for (uint32_t k = 0; k < n_act; k++) {
      dt_completed(true);
      act_sched(10, 60, 30, 0, false);
      act_started(0, true);
      act_close(0, CDR_EV_AT_COMPLETED, true);
      dt_sched(false);
      dt_started();
    }
    dt_completed(true);
    emit(CDR_EV_WF_COMPLETED, false);
  }

  // one injected fault (error-path coverage)
  void inject_fault(uint32_t mask) {
    std::vector<cdr_event>& ev = o.ev;
    if (ev.size() < 4) return;
    size_t k = 2 + r.below((uint32_t)ev.size() - 2);
    cdr_event& e = ev[k];
    uint32_t kind = r.below(8);
    while (mask && !(mask & (1u << kind))) kind = (kind + 1) & 7;
    switch (kind) {
      case 0:
        e.type = 42 + r.below(10);  // unknown event type
        break;
      case 1:
        if (e.type == CDR_EV_DT_STARTED) e.a.dt.scheduled_event_id += 1;
        else e.version -= 7;  // lower version (NDC) / unknown cluster (2DC)
        break;
      case 2:
        e.type = CDR_EV_AT_COMPLETED;  // close of a missing activity
        e.a.at.scheduled_event_id = 100000;
        break;
      case 3:
        e.type = CDR_EV_AT_STARTED;  // nil-deref panic
        e.a.at.scheduled_event_id = 100001;
        break;
      case 4:
        e.type = CDR_EV_CHILD_STARTED;  // nil-deref panic
        e.a.ref.initiated_event_id = 100002;
        break;
      case 5:
        e.type = CDR_EV_WF_COMPLETED;  // may be an invalid transition (Created -> Completed)
        break;
      case 6:
        e.type = CDR_EV_AT_CANCEL_REQUESTED;  // missing activity info
        e.a.at.activity_id = H_ACTID0 + 2998;
        break;
      default:
        e.type = CDR_EV_WF_CONTINUED_AS_NEW;  // continue-as-new without newRunHistory
        e.a.can.new_execution_run_id = wf_handle(wf, 30);
        break;
    }
  }
};

uint32_t lognormal_len(Rng& r, double median, uint32_t cap) {
  double u1 = std::max(r.uni(), 1e-12), u2 = r.uni();
  double z = std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
  double v = median * std::exp(0.8 * z);
  uint32_t n = (uint32_t)std::max(8.0, std::min((double)cap, v));
  return n;
}

int default_builder(int cfg, Rng& r) {
  switch (cfg) {
    case 1:
    case 2:
    case 5:
      return CDR_BUILDER_NDC;
    case 3:
      return CDR_BUILDER_2DC;
    case 4:
      return r.p(0.5) ? CDR_BUILDER_NDC : CDR_BUILDER_2DC;
    default:
      return (int)r.below(3);
  }
}

inline uint32_t global_index(const cdr_synth_params& P, uint32_t local) {
  return P.index_map ? P.index_map[local] : local;
}

// the per-workflow draws that precede generation (builder, version origin, target
// length), from the workflow's second stream; shared by gen_one and cdr_synth_weights
struct WfPlan {
  int builder;
  int64_t version;
  uint32_t target;  // target event count of the walk (0: fixed-shape configs)
};
WfPlan plan_one(const cdr_synth_params& P, uint32_t w, Rng& r2) {
  WfPlan q{};
  q.builder = P.builder >= 0 ? P.builder : default_builder(P.config, r2);
  const uint32_t cap = P.max_len ? P.max_len : 204800u;
  q.version = 1;
  if (q.builder == CDR_BUILDER_LOCAL) q.version = CDR_EMPTY_VERSION;
  else if (q.builder == CDR_BUILDER_2DC) q.version = 1 + r2.below(3);
  switch (P.config) {
    case 1:
      q.target = 11;
      break;
    case 2:
      q.target = P.target_len ? 5 + 6 * ((P.target_len - 5) / 6) : 203;
      break;
    case 3:
      q.target = P.target_len ? P.target_len : 200;
      break;
    case 4:
      q.target = lognormal_len(r2, P.target_len ? P.target_len : 200, cap);
      break;
    case 5:
      q.target = lognormal_len(r2, P.target_len ? P.target_len : 120, cap);
      break;
    default:
      q.target = lognormal_len(r2, P.target_len ? P.target_len : 60, cap);
      break;
  }
  if (P.long_stride && w % P.long_stride == P.long_stride / 2 && P.config != 1 && P.config != 2)
    q.target = cap;  // at the history count limit (the draws above are kept: the stream stays aligned)
  return q;
}

// generate workflow `w` (pure function of params and w)
void gen_one(const cdr_synth_params& P, uint32_t local, WfOut& o) {
  const uint32_t w = global_index(P, local);  // global workflow index
  Gen g(P, w, o);
  Rng r2(P.seed ^ cdr_mix64(0xB17D + (uint64_t)w));
  const WfPlan q = plan_one(P, w, r2);
  const int builder = q.builder;
  Gen* gp = &g;
  g.version = q.version;
  // config 5 (NDC): the fork snapshot (a DeepCopy of the generator, nDC_integration_test.go:
  // 224-308) is taken at a round boundary 40-70% into the walk, from its own stream so
  // that the base history is the same with or without forks
  std::vector<Gen> snap;
  Rng rf(P.seed ^ cdr_mix64(0xF0C5 + (uint64_t)w));
  if (P.config == 5 && q.builder == CDR_BUILDER_NDC) {
    g.fork_snap = &snap;
    g.fork_at = (uint32_t)(q.target * (0.4 + 0.3 * rf.uni()));
  }
  switch (P.config) {
    case 1:
      gp->echo();
      break;
    case 2:
      gp->activity_heavy(P.target_len ? (P.target_len - 5) / 6 : 33);
      break;
    case 3:
      gp->random_walk(q.target, false, 0.5, 1.5, 0.7);
      break;
    case 4:
      gp->random_walk(q.target, true, 0.6, 0.6, 1.2);
      break;
    case 5:
      gp->random_walk(q.target, false, 1.0, 0.8, 0.5);
      break;
    default:
      gp->random_walk(q.target, r2.p(0.2), 1.0, 1.0, 1.0);
      break;
  }
  if (!snap.empty()) {
    // the two continuations from the fork point: fork A above every base version (a
    // failover to another cluster), fork B above A or between the fork point's version
    // and A's, half the workflows each; one version per continuation (one replication task)
    const Gen& at = snap[0];
    o.forked = true;
    o.fork_F = at.id - 1;
    o.fork_vF = at.version;
    int64_t maxv = 0;
    for (const cdr_event& e : o.ev) maxv = std::max(maxv, e.version);
    const int64_t inc = at.ver_inc;
    o.fork_ver[0] = (maxv / inc + 1) * inc + 1 + rf.below(3);
    o.fork_ver[1] = rf.p(0.5) ? (o.fork_ver[0] / inc + 1) * inc + 1 + rf.below(3) : at.version + 1;
    for (int k = 0; k < 2; k++) {
      Gen f = at;
      f.fork_snap = nullptr;
      f.cur = &o.fork[k];
      f.r = Rng(P.seed ^ cdr_mix64(0xF0C50000ull + 2 * (uint64_t)w + (uint64_t)k));
      f.version = o.fork_ver[k];
      f.no_failover = true;
      f.walk_body(8 + (uint32_t)f.r.below(q.target / 2 + 8), 1.0, 0.8, 0.5);
      f.walk_end(false);
    }
  }
  if (builder == CDR_BUILDER_LOCAL) {
    for (auto& e : o.ev) e.version = CDR_EMPTY_VERSION;
    for (auto& e : o.newrun) e.version = CDR_EMPTY_VERSION;
  }
  if (P.error_rate > 0 && r2.uni() < P.error_rate) g.inject_fault(P.fault_kinds);
  if (P.ndc_part != CDR_SYNTH_PART_BASE) {  // one part of a config-5 forked history
    if (!o.forked) {
      o.ev.clear();
    } else if (P.ndc_part == CDR_SYNTH_PART_REBUILD) {
      o.ev.resize((size_t)o.fork_F);  // event ids are 1..n: events 1..F
    } else {
      o.ev = o.fork[P.ndc_part == CDR_SYNTH_PART_FORK_A ? 0 : 1];
    }
  }
  o.d.wf_key = cdr_mix64(P.seed ^ (0xC0FFEEull + w));
  o.d.domain_id = H_DOMAIN0 + 15;
  o.d.workflow_id = wf_handle(w, 0);
  o.d.run_id = wf_handle(w, 10);
  o.d.request_id = wf_handle(w, 11);
  o.d.builder = (uint32_t)builder;
  o.d.retention_days = 1 + (int32_t)r2.below(30);
  o.d.failover_version = builder == CDR_BUILDER_LOCAL ? CDR_EMPTY_VERSION : 1;
  o.d.expected_next_event_id = P.ndc_part == CDR_SYNTH_PART_REBUILD ? o.fork_F + 1
                               : (P.rebuild && P.ndc_part == CDR_SYNTH_PART_BASE) ? (int64_t)o.ev.size() + 1
                                                                                   : 0;
  o.d.parent = -1;
  o.d.newrun = -1;
  o.d.newrun_call = o.newrun_call;
  o.d.newrun_ndc = o.newrun_ndc ? 1u : 0u;
}

int threads_for(int t) {
  if (t > 0) return t;
  unsigned h = std::thread::hardware_concurrency();
  return h ? (int)std::min(h, 32u) : 4;
}

template <class F>
void par(uint32_t n, int threads, F&& f) {
  threads = threads_for(threads);
  std::atomic<uint32_t> next{0};
  std::vector<std::thread> pool;
  auto work = [&] {
    for (;;) {
      uint32_t i0 = next.fetch_add(64);
      if (i0 >= n) break;
      uint32_t i1 = std::min(n, i0 + 64);
      for (uint32_t i = i0; i < i1; i++) f(i);
    }
  };
  for (int t = 1; t < threads && n > 64; t++) {
    try {
      pool.emplace_back(work);
    } catch (const std::system_error&) {
      break;  // thread limit reached: the caller's thread still drains the queue
    }
  }
  work();
  for (auto& th : pool) th.join();
}

struct Sizes {
  std::vector<uint32_t> n_ev, n_nr, n_kv, n_rp;
  std::vector<uint8_t> has_nr;
  std::vector<cdr_wf_caps> cap_ev, cap_nr;  // only filled when want_caps
  std::vector<uint32_t> aw_ev, aw_nr;       // arena words
};

uint32_t arena_of(const std::vector<cdr_event>& ev) {
  uint32_t a = 0;
  for (auto& e : ev) a += cdr_internal::arena_words_for(e.type);
  return a;
}

void size_pass(const cdr_synth_params& P, Sizes& S, int threads, bool want_caps = false) {
  if (want_caps) {
    S.cap_ev.assign(P.n_wfs, cdr_wf_caps{});
    S.cap_nr.assign(P.n_wfs, cdr_wf_caps{});
    S.aw_ev.assign(P.n_wfs, 0);
    S.aw_nr.assign(P.n_wfs, 0);
  }
  S.n_ev.assign(P.n_wfs, 0);
  S.n_nr.assign(P.n_wfs, 0);
  S.n_kv.assign(P.n_wfs, 0);
  S.n_rp.assign(P.n_wfs, 0);
  S.has_nr.assign(P.n_wfs, 0);
  par(P.n_wfs, threads, [&](uint32_t w) {
    WfOut o;
    gen_one(P, w, o);
    S.n_ev[w] = (uint32_t)o.ev.size();
    S.n_nr[w] = (uint32_t)o.newrun.size();
    S.has_nr[w] = o.has_newrun;
    S.n_kv[w] = (uint32_t)o.kvs.size();
    S.n_rp[w] = (uint32_t)o.rps.size();
    if (want_caps) {
      cdr_internal::caps_one(o.ev.data(), o.ev.size(), o.d.builder, &S.cap_ev[w], o.kvs.data(), o.rps.data());
      cdr_internal::caps_one(o.newrun.data(), o.newrun.size(),
                             o.newrun_ndc ? (uint32_t)CDR_BUILDER_NDC : (uint32_t)CDR_BUILDER_2DC, &S.cap_nr[w],
                             o.kvs.data(), o.rps.data());
      // task-list capacities too (cdr_out.transfer / timer_tasks: bench.py --tasks)
      cdr_internal::task_caps(o.ev.data(), o.ev.size(), &S.cap_ev[w].xfer_cap, &S.cap_ev[w].ttask_cap);
      if (!o.newrun.empty())
        cdr_internal::task_caps(o.newrun.data(), o.newrun.size(), &S.cap_nr[w].xfer_cap, &S.cap_nr[w].ttask_cap);
      S.aw_ev[w] = arena_of(o.ev);
      S.aw_nr[w] = arena_of(o.newrun);
    }
  });
}

void rebase(std::vector<cdr_event>& ev, uint32_t kv_base, uint32_t rp_base) {
  for (auto& e : ev) {
    if (e.type == CDR_EV_WF_STARTED) {
      e.a.started.search_attr_off += kv_base;
      e.a.started.reset_points_off += rp_base;
    } else if (e.type == CDR_EV_UPSERT_SA) {
      e.a.upsert.search_attr_off += kv_base;
    }
  }
}

void cluster_meta(cdr_cluster_meta* c) {
  std::memset(c, 0, sizeof(*c));
  c->failover_version_increment = 10;
  c->current_cluster = 0;
  c->n_clusters = 3;
  c->initial_version[0] = 1;
  c->initial_version[1] = 2;
  c->initial_version[2] = 3;
}

}  // namespace

extern "C" {

// Sizes of the natural-order batch for `p`.
int cdr_synth_size(const cdr_synth_params* p, cdr_synth_sizes* out) {
  if (!p || !out) return CDR_API_EINVAL;
  Sizes S;
  size_pass(*p, S, 0);
  cdr_synth_sizes z{};
  for (uint32_t w = 0; w < p->n_wfs; w++) {
    z.n_events += S.n_ev[w] + S.n_nr[w];
    z.n_entries += 1 + (S.has_nr[w] ? 1 : 0);
    z.n_kvs += S.n_kv[w];
    z.n_rps += S.n_rp[w];
  }
  *out = z;
  return CDR_API_OK;
}

// Fill a natural-order batch (arrays sized by cdr_synth_size).  Entry order: each
// top-level workflow followed by its continue-as-new run (if any).  `b` receives the
// pointers, cluster metadata, now and seed.
int cdr_synth_fill(const cdr_synth_params* p, cdr_event* ev, cdr_wf_desc* wfs, cdr_kv* kvs, cdr_reset_point* rps,
                   cdr_batch* b) {
  if (!p || !ev || !wfs || !b) return CDR_API_EINVAL;
  Sizes S;
  size_pass(*p, S, 0);
  std::vector<uint64_t> ev_base(p->n_wfs), kv_base(p->n_wfs), rp_base(p->n_wfs);
  std::vector<uint32_t> ent_base(p->n_wfs);
  uint64_t e = 0, kv = 0, rp = 0;
  uint32_t ent = 0;
  for (uint32_t w = 0; w < p->n_wfs; w++) {
    ev_base[w] = e;
    kv_base[w] = kv;
    rp_base[w] = rp;
    ent_base[w] = ent;
    e += S.n_ev[w] + S.n_nr[w];
    kv += S.n_kv[w];
    rp += S.n_rp[w];
    ent += 1 + (S.has_nr[w] ? 1 : 0);
  }
  par(p->n_wfs, 0, [&](uint32_t w) {
    WfOut o;
    gen_one(*p, w, o);
    rebase(o.ev, (uint32_t)kv_base[w], (uint32_t)rp_base[w]);
    rebase(o.newrun, (uint32_t)kv_base[w], (uint32_t)rp_base[w]);
    std::copy(o.ev.begin(), o.ev.end(), ev + ev_base[w]);
    std::copy(o.newrun.begin(), o.newrun.end(), ev + ev_base[w] + o.ev.size());
    if (kvs) std::copy(o.kvs.begin(), o.kvs.end(), kvs + kv_base[w]);
    if (rps) std::copy(o.rps.begin(), o.rps.end(), rps + rp_base[w]);
    const uint32_t i = ent_base[w];
    cdr_wf_desc d = o.d;
    d.ev_off = ev_base[w];
    d.ev_len = o.ev.size();
    if (o.has_newrun) {
      d.newrun = (int32_t)(i + 1);
      cdr_wf_desc n = o.d;
      n.wf_key = cdr_mix64(o.d.wf_key ^ CDR_UUID_NEWRUN_KEY);
      n.ev_off = ev_base[w] + o.ev.size();
      n.ev_len = o.newrun.size();
      n.run_id = wf_handle(global_index(*p, w), 30);  // == the CAN event's NewExecutionRunId
      uint64_t lo, hi;
      cdr_uuid(p->seed, o.d.wf_key, CDR_UUID_NEWRUN_REQ, 0, &lo, &hi);
      n.request_id = wf_handle(global_index(*p, w), 12);  // host-interned uuid.New() (stateBuilder.go:566)
      (void)lo;
      (void)hi;
      n.builder = o.newrun_ndc ? CDR_BUILDER_NDC : CDR_BUILDER_2DC;
      n.expected_next_event_id = 0;
      n.parent = (int32_t)i;
      n.newrun = -1;
      n.newrun_call = 0;
      n.newrun_ndc = 0;
      wfs[i + 1] = n;
    }
    wfs[i] = d;
  });
  std::memset(b, 0, sizeof(*b));
  b->events = ev;
  b->n_events = e;
  b->wfs = wfs;
  b->n_wfs = ent;
  b->empty_uuid = H_EMPTY_UUID;
  b->kvs = kvs;
  b->n_kvs = kv;
  b->rps = rps;
  b->n_rps = rp;
  cluster_meta(&b->cluster);
  b->now_ns = 1700000000000000000ll;
  b->uuid_seed = p->seed * 0x9E3779B97F4A7C15ull + 1;
  return CDR_API_OK;
}



// Plan a directly-sliced synthetic batch (no natural-order intermediate: the bench
// path for 1M-workflow configs).
int cdr_synth_sliced_plan(const cdr_synth_params* p, cdr_synth_plan_info* info) {
  if (!p || !info) return CDR_API_EINVAL;
  Sizes S;
  size_pass(*p, S, 0, true);
  cdr_synth_plan_info z{};
  std::vector<cdr_wf_desc> lens;
  std::vector<cdr_wf_caps> lcaps;
  for (uint32_t w = 0; w < p->n_wfs; w++) {
    z.n_events += S.n_ev[w] + S.n_nr[w];
    z.n_entries += 1 + (S.has_nr[w] ? 1 : 0);
    z.n_kvs += S.n_kv[w];
    z.n_rps += S.n_rp[w];
    z.arena_words += S.aw_ev[w] + S.aw_nr[w];
    const cdr_wf_caps* cs[2] = {&S.cap_ev[w], &S.cap_nr[w]};
    for (int j = 0; j < (S.has_nr[w] ? 2 : 1); j++) {
      z.totals.act += cs[j]->act_cap;
      z.totals.timer += cs[j]->timer_cap;
      z.totals.child += cs[j]->child_cap;
      z.totals.cancel += cs[j]->cancel_cap;
      z.totals.signal += cs[j]->signal_cap;
      z.totals.vh += cs[j]->vh_cap;
      z.totals.rp += cs[j]->rp_cap;
      z.totals.sa += cs[j]->sa_cap;
      z.totals.xfer += cs[j]->xfer_cap;
      z.totals.ttask += cs[j]->ttask_cap;
      cdr_wf_desc d{};
      d.ev_len = j == 0 ? S.n_ev[w] : S.n_nr[w];
      lens.push_back(d);
      lcaps.push_back(*cs[j]);
    }
  }
  uint32_t ns = 0;
  uint64_t rows = 0;
  cdr_plan_slices_ex(lens.data(), lcaps.data(), (uint32_t)lens.size(), p->plan_mode, nullptr, nullptr, nullptr,
                     nullptr, &ns, &rows, nullptr);
  z.n_slices = ns;
  z.n_rows = rows;
  *info = z;
  return CDR_API_OK;
}

// Fill the sliced columns (host buffers sized by the plan: columns n_rows*64,
// lane_wf n_slices*64, slice_len/row0 n_slices, arena arena_words) plus per-entry
// descriptors and output capacities, and the kv/reset-point tables.
int cdr_synth_sliced_fill(const cdr_synth_params* p, cdr_slices* o, cdr_wf_desc* wfs, cdr_wf_caps* caps,
                          cdr_kv* kvs, cdr_reset_point* rps, cdr_batch* meta, int threads) {
  if (!p || !o || !wfs || !caps || !meta) return CDR_API_EINVAL;
  if (p->plan_mode && !o->slice_flags) return CDR_API_EINVAL;  // wave slices are marked there
  Sizes S;
  size_pass(*p, S, threads, true);
  const uint32_t nw = p->n_wfs;
  std::vector<uint32_t> ent_base(nw);
  std::vector<uint64_t> kv_base(nw), rp_base(nw);
  uint32_t ent = 0;
  uint64_t kv = 0, rp = 0;
  std::vector<cdr_wf_desc> lens;
  std::vector<uint64_t> arena_base;
  uint64_t ab = 0;
  cdr_totals t{};
  for (uint32_t w = 0; w < nw; w++) {
    ent_base[w] = ent;
    kv_base[w] = kv;
    rp_base[w] = rp;
    kv += S.n_kv[w];
    rp += S.n_rp[w];
    const int m = S.has_nr[w] ? 2 : 1;
    for (int j = 0; j < m; j++) {
      cdr_wf_caps c = j == 0 ? S.cap_ev[w] : S.cap_nr[w];
      c.act_off = t.act;
      t.act += c.act_cap;
      c.timer_off = t.timer;
      t.timer += c.timer_cap;
      c.child_off = t.child;
      t.child += c.child_cap;
      c.cancel_off = t.cancel;
      t.cancel += c.cancel_cap;
      c.signal_off = t.signal;
      t.signal += c.signal_cap;
      c.vh_off = t.vh;
      t.vh += c.vh_cap;
      c.rp_off = t.rp;
      t.rp += c.rp_cap;
      c.sa_off = t.sa;
      t.sa += c.sa_cap;
      c.xfer_off = t.xfer;
      t.xfer += c.xfer_cap;
      c.ttask_off = t.ttask;
      t.ttask += c.ttask_cap;
      caps[ent + j] = c;
      cdr_wf_desc d{};
      d.ev_len = j == 0 ? S.n_ev[w] : S.n_nr[w];
      lens.push_back(d);
      arena_base.push_back(ab);
      ab += j == 0 ? S.aw_ev[w] : S.aw_nr[w];
    }
    ent += m;
  }
  if (ab > o->arena_words || ab >= (1ull << 32)) return CDR_API_EINVAL;  // u32 arena offsets (cdr.h)
  uint32_t ns = 0;
  uint64_t rows = 0;
  int rc = cdr_plan_slices_ex(lens.data(), caps, ent, p->plan_mode, const_cast<int32_t*>(o->lane_wf),
                              const_cast<uint32_t*>(o->slice_len), const_cast<uint64_t*>(o->slice_row0),
                              const_cast<uint32_t*>(o->slice_flags), &ns, &rows, nullptr);
  if (rc) return rc;
  if (ns != o->n_slices || rows != o->n_rows) return CDR_API_EINVAL;
  if (o->slice_scratch_off && o->slice_act_slots && o->slice_tim_slots) {
    uint64_t words = 0;
    rc = cdr_plan_scratch(caps, o->lane_wf, ns, const_cast<uint64_t*>(o->slice_scratch_off),
                          const_cast<uint32_t*>(o->slice_act_slots), const_cast<uint32_t*>(o->slice_tim_slots),
                          const_cast<uint32_t*>(o->slice_flags), &words, nullptr);
    if (rc) return rc;
  }
  // entry -> (slice, lane)
  std::vector<uint32_t> where(ent);
  for (uint32_t i = 0; i < ns * (uint32_t)CDR_SLICE_WIDTH; i++)
    if (o->lane_wf[i] >= 0) where[o->lane_wf[i]] = i;
  // empty lanes of lane slices (wave slices pad their own last row)
  auto is_wave = [&](uint32_t s) { return o->slice_flags && (o->slice_flags[s] & CDR_SLICE_WAVE); };
  for (uint32_t i = 0; i < ns * (uint32_t)CDR_SLICE_WIDTH; i++) {
    const uint32_t s = i / CDR_SLICE_WIDTH;
    if (o->lane_wf[i] < 0 && !is_wave(s))
      cdr_internal::pack_lane(nullptr, 0, o->slice_row0[s], o->slice_len[s], i % CDR_SLICE_WIDTH, 0, o);
  }
  auto pack = [&](const std::vector<cdr_event>& ev, uint32_t at, uint64_t apos) {
    const uint32_t s = at / CDR_SLICE_WIDTH;
    if (is_wave(s))
      cdr_internal::pack_chunked(ev.data(), ev.size(), o->slice_row0[s], o->slice_len[s], apos, o);
    else
      cdr_internal::pack_lane(ev.data(), ev.size(), o->slice_row0[s], o->slice_len[s], at % CDR_SLICE_WIDTH, apos, o);
  };
  par(nw, threads, [&](uint32_t w) {
    WfOut g;
    gen_one(*p, w, g);
    rebase(g.ev, (uint32_t)kv_base[w], (uint32_t)rp_base[w]);
    rebase(g.newrun, (uint32_t)kv_base[w], (uint32_t)rp_base[w]);
    if (kvs) std::copy(g.kvs.begin(), g.kvs.end(), kvs + kv_base[w]);
    if (rps) std::copy(g.rps.begin(), g.rps.end(), rps + rp_base[w]);
    const uint32_t i = ent_base[w];
    cdr_wf_desc d = g.d;
    d.ev_off = 0;
    d.ev_len = g.ev.size();
    pack(g.ev, where[i], arena_base[i]);
    if (g.has_newrun) {
      d.newrun = (int32_t)(i + 1);
      cdr_wf_desc n = g.d;
      n.wf_key = cdr_mix64(g.d.wf_key ^ CDR_UUID_NEWRUN_KEY);
      n.ev_off = 0;
      n.ev_len = g.newrun.size();
      n.run_id = wf_handle(global_index(*p, w), 30);
      n.request_id = wf_handle(global_index(*p, w), 12);
      n.builder = g.newrun_ndc ? CDR_BUILDER_NDC : CDR_BUILDER_2DC;
      n.expected_next_event_id = 0;
      n.parent = (int32_t)i;
      n.newrun = -1;
      n.newrun_call = 0;
      n.newrun_ndc = 0;
      wfs[i + 1] = n;
      pack(g.newrun, where[i + 1], arena_base[i + 1]);
    }
    wfs[i] = d;
  });
  std::memset(meta, 0, sizeof(*meta));
  meta->n_wfs = ent;
  meta->empty_uuid = H_EMPTY_UUID;
  meta->n_kvs = kv;
  meta->n_rps = rp;
  cluster_meta(&meta->cluster);
  meta->now_ns = 1700000000000000000ll;
  meta->uuid_seed = p->seed * 0x9E3779B97F4A7C15ull + 1;
  return CDR_API_OK;
}

// Planned event count of every workflow of the population (index_map ignored: global
// indices 0..n-1), without generating it: the walk's target length (the generated
// history ends within a few events of it) — the weights of the shard->GPU assignment.
int cdr_synth_weights(const cdr_synth_params* p, uint64_t n, uint32_t* out) {
  if (!p || !out) return CDR_API_EINVAL;
  par((uint32_t)n, 0, [&](uint32_t w) {
    Rng r2(p->seed ^ cdr_mix64(0xB17D + (uint64_t)w));
    out[w] = plan_one(*p, w, r2).target;
  });
  return CDR_API_OK;
}

int cdr_synth_ndc_tasks(const cdr_synth_params* p, int fork, cdr_ndc_task* tasks, cdr_vh_item* items,
                        uint32_t items_cap) {
  if (!p || !tasks || !items || (fork != 0 && fork != 1)) return CDR_API_EINVAL;
  std::atomic<int> bad{0};
  cdr_synth_params q = *p;
  q.ndc_part = CDR_SYNTH_PART_BASE;
  par(p->n_wfs, 0, [&](uint32_t w) {
    WfOut o;
    gen_one(q, w, o);
    cdr_ndc_task t{};
    t.items_off = (uint64_t)w * items_cap;
    if (o.forked) {
      cdr_vh_item* it = items + t.items_off;
      uint32_t n = 0;
      bool ok = true;
      auto add = [&](int64_t id, int64_t v) {  // AddOrUpdateItem on a well-formed history
        if (n > 0 && it[n - 1].version == v) {
          it[n - 1].event_id = id;
        } else if (n < items_cap) {
          it[n++] = cdr_vh_item{id, v};
        } else {
          ok = false;
        }
      };
      for (int64_t k = 0; k < o.fork_F; k++) add(o.ev[k].event_id, o.ev[k].version);
      const std::vector<cdr_event>& f = o.fork[fork];
      for (const cdr_event& e : f) add(e.event_id, e.version);
      if (!ok) bad = 1;
      t.n_items = n;
      t.first_event_id = f.empty() ? 0 : f.front().event_id;
      t.last_event_id = f.empty() ? 0 : f.back().event_id;
      t.last_version = f.empty() ? 0 : f.back().version;
      t.version = o.fork_ver[fork];
      uint64_t lo, hi;
      cdr_uuid(p->seed, o.d.wf_key, CDR_UUID_FORK, fork, &lo, &hi);
      t.new_token.tree = o.d.run_id;
      t.new_token.branch_lo = lo;
      t.new_token.branch_hi = hi;
    }
    tasks[w] = t;
  });
  return bad ? CDR_API_EINVAL : CDR_API_OK;
}

int cdr_synth_shards(uint64_t n, int32_t num_shards, int32_t* out) {
  if (!out || num_shards <= 0) return CDR_API_EINVAL;
  par((uint32_t)n, 0, [&](uint32_t i) {
    char buf[32];
    int len = snprintf(buf, sizeof buf, "wf-%u", i);
    out[i] = cdr_workflow_id_to_shard(buf, (size_t)len, num_shards);
  });
  return CDR_API_OK;
}

}  // extern "C"
