// replay.hip — MI355X (gfx950) kernels of the batched workflow-history replay engine.
//
// Reference hot path: stateBuilderImpl.applyEvents (service/history/stateBuilder.go:
// 112-611) driving mutableStateBuilder.Replicate*Event, one goroutine per workflow.
//
// MI355X design (DESIGN.md has the full argument):
//   * Input arrives in the sliced layout of cdr.h: 64 workflows of similar length per
//     slice, event k of all 64 stored contiguously per column.  One wavefront owns one
//     slice, one lane owns one workflow; at step k the wave loads event k of its 64
//     workflows with fully coalesced 256-512 B column loads.  A column is only loaded
//     when some lane's event type needs it, so HBM traffic tracks the algorithmic bytes.
//   * Per-workflow scalar state (ExecutionInfo, decision FSM, version history head,
//     replication state, call bookkeeping) lives in VGPRs for the whole history.
//   * Pending entities live in the workflow's slot range of the output tables
//     (capacity planned on the host); a deleted entity frees its slot and the next
//     creation reuses the lowest free slot, so a steady-state workflow keeps touching
//     the same few L2-resident lines and only its final rows reach HBM.
//   * The order-dependent timer picks (timerBuilder.go:171-312) are a min-scan over the
//     workflow's live slots after each activity/timer event.
//   * Errors: the first error/panic of a workflow stops it (the caller discards the
//     mutable state); its code and event are reported per workflow.
//   * Continue-as-new runs are separate lanes; k_finalize stitches their status into
//     the parent afterwards (stateBuilder.go:537-595).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "cdr/cdr.h"

#define DEAD_KEY ((int64_t)0x8000000000000000ll)
#define AI_IN_AID_MAP 0x80000000u /* kernel-private: this row holds byActivityID[aid] */
#define NS_PER_S 1000000000ll

namespace {

struct Ctl {  // per-lane scalar replay state (all in registers)
  int32_t err;
  int64_t err_id, err_k;
  bool dead;
};

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

__device__ __forceinline__ int cluster_for_version(const cdr_cluster_meta& m, int64_t v) {
  if (v == CDR_EMPTY_VERSION) return m.current_cluster;
  int64_t init = v % m.failover_version_increment;
  int r = -1;
#pragma unroll
  for (int i = 0; i < CDR_MAX_CLUSTERS; i++)
    if (i < m.n_clusters && m.initial_version[i] == init && r < 0) r = i;
  return r;
}

// activity timer pick over the live slots (timerBuilder.go:211-312): head candidate by
// (time, scheduleID, candidate order); OR its bit into TimerTaskStatus if not set.
__device__ void activity_timer_pick(cdr_activity_info* rows, uint32_t hw) {
  int best = -1;
  int64_t bt = 0, bs = 0;
  int bo = 0;
  int32_t bbit = 0;
  for (uint32_t j = 0; j < hw; j++) {
    const cdr_activity_info& r = rows[j];
    const int64_t sched = r.schedule_id;
    if (sched == DEAD_KEY) continue;
    int64_t t = r.scheduled_time + (int64_t)r.s2c * NS_PER_S;
    if (r.expiration_time < t) t = r.expiration_time;  // ExpirationTime is always set on replay
    int o = 0;
    int32_t bit = CDR_TTS_SCHEDULE_TO_CLOSE;
    int64_t t2, t3 = 0;
    int32_t bit2;
    bool has3 = false;
    if (r.started_id != CDR_EMPTY_EVENT_ID) {
      const int64_t st = r.started_time;
      t2 = st + (int64_t)r.stc * NS_PER_S;
      bit2 = CDR_TTS_START_TO_CLOSE;
      if (r.hb > 0) {
        int64_t lhb = r.last_heartbeat_time;
        if (lhb < st) lhb = st;
        t3 = lhb + (int64_t)r.hb * NS_PER_S;
        has3 = true;
      }
    } else {
      t2 = r.scheduled_time + (int64_t)r.s2s * NS_PER_S;
      bit2 = CDR_TTS_SCHEDULE_TO_START;
    }
    // best of this activity (append order breaks ties: S2C, then STC/S2S, then HB)
    if (t2 < t) {
      t = t2;
      o = 1;
      bit = bit2;
    }
    if (has3 && t3 < t) {
      t = t3;
      o = 2;
      bit = CDR_TTS_HEARTBEAT;
    }
    if (best < 0 || t < bt || (t == bt && (sched < bs || (sched == bs && o < bo)))) {
      best = (int)j;
      bt = t;
      bs = sched;
      bo = o;
      bbit = bit;
    }
  }
  if (best >= 0) {
    int32_t st = rows[best].timer_task_status;
    if (!(st & bbit)) rows[best].timer_task_status = st | bbit;
  }
}

// user timer pick (timerBuilder.go:171-184,233-247): head by (ExpiryTime, StartedID)
__device__ void user_timer_pick(cdr_timer_info* rows, uint32_t hw) {
  int best = -1;
  int64_t be = 0, bs = 0;
  for (uint32_t j = 0; j < hw; j++) {
    const int64_t s = rows[j].started_id;
    if (s == DEAD_KEY) continue;
    const int64_t e = rows[j].expiry_time;
    if (best < 0 || e < be || (e == be && s < bs)) {
      best = (int)j;
      be = e;
      bs = s;
    }
  }
  if (best >= 0 && rows[best].task_id != CDR_TIMER_TASK_STATUS_CREATED)
    rows[best].task_id = CDR_TIMER_TASK_STATUS_CREATED;
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

template <class Row>
__device__ __forceinline__ int find_initiated(const Row* rows, uint32_t hw, int64_t id) {
  for (uint32_t j = 0; j < hw; j++)
    if (rows[j].initiated_id == id) return (int)j;
  return -1;
}
template <class Row>
__device__ __forceinline__ int alloc_initiated(const Row* rows, uint32_t& hw, uint32_t cap) {
  for (uint32_t j = 0; j < hw; j++)
    if (rows[j].initiated_id == DEAD_KEY) return (int)j;
  if (hw < cap) return (int)(hw++);
  return -1;
}

}  // namespace

// ============================================================== replay kernel
__global__ __launch_bounds__(256) void k_replay(cdr_dev_batch B, cdr_out O) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t s = g >> 6;
  if (s >= B.ev.n_slices) return;
  const int32_t w = B.ev.lane_wf[g];
  if (w < 0) return;
  const cdr_wf_desc d = B.wfs[w];
  const cdr_wf_caps cp = B.caps[w];
  const uint32_t len = (uint32_t)d.ev_len;
  const uint64_t base = B.ev.slice_row0[s] * CDR_SLICE_WIDTH + (g & 63);
  const uint32_t EU = B.empty_uuid;

  cdr_activity_info* act = O.act + cp.act_off;
  cdr_timer_info* tim = O.timer + cp.timer_off;
  cdr_child_info* chi = O.child + cp.child_off;
  cdr_cancel_info* can = O.cancel + cp.cancel_off;
  cdr_signal_info* sig = O.signal + cp.signal_off;
  cdr_vh_item* vh = O.vh + cp.vh_off;
  cdr_reset_point* rp = O.rp + cp.rp_off;
  cdr_kv* sa = O.sa + cp.sa_off;
  cdr_repl_state* RS = O.repl + w;

  const bool isRS = d.builder == CDR_BUILDER_2DC;
  const bool isVH = d.builder == CDR_BUILDER_NDC;

  // ---- ExecutionInfo (mutableStateBuilder.go:185-196 defaults)
  uint32_t x_create_req = 0, x_task_list = 0, x_wf_type = 0, x_cron = 0, x_pdom = 0, x_pwf = 0, x_prun = 0,
           x_memo = 0, x_nonretr = 0, x_flags = 0;
  int64_t x_initiated = 0, x_completion_batch = 0, x_last_first = 0, x_last_task = 0,
          x_next_event = CDR_FIRST_EVENT_ID, x_last_processed = CDR_EMPTY_EVENT_ID;
  int32_t x_wf_timeout = 0, x_dt_timeout_value = 0, x_state = CDR_STATE_CREATED, x_close = CDR_CLOSE_NONE,
          x_signals = 0, x_attempt = 0, x_init_int = 0, x_max_int = 0, x_max_att = 0, x_exp_s = 0;
  double x_backoff = 0.0;
  int64_t x_exp_time = 0;
  uint64_t x_br_lo = 0, x_br_hi = 0;
  // decision (decisionInfo)
  int64_t dv = CDR_EMPTY_VERSION, dsched = CDR_EMPTY_EVENT_ID, dstart = CDR_EMPTY_EVENT_ID, datt = 0, dst_ts = 0,
          dsc_ts = 0, dorig_ts = 0;
  uint32_t dreq = EU;
  int32_t dto = 0;
  // versions
  int64_t curv = d.failover_version;  // NDC currentVersion
  int64_t rs_cur = d.failover_version, rs_start = d.failover_version, rs_lwv = CDR_EMPTY_VERSION,
          rs_lwid = CDR_EMPTY_EVENT_ID;
  uint32_t rs_mask = 0;
  int64_t vh_last_id = 0, vh_last_ver = 0;
  uint32_t n_vh = 0;
  // tables
  uint32_t hw_act = 0, hw_tim = 0, hw_chi = 0, hw_can = 0, hw_sig = 0;
  uint32_t live_chi = 0, live_can = 0, live_sig = 0;
  uint32_t n_rp = 0, n_sa = 0;
  // calls / errors
  int64_t call_first_id = 0, call_first_k = 0, prev_id = 0, prev_ver = 0;
  uint32_t call_idx = 0;
  bool newrun_applied = false;
  int32_t err = CDR_OK;
  int64_t err_id = 0, err_k = 0;
  bool stop_at_call_end = false;

#define FAIL(code)             \
  do {                         \
    err = (code);              \
    err_id = e_id;             \
    err_k = k;                 \
    stop_at_call_end = true;   \
  } while (0)

  // close the call that ended with event (prev_id, prev_ver): stateBuilder.go:603-604
  // plus the replication-state writes whose source is the call's last event
  // (UpdateReplicationStateLastEventID mutableStateBuilder.go:561-581).
  auto finish_call = [&]() {
    if (isRS) {
      rs_lwv = prev_ver;
      rs_lwid = prev_id;
      const int src = cluster_for_version(B.cluster, prev_ver);
      if (src < 0) {
        // the panic fires at the call's first event, before anything else in the call
        err = CDR_P_UNKNOWN_CLUSTER;
        err_id = call_first_id;
        err_k = call_first_k;
        return;
      }
      if (src != B.cluster.current_cluster) {
        RS->lri_version[src] = prev_ver;
        RS->lri_last_event_id[src] = prev_id;
        rs_mask |= 1u << src;
      }
    }
    if (err == CDR_OK) {
      x_last_first = call_first_id;
      x_next_event = prev_id + 1;
    }
  };

  if (len == 0) err = CDR_E_HISTORY_EMPTY;

  for (uint32_t k = 0; k < len; k++) {
    const uint64_t i = base + (uint64_t)k * CDR_SLICE_WIDTH;
    const uint32_t tf = B.ev.type_flags[i];
    const uint32_t type = tf & 0xFFu;
    const int64_t e_id = B.ev.event_id[i];
    const int64_t e_ver = B.ev.version[i];
    if ((tf & CDR_SEF_BATCH_FIRST) || k == 0) {
      if (k > 0) {
        finish_call();
        if (err != CDR_OK) break;
        call_idx++;
      }
      call_first_id = e_id;
      call_first_k = k;
    } else if (stop_at_call_end) {
      prev_id = e_id;
      prev_ver = e_ver;
      continue;  // skip the rest of the failed call; only its last event matters for 2DC
    }
    prev_id = e_id;
    prev_ver = e_ver;
    if (stop_at_call_end) continue;

    // ---- version prelude (stateBuilder.go:134-154)
    if (isRS) {
      rs_cur = e_ver;  // UpdateReplicationStateVersion(v, true)
    } else if (isVH) {
      if (x_state == CDR_STATE_CREATED || x_state == CDR_STATE_RUNNING) {
        if (n_vh) curv = vh_last_ver;  // UpdateCurrentVersion (:445-489)
        curv = e_ver;
      }
      // NewVersionHistoryItem + AddOrUpdateItem (versionHistory.go:31-42,203-236)
      if (e_id < 0 || (e_ver < 0 && e_ver != CDR_EMPTY_VERSION)) {
        FAIL(CDR_P_VH_ITEM_INVALID);
        continue;
      }
      if (n_vh == 0) {
        if (cp.vh_cap == 0) {
          FAIL(CDR_E_BAD_INPUT);
          continue;
        }
        vh[0] = cdr_vh_item{e_id, e_ver};
        n_vh = 1;
        vh_last_id = e_id;
        vh_last_ver = e_ver;
      } else {
        if (e_ver < vh_last_ver) {
          FAIL(CDR_E_VH_LOWER_VERSION);
          continue;
        }
        if (e_id <= vh_last_id) {
          FAIL(CDR_E_VH_LOWER_EVENT_ID);
          continue;
        }
        if (e_ver > vh_last_ver) {
          if (n_vh >= cp.vh_cap) {
            FAIL(CDR_E_BAD_INPUT);
            continue;
          }
          vh[n_vh++] = cdr_vh_item{e_id, e_ver};
        } else {
          vh[n_vh - 1].event_id = e_id;
        }
        vh_last_id = e_id;
        vh_last_ver = e_ver;
      }
    }
    x_last_task = B.ev.task_id[i];  // :155

    switch (type) {
      case CDR_EV_WF_STARTED: {  // stateBuilder.go:158-184 -> mutableStateBuilder.go:1639-1716
        const cdr_attr_wf_started* a =
            reinterpret_cast<const cdr_attr_wf_started*>(B.ev.arena + (uint64_t)B.ev.aux[i]);
        const uint32_t af = a->flags;
        if ((af & CDR_SF_HAS_PARENT_DOMAIN) && (af & CDR_SF_PARENT_DOMAIN_MISSING)) {
          FAIL(CDR_E_DOMAIN_NOT_FOUND);
          break;
        }
        x_create_req = d.request_id;
        x_task_list = a->task_list;
        x_wf_type = a->workflow_type;
        x_wf_timeout = a->exec_timeout_s;
        x_dt_timeout_value = a->task_timeout_s;
        if (!transition_ok(x_state, x_close, CDR_STATE_CREATED, CDR_CLOSE_NONE)) {
          FAIL(CDR_E_INVALID_STATE_TRANSITION);
          break;
        }
        x_state = CDR_STATE_CREATED;
        x_close = CDR_CLOSE_NONE;
        x_last_processed = CDR_EMPTY_EVENT_ID;
        x_last_first = e_id;
        dv = CDR_EMPTY_VERSION;
        dsched = CDR_EMPTY_EVENT_ID;
        dstart = CDR_EMPTY_EVENT_ID;
        dreq = EU;
        dto = 0;
        x_cron = a->cron_schedule;
        if (af & CDR_SF_HAS_PARENT_DOMAIN) x_pdom = a->parent_domain_id;
        if (af & CDR_SF_HAS_PARENT_EXEC) {
          x_pwf = a->parent_workflow_id;
          x_prun = a->parent_run_id;
        }
        x_initiated = (af & CDR_SF_HAS_PARENT_INITIATED) ? a->parent_initiated_id : CDR_EMPTY_EVENT_ID;
        x_attempt = a->attempt;
        if (a->expiration_ts != 0) {
          x_exp_time = a->expiration_ts;
          x_flags |= CDR_XI_HAS_EXPIRATION;
        }
        if (af & CDR_SF_HAS_RETRY) {
          x_flags |= CDR_XI_HAS_RETRY;
          x_backoff = a->backoff_coefficient;
          x_exp_s = a->retry_expiration_s;
          x_init_int = a->retry_initial_s;
          x_max_att = a->retry_max_attempts;
          x_max_int = a->retry_max_interval_s;
          x_nonretr = a->nonretriable;
        }
        // rolloverAutoResetPointsWithExpiringTime (:3184-3205)
        n_rp = 0;
        x_flags &= ~CDR_XI_HAS_RESET_POINTS;
        if (af & CDR_SF_HAS_RESET_POINTS) {
          x_flags |= CDR_XI_HAS_RESET_POINTS;
          const int64_t expiring = B.ev.timestamp[i] + (int64_t)d.retention_days * 24ll * 3600ll * NS_PER_S;
          for (uint32_t q = 0; q < a->reset_points_len && q < cp.rp_cap; q++) {
            cdr_reset_point p = B.rps[a->reset_points_off + q];
            const uint32_t run = (p.flags & CDR_RP_HAS_RUN_ID) ? p.run_id : 0u;
            if (run == a->continued_run_id) {
              p.flags |= CDR_RP_HAS_EXPIRING;
              p.expiring_time_nano = expiring;
            }
            rp[n_rp++] = p;
          }
        }
        if (af & CDR_SF_HAS_MEMO) {
          x_flags |= CDR_XI_HAS_MEMO;
          x_memo = a->memo;
        }
        if (af & CDR_SF_HAS_SEARCH_ATTR) {
          n_sa = 0;
          for (uint32_t q = 0; q < a->search_attr_len && q < cp.sa_cap; q++) sa[n_sa++] = B.kvs[a->search_attr_off + q];
          if (n_sa) x_flags |= CDR_XI_HAS_SEARCH_ATTR;
          else x_flags &= ~CDR_XI_HAS_SEARCH_ATTR;
        }
        x_flags |= CDR_XI_STARTED;
        // SetHistoryTree (:313-339): branch token on ExecutionInfo, or on the VH for NDC
        cdr_uuid(B.uuid_seed, d.wf_key, CDR_UUID_BRANCH, e_id, &x_br_lo, &x_br_hi);
        x_flags |= isVH ? CDR_XI_VH_BRANCH : CDR_XI_HAS_BRANCH;
        if (isRS) rs_start = e_ver;  // :182-184
        break;
      }
      case CDR_EV_DT_SCHEDULED:  // :186-200 -> mutableStateDecisionTaskManager.go:143-167
        dv = e_ver;
        dsched = e_id;
        dstart = CDR_EMPTY_EVENT_ID;
        dreq = EU;
        dto = B.ev.n[i];
        datt = B.ev.aux[i];
        dsc_ts = B.ev.timestamp[i];
        dst_ts = 0;
        dorig_ts = dsc_ts;
        break;
      case CDR_EV_DT_STARTED: {  // :202-213 -> :200-253
        const int64_t sid = B.ev.key[i];
        if (sid != dsched) {
          FAIL(CDR_E_DECISION_NOT_FOUND);
          break;
        }
        if (x_state == CDR_STATE_CREATED) {
          // Created -> Running is always accepted (workflowExecutionInfo.go:56-60)
          x_state = CDR_STATE_RUNNING;
          x_close = CDR_CLOSE_NONE;
        }
        dv = e_ver;
        dstart = e_id;
        dreq = B.ev.h[i];
        datt = 0;
        dst_ts = B.ev.timestamp[i];
        break;
      }
      case CDR_EV_DT_COMPLETED: {  // :215-219 -> :255-262,659-674,789-800
        dv = CDR_EMPTY_VERSION;
        dsched = CDR_EMPTY_EVENT_ID;
        dstart = CDR_EMPTY_EVENT_ID;
        dreq = EU;
        dto = 0;
        datt = 0;
        dst_ts = 0;
        dsc_ts = 0;  // OriginalScheduledTimestamp kept
        x_last_processed = B.ev.aux[i];
        const uint32_t cks = B.ev.h[i];
        if (cks) {  // addBinaryCheckSumIfNotExists (mutableStateBuilder.go:1798-1842)
          bool exists = false;
          for (uint32_t q = 0; q < n_rp; q++) {
            const uint32_t c = (rp[q].flags & CDR_RP_HAS_CHECKSUM) ? rp[q].binary_checksum : 0u;
            exists |= c == cks;
          }
          if (!exists) {
            if (n_rp >= cp.rp_cap) {
              FAIL(CDR_E_BAD_INPUT);
              break;
            }
            const bool resettable = live_chi == 0 && live_can == 0 && live_sig == 0;
            cdr_reset_point p;
            p.binary_checksum = cks;
            p.run_id = d.run_id;
            p.first_decision_completed_id = e_id;
            p.created_time_nano = B.now_ns;
            p.expiring_time_nano = 0;
            p.flags = CDR_RP_HAS_CHECKSUM | CDR_RP_HAS_RUN_ID | CDR_RP_HAS_FIRST_DC_ID | CDR_RP_HAS_CREATED |
                      CDR_RP_HAS_RESETTABLE | (resettable ? CDR_RP_RESETTABLE : 0u);
            p._pad = 0;
            rp[n_rp++] = p;
            x_flags |= CDR_XI_HAS_RESET_POINTS;
          }
        }
        break;
      }
      case CDR_EV_DT_TIMED_OUT:  // :221-239 -> FailDecision :635-656 + transient :169-198
      case CDR_EV_DT_FAILED: {   // :241-257
        const bool inc = type == CDR_EV_DT_FAILED || B.ev.n[i] != CDR_TIMEOUT_SCHEDULE_TO_START;
        const int64_t a1 = inc ? datt + 1 : 0;
        dv = CDR_EMPTY_VERSION;
        dsched = CDR_EMPTY_EVENT_ID;
        dstart = CDR_EMPTY_EVENT_ID;
        dreq = EU;
        dto = 0;
        dst_ts = 0;
        dorig_ts = 0;
        datt = a1;
        dsc_ts = inc ? B.now_ns : 0;
        if (datt != 0) {  // no pending decision here by construction
          dv = isRS ? rs_cur : (isVH ? curv : CDR_EMPTY_VERSION);
          dsched = x_next_event;  // NextEventID as of the call's start
          dto = x_dt_timeout_value;
          dsc_ts = B.now_ns;
        }
        break;
      }
      case CDR_EV_AT_SCHEDULED: {  // :259-269 -> mutableStateBuilder.go:1982-2028
        const cdr_attr_at_scheduled* a =
            reinterpret_cast<const cdr_attr_at_scheduled*>(B.ev.arena + (uint64_t)B.ev.aux[i]);
        const uint32_t aid = (uint32_t)B.ev.key[i];
        int slot = -1;
        for (uint32_t j = 0; j < hw_act; j++) {
          if (act[j].schedule_id == DEAD_KEY) {
            if (slot < 0) slot = (int)j;
          } else if (act[j].activity_id == aid && (act[j].flags & AI_IN_AID_MAP)) {
            act[j].flags &= ~AI_IN_AID_MAP;  // byActivityID[aid] is overwritten
          }
        }
        if (slot < 0) {
          if (hw_act >= cp.act_cap) {
            FAIL(CDR_E_BAD_INPUT);
            break;
          }
          slot = (int)hw_act++;
        }
        const int64_t ts = B.ev.timestamp[i];
        cdr_activity_info r;
        r.version = e_ver;
        r.schedule_id = e_id;
        r.scheduled_event_batch_id = call_first_id;
        r.scheduled_time = ts;
        r.started_id = CDR_EMPTY_EVENT_ID;
        r.started_time = 0;
        r.last_heartbeat_time = 0;
        r.expiration_time = ts + (int64_t)a->s2c_s * NS_PER_S;
        r.cancel_request_id = CDR_EMPTY_EVENT_ID;
        r.activity_id = aid;
        r.request_id = 0;
        r.task_list = a->task_list;
        r.s2s = a->s2s_s;
        r.s2c = a->s2c_s;
        r.stc = a->stc_s;
        r.hb = a->hb_s;
        r.timer_task_status = CDR_TIMER_TASK_STATUS_NONE;
        r.attempt = 0;
        const bool retry = (a->flags & CDR_AF_HAS_RETRY) != 0;
        r.initial_interval = retry ? a->retry_initial_s : 0;
        r.maximum_interval = retry ? a->retry_max_interval_s : 0;
        r.maximum_attempts = retry ? a->retry_max_attempts : 0;
        r.nonretriable = retry ? a->nonretriable : 0u;
        r.backoff_coefficient = retry ? a->backoff_coefficient : 0.0;
        if (retry && a->retry_expiration_s > a->s2c_s) r.expiration_time = ts + (int64_t)a->retry_expiration_s * NS_PER_S;
        r.flags = (retry ? CDR_AI_HAS_RETRY : 0u) | AI_IN_AID_MAP;
        act[slot] = r;
        activity_timer_pick(act, hw_act);
        break;
      }
      case CDR_EV_AT_STARTED: {  // :271-278 -> :2083-2098
        const int64_t sid = B.ev.key[i];
        int slot = -1;
        for (uint32_t j = 0; j < hw_act; j++)
          if (act[j].schedule_id == sid) slot = (int)j;
        if (slot < 0) {
          FAIL(CDR_P_ACTIVITY_STARTED_NIL);  // nil deref in Go
          break;
        }
        const int64_t ts = B.ev.timestamp[i];
        act[slot].version = e_ver;
        act[slot].started_id = e_id;
        act[slot].request_id = B.ev.h[i];
        act[slot].started_time = ts;
        act[slot].last_heartbeat_time = ts;
        act[slot].flags |= CDR_AI_STARTED_TIME_SET;
        activity_timer_pick(act, hw_act);
        break;
      }
      case CDR_EV_AT_COMPLETED:  // :280-305,312-319 -> DeleteActivity :1247-1269
      case CDR_EV_AT_FAILED:
      case CDR_EV_AT_TIMED_OUT:
      case CDR_EV_AT_CANCELED: {
        const int64_t sid = B.ev.key[i];
        int slot = -1;
        for (uint32_t j = 0; j < hw_act; j++)
          if (act[j].schedule_id == sid) slot = (int)j;
        if (slot < 0) {
          FAIL(CDR_E_ACTIVITY_NOT_FOUND);
          break;
        }
        const uint32_t aid = act[slot].activity_id;
        const bool own = (act[slot].flags & AI_IN_AID_MAP) != 0;
        act[slot].schedule_id = DEAD_KEY;
        act[slot].flags &= ~AI_IN_AID_MAP;
        bool found = own;
        if (!own)
          for (uint32_t j = 0; j < hw_act; j++)
            if (act[j].schedule_id != DEAD_KEY && act[j].activity_id == aid && (act[j].flags & AI_IN_AID_MAP)) {
              act[j].flags &= ~AI_IN_AID_MAP;
              found = true;
            }
        if (!found) {
          FAIL(CDR_E_ACTIVITY_ID_NOT_FOUND);
          break;
        }
        activity_timer_pick(act, hw_act);
        break;
      }
      case CDR_EV_AT_CANCEL_REQUESTED: {  // :307-310 -> :2264-2285
        const uint32_t aid = (uint32_t)B.ev.key[i];
        int slot = -1;
        for (uint32_t j = 0; j < hw_act; j++)
          if (act[j].schedule_id != DEAD_KEY && act[j].activity_id == aid && (act[j].flags & AI_IN_AID_MAP))
            slot = (int)j;
        if (slot < 0) {
          FAIL(CDR_E_MISSING_ACTIVITY_INFO);
          break;
        }
        act[slot].version = e_ver;
        act[slot].flags |= CDR_AI_CANCEL_REQUESTED;
        act[slot].cancel_request_id = e_id;
        break;
      }
      case CDR_EV_TIMER_STARTED: {  // :324-332 -> :2877-2900
        const uint32_t tid = (uint32_t)B.ev.key[i];
        int slot = -1, free_slot = -1;
        for (uint32_t j = 0; j < hw_tim; j++) {
          if (tim[j].started_id == DEAD_KEY) {
            if (free_slot < 0) free_slot = (int)j;
          } else if (tim[j].timer_id == tid) {
            slot = (int)j;
          }
        }
        if (slot < 0) slot = free_slot;
        if (slot < 0) {
          if (hw_tim >= cp.timer_cap) {
            FAIL(CDR_E_BAD_INPUT);
            break;
          }
          slot = (int)hw_tim++;
        }
        cdr_timer_info t;
        t.version = e_ver;
        t.started_id = e_id;
        t.expiry_time = B.ev.timestamp[i] + B.ev.aux[i] * NS_PER_S;
        t.task_id = CDR_TIMER_TASK_STATUS_NONE;
        t.timer_id = tid;
        t._pad = 0;
        tim[slot] = t;
        user_timer_pick(tim, hw_tim);
        break;
      }
      case CDR_EV_TIMER_FIRED:     // :334-341
      case CDR_EV_TIMER_CANCELED: {  // :343-350
        const uint32_t tid = (uint32_t)B.ev.key[i];
        for (uint32_t j = 0; j < hw_tim; j++)
          if (tim[j].started_id != DEAD_KEY && tim[j].timer_id == tid) tim[j].started_id = DEAD_KEY;
        user_timer_pick(tim, hw_tim);
        break;
      }
      case CDR_EV_CHILD_INITIATED: {  // :355-371 -> :3256-3280
        int slot = alloc_initiated(chi, hw_chi, cp.child_cap);
        if (slot < 0) {
          FAIL(CDR_E_BAD_INPUT);
          break;
        }
        cdr_child_info c;
        c.version = e_ver;
        c.initiated_id = e_id;
        c.initiated_event_batch_id = call_first_id;
        c.started_id = CDR_EMPTY_EVENT_ID;
        cdr_uuid(B.uuid_seed, d.wf_key, CDR_UUID_CHILD_REQ, e_id, &c.create_request_lo, &c.create_request_hi);
        c.started_workflow_id = B.ev.h[i];
        c.started_run_id = 0;
        c.domain_name = (uint32_t)B.ev.key[i];
        c.workflow_type = (uint32_t)B.ev.aux[i];
        c.parent_close_policy = B.ev.n[i];
        c._pad = 0;
        chi[slot] = c;
        live_chi++;
        if (tf & CDR_SEF_DOMAIN_MISSING) FAIL(CDR_E_DOMAIN_NOT_FOUND);
        break;
      }
      case CDR_EV_CHILD_STARTED: {  // :378-381 -> :3312-3325
        const int slot = find_initiated(chi, hw_chi, B.ev.key[i]);
        if (slot < 0) {
          FAIL(CDR_P_CHILD_STARTED_NIL);
          break;
        }
        chi[slot].started_id = e_id;
        chi[slot].started_run_id = B.ev.h[i];
        break;
      }
      case CDR_EV_CHILD_START_FAILED:
      case CDR_EV_CHILD_COMPLETED:
      case CDR_EV_CHILD_FAILED:
      case CDR_EV_CHILD_CANCELED:
      case CDR_EV_CHILD_TIMED_OUT:
      case CDR_EV_CHILD_TERMINATED: {  // DeletePendingChildExecution :1138-1144
        const int slot = find_initiated(chi, hw_chi, B.ev.key[i]);
        if (slot >= 0) {
          chi[slot].initiated_id = DEAD_KEY;
          live_chi--;
        }
        break;
      }
      case CDR_EV_RCE_INITIATED: {  // :408-427 -> :2577-2596
        int slot = alloc_initiated(can, hw_can, cp.cancel_cap);
        if (slot < 0) {
          FAIL(CDR_E_BAD_INPUT);
          break;
        }
        cdr_cancel_info c;
        c.version = e_ver;
        c.initiated_event_batch_id = call_first_id;
        c.initiated_id = e_id;
        cdr_uuid(B.uuid_seed, d.wf_key, CDR_UUID_CANCEL_REQ, e_id, &c.cancel_request_lo, &c.cancel_request_hi);
        can[slot] = c;
        live_can++;
        if (tf & CDR_SEF_DOMAIN_MISSING) FAIL(CDR_E_DOMAIN_NOT_FOUND);
        break;
      }
      case CDR_EV_RCE_FAILED:
      case CDR_EV_EXT_CANCEL_REQUESTED: {  // DeletePendingRequestCancel :1147-1153
        const int slot = find_initiated(can, hw_can, B.ev.key[i]);
        if (slot >= 0) {
          can[slot].initiated_id = DEAD_KEY;
          live_can--;
        }
        break;
      }
      case CDR_EV_SE_INITIATED: {  // :439-458 -> :2701-2723
        int slot = alloc_initiated(sig, hw_sig, cp.signal_cap);
        if (slot < 0) {
          FAIL(CDR_E_BAD_INPUT);
          break;
        }
        const uint64_t io = (uint64_t)B.ev.aux[i];
        cdr_signal_info c;
        c.version = e_ver;
        c.initiated_event_batch_id = call_first_id;
        c.initiated_id = e_id;
        cdr_uuid(B.uuid_seed, d.wf_key, CDR_UUID_SIGNAL_REQ, e_id, &c.signal_request_lo, &c.signal_request_hi);
        c.signal_name = B.ev.h[i];
        c.input = (uint32_t)(io >> 32);
        c.control = (uint32_t)io;
        c._pad = 0;
        sig[slot] = c;
        live_sig++;
        if (tf & CDR_SEF_DOMAIN_MISSING) FAIL(CDR_E_DOMAIN_NOT_FOUND);
        break;
      }
      case CDR_EV_SE_FAILED:
      case CDR_EV_EXT_SIGNALED: {  // DeletePendingSignal :1156-1162
        const int slot = find_initiated(sig, hw_sig, B.ev.key[i]);
        if (slot >= 0) {
          sig[slot].initiated_id = DEAD_KEY;
          live_sig--;
        }
        break;
      }
      case CDR_EV_AT_REQ_CANCEL_FAILED:
      case CDR_EV_CANCEL_TIMER_FAILED:
      case CDR_EV_MARKER_RECORDED:
        break;
      case CDR_EV_WF_SIGNALED:  // :473-476
        x_signals++;
        break;
      case CDR_EV_WF_CANCEL_REQUESTED:  // :478-481
        x_flags |= CDR_XI_CANCEL_REQUESTED;
        break;
      case CDR_EV_WF_COMPLETED:
      case CDR_EV_WF_FAILED:
      case CDR_EV_WF_TIMED_OUT:
      case CDR_EV_WF_CANCELED:
      case CDR_EV_WF_TERMINATED: {  // :483-531
        const int cs = type == CDR_EV_WF_COMPLETED   ? CDR_CLOSE_COMPLETED
                       : type == CDR_EV_WF_FAILED    ? CDR_CLOSE_FAILED
                       : type == CDR_EV_WF_TIMED_OUT ? CDR_CLOSE_TIMED_OUT
                       : type == CDR_EV_WF_CANCELED  ? CDR_CLOSE_CANCELED
                                                     : CDR_CLOSE_TERMINATED;
        if (!transition_ok(x_state, x_close, CDR_STATE_COMPLETED, cs)) {
          FAIL(CDR_E_INVALID_STATE_TRANSITION);
          break;
        }
        x_state = CDR_STATE_COMPLETED;
        x_close = cs;
        x_completion_batch = call_first_id;
        break;
      }
      case CDR_EV_UPSERT_SA: {  // :533-535 -> :2746-2768
        const uint64_t off = (uint64_t)B.ev.aux[i];
        const uint32_t cnt = B.ev.h[i];
        for (uint32_t q = 0; q < cnt; q++) {
          const cdr_kv kv = B.kvs[off + q];
          bool found = false;
          for (uint32_t j = 0; j < n_sa; j++)
            if (sa[j].key == kv.key) {
              sa[j].value = kv.value;
              found = true;
            }
          if (!found) {
            if (n_sa >= cp.sa_cap) break;
            sa[n_sa++] = kv;
          }
        }
        x_flags |= CDR_XI_HAS_SEARCH_ATTR;
        break;
      }
      case CDR_EV_WF_CONTINUED_AS_NEW: {  // :537-595
        if (d.newrun < 0 || call_idx != d.newrun_call || B.wfs[d.newrun].ev_len == 0) {
          FAIL(CDR_E_NEWRUN_HISTORY_EMPTY);
          break;
        }
        newrun_applied = true;  // the new run replays in its own lane; k_finalize joins
        if (!transition_ok(x_state, x_close, CDR_STATE_COMPLETED, CDR_CLOSE_CONTINUED_AS_NEW)) {
          FAIL(CDR_E_INVALID_STATE_TRANSITION);
          break;
        }
        x_state = CDR_STATE_COMPLETED;
        x_close = CDR_CLOSE_CONTINUED_AS_NEW;
        x_completion_batch = call_first_id;
        break;
      }
      default:
        FAIL(CDR_E_UNKNOWN_EVENT_TYPE);  // :597-599
        break;
    }
  }
  if (len > 0 && err == CDR_OK) finish_call();
  else if (len > 0 && stop_at_call_end && isRS) {
    // a failed call still raises the cluster panic first if its last event's version is unknown
    const int src = cluster_for_version(B.cluster, prev_ver);
    if (src < 0) {
      err = CDR_P_UNKNOWN_CLUSTER;
      err_id = call_first_id;
      err_k = call_first_k;
    }
  }
  if (err == CDR_OK && d.parent < 0 && d.expected_next_event_id != 0 && x_next_event != d.expected_next_event_id) {
    err = CDR_E_REBUILD_NEXT_EVENT_ID;  // nDCStateRebuilder.go:139-143
    err_id = prev_id;
    err_k = len;
  }
#undef FAIL

  cdr_wf_result r;
  r.code = err;
  r.flags = newrun_applied ? CDR_RF_NEWRUN_APPLIED : 0u;
  if (d.parent >= 0) r.flags |= CDR_RF_IS_NEWRUN;
  r.fail_event_id = err_id;
  r.fail_index = err_k;
  r.n_activity = r.n_timer = r.n_child = r.n_cancel = r.n_signal = 0;
  r.n_vh = r.n_reset_points = r.n_search_attr = 0;
  if (err == CDR_OK) {
    r.n_activity = compact_sorted(act, hw_act, ActKey{});
    for (uint32_t j = 0; j < r.n_activity; j++) act[j].flags &= ~AI_IN_AID_MAP;
    r.n_timer = compact_sorted(tim, hw_tim, TimerKey{});
    r.n_child = compact_sorted(chi, hw_chi, ChildKey{});
    r.n_cancel = compact_sorted(can, hw_can, CancelKey{});
    r.n_signal = compact_sorted(sig, hw_sig, SignalKey{});
    r.n_vh = n_vh;
    r.n_reset_points = n_rp;
    // SearchAttributes is a Go map: canonical output order is ascending key
    for (uint32_t a = 1; a < n_sa; a++) {
      cdr_kv v = sa[a];
      uint32_t b = a;
      while (b > 0 && sa[b - 1].key > v.key) {
        sa[b] = sa[b - 1];
        b--;
      }
      sa[b] = v;
    }
    r.n_search_attr = n_sa;

    cdr_exec_info x;
    x.domain_id = (x_flags & CDR_XI_STARTED) ? d.domain_id : 0u;
    x.workflow_id = (x_flags & CDR_XI_STARTED) ? d.workflow_id : 0u;
    x.run_id = (x_flags & CDR_XI_STARTED) ? d.run_id : 0u;
    x.create_request_id = x_create_req;
    x.parent_domain_id = x_pdom;
    x.parent_workflow_id = x_pwf;
    x.parent_run_id = x_prun;
    x.task_list = x_task_list;
    x.workflow_type = x_wf_type;
    x.decision_request_id = dreq;
    x.cron_schedule = x_cron;
    x.memo = x_memo;
    x.nonretriable = x_nonretr;
    x.branch_tree_id = (x_flags & (CDR_XI_HAS_BRANCH | CDR_XI_VH_BRANCH)) ? d.run_id : 0u;
    x.flags = x_flags;
    x._pad0 = 0;
    x.initiated_id = x_initiated;
    x.completion_event_batch_id = x_completion_batch;
    x.workflow_timeout = x_wf_timeout;
    x.decision_timeout_value = x_dt_timeout_value;
    x.state = x_state;
    x.close_status = x_close;
    x.last_first_event_id = x_last_first;
    x.last_event_task_id = x_last_task;
    x.next_event_id = x_next_event;
    x.last_processed_event = x_last_processed;
    x.signal_count = x_signals;
    x.decision_timeout = dto;
    x.decision_version = dv;
    x.decision_schedule_id = dsched;
    x.decision_started_id = dstart;
    x.decision_attempt = datt;
    x.decision_started_ts = dst_ts;
    x.decision_scheduled_ts = dsc_ts;
    x.decision_original_scheduled_ts = dorig_ts;
    x.attempt = x_attempt;
    x.initial_interval = x_init_int;
    x.backoff_coefficient = x_backoff;
    x.maximum_interval = x_max_int;
    x.maximum_attempts = x_max_att;
    x.expiration_time = x_exp_time;
    x.expiration_seconds = x_exp_s;
    x._pad1 = 0;
    x.branch_id_lo = x_br_lo;
    x.branch_id_hi = x_br_hi;
    x.reset_points_len = n_rp;
    x.search_attr_len = n_sa;
    O.exec[w] = x;
    if (isRS) {
      RS->current_version = rs_cur;
      RS->start_version = rs_start;
      RS->last_write_version = rs_lwv;
      RS->last_write_event_id = rs_lwid;
      for (int c = 0; c < CDR_MAX_CLUSTERS; c++)
        if (!(rs_mask & (1u << c))) {
          RS->lri_version[c] = 0;
          RS->lri_last_event_id[c] = 0;
        }
      RS->lri_mask = rs_mask;
      RS->present = 1;
    } else {
      cdr_repl_state z = {};
      *RS = z;
    }
  }
  O.result[w] = r;
}

// continue-as-new stitching (stateBuilder.go:557-574): a parent that applied its new
// run inherits the new run's error; a new run its parent never reached is NOT_APPLIED.
__global__ void k_finalize(cdr_dev_batch B, cdr_out O) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= B.n_wfs) return;
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
struct cdr_ctx {
  int device;
  hipEvent_t ev[4];
  float replay_ms, finalize_ms;
  bool timed;
};

#define HIPCHK(x)                                                                      \
  do {                                                                                 \
    hipError_t _e = (x);                                                               \
    if (_e != hipSuccess) {                                                            \
      fprintf(stderr, "cdr: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(_e), __FILE__, __LINE__); \
      return CDR_API_EDEVICE;                                                          \
    }                                                                                  \
  } while (0)

extern "C" {

cdr_ctx* cdr_create(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= device || device < 0) return nullptr;
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  cdr_ctx* c = new cdr_ctx();
  c->device = device;
  for (int i = 0; i < 4; i++)
    if (hipEventCreate(&c->ev[i]) != hipSuccess) {
      delete c;
      return nullptr;
    }
  c->timed = false;
  return c;
}

void cdr_destroy(cdr_ctx* c) {
  if (!c) return;
  for (int i = 0; i < 4; i++) (void)hipEventDestroy(c->ev[i]);
  delete c;
}

int cdr_replay_sliced_async(cdr_ctx* c, const cdr_dev_batch* in, const cdr_out* out, void* stream) {
  if (!c || !in || !out) return CDR_API_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  HIPCHK(hipSetDevice(c->device));
  const uint32_t threads = in->ev.n_slices * CDR_SLICE_WIDTH;
  const uint32_t blocks = (threads + 255) / 256;
  HIPCHK(hipEventRecord(c->ev[0], st));
  if (blocks) hipLaunchKernelGGL(k_replay, dim3(blocks), dim3(256), 0, st, *in, *out);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(c->ev[1], st));
  const uint32_t fb = (in->n_wfs + 255) / 256;
  if (fb) hipLaunchKernelGGL(k_finalize, dim3(fb), dim3(256), 0, st, *in, *out);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(c->ev[2], st));
  c->timed = true;
  return CDR_API_OK;
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

}  // extern "C"
