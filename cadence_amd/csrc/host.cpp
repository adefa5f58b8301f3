// host.cpp — host-side planning and packing for the replay engine (CPU only).
//
// The reference decodes each history batch into []*shared.HistoryEvent and walks it
// in one goroutine (stateBuilder.go:132-601).  Here the host instead lays a whole
// batch of decoded histories out as sliced columns (cdr.h: "SELL-64") so that one
// wavefront replays 64 workflows in lockstep with coalesced loads, and sizes the
// per-workflow output regions the kernels write into.
#include <algorithm>
#include <cmath>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <queue>
#include <system_error>
#include <thread>
#include <vector>

#include "cdr/cdr.h"
#include "cdr/ingest.h"
#include "internal.h"
#include "pack_event.h"

namespace {

int hw_threads(int threads) {
  if (threads > 0) return threads;
  unsigned h = std::thread::hardware_concurrency();
  return h ? (int)std::min(h, 64u) : 4;
}

template <class F>
void parallel_for(uint64_t n, int threads, F&& f, uint64_t grain = 256, uint64_t serial_below = 4096) {
  threads = hw_threads(threads);
  if (threads <= 1 || n < serial_below) {
    for (uint64_t i = 0; i < n; i++) f(i);
    return;
  }
  std::atomic<uint64_t> next{0};
  std::vector<std::thread> pool;
  auto work = [&] {
    for (;;) {
      uint64_t i0 = next.fetch_add(grain);
      if (i0 >= n) break;
      uint64_t i1 = std::min(n, i0 + grain);
      for (uint64_t i = i0; i < i1; i++) f(i);
    }
  };
  for (int t = 1; t < threads; t++) {
    try {
      pool.emplace_back(work);
    } catch (const std::system_error&) {
      break;  // thread limit reached: the caller's thread still drains the queue
    }
  }
  work();
  for (auto& th : pool) th.join();
}

// std::stable_sort over `threads` host threads: contiguous chunks sorted in parallel, then
// merged pairwise (std::merge takes the earlier chunk's element first on a tie), so the result
// is the serial stable sort's, element for element
template <class T, class Cmp>
void par_stable_sort(std::vector<T>& v, Cmp cmp, int threads) {
  const size_t n = v.size();
  size_t t = (size_t)std::max(1, threads);
  while (t > 1 && n / t < 32768) t >>= 1;
  if (t <= 1) {
    std::stable_sort(v.begin(), v.end(), cmp);
    return;
  }
  std::vector<size_t> cut(t + 1);
  for (size_t i = 0; i <= t; i++) cut[i] = n * i / t;
  {
    std::vector<std::thread> pool;
    for (size_t i = 0; i < t; i++)
      pool.emplace_back([&, i] { std::stable_sort(v.begin() + cut[i], v.begin() + cut[i + 1], cmp); });
    for (auto& th : pool) th.join();
  }
  std::vector<T> buf(n);
  std::vector<T>* src = &v;
  std::vector<T>* dst = &buf;
  for (size_t w = 1; w < t; w *= 2) {  // runs of w chunks -> runs of 2w chunks
    std::vector<std::thread> pool;
    for (size_t i = 0; i < t; i += 2 * w) {
      const size_t a = cut[i], m = cut[std::min(t, i + w)], e = cut[std::min(t, i + 2 * w)];
      pool.emplace_back([=] {
        std::merge(src->begin() + a, src->begin() + m, src->begin() + m, src->begin() + e, dst->begin() + a, cmp);
      });
    }
    for (auto& th : pool) th.join();
    std::swap(src, dst);
  }
  if (src != &v) v.swap(*src);
}

}  // namespace


namespace cdr_internal {

uint32_t arena_words_for(uint32_t type) { return cdr_arena_words_for(type); }

void caps_one(const cdr_event* ev, uint64_t n, uint32_t builder, cdr_wf_caps* out, const cdr_kv* kvs,
              const cdr_reset_point* rps, const loaded_rows* loaded) {
  cdr_wf_caps c{};
  bool fast = builder != CDR_BUILDER_2DC && n > 0 && ev[0].type == CDR_EV_WF_STARTED;
  bool have_ver = false;
  int64_t last_ver = 0;
  uint32_t vh = 0;
  int64_t live = 0, live_max = 0;
  // live sets of the wave kernel's lane tables, simulated by key (its slots are
  // reused first-free, so a table's high-water mark is its peak live count)
  std::vector<int64_t> lv[4];  // user timers (timer id), children, request-cancels, signals (initiated id)
  size_t lv_max[4] = {0, 0, 0, 0};
  // k_replay_reg envelope (CDR_CAP_REG): ids, call lengths, reset-point rows (Started's
  // plus new distinct checksums), distinct search-attribute keys
  bool reg = n > 0 && n < (1u << 20);
  int64_t last_id = 0;
  uint64_t call_start = 0;
  std::vector<uint32_t> rp_cks, sa_keys;
  auto lv_add = [&](int t, int64_t key, bool unique) {
    if (unique && std::find(lv[t].begin(), lv[t].end(), key) != lv[t].end()) return;
    lv[t].push_back(key);
    lv_max[t] = std::max(lv_max[t], lv[t].size());
  };
  auto lv_del = [&](int t, int64_t key) {
    auto it = std::find(lv[t].begin(), lv[t].end(), key);
    if (it != lv[t].end()) lv[t].erase(it);
  };
  if (loaded) {  // a loaded state's rows (by key when known; else keys no event names)
    const loaded_rows& L = *loaded;
    live = live_max = L.n[0];
    for (uint32_t i = 0; i < L.n[1]; i++) lv_add(0, L.timer ? (int64_t)L.timer[i].timer_id : INT64_MIN + i, false);
    for (uint32_t i = 0; i < L.n[2]; i++) lv_add(1, L.child ? L.child[i].initiated_id : INT64_MIN + i, false);
    for (uint32_t i = 0; i < L.n[3]; i++) lv_add(2, L.cancel ? L.cancel[i].initiated_id : INT64_MIN + i, false);
    for (uint32_t i = 0; i < L.n[4]; i++) lv_add(3, L.signal ? L.signal[i].initiated_id : INT64_MIN + i, false);
    for (uint32_t i = 0; i < L.n[5]; i++)
      rp_cks.push_back(L.rp ? ((L.rp[i].flags & CDR_RP_HAS_CHECKSUM) ? L.rp[i].binary_checksum : 0u) : 0xFFFFFFFFu - i);
    for (uint32_t i = 0; i < L.n[6]; i++) sa_keys.push_back(L.sa ? L.sa[i].key : 0xFFFFFFFFu - i);
  }
  for (uint64_t k = 0; k < n; k++) {
    const cdr_event& e = ev[k];
    if (k == 0 || (e.flags & CDR_EVF_BATCH_FIRST)) call_start = k;
    reg = reg && e.event_id > last_id && e.event_id < (1ll << 31) && e.version < (1ll << 31) &&
          k - call_start < 4096;
    last_id = e.event_id;
    if (e.type == CDR_EV_WF_STARTED) {  // rows from the start attributes (a second Started resets them)
      const cdr_attr_wf_started& a = e.a.started;
      rp_cks.clear();
      sa_keys.clear();
      if (a.flags & CDR_SF_HAS_RESET_POINTS)
        for (uint32_t q = 0; q < a.reset_points_len; q++) {  // a row each; unknown checksums match nothing
          const cdr_reset_point* p = rps ? rps + a.reset_points_off + q : nullptr;
          rp_cks.push_back(p && (p->flags & CDR_RP_HAS_CHECKSUM) ? p->binary_checksum : 0u);
        }
      if (a.flags & CDR_SF_HAS_SEARCH_ATTR)
        for (uint32_t q = 0; q < a.search_attr_len; q++)
          sa_keys.push_back(kvs ? kvs[a.search_attr_off + q].key : 0xFFFFFFF0u - q);
    } else if (e.type == CDR_EV_DT_COMPLETED && e.a.dt.binary_checksum) {
      if (std::find(rp_cks.begin(), rp_cks.end(), e.a.dt.binary_checksum) == rp_cks.end())
        rp_cks.push_back(e.a.dt.binary_checksum);
    } else if (e.type == CDR_EV_UPSERT_SA) {
      for (uint32_t q = 0; q < e.a.upsert.search_attr_len && sa_keys.size() <= CDR_REG_NSA; q++) {
        const uint32_t key = kvs ? kvs[e.a.upsert.search_attr_off + q].key : 0xFFFFFF00u - (uint32_t)sa_keys.size();
        if (std::find(sa_keys.begin(), sa_keys.end(), key) == sa_keys.end()) sa_keys.push_back(key);
      }
    }
    // live-activity bound: a close of a missing activity stops the replay, so before
    // the first error every close removed one live activity
    if (e.type == CDR_EV_AT_SCHEDULED) live_max = std::max(live_max, ++live);
    if (e.type == CDR_EV_AT_COMPLETED || e.type == CDR_EV_AT_FAILED || e.type == CDR_EV_AT_TIMED_OUT ||
        e.type == CDR_EV_AT_CANCELED)
      live = std::max<int64_t>(0, live - 1);
    switch (e.type) {
      case CDR_EV_TIMER_STARTED: lv_add(0, e.a.timer.timer_id, true); break;
      case CDR_EV_TIMER_FIRED: case CDR_EV_TIMER_CANCELED: lv_del(0, e.a.timer.timer_id); break;
      case CDR_EV_CHILD_INITIATED: lv_add(1, e.event_id, false); break;
      case CDR_EV_CHILD_START_FAILED: case CDR_EV_CHILD_COMPLETED: case CDR_EV_CHILD_FAILED:
      case CDR_EV_CHILD_CANCELED: case CDR_EV_CHILD_TIMED_OUT: case CDR_EV_CHILD_TERMINATED:
        lv_del(1, e.a.ref.initiated_event_id);
        break;
      case CDR_EV_RCE_INITIATED: lv_add(2, e.event_id, false); break;
      case CDR_EV_RCE_FAILED: case CDR_EV_EXT_CANCEL_REQUESTED: lv_del(2, e.a.ref.initiated_event_id); break;
      case CDR_EV_SE_INITIATED: lv_add(3, e.event_id, false); break;
      case CDR_EV_SE_FAILED: case CDR_EV_EXT_SIGNALED: lv_del(3, e.a.ref.initiated_event_id); break;
      default: break;
    }
    fast = fast && e.type < 64 && (CDR_FAST_TYPES & (1ull << e.type)) && (k == 0 || e.type != CDR_EV_WF_STARTED);
    if (!have_ver || e.version > last_ver) {
      vh++;
      last_ver = e.version;
      have_ver = true;
    }
    switch (e.type) {
      case CDR_EV_WF_STARTED:
        c.rp_cap += e.a.started.reset_points_len;
        c.sa_cap += e.a.started.search_attr_len;
        break;
      case CDR_EV_DT_COMPLETED:
        if (e.a.dt.binary_checksum) c.rp_cap++;
        break;
      case CDR_EV_AT_SCHEDULED:
        c.act_cap++;
        break;
      case CDR_EV_TIMER_STARTED:
        c.timer_cap++;
        break;
      case CDR_EV_CHILD_INITIATED:
        c.child_cap++;
        break;
      case CDR_EV_RCE_INITIATED:
        c.cancel_cap++;
        break;
      case CDR_EV_SE_INITIATED:
        c.signal_cap++;
        break;
      case CDR_EV_UPSERT_SA:
        c.sa_cap += e.a.upsert.search_attr_len;
        break;
      default:
        break;
    }
  }
  c.vh_cap = vh;
  c.act_live = (uint32_t)live_max;
  c.timer_live = (uint32_t)lv_max[0];  // peak live user timers: the kernels reuse freed slots first
  // the lane planner's ordering key: the entity counts (cdr_wf_caps.order_key)
  {
    auto sat = [](uint32_t v, uint32_t bits) { return v < (1u << bits) ? v : (1u << bits) - 1u; };
    c.order_key = sat(c.act_cap, 10) << 22 | sat(c.timer_cap, 11) << 11 |
                  sat(c.child_cap + c.cancel_cap + c.signal_cap, 11);
  }
  // the pending tables' row capacities: the peak live sets (the rows still pending at the
  // end are at most those), or the creating-event counts past the device planner's tracked
  // bound (k_caps: CDR_WAVE_SLOTS + 1 keys per set)
  {
    const size_t T = CDR_WAVE_SLOTS + 1;
    c.act_cap = (uint32_t)live_max;
    c.timer_cap = lv_max[0] > T ? c.timer_cap : (uint32_t)lv_max[0];
    c.child_cap = lv_max[1] > T ? c.child_cap : (uint32_t)lv_max[1];
    c.cancel_cap = lv_max[2] > T ? c.cancel_cap : (uint32_t)lv_max[2];
    c.signal_cap = lv_max[3] > T ? c.signal_cap : (uint32_t)lv_max[3];
  }
  c.flags = (fast && live_max <= 1) ? CDR_CAP_FAST : 0u;
  const uint32_t W = CDR_WAVE_SLOTS;
  // the wave kernel keeps one slot per lane and reuses freed slots first, so its
  // high-water marks are the peak live counts
  if (!(c.flags & CDR_CAP_FAST) && live_max <= (int64_t)W && lv_max[0] <= W && lv_max[1] <= W && lv_max[2] <= W &&
      lv_max[3] <= W)
    c.flags |= CDR_CAP_WAVE;
  // small working sets and a moderate length: cheaper in a lane slice than on a wave of
  // its own (the lane kernel's slot scans are short; the wave kernel pays its scalar
  // per-event cost regardless) — measured on C3/C5 shapes, DESIGN.md §3
  {
    static const uint32_t* lim = [] {
      static uint32_t v[4] = {CDR_LANE_MAX_ACT, CDR_LANE_MAX_TIMERS, CDR_LANE_MAX_EXT, CDR_LANE_MAX_LEN};
      if (const char* e = std::getenv("CDR_LANE_MAX"))  // tuning override "act,timers,ext,len"
        std::sscanf(e, "%u,%u,%u,%u", &v[0], &v[1], &v[2], &v[3]);
      return v;
    }();
    if ((c.flags & CDR_CAP_WAVE) && live_max <= (int64_t)lim[0] && lv_max[0] <= lim[1] &&
        lv_max[1] + lv_max[2] + lv_max[3] <= lim[2] && n <= lim[3])
      c.flags |= CDR_CAP_LANE;
  }
  reg = reg && !(c.flags & CDR_CAP_FAST) && lv_max[0] <= CDR_REG_NT && lv_max[1] <= CDR_REG_NX &&
        lv_max[2] <= CDR_REG_NX && lv_max[3] <= CDR_REG_NX && sa_keys.size() <= CDR_REG_NSA;
  // the 12-activity variant also keeps more reset points (CDR_REG2_NRP): histories with more
  // distinct checksums than CDR_REG_NRP go there rather than to the wave kernel
  if (reg && live_max <= (int64_t)CDR_REG_NA && rp_cks.size() <= CDR_REG_NRP) c.flags |= CDR_CAP_REG;
  else if (reg && live_max <= (int64_t)CDR_REG2_NA && rp_cks.size() <= CDR_REG2_NRP) c.flags |= CDR_CAP_REG2;
  if ((c.flags & CDR_CAP_REG) && live_max <= (int64_t)CDR_REG0_NA && lv_max[0] <= CDR_REG0_NT &&
      lv_max[1] <= CDR_REG0_NX && lv_max[2] <= CDR_REG0_NX && lv_max[3] <= CDR_REG0_NX)
    c.flags |= CDR_CAP_REG0;
  *out = c;
}

// upper bounds of the transfer / timer tasks an entry's events append
// (stateBuilder.go:157-595: at most one of each kind per event, two timer tasks for
// WorkflowExecutionStarted — backoff + timeout)
void task_caps(const cdr_event* ev, uint64_t n, uint32_t* xfer, uint32_t* ttask) {
  uint32_t x = 0, t = 0;
  for (uint64_t k = 0; k < n; k++) {
    switch (ev[k].type) {
      case CDR_EV_WF_STARTED:
        x += 1;
        t += 2;
        break;
      case CDR_EV_DT_SCHEDULED:
      case CDR_EV_DT_TIMED_OUT:
      case CDR_EV_DT_FAILED:
      case CDR_EV_CHILD_INITIATED:
      case CDR_EV_RCE_INITIATED:
      case CDR_EV_SE_INITIATED:
      case CDR_EV_UPSERT_SA:
        x += 1;
        break;
      case CDR_EV_AT_SCHEDULED:
      case CDR_EV_WF_COMPLETED:
      case CDR_EV_WF_FAILED:
      case CDR_EV_WF_TIMED_OUT:
      case CDR_EV_WF_CANCELED:
      case CDR_EV_WF_TERMINATED:
      case CDR_EV_WF_CONTINUED_AS_NEW:
        x += 1;
        t += 1;
        break;
      case CDR_EV_DT_STARTED:
      case CDR_EV_AT_STARTED:
      case CDR_EV_AT_COMPLETED:
      case CDR_EV_AT_FAILED:
      case CDR_EV_AT_TIMED_OUT:
      case CDR_EV_AT_CANCELED:
      case CDR_EV_TIMER_STARTED:
      case CDR_EV_TIMER_FIRED:
      case CDR_EV_TIMER_CANCELED:
        t += 1;
        break;
      default:
        break;
    }
  }
  // refreshTasks (mutableStateTaskRefresher.go:66-160) writes into the same slices: its
  // transfer tasks are bounded by the same events plus one UpsertWorkflowSearchAttributes
  // task; its timer tasks (at most one per kind) by Started's two, a close event's, a
  // DecisionTaskStarted's, an ActivityTaskScheduled's and a TimerStarted's
  *xfer = x + 1;
  *ttask = t;
}

void pack_lane(const cdr_event* ev, uint64_t n_ev, uint64_t row0, uint32_t len, uint32_t l, uint64_t apos,
               const cdr_slices* o) {
  uint8_t* const blk0 = const_cast<uint8_t*>(o->slab) + row0 * CDR_ROW_BYTES;
  uint64_t* arena = const_cast<uint64_t*>(o->arena);
  for (uint32_t k = 0; k < len; k++)
    cdr_put_event(blk0 + (uint64_t)k * CDR_ROW_BYTES, l, k < n_ev ? ev + k : nullptr, k == 0, &apos, arena);
}

// a wave slice: event k of the one workflow in row k/64, lane k%64 (cdr.h)
void pack_chunked(const cdr_event* ev, uint64_t n_ev, uint64_t row0, uint32_t rows, uint64_t apos,
                  const cdr_slices* o) {
  uint8_t* const blk0 = const_cast<uint8_t*>(o->slab) + row0 * CDR_ROW_BYTES;
  uint64_t* arena = const_cast<uint64_t*>(o->arena);
  for (uint64_t k = 0; k < (uint64_t)rows * CDR_SLICE_WIDTH; k++)
    cdr_put_event(blk0 + (k / CDR_SLICE_WIDTH) * CDR_ROW_BYTES, (uint32_t)(k % CDR_SLICE_WIDTH),
              k < n_ev ? ev + k : nullptr, k == 0, &apos, arena);
}

}  // namespace cdr_internal

extern "C" {

static int plan_caps_impl(const cdr_batch* b, cdr_wf_caps* caps, cdr_totals* totals, const cdr_wf_caps* bound);

int cdr_plan_caps(const cdr_batch* b, cdr_wf_caps* caps, cdr_totals* totals) {
  return plan_caps_impl(b, caps, totals, nullptr);
}

int cdr_plan_ndc_apply(const cdr_batch* b, const cdr_wf_caps* state_caps, cdr_wf_caps* caps, cdr_totals* totals) {
  if (!state_caps || (b && b->carry)) return CDR_API_EINVAL;
  return plan_caps_impl(b, caps, totals, state_caps);
}

}  // extern "C"

// `bound` (cdr_plan_ndc_apply): every entry replays onto a loaded state whose rows are at
// most its state capacities (known only on the device when the launch is planned)
static int plan_caps_impl(const cdr_batch* b, cdr_wf_caps* caps, cdr_totals* totals, const cdr_wf_caps* bound) {
  if (!b || !caps || !totals) return CDR_API_EINVAL;
  // per entry (in parallel: every entry's simulation is independent), then the offsets as a
  // prefix over the entries
  std::atomic<int> bad{0};
  parallel_for(b->n_wfs, 0, [&](uint64_t wi) {
    const uint32_t w = (uint32_t)wi;
    const cdr_wf_desc& d = b->wfs[w];
    if (d.ev_off + d.ev_len > b->n_events) {
      bad = 1;
      return;
    }
    // a continue-as-new entry must describe the run the parent's CAN event names
    // (stateBuilder.go:559-563): same workflow, RunId = NewExecutionRunId, builder
    // from newRunNDC
    if (d.newrun >= 0) {
      if ((uint32_t)d.newrun >= b->n_wfs) {
        bad = 1;
        return;
      }
      const cdr_wf_desc& n = b->wfs[d.newrun];
      if (n.parent != (int32_t)w || n.workflow_id != d.workflow_id ||
          n.builder != (d.newrun_ndc ? (uint32_t)CDR_BUILDER_NDC : (uint32_t)CDR_BUILDER_2DC)) {
        bad = 1;
        return;
      }
      uint32_t call = 0;
      for (uint64_t k = 0; k < d.ev_len; k++) {
        const cdr_event& e = b->events[d.ev_off + k];
        if (k > 0 && (e.flags & CDR_EVF_BATCH_FIRST)) call++;
        if (call == d.newrun_call && e.type == CDR_EV_WF_CONTINUED_AS_NEW &&
            e.a.can.new_execution_run_id != n.run_id) {
          bad = 1;
          return;
        }
      }
    }
    cdr_wf_caps c{};
    const bool carried = b->carry && b->carry->src && b->carry->src[w] >= 0;
    if (carried) {
      // a loaded state (cdr_carry): its rows are live from the start (the peak live sets
      // and the register-table envelope count them); the fast and wave kernels take no
      // loaded state, the register-table kernels' carry-in instantiations do
      const cdr_carry& cy = *b->carry;
      const uint32_t src = (uint32_t)cy.src[w];
      if (src >= cy.n_src || d.parent >= 0 || !cy.state.result || cy.state.result[src].code != CDR_OK) {
        bad = 1;
        return;
      }
      const cdr_wf_result& r = cy.state.result[src];
      cdr_internal::loaded_rows ld{{r.n_activity, r.n_timer, r.n_child, r.n_cancel, r.n_signal, r.n_reset_points,
                                    r.n_search_attr},
                                   nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
      if (cy.caps) {  // host-visible rows: the simulation follows their keys
        const cdr_wf_caps& sc = cy.caps[src];
        ld.timer = cy.state.timer ? cy.state.timer + sc.timer_off : nullptr;
        ld.child = cy.state.child ? cy.state.child + sc.child_off : nullptr;
        ld.cancel = cy.state.cancel ? cy.state.cancel + sc.cancel_off : nullptr;
        ld.signal = cy.state.signal ? cy.state.signal + sc.signal_off : nullptr;
        ld.rp = cy.state.rp ? cy.state.rp + sc.rp_off : nullptr;
        ld.sa = cy.state.sa ? cy.state.sa + sc.sa_off : nullptr;
      }
      cdr_internal::caps_one(b->events + d.ev_off, d.ev_len, d.builder, &c, b->kvs, b->rps, &ld);
      // (the pending tables' capacities are peak live sets that already count the loaded rows)
      c.vh_cap += r.n_vh;
      c.rp_cap += r.n_reset_points;
      c.sa_cap += r.n_search_attr;
      c.flags = (c.flags & ~(CDR_CAP_FAST | CDR_CAP_WAVE | CDR_CAP_LANE)) | CDR_CAP_LOADED;
    } else {
      cdr_internal::caps_one(b->events + d.ev_off, d.ev_len, d.builder, &c, b->kvs, b->rps);
    }
    if (bound) {  // the loaded rows' bound: the state's capacities
      if (d.parent >= 0 || d.newrun >= 0) {  // one run per entry
        bad = 1;
        return;
      }
      const cdr_wf_caps& s = bound[w];
      c.act_cap += s.act_cap;
      c.timer_cap += s.timer_cap;
      c.child_cap += s.child_cap;
      c.cancel_cap += s.cancel_cap;
      c.signal_cap += s.signal_cap;
      c.vh_cap += s.vh_cap;
      c.rp_cap += s.rp_cap;
      c.sa_cap += s.sa_cap;
      // live rows: at most the state's peak live sets (the sum of its parts' simulated
      // peaks, cadence_amd/ndc.py state_caps_for), not its capacities (every row any part
      // ever added): the general kernel sizes its working slots by these
      c.act_live += s.act_live;
      c.timer_live += s.timer_live;
      // the loaded rows are not known here: the register-table envelope is the history's
      // own, and an entry goes to the 12-activity variant (a loaded state plus the history's
      // own rows outgrow the 6-activity tables for ~1 entry in 4 on the forked C5 population,
      // and a slice runs as its largest lane needs); an entry whose loaded state outgrows even
      // that is handed on to the general kernel (replay_reg.inc).  CDR_CARRY_REG2=0 keeps the
      // history's own variant and relies on the hand-on chain (C5 forks 1M: 53.6 vs 48.5 ms)
      c.flags = (c.flags & ~(CDR_CAP_FAST | CDR_CAP_WAVE | CDR_CAP_LANE | CDR_CAP_REG0)) | CDR_CAP_LOADED;
      static const int all12 = [] {
        const char* e = std::getenv("CDR_CARRY_REG2");
        return e ? std::atoi(e) : 1;
      }();
      if (all12 && (c.flags & CDR_CAP_REG)) c.flags = (c.flags & ~CDR_CAP_REG) | CDR_CAP_REG2;
    }
    cdr_internal::task_caps(b->events + d.ev_off, d.ev_len, &c.xfer_cap, &c.ttask_cap);
    caps[w] = c;
  }, 64);
  if (bad) return CDR_API_EINVAL;
  cdr_totals t{};
  for (uint32_t w = 0; w < b->n_wfs; w++) {
    cdr_wf_caps& c = caps[w];
    c.xfer_off = t.xfer;
    t.xfer += c.xfer_cap;
    c.ttask_off = t.ttask;
    t.ttask += c.ttask_cap;
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
  }
  *totals = t;
  return CDR_API_OK;
}

// cdr_plan_slices_ex's body; with `pv` set, the outputs go to its vectors (sized here: one
// call plans and fills, where the C ABI takes a size query and a second call)
static int plan_slices_impl(const cdr_wf_desc* wfs, const cdr_wf_caps* caps, uint32_t n_wfs, uint32_t mode,
                            cdr_internal::plan_vecs* pv, int32_t* lane_wf, uint32_t* slice_len, uint64_t* slice_row0,
                            uint32_t* slice_flags, uint32_t* n_slices, uint64_t* n_rows, uint32_t* n_wave) {
  if (!wfs && n_wfs) return CDR_API_EINVAL;
  if ((mode & CDR_PLAN_WAVE) && !caps && n_wfs) return CDR_API_EINVAL;
  std::vector<uint32_t> lanes, waves, pars;
  lanes.reserve(n_wfs);
  // long histories: a lane slice advances one event per step, so a history much longer
  // than the batch's lane work per resident wave (its steps / CDR_LANE_RESIDENT) sets
  // the lane kernels' critical path alone; on a wave of its own it replays ~10x faster
  // per event and co-runs with the lane slices (replay.hip, side stream).  The
  // 12-activity register kernel runs one wave per SIMD, so its threshold is lower.
  // PAR slices replay a long history ~4x faster than a lane slice, so their threshold is
  // lower (CDR_PAR_FACTOR), within the CDR_PAR_MAX_SLICES cap below
  uint64_t long_thr = UINT64_MAX, long_thr2 = UINT64_MAX, par_thr = UINT64_MAX, par_thr2 = UINT64_MAX;
  if ((mode & CDR_PLAN_WAVE) && !(mode & CDR_PLAN_NO_LONG)) {
    static const uint32_t* lp = [] {
      static uint32_t v[4] = {CDR_LONG_MIN, CDR_LONG_FACTOR, CDR_LONG_REG2_DIV, CDR_PAR_FACTOR};
      if (const char* e = std::getenv("CDR_LONG"))  // tuning override "min,factor,reg2 divisor[,PAR factor]"
        std::sscanf(e, "%u,%u,%u,%u", &v[0], &v[1], &v[2], &v[3]);
      return v;
    }();
    uint64_t lane_ev = 0;
    for (uint32_t w = 0; w < n_wfs; w++)
      if (!(caps[w].flags & CDR_CAP_WAVE) || (caps[w].flags & (CDR_CAP_REG | CDR_CAP_REG2)))
        lane_ev += wfs[w].ev_len;
    const uint64_t per_slot = lane_ev / ((uint64_t)CDR_SLICE_WIDTH * CDR_LANE_RESIDENT);
    long_thr = std::max<uint64_t>(lp[0], (uint64_t)lp[1] * per_slot);
    long_thr2 = std::max<uint64_t>(lp[0] / 2, long_thr / std::max(1u, lp[2]));
    par_thr = std::max<uint64_t>(lp[0], (uint64_t)lp[3] * per_slot);
    par_thr2 = std::max<uint64_t>(lp[0] / 2, par_thr / std::max(1u, lp[2]));
  }
  // wave slices: every CDR_CAP_WAVE entry no register-table kernel takes (the general
  // lane kernel is the slow fallback for what fits neither), and the long ones
  // (CDR_PLAN_PAR: the long register-table ones to PAR lane slices instead)
  for (uint32_t w = 0; w < n_wfs; w++) {
    const uint32_t f = caps ? caps[w].flags : 0u;
    const uint64_t thr = (f & CDR_CAP_REG) ? long_thr : long_thr2;
    if ((mode & CDR_PLAN_WAVE) && (mode & CDR_PLAN_PAR) && !(mode & CDR_PLAN_WAVE_ALL) &&
        (f & (CDR_CAP_REG | CDR_CAP_REG2)) && !(f & CDR_CAP_LOADED) && (uint64_t)wfs[w].ev_len > ((f & CDR_CAP_REG) ? par_thr : par_thr2)) {
      pars.push_back(w);
      continue;
    }
    ((mode & CDR_PLAN_WAVE) && (f & CDR_CAP_WAVE) &&
             ((mode & CDR_PLAN_WAVE_ALL) || !(f & (CDR_CAP_REG | CDR_CAP_REG2)) || (uint64_t)wfs[w].ev_len > thr)
         ? waves
         : lanes)
        .push_back(w);
  }
  // longest first: a slice's rows = its longest lane, so neighbours in length
  // share slices and padding stays small (SELL-C-sigma with sigma = batch); wave
  // slices longest first too, so the longest histories start first
  auto longer = [&](uint32_t a, uint32_t c) { return wfs[a].ev_len > wfs[c].ev_len; };
  // lane slices: within a length class (~4% wide, so padding stays small) order by the
  // working-slot footprint, so that a slice's slot count (max over its lanes) is close
  // to its lanes' own and more slices fit the LDS tier of the general kernel
  auto lclass = [&](uint32_t a) { return (uint32_t)(std::log2((double)wfs[a].ev_len + 1.0) * 16.0); };
  auto slots = [&](uint32_t a) { return caps ? caps[a].act_live * CDR_ACT_PLANES + caps[a].timer_live * CDR_TIM_PLANES : 0u; };
  // kernel groups first (fast-path, register-table, general), so that slices are
  // homogeneous and go to the specialised kernels whole
  auto group = [&](uint32_t a) {
    return !caps                               ? 0u
           : (caps[a].flags & CDR_CAP_FAST)  ? 0u
           : (caps[a].flags & CDR_CAP_REG0)  ? 1u
           : (caps[a].flags & CDR_CAP_REG)   ? 2u
           : (caps[a].flags & CDR_CAP_REG2)  ? 3u
                                             : 4u;
  };
  // register-table groups: within a length class by their entity counts (scheduled
  // activities, started timers, initiated externals: cdr_wf_caps.order_key), so that a slice's lanes have similar
  // class counts and the class-sorted block's aligned regions (replay_cls.inc) carry little
  // padding (C3: 13% fewer class rows than ordering by footprint)
  // a PAR slice holds a whole CU (four 256-VGPR waves), so beyond about one round of them the
  // PAR kernel queues behind itself: the longest CDR_PAR_MAX_SLICES slices' worth stay PAR,
  // the rest go back to the register-table lanes
  std::stable_sort(pars.begin(), pars.end(), longer);
  {
    static const uint64_t par_max = [] {
      const char* e = std::getenv("CDR_PAR_MAX");  // tuning override (slices)
      return (uint64_t)(e ? std::strtoul(e, nullptr, 0) : CDR_PAR_MAX_SLICES) * CDR_PAR_LANES;
    }();
    const uint64_t pmax = (mode & CDR_PLAN_PAR_SOLO) ? (uint64_t)CDR_PAR_SOLO_MAX : par_max;
    if (pars.size() > pmax) {
      lanes.insert(lanes.end(), pars.begin() + pmax, pars.end());
      pars.resize(pmax);
    }
  }
  std::vector<uint32_t> lane_len;  // ev_len of lanes[i] (0: padding)
  {  // lane order: kernel group, length class (descending), then (register-table groups)
     // entity counts, footprint and length, all descending; the keys are computed once per
     // entry (a log2 and the caps reads per comparison dominated the planner: C3 100k 145 ms)
    struct LaneKey {
      uint32_t group, lclass, counts, slots;
      uint64_t len;
      uint32_t w;
    };
    static const bool by_counts = !std::getenv("CDR_LANE_ORDER_FOOTPRINT");  // A/B knob: the round-1 order
    std::vector<LaneKey> keys(lanes.size());
    for (size_t i = 0; i < lanes.size(); i++) {
      const uint32_t a = lanes[i], g = group(a);
      const bool counts = caps && by_counts && g >= 1 && g <= 3;
      keys[i] = LaneKey{g, lclass(a), counts ? caps[a].order_key : 0u, slots(a), (uint64_t)wfs[a].ev_len, a};
    }
    // (on the host's threads: the serial sort was most of a 1M-entry plan)
    par_stable_sort(keys, [](const LaneKey& x, const LaneKey& y) {
      if (x.group != y.group) return x.group < y.group;
      if (x.lclass != y.lclass) return x.lclass > y.lclass;
      if (x.counts != y.counts) return x.counts > y.counts;
      if (x.slots != y.slots) return x.slots > y.slots;
      return x.len > y.len;
    }, std::min(hw_threads(0), 16));
    for (size_t i = 0; i < lanes.size(); i++) lanes[i] = keys[i].w;
    // each kernel group starts a slice of its own (a mixed slice would replay on the
    // general kernel at the length of the next group's longest histories); the lanes' lengths
    // ride along from the keys (the slice loop below would otherwise read every entry's
    // descriptor again, in sorted — random — order)
    std::vector<uint32_t> padded;
    padded.reserve(lanes.size() + 3 * CDR_SLICE_WIDTH);
    lane_len.reserve(lanes.size() + 3 * CDR_SLICE_WIDTH);
    for (size_t i = 0; i < lanes.size(); i++) {
      if (i > 0 && keys[i].group != keys[i - 1].group)
        while (padded.size() % CDR_SLICE_WIDTH) {
          padded.push_back(UINT32_MAX);
          lane_len.push_back(0);
        }
      padded.push_back(lanes[i]);
      lane_len.push_back((uint32_t)keys[i].len);
    }
    lanes.swap(padded);
  }
  std::stable_sort(waves.begin(), waves.end(), longer);
  // PAR slices first (slices 0 .. np - 1, CDR_PAR_LANES histories each: their P loop runs
  // one history at a time), then the lane slices, then the wave slices
  // (the CDR_PAR_SOLO longest get a slice each: a W step over one lane runs one handler group)
  static const uint32_t solo_max = [] {
    const char* e = std::getenv("CDR_PAR_SOLO");
    return e ? (uint32_t)std::strtoul(e, nullptr, 0) : (uint32_t)CDR_PAR_SOLO;
  }();
  // ... and every history of at least CDR_PAR_SOLO_LEN events (up to the history count
  // limit): alone in its slice, k_replay_cls replays its activity / timer / external classes
  // in wave form (one event per step, the tables spread over the lanes) instead of one lane
  static const uint64_t solo_len = [] {
    const char* e = std::getenv("CDR_PAR_SOLO_LEN");  // A/B knob (events; 0 = none)
    const uint64_t v = e ? std::strtoull(e, nullptr, 0) : (uint64_t)CDR_PAR_SOLO_LEN;
    return v ? v : UINT64_MAX;
  }();
  uint32_t n_solo_len = 0;
  while (n_solo_len < pars.size() && wfs[pars[n_solo_len]].ev_len >= solo_len) n_solo_len++;
  // (CDR_PLAN_PAR_SOLO: every PAR history alone in its slice)
  const uint32_t solo = (mode & CDR_PLAN_PAR_SOLO) ? (uint32_t)pars.size()
                                                   : std::min<uint32_t>(std::max(solo_max, n_solo_len), (uint32_t)pars.size());
  // balanced PAR slices: a PAR slice's roles each walk its histories one at a time, so the
  // slice's time follows the summed lengths of its histories, and the kernel ends with its
  // heaviest slice (longest-first runs of 16 put the 16 longest histories in slice 0).
  // Longest-processing-time-first over the non-solo slices: each history (longest first)
  // joins the lightest slice with room; pars is then laid out slice by slice, UINT32_MAX
  // filling short slices
  static const bool par_lpt = [] {
    const char* e = std::getenv("CDR_PAR_PACK");  // A/B knob: "sorted" = the round-3 runs of 16
    return !(e && std::strcmp(e, "sorted") == 0);
  }();
  if (par_lpt && pars.size() > solo + CDR_PAR_LANES) {
    const uint32_t nb = (uint32_t)((pars.size() - solo + CDR_PAR_LANES - 1) / CDR_PAR_LANES);
    std::vector<std::vector<uint32_t>> bins(nb);
    typedef std::pair<uint64_t, uint32_t> Load;  // (summed events, bin)
    std::priority_queue<Load, std::vector<Load>, std::greater<Load>> light;
    for (uint32_t b = 0; b < nb; b++) light.push(Load(0, b));
    for (size_t i = solo; i < pars.size(); i++) {
      const Load l = light.top();
      light.pop();
      bins[l.second].push_back(pars[i]);
      if (bins[l.second].size() < CDR_PAR_LANES) light.push(Load(l.first + wfs[pars[i]].ev_len, l.second));
    }
    pars.resize(solo);
    for (uint32_t b = 0; b < nb; b++) {
      pars.insert(pars.end(), bins[b].begin(), bins[b].end());
      pars.resize(solo + (size_t)(b + 1) * CDR_PAR_LANES, UINT32_MAX);
    }
  }
  // PAR slice s takes pars[par_at(s) ...] (solo slices first, then CDR_PAR_LANES per slice)
  auto par_at = [&](uint32_t s) -> size_t { return s < solo ? s : solo + (size_t)(s - solo) * CDR_PAR_LANES; };
  const uint32_t np = solo + (uint32_t)((pars.size() - solo + CDR_PAR_LANES - 1) / CDR_PAR_LANES);
  const uint32_t nl = np + (uint32_t)((lanes.size() + CDR_SLICE_WIDTH - 1) / CDR_SLICE_WIDTH);
  const uint32_t nw = (uint32_t)waves.size();
  if (pv) {
    pv->lane_wf.resize((size_t)(nl + nw) * CDR_SLICE_WIDTH);
    pv->slice_len.resize(nl + nw);
    pv->slice_row0.resize(nl + nw);
    pv->slice_flags.resize(nl + nw);
    lane_wf = pv->lane_wf.data();
    slice_len = pv->slice_len.data();
    slice_row0 = pv->slice_row0.data();
    slice_flags = pv->slice_flags.data();
  }
  uint64_t rows = 0;
  for (uint32_t s = 0; s < nl; s++) {
    const std::vector<uint32_t>& src = s < np ? pars : lanes;
    const uint32_t width = s < solo ? 1u : s < np ? CDR_PAR_LANES : CDR_SLICE_WIDTH;  // lanes taken from src
    const size_t first = s < np ? par_at(s) : (size_t)(s - np) * CDR_SLICE_WIDTH;
    auto at = [&](uint32_t l) -> uint32_t {  // workflow of lane l, UINT32_MAX = empty
      const size_t i = first + l;
      return (l < width && i < src.size()) ? src[i] : UINT32_MAX;
    };
    uint32_t len = 0;  // the slice's longest lane
    for (uint32_t l = 0; l < CDR_SLICE_WIDTH; l++) {
      const uint32_t w = at(l);
      if (w != UINT32_MAX) len = std::max(len, s < np ? (uint32_t)wfs[w].ev_len : lane_len[first + l]);
    }
    if (slice_len) slice_len[s] = len;
    if (slice_row0) slice_row0[s] = rows;
    if (slice_flags) slice_flags[s] = s < np ? CDR_SLICE_PAR : 0u;
    rows += len;
    if (lane_wf)
      for (uint32_t l = 0; l < CDR_SLICE_WIDTH; l++) {
        const uint32_t w = at(l);
        lane_wf[(size_t)s * CDR_SLICE_WIDTH + l] = w != UINT32_MAX ? (int32_t)w : -1;
      }
  }
  for (uint32_t q = 0; q < nw; q++) {
    const uint32_t s = nl + q;
    const uint32_t len = (uint32_t)((wfs[waves[q]].ev_len + CDR_SLICE_WIDTH - 1) / CDR_SLICE_WIDTH);
    if (slice_len) slice_len[s] = len;
    if (slice_row0) slice_row0[s] = rows;
    if (slice_flags) slice_flags[s] = CDR_SLICE_WAVE;
    rows += len;
    if (lane_wf)
      for (uint32_t l = 0; l < CDR_SLICE_WIDTH; l++)
        lane_wf[(size_t)s * CDR_SLICE_WIDTH + l] = l == 0 ? (int32_t)waves[q] : -1;
  }
  if (n_slices) *n_slices = nl + nw;
  if (n_rows) *n_rows = rows;
  if (n_wave) *n_wave = nw;
  return CDR_API_OK;
}

int cdr_internal::plan_slices_vec(const cdr_wf_desc* wfs, const cdr_wf_caps* caps, uint32_t n_wfs, uint32_t mode,
                                  plan_vecs& out, uint32_t* n_slices, uint64_t* n_rows, uint32_t* n_wave) {
  return plan_slices_impl(wfs, caps, n_wfs, mode, &out, nullptr, nullptr, nullptr, nullptr, n_slices, n_rows, n_wave);
}

extern "C" {

int cdr_plan_slices_ex(const cdr_wf_desc* wfs, const cdr_wf_caps* caps, uint32_t n_wfs, uint32_t mode,
                       int32_t* lane_wf, uint32_t* slice_len, uint64_t* slice_row0, uint32_t* slice_flags,
                       uint32_t* n_slices, uint64_t* n_rows, uint32_t* n_wave) {
  return plan_slices_impl(wfs, caps, n_wfs, mode, nullptr, lane_wf, slice_len, slice_row0, slice_flags, n_slices,
                          n_rows, n_wave);
}

int cdr_plan_slices(const cdr_wf_desc* wfs, uint32_t n_wfs, int32_t* lane_wf, uint32_t* slice_len,
                    uint64_t* slice_row0, uint32_t* n_slices, uint64_t* n_rows) {
  return cdr_plan_slices_ex(wfs, nullptr, n_wfs, 0, lane_wf, slice_len, slice_row0, nullptr, n_slices, n_rows,
                            nullptr);
}

int cdr_plan_class_ranges(const uint32_t* slice_flags, uint32_t n_slices, uint32_t* lo, uint32_t* hi) {
  if (!lo || !hi || (!slice_flags && n_slices)) return CDR_API_EINVAL;
  for (int c = 0; c < 6; c++) lo[c] = hi[c] = 0;
  for (uint32_t s = 0; s < n_slices; s++) {
    const uint32_t f = slice_flags[s];
    if (f & CDR_SLICE_PAR) continue;  // slices 0 .. n_par_slices - 1, launched on their own
    const int c = (f & CDR_SLICE_WAVE)   ? CDR_CLASS_WAVE
                  : (f & CDR_SLICE_FAST) ? CDR_CLASS_FAST
                  : (f & CDR_SLICE_REG0) ? CDR_CLASS_REG0
                  : (f & CDR_SLICE_REG)  ? CDR_CLASS_REG
                  : (f & CDR_SLICE_REG2) ? CDR_CLASS_REG2
                                         : CDR_CLASS_GENERAL;
    if (hi[c] == 0) lo[c] = s;
    hi[c] = s + 1;
  }
  return CDR_API_OK;
}

int cdr_plan_scratch(const cdr_wf_caps* caps, const int32_t* lane_wf, uint32_t n_slices, uint64_t* scratch_off,
                     uint32_t* act_slots, uint32_t* tim_slots, uint32_t* slice_flags, uint64_t* total_words,
                     uint32_t* n_fast) {
  if (!caps || !lane_wf || !total_words) return CDR_API_EINVAL;
  uint64_t off = 0;
  uint32_t nf = 0;
  for (uint32_t s = 0; s < n_slices; s++) {
    if (slice_flags && (slice_flags[s] & CDR_SLICE_WAVE)) {  // lane-distributed tables: no scratch
      if (scratch_off) scratch_off[s] = off;
      if (act_slots) act_slots[s] = 0;
      if (tim_slots) tim_slots[s] = 0;
      slice_flags[s] = CDR_SLICE_WAVE;
      continue;
    }
    uint32_t a = 0, t = 0, lanes = 0;
    bool fast = true, reg0 = true, reg = true, reg2 = true;
    for (uint32_t l = 0; l < CDR_SLICE_WIDTH; l++) {
      const int32_t w = lane_wf[(size_t)s * CDR_SLICE_WIDTH + l];
      if (w < 0) continue;
      a = std::max(a, caps[w].act_live);
      t = std::max(t, caps[w].timer_live);
      fast = fast && (caps[w].flags & CDR_CAP_FAST);
      reg0 = reg0 && (caps[w].flags & CDR_CAP_REG0);
      reg = reg && (caps[w].flags & CDR_CAP_REG);
      reg2 = reg2 && (caps[w].flags & (CDR_CAP_REG | CDR_CAP_REG2));
      lanes++;
    }
    fast = fast && lanes > 0;
    reg0 = reg0 && lanes > 0 && !fast;
    reg = reg && lanes > 0 && !fast && !reg0;
    reg2 = reg2 && lanes > 0 && !fast && !reg0 && !reg;
    nf += fast ? 1u : 0u;
    if (scratch_off) scratch_off[s] = off;
    if (act_slots) act_slots[s] = a;
    if (tim_slots) tim_slots[s] = t;
    if (slice_flags && (slice_flags[s] & CDR_SLICE_PAR))  // register-table lanes, any class
      slice_flags[s] = (reg0 || reg || reg2) ? CDR_SLICE_PAR : 0u;
    else if (slice_flags)
      slice_flags[s] = fast ? CDR_SLICE_FAST : reg0 ? CDR_SLICE_REG0 : reg ? CDR_SLICE_REG : reg2 ? CDR_SLICE_REG2 : 0u;
    off += ((uint64_t)a * CDR_ACT_PLANES + (uint64_t)t * CDR_TIM_PLANES) * CDR_SLICE_WIDTH;
  }
  *total_words = off;
  if (n_fast) *n_fast = nf;
  return CDR_API_OK;
}

// one pass over every event's type word (a cache line per 152-B record): on the host's
// threads, in chunks, since a serial pass over a 200k-entry C2 batch cost as much as the pack
uint64_t cdr_plan_arena_words(const cdr_batch* b) {
  constexpr uint64_t CH = 1u << 16;
  const uint64_t nc = (b->n_events + CH - 1) / CH;
  std::vector<uint64_t> part(nc, 0);
  parallel_for(nc, 0, [&](uint64_t c) {
    uint64_t w = 0;
    for (uint64_t i = c * CH, e = std::min(b->n_events, (c + 1) * CH); i < e; i++)
      w += cdr_arena_words_for(b->events[i].type);
    part[c] = w;
  }, 1, 2);
  uint64_t w = 0;
  for (uint64_t v : part) w += v;
  return w;
}

int cdr_pack_slices(const cdr_batch* b, cdr_slices* o, int threads) {
  if (!b || !o) return CDR_API_EINVAL;
  // arena offsets: per workflow prefix (natural order), records in event order
  // (per-entry word counts on the host's threads, then their prefix)
  std::vector<uint64_t> arena_base(b->n_wfs + 1, 0);
  parallel_for(b->n_wfs, threads, [&](uint64_t w) {
    const cdr_wf_desc& d = b->wfs[w];
    uint64_t words = 0;
    for (uint64_t k = 0; k < d.ev_len; k++) words += cdr_arena_words_for(b->events[d.ev_off + k].type);
    arena_base[w + 1] = words;
  });
  for (uint32_t w = 0; w < b->n_wfs; w++) arena_base[w + 1] += arena_base[w];
  if (arena_base[b->n_wfs] > o->arena_words) return CDR_API_EINVAL;
  if (o->arena_words >= (1ull << 32)) return CDR_API_EINVAL;  // u32 arena offsets (cdr.h)
  std::atomic<int> bad{0};
  parallel_for(o->n_slices, threads, [&](uint64_t s) {
    const uint64_t row0 = o->slice_row0[s];
    const uint32_t len = o->slice_len[s];
    if (o->slice_flags && (o->slice_flags[s] & CDR_SLICE_WAVE)) {
      const int32_t w = o->lane_wf[s * CDR_SLICE_WIDTH];
      if (w < 0 || b->wfs[w].ev_len > (uint64_t)len * CDR_SLICE_WIDTH) {
        bad = 1;
        return;
      }
      cdr_internal::pack_chunked(b->events + b->wfs[w].ev_off, b->wfs[w].ev_len, row0, len, arena_base[w], o);
      return;
    }
    // blocks of rows, lane by lane within a block: the block's rows (~60 KB) stay in cache
    // while each lane's events stream in order (a lane-major walk over the whole slice
    // revisits ~0.8 MB of rows once per lane; a row-major one interleaves 64 input streams)
    const cdr_event* evl[CDR_SLICE_WIDTH];
    uint32_t n_ev[CDR_SLICE_WIDTH];
    uint64_t apos[CDR_SLICE_WIDTH];
    for (uint32_t l = 0; l < CDR_SLICE_WIDTH; l++) {
      const int32_t w = o->lane_wf[s * CDR_SLICE_WIDTH + l];
      evl[l] = w >= 0 ? b->events + b->wfs[w].ev_off : nullptr;
      n_ev[l] = w >= 0 ? (uint32_t)b->wfs[w].ev_len : 0u;
      apos[l] = w >= 0 ? arena_base[w] : 0;
      if (w >= 0 && b->wfs[w].ev_len > len) {
        bad = 1;
        n_ev[l] = 0;
        evl[l] = nullptr;
      }
    }
    uint8_t* const blk0 = const_cast<uint8_t*>(o->slab) + row0 * CDR_ROW_BYTES;
    uint64_t* arena = const_cast<uint64_t*>(o->arena);
    constexpr uint32_t KB = 16;
    for (uint32_t k0 = 0; k0 < len; k0 += KB) {
      const uint32_t k1 = k0 + KB < len ? k0 + KB : len;
      for (uint32_t l = 0; l < CDR_SLICE_WIDTH; l++)
        for (uint32_t k = k0; k < k1; k++)
          cdr_put_event(blk0 + (uint64_t)k * CDR_ROW_BYTES, l, k < n_ev[l] ? evl[l] + k : nullptr, k == 0, &apos[l],
                        arena);
    }
  }, 2, 8);  // a slice is ~0.8 MB of rows: small grains, parallel from a few slices on
  return bad ? CDR_API_EINVAL : CDR_API_OK;
}

// ---- class-sorted blocks on the host (cdr.h; the device twins are k_cls_count /
// k_cls_fill in replay_cls.inc): the packer regroups each register-table lane's events
// by entity class, so the class-decomposed replay reads one class per step (the
// per-event type switch of stateBuilder.go:157-600, regrouped)
static uint32_t cls_lane_len(const cdr_slices* s, const cdr_wf_desc* wfs, uint64_t sl, uint32_t lane) {
  const int32_t w = s->lane_wf[sl * CDR_SLICE_WIDTH + lane];
  return w >= 0 ? (uint32_t)wfs[w].ev_len : 0u;
}
static inline uint32_t slab_u32(const uint8_t* rows, uint64_t k, int c, uint32_t lane) {
  uint32_t v;
  std::memcpy(&v, rows + k * CDR_ROW_BYTES + cdr_col_off(c) + lane * 4u, 4);
  return v;
}
static inline int64_t slab_i64(const uint8_t* rows, uint64_t k, int c, uint32_t lane) {
  int64_t v;
  std::memcpy(&v, rows + k * CDR_ROW_BYTES + cdr_col_off(c) + lane * 8u, 8);
  return v;
}

int cdr_plan_cls(const cdr_slices* s, const cdr_wf_desc* wfs, uint32_t* cls_rows, uint64_t* cls_row0) {
  if (!s || !wfs || !cls_rows || !cls_row0 || !s->slice_flags) return CDR_API_EINVAL;
  uint64_t acc = 0;
  for (uint64_t sl = 0; sl < s->n_slices; sl++) {
    uint32_t m[4] = {0, 0, 0, 0};
    if (s->slice_flags[sl] & CDR_CLS_SLICES) {
      const uint8_t* rows = s->slab + s->slice_row0[sl] * CDR_ROW_BYTES;
      for (uint32_t l = 0; l < CDR_SLICE_WIDTH; l++) {
        const uint32_t len = cls_lane_len(s, wfs, sl, l);
        if (len > s->slice_len[sl]) return CDR_API_EINVAL;
        uint32_t n[4] = {0, 0, 0, 0};
        for (uint32_t k = 0; k < len; k++) {
          const uint32_t c = cdr_cls_of(slab_u32(rows, k, CDR_COL_TYPE_FLAGS, l) & 0xFFu);
          if (c < 4) n[c]++;
        }
        for (int j = 0; j < 4; j++) m[j] = std::max(m[j], n[j]);
      }
    }
    cls_row0[sl] = acc;
    for (int j = 0; j < 4; j++) {
      cls_rows[4 * sl + j] = m[j];
      acc += m[j];
    }
  }
  cls_row0[s->n_slices] = acc;
  return CDR_API_OK;
}

int cdr_pack_cls(const cdr_slices* s, const cdr_wf_desc* wfs, const uint32_t* cls_rows, const uint64_t* cls_row0,
                 uint8_t* cls_slab, int threads) {
  if (!s || !wfs || !cls_rows || !cls_row0 || !cls_slab || !s->slice_flags) return CDR_API_EINVAL;
  std::atomic<int> bad{0};
  parallel_for(
      s->n_slices, threads,
      [&](uint64_t sl) {
        if (!(s->slice_flags[sl] & CDR_CLS_SLICES)) return;
        const uint8_t* src = s->slab + s->slice_row0[sl] * CDR_ROW_BYTES;
        uint8_t* dst = cls_slab + cls_row0[sl] * CDR_ROW_BYTES;
        uint32_t M[4], off[4], acc = 0;
        for (int j = 0; j < 4; j++) {
          M[j] = cls_rows[4 * sl + j];
          off[j] = acc;
          acc += M[j];
        }
        if (cls_row0[sl + 1] - cls_row0[sl] != acc) {
          bad = 1;
          return;
        }
        std::memset(dst, 0, (size_t)acc * CDR_ROW_BYTES);
        auto put = [&](uint64_t row, int c, uint32_t lane, const void* v) {
          std::memcpy(dst + row * CDR_ROW_BYTES + cdr_col_off(c) + lane * cdr_col_size(c), v, cdr_col_size(c));
        };
        // per lane state, walked row by row (each source row read once, contiguously)
        uint32_t len[CDR_SLICE_WIDTH], pos[CDR_SLICE_WIDTH][4], k0[CDR_SLICE_WIDTH];
        int64_t prev_id[CDR_SLICE_WIDTH], x_next[CDR_SLICE_WIDTH], wver[CDR_SLICE_WIDTH];
        bool any_w[CDR_SLICE_WIDTH];
        uint32_t maxlen = 0;
        for (uint32_t l = 0; l < CDR_SLICE_WIDTH; l++) {
          len[l] = cls_lane_len(s, wfs, sl, l);
          if (len[l] > s->slice_len[sl]) bad = 1;
          maxlen = std::max(maxlen, len[l]);
          pos[l][0] = pos[l][1] = pos[l][2] = pos[l][3] = 0;
          k0[l] = 0;
          prev_id[l] = 0;
          x_next[l] = CDR_FIRST_EVENT_ID;
          wver[l] = 0;
          any_w[l] = false;
        }
        if (bad) return;
        for (uint32_t k = 0; k < maxlen; k++) {
          for (uint32_t l = 0; l < CDR_SLICE_WIDTH; l++) {
            if (k >= len[l]) continue;
            const uint32_t tf = slab_u32(src, k, CDR_COL_TYPE_FLAGS, l);
            const int64_t id = slab_i64(src, k, CDR_COL_EVENT_ID, l), ver = slab_i64(src, k, CDR_COL_VERSION, l);
            const bool bf = (tf & CDR_SEF_BATCH_FIRST) || k == 0;
            if (bf && k > 0) x_next[l] = prev_id[l] + 1;  // NextEventID after the previous call (stateBuilder.go:603-604)
            if (bf) k0[l] = k;
            prev_id[l] = id;
            const uint32_t type = tf & 0xFFu;
            const uint32_t c = cdr_cls_of(type);
            if (c == CDR_CLS_DROP) continue;
            if (pos[l][c] >= M[c]) {  // the plan does not belong to this slab
              bad = 1;
              return;
            }
            const uint64_t row = off[c] + pos[l][c]++;
            const bool need_id = type < 64 && ((1ull << type) & CDR_CLS_NEED_ID);
            const bool same_v = c != CDR_CLS_W || (any_w[l] && ver == wver[l]);
            if (c == CDR_CLS_W) {
              wver[l] = ver;
              any_w[l] = true;
            }
            const uint32_t tf2 = (tf & ~(CDR_SEF_ID_NEXT | CDR_SEF_VER_SAME)) | (need_id ? 0u : CDR_SEF_CLS_NO_ID) |
                                 (same_v ? CDR_SEF_CLS_VER_SAME : 0u);
            const uint64_t d = (uint64_t)id - (uint64_t)x_next[l];
            const uint32_t xd = (id >= x_next[l] && d < 0xFFFFFFFFull) ? (uint32_t)d : 0xFFFFFFFFu;
            const uint64_t ann = CDR_CLS_ANN(k, (k - k0[l]) & 0xFFFu, xd);
            const int64_t ts = slab_i64(src, k, CDR_COL_TIMESTAMP, l), key = slab_i64(src, k, CDR_COL_KEY, l),
                          aux = slab_i64(src, k, CDR_COL_AUX, l);
            const uint32_t h = slab_u32(src, k, CDR_COL_H, l), nn = slab_u32(src, k, CDR_COL_N, l);
            put(row, CDR_COL_TYPE_FLAGS, l, &tf2);
            put(row, CDR_COL_EVENT_ID, l, &id);
            put(row, CDR_COL_VERSION, l, &ver);
            put(row, CDR_COL_TIMESTAMP, l, &ts);
            put(row, CDR_COL_TASK_ID, l, &ann);
            put(row, CDR_COL_KEY, l, &key);
            put(row, CDR_COL_AUX, l, &aux);
            put(row, CDR_COL_H, l, &h);
            put(row, CDR_COL_N, l, &nn);
          }
        }
        const uint32_t pad = CDR_EV_PAD | CDR_SEF_CLS_NO_ID | CDR_SEF_CLS_VER_SAME;
        for (uint32_t l = 0; l < CDR_SLICE_WIDTH; l++)
          for (int j = 0; j < 4; j++)
            for (uint32_t p = pos[l][j]; p < M[j]; p++) put(off[j] + p, CDR_COL_TYPE_FLAGS, l, &pad);
      },
      1, 2);
  return bad ? CDR_API_EINVAL : CDR_API_OK;
}

// ---------------------------------------------------------------- farmhash
// Fingerprint32 == farmhashmk::Hash32 (github.com/dgryski/go-farm
// v0.0.0-20190423205320-6a90982ecee2, a port of google/farmhash), used by
// common.WorkflowIDToHistoryShard (common/util.go:249-252).  Restated from the
// published algorithm; no reference test pins concrete values (parity unpinned,
// affects partitioning only).
static inline uint32_t fh_fetch(const unsigned char* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}
static inline uint32_t fh_rot(uint32_t v, int s) { return s == 0 ? v : (v >> s) | (v << (32 - s)); }
static const uint32_t fh_c1 = 0xcc9e2d51u, fh_c2 = 0x1b873593u;
static inline uint32_t fh_fmix(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}
static inline uint32_t fh_mur(uint32_t a, uint32_t h) {
  a *= fh_c1;
  a = fh_rot(a, 17);
  a *= fh_c2;
  h ^= a;
  h = fh_rot(h, 19);
  return h * 5 + 0xe6546b64u;
}
static uint32_t fh_len0to4(const unsigned char* s, size_t len) {
  uint32_t b = 0, c = 9;
  for (size_t i = 0; i < len; i++) {
    int8_t v = (int8_t)s[i];
    b = b * fh_c1 + (uint32_t)(int32_t)v;
    c ^= b;
  }
  return fh_fmix(fh_mur(b, fh_mur((uint32_t)len, c)));
}
static uint32_t fh_len5to12(const unsigned char* s, size_t len) {
  uint32_t a = (uint32_t)len, b = (uint32_t)len * 5, c = 9, d = b;
  a += fh_fetch(s);
  b += fh_fetch(s + len - 4);
  c += fh_fetch(s + ((len >> 1) & 4));
  return fh_fmix(fh_mur(c, fh_mur(b, fh_mur(a, d))));
}
static uint32_t fh_len13to24(const unsigned char* s, size_t len) {
  uint32_t a = fh_fetch(s - 4 + (len >> 1));
  uint32_t b = fh_fetch(s + 4);
  uint32_t c = fh_fetch(s + len - 8);
  uint32_t d = fh_fetch(s + (len >> 1));
  uint32_t e = fh_fetch(s);
  uint32_t f = fh_fetch(s + len - 4);
  uint32_t h = d * fh_c1 + (uint32_t)len;
  a = fh_rot(a, 12) + f;
  h = fh_mur(c, h) + a;
  a = fh_rot(a, 3) + c;
  h = fh_mur(e, h) + a;
  a = fh_rot(a + f, 12) + d;
  h = fh_mur(b, h) + a;
  return fh_fmix(h);
}

uint32_t cdr_fingerprint32(const char* str, size_t len) {
  const unsigned char* s = (const unsigned char*)str;
  if (len <= 24) {
    return len <= 12 ? (len <= 4 ? fh_len0to4(s, len) : fh_len5to12(s, len)) : fh_len13to24(s, len);
  }
  uint32_t h = (uint32_t)len, g = fh_c1 * (uint32_t)len, f = g;
  uint32_t a0 = fh_rot(fh_fetch(s + len - 4) * fh_c1, 17) * fh_c2;
  uint32_t a1 = fh_rot(fh_fetch(s + len - 8) * fh_c1, 17) * fh_c2;
  uint32_t a2 = fh_rot(fh_fetch(s + len - 16) * fh_c1, 17) * fh_c2;
  uint32_t a3 = fh_rot(fh_fetch(s + len - 12) * fh_c1, 17) * fh_c2;
  uint32_t a4 = fh_rot(fh_fetch(s + len - 20) * fh_c1, 17) * fh_c2;
  h ^= a0;
  h = fh_rot(h, 19);
  h = h * 5 + 0xe6546b64u;
  h ^= a2;
  h = fh_rot(h, 19);
  h = h * 5 + 0xe6546b64u;
  g ^= a1;
  g = fh_rot(g, 19);
  g = g * 5 + 0xe6546b64u;
  g ^= a3;
  g = fh_rot(g, 19);
  g = g * 5 + 0xe6546b64u;
  f += a4;
  f = fh_rot(f, 19) + 113;
  size_t iters = (len - 1) / 20;
  do {
    uint32_t a = fh_fetch(s), b = fh_fetch(s + 4), c = fh_fetch(s + 8), d = fh_fetch(s + 12), e = fh_fetch(s + 16);
    h += a;
    g += b;
    f += c;
    h = fh_mur(d, h) + e;
    g = fh_mur(c, g) + a;
    f = fh_mur(b + e * fh_c1, f) + d;
    f += g;
    g += f;
    s += 20;
  } while (--iters != 0);
  g = fh_rot(g, 11) * fh_c1;
  g = fh_rot(g, 17) * fh_c1;
  f = fh_rot(f, 11) * fh_c1;
  f = fh_rot(f, 17) * fh_c1;
  h = fh_rot(h + g, 19);
  h = h * 5 + 0xe6546b64u;
  h = fh_rot(h, 17) * fh_c1;
  h = fh_rot(h + f, 19);
  h = h * 5 + 0xe6546b64u;
  h = fh_rot(h, 17) * fh_c1;
  return h;
}

int32_t cdr_workflow_id_to_shard(const char* workflow_id, size_t len, int32_t num_shards) {
  if (num_shards <= 0) return -1;
  return (int32_t)(cdr_fingerprint32(workflow_id, len) % (uint32_t)num_shards);
}

const char* cdr_version(void) { return "cadence_amd-cdr 0.1 (gfx950)"; }

}  // extern "C"

extern "C" {
// sizeof of the ABI structs, so language bindings can verify their mirrors.
uint64_t cdr_struct_size(const char* name) {
  struct E {
    const char* n;
    uint64_t s;
  };
  static const E table[] = {
      {"cdr_event", sizeof(cdr_event)},
      {"cdr_wf_desc", sizeof(cdr_wf_desc)},
      {"cdr_cluster_meta", sizeof(cdr_cluster_meta)},
      {"cdr_batch", sizeof(cdr_batch)},
      {"cdr_kv", sizeof(cdr_kv)},
      {"cdr_reset_point", sizeof(cdr_reset_point)},
      {"cdr_attr_wf_started", sizeof(cdr_attr_wf_started)},
      {"cdr_attr_at_scheduled", sizeof(cdr_attr_at_scheduled)},
      {"cdr_exec_info", sizeof(cdr_exec_info)},
      {"cdr_repl_state", sizeof(cdr_repl_state)},
      {"cdr_vh_item", sizeof(cdr_vh_item)},
      {"cdr_activity_info", sizeof(cdr_activity_info)},
      {"cdr_timer_info", sizeof(cdr_timer_info)},
      {"cdr_child_info", sizeof(cdr_child_info)},
      {"cdr_cancel_info", sizeof(cdr_cancel_info)},
      {"cdr_signal_info", sizeof(cdr_signal_info)},
      {"cdr_wf_result", sizeof(cdr_wf_result)},
      {"cdr_wf_caps", sizeof(cdr_wf_caps)},
      {"cdr_totals", sizeof(cdr_totals)},
      {"cdr_out", sizeof(cdr_out)},
      {"cdr_slices", sizeof(cdr_slices)},
      {"cdr_dev_batch", sizeof(cdr_dev_batch)},
      {"cdr_carry", sizeof(cdr_carry)},
      {"cdr_task", sizeof(cdr_task)},
      {"cdr_last_decision", sizeof(cdr_last_decision)},
      {"cdr_opts", sizeof(cdr_opts)},
      {"cdr_strtab", sizeof(cdr_strtab)},
      {"cdr_exec_persist", sizeof(cdr_exec_persist)},
      {"cdr_ingest_in", sizeof(cdr_ingest_in)},
      {"cdr_ingest_out", sizeof(cdr_ingest_out)},
      {"cdr_vh_token", sizeof(cdr_vh_token)},
      {"cdr_vh_branch", sizeof(cdr_vh_branch)},
      {"cdr_vhs", sizeof(cdr_vhs)},
      {"cdr_ndc_task", sizeof(cdr_ndc_task)},
      {"cdr_ndc_decision", sizeof(cdr_ndc_decision)},
      {"cdr_ndc_round", sizeof(cdr_ndc_round)},
  };
  for (const E& e : table)
    if (std::strcmp(e.n, name) == 0) return e.s;
  return 0;
}
}  // extern "C"
