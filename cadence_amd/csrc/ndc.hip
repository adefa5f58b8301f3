// ndc.hip — NDC branch management and conflict-resolution rebuild bookkeeping.
//
// When a replication task forks a workflow's history, the history
// service decides per task, before any replay (paths relative to /root/reference):
//   nDCBranchMgr.prepareVersionHistory       service/history/nDCBranchMgr.go:80-249
//     FindLCAVersionHistoryIndexAndItem / IsLCAAppendable / DuplicateUntilLCAItem /
//     AddVersionHistory                      common/persistence/versionHistory.go:152-520
//   nDCConflictResolver.prepareMutableState   service/history/nDCConflictResolver.go:73-114
// and, after the stateRebuilder replay of a branch (cdr_replay_* with
// expected_next_event_id = the branch's last item + 1), verifies the rebuilt version
// history against the branch's (nDCConflictResolver.go:154-165) and switches the current
// branch (:172-174).  These kernels do that bookkeeping for a whole batch of workflows,
// one thread per workflow: the work is a few dozen version-history items per workflow
// (no events), so it is latency-, not bandwidth-bound; what matters is that it runs on
// the device next to the replays it routes, with no host round trip per workflow.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "cdr/cdr.h"
#include "ctx.h"

#define HIPCHK(x)                                                                                     \
  do {                                                                                                \
    hipError_t _e = (x);                                                                              \
    if (_e != hipSuccess) {                                                                           \
      fprintf(stderr, "cdr: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(_e), __FILE__, __LINE__); \
      return CDR_API_EDEVICE;                                                                         \
    }                                                                                                 \
  } while (0)

extern "C" int cdr_ctx_device(const cdr_ctx* ctx);  // replay.hip

namespace {

struct It {
  int64_t e, v;
};
__device__ __forceinline__ It ld(const cdr_vh_item* p) {
  const cdr_vh_item x = *p;
  return It{x.event_id, x.version};
}
__device__ __forceinline__ bool tok_eq(const cdr_vh_token& a, const cdr_vh_token& b) {
  return a.tree == b.tree && a.branch_lo == b.branch_lo && a.branch_hi == b.branch_hi;
}

// FindLCAItem (versionHistory.go:262-290): walk both histories back from their last items
__device__ int32_t find_lca(const cdr_vh_item* a, uint32_t na, const cdr_vh_item* b, uint32_t nb, It* out) {
  int li = (int)na - 1, ri = (int)nb - 1;
  while (li >= 0 && ri >= 0) {
    const It l = ld(a + li), r = ld(b + ri);
    if (l.v == r.v) {
      *out = l.e > r.e ? r : l;
      return CDR_OK;
    }
    if (l.v > r.v) li--;
    else ri--;
  }
  return CDR_E_VH_NO_LCA;
}

// AddOrUpdateItem (versionHistory.go:203-236) onto a history whose items live at dst
// (count n, last item in `last`); items past `cap` are tracked but not stored
__device__ int32_t add_or_update(cdr_vh_item* dst, uint32_t cap, uint32_t* n, It* last, It it, bool* over) {
  if (*n == 0) {
    if (cap > 0) dst[0] = cdr_vh_item{it.e, it.v};
    else *over = true;
    *n = 1;
    *last = it;
    return CDR_OK;
  }
  if (it.v < last->v) return CDR_E_VH_LOWER_VERSION;
  if (it.e <= last->e) return CDR_E_VH_LOWER_EVENT_ID;
  if (it.v > last->v) {
    if (*n < cap) dst[*n] = cdr_vh_item{it.e, it.v};
    else *over = true;
    (*n)++;
  } else if (*n <= cap) {
    dst[*n - 1].event_id = it.e;
  }
  *last = it;
  return CDR_OK;
}

__device__ int32_t branch_one(const cdr_ndc_task& t, const cdr_vh_item* ti, cdr_vhs& s, cdr_vh_item* pool,
                              cdr_ndc_decision& d) {
  const cdr_vh_item* inc = ti + t.items_off;
  const uint32_t ni = t.n_items;
  cdr_vh_item* base = pool + s.items_off;
  const uint32_t cap = s.items_cap;
  // FindLCAVersionHistoryIndexAndItem (versionHistory.go:489-520)
  uint32_t idx = 0, len = 0;
  It lca{0, 0};
  bool set = false;
  for (uint32_t b = 0; b < s.n_branches; b++) {
    It it;
    const int32_t rc = find_lca(base + (uint64_t)b * cap, s.branch[b].n_items, inc, ni, &it);
    if (rc) return rc;
    if (!set || it.e > lca.e || (it.e == lca.e && s.branch[b].n_items < len)) {
      set = true;
      idx = b;
      len = s.branch[b].n_items;
      lca = it;
    }
  }
  if (!set) return CDR_E_VH_NO_LCA;  // no branch at all: NewVersionHistories never ran
  d.lca = cdr_vh_item{lca.e, lca.v};
  const cdr_vh_item* src = base + (uint64_t)idx * cap;
  const uint32_t ns = s.branch[idx].n_items;
  uint32_t branch = idx, n_br = s.n_branches, cur = s.current;
  bool over = false;
  uint32_t tgt_n = ns;  // target branch's item count after the task
  It tgt_last = ns ? ld(src + ns - 1) : It{0, 0};
  cdr_vh_item* tgt = base + (uint64_t)idx * cap;
  bool created = false;
  if (ns > 0 && tgt_last.e == lca.e && tgt_last.v == lca.v) {  // IsLCAAppendable
    const int64_t next = tgt_last.e + 1;                        // verifyEventsOrder :171-193
    if (t.first_event_id < next) {
      d.action = CDR_NDC_SKIP;
      d.branch_index = idx;
      return CDR_OK;
    }
    if (t.first_event_id > next) return CDR_E_NDC_RETRY_TASK;
  } else {
    // DuplicateUntilLCAItem (versionHistory.go:152-186) into the next branch slot
    const uint32_t nb = s.n_branches;
    const bool slot = nb < CDR_VHS_MAX_BRANCHES;
    cdr_vh_item* dst = base + (uint64_t)nb * cap;
    uint32_t n = 0;
    It last{0, 0}, first{0, 0};
    bool found = false;
    for (uint32_t i = 0; i < ns && !found; i++) {
      const It it = ld(src + i);
      if (n == 0) first = it.v < lca.v ? it : lca;
      int32_t rc;
      if (it.v < lca.v) {
        rc = add_or_update(dst, slot ? cap : 0, &n, &last, it, &over);
      } else if (it.v == lca.v) {
        if (lca.e > it.e) return CDR_E_VH_LCA_NOT_CONTAINED;
        rc = add_or_update(dst, slot ? cap : 0, &n, &last, lca, &over);
        found = true;
      } else {
        return CDR_E_VH_LCA_NOT_CONTAINED;
      }
      if (rc) return rc;
    }
    if (!found) return CDR_E_VH_LCA_NOT_CONTAINED;
    const int64_t next = last.e + 1;
    if (t.first_event_id < next) {  // doContinue = false
      d.action = CDR_NDC_SKIP;
      d.branch_index = idx;
      return CDR_OK;
    }
    if (t.first_event_id > next) return CDR_E_NDC_RETRY_TASK;
    // createNewBranch (nDCBranchMgr.go:195-249) -> AddVersionHistory (versionHistory.go:438-487)
    const cdr_vh_branch& cb = s.branch[cur];
    const uint32_t cn = cb.n_items;
    if (cn == 0) return CDR_E_VH_EMPTY;
    const cdr_vh_item* cur_items = base + (uint64_t)cur * cap;
    if (first.v != ld(cur_items).v) return CDR_E_VH_FIRST_ITEM_MISMATCH;
    if (last.v > ld(cur_items + cn - 1).v) return CDR_E_NDC_BRANCH_CHANGED;  // the index switch is an error here
    if (!slot) over = true;
    branch = nb;
    n_br = nb + 1;
    tgt = dst;
    tgt_n = n;
    tgt_last = last;
    created = true;
  }
  // prepareMutableState (nDCConflictResolver.go:73-114)
  if (branch == cur) {
    d.action = CDR_NDC_APPLY_CURRENT;
  } else {
    const uint32_t cn = s.branch[cur].n_items;
    if (cn == 0) return CDR_E_VH_EMPTY;
    const It cur_last = ld(base + (uint64_t)cur * cap + cn - 1);
    if (t.version < cur_last.v) {
      // applyNonStartEventsToNoneCurrentBranch: the branch's VH gets the last event
      const int32_t rc = add_or_update(tgt, branch < CDR_VHS_MAX_BRANCHES ? cap : 0, &tgt_n, &tgt_last,
                                       It{t.last_event_id, t.last_version}, &over);
      if (rc) return rc;
      d.action = CDR_NDC_BACKFILL;
    } else if (t.version == cur_last.v) {
      return CDR_E_NDC_SAME_VERSION;
    } else {
      if (tgt_n == 0) return CDR_E_VH_EMPTY;
      d.action = CDR_NDC_REBUILD;
      d.rebuild_next_event_id = tgt_last.e + 1;
      d.rebuild_token = created ? t.new_token : s.branch[branch].token;
    }
  }
  if (over) return CDR_E_VHS_CAPACITY;
  // commit
  d.branch_index = branch;
  d.created = created ? 1u : 0u;
  if (created) {
    s.branch[branch].token = t.new_token;
    s.branch[branch]._pad = 0;
  }
  s.branch[branch].n_items = tgt_n;
  s.n_branches = n_br;
  return CDR_OK;
}

__global__ __launch_bounds__(256) void k_ndc_branch(const cdr_ndc_task* tasks, const cdr_vh_item* task_items,
                                                    uint32_t n, cdr_vhs* vhs, cdr_vh_item* pool,
                                                    cdr_ndc_decision* dec) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= n) return;
  const cdr_ndc_task t = tasks[w];
  cdr_vhs& s = vhs[w];
  cdr_ndc_decision d{};
  const int32_t rc = branch_one(t, task_items, s, pool, d);
  if (rc) {
    d = cdr_ndc_decision{};
    d.code = rc;
  }
  dec[w] = d;
}

__global__ __launch_bounds__(256) void k_ndc_rebuild_verify(uint32_t n, const cdr_ndc_decision* dec, cdr_vhs* vhs,
                                                            const cdr_vh_item* pool, const cdr_wf_caps* caps,
                                                            cdr_out O) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= n) return;
  const cdr_ndc_decision d = dec[w];
  if (d.code != CDR_OK || d.action != CDR_NDC_REBUILD) return;
  cdr_wf_result& r = O.result[w];
  if (r.code != CDR_OK) return;
  cdr_exec_info& x = O.exec[w];  // SetCurrentBranchToken(target) (nDCStateRebuilder.go:144-146)
  x.branch_tree_id = d.rebuild_token.tree;
  x.branch_id_lo = d.rebuild_token.branch_lo;
  x.branch_id_hi = d.rebuild_token.branch_hi;
  cdr_vhs& s = vhs[w];
  const cdr_vh_branch& b = s.branch[d.branch_index];
  const cdr_vh_item* want = pool + s.items_off + (uint64_t)d.branch_index * s.items_cap;
  const cdr_vh_item* got = O.vh + caps[w].vh_off;
  bool eq = b.n_items == r.n_vh && tok_eq(b.token, d.rebuild_token);
  for (uint32_t i = 0; eq && i < r.n_vh; i++) eq = got[i].event_id == want[i].event_id && got[i].version == want[i].version;
  if (!eq) {  // nDCConflictResolver.go:161-165
    r.code = CDR_E_REBUILD_VH_MISMATCH;
    r.fail_event_id = 0;
    r.fail_index = 0;
    r.n_activity = r.n_timer = r.n_child = r.n_cancel = r.n_signal = 0;
    r.n_vh = r.n_reset_points = r.n_search_attr = 0;
    return;
  }
  s.current = d.branch_index;  // SetCurrentVersionHistoryIndex (:172-174)
}

__device__ void zero_result(cdr_wf_result& r, int32_t code);

__global__ __launch_bounds__(256) void k_vhs_sync(uint32_t n, cdr_vhs* vhs, cdr_vh_item* pool,
                                                  const cdr_wf_caps* caps, cdr_out O) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= n) return;
  const cdr_wf_result& r = O.result[w];
  if (r.code != CDR_OK) return;
  cdr_vhs& s = vhs[w];
  if (r.n_vh > s.items_cap) {  // the caller's item slots are too few: the workflow fails visibly
    zero_result(O.result[w], CDR_E_VHS_CAPACITY);
    return;
  }
  if (s.n_branches == 0) {  // NewVersionHistories (versionHistory.go:350-363)
    s.n_branches = 1;
    s.current = 0;
  }
  cdr_vh_branch& b = s.branch[s.current];
  const cdr_exec_info& x = O.exec[w];
  b.token.tree = x.branch_tree_id;
  b.token._pad = 0;
  b.token.branch_lo = x.branch_id_lo;
  b.token.branch_hi = x.branch_id_hi;
  b.n_items = r.n_vh;
  b._pad = 0;
  cdr_vh_item* dst = pool + s.items_off + (uint64_t)s.current * s.items_cap;
  const cdr_vh_item* src = O.vh + caps[w].vh_off;
  for (uint32_t i = 0; i < r.n_vh; i++) dst[i] = src[i];
}

// ---- cdr_ndc_replicate_async's steps (one thread per workflow)

__device__ void zero_result(cdr_wf_result& r, int32_t code) {
  r = cdr_wf_result{};
  r.code = code;
}

// the state records of entry w := the source's (rows at the destination's capacities)
__device__ void copy_state(const cdr_out& S, const cdr_wf_caps& sc, const cdr_out& D, const cdr_wf_caps& dc, uint32_t w) {
  const cdr_wf_result r = S.result[w];
  D.exec[w] = S.exec[w];
  D.repl[w] = S.repl[w];
  D.result[w] = r;
  if (r.code != CDR_OK) return;
  bool ok = true;
  auto cp = [&](auto* src, auto* dst, uint64_t so, uint64_t doff, uint32_t n, uint32_t cap) {
    if (n > cap) {
      ok = false;
      return;
    }
    for (uint32_t i = 0; i < n; i++) dst[doff + i] = src[so + i];
  };
  cp(S.act, D.act, sc.act_off, dc.act_off, r.n_activity, dc.act_cap);
  cp(S.timer, D.timer, sc.timer_off, dc.timer_off, r.n_timer, dc.timer_cap);
  cp(S.child, D.child, sc.child_off, dc.child_off, r.n_child, dc.child_cap);
  cp(S.cancel, D.cancel, sc.cancel_off, dc.cancel_off, r.n_cancel, dc.cancel_cap);
  cp(S.signal, D.signal, sc.signal_off, dc.signal_off, r.n_signal, dc.signal_cap);
  cp(S.vh, D.vh, sc.vh_off, dc.vh_off, r.n_vh, dc.vh_cap);
  cp(S.rp, D.rp, sc.rp_off, dc.rp_off, r.n_reset_points, dc.rp_cap);
  cp(S.sa, D.sa, sc.sa_off, dc.sa_off, r.n_search_attr, dc.sa_cap);
  if (!ok) D.result[w].code = CDR_E_BAD_INPUT;
}

// which workflows the rebuild replays (CDR_NDC_REBUILD of a live state); every output
// record a step will not write is marked CDR_NOT_RUN; the apply carry's src map
__global__ __launch_bounds__(256) void k_ndc_round_begin(uint32_t n, const cdr_ndc_decision* dec, cdr_out S,
                                                         cdr_out RB, cdr_out AP, uint8_t* skip_rb, int32_t* src) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= n) return;
  const cdr_ndc_decision d = dec[w];
  const bool rb = S.result[w].code == CDR_OK && d.code == CDR_OK && d.action == CDR_NDC_REBUILD;
  skip_rb[w] = rb ? 0 : 1;
  if (!rb) zero_result(RB.result[w], CDR_NOT_RUN);
  zero_result(AP.result[w], CDR_NOT_RUN);
  src[w] = (int32_t)w;
}

// after the rebuild (+ refresh + verification): the rebuilt state replaces the workflow's
// (nDCConflictResolver.prepareMutableState returns it, :107-113) and is applied onto in
// memory; which workflows the apply replays
__global__ __launch_bounds__(256) void k_ndc_round_adopt_rebuilt(uint32_t n, const cdr_ndc_decision* dec,
                                                                 const cdr_wf_caps* sc, cdr_out S,
                                                                 const cdr_wf_caps* rc, cdr_out RB, uint8_t* skip_ap,
                                                                 uint8_t* in_mem) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= n) return;
  const cdr_ndc_decision d = dec[w];
  skip_ap[w] = 1;
  in_mem[w] = 0;
  if (S.result[w].code != CDR_OK) return;  // a failed workflow stays failed
  if (d.code != CDR_OK) {                  // the branch manager's / conflict resolver's error
    zero_result(S.result[w], d.code);
    return;
  }
  if (d.action == CDR_NDC_REBUILD) {
    if (RB.result[w].code != CDR_OK) {  // rebuild, refresh or verification failed
      S.result[w] = RB.result[w];
      return;
    }
    copy_state(RB, rc[w], S, sc[w], w);
    if (S.result[w].code != CDR_OK) return;
    in_mem[w] = 1;
    skip_ap[w] = 0;
  } else if (d.action == CDR_NDC_APPLY_CURRENT) {
    skip_ap[w] = 0;
  }
}

__global__ void k_ndc_carry_desc(cdr_carry* dst, cdr_carry c) { *dst = c; }

// after the apply (+ VH sync): the applied state is the workflow's
__global__ __launch_bounds__(256) void k_ndc_round_adopt_applied(uint32_t n, const uint8_t* skip_ap,
                                                                 const cdr_wf_caps* sc, cdr_out S,
                                                                 const cdr_wf_caps* ac, cdr_out AP) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= n || skip_ap[w]) return;
  if (AP.result[w].code != CDR_OK)
    S.result[w] = AP.result[w];
  else
    copy_state(AP, ac[w], S, sc[w], w);
}

}  // namespace

extern "C" {

int cdr_ndc_replicate_async(cdr_ctx* ctx, uint32_t n, const cdr_ndc_round* R, cdr_vhs* vhs, cdr_vh_item* pool,
                            const cdr_wf_caps* state_caps, const cdr_out* state, void* stream) {
  if (!ctx || !R || !state || (n && (!R->tasks || !R->task_items || !vhs || !pool || !R->dec || !state_caps)))
    return CDR_API_EINVAL;
  if (n > R->rebuild.n_wfs || n > R->apply.n_wfs || R->apply.carry || !R->rebuild_out.transfer ||
      !R->rebuild_out.timer_tasks || !R->rebuild_out.n_tasks)
    return CDR_API_EINVAL;
  // every apply entry replays onto a loaded state: only the general and the register-table
  // kernels take one (cdr_plan_ndc_apply never plans fast or wave slices)
  if (R->apply.n_fast_slices || R->apply.n_wave_slices) return CDR_API_EINVAL;
  if (n == 0) return CDR_API_OK;
  hipStream_t st = (hipStream_t)stream;
  HIPCHK(hipSetDevice(cdr_ctx_device(ctx)));
  uint8_t* skip_rb = (uint8_t*)cdr_ws_get(ctx, WS_NDC_SKIP_RB, n);
  uint8_t* skip_ap = (uint8_t*)cdr_ws_get(ctx, WS_NDC_SKIP_AP, n);
  uint8_t* in_mem = (uint8_t*)cdr_ws_get(ctx, WS_NDC_INMEM, n);
  int32_t* src = (int32_t*)cdr_ws_get(ctx, WS_NDC_SRC, n * 4ull);
  cdr_carry* carry_d = (cdr_carry*)cdr_ws_get(ctx, WS_NDC_CARRY, sizeof(cdr_carry));
  if (!skip_rb || !skip_ap || !in_mem || !src || !carry_d) return CDR_API_ENOMEM;
  const dim3 g((n + 255) / 256), b(256);
  // 1. prepareVersionHistory + prepareMutableState
  int rc = cdr_ndc_branch_async(ctx, R->tasks, R->task_items, n, vhs, pool, R->dec, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(k_ndc_round_begin, g, b, 0, st, n, R->dec, *state, R->rebuild_out, R->apply_out, skip_rb, src);
  HIPCHK(hipGetLastError());
  // 2. nDCStateRebuilder.rebuild of the REBUILD workflows, refreshTasks, verification
  cdr_dev_batch rb = R->rebuild;  // its class-sorted blocks, if any, go to k_replay_cls (skip-aware)
  rb.skip = skip_rb;
  cdr_out rbo = R->rebuild_out;
  rbo.transfer = rbo.timer_tasks = nullptr;  // the replay emits no stateBuilder tasks here
  rbo.n_tasks = nullptr;
  if ((rc = cdr_replay_sliced_async(ctx, &rb, &rbo, stream))) return rc;
  if ((rc = cdr_refresh_tasks_async(ctx, &rb, &R->rebuild_out, R->refresh_now, R->refresh_flags, stream))) return rc;
  if ((rc = cdr_ndc_rebuild_verify_async(ctx, n, R->dec, vhs, pool, R->rebuild.caps, &R->rebuild_out, stream)))
    return rc;
  hipLaunchKernelGGL(k_ndc_round_adopt_rebuilt, g, b, 0, st, n, R->dec, state_caps, *state, R->rebuild.caps,
                     R->rebuild_out, skip_ap, in_mem);
  HIPCHK(hipGetLastError());
  // 3. applyNonStartEventsToCurrentBranch: carry-in replay onto the (rebuilt or loaded) state
  cdr_carry cy{};
  cy.src = src;
  cy.caps = state_caps;
  cy.n_src = n;
  cy.state = *state;
  cy.state.transfer = cy.state.timer_tasks = nullptr;
  cy.state.n_tasks = nullptr;
  cy.state.last_decision = nullptr;
  cy.in_memory = in_mem;
  hipLaunchKernelGGL(k_ndc_carry_desc, dim3(1), dim3(1), 0, st, carry_d, cy);
  HIPCHK(hipGetLastError());
  cdr_dev_batch ap = R->apply;
  ap.skip = skip_ap;
  ap.carry = carry_d;
  ap.cls_slab = nullptr;
  ap.cls_row0 = nullptr;
  ap.cls_rows = nullptr;
  cdr_out apo = R->apply_out;
  apo.transfer = apo.timer_tasks = nullptr;
  apo.n_tasks = nullptr;
  if ((rc = cdr_replay_sliced_async(ctx, &ap, &apo, stream))) return rc;
  if ((rc = cdr_vhs_sync_async(ctx, n, vhs, pool, R->apply.caps, &R->apply_out, stream))) return rc;
  // 4. the applied states become the workflows'
  hipLaunchKernelGGL(k_ndc_round_adopt_applied, g, b, 0, st, n, skip_ap, state_caps, *state, R->apply.caps,
                     R->apply_out);
  HIPCHK(hipGetLastError());
  return CDR_API_OK;
}

int cdr_ndc_branch_async(cdr_ctx* ctx, const cdr_ndc_task* tasks, const cdr_vh_item* task_items, uint32_t n,
                         cdr_vhs* vhs, cdr_vh_item* pool, cdr_ndc_decision* dec, void* stream) {
  if (!ctx || (n && (!tasks || !task_items || !vhs || !pool || !dec))) return CDR_API_EINVAL;
  HIPCHK(hipSetDevice(cdr_ctx_device(ctx)));
  if (n) hipLaunchKernelGGL(k_ndc_branch, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, tasks, task_items,
                            n, vhs, pool, dec);
  HIPCHK(hipGetLastError());
  return CDR_API_OK;
}

int cdr_ndc_rebuild_verify_async(cdr_ctx* ctx, uint32_t n, const cdr_ndc_decision* dec, cdr_vhs* vhs,
                                 const cdr_vh_item* pool, const cdr_wf_caps* caps, const cdr_out* out, void* stream) {
  if (!ctx || !out || (n && (!dec || !vhs || !pool || !caps))) return CDR_API_EINVAL;
  HIPCHK(hipSetDevice(cdr_ctx_device(ctx)));
  if (n) hipLaunchKernelGGL(k_ndc_rebuild_verify, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, n, dec,
                            vhs, pool, caps, *out);
  HIPCHK(hipGetLastError());
  return CDR_API_OK;
}

int cdr_vhs_sync_async(cdr_ctx* ctx, uint32_t n, cdr_vhs* vhs, cdr_vh_item* pool, const cdr_wf_caps* caps,
                       const cdr_out* out, void* stream) {
  if (!ctx || !out || (n && (!vhs || !pool || !caps))) return CDR_API_EINVAL;
  HIPCHK(hipSetDevice(cdr_ctx_device(ctx)));
  if (n) hipLaunchKernelGGL(k_vhs_sync, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, n, vhs, pool, caps,
                            *out);
  HIPCHK(hipGetLastError());
  return CDR_API_OK;
}

}  // extern "C"
