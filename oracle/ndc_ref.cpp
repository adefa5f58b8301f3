// oracle/ndc_ref.cpp — TEST INFRASTRUCTURE ONLY (parity checker for ndc.hip).
//
// A literal restatement of the reference's NDC version-history bookkeeping and of the
// branch-management / conflict-resolution decisions that surround the replay path when
// a replication task forks a workflow's history:
//   VersionHistory / VersionHistories        common/persistence/versionHistory.go:31-607
//   nDCBranchMgr.prepareVersionHistory        service/history/nDCBranchMgr.go:80-249
//   nDCConflictResolver.prepareMutableState   service/history/nDCConflictResolver.go:73-114
//   nDCConflictResolver.rebuild (verification) service/history/nDCConflictResolver.go:116-184
//   applyNonStartEventsToNoneCurrentBranch    service/history/nDCHistoryReplicator.go:420-454
// Nothing in the product links this file; tests/ use it as the checker of the GPU
// kernels in cadence_amd/csrc/ndc.hip and to pin the reference's versionHistory_test.go
// known answers.
#include <cstdint>
#include <cstring>
#include <vector>

#include "cdr/schema.h"

namespace {

struct Item {
  int64_t eventID, version;
  bool operator==(const Item& o) const { return eventID == o.eventID && version == o.version; }
};

struct VersionHistory {
  cdr_vh_token token{};
  std::vector<Item> items;

  // AddOrUpdateItem versionHistory.go:203-236
  int32_t AddOrUpdateItem(Item it) {
    if (items.empty()) {
      items.push_back(it);
      return CDR_OK;
    }
    Item& last = items.back();
    if (it.version < last.version) return CDR_E_VH_LOWER_VERSION;
    if (it.eventID <= last.eventID) return CDR_E_VH_LOWER_EVENT_ID;
    if (it.version > last.version)
      items.push_back(it);
    else
      last.eventID = it.eventID;
    return CDR_OK;
  }
  // DuplicateUntilLCAItem versionHistory.go:152-186
  int32_t DuplicateUntilLCAItem(Item lca, VersionHistory* out) const {
    VersionHistory v;
    for (const Item& it : items) {
      if (it.version < lca.version) {
        int32_t rc = v.AddOrUpdateItem(it);
        if (rc) return rc;
      } else if (it.version == lca.version) {
        if (lca.eventID > it.eventID) return CDR_E_VH_LCA_NOT_CONTAINED;
        int32_t rc = v.AddOrUpdateItem(lca);
        if (rc) return rc;
        *out = v;
        return CDR_OK;
      } else {
        return CDR_E_VH_LCA_NOT_CONTAINED;
      }
    }
    return CDR_E_VH_LCA_NOT_CONTAINED;
  }
  // ContainsItem versionHistory.go:238-260
  bool ContainsItem(Item it) const {
    int64_t prev = CDR_FIRST_EVENT_ID - 1;
    for (const Item& cur : items) {
      if (it.version == cur.version) {
        if (it.eventID == CDR_FIRST_EVENT_ID - 1 && it.eventID <= cur.eventID) return true;
        if (prev < it.eventID && it.eventID <= cur.eventID) return true;
      } else if (it.version < cur.version) {
        return false;
      }
      prev = cur.eventID;
    }
    return false;
  }
  // FindLCAItem versionHistory.go:262-290
  int32_t FindLCAItem(const VersionHistory& remote, Item* out) const {
    long li = (long)items.size() - 1, ri = (long)remote.items.size() - 1;
    while (li >= 0 && ri >= 0) {
      const Item& l = items[li];
      const Item& r = remote.items[ri];
      if (l.version == r.version) {
        *out = l.eventID > r.eventID ? r : l;
        return CDR_OK;
      } else if (l.version > r.version) {
        li--;
      } else {
        ri--;
      }
    }
    return CDR_E_VH_NO_LCA;
  }
  // IsLCAAppendable versionHistory.go:292-305 (non-empty histories only)
  bool IsLCAAppendable(Item it) const { return !items.empty() && items.back() == it; }
  bool Equals(const VersionHistory& o) const {  // versionHistory.go:330-348
    return std::memcmp(&token, &o.token, sizeof token) == 0 && items == o.items;
  }
};

struct VersionHistories {
  uint32_t current = 0;
  std::vector<VersionHistory> h;

  // AddVersionHistory versionHistory.go:438-487
  int32_t AddVersionHistory(const VersionHistory& v, bool* changed, uint32_t* idx) {
    *changed = false;
    *idx = 0;
    if (v.items.empty()) return CDR_E_VH_EMPTY;
    const VersionHistory& cur = h[current];
    if (cur.items.empty()) return CDR_E_VH_EMPTY;
    if (v.items.front().version != cur.items.front().version) return CDR_E_VH_FIRST_ITEM_MISMATCH;
    const Item curLast = cur.items.back();
    h.push_back(v);
    *idx = (uint32_t)h.size() - 1;
    if (v.items.back().version > curLast.version) {
      *changed = true;
      current = *idx;
    }
    return CDR_OK;
  }
  // FindLCAVersionHistoryIndexAndItem versionHistory.go:489-520
  int32_t FindLCAVersionHistoryIndexAndItem(const VersionHistory& incoming, uint32_t* idx, Item* item) const {
    bool set = false;
    size_t len = 0;
    if (h.empty()) return CDR_E_VH_NO_LCA;  // no history at all (NewVersionHistories never ran)
    for (size_t i = 0; i < h.size(); i++) {
      Item it;
      int32_t rc = h[i].FindLCAItem(incoming, &it);
      if (rc) return rc;
      if (!set || it.eventID > item->eventID || (it.eventID == item->eventID && h[i].items.size() < len)) {
        set = true;
        *idx = (uint32_t)i;
        len = h[i].items.size();
        *item = it;
      }
    }
    return CDR_OK;
  }
  // FindFirstVersionHistoryIndexByItem versionHistory.go:522-534
  int32_t FindFirstVersionHistoryIndexByItem(Item it, uint32_t* idx) const {
    for (size_t i = 0; i < h.size(); i++)
      if (h[i].ContainsItem(it)) {
        *idx = (uint32_t)i;
        return CDR_OK;
      }
    return CDR_E_VH_LCA_NOT_CONTAINED;
  }
  // IsRebuilt versionHistory.go:536-560
  bool IsRebuilt() const {
    const Item curLast = h[current].items.back();
    for (const VersionHistory& v : h)
      if (v.items.back().version > curLast.version) return true;
    return false;
  }
};

VersionHistory from_items(const cdr_vh_item* it, uint32_t n) {
  VersionHistory v;
  for (uint32_t i = 0; i < n; i++) v.items.push_back({it[i].event_id, it[i].version});
  return v;
}

VersionHistories load(const cdr_vhs& s, const cdr_vh_item* pool) {
  VersionHistories v;
  v.current = s.current;
  for (uint32_t b = 0; b < s.n_branches; b++) {
    VersionHistory x = from_items(pool + s.items_off + (uint64_t)b * s.items_cap, s.branch[b].n_items);
    x.token = s.branch[b].token;
    v.h.push_back(x);
  }
  return v;
}

int32_t store(const VersionHistories& v, cdr_vhs* s, cdr_vh_item* pool) {
  if (v.h.size() > CDR_VHS_MAX_BRANCHES) return CDR_E_VHS_CAPACITY;
  for (const VersionHistory& x : v.h)
    if (x.items.size() > s->items_cap) return CDR_E_VHS_CAPACITY;
  s->current = v.current;
  s->n_branches = (uint32_t)v.h.size();
  for (uint32_t b = 0; b < s->n_branches; b++) {
    s->branch[b].token = v.h[b].token;
    s->branch[b].n_items = (uint32_t)v.h[b].items.size();
    cdr_vh_item* dst = pool + s->items_off + (uint64_t)b * s->items_cap;
    for (size_t i = 0; i < v.h[b].items.size(); i++) dst[i] = cdr_vh_item{v.h[b].items[i].eventID, v.h[b].items[i].version};
  }
  return CDR_OK;
}

// one task: prepareVersionHistory (nDCBranchMgr.go:80-125) + prepareMutableState
// (nDCConflictResolver.go:73-114) + the non-current-branch backfill's VH update
// (nDCHistoryReplicator.go:437-447); vhs updated in place only when the task succeeds
int32_t ndc_branch_one(const cdr_ndc_task& t, const cdr_vh_item* task_items, VersionHistories& v, cdr_ndc_decision* d) {
  std::memset(d, 0, sizeof *d);
  VersionHistory incoming = from_items(task_items + t.items_off, t.n_items);
  uint32_t idx = 0;
  Item lca{};
  int32_t rc = v.FindLCAVersionHistoryIndexAndItem(incoming, &idx, &lca);  // flushBufferedEvents :127-134
  if (rc) return rc;
  d->lca = cdr_vh_item{lca.eventID, lca.version};
  VersionHistories nv = v;
  const VersionHistory& vh = nv.h[idx];
  uint32_t branch = idx;
  if (vh.IsLCAAppendable(lca)) {
    // verifyEventsOrder :171-193
    const int64_t next = vh.items.back().eventID + 1;
    if (t.first_event_id < next) {
      d->action = CDR_NDC_SKIP;
      d->branch_index = idx;
      return CDR_OK;
    }
    if (t.first_event_id > next) return CDR_E_NDC_RETRY_TASK;
  } else {
    VersionHistory dup;
    rc = vh.DuplicateUntilLCAItem(lca, &dup);
    if (rc) return rc;
    if (dup.items.empty()) return CDR_E_VH_EMPTY;
    const int64_t next = dup.items.back().eventID + 1;
    if (t.first_event_id < next) {  // doContinue = false: nothing happens
      d->action = CDR_NDC_SKIP;
      d->branch_index = idx;
      return CDR_OK;
    }
    if (t.first_event_id > next) return CDR_E_NDC_RETRY_TASK;
    dup.token = t.new_token;  // createNewBranch :195-249 (ForkHistoryBranch's token)
    bool changed = false;
    rc = nv.AddVersionHistory(dup, &changed, &branch);
    if (rc) return rc;
    if (changed) return CDR_E_NDC_BRANCH_CHANGED;
    d->created = 1;
  }
  d->branch_index = branch;
  // prepareMutableState
  if (branch == nv.current) {
    d->action = CDR_NDC_APPLY_CURRENT;
  } else {
    const VersionHistory& cur = nv.h[nv.current];
    if (cur.items.empty()) return CDR_E_VH_EMPTY;
    const Item curLast = cur.items.back();
    if (t.version < curLast.version) {
      // applyNonStartEventsToNoneCurrentBranch: the branch's VH gets the last event
      rc = nv.h[branch].AddOrUpdateItem(Item{t.last_event_id, t.last_version});
      if (rc) return rc;
      d->action = CDR_NDC_BACKFILL;
    } else if (t.version == curLast.version) {
      return CDR_E_NDC_SAME_VERSION;
    } else {
      const VersionHistory& rb = nv.h[branch];
      if (rb.items.empty()) return CDR_E_VH_EMPTY;
      d->action = CDR_NDC_REBUILD;
      d->rebuild_next_event_id = rb.items.back().eventID + 1;
      d->rebuild_token = rb.token;
    }
  }
  v = nv;
  return CDR_OK;
}

}  // namespace

extern "C" {

// ---- single-history known-answer helpers (versionHistory_test.go)
int cdro_vh_duplicate_until_lca(const cdr_vh_item* items, uint32_t n, cdr_vh_item lca, cdr_vh_item* out,
                                uint32_t* n_out) {
  VersionHistory dup;
  int32_t rc = from_items(items, n).DuplicateUntilLCAItem(Item{lca.event_id, lca.version}, &dup);
  if (rc) return rc;
  for (size_t i = 0; i < dup.items.size(); i++) out[i] = cdr_vh_item{dup.items[i].eventID, dup.items[i].version};
  *n_out = (uint32_t)dup.items.size();
  return CDR_OK;
}
int cdro_vh_contains(const cdr_vh_item* items, uint32_t n, cdr_vh_item it) {
  return from_items(items, n).ContainsItem(Item{it.event_id, it.version}) ? 1 : 0;
}
int cdro_vh_is_lca_appendable(const cdr_vh_item* items, uint32_t n, cdr_vh_item it) {
  return from_items(items, n).IsLCAAppendable(Item{it.event_id, it.version}) ? 1 : 0;
}
int cdro_vh_find_lca(const cdr_vh_item* local, uint32_t nl, const cdr_vh_item* remote, uint32_t nr,
                     cdr_vh_item* out) {
  Item it{};
  int32_t rc = from_items(local, nl).FindLCAItem(from_items(remote, nr), &it);
  if (rc == CDR_OK) *out = cdr_vh_item{it.eventID, it.version};
  return rc;
}

// ---- VersionHistories over a cdr_vhs record (items in `pool`)
int cdro_vhs_add(cdr_vhs* s, cdr_vh_item* pool, const cdr_vh_token* token, const cdr_vh_item* items, uint32_t n,
                 int* changed, uint32_t* idx) {
  VersionHistories v = load(*s, pool);
  VersionHistory x = from_items(items, n);
  x.token = *token;
  bool ch = false;
  int32_t rc = v.AddVersionHistory(x, &ch, idx);
  if (rc) return rc;
  *changed = ch ? 1 : 0;
  return store(v, s, pool);
}
int cdro_vhs_find_lca_index(const cdr_vhs* s, const cdr_vh_item* pool, const cdr_vh_item* items, uint32_t n,
                            uint32_t* idx, cdr_vh_item* item) {
  Item it{};
  int32_t rc = load(*s, pool).FindLCAVersionHistoryIndexAndItem(from_items(items, n), idx, &it);
  if (rc == CDR_OK) *item = cdr_vh_item{it.eventID, it.version};
  return rc;
}
int cdro_vhs_find_first_index_by_item(const cdr_vhs* s, const cdr_vh_item* pool, cdr_vh_item it, uint32_t* idx) {
  return load(*s, pool).FindFirstVersionHistoryIndexByItem(Item{it.event_id, it.version}, idx);
}
int cdro_vhs_is_rebuilt(const cdr_vhs* s, const cdr_vh_item* pool) { return load(*s, pool).IsRebuilt() ? 1 : 0; }

// ---- batch operations restated (the checker of ndc.hip's kernels)

// For every workflow w: task[w] against vhs[w] (updated in place when the decision is
// CDR_OK); decision in dec[w].
int cdro_ndc_branch(const cdr_ndc_task* tasks, const cdr_vh_item* task_items, uint32_t n, cdr_vhs* vhs,
                    cdr_vh_item* pool, cdr_ndc_decision* dec) {
  for (uint32_t w = 0; w < n; w++) {
    VersionHistories v = load(vhs[w], pool);
    cdr_ndc_decision d;
    int32_t rc = ndc_branch_one(tasks[w], task_items, v, &d);
    if (rc == CDR_OK) rc = store(v, &vhs[w], pool);
    if (rc) {
      std::memset(&d, 0, sizeof d);
      d.code = rc;
    }
    dec[w] = d;
  }
  return 0;
}

// After the rebuild replay of every CDR_NDC_REBUILD workflow (entry w of `out`):
// SetCurrentBranchToken(target) on the rebuilt state (nDCStateRebuilder.go:144-146), the
// rebuilt current VersionHistory must equal the branch's (nDCConflictResolver.go:154-165),
// then SetCurrentVersionHistoryIndex(branchIndex) (:172-174).  A mismatch sets the
// entry's result code; other workflows are untouched.
int cdro_ndc_rebuild_verify(uint32_t n, const cdr_ndc_decision* dec, cdr_vhs* vhs, const cdr_vh_item* pool,
                            const cdr_wf_caps* caps, cdr_out* out) {
  for (uint32_t w = 0; w < n; w++) {
    const cdr_ndc_decision& d = dec[w];
    if (d.code != CDR_OK || d.action != CDR_NDC_REBUILD) continue;
    cdr_wf_result& r = out->result[w];
    if (r.code != CDR_OK) continue;
    cdr_exec_info& x = out->exec[w];
    x.branch_tree_id = d.rebuild_token.tree;
    x.branch_id_lo = d.rebuild_token.branch_lo;
    x.branch_id_hi = d.rebuild_token.branch_hi;
    const cdr_vhs& s = vhs[w];
    const cdr_vh_branch& b = s.branch[d.branch_index];
    const cdr_vh_item* want = pool + s.items_off + (uint64_t)d.branch_index * s.items_cap;
    const cdr_vh_item* got = out->vh + caps[w].vh_off;
    bool eq = b.n_items == r.n_vh && std::memcmp(&b.token, &d.rebuild_token, sizeof b.token) == 0;
    for (uint32_t i = 0; eq && i < r.n_vh; i++) eq = got[i].event_id == want[i].event_id && got[i].version == want[i].version;
    if (!eq) {
      r.code = CDR_E_REBUILD_VH_MISMATCH;
      r.fail_event_id = 0;
      r.fail_index = 0;
      r.n_activity = r.n_timer = r.n_child = r.n_cancel = r.n_signal = 0;
      r.n_vh = r.n_reset_points = r.n_search_attr = 0;
      continue;
    }
    vhs[w].current = d.branch_index;
  }
  return 0;
}

// The mutable state's current VersionHistory after a replay of entry w (OK entries; the
// NDC builder) becomes branch vhs[w].current (with the exec record's VH token); a
// workflow without branches gets its first one (NewVersionHistories, versionHistory.go:350-363).
int cdro_vhs_sync(uint32_t n, cdr_vhs* vhs, cdr_vh_item* pool, const cdr_wf_caps* caps, const cdr_out* out) {
  for (uint32_t w = 0; w < n; w++) {
    const cdr_wf_result& r = out->result[w];
    if (r.code != CDR_OK) continue;
    cdr_vhs& s = vhs[w];
    if (r.n_vh > s.items_cap) {  // the caller's item slots are too few: the workflow fails visibly
      out->result[w] = cdr_wf_result{};
      out->result[w].code = CDR_E_VHS_CAPACITY;
      continue;
    }
    if (s.n_branches == 0) {
      s.n_branches = 1;
      s.current = 0;
    }
    cdr_vh_branch& b = s.branch[s.current];
    const cdr_exec_info& x = out->exec[w];
    b.token.tree = x.branch_tree_id;
    b.token._pad = 0;
    b.token.branch_lo = x.branch_id_lo;
    b.token.branch_hi = x.branch_id_hi;
    b.n_items = r.n_vh;
    b._pad = 0;
    std::memcpy(pool + s.items_off + (uint64_t)s.current * s.items_cap, out->vh + caps[w].vh_off,
                (size_t)r.n_vh * sizeof(cdr_vh_item));
  }
  return 0;
}

}  // extern "C"
