"""Builders for the NDC conflict-resolution tests: the reference's hand-crafted 3-branch
history (host/ndc/nDC_integration_test.go:310-613, transcribed in
tests/golden/ndc_handcrafted_3branch.input.json) as the base / rebuild / fork batches and
the replication task that cadence_amd.ndc.replicate consumes."""
import ctypes as C
import json
import os

from cadence_amd import abi
from cadence_amd.history import HistoryBuilder

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURE = os.path.join(HERE, "golden", "ndc_handcrafted_3branch.input.json")
FORK_TOKEN = (0xF0F0, 0xB2B2)  # ForkHistoryBranch's NewBranchToken BranchID (fixed here)


def handcrafted():
    """(base, rebuild, [(fork batch, tasks, items)], doc): base = eventsBatch1 + eventsBatch3
    (both applied to the one branch in the test's order), rebuild = eventsBatch1 (the new
    branch's events 1..14), fork = eventsBatch2 with versionHistory2 as its task's
    incoming VersionHistory."""
    doc = json.load(open(FIXTURE))
    hb = HistoryBuilder()
    kw = dict(workflow_id=doc["workflow_id"], run_id=doc["run_id"], request_id="replication-request",
              builder=abi.BUILDER_NDC, failover_version=21)

    def batch(calls, expected_next=0):
        hb.workflows = []
        w = hb.workflow(expected_next_event_id=expected_next, **kw)
        w.calls = calls
        return hb.build()
    base = batch(doc["eventsBatch1"] + doc["eventsBatch3"])
    rebuild = batch(doc["eventsBatch1"], expected_next=15)
    fork = batch(doc["eventsBatch2"])
    vh2 = doc["versionHistory2"]
    items = (abi.CdrVHItem * len(vh2))()
    for i, (e, v) in enumerate(vh2):
        items[i].event_id, items[i].version = e, v
    t = (abi.CdrNdcTask * 1)()
    t[0].items_off, t[0].n_items = 0, len(vh2)
    last = doc["eventsBatch2"][-1][-1]
    t[0].first_event_id = doc["eventsBatch2"][0][0]["eventId"]
    t[0].last_event_id, t[0].last_version = last["eventId"], last["version"]
    t[0].version = last["version"]
    t[0].new_token.tree = base.wfs[0].run_id
    t[0].new_token.branch_lo, t[0].new_token.branch_hi = FORK_TOKEN
    # every batch's handles come from the same interner: the last build holds them all
    for b in (base, rebuild):
        b.strings = fork.strings
    return base, rebuild, [(fork, t, items)], doc


def check_reference_outcome(final, vhs, pool, decs, doc):
    """The outcome for TestHandcraftedMultipleBranches (nDC_integration_test.go:323-613).

    Pinned by the reference: every replication task applies without an error (the test's
    s.applyEvents asserts NoError), and the two branches' VersionHistories are the ones the
    test itself builds from the event batches (versionHistory2 / versionHistory3 via
    DuplicateUntilLCAItem((14, 21)) + eventBatchesToVersionHistory, :571-584).
    DERIVED, not asserted by the reference (restating nDCBranchMgr / nDCConflictResolver /
    nDCStateRebuilder on these events — the builder's reading of the flow): the decision's
    action, branch index and rebuild point, the branch token, and the final
    ExecutionInfo / pending-row values below the marker."""
    from cadence_amd import ndc
    d = decs[0][0]
    assert (abi.STATUS[d.code], abi.NDC_ACTIONS[d.action], d.branch_index, d.created) == ("OK", "REBUILD", 1, 1)
    assert (d.lca.event_id, d.lca.version) == (14, 21) and d.rebuild_next_event_id == 15
    assert vhs[0].n_branches == 2 and vhs[0].current == 1
    assert ndc.branch_items(vhs, pool, 0, 0) == [tuple(x) for x in doc["versionHistory3"]]
    assert ndc.branch_items(vhs, pool, 0, 1) == [tuple(x) for x in doc["versionHistory2"]]
    assert (vhs[0].branch[1].token.branch_lo, vhs[0].branch[1].token.branch_hi) == FORK_TOKEN
    r, x = final.result[0], final.exec[0]
    assert abi.STATUS[r.code] == "OK"  # pinned: the applies succeed
    # ---- derived from the restated flow (not asserted by the reference test)
    assert (x.state, x.close_status) == (abi.STATE_COMPLETED, abi.CLOSE_TIMED_OUT)
    assert (x.next_event_id, x.last_first_event_id, x.completion_event_batch_id) == (16, 15, 15)
    assert x.signal_count == 2
    assert (x.branch_id_lo, x.branch_id_hi) == FORK_TOKEN  # SetCurrentBranchToken(target)
    # the activity timed out only on branch 0: on the rebuilt branch it is still pending
    acts = final.rows(0, "act")
    assert [(a.schedule_id, a.started_id) for a in acts] == [(6, 7)]
    # the decision started at 14 is still pending (the workflow timed out around it)
    assert (x.decision_schedule_id, x.decision_started_id) == (13, 14)
    assert C.sizeof(x) == 256
