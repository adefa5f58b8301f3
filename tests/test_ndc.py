"""NDC conflict resolution on the CPU restatement (oracle.ndc_replicate, replay_ref.cpp
cdro_ndc_replicate_round): the reference's hand-crafted 3-branch history and the forked
synthetic config 5 — branch decisions, nDCStateRebuilder.rebuild (replay, refreshTasks,
VersionHistory verification) and apply onto the rebuilt state kept in memory
(nDCConflictResolver.go:117-184, nDCHistoryReplicator.go:330-398)."""
import collections
import ctypes as C

from cadence_amd import abi, engine, ndc

from . import ndc_fixture


def test_handcrafted_three_branches_oracle():
    import oracle
    base, rebuild, forks, doc = ndc_fixture.handcrafted()
    final, vhs, pool, decs, rounds = oracle.ndc_replicate(base, rebuild, forks)
    ndc_fixture.check_reference_outcome(final, vhs, pool, decs, doc)
    rb, ap = rounds[0]
    assert abi.STATUS[rb.result[0].code] == "OK" and rb.exec[0].next_event_id == 15  # events 1..14 rebuilt
    # refreshTasks after the rebuild (nDCStateRebuilder.go:154-157): the pending activity's
    # timeout task and its marked TimerTaskStatus carry into the applied state
    tt = [abi.TASK_TYPES[t.type] for t in rb.task_rows(0, "ttask")]
    assert "ActivityTimeout" in tt
    assert [a.timer_task_status for a in final.rows(0, "act")] == [a.timer_task_status for a in rb.rows(0, "act")]


def test_forked_config5_oracle_invariants():
    """Every fork A forces a rebuild (its version is above every base version); fork B
    rebuilds or backfills; rebuilt version histories always verify; the final current
    branch holds the highest last-write version (IsRebuilt false) and its items are the
    replayed state's version history."""
    import oracle
    n = 200
    base, rebuild, forks = ndc.synth_forked(5, n, 0x5EED0C05)
    final, vhs, pool, decs, rounds = oracle.ndc_replicate(base, rebuild, forks, threads=4)
    assert engine.status_histogram(final) == {"OK": n}
    a = collections.Counter(abi.NDC_ACTIONS[decs[0][w].action] for w in range(n) if decs[0][w].code == abi.OK)
    b = collections.Counter(abi.NDC_ACTIONS[decs[1][w].action] for w in range(n) if decs[1][w].code == abi.OK)
    assert a == {"REBUILD": n}
    assert set(b) == {"REBUILD", "BACKFILL"}
    for w in range(n):
        s = vhs[w]
        assert s.n_branches == 3
        assert oracle.lib().cdro_vhs_is_rebuilt(C.byref(s), pool) == 0  # IsRebuilt: current = newest
        last = [ndc.branch_items(vhs, pool, w, k)[-1][1] for k in range(3)]
        assert last[s.current] == max(last)
        cur = ndc.branch_items(vhs, pool, w, s.current)
        assert [(i.event_id, i.version) for i in final.rows(w, "vh")] == cur
        # fork point: every branch shares the base's items up to it
        f = forks[0][1][w].first_event_id - 1
        pre = [it for it in ndc.branch_items(vhs, pool, w, 0) if it[0] < f]
        for k in (1, 2):
            assert ndc.branch_items(vhs, pool, w, k)[:len(pre)] == pre
    # round 2's backfills touched no state: their apply records were never run
    for w in range(n):
        if abi.NDC_ACTIONS[decs[1][w].action] == "BACKFILL":
            assert rounds[1][1].result[w].code == 65  # CDR_NOT_RUN


def in_memory_case():
    """(suffix batch, loaded state, {in_memory flag: oracle outputs}) of the in-memory KAT."""
    import numpy as np
    import oracle
    from cadence_amd.history import HistoryBuilder
    NS = 10 ** 9

    def ev(i, ty, ver=3, **a):
        return dict(eventId=i, version=ver, timestamp=1_600_000_000 * NS + i * NS, eventType=ty, **a)
    started = ev(1, "WorkflowExecutionStarted", workflowExecutionStartedEventAttributes={
        "workflowType": {"name": "wt"}, "taskList": {"name": "tl"}, "executionStartToCloseTimeoutSeconds": 100,
        "taskStartToCloseTimeoutSeconds": 10})
    dts = ev(2, "DecisionTaskScheduled", decisionTaskScheduledEventAttributes={"taskList": {"name": "tl"},
                                                                              "startToCloseTimeoutSeconds": 10})
    dtst = ev(3, "DecisionTaskStarted", decisionTaskStartedEventAttributes={"scheduledEventId": 2})
    term = ev(4, "WorkflowExecutionTerminated", workflowExecutionTerminatedEventAttributes={})
    hb = HistoryBuilder()
    kw = dict(workflow_id="wf", run_id="run", request_id="req", builder=abi.BUILDER_NDC, failover_version=3)
    w = hb.workflow(**kw)
    w.calls = [[started, dts], [dtst], [term]]
    pre = hb.build()
    pre_out = oracle.replay(pre)
    assert pre_out.result[0].code == abi.OK
    hb.workflows = []
    w = hb.workflow(**kw)
    w.calls = [[ev(5, "DecisionTaskTimedOut", ver=9, decisionTaskTimedOutEventAttributes={
        "scheduledEventId": 2, "startedEventId": 3, "timeoutType": "START_TO_CLOSE"})]]
    suf = hb.build()
    outs = {}
    for mem in (0, 1):
        suf.carry = engine.Carry(src=np.array([0], np.int32), state=pre_out, in_memory=np.array([mem], np.uint8))
        outs[mem] = oracle.replay(suf)
    return suf, pre_out, outs


def test_in_memory_carry_keeps_the_rebuilt_current_version():
    """cdr_carry.in_memory (the rebuilt builder never goes through Load): a closed NDC
    workflow that receives a decision failure keeps the rebuilt currentVersion for the
    transient decision's version, where a Load gives EmptyVersion (mutableStateBuilder.go:291)."""
    suf, pre_out, outs = in_memory_case()
    x0, x1 = outs[0].exec[0], outs[1].exec[0]
    assert outs[0].result[0].code == outs[1].result[0].code == abi.OK
    # the transient decision (ReplicateTransientDecisionTaskScheduled) takes GetCurrentVersion()
    assert (x0.decision_schedule_id, x0.decision_attempt) == (x1.decision_schedule_id, x1.decision_attempt) == (5, 1)
    assert (x0.decision_version, x1.decision_version) == (-24, 3)  # Load: EmptyVersion; in memory: the last item's


def test_apply_working_slots_bounded_by_live_rows():
    """cdr_plan_ndc_apply sizes an apply entry's live sets (the general kernel's working
    slots) by the loaded state's peak live rows — the sum of the parts' simulated peaks —
    and its pending tables by the same bound (the table capacities are peak live sets,
    cdr_wf_caps), never by every row any part ever added."""
    import ctypes as C
    base, rebuild, forks = ndc.synth_forked(5, 200, 0x5EED0C05)
    caps_tab = ndc.state_caps_for(base, rebuild, forks).caps
    bound = ndc.state_caps_for(base, rebuild, forks, live_sum=True).caps
    parts = [engine.plan(base), engine.plan(rebuild)] + [engine.plan(fb) for fb, _, _ in forks]
    L = abi.lib()
    fb = forks[0][0]
    own = engine.plan(fb).caps
    caps = (abi.CdrWfCaps * fb.n_wfs)()
    tot = abi.CdrTotals()
    assert L.cdr_plan_ndc_apply(C.byref(fb.cstruct()), bound, caps, C.byref(tot)) == 0
    scheduled = 0
    for w in range(fb.n_wfs):
        peak = sum(p.caps[w].act_live for p in parts)
        assert bound[w].act_live == peak
        assert bound[w].act_cap == caps_tab[w].act_cap == peak  # pending rows: the peak live sets
        assert caps[w].act_live == own[w].act_live + peak
        assert caps[w].act_cap == own[w].act_cap + caps_tab[w].act_cap
        scheduled += sum(1 for p in (base, rebuild, fb) for k in range(p.wfs[w].ev_len)
                         if p.events[p.wfs[w].ev_off + k].type == abi.EV["ActivityTaskScheduled"])
    assert sum(caps[w].act_cap for w in range(fb.n_wfs)) < scheduled


def test_vh_item_capacity_is_reported():
    """The VersionHistories item slots are the caller's (cdr_vhs.items_cap): a state whose
    version history outgrows them fails with CDR_E_VHS_CAPACITY (it is not silently left
    without a branch — which surfaced as E_VH_NO_LCA at the next task); the default slots
    come from the run's own histories (ndc.items_cap_for) and never overflow."""
    import oracle
    base, rebuild, forks = ndc.synth_forked(5, 64, 0x5EED0C07)
    need = ndc.items_cap_for(base, rebuild, forks)
    assert (need >= ndc.ITEMS_CAP).all()
    small = 4
    st, _, _, _, _ = oracle.ndc_replicate(base, rebuild, forks, items_cap=small)
    hist = engine.status_histogram(st)
    assert hist.get("E_VHS_CAPACITY", 0) > 0, hist
    st, _, _, _, _ = oracle.ndc_replicate(base, rebuild, forks)
    assert engine.status_histogram(st) == {"OK": 64}
