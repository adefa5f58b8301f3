"""refreshTasks after a rebuild (mutableStateTaskRefresher.go:66-160, called by
nDCStateRebuilder.rebuild :154-157).

CPU: the oracle (oracle/refresh_ref.cpp) on small hand-written histories, against
expectations derived line by line from mutableStateTaskRefresher.go and
mutableStateTaskGenerator.go (the reference has no unit test of the refresher:
nDCStateRebuilder_test.go:321 mocks it — parity unpinned by reference vectors).
GPU (-m gpu): refresh.hip through cdr_rebuild_batch == the oracle, task lists and the
refreshed activity / timer rows, on every config, builder and plan mode.
"""
import pytest

from cadence_amd import abi, engine
from cadence_amd.history import HistoryBuilder

NS = 10 ** 9
T0 = 1_600_000_000 * NS
NOW = 1_700_000_000 * NS


def _ev(i, ty, **a):
    return dict(eventId=i, version=7, timestamp=T0 + i * NS, eventType=ty, **a)


def _started(backoff=0, initiator=None, timeout=100, expiration=0):
    x = {"workflowType": {"name": "wt"}, "taskList": {"name": "tl"},
         "executionStartToCloseTimeoutSeconds": timeout, "taskStartToCloseTimeoutSeconds": 10}
    if backoff:
        x["firstDecisionTaskBackoffSeconds"] = backoff
    if initiator is not None:
        x["initiator"] = initiator
    if expiration:
        x["expirationTimestamp"] = expiration
    return _ev(1, "WorkflowExecutionStarted", workflowExecutionStartedEventAttributes=x)


def _dt(i):
    return [_ev(i, "DecisionTaskScheduled", decisionTaskScheduledEventAttributes={
        "taskList": {"name": "tl"}, "startToCloseTimeoutSeconds": 10}),
        _ev(i + 1, "DecisionTaskStarted", decisionTaskStartedEventAttributes={"scheduledEventId": i}),
        _ev(i + 2, "DecisionTaskCompleted", decisionTaskCompletedEventAttributes={
            "scheduledEventId": i, "startedEventId": i + 1})]


def _hb(calls, retention=2, **kw):
    hb = HistoryBuilder()
    w = hb.workflow(workflow_id="wf", run_id="run", request_id="req", retention_days=retention, **kw)
    w.calls = calls
    return hb, hb.build(now_ns=NOW)


def _rebuild(calls, adv=True, **kw):
    import oracle
    hb, b = _hb(calls, **kw)
    out = oracle.rebuild(b, advanced_visibility=adv)
    return out, hb.intern


def _types(rows):
    return [abi.TASK_TYPES[r.type] for r in rows]


def test_running_workflow_tasks():
    """Started + a completed decision + a pending activity + two user timers:
    WorkflowTimeout (now + timeout, start version), RecordWorkflowStarted (running),
    ActivityTask (not started), the activity and user-timer picks, Upsert SA."""
    calls = [[_started()] + _dt(2)[:1], _dt(2)[1:2],
             _dt(2)[2:] + [
                 _ev(5, "ActivityTaskScheduled", activityTaskScheduledEventAttributes={
                     "activityId": "a", "taskList": {"name": "atl"}, "scheduleToStartTimeoutSeconds": 5,
                     "scheduleToCloseTimeoutSeconds": 60, "startToCloseTimeoutSeconds": 30}),
                 _ev(6, "TimerStarted", timerStartedEventAttributes={"timerId": "t1", "startToFireTimeoutSeconds": 50}),
                 _ev(7, "TimerStarted", timerStartedEventAttributes={"timerId": "t2", "startToFireTimeoutSeconds": 20})]]
    out, I = _rebuild(calls)
    assert out.result[0].code == abi.OK
    xt, tt = out.task_rows(0, "xfer"), out.task_rows(0, "ttask")
    assert _types(xt) == ["RecordWorkflowStarted", "ActivityTask", "UpsertWorkflowSearchAttributes"]
    assert all(t.visibility_ts == NOW for t in xt)
    assert (xt[0].version, xt[2].version) == (7, 7)  # start version; NDC current version
    a = xt[1]
    assert (a.event_id, a.domain_id, a.task_list, a.version) == (5, I("domain-id"), I("atl"), 7)
    assert _types(tt) == ["WorkflowTimeout", "ActivityTimeout", "UserTimer"]
    assert (tt[0].visibility_ts, tt[0].version) == (NOW + 100 * NS, 7)
    # ScheduleToStart (T0+5s + 5s) is the earliest activity candidate
    assert (tt[1].event_id, tt[1].timeout_type, tt[1].visibility_ts, tt[1].version) == (5, 1, T0 + 10 * NS, 0)
    assert (tt[2].event_id, tt[2].visibility_ts) == (7, T0 + 27 * NS)
    act, tim = out.rows(0, "act"), out.rows(0, "timer")
    assert [r.timer_task_status for r in act] == [abi.TTS_SCHEDULE_TO_START]
    assert sorted((r.started_id, r.task_id) for r in tim) == [(6, 0), (7, 1)]


def test_no_advanced_visibility():
    out, _ = _rebuild([[_started()] + _dt(2)[:1]], adv=False)
    assert "UpsertWorkflowSearchAttributes" not in _types(out.task_rows(0, "xfer"))


@pytest.mark.parametrize("initiator,ttype", [(None, 1), ("CronSchedule", 1), ("RetryPolicy", 0)])
def test_delayed_decision(initiator, ttype):
    """No decision processed or pending + a first-decision backoff: WorkflowTimeout at
    now + timeout + backoff, WorkflowBackoffTimer at now + backoff, timeout type by
    initiator (nil -> Cron, mutableStateTaskGenerator.go:190-211)."""
    out, _ = _rebuild([[_started(backoff=60, initiator=initiator)]])
    tt = out.task_rows(0, "ttask")
    assert _types(tt) == ["WorkflowTimeout", "WorkflowBackoffTimer"]
    assert tt[0].visibility_ts == NOW + 160 * NS
    assert (tt[1].visibility_ts, tt[1].timeout_type, tt[1].version) == (NOW + 60 * NS, ttype, 7)


def test_delayed_decision_decider_is_an_error():
    import oracle
    _, b = _hb([[_started(backoff=60, initiator="Decider")]])
    out = oracle.rebuild(b)
    assert out.result[0].code == 15  # E_REFRESH_BACKOFF_INITIATOR
    assert out.tasks["n"][0] == out.tasks["n"][1] == 0


def test_expiration_caps_workflow_timeout():
    exp = NOW + 30 * NS
    out, _ = _rebuild([[_started(expiration=exp)] + _dt(2)[:1]])
    assert out.task_rows(0, "ttask")[0].visibility_ts == exp


def test_decision_tasks():
    """Scheduled decision -> DecisionTask (domain, task list, schedule ID, version);
    started -> DecisionTimeout at now + StartToClose (:233-300)."""
    out, I = _rebuild([[_started()] + _dt(2)[:1]])
    d = out.task_rows(0, "xfer")[1]
    assert (abi.TASK_TYPES[d.type], d.event_id, d.domain_id, d.task_list, d.version) == (
        "DecisionTask", 2, I("domain-id"), I("tl"), 7)
    out, _ = _rebuild([[_started()] + _dt(2)[:1], _dt(2)[1:2]])
    tt = out.task_rows(0, "ttask")
    assert _types(tt) == ["WorkflowTimeout", "DecisionTimeout"]
    assert (tt[1].event_id, tt[1].timeout_type, tt[1].visibility_ts, tt[1].version) == (2, 0, NOW + 10 * NS, 7)


def test_closed_workflow():
    """Closed: CloseExecution + DeleteHistoryEvent at now + retention days, no
    RecordWorkflowStarted (:193-231)."""
    calls = [[_started()] + _dt(2)[:1], _dt(2)[1:2],
             _dt(2)[2:] + [_ev(5, "WorkflowExecutionCompleted", workflowExecutionCompletedEventAttributes={})]]
    out, _ = _rebuild(calls, retention=3)
    xt, tt = out.task_rows(0, "xfer"), out.task_rows(0, "ttask")
    assert _types(xt) == ["CloseExecution", "UpsertWorkflowSearchAttributes"]
    assert _types(tt) == ["WorkflowTimeout", "DeleteHistoryEvent"]
    assert tt[1].visibility_ts == NOW + 3 * 86400 * NS


def test_external_tasks():
    """Pending child (not started), request-cancel and signal: target domain ID (the
    execution's for an empty domain), workflow / run, child-only, version (:344-461)."""
    we = {"workflowId": "target-wf", "runId": "target-run"}
    calls = [[_started()] + _dt(2)[:1], _dt(2)[1:2],
             _dt(2)[2:] + [
                 _ev(5, "StartChildWorkflowExecutionInitiated", startChildWorkflowExecutionInitiatedEventAttributes={
                     "domain": "child-dom", "workflowId": "child-wf", "workflowType": {"name": "ct"}}),
                 _ev(6, "SignalExternalWorkflowExecutionInitiated",
                     signalExternalWorkflowExecutionInitiatedEventAttributes={
                         "domain": "", "workflowExecution": we, "signalName": "s", "childWorkflowOnly": True}),
                 _ev(7, "RequestCancelExternalWorkflowExecutionInitiated",
                     requestCancelExternalWorkflowExecutionInitiatedEventAttributes={
                         "domain": "can-dom", "workflowExecution": we})]]
    out, I = _rebuild(calls)
    xt = out.task_rows(0, "xfer")
    assert _types(xt) == ["RecordWorkflowStarted", "StartChildExecution", "CancelExecution", "SignalExecution",
                          "UpsertWorkflowSearchAttributes"]
    c, k, s = xt[1:4]
    assert (c.event_id, c.domain_id, c.target_workflow_id, c.version) == (5, I("id-of-child-dom"), I("child-wf"), 7)
    assert (k.event_id, k.domain_id, k.target_workflow_id, k.target_run_id, k.flags) == (
        7, I("id-of-can-dom"), I("target-wf"), I("target-run"), 0)
    assert (s.event_id, s.domain_id, s.target_run_id, s.flags) == (6, I("domain-id"), I("target-run"), 1)


def _act(i, aid, domain=None):
    x = {"activityId": aid, "taskList": {"name": "atl"}, "scheduleToStartTimeoutSeconds": 5,
         "scheduleToCloseTimeoutSeconds": 60, "startToCloseTimeoutSeconds": 30}
    if domain is not None:
        x["domain"] = domain
    return _ev(i, "ActivityTaskScheduled", activityTaskScheduledEventAttributes=x)


def _cross_domain_calls():
    return [[_started()] + _dt(2)[:1], _dt(2)[1:2],
            _dt(2)[2:] + [_act(5, "local"), _act(6, "empty", ""), _act(7, "remote", "remote-dom")]]


def test_activity_target_domain():
    """generateActivityTransferTasks (mutableStateTaskGenerator.go:302-333): the ActivityTask's
    DomainID is getTargetDomainID(attr.GetDomain()) (:531-545) — the execution's domain for a
    nil or empty domain, the domain cache's ID for a named one."""
    out, I = _rebuild(_cross_domain_calls())
    assert out.result[0].code == abi.OK
    xt = [t for t in out.task_rows(0, "xfer") if abi.TASK_TYPES[t.type] == "ActivityTask"]
    assert [(t.event_id, t.domain_id) for t in xt] == [
        (5, I("domain-id")), (6, I("domain-id")), (7, I("id-of-remote-dom"))]
    assert all(t.task_list == I("atl") for t in xt)


def test_activity_target_domain_missing():
    """A named target domain the domain cache does not know: getTargetDomainID's error
    (:538-541) fails the refresh (CDR_E_DOMAIN_NOT_FOUND), the entry keeps no tasks."""
    import oracle
    hb = HistoryBuilder()
    hb.domains_missing.add("remote-dom")
    w = hb.workflow(workflow_id="wf", run_id="run", request_id="req", retention_days=2)
    w.calls = _cross_domain_calls()
    b = hb.build(now_ns=NOW)
    ref = oracle.replay(b)
    assert ref.result[0].code == abi.OK  # the replay itself never reads the activity's domain
    out = oracle.rebuild(b)
    assert out.result[0].code == 11  # CDR_E_DOMAIN_NOT_FOUND
    assert out.tasks["n"][0] == out.tasks["n"][1] == 0


def test_snapshot_passive_task_versions():
    """CloseTransactionAsSnapshot(passive): setTaskInfo sets every task's Version to the
    current version (historyEngine.go:2383-2397) — timer picks included."""
    import oracle
    calls = [[_started()] + _dt(2)[:1], _dt(2)[1:2], _dt(2)[2:] + [
        dict(_ev(5, "TimerStarted", timerStartedEventAttributes={"timerId": "t", "startToFireTimeoutSeconds": 9}),
             version=9)]]
    _, b = _hb(calls)
    plain, snap = oracle.rebuild(b), oracle.rebuild(b, snapshot=True)
    for kind in ("xfer", "ttask"):
        p, q = plain.task_rows(0, kind), snap.task_rows(0, kind)
        assert len(p) == len(q) > 0
        assert all(t.version == 9 for t in q)
        assert [t.type for t in p] == [t.type for t in q]
    assert [t.version for t in plain.task_rows(0, "ttask")] == [7, 0]  # start version; user timer unset


def test_refresh_caps_bound_oracle():
    """The planner's task capacities bound what the refresher emits on every config."""
    import oracle
    for cfg in range(6):
        b = engine.synth_batch(cfg, 120, seed=cfg + 21, error_rate=0.1)
        out = oracle.rebuild(b)
        assert not [w for w in range(b.n_wfs) if out.result[w].code == 16]  # E_REFRESH_CAPACITY
        assert sum(out.tasks["n"][:2 * b.n_wfs]) > 0


def test_carry_entries_miss_the_start_event():
    """A carried-in entry's start event is not among its own events: the refresher's
    events-cache miss (E_REFRESH_EVENT_NOT_FOUND) — those go through the caller's cache."""
    import oracle
    b = engine.synth_batch(2, 64, seed=5)
    pre, cut = engine.split_batch(b, 2)
    sb = engine.suffix_batch(b, cut, pre, oracle.replay(pre))
    out = oracle.rebuild(sb)
    codes = {out.result[w].code for w in range(sb.n_wfs)}
    assert 14 in codes


# ------------------------------------------------------------------ GPU
def _check(eng, b, adv=True, snapshot=False):
    import oracle
    ref = oracle.rebuild(b, advanced_visibility=adv, snapshot=snapshot)
    got = eng.rebuild(b, advanced_visibility=adv, snapshot=snapshot)
    bad = engine.compare(b, got, ref) + engine.compare_tasks(b, got, ref)
    for w in range(b.n_wfs):
        if got.result[w].code != ref.result[w].code:
            bad.append(f"wf {w}: code {got.result[w].code} != {ref.result[w].code}")
            break
    assert not bad, "\n".join(bad[:10])
    return ref


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5])
def test_gpu_refresh_configs(engine_gpu, cfg):
    b = engine.synth_batch(cfg, 400, seed=0x5EED0400 + cfg, error_rate=0.1 if cfg in (0, 3, 4) else 0.0)
    ref = _check(engine_gpu, b)
    assert sum(ref.tasks["n"][:2 * b.n_wfs]) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("builder", [abi.BUILDER_LOCAL, abi.BUILDER_2DC, abi.BUILDER_NDC])
def test_gpu_refresh_builders(engine_gpu, builder):
    b = engine.synth_batch(0, 300, seed=71 + builder, builder=builder, error_rate=0.2)
    _check(engine_gpu, b, adv=False)
    _check(engine_gpu, b, snapshot=True)


@pytest.mark.gpu
def test_gpu_refresh_lane_only_and_carry(engine_gpu):
    """Every entry on lane slices (no wave slices), and a carried-in batch (misses)."""
    prev = engine_gpu.set_wave(False)
    try:
        _check(engine_gpu, engine.synth_batch(4, 300, seed=81))
    finally:
        engine_gpu.set_wave(prev)
    b = engine.synth_batch(3, 200, seed=83)
    pre, cut = engine.split_batch(b, 2)
    _check(engine_gpu, engine.suffix_batch(b, cut, pre, engine_gpu.replay(pre)))


@pytest.mark.gpu
def test_gpu_refresh_fixture_histories(engine_gpu):
    """The hand-written histories above on the GPU (delayed decision, Decider error,
    expiration cap, externals)."""
    we = {"workflowId": "target-wf", "runId": "target-run"}
    cases = [
        [[_started(backoff=60, initiator="RetryPolicy")]],
        [[_started(backoff=60, initiator="Decider")]],
        [[_started(expiration=NOW + 30 * NS)] + _dt(2)[:1]],
        [[_started()] + _dt(2)[:1], _dt(2)[1:2], _dt(2)[2:] + [
            _ev(5, "StartChildWorkflowExecutionInitiated", startChildWorkflowExecutionInitiatedEventAttributes={
                "domain": "child-dom", "workflowId": "child-wf", "workflowType": {"name": "ct"}}),
            _ev(6, "SignalExternalWorkflowExecutionInitiated", signalExternalWorkflowExecutionInitiatedEventAttributes={
                "domain": "", "workflowExecution": we, "signalName": "s", "childWorkflowOnly": True}),
            _ev(7, "ActivityTaskScheduled", activityTaskScheduledEventAttributes={
                "activityId": "a", "taskList": {"name": "atl"}, "scheduleToStartTimeoutSeconds": 5,
                "scheduleToCloseTimeoutSeconds": 60, "startToCloseTimeoutSeconds": 30}),
            _ev(8, "TimerStarted", timerStartedEventAttributes={"timerId": "t1", "startToFireTimeoutSeconds": 50})]],
    ]
    for calls in cases:
        _, b = _hb(calls)
        _check(engine_gpu, b)


@pytest.mark.gpu
@pytest.mark.parametrize("missing", [False, True])
def test_gpu_activity_target_domain(engine_gpu, missing):
    """GPU twin of the cross-domain activity KATs: refresh.hip reads the scheduled event's
    target domain from the arena record, a missing one fails the entry."""
    hb = HistoryBuilder()
    if missing:
        hb.domains_missing.add("remote-dom")
    w = hb.workflow(workflow_id="wf", run_id="run", request_id="req", retention_days=2)
    w.calls = _cross_domain_calls()
    ref = _check(engine_gpu, hb.build(now_ns=NOW))
    assert ref.result[0].code == (11 if missing else abi.OK)
