"""More of the reference's known-answer tests restated on the CPU restatement (oracle/),
each with a GPU twin (the same batch through libcdr, compared field by field).

  * stateBuilder_test.go:367-520  continue-as-new: the new run's mutable state, the
    outer run's close tasks and the new run's tasks
  * stateBuilder_test.go:775-1050 child / signal-external / request-cancel initiation
    (the pending rows ReplicateXInitiated builds, InitiatedEventBatchID = the call's
    first event, and the transfer task each call appends) and their failures
  * stateBuilder_test.go:1433-1625 child closes (the row goes, no task)
  * mutableStateBuilder_test.go:111-129,233-257 with its prepare helper :493-645 — the
    replicated transient-decision sequence and a failover before the next failure.

The reference's expectations are mock-call assertions or a hand-built expected builder;
the values below are what those builders hold (file:line on each assertion)."""
import pytest

import oracle
from cadence_amd import abi, engine
from cadence_amd.history import HistoryBuilder

NS = 1_000_000_000
NOW = 1_650_000_000_000_000_000  # the test's time.Now()
T_BATCH = 1_700_000_000_000_000_000  # cdr_batch.now_ns (timeSource.Now() of the replay)
TARGET_DOMAIN, TARGET_DOMAIN_ID = "some random target domain name", "deadbeef-0123-4567-890a-bcdef0123458"
PARENT_DOMAIN, PARENT_DOMAIN_ID = "some random parent domain name", "deadbeef-0123-4567-890a-bcdef0123457"
DOMAIN_ID = "deadbeef-0123-4567-890a-bcdef0123456"
TF_CHILD_ONLY = 0x1  # schema.h CDR_TF_CHILD_ONLY


def ev(eid, etype, version=1, ts=NOW, **attrs):
    e = {"eventId": eid, "version": version, "timestamp": ts, "eventType": etype}
    if attrs:
        e[etype[0].lower() + etype[1:] + "EventAttributes"] = attrs
    return e


def started(eid=1, version=1, ts=NOW, **kw):
    a = {"workflowType": {"name": "some random workflow type"}, "taskList": {"name": "some random tasklist"},
         "executionStartToCloseTimeoutSeconds": 110, "taskStartToCloseTimeoutSeconds": 11}
    a.update(kw)
    return ev(eid, "WorkflowExecutionStarted", version, ts, **a)


def decision_round(first_id, version=1, ts=NOW):
    """DecisionTaskScheduled / Started / Completed as three calls starting at first_id."""
    return [[ev(first_id, "DecisionTaskScheduled", version, ts, startToCloseTimeoutSeconds=11)],
            [ev(first_id + 1, "DecisionTaskStarted", version, ts, scheduledEventId=first_id, requestId="r")],
            [ev(first_id + 2, "DecisionTaskCompleted", version, ts, scheduledEventId=first_id,
                startedEventId=first_id + 1)]]


def builder():
    hb = HistoryBuilder()
    hb.domain_ids = {TARGET_DOMAIN: TARGET_DOMAIN_ID, PARENT_DOMAIN: PARENT_DOMAIN_ID}
    return hb


def wf(hb, calls, b=abi.BUILDER_2DC, **kw):
    w = hb.workflow(workflow_id="some random workflow ID", run_id="some-run-id", request_id="req",
                    domain_id=DOMAIN_ID, builder=b, failover_version=1, **kw)
    w.calls = calls
    return w


def cluster(v0=1, v1=2):
    c = abi.CdrClusterMeta()
    c.failover_version_increment = 10
    c.current_cluster = 0
    c.n_clusters = 2
    c.initial_version[0] = v0
    c.initial_version[1] = v1
    return c


def replay_both(b, gpu=None, tasks=True):
    ref = oracle.replay(b, tasks=tasks)
    if gpu is not None:
        old = gpu.set_plan_mode(0)  # task emission lives in the general kernel's plan
        try:
            got = gpu.replay(b, tasks=tasks)
        finally:
            gpu.set_plan_mode(old)
        bad = engine.compare(b, got, ref)
        assert not bad, "\n".join(bad)
        if tasks:
            bad = engine.compare_tasks(b, got, ref)
            assert not bad, "\n".join(bad)
    return ref


def tasks_of(out, w, kind):
    return [(abi.TASK_TYPES[t.type], t) for t in out.task_rows(w, kind)]


# ---------------------------------------------------------------- continue-as-new
def can_batch():
    """stateBuilder_test.go:367-520: the outer run closes with ContinuedAsNew (event 130);
    the new run is Started (parent domain / execution / initiated 144) + Signaled +
    DecisionTaskScheduled (attempt 123), replayed with the replication-state builder
    (newRunNDC false)."""
    hb = builder()
    calls = [[started(1)]] + decision_round(2) + [[ev(130, "WorkflowExecutionContinuedAsNew",
                                                       newExecutionRunId="new-run-id")]]
    w = wf(hb, calls, new_run_call=4, new_run_ndc=False)
    w.new_run_history = [
        started(1, parentWorkflowDomain=PARENT_DOMAIN,
                parentWorkflowExecution={"workflowId": "some random parent workflow ID", "runId": "parent-run"},
                parentInitiatedEventId=144),
        ev(2, "WorkflowExecutionSignaled", signalName="some random signal name"),
        ev(3, "DecisionTaskScheduled", taskList={"name": "some random tasklist"}, startToCloseTimeoutSeconds=11,
           attempt=123)]
    return hb.build(now_ns=T_BATCH, cluster=cluster())


def check_can(b, out):
    S = b.strings
    assert abi.STATUS[out.result[0].code] == "OK" and abi.STATUS[out.result[1].code] == "OK"
    assert out.result[0].flags & abi.RF_NEWRUN_APPLIED
    x = out.exec[1]  # expectedNewRunStateBuilder (:470-504)
    assert (S[x.domain_id], S[x.workflow_id], S[x.run_id]) == (DOMAIN_ID, "some random workflow ID", "new-run-id")
    assert (S[x.parent_domain_id], S[x.parent_workflow_id], S[x.parent_run_id], x.initiated_id) == (
        PARENT_DOMAIN_ID, "some random parent workflow ID", "parent-run", 144)
    assert (S[x.task_list], S[x.workflow_type], x.workflow_timeout, x.decision_timeout_value) == (
        "some random tasklist", "some random workflow type", 110, 11)
    assert (x.state, x.close_status, x.signal_count) == (abi.STATE_CREATED, abi.CLOSE_NONE, 1)
    assert (x.decision_version, x.decision_schedule_id, x.decision_started_id, x.decision_attempt) == (1, 3, -23, 123)
    assert (x.decision_timeout, x.decision_scheduled_ts, x.decision_original_scheduled_ts) == (11, NOW, NOW)
    assert S[x.decision_request_id] == "emptyUuid"
    assert (x.last_first_event_id, x.next_event_id, x.last_processed_event) == (1, 4, -23)  # :496-497
    rs = out.repl[1]  # :500-504
    assert (rs.start_version, rs.current_version, rs.last_write_version, rs.last_write_event_id) == (1, 1, 1, 3)
    # the outer run's tasks of the CAN call (:506-511) and the new run's (:513-521)
    xo = [(n, t.event_id) for n, t in tasks_of(out, 0, "xfer")][-1:]
    to = [(n, t.visibility_ts) for n, t in tasks_of(out, 0, "ttask")][-1:]
    assert xo == [("CloseExecution", 0)]
    assert to == [("DeleteHistoryEvent", NOW + 1 * 24 * 3600 * NS)]  # retention 1 day after the CAN event
    assert [(n, t.visibility_ts) for n, t in tasks_of(out, 1, "ttask")] == [("WorkflowTimeout", NOW + 110 * NS)]
    nx = tasks_of(out, 1, "xfer")
    assert [n for n, _ in nx] == ["RecordWorkflowStarted", "DecisionTask"]
    assert (S[nx[1][1].domain_id], S[nx[1][1].task_list], nx[1][1].event_id) == (DOMAIN_ID, "some random tasklist", 3)


def test_continue_as_new_new_run_oracle():
    b = can_batch()
    check_can(b, replay_both(b))


@pytest.mark.gpu
def test_continue_as_new_new_run_gpu(engine_gpu):
    b = can_batch()
    check_can(b, replay_both(b, engine_gpu))


# ------------------------------------------------- child / signal / cancel initiation
def initiated_batch(kind, fail=False):
    """stateBuilder_test.go:775-1050: one initiating event 130 in a call of its own (its
    batch id is itself), optionally followed by the failure event in the next call."""
    hb = builder()
    base = [[started(1)]] + decision_round(2)
    tgt = {"domain": TARGET_DOMAIN,
           "workflowExecution": {"workflowId": "some random target workflow ID", "runId": "target-run-id"}}
    if kind == "child":
        e = ev(130, "StartChildWorkflowExecutionInitiated", domain=TARGET_DOMAIN,
               workflowId="some random target workflow ID", workflowType={"name": "child-type"})
        f = ev(131, "StartChildWorkflowExecutionFailed", initiatedEventId=130)
    elif kind == "signal":
        e = ev(130, "SignalExternalWorkflowExecutionInitiated", signalName="some random signal name",
               input="some random signal input", childWorkflowOnly=True, **tgt)
        f = ev(131, "SignalExternalWorkflowExecutionFailed", initiatedEventId=130)
    else:
        e = ev(130, "RequestCancelExternalWorkflowExecutionInitiated", childWorkflowOnly=True,
               control="some random control", **tgt)
        f = ev(131, "RequestCancelExternalWorkflowExecutionFailed", initiatedEventId=130)
    calls = base + [[e]] + ([[f]] if fail else [])
    wf(hb, calls)
    return hb.build(now_ns=T_BATCH, cluster=cluster())


def check_initiated(kind, b, out, fail):
    S = b.strings
    assert abi.STATUS[out.result[0].code] == "OK"
    table = {"child": "child", "signal": "signal", "cancel": "cancel"}[kind]
    rows = out.rows(0, table)
    xfer = tasks_of(out, 0, "xfer")
    if fail:  # ReplicateXFailed removes the row; the failure call adds no task (:829-860, :926-957, :1019-1050)
        assert rows == []
        assert xfer[-1][0] != "CloseExecution" and len([n for n, _ in xfer if n in (
            "StartChildExecution", "SignalExecution", "CancelExecution")]) == 1
        return
    (r,) = rows
    assert (r.version, r.initiated_id, r.initiated_event_batch_id) == (1, 130, 130)
    name, t = xfer[-1]
    if kind == "child":  # ChildExecutionInfo (:800-807), StartChildExecutionTask (:818-822)
        assert r.started_id == abi.EMPTY_EVENT_ID and S[r.domain_name] == TARGET_DOMAIN
        assert (name, S[t.domain_id], S[t.target_workflow_id], t.event_id) == (
            "StartChildExecution", TARGET_DOMAIN_ID, "some random target workflow ID", 130)
    else:  # SignalExecutionTask (:915-921) / CancelExecutionTask (:1008-1014)
        if kind == "signal":
            assert S[r.signal_name] == "some random signal name"
        want = "SignalExecution" if kind == "signal" else "CancelExecution"
        assert (name, S[t.domain_id], S[t.target_workflow_id], S[t.target_run_id], t.flags, t.event_id) == (
            want, TARGET_DOMAIN_ID, "some random target workflow ID", "target-run-id", TF_CHILD_ONLY, 130)
    assert tasks_of(out, 0, "ttask")[-1][0] != "DeleteHistoryEvent"


@pytest.mark.parametrize("kind", ["child", "signal", "cancel"])
@pytest.mark.parametrize("fail", [False, True])
def test_initiated_oracle(kind, fail):
    b = initiated_batch(kind, fail)
    check_initiated(kind, b, replay_both(b), fail)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["child", "signal", "cancel"])
@pytest.mark.parametrize("fail", [False, True])
def test_initiated_gpu(engine_gpu, kind, fail):
    b = initiated_batch(kind, fail)
    check_initiated(kind, b, replay_both(b, engine_gpu), fail)


# ------------------------------------------------------------------ child closes
CHILD_CLOSES = ["ChildWorkflowExecutionCompleted", "ChildWorkflowExecutionFailed", "ChildWorkflowExecutionCanceled",
                "ChildWorkflowExecutionTimedOut", "ChildWorkflowExecutionTerminated"]


def child_close_batch(close):
    hb = builder()
    calls = [[started(1)]] + decision_round(2) + [
        [ev(130, "StartChildWorkflowExecutionInitiated", domain=TARGET_DOMAIN, workflowId="child-wid")],
        [ev(131, "ChildWorkflowExecutionStarted", initiatedEventId=130,
            workflowExecution={"workflowId": "child-wid", "runId": "child-run"})]]
    if close:
        calls.append([ev(132, close, initiatedEventId=130)])
    wf(hb, calls)
    return hb.build(now_ns=T_BATCH, cluster=cluster())


def check_child_close(b, out, close):
    S = b.strings
    assert abi.STATUS[out.result[0].code] == "OK"
    n_x, n_t = len(out.task_rows(0, "xfer")), len(out.task_rows(0, "ttask"))
    if close is None:  # ChildWorkflowExecutionStarted (:1497-1528): StartedID / run id set, no task
        (r,) = out.rows(0, "child")
        assert (r.started_id, S[r.started_workflow_id], S[r.started_run_id]) == (131, "child-wid", "child-run")
        return n_x, n_t
    assert out.rows(0, "child") == []  # ReplicateChildWorkflowExecution*Event deletes the row
    return n_x, n_t


@pytest.mark.parametrize("close", CHILD_CLOSES)
def test_child_close_oracle(close):
    """:1433-1625: a child close appends no transfer / timer task."""
    b0 = child_close_batch(None)
    n0 = check_child_close(b0, replay_both(b0), None)
    b = child_close_batch(close)
    assert check_child_close(b, replay_both(b), close) == n0


@pytest.mark.gpu
@pytest.mark.parametrize("close", CHILD_CLOSES + [None])
def test_child_close_gpu(engine_gpu, close):
    b = child_close_batch(close)
    check_child_close(b, replay_both(b, engine_gpu), close)


# ---------------------------------------------- replicated transient decisions + failover
def transient_batch(last):
    """mutableStateBuilder_test.go:493-645 as replicated batches (version 12, 2DC):
    Started, DT scheduled / started / failed (-> transient decision, attempt 1), the
    next DT scheduled with attempt 123 and started (the replicated Started resets the
    attempt to 0, mutableStateDecisionTaskManager.go:216-224); then `last`: the
    decision completes (:83-108), or a failover to version 13 times it out / fails it
    (:111-129, :233-257) -> a transient decision of the failover version."""
    hb = builder()
    v, t = 12, NOW
    calls = [[started(1, v, t, taskStartToCloseTimeoutSeconds=11, executionStartToCloseTimeoutSeconds=222)],
             [ev(2, "DecisionTaskScheduled", v, t, startToCloseTimeoutSeconds=11, attempt=0)],
             [ev(3, "DecisionTaskStarted", v, t, scheduledEventId=2, requestId="r3")],
             [ev(4, "DecisionTaskFailed", v, t, scheduledEventId=2, startedEventId=3)],
             [ev(5, "DecisionTaskScheduled", v, t, startToCloseTimeoutSeconds=11, attempt=123)],
             [ev(6, "DecisionTaskStarted", v, t, scheduledEventId=5, requestId="r6")]]
    if last == "completed":
        calls.append([ev(7, "DecisionTaskCompleted", v, t + 1, scheduledEventId=5, startedEventId=6)])
    elif last == "timedout":
        calls.append([ev(7, "DecisionTaskTimedOut", v + 1, t + 1, scheduledEventId=5, startedEventId=6,
                         timeoutType="START_TO_CLOSE")])
    elif last == "failed":
        calls.append([ev(7, "DecisionTaskFailed", v + 1, t + 1, scheduledEventId=5, startedEventId=6)])
    w = wf(hb, calls)
    w.failover_version = v
    return hb.build(now_ns=T_BATCH, cluster=cluster(2, 3))  # 12: this cluster, 13: the other


def check_transient(b, out, last):
    assert abi.STATUS[out.result[0].code] == "OK"
    x, ld = out.exec[0], out.last_decision[0]
    if last is None:  # after the prepare helper: decision 5 started at 6, attempt reset to 0
        assert (x.decision_schedule_id, x.decision_started_id, x.decision_attempt, x.decision_version) == (5, 6, 0, 12)
        assert (ld.source, ld.schedule_id, ld.attempt) == (abi.LD_STARTED, 5, 0)
        return
    if last == "completed":  # no decision left, none transient
        assert (x.decision_schedule_id, x.decision_started_id, x.decision_attempt) == (-23, -23, 0)
        assert x.last_processed_event == 6 and ld.source == abi.LD_NONE
        return
    # the failover failure: attempt 0 + 1 -> a transient decision at NextEventID 7 of
    # the failover version, scheduled now (:169-198)
    assert (x.decision_schedule_id, x.decision_started_id, x.decision_attempt) == (7, -23, 1)
    assert (x.decision_version, x.decision_timeout, x.decision_scheduled_ts) == (13, 11, T_BATCH)
    assert (ld.source, ld.version, ld.schedule_id, ld.attempt) == (abi.LD_TRANSIENT, 13, 7, 1)
    assert out.repl[0].current_version == 13


@pytest.mark.parametrize("last", [None, "completed", "timedout", "failed"])
def test_transient_failover_oracle(last):
    b = transient_batch(last)
    check_transient(b, replay_both(b), last)


@pytest.mark.gpu
@pytest.mark.parametrize("last", [None, "completed", "timedout", "failed"])
def test_transient_failover_gpu(engine_gpu, last):
    b = transient_batch(last)
    check_transient(b, replay_both(b, engine_gpu), last)
