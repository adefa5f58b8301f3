"""Transfer / timer task emission (stateBuilder.go:613-804).

CPU: the oracle's task lists against the reference's own expectations in
stateBuilder_test.go (restated through small hand-written histories): the Started
event's WorkflowTimeout / WorkflowBackoffTimer / RecordWorkflowStarted tasks
(:153-220), the transient decision's DecisionTask (:1180-1230), the close tasks
(:251), the child / signal / cancel transfer tasks (:818, :913, :1006) and the
timer-builder tasks.  GPU (-m gpu): the general kernel's task lists == the oracle's,
field by field, for every config, builder and carried-in state.
"""
import pytest

from cadence_amd import abi, engine
from cadence_amd.history import HistoryBuilder

NS = 10 ** 9
T0 = 1_600_000_000 * NS


def _ev(i, ty, ts=None, **a):
    return dict(eventId=i, version=1, timestamp=T0 + i * NS if ts is None else ts, eventType=ty, **a)


def _started(i=1, backoff=0, cron=False, timeout=100):
    x = {"workflowType": {"name": "wt"}, "taskList": {"name": "tl"},
         "executionStartToCloseTimeoutSeconds": timeout, "taskStartToCloseTimeoutSeconds": 10}
    if backoff:
        x["firstDecisionTaskBackoffSeconds"] = backoff
    if cron:
        x["initiator"] = "CronSchedule"
        x["cronSchedule"] = "* * * * *"
    return _ev(i, "WorkflowExecutionStarted", workflowExecutionStartedEventAttributes=x)


def _dt_sched(i, att=0):
    return _ev(i, "DecisionTaskScheduled", decisionTaskScheduledEventAttributes={
        "taskList": {"name": "tl"}, "startToCloseTimeoutSeconds": 10, "attempt": att})


def _replay(calls, retention=1, **kw):
    import oracle
    hb = HistoryBuilder()
    w = hb.workflow(workflow_id="wf", run_id="run", request_id="req", retention_days=retention, **kw)
    w.calls = calls
    b = hb.build()
    out = oracle.replay(b, tasks=True)
    assert out.result[0].code == abi.OK, out.result[0].code
    I = hb.intern
    return out, I


def _types(rows):
    return [abi.TASK_TYPES[r.type] for r in rows]


@pytest.mark.parametrize("backoff,cron", [(0, False), (60, True), (30, False)])
def test_started_tasks(backoff, cron):
    """stateBuilder_test.go:153-220: WorkflowTimeoutTask at now + WorkflowTimeout (+
    backoff), a WorkflowBackoffTimerTask at now + backoff when there is one (timeout
    type Cron for a cron initiator), one RecordWorkflowStartedTask."""
    out, I = _replay([[_started(backoff=backoff, cron=cron)]])
    tt, xt = out.task_rows(0, "ttask"), out.task_rows(0, "xfer")
    assert _types(xt) == ["RecordWorkflowStarted"]
    ts = T0 + NS
    if backoff:
        assert _types(tt) == ["WorkflowBackoffTimer", "WorkflowTimeout"]
        assert tt[0].visibility_ts == ts + backoff * NS
        assert tt[0].timeout_type == (1 if cron else 0)  # WorkflowBackoffTimeoutType{Retry,Cron}
        assert tt[1].visibility_ts == ts + (100 + backoff) * NS
    else:
        assert _types(tt) == ["WorkflowTimeout"]
        assert tt[0].visibility_ts == ts + 100 * NS


def test_decision_tasks_and_transient():
    """DecisionTask per scheduled decision (DomainID, TaskList, ScheduleID); a
    DecisionTimeoutTask at Started + StartToClose; a timed-out decision schedules a
    transient DecisionTask at the call's NextEventID (stateBuilder_test.go:1180-1230)."""
    calls = [[_started(), _dt_sched(2)],
             [_ev(3, "DecisionTaskStarted", decisionTaskStartedEventAttributes={"scheduledEventId": 2,
                                                                                 "requestId": "r"})],
             [_ev(4, "DecisionTaskTimedOut", decisionTaskTimedOutEventAttributes={
                 "scheduledEventId": 2, "startedEventId": 3, "timeoutType": 0})]]
    out, I = _replay(calls)
    xt, tt = out.task_rows(0, "xfer"), out.task_rows(0, "ttask")
    assert _types(xt) == ["RecordWorkflowStarted", "DecisionTask", "DecisionTask"]
    assert (xt[1].event_id, xt[1].domain_id, xt[1].task_list) == (2, I("domain-id"), I("tl"))
    assert xt[2].event_id == 4  # NextEventID as of the call's start (transient ScheduleID)
    assert _types(tt) == ["WorkflowTimeout", "DecisionTimeout"]
    d = tt[1]
    assert (d.event_id, d.visibility_ts, d.timeout_type, d.attempt) == (2, T0 + 3 * NS + 10 * NS, 0, 0)


def test_close_tasks_retention():
    """appendTasksForFinishedExecutions: CloseExecutionTask + DeleteHistoryEventTask at
    the close event's time + retention days (stateBuilder_test.go:251)."""
    calls = [[_started(), _dt_sched(2)],
             [_ev(3, "DecisionTaskStarted", decisionTaskStartedEventAttributes={"scheduledEventId": 2})],
             [_ev(4, "DecisionTaskCompleted", decisionTaskCompletedEventAttributes={"scheduledEventId": 2,
                                                                                    "startedEventId": 3}),
              _ev(5, "WorkflowExecutionCompleted", workflowExecutionCompletedEventAttributes={})]]
    out, _ = _replay(calls, retention=3)
    xt, tt = out.task_rows(0, "xfer"), out.task_rows(0, "ttask")
    assert _types(xt)[-1] == "CloseExecution"
    assert _types(tt)[-1] == "DeleteHistoryEvent"
    assert tt[-1].visibility_ts == T0 + 5 * NS + 3 * 86400 * NS


def test_external_tasks():
    """StartChildExecutionTask / SignalExecutionTask / CancelExecutionTask carry the
    target domain's ID, workflow, run and child-only flag (stateBuilder_test.go:818,
    :913, :1006) and the initiated event ID."""
    we = {"workflowId": "target-wf", "runId": "target-run"}
    calls = [[_started(), _dt_sched(2)],
             [_ev(3, "DecisionTaskStarted", decisionTaskStartedEventAttributes={"scheduledEventId": 2})],
             [_ev(4, "DecisionTaskCompleted", decisionTaskCompletedEventAttributes={"scheduledEventId": 2,
                                                                                    "startedEventId": 3}),
              _ev(5, "StartChildWorkflowExecutionInitiated", startChildWorkflowExecutionInitiatedEventAttributes={
                  "domain": "child-dom", "workflowId": "child-wf", "workflowType": {"name": "ct"}}),
              _ev(6, "SignalExternalWorkflowExecutionInitiated",
                  signalExternalWorkflowExecutionInitiatedEventAttributes={
                      "domain": "sig-dom", "workflowExecution": we, "signalName": "s", "childWorkflowOnly": True}),
              _ev(7, "RequestCancelExternalWorkflowExecutionInitiated",
                  requestCancelExternalWorkflowExecutionInitiatedEventAttributes={
                      "domain": "can-dom", "workflowExecution": we})]]
    out, I = _replay(calls)
    xt = out.task_rows(0, "xfer")
    assert _types(xt)[-3:] == ["StartChildExecution", "SignalExecution", "CancelExecution"]
    c, s, k = xt[-3:]
    assert (c.event_id, c.domain_id, c.target_workflow_id) == (5, I("id-of-child-dom"), I("child-wf"))
    assert (s.event_id, s.domain_id, s.target_workflow_id, s.target_run_id, s.flags) == (
        6, I("id-of-sig-dom"), I("target-wf"), I("target-run"), 1)
    assert (k.event_id, k.domain_id, k.target_run_id, k.flags) == (7, I("id-of-can-dom"), I("target-run"), 0)


def test_timer_builder_tasks():
    """UserTimerTask for the earliest timer when it is first picked (EventID = its
    StartedID, visibility = its expiry); ActivityTimeoutTask for the earliest activity
    candidate (ScheduleToStart before start, timerBuilder_test.go:85-215)."""
    calls = [[_started(), _dt_sched(2)],
             [_ev(3, "DecisionTaskStarted", decisionTaskStartedEventAttributes={"scheduledEventId": 2})],
             [_ev(4, "DecisionTaskCompleted", decisionTaskCompletedEventAttributes={"scheduledEventId": 2,
                                                                                    "startedEventId": 3}),
              _ev(5, "TimerStarted", timerStartedEventAttributes={"timerId": "t1", "startToFireTimeoutSeconds": 50}),
              _ev(6, "TimerStarted", timerStartedEventAttributes={"timerId": "t2", "startToFireTimeoutSeconds": 20}),
              _ev(7, "ActivityTaskScheduled", activityTaskScheduledEventAttributes={
                  "activityId": "a", "taskList": {"name": "atl"}, "scheduleToStartTimeoutSeconds": 5,
                  "scheduleToCloseTimeoutSeconds": 60, "startToCloseTimeoutSeconds": 30,
                  "heartbeatTimeoutSeconds": 0})]]
    out, I = _replay(calls)
    tt = out.task_rows(0, "ttask")
    ut = [t for t in tt if abi.TASK_TYPES[t.type] == "UserTimer"]
    at = [t for t in tt if abi.TASK_TYPES[t.type] == "ActivityTimeout"]
    assert [(t.event_id, t.visibility_ts) for t in ut] == [(5, T0 + 5 * NS + 50 * NS), (6, T0 + 6 * NS + 20 * NS)]
    assert [(t.event_id, t.timeout_type, t.visibility_ts) for t in at] == [(7, 1, T0 + 7 * NS + 5 * NS)]
    assert _types(out.task_rows(0, "xfer"))[-1] == "ActivityTask"


def test_task_caps_bound_oracle():
    """The planner's task capacities bound what the oracle emits on every config."""
    import oracle
    for cfg in range(6):
        b = engine.synth_batch(cfg, 120, seed=cfg + 11, error_rate=0.1)
        out = oracle.replay(b, tasks=True)
        for w in range(b.n_wfs):
            if out.result[w].code == abi.OK:
                c = out.plan.caps[w]
                assert out.tasks["n"][2 * w] <= c.xfer_cap and out.tasks["n"][2 * w + 1] <= c.ttask_cap


# ------------------------------------------------------------------ GPU
def _check_tasks(eng, b):
    import oracle
    ref = oracle.replay(b, tasks=True)
    got = eng.replay(b, tasks=True)
    bad = engine.compare(b, got, ref) + engine.compare_tasks(b, got, ref)
    assert not bad, "\n".join(bad[:10])
    return ref


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5])
def test_gpu_tasks_configs(engine_gpu, cfg):
    b = engine.synth_batch(cfg, 300, seed=0x5EED0300 + cfg, error_rate=0.1 if cfg in (0, 3, 4) else 0.0)
    ref = _check_tasks(engine_gpu, b)
    assert sum(ref.tasks["n"][:2 * b.n_wfs]) > 0


@pytest.mark.gpu
def test_gpu_tasks_staging_follows_each_batch(engine_gpu):
    """Two task batches of the same size through one context: the class kernels'
    task staging is sized from each launch's own task rows, not from the previous batch that
    happened to use the same capacity buffer — a second batch with more tasks per entry must
    still equal the oracle (with the staging sized by the first, its records would overrun)."""
    import oracle
    small = engine.synth_batch(3, 320, seed=0x5EED0601, target_len=40)
    big = engine.synth_batch(5, 320, seed=0x5EED0602)
    assert small.n_wfs == big.n_wfs
    old = engine_gpu.set_cls(abi.CLS_BUILD)
    try:
        for b in (small, big):
            ref = oracle.replay(b, tasks=True)
            got = engine_gpu.replay(b, tasks=True)
            bad = engine.compare(b, got, ref) + engine.compare_tasks(b, got, ref)
            assert not bad, "\n".join(bad[:10])
    finally:
        engine_gpu.set_cls(old)
    assert sum(oracle.replay(big, tasks=True).tasks["n"][:2 * big.n_wfs]) > \
        sum(oracle.replay(small, tasks=True).tasks["n"][:2 * small.n_wfs])


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [3, 4, 5])
@pytest.mark.parametrize("err", [0.0, 0.2])
def test_gpu_tasks_class_path(engine_gpu, cfg, err):
    """Task lists from the class kernels (k_replay_cls<TASKS> staging + k_tasks_merge) through
    the host-buffer call: with the k_replay_reg<TASKS> pass behind them (CLS_BUILD) every
    entry's state and lists equal the oracle's — injected faults included, whose entries the
    class kernel hands on; alone (CLS_ALONE) every entry it kept has the oracle's lists, and on
    a clean batch it keeps every entry."""
    import oracle
    b = engine.synth_batch(cfg, 600, seed=0x5EED0500 + cfg + int(err * 10), error_rate=err)
    ref = oracle.replay(b, tasks=True)
    old = engine_gpu.set_cls(abi.CLS_BUILD)
    try:
        got = engine_gpu.replay(b, tasks=True)
        bad = engine.compare(b, got, ref) + engine.compare_tasks(b, got, ref)
        assert not bad, "\n".join(bad[:10])
        engine_gpu.set_cls(abi.CLS_ALONE)
        alone = engine_gpu.replay(b, tasks=True)
    finally:
        engine_gpu.set_cls(old)
    kept = [w for w in range(b.n_wfs) if alone.result[w].code == abi.OK]
    assert not engine.compare_tasks(b, alone, ref)  # (entries OK in both)
    assert sum(alone.task_rows(w, "xfer").__len__() for w in kept) > 0
    if err == 0.0:
        assert len(kept) == b.n_wfs


@pytest.mark.gpu
@pytest.mark.parametrize("builder", [abi.BUILDER_LOCAL, abi.BUILDER_2DC, abi.BUILDER_NDC])
def test_gpu_tasks_builders(engine_gpu, builder):
    _check_tasks(engine_gpu, engine.synth_batch(0, 300, seed=51 + builder, builder=builder, error_rate=0.2))


@pytest.mark.gpu
def test_gpu_tasks_carry(engine_gpu):
    """Tasks of a replay onto loaded state (ActivityTimeoutTask.Attempt from the row)."""
    b = engine.synth_batch(3, 300, seed=61)
    pre, cut = engine.split_batch(b, 2)
    sb = engine.suffix_batch(b, cut, pre, engine_gpu.replay(pre))
    _check_tasks(engine_gpu, sb)


@pytest.mark.gpu
def test_gpu_tasks_fixture_histories(engine_gpu):
    """The hand-written KAT histories above, on the GPU."""
    import oracle
    hb = HistoryBuilder()
    w = hb.workflow(workflow_id="wf", run_id="run", request_id="req")
    w.calls = [[_started(backoff=60, cron=True), _dt_sched(2)],
               [_ev(3, "DecisionTaskStarted", decisionTaskStartedEventAttributes={"scheduledEventId": 2})],
               [_ev(4, "DecisionTaskTimedOut", decisionTaskTimedOutEventAttributes={
                   "scheduledEventId": 2, "startedEventId": 3, "timeoutType": 0})]]
    b = hb.build()
    ref = oracle.replay(b, tasks=True)
    got = engine_gpu.replay(b, tasks=True)
    assert not engine.compare_tasks(b, got, ref)
    assert _types(got.task_rows(0, "xfer")) == ["RecordWorkflowStarted", "DecisionTask", "DecisionTask"]


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [1, 2])
def test_gpu_tasks_fast_kernel(engine_gpu, cfg):
    """C1 / C2 with tasks stay on k_replay_fast (its TASKS instantiation, replay_fast.inc):
    the task lists equal the oracle's and the general kernel's (fast path off)."""
    b = engine.synth_batch(cfg, 1500, seed=0x5EED0310 + cfg)
    nf, ns = engine.fast_slices(b)
    assert nf == ns > 0  # every slice of the task plan is a fast-path slice
    ref = _check_tasks(engine_gpu, b)
    old = engine_gpu.set_fast_path(False)
    try:
        gen = engine_gpu.replay(b, tasks=True)
    finally:
        engine_gpu.set_fast_path(old)
    assert not engine.compare_tasks(b, gen, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,reg,cls", [(2, True, None), (3, True, None), (3, False, None), (3, True, "host"),
                                         (4, True, "host"), (5, True, "host")])
def test_gpu_tasks_device_batch(engine_gpu, cfg, reg, cls):
    """The `bench.py --tasks` path: a synthetic sliced batch carrying task capacities
    (DeviceBatch(tasks=True), a plan without wave / PAR slices) replayed by
    cdr_replay_sliced_async — C2 on k_replay_fast<TASKS>; C3's register-table slices on
    k_replay_reg<..., TASKS> without class blocks (and, with the register-table path off, every
    C3 slice on the general kernel's TASKS instantiation); with class blocks (cls="host", C3-C5)
    on k_replay_cls<..., TASKS> + k_tasks_merge, the entries they hand on on k_replay_reg<TASKS>
    — equals the oracle's task lists for the same workflows, entry by entry and byte for byte."""
    import ctypes as C

    import numpy as np
    import torch

    import oracle
    from cadence_amd.synth import DeviceBatch
    n, seed = 1500, 0x5EED0410 + cfg
    db = DeviceBatch(torch, cfg, np.arange(n, dtype=np.uint32), seed, plan_mode=0, cls=cls, tasks=True)
    L = abi.lib()
    ctx = L.cdr_create(torch.cuda.current_device(), None)
    try:
        if not reg:
            L.cdr_set_reg_path(ctx, 0)
        stream = torch.cuda.current_stream().cuda_stream
        assert L.cdr_replay_sliced_async(ctx, C.byref(db.db), C.byref(db.out), C.c_void_p(stream)) == 0
        torch.cuda.synchronize()
    finally:
        L.cdr_destroy(ctx)
    ref = oracle.replay(engine.synth_batch(cfg, n, seed), tasks=True)
    ne = db.info.n_entries
    assert ne == ref.n_wfs
    nt = db.out_t["n_tasks"][: 8 * ne].view(torch.int32).cpu().numpy().reshape(-1, 2)
    bufs = {"xfer": db.out_t["transfer"].cpu().numpy().tobytes(), "ttask": db.out_t["timer_tasks"].cpu().numpy().tobytes()}
    sz = C.sizeof(abi.CdrTask)
    bad, total = [], 0
    for w in range(ne):
        assert ref.result[w].code == abi.OK
        cap = db.h_caps[w]
        for kind, off, k in (("xfer", cap.xfer_off, 0), ("ttask", cap.ttask_off, 1)):
            want = [bytes(r) for r in ref.task_rows(w, kind)]
            got = [bufs[kind][(off + j) * sz:(off + j + 1) * sz] for j in range(int(nt[w, k]))]
            total += len(want)
            if got != want:
                bad.append((w, kind, len(got), len(want)))
    assert not bad, bad[:5]
    assert total > n


@pytest.mark.parametrize("cfg", [2, 3, 4, 5])
def test_synth_sliced_task_caps(cfg):
    """The synthetic sliced plan's task capacities (bench.py --tasks) are cdr_plan_caps's for
    the same workflows, entry by entry, with prefix offsets in entry order."""
    import ctypes as C

    import numpy as np
    L = abi.lib()
    n, seed = 700, 0x5EED0420 + cfg
    idx = np.arange(n, dtype=np.uint32)
    p = abi.CdrSynthParams(config=cfg, n_wfs=n, seed=seed, target_len=0, max_len=0, error_rate=0.0, builder=-1,
                           rebuild=0, index_map=idx.ctypes.data, plan_mode=0, long_stride=0)
    info = abi.CdrSynthPlanInfo()
    assert L.cdr_synth_sliced_plan(C.byref(p), C.byref(info)) == 0
    slab = np.empty(info.n_rows * 64 * abi.EL_BYTES, np.uint8)
    lane = np.empty(info.n_slices * 64, np.int32)
    slen, row0 = np.empty(info.n_slices, np.uint32), np.empty(info.n_slices, np.uint64)
    z = [np.zeros(info.n_slices, t) for t in (np.uint64, np.uint32, np.uint32, np.uint32)]
    arena = np.empty(max(1, info.arena_words), np.uint64)
    wfs, caps = (abi.CdrWfDesc * info.n_entries)(), (abi.CdrWfCaps * info.n_entries)()
    kvs, rps = np.zeros(max(1, info.n_kvs) * 2, np.uint32), (abi.CdrResetPoint * max(1, info.n_rps))()
    s = abi.CdrSlices(n_slices=info.n_slices, n_rows=info.n_rows, arena_words=info.arena_words)
    s.slice_row0, s.slice_len, s.lane_wf, s.slab, s.arena = (row0.ctypes.data, slen.ctypes.data, lane.ctypes.data,
                                                             slab.ctypes.data, arena.ctypes.data)
    s.slice_scratch_off, s.slice_act_slots, s.slice_tim_slots, s.slice_flags = [a.ctypes.data for a in z]
    meta = abi.CdrBatch()
    assert L.cdr_synth_sliced_fill(C.byref(p), C.byref(s), wfs, caps, kvs.ctypes.data, rps, C.byref(meta), 4) == 0
    ref = engine.plan(engine.synth_batch(cfg, n, seed))
    assert info.totals.xfer == ref.totals.xfer and info.totals.ttask == ref.totals.ttask
    for w in range(info.n_entries):
        a, b = caps[w], ref.caps[w]
        assert (a.xfer_cap, a.ttask_cap, a.xfer_off, a.ttask_off) == (b.xfer_cap, b.ttask_cap, b.xfer_off, b.ttask_off), w
