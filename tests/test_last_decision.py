"""applyEvents' second return value, lastDecision *decisionInfo (stateBuilder.go:126,200,
213,238,256,610), per entry in cdr_out.last_decision.

The reference's tests discard it (every stateBuilder_test.go call is `_, _, _, err :=`),
so the CPU cases below restate the Go directly: the decisionInfo returned by
ReplicateDecisionTaskScheduledEvent / ReplicateDecisionTaskStartedEvent /
ReplicateTransientDecisionTaskScheduled (mutableStateDecisionTaskManager.go:143-253) of
the LAST call, nil when that call has none.  The GPU cases check every kernel against
that restatement on synthetic populations whose calls are split at random, so the
in-call capture path (a source event followed by a clearing event in the same call) is
exercised."""
import ctypes as C
import dataclasses

import numpy as np
import pytest

import oracle
from cadence_amd import abi, engine
from cadence_amd.history import HistoryBuilder

T0 = 1_600_000_000_000_000_000
NOW = 1_700_000_000_000_000_000
STARTED = {"eventId": 1, "version": 5, "timestamp": T0, "eventType": "WorkflowExecutionStarted",
           "workflowExecutionStartedEventAttributes": {"taskList": {"name": "tl"},
                                                       "taskStartToCloseTimeoutSeconds": 17}}


def dts(eid, ts, timeout=10, attempt=0):
    return {"eventId": eid, "version": 5, "timestamp": ts, "eventType": "DecisionTaskScheduled",
            "decisionTaskScheduledEventAttributes": {"startToCloseTimeoutSeconds": timeout, "attempt": attempt}}


def dtst(eid, ts, sched, req="req"):
    return {"eventId": eid, "version": 6, "timestamp": ts, "eventType": "DecisionTaskStarted",
            "decisionTaskStartedEventAttributes": {"scheduledEventId": sched, "requestId": req}}


def dtc(eid, ts, sched, started):
    return {"eventId": eid, "version": 6, "timestamp": ts, "eventType": "DecisionTaskCompleted",
            "decisionTaskCompletedEventAttributes": {"scheduledEventId": sched, "startedEventId": started}}


def dtf(eid, ts, sched, started):
    return {"eventId": eid, "version": 6, "timestamp": ts, "eventType": "DecisionTaskFailed",
            "decisionTaskFailedEventAttributes": {"scheduledEventId": sched, "startedEventId": started}}


def replay(calls, builder=abi.BUILDER_LOCAL):
    hb = HistoryBuilder()
    w = hb.workflow(workflow_id="wid", run_id="rid", request_id="req", builder=builder, failover_version=5)
    w.calls = calls
    b = hb.build(now_ns=NOW)
    out = oracle.replay(b)
    assert out.result[0].code == abi.OK, abi.STATUS[out.result[0].code]
    return b, out.last_decision[0]


def test_scheduled_in_last_call():
    b, ld = replay([[STARTED, dts(2, T0 + 1, timeout=11, attempt=0)]])
    assert ld.source == abi.LD_SCHEDULED and ld.event_index == 1
    assert (ld.version, ld.schedule_id, ld.started_id, ld.attempt) == (5, 2, abi.EMPTY_EVENT_ID, 0)
    assert (ld.scheduled_ts, ld.started_ts, ld.original_scheduled_ts, ld.decision_timeout) == (T0 + 1, 0, T0 + 1, 11)
    assert b.strings[ld.request_id] == "emptyUuid"


def test_started_in_last_call():
    b, ld = replay([[STARTED, dts(2, T0 + 1, attempt=3)], [dtst(3, T0 + 2, 2, "r-3")]])
    assert ld.source == abi.LD_STARTED and ld.event_index == 2
    # the replicated Started resets the attempt (:224); timeout / scheduled times carried
    assert (ld.version, ld.schedule_id, ld.started_id, ld.attempt) == (6, 2, 3, 0)
    assert (ld.scheduled_ts, ld.started_ts, ld.original_scheduled_ts, ld.decision_timeout) == (T0 + 1, T0 + 2,
                                                                                              T0 + 1, 10)
    assert b.strings[ld.request_id] == "r-3"


def test_completed_after_started_in_the_same_call():
    """The pointer returned at Started keeps its values after DecisionTaskCompleted
    deletes the decision (DeleteDecision builds a new record, :659-674)."""
    _, ld = replay([[STARTED, dts(2, T0 + 1)], [dtst(3, T0 + 2, 2), dtc(4, T0 + 3, 2, 3),
                                                 {"eventId": 5, "version": 6, "timestamp": T0 + 3,
                                                  "eventType": "WorkflowExecutionSignaled"}]])
    assert ld.source == abi.LD_STARTED and ld.event_index == 2
    assert (ld.schedule_id, ld.started_id, ld.started_ts) == (2, 3, T0 + 2)


def test_transient_after_failure():
    """DecisionTaskFailed then the transient decision: ScheduleID = NextEventID as of the
    call's start, Attempt = 1, ScheduledTimestamp = now, Version = GetCurrentVersion()."""
    _, ld = replay([[STARTED, dts(2, T0 + 1)], [dtst(3, T0 + 2, 2)], [dtf(4, T0 + 3, 2, 3)]])
    assert ld.source == abi.LD_TRANSIENT and ld.event_index == 3
    assert (ld.schedule_id, ld.started_id, ld.attempt, ld.scheduled_ts) == (4, abi.EMPTY_EVENT_ID, 1, NOW)
    assert (ld.original_scheduled_ts, ld.decision_timeout, ld.version) == (0, 17, abi.EMPTY_VERSION)


def test_transient_version_ndc():
    _, ld = replay([[STARTED, dts(2, T0 + 1)], [dtst(3, T0 + 2, 2)], [dtf(4, T0 + 3, 2, 3)]], abi.BUILDER_NDC)
    assert ld.source == abi.LD_TRANSIENT and ld.version == 6  # the current version: the failure event's


def test_no_decision_in_last_call():
    _, ld = replay([[STARTED, dts(2, T0 + 1)], [dtst(3, T0 + 2, 2)],
                    [dtc(4, T0 + 3, 2, 3), {"eventId": 5, "version": 6, "timestamp": T0 + 3,
                                             "eventType": "WorkflowExecutionSignaled"}]])
    assert ld.source == abi.LD_NONE and bytes(ld) == bytes(abi.CdrLastDecision())


def merge_calls(batch, seed, p=0.5):
    """The same histories with adjacent applyEvents calls merged at random (batch-first
    flags cleared), for entries without a continue-as-new call: a source event and a
    clearing event then share a call."""
    rng = np.random.default_rng(seed)
    ev = (abi.CdrEvent * len(batch.events))()
    C.memmove(ev, batch.events, C.sizeof(ev))
    for w in range(batch.n_wfs):
        d = batch.wfs[w]
        if d.parent >= 0 or d.newrun >= 0:
            continue
        for k in range(1, d.ev_len):
            e = ev[d.ev_off + k]
            if (e.flags & abi.EVF_BATCH_FIRST) and rng.random() < p:
                e.flags &= ~abi.EVF_BATCH_FIRST
    return dataclasses.replace(batch, events=ev)


def _in_call_captures(batch, out):
    """Entries whose lastDecision source event is followed, in its call, by a clearing
    event (DecisionTaskCompleted / Failed / TimedOut): the kernels' in-loop capture."""
    n = 0
    clear = {abi.EV["DecisionTaskCompleted"], abi.EV["DecisionTaskFailed"], abi.EV["DecisionTaskTimedOut"]}
    for w in range(batch.n_wfs):
        ld = out.last_decision[w]
        if out.result[w].code != abi.OK or ld.source == abi.LD_NONE:
            continue
        d = batch.wfs[w]
        for k in range(int(ld.event_index) + 1, d.ev_len):
            ev = batch.events[d.ev_off + k]
            if ev.flags & abi.EVF_BATCH_FIRST:
                break
            if ev.type in clear:
                n += 1
                break
    return n


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [1, 2, 3, 4, 5])
@pytest.mark.parametrize("kernels", ["default", "general", "wave_all"])
def test_gpu_last_decision_matches_oracle(engine_gpu, cfg, kernels):
    b = merge_calls(engine.synth_batch(cfg, 300, seed=0x1D0 + cfg), seed=cfg)  # in-call captures
    ref = oracle.replay(b, threads=8)
    old_fast = engine_gpu.set_fast_path(kernels != "general")
    old_mode = engine_gpu.set_plan_mode(abi.PLAN_WAVE | abi.PLAN_WAVE_ALL if kernels == "wave_all" else
                                        (0 if kernels == "general" else abi.PLAN_WAVE))
    try:
        got = engine_gpu.replay(b)
    finally:
        engine_gpu.set_fast_path(old_fast)
        engine_gpu.set_plan_mode(old_mode)
    bad = engine.compare(b, got, ref)
    assert not bad, "\n".join(bad)
    src = np.bincount([ref.last_decision[w].source for w in range(b.n_wfs) if ref.result[w].code == abi.OK],
                      minlength=4)
    assert src[abi.LD_SCHEDULED] + src[abi.LD_STARTED] > 0, src


def test_split_batches_reach_the_capture_path():
    """The GPU cases above cover the in-call capture (CPU check of the population)."""
    total = 0
    for cfg in (1, 2, 3, 4, 5):
        b = merge_calls(engine.synth_batch(cfg, 300, seed=0x1D0 + cfg), seed=cfg)
        total += _in_call_captures(b, oracle.replay(b, threads=8))
    assert total > 0


def one_entry(batch, w):
    """Entry w of `batch` (plus its continue-as-new run) as a batch of its own."""
    d = batch.wfs[w]
    ids = [w] + ([d.newrun] if d.newrun >= 0 else [])
    wfs = (abi.CdrWfDesc * len(ids))()
    for i, x in enumerate(ids):
        C.memmove(C.byref(wfs[i]), C.byref(batch.wfs[x]), C.sizeof(abi.CdrWfDesc))
    if len(ids) == 2:
        wfs[0].newrun, wfs[1].parent = 1, 0
    return dataclasses.replace(batch, wfs=wfs, carry=None)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [1, 3, 4, 5])
def test_gpu_replay_one_matches_oracle(engine_gpu, cfg):
    """cdr_replay_one (the shim's single-workflow call, persistent per-context buffers)
    on 40 workflows one after another, each against the oracle."""
    b = merge_calls(engine.synth_batch(cfg, 40, seed=0x0E + cfg), seed=cfg)
    for w in range(b.n_wfs):
        if b.wfs[w].parent >= 0:
            continue
        one = one_entry(b, w)
        got = engine_gpu.replay_one(one)
        ref = oracle.replay(one)
        bad = engine.compare(one, got, ref)
        assert not bad, (w, bad)
