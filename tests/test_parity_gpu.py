"""GPU parity: the HIP replay engine vs the CPU restatement (oracle/), field by field.

Inputs are the deterministic synthetic configs of SURVEY §8(d) (small sizes the
oracle finishes in seconds), with and without injected faults so that every error
and panic site is exercised.  Bar: bit-exact (integer/handle state; the only float,
BackoffCoefficient, is a verbatim copy).
"""
import pytest

from cadence_amd import abi, engine

pytestmark = pytest.mark.gpu


def _check(batch, eng, both_paths=False, lanes=True):
    """Default routing (fast-path, wave and lane slices) vs the oracle; `lanes`: again
    with no wave slices (divergent histories on the lane-per-workflow general kernel);
    `both_paths`: again with the fast path off too (everything on the general kernel)."""
    import oracle
    ref = oracle.replay(batch)
    got = eng.replay(batch)
    bad = engine.compare(batch, got, ref)
    assert not bad, "default routing: " + "\n".join(bad[:10])
    old = eng.set_cls(False)  # register-table slices on k_replay_reg alone
    try:
        got = eng.replay(batch)
    finally:
        eng.set_cls(old)
    bad = engine.compare(batch, got, ref)
    assert not bad, "no class-sorted blocks: " + "\n".join(bad[:10])
    old = eng.set_plan_mode(abi.PLAN_WAVE | abi.PLAN_WAVE_ALL)  # every divergent history on a wave
    try:
        got = eng.replay(batch)
    finally:
        eng.set_plan_mode(old)
    bad = engine.compare(batch, got, ref)
    assert not bad, "all divergent on the wave kernel: " + "\n".join(bad[:10])
    if lanes:
        old = eng.set_wave(False)
        try:
            got = eng.replay(batch)
        finally:
            eng.set_wave(old)
        bad = engine.compare(batch, got, ref)
        assert not bad, "lane slices only: " + "\n".join(bad[:10])
    if both_paths:  # the same batch through the general kernel only
        old, oldw = eng.set_fast_path(False), eng.set_wave(False)
        try:
            got = eng.replay(batch)
        finally:
            eng.set_fast_path(old)
            eng.set_wave(oldw)
        bad = engine.compare(batch, got, ref)
        assert not bad, "general kernel: " + "\n".join(bad[:10])
    return ref


@pytest.mark.parametrize("cfg", [1, 2, 3, 4, 5, 0])
def test_synth_configs_clean(engine_gpu, cfg):
    b = engine.synth_batch(cfg, 300, seed=0x5EED0000 + cfg)
    if cfg in (3, 4, 5, 0):  # divergent shapes: the wave kernel must be exercised
        assert engine.slice_kinds(b, mode=abi.PLAN_WAVE | abi.PLAN_WAVE_ALL)[1] > 0
    ref = _check(b, engine_gpu)
    assert engine.status_histogram(ref).get("OK", 0) > 0


@pytest.mark.parametrize("cfg", [0, 3, 4, 5])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_synth_configs_faults(engine_gpu, cfg, seed):
    b = engine.synth_batch(cfg, 400, seed=seed * 1000 + cfg, error_rate=0.3)
    ref = _check(b, engine_gpu)
    hist = engine.status_histogram(ref)
    assert len(hist) > 1, hist


@pytest.mark.parametrize("builder", [abi.BUILDER_LOCAL, abi.BUILDER_2DC, abi.BUILDER_NDC])
def test_builders(engine_gpu, builder):
    b = engine.synth_batch(0, 300, seed=77 + builder, builder=builder, error_rate=0.1)
    _check(b, engine_gpu)


def test_rebuild_next_event_check(engine_gpu):
    b = engine.synth_batch(5, 200, seed=99, rebuild=True, error_rate=0.2)
    _check(b, engine_gpu)


def test_long_histories(engine_gpu):
    b = engine.synth_batch(4, 40, seed=5, target_len=3000, max_len=20000)
    _check(b, engine_gpu)


@pytest.mark.parametrize("cfg", [3, 4, 5])
def test_wave_kernel_configs(engine_gpu, cfg):
    """Larger divergent batches (every entry that fits the wave kernel gets a wave
    slice), checked against the oracle only."""
    b = engine.synth_batch(cfg, 1500, seed=0x5EED0100 + cfg, error_rate=0.1)
    nf, nw, ns = engine.slice_kinds(b, mode=abi.PLAN_WAVE | abi.PLAN_WAVE_ALL)
    assert nw > 0, (nf, nw, ns)
    _check(b, engine_gpu, lanes=False)


@pytest.mark.parametrize("cfg", [1, 2])
@pytest.mark.parametrize("err", [0.0, 0.3])
def test_fast_path(engine_gpu, cfg, err):
    """Sequential-activity shapes run on the fast-path kernel; with and without
    injected faults it must agree with the oracle and with the general kernel."""
    b = engine.synth_batch(cfg, 700, seed=0x5EED0000 + cfg + int(err * 10), error_rate=err,
                           fault_kinds=abi.FAULTS_FAST)
    nf, ns = engine.fast_slices(b)
    assert nf > 0, (nf, ns)
    _check(b, engine_gpu, both_paths=True)


@pytest.mark.parametrize("builder", [abi.BUILDER_LOCAL, abi.BUILDER_NDC])
@pytest.mark.parametrize("err", [0.0, 0.2])
def test_fast_path_builders(engine_gpu, builder, err):
    b = engine.synth_batch(2, 300, seed=91 + builder, builder=builder, error_rate=err, fault_kinds=abi.FAULTS_FAST)
    nf, ns = engine.fast_slices(b)
    if err == 0.0:  # faults may leave two activities pending (not a fast-path shape)
        assert nf == ns
    _check(b, engine_gpu, both_paths=True)


def _overflow_history(hb, wid, n_sa, n_rp, builder):
    from cadence_amd.history import HistoryBuilder  # noqa: F401  (hb is one)
    w = hb.workflow(workflow_id=wid, run_id=wid + "-run", request_id="q", builder=builder, failover_version=1)
    t = 1_600_000_000 * 10 ** 9
    ev = lambda i, ty, **a: dict(eventId=i, version=1, timestamp=t + i, eventType=ty, **a)  # noqa: E731
    started = ev(1, "WorkflowExecutionStarted", workflowExecutionStartedEventAttributes={
        "workflowType": {"name": "wt"}, "taskList": {"name": "tl"}, "executionStartToCloseTimeoutSeconds": 60,
        "taskStartToCloseTimeoutSeconds": 10,
        "searchAttributes": {"indexedFields": {f"key-{i}": f"v-{i}" for i in range(n_sa)}},
        "prevAutoResetPoints": {"points": [{"binaryChecksum": f"cks-{i}", "runId": "old-run",
                                            "firstDecisionCompletedId": 4, "createdTimeNano": 5,
                                            "resettable": True} for i in range(n_rp)]}})
    calls = [[started, ev(2, "DecisionTaskScheduled", decisionTaskScheduledEventAttributes={
        "startToCloseTimeoutSeconds": 10, "attempt": 0})]]
    i = 3
    for cks in [f"cks-{n_rp - 1}", "cks-3", "brand-new", f"cks-{n_rp // 2}", "brand-new", "another"]:
        calls.append([ev(i, "DecisionTaskStarted", decisionTaskStartedEventAttributes={
            "scheduledEventId": i - 1, "requestId": f"r{i}"})])
        calls.append([ev(i + 1, "DecisionTaskCompleted", decisionTaskCompletedEventAttributes={
            "scheduledEventId": i - 1, "startedEventId": i, "binaryChecksum": cks}),
            ev(i + 2, "UpsertWorkflowSearchAttributes", upsertWorkflowSearchAttributesEventAttributes={
                "searchAttributes": {"indexedFields": {f"key-{n_sa - 1}": f"w{i}", "key-1": f"w{i}",
                                                       f"fresh-{i}": "x"}}}),
            ev(i + 3, "DecisionTaskScheduled", decisionTaskScheduledEventAttributes={
                "startToCloseTimeoutSeconds": 10, "attempt": 0})])
        i += 4
    calls.append([ev(i, "DecisionTaskStarted", decisionTaskStartedEventAttributes={
        "scheduledEventId": i - 1, "requestId": "r"})])
    calls.append([ev(i + 1, "DecisionTaskCompleted", decisionTaskCompletedEventAttributes={
        "scheduledEventId": i - 1, "startedEventId": i}),
        ev(i + 2, "WorkflowExecutionCompleted", workflowExecutionCompletedEventAttributes={})])
    w.calls = calls


@pytest.mark.parametrize("n", [10, 64, 65, 150])
def test_wave_kernel_table_overflow(engine_gpu, n):
    """More than 64 search attributes and reset points: the wave kernel's lane tables
    hold the first 64, the rest are looked up in their output rows."""
    from cadence_amd.history import HistoryBuilder
    hb = HistoryBuilder()
    for j, bld in enumerate([abi.BUILDER_NDC, abi.BUILDER_2DC, abi.BUILDER_LOCAL]):
        _overflow_history(hb, f"wf-{j}", n, n, bld)
    b = hb.build()
    nf, nw, ns = engine.slice_kinds(b, mode=abi.PLAN_WAVE | abi.PLAN_WAVE_ALL)
    assert nw == 3, (nf, nw, ns)
    ref = _check(b, engine_gpu)
    assert engine.status_histogram(ref) == {"OK": 3}
