"""Edge cases of the batch boundary (the reference's own: an empty history is an
InternalFailureError, stateBuilder.go:121-123; histories up to the history count
limit, service/history/service.go:264 = 204,800 events; ragged batches).

CPU: the planner and the oracle on those shapes.  GPU: the HIP path == the oracle.
"""
import pytest

from cadence_amd import abi, engine
from cadence_amd.history import HistoryBuilder

MAX_EVENTS = 204_800  # HistoryCountLimitError default (service.go:264)


def _empty_and_tiny():
    hb = HistoryBuilder()
    hb.workflow(workflow_id="empty", run_id="r0", request_id="q").calls = []
    w = hb.workflow(workflow_id="one", run_id="r1", request_id="q")
    w.calls = [[dict(eventId=1, version=1, timestamp=10 ** 18, eventType="WorkflowExecutionStarted",
                     workflowExecutionStartedEventAttributes={"taskList": {"name": "tl"}})]]
    hb.workflow(workflow_id="empty2", run_id="r2", request_id="q").calls = []
    return hb.build()


def test_oracle_empty_and_single_event_entries():
    import oracle
    b = _empty_and_tiny()
    out = oracle.replay(b)
    assert [out.result[w].code for w in range(3)] == [1, abi.OK, 1]  # CDR_E_HISTORY_EMPTY
    assert out.exec[1].next_event_id == 2


def test_plan_max_length_history():
    b = engine.synth_batch(3, 2, seed=9, target_len=MAX_EVENTS, max_len=MAX_EVENTS)
    lens = sorted(b.wfs[w].ev_len for w in range(b.n_wfs) if b.wfs[w].parent < 0)
    assert lens[-1] >= MAX_EVENTS * 0.9
    pl = engine.plan(b)
    assert pl.totals.vh >= 1


@pytest.mark.gpu
def test_gpu_empty_and_single_event_entries(engine_gpu):
    import oracle
    b = _empty_and_tiny()
    bad = engine.compare(b, engine_gpu.replay(b), oracle.replay(b))
    assert not bad, bad


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [2, 3])
def test_gpu_max_length_histories(engine_gpu, cfg):
    """Histories at the history count limit (C2: the fast kernel, ~34k activities; C3:
    the wave kernel) next to short ones in the same batch (ragged)."""
    import oracle
    b = engine.synth_batch(cfg, 3, seed=17 + cfg, target_len=MAX_EVENTS, max_len=MAX_EVENTS)
    small = engine.synth_batch(cfg, 200, seed=23 + cfg)
    assert max(b.wfs[w].ev_len for w in range(b.n_wfs)) >= MAX_EVENTS * 0.9
    for batch in (b, small):
        bad = engine.compare(batch, engine_gpu.replay(batch), oracle.replay(batch))
        assert not bad, "\n".join(bad[:5])


def _par_slices(batch, pl=None):
    """(lanes of each PAR slice, flags) of the batch's default slice plan (PLAN_WAVE | PLAN_PAR)."""
    import ctypes as C
    import numpy as np
    L = abi.lib()
    pl = pl or engine.plan(batch)
    mode = abi.PLAN_WAVE | abi.PLAN_PAR
    ns, rows, nw = C.c_uint32(), C.c_uint64(), C.c_uint32()
    L.cdr_plan_slices_ex(batch.wfs, pl.caps, batch.n_wfs, mode, None, None, None, None, C.byref(ns), C.byref(rows),
                         C.byref(nw))
    lane = np.zeros(max(1, ns.value) * 64, np.int32)
    flags = np.zeros(max(1, ns.value), np.uint32)
    L.cdr_plan_slices_ex(batch.wfs, pl.caps, batch.n_wfs, mode, lane.ctypes.data, None, None, flags.ctypes.data,
                         C.byref(ns), C.byref(rows), C.byref(nw))
    lanes = lane[:ns.value * 64].reshape(-1, 64)
    return [sorted(int(w) for w in lanes[s] if w >= 0) for s in range(ns.value) if flags[s] & abi.SLICE_PAR]


def test_plan_solo_par_slices_at_the_limit():
    """configs[3] load balance: every register-table history of CDR_PAR_SOLO_LEN (16,384)
    events or more gets a PAR slice of its own (k_replay_cls replays its A / T / X classes
    in wave form there), the shorter long ones share PAR slices."""
    b = engine.synth_batch(4, 40, seed=0x5EED0004, long_stride=20)
    long_ = {w for w in range(b.n_wfs) if b.wfs[w].ev_len >= 16384}
    assert len(long_) == 2 and min(b.wfs[w].ev_len for w in long_) >= MAX_EVENTS * 0.99
    par = _par_slices(b)
    assert all([w] in par for w in long_)  # each alone in a PAR slice
    assert all(len(s) == 1 for s in par[:len(long_)])  # the solo slices come first


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [4, 3])
def test_gpu_limit_histories_solo_par(engine_gpu, cfg):
    """Histories at the history count limit (204,800 events, configs[3]'s C4 shape: children,
    continue-as-new) on solo PAR slices next to short ones: the class kernel ALONE replays
    them (none handed on to k_replay_reg), and every entry equals the oracle; the default
    path (with the fallback) too."""
    import oracle
    b = engine.synth_batch(cfg, 40, seed=0x5EED0404 + cfg, long_stride=20)
    assert sum(1 for s in _par_slices(b) if len(s) == 1) >= 1
    ref = oracle.replay(b)
    old = engine_gpu.set_cls(abi.CLS_ALONE)
    try:
        got = engine_gpu.replay(b)
    finally:
        engine_gpu.set_cls(old)
    retried = [w for w in range(b.n_wfs) if got.result[w].code == abi.CLS_RETRY]
    assert not retried, retried[:10]
    bad = engine.compare(b, got, ref)
    assert not bad, "\n".join(bad[:10])
    bad = engine.compare(b, engine_gpu.replay(b), ref)
    assert not bad, "\n".join(bad[:10])
