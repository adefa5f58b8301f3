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
