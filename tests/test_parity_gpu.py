"""GPU parity: the HIP replay engine vs the CPU restatement (oracle/), field by field.

Inputs are the deterministic synthetic configs of SURVEY §8(d) (small sizes the
oracle finishes in seconds), with and without injected faults so that every error
and panic site is exercised.  Bar: bit-exact (integer/handle state; the only float,
BackoffCoefficient, is a verbatim copy).
"""
import pytest

from cadence_amd import abi, engine

pytestmark = pytest.mark.gpu


def _check(batch, eng):
    import oracle
    ref = oracle.replay(batch)
    got = eng.replay(batch)
    bad = engine.compare(batch, got, ref)
    assert not bad, "\n".join(bad[:10])
    return ref


@pytest.mark.parametrize("cfg", [1, 2, 3, 4, 5, 0])
def test_synth_configs_clean(engine_gpu, cfg):
    b = engine.synth_batch(cfg, 300, seed=0x5EED0000 + cfg)
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
