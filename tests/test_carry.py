"""Carry-in replay (cdr_carry): applyEvents onto a LOADED mutable state, the
mutableStateBuilder.Load path (mutableStateBuilder.go:272-295) used by the NDC
replicator's apply-to-current-branch (nDCHistoryReplicator.go:330-398).

The size-independent property: cut every history at a call boundary, replay the
prefix, load its persisted records and replay the rest onto them — the result must
equal replaying the whole history in one go (same persisted state, same outcome).
The reference holds no fixture for a loaded state, so the property (checked on the
oracle here and on the GPU in the gpu-marked tests) and GPU == oracle on the same
carry-in batches are what pin this path.
"""
import pytest

from cadence_amd import abi, engine


def _assert_split_equal(batch, full, suf_batch, suf, prefix_cut):
    """suffix-on-loaded-state results == whole-history results, entry by entry (an
    entry that failed in the whole replay must fail the same way; its fail_index is
    relative to the entry's own events, so it shifts by the cut)."""
    for w in range(batch.n_wfs):
        a, b = suf.result[w], full.result[w]
        carried = suf_batch.carry.src[w] >= 0
        if b.code != abi.OK:
            assert (a.code, a.fail_event_id) == (b.code, b.fail_event_id), w
            assert a.fail_index + (prefix_cut[w] if carried else 0) == b.fail_index, w
            a.fail_index = b.fail_index  # compared above
    bad = engine.compare(batch, suf, full)
    assert not bad, "\n".join(bad[:10])


def _split_replay(replay, batch, seed):
    full = replay(batch)
    pre, cut = engine.split_batch(batch, seed)
    pre_out = replay(pre)
    suf_batch = engine.suffix_batch(batch, cut, pre, pre_out)
    n_carried = int((suf_batch.carry.src >= 0).sum())
    suf = replay(suf_batch)
    return full, suf_batch, suf, cut, n_carried


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5])
def test_oracle_split_equals_whole(cfg):
    import oracle
    b = engine.synth_batch(cfg, 150, seed=0x5EED0000 + cfg)
    full, sb, suf, cut, n = _split_replay(oracle.replay, b, seed=cfg)
    assert n > 0
    _assert_split_equal(b, full, sb, suf, cut)


@pytest.mark.parametrize("builder", [abi.BUILDER_LOCAL, abi.BUILDER_2DC, abi.BUILDER_NDC])
def test_oracle_split_builders_faults(builder):
    import oracle
    b = engine.synth_batch(0, 200, seed=31 + builder, builder=builder, error_rate=0.2)
    full, sb, suf, cut, n = _split_replay(oracle.replay, b, seed=builder)
    assert n > 0
    _assert_split_equal(b, full, sb, suf, cut)


def test_carry_plan_caps():
    """Loaded rows count toward the entry's capacities; loaded entries leave the
    fast/wave kernels (the general kernel replays onto loaded state)."""
    import oracle
    b = engine.synth_batch(3, 64, seed=5)
    pre, cut = engine.split_batch(b, 1)
    pre_out = oracle.replay(pre)
    sb = engine.suffix_batch(b, cut, pre, pre_out)
    pl0, pl = engine.plan(b), engine.plan(sb)
    for w in range(b.n_wfs):
        c = pl.caps[w]
        if sb.carry.src[w] < 0:
            continue
        r = pre_out.result[w]
        assert c.flags & (abi.CAP_FAST | abi.CAP_WAVE) == 0
        assert c.timer_live >= r.n_timer and c.act_live >= r.n_activity
        assert c.vh_cap >= r.n_vh and c.rp_cap >= r.n_reset_points and c.sa_cap >= r.n_search_attr
        assert c.child_cap >= r.n_child and c.signal_cap >= r.n_signal and c.cancel_cap >= r.n_cancel
        assert c.act_cap <= pl0.caps[w].act_cap + r.n_activity


def test_carry_rejects_failed_state():
    import ctypes as C
    import numpy as np
    import oracle
    b = engine.synth_batch(0, 100, seed=3, error_rate=0.5)
    out = oracle.replay(b)
    bad = [w for w in range(b.n_wfs) if out.result[w].code != abi.OK and b.wfs[w].parent < 0]
    assert bad
    src = np.full(b.n_wfs, -1, np.int32)
    src[bad[0]] = bad[0]
    sb = engine.Batch(events=b.events, wfs=b.wfs, kvs=b.kvs, rps=b.rps, cluster=b.cluster, now_ns=b.now_ns,
                      uuid_seed=b.uuid_seed, empty_uuid=b.empty_uuid, carry=engine.Carry(src=src, state=out))
    caps = (abi.CdrWfCaps * b.n_wfs)()
    tot = abi.CdrTotals()
    assert abi.lib().cdr_plan_caps(C.byref(sb.cstruct()), caps, C.byref(tot)) == -1  # CDR_API_EINVAL


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [0, 2, 3, 4, 5])
def test_gpu_carry_matches_oracle(engine_gpu, cfg):
    """The same carry-in batch on the GPU and on the oracle: bit-exact; and the
    split property on the GPU's own outputs."""
    import oracle
    b = engine.synth_batch(cfg, 300, seed=0x5EED0200 + cfg, error_rate=0.1 if cfg in (0, 3) else 0.0)
    pre, cut = engine.split_batch(b, cfg + 7)
    pre_gpu, pre_ref = engine_gpu.replay(pre), oracle.replay(pre)
    assert not engine.compare(pre, pre_gpu, pre_ref)
    sb = engine.suffix_batch(b, cut, pre, pre_gpu)
    assert (sb.carry.src >= 0).sum() > 0
    got, ref = engine_gpu.replay(sb), oracle.replay(sb)
    bad = engine.compare(sb, got, ref)
    assert not bad, "\n".join(bad[:10])
    _assert_split_equal(b, engine_gpu.replay(b), sb, got, cut)


@pytest.mark.gpu
@pytest.mark.parametrize("builder", [abi.BUILDER_LOCAL, abi.BUILDER_2DC, abi.BUILDER_NDC])
def test_gpu_carry_builders(engine_gpu, builder):
    import oracle
    b = engine.synth_batch(0, 300, seed=41 + builder, builder=builder, error_rate=0.2)
    pre, cut = engine.split_batch(b, builder + 3)
    pre_gpu = engine_gpu.replay(pre)
    sb = engine.suffix_batch(b, cut, pre, pre_gpu)
    got, ref = engine_gpu.replay(sb), oracle.replay(sb)
    bad = engine.compare(sb, got, ref)
    assert not bad, "\n".join(bad[:10])
