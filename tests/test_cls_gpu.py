"""Class-decomposed register-table replay (k_replay_cls, replay_cls.inc) vs the oracle.

k_replay_cls replays each register-table slice from its class-sorted block and hands
every entry it does not replay itself (errors, panics, a second Started, ...) to
k_replay_reg.  The default path (both kernels) is covered by every parity test; here
the class kernel runs ALONE (cdr_set_cls_path mode 2: entries it hands on keep the
internal code CLS_RETRY), so that an entry it did replay cannot hide behind the
fallback: every entry it did not hand on must equal the oracle field by field, and on
clean batches it must hand on none.
"""
import re

import pytest

from cadence_amd import abi, engine

pytestmark = pytest.mark.gpu


def _cls_alone(eng, batch):
    old = eng.set_cls(2)
    try:
        return eng.replay(batch)
    finally:
        eng.set_cls(old)


def _split(batch, got, ref):
    retried = {w for w in range(batch.n_wfs) if got.result[w].code == abi.CLS_RETRY}
    # a handed-on entry's continue-as-new run is left CDR_NOT_APPLIED by k_finalize
    retried |= {w for w in range(batch.n_wfs) if batch.wfs[w].parent in retried}
    bad = engine.compare(batch, got, ref, limit=10 ** 9)
    wrong = [b for b in bad if int(re.match(r"wf (\d+):", b).group(1)) not in retried]
    return retried, wrong


@pytest.mark.parametrize("cfg", [3, 4, 5, 0])
def test_cls_alone_clean(engine_gpu, cfg):
    import oracle
    b = engine.synth_batch(cfg, 1500, seed=0x5EED0200 + cfg)
    ref = oracle.replay(b)
    got = _cls_alone(engine_gpu, b)
    retried, wrong = _split(b, got, ref)
    assert not wrong, "\n".join(wrong[:10])
    assert not retried, sorted(retried)[:10]  # clean: nothing handed on


@pytest.mark.parametrize("cfg", [0, 3, 4, 5])
@pytest.mark.parametrize("seed", [1, 2])
def test_cls_alone_faults(engine_gpu, cfg, seed):
    """Injected faults: the class kernel hands the failing entries on; the rest match."""
    import oracle
    b = engine.synth_batch(cfg, 800, seed=seed * 7000 + cfg, error_rate=0.3)
    ref = oracle.replay(b)
    got = _cls_alone(engine_gpu, b)
    retried, wrong = _split(b, got, ref)
    assert not wrong, "\n".join(wrong[:10])
    if cfg in (3, 4, 5):  # the class kernel ran (and handed its failing entries on)
        assert retried, "no entry handed on: k_replay_cls did not run"
    # and with k_replay_reg behind it, everything matches
    bad = engine.compare(b, engine_gpu.replay(b), ref)
    assert not bad, "\n".join(bad[:10])


@pytest.mark.parametrize("cfg", [3, 4, 5])
def test_cls_on_off_equal(engine_gpu, cfg):
    """The same batch with the class kernel on and off: identical outputs."""
    b = engine.synth_batch(cfg, 1000, seed=0x5EED0300 + cfg, error_rate=0.05)
    on = engine_gpu.replay(b)
    old = engine_gpu.set_cls(False)
    try:
        off = engine_gpu.replay(b)
    finally:
        engine_gpu.set_cls(old)
    bad = engine.compare(b, on, off)
    assert not bad, "\n".join(bad[:10])


def test_cls_long_and_2dc(engine_gpu):
    """Register-table entries with long histories (NO_LONG keeps them in lane slices) and
    every builder."""
    import oracle
    for builder in (abi.BUILDER_LOCAL, abi.BUILDER_2DC, abi.BUILDER_NDC):
        b = engine.synth_batch(3, 300, seed=4242 + builder, builder=builder, target_len=900)
        ref = oracle.replay(b)
        old = engine_gpu.set_plan_mode(abi.PLAN_WAVE | abi.PLAN_NO_LONG)
        try:
            got = _cls_alone(engine_gpu, b)
        finally:
            engine_gpu.set_plan_mode(old)
        retried, wrong = _split(b, got, ref)
        assert not wrong, f"builder {builder}: " + "\n".join(wrong[:10])
        assert not retried - {w for w in range(b.n_wfs) if ref.result[w].code != abi.OK}


def _n_par(batch, mode):
    import ctypes as C
    import numpy as np
    pl = engine.plan(batch)
    L = abi.lib()
    ns, rows, nw = C.c_uint32(), C.c_uint64(), C.c_uint32()
    L.cdr_plan_slices_ex(batch.wfs, pl.caps, batch.n_wfs, mode, None, None, None, None, C.byref(ns), C.byref(rows),
                         C.byref(nw))
    lane = np.zeros(ns.value * 64, np.int32)
    flags = np.zeros(ns.value, np.uint32)
    L.cdr_plan_slices_ex(batch.wfs, pl.caps, batch.n_wfs, mode, lane.ctypes.data, None, None, flags.ctypes.data,
                         C.byref(ns), C.byref(rows), C.byref(nw))
    return int(((flags & abi.SLICE_PAR) != 0).sum())


@pytest.mark.parametrize("cfg", [3, 4, 5])
@pytest.mark.parametrize("err", [0.0, 0.2])
def test_par_long_histories(engine_gpu, cfg, err):
    """Long register-table histories in CDR_SLICE_PAR slices: the class kernel's four-wave
    variant (its loops at once, the X wave waiting on the W wave's progress) alone, then
    with k_replay_reg behind it, against the oracle."""
    import oracle
    b = engine.synth_batch(cfg, 160, seed=0x5EED0400 + cfg + int(err * 10), target_len=1500, max_len=6000,
                           error_rate=err)
    mode = abi.PLAN_WAVE | abi.PLAN_PAR
    assert _n_par(b, mode) > 0
    ref = oracle.replay(b)
    old = engine_gpu.set_plan_mode(mode)
    try:
        got = _cls_alone(engine_gpu, b)
        retried, wrong = _split(b, got, ref)
        assert not wrong, "\n".join(wrong[:10])
        if err == 0.0:
            assert not retried, sorted(retried)[:10]
        full = engine_gpu.replay(b)
        bad = engine.compare(b, full, ref)
        assert not bad, "\n".join(bad[:10])
        oldc = engine_gpu.set_cls(False)  # PAR slices on k_replay_reg <12, 10, 4>
        try:
            bad = engine.compare(b, engine_gpu.replay(b), ref)
        finally:
            engine_gpu.set_cls(oldc)
        assert not bad, "\n".join(bad[:10])
    finally:
        engine_gpu.set_plan_mode(old)


@pytest.mark.parametrize("cfg,n", [(3, 20000), (4, 30000), (5, 20000)])
def test_host_blocks_equal_device_blocks(engine_gpu, cfg, n):
    """The host packer's class-sorted blocks (cdr_pack_cls) are the device build's
    (k_cls_count / k_cls_fill) byte for byte — padding elements' type_flags included, their
    other columns (unwritten by the device build) aside — and both replay to the same
    outputs."""
    import numpy as np
    import torch
    from cadence_amd.synth import DeviceBatch
    idx = np.arange(n, dtype=np.uint32)
    seed = 0x5EED0000 + cfg
    h = DeviceBatch(torch, cfg, idx, seed, cls="host")
    d = DeviceBatch(torch, cfg, idx, seed, ctx_for_cls=engine_gpu.ctx, cls="device")
    assert h.cls_rows == d.cls_rows > 0
    ns = h.info.n_slices
    for a, b in zip(h.cls_dev[:2], d.cls_dev[:2]):
        assert torch.equal(a[:b.numel()].cpu() if a.numel() >= b.numel() else a.cpu(), b[:a.numel()].cpu())
    hb = abi.slab_columns(h.cls_dev[2][:h.cls_rows * abi.ROW_BYTES].cpu().numpy())
    db_ = abi.slab_columns(d.cls_dev[2][:d.cls_rows * abi.ROW_BYTES].cpu().numpy())
    pad = (hb["type_flags"] & 0xFF) == 0xFF
    assert (hb["type_flags"] == db_["type_flags"]).all()
    for col in ("event_id", "version", "timestamp", "task_id", "key", "aux", "h", "n"):
        diff = np.nonzero((hb[col] != db_[col]) & ~pad)[0]
        assert len(diff) == 0, (col, diff[:5])
    stream = torch.cuda.current_stream().cuda_stream
    import ctypes as C
    for x in (h, d):
        assert abi.lib().cdr_replay_sliced_async(engine_gpu.ctx, C.byref(x.db), C.byref(x.out), C.c_void_p(stream)) == 0
    assert (h.digests(engine_gpu.ctx, stream)[0] == d.digests(engine_gpu.ctx, stream)[0]).all()
    assert ns == d.info.n_slices


def test_newrun_cluster_panic_all_kernels(engine_gpu):
    """A 2DC entry whose continue-as-new call ends on a version of no known cluster: the
    reference's ClusterNameForFailoverVersion panic fires at that call's first event
    (mutableStateBuilder.go:561-581, before the events), so the new run is never attempted —
    result code CDR_P_UNKNOWN_CLUSTER without CDR_RF_NEWRUN_APPLIED — on every kernel that
    checks the call ends lazily (register-table, general, wave) and through the class path."""
    import oracle
    b = engine.synth_batch(4, 600, seed=0x5EED0506, error_rate=0.2)
    ref = oracle.replay(b)
    case = [w for w in range(b.n_wfs) if ref.result[w].code == 35 and b.wfs[w].newrun >= 0]  # CDR_P_UNKNOWN_CLUSTER
    assert case and all(ref.result[w].flags & abi.RF_NEWRUN_APPLIED == 0 for w in case)
    L = abi.lib()
    runs = {}
    old_mode = engine_gpu.set_plan_mode(0)  # lane slices: register-table / general kernels
    try:
        runs["reg"] = engine_gpu.replay(b)
        L.cdr_set_reg_path(engine_gpu.ctx, 0)
        runs["general"] = engine_gpu.replay(b)
        L.cdr_set_reg_path(engine_gpu.ctx, 1)
        engine_gpu.set_plan_mode(abi.PLAN_WAVE | abi.PLAN_WAVE_ALL)
        runs["wave"] = engine_gpu.replay(b)
        engine_gpu.set_plan_mode(abi.PLAN_WAVE | abi.PLAN_PAR)
        old_cls = engine_gpu.set_cls(abi.CLS_BUILD)
        try:
            runs["class"] = engine_gpu.replay(b)
        finally:
            engine_gpu.set_cls(old_cls)
    finally:
        L.cdr_set_reg_path(engine_gpu.ctx, 1)
        engine_gpu.set_plan_mode(old_mode)
    for name, got in runs.items():
        bad = engine.compare(b, got, ref)
        assert not bad, f"{name}: " + "\n".join(bad[:5])
