"""The host-buffer boundary (cdr_create with cdr_opts, cdr_replay_batch on a stream with
the context's grow-only workspace, error returns) on the GPU."""
import ctypes as C

import pytest

import oracle
from cadence_amd import abi, engine

pytestmark = pytest.mark.gpu


def test_create_with_opts_and_reserved_workspace():
    L = abi.lib()
    o = abi.CdrOpts()
    L.cdr_opts_default(C.byref(o))
    assert (o.plan_mode, o.fast_path, o.reg_path, o.concurrent) == (abi.PLAN_WAVE | abi.PLAN_PAR, 1, 1, 1)
    o.fast_path, o.concurrent, o.workspace_bytes = 0, 0, 64 << 20
    ctx = L.cdr_create(0, C.byref(o))
    assert ctx
    try:
        assert L.cdr_set_fast_path(ctx, 1) == 0  # the option took effect
        bad = abi.CdrOpts()
        L.cdr_opts_default(C.byref(bad))
        bad.plan_mode = 0x80
        assert not L.cdr_create(0, C.byref(bad))
        assert not L.cdr_create(64, None)  # no such device
    finally:
        L.cdr_destroy(ctx)


def test_replay_on_a_stream_reuses_the_workspace(engine_gpu):
    """Two calls on a caller-created stream (the HIP runtime libcdr uses, through
    ctypes); the second, smaller batch needs no new device memory (the workspace only
    grows) and both match the oracle."""
    hip = engine._hip()
    st = C.c_void_p()
    assert hip.hipStreamCreate(C.byref(st)) == 0
    L = abi.lib()

    def free_bytes():
        f, t = C.c_size_t(), C.c_size_t()
        assert hip.hipMemGetInfo(C.byref(f), C.byref(t)) == 0
        return f.value
    try:
        for n in (300, 120):
            b = engine.synth_batch(4, n, seed=n)
            pl = engine.plan(b)
            out = engine.Outputs(b, pl)
            free0 = free_bytes()
            rc = L.cdr_replay_batch(engine_gpu.ctx, C.byref(b.cstruct()), pl.caps, C.byref(pl.totals),
                                    C.byref(out.cstruct()), st)
            assert rc == 0
            if n == 120:
                assert free_bytes() >= free0 - (2 << 20)
            assert not engine.compare(b, out, oracle.replay(b))
    finally:
        hip.hipStreamDestroy(st)


def test_oversized_totals_return_enomem_and_the_context_survives(engine_gpu):
    """An allocation the device cannot satisfy is reported as CDR_API_ENOMEM before any
    launch (no kernel sees a null buffer), and the same context replays afterwards."""
    b = engine.synth_batch(3, 64, seed=5)
    pl = engine.plan(b)
    out = engine.Outputs(b, pl)
    huge = abi.CdrTotals()
    C.memmove(C.byref(huge), C.byref(pl.totals), C.sizeof(huge))
    huge.act = 1 << 44  # 2 PiB of activity rows
    rc = abi.lib().cdr_replay_batch(engine_gpu.ctx, C.byref(b.cstruct()), pl.caps, C.byref(huge),
                                    C.byref(out.cstruct()), None)
    assert rc == -4  # CDR_API_ENOMEM
    got = engine_gpu.replay(b)
    assert not engine.compare(b, got, oracle.replay(b))
