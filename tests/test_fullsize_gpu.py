"""Full-size parity: 1M-workflow synthetic populations replayed on the GPU, compared entry
by entry with the CPU restatement (oracle/) through the restated output digest.

The north star's acceptance bar is "bit-exact mutable state on 1M-workflow synthetic
histories".  Moving 1M persisted states off the device to compare them record by record
would dominate the test, so both sides reduce each entry's persisted projection
(result code / fail event id and, for OK entries, every byte of ExecutionInfo,
ReplicationState, version history, pending rows, reset points and search attributes —
mutableStateBuilder.CopyToPersistence, service/history/mutableStateBuilder.go:257-270) to
a 64-bit digest: k_digest on the device (cdr_entry_digests_async), digest_ref.cpp on the
host.  Equal digest arrays entry by entry is the bar; a mismatch names the first entries
that differ.  Sizes default to the bench's 1M per GPU (CDR_FULLSIZE_WFS overrides), so the
12-17 GB slabs, >4 GB offsets and ~15k-slice plans of the benchmark are the ones checked.
"""
import os

import numpy as np
import pytest

from cadence_amd import abi

pytestmark = pytest.mark.gpu

N_WFS = int(os.environ.get("CDR_FULLSIZE_WFS", "1000000"))
THREADS = int(os.environ.get("CDR_CPU_THREADS", "16"))


def _gpu_digests(ctx, cfg, index_map, seed, plan_mode, reg, cls="host"):
    import torch
    from cadence_amd.synth import DeviceBatch
    import ctypes as C
    # cls: where the register-table slices' class-sorted blocks come from (k_replay_cls):
    # "host" the packer (the default), "device" k_cls_fill, None no blocks
    db = DeviceBatch(torch, cfg, index_map, seed, plan_mode=plan_mode, ctx_for_cls=ctx, cls=cls)
    stream = torch.cuda.current_stream().cuda_stream
    L = abi.lib()
    L.cdr_set_reg_path(ctx, int(reg))
    try:
        rc = L.cdr_replay_sliced_async(ctx, C.byref(db.db), C.byref(db.out), C.c_void_p(stream))
    finally:
        L.cdr_set_reg_path(ctx, 1)
    assert rc == 0, rc
    per, tot = db.digests(ctx, stream)
    kinds = {"cls_where": db.cls_where, "wave": db.n_wave, "reg": db.n_reg, "reg2": db.n_reg2, "reg0": db.n_reg0, "cls_rows": db.cls_rows,
             "par": db.n_par}
    del db
    torch.cuda.empty_cache()
    return per, tot, kinds


@pytest.mark.parametrize("cfg,plan_mode,reg", [
    (2, abi.PLAN_WAVE, True),
    (3, abi.PLAN_WAVE, True),
    (3, abi.PLAN_WAVE, "nocls"),  # register-table slices on k_replay_reg alone (no class-sorted blocks)
    (3, abi.PLAN_WAVE, "devcls"),  # class-sorted blocks built on the device (k_cls_fill)
    (3, abi.PLAN_WAVE | abi.PLAN_WAVE_ALL, True),
    (4, abi.PLAN_WAVE, True),
    (4, abi.PLAN_WAVE | abi.PLAN_PAR, True),  # the long histories on four-wave PAR slices (the default)
    (4, abi.PLAN_WAVE | abi.PLAN_NO_LONG, True),  # long histories kept in register-table lane slices
    (5, abi.PLAN_WAVE, True),
    (5, abi.PLAN_WAVE | abi.PLAN_PAR, True),
    (5, abi.PLAN_WAVE, False),  # register-table slices on the general kernel
])
def test_fullsize_entry_digests(engine_gpu, cfg, plan_mode, reg):
    import oracle
    seed = 0x5EED0000 + cfg
    index_map = np.arange(N_WFS, dtype=np.uint32)
    cls = None if reg == "nocls" else "device" if reg == "devcls" else "host"
    got, got_sum, kinds = _gpu_digests(engine_gpu.ctx, cfg, index_map, seed, plan_mode, bool(reg), cls)
    want, want_sum, hist = oracle.synth_digests(cfg, index_map, seed, threads=THREADS)
    assert len(got) == len(want)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, f"C{cfg}: {len(bad)} of {len(want)} entries differ, first {bad[:10].tolist()}"
    assert got_sum == want_sum
    assert hist.get("OK", 0) == len(want), hist  # clean populations replay OK throughout
    # the kernels that took part
    if plan_mode & abi.PLAN_WAVE_ALL:
        assert kinds["wave"] > 0
    elif cfg in (3, 4, 5):
        assert kinds["reg"] > 0, kinds
        assert (kinds["cls_rows"] > 0) == (cls is not None), kinds  # the class-sorted blocks were built (or not)
    if cfg in (4, 5) and not plan_mode & abi.PLAN_WAVE_ALL:
        assert kinds["reg2"] > 0, kinds
    if cfg in (4, 5) and plan_mode & abi.PLAN_PAR:  # the long register-table histories on PAR slices
        assert kinds["par"] > 0, kinds
    if cfg in (4, 5) and plan_mode == abi.PLAN_WAVE:  # the long-history rule (cdr.h CDR_PLAN_NO_LONG)
        assert kinds["wave"] > 0, kinds
