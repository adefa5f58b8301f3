"""TEST INFRASTRUCTURE ONLY: Python binding of the CPU restatement (replay_ref.cpp).

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
parity checker / CPU baseline.  The product (cadence_amd/) never imports this.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libcdr_oracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        from cadence_amd import abi
        L = C.CDLL(LIB)
        L.cdro_replay_batch.restype = C.c_int
        L.cdro_replay_batch.argtypes = [C.POINTER(abi.CdrBatch), C.POINTER(abi.CdrWfCaps), C.POINTER(abi.CdrOut),
                                        C.c_int]
        L.cdro_refresh_tasks.restype = C.c_int
        L.cdro_refresh_tasks.argtypes = [C.POINTER(abi.CdrBatch), C.POINTER(abi.CdrWfCaps), C.POINTER(abi.CdrOut),
                                         C.c_int64, C.c_uint32]
        L.cdro_vh_add_or_update.restype = C.c_int
        L.cdro_vh_add_or_update.argtypes = [C.POINTER(abi.CdrVHItem), C.POINTER(C.c_uint32), C.c_uint32,
                                            C.c_int64, C.c_int64]
        L.cdro_state_transition.restype = C.c_int
        L.cdro_state_transition.argtypes = [C.c_int] * 4
        P = C.POINTER
        VH = abi.CdrVHItem
        for name, args in (
                ("cdro_vh_duplicate_until_lca", [P(VH), C.c_uint32, VH, P(VH), P(C.c_uint32)]),
                ("cdro_vh_contains", [P(VH), C.c_uint32, VH]),
                ("cdro_vh_is_lca_appendable", [P(VH), C.c_uint32, VH]),
                ("cdro_vh_find_lca", [P(VH), C.c_uint32, P(VH), C.c_uint32, P(VH)]),
                ("cdro_vhs_add", [P(abi.CdrVHS), P(VH), P(abi.CdrVHToken), P(VH), C.c_uint32, P(C.c_int),
                                  P(C.c_uint32)]),
                ("cdro_vhs_find_lca_index", [P(abi.CdrVHS), P(VH), P(VH), C.c_uint32, P(C.c_uint32), P(VH)]),
                ("cdro_vhs_find_first_index_by_item", [P(abi.CdrVHS), P(VH), VH, P(C.c_uint32)]),
                ("cdro_vhs_is_rebuilt", [P(abi.CdrVHS), P(VH)]),
                ("cdro_ndc_branch", [P(abi.CdrNdcTask), P(VH), C.c_uint32, P(abi.CdrVHS), P(VH),
                                     P(abi.CdrNdcDecision)]),
                ("cdro_ndc_rebuild_verify", [C.c_uint32, P(abi.CdrNdcDecision), P(abi.CdrVHS), P(VH),
                                             P(abi.CdrWfCaps), P(abi.CdrOut)]),
                ("cdro_vhs_sync", [C.c_uint32, P(abi.CdrVHS), P(VH), P(abi.CdrWfCaps), P(abi.CdrOut)])):
            fn = getattr(L, name)
            fn.restype = C.c_int
            fn.argtypes = args
        L.cdro_entry_digests.restype = C.c_int
        L.cdro_entry_digests.argtypes = [C.POINTER(abi.CdrBatch), C.POINTER(abi.CdrWfCaps), C.POINTER(abi.CdrOut),
                                         C.c_void_p, C.POINTER(C.c_uint64), C.c_int]
        _lib = L
    return _lib


def replay(batch, pl=None, threads: int = 1, tasks: bool = False):
    """Oracle replay of a cadence_amd.engine.Batch into host Outputs (`tasks`: also
    the transfer / timer task lists)."""
    from cadence_amd import engine
    pl = pl or engine.plan(batch)
    out = engine.Outputs(batch, pl, tasks)
    rc = lib().cdro_replay_batch(C.byref(batch.cstruct()), pl.caps, C.byref(out.cstruct()), threads)
    if rc:
        raise RuntimeError(f"cdro_replay_batch rc={rc}")
    return out


def rebuild(batch, pl=None, advanced_visibility: bool = True, snapshot: bool = False):
    """Oracle of nDCStateRebuilder's replay + refreshTasks (refresh_ref.cpp): the
    rebuilt state with the refresher's task lists (now = batch.now_ns)."""
    from cadence_amd import abi, engine
    pl = pl or engine.plan(batch)
    out = replay(batch, pl)
    out.alloc_tasks(pl)
    flags = (abi.REFRESH_ADVANCED_VISIBILITY if advanced_visibility else 0) | (
        abi.REFRESH_SNAPSHOT_PASSIVE if snapshot else 0)
    bs = batch.cstruct()
    rc = lib().cdro_refresh_tasks(C.byref(bs), pl.caps, C.byref(out.cstruct()), bs.now_ns, flags)
    if rc:
        raise RuntimeError(f"cdro_refresh_tasks rc={rc}")
    return out


def entry_digests(batch, pl, out, threads: int = 1):
    """(per-entry digests uint64[n_wfs], wrapping sum) of oracle outputs — the restated
    k_digest hash (digest_ref.cpp)."""
    import numpy as np
    per = np.zeros(max(1, batch.n_wfs), np.uint64)
    tot = C.c_uint64()
    rc = lib().cdro_entry_digests(C.byref(batch.cstruct()), pl.caps, C.byref(out.cstruct()), per.ctypes.data,
                                  C.byref(tot), threads)
    if rc:
        raise RuntimeError(f"cdro_entry_digests rc={rc}")
    return per[:batch.n_wfs], tot.value


def synth_digests(config: int, index_map, seed: int, threads: int = 16, chunk: int = 65536, **kw):
    """Oracle digests of a synthetic population at full size: the workflows of
    `index_map` (global indices, in order) generated in natural order chunk by chunk,
    replayed by the restatement on `threads` host threads and hashed entry by entry.
    Returns (per-entry digests in cadence_amd.synth.DeviceBatch's entry order, sum,
    {status name: count})."""
    import numpy as np
    from cadence_amd import abi, engine
    index_map = np.ascontiguousarray(index_map, dtype=np.uint32)
    parts, total, hist = [], 0, {}
    bufs = engine.SynthBuffers()
    for i in range(0, len(index_map), chunk):
        im = index_map[i:i + chunk]
        b = engine.synth_batch(config, len(im), seed, index_map=im, buffers=bufs, **kw)
        pl = engine.plan(b)
        out = replay(b, pl, threads=threads)
        per, s = entry_digests(b, pl, out, threads)
        parts.append(per)
        total = (total + s) & 0xFFFFFFFFFFFFFFFF
        codes = np.frombuffer(out.result, dtype=np.int32).reshape(-1, C.sizeof(abi.CdrWfResult) // 4)[:b.n_wfs, 0]
        for v, c in zip(*np.unique(codes, return_counts=True)):
            k = abi.STATUS.get(int(v), str(int(v)))
            hist[k] = hist.get(k, 0) + int(c)
        del b, pl, out
    return (np.concatenate(parts) if parts else np.zeros(0, np.uint64)), total, hist


class NdcBackend:
    """ndc_ref.cpp's branch bookkeeping alone (the branch-kernel parity test)."""

    def branch(self, tasks, items, vhs, pool, n):
        from cadence_amd import abi
        dec = (abi.CdrNdcDecision * max(1, n))()
        lib().cdro_ndc_branch(tasks, items, n, vhs, pool, dec)
        return dec


def ndc_replicate(base, rebuild, forks, items_cap=None, refresh_flags: int = 1, threads: int = 1):
    """The NDC replication run restated on the CPU (replay_ref.cpp cdro_ndc_replicate_round:
    per workflow, the rebuilt MutableState kept in memory between nDCStateRebuilder.rebuild
    and applyEvents, nDCConflictResolver.go:117-184, nDCHistoryReplicator.go:330-398): the
    base branch replayed into the state buffer, then each fork round.  Returns what
    cadence_amd.ndc.DeviceReplicator.run returns: (state Outputs, vhs, pool, [decisions],
    [(rebuild Outputs, apply Outputs) per round])."""
    from cadence_amd import abi, engine, ndc
    L = lib()
    if not hasattr(L, "_ndc_round_bound"):
        P = C.POINTER
        L.cdro_ndc_replicate_round.restype = C.c_int
        L.cdro_ndc_replicate_round.argtypes = [
            C.c_uint32, P(abi.CdrNdcTask), P(abi.CdrVHItem), P(abi.CdrBatch), P(abi.CdrWfCaps), P(abi.CdrOut),
            P(abi.CdrBatch), P(abi.CdrWfCaps), P(abi.CdrOut), P(abi.CdrVHS), P(abi.CdrVHItem), P(abi.CdrNdcDecision),
            P(abi.CdrWfCaps), P(abi.CdrOut), C.c_int64, C.c_uint32, C.c_int]
        L._ndc_round_bound = True
    n = base.n_wfs
    sp = ndc.state_caps_for(base, rebuild, forks)
    state = engine.Outputs(base, sp)
    rc = L.cdro_replay_batch(C.byref(base.cstruct()), sp.caps, C.byref(state.cstruct()), threads)
    if rc:
        raise RuntimeError(f"cdro_replay_batch rc={rc}")
    vhs, pool = ndc.new_vhs(n, ndc.items_cap_for(base, rebuild, forks) if items_cap is None else items_cap)
    L.cdro_vhs_sync(n, vhs, pool, sp.caps, C.byref(state.cstruct()))
    rp = engine.plan(rebuild)
    decs, per_round = [], []
    for fb, tasks, items in forks:
        caps = (abi.CdrWfCaps * max(1, n))()
        tot = abi.CdrTotals()
        rc = abi.lib().cdr_plan_ndc_apply(C.byref(fb.cstruct()), sp.caps, caps, C.byref(tot))
        if rc:
            raise RuntimeError(f"cdr_plan_ndc_apply rc={rc}")
        ap = engine.Plan(caps=caps, totals=tot)
        rb_out = engine.Outputs(rebuild, rp, tasks=True)
        ap_out = engine.Outputs(fb, ap)
        dec = (abi.CdrNdcDecision * max(1, n))()
        rc = L.cdro_ndc_replicate_round(n, tasks, items, C.byref(rebuild.cstruct()), rp.caps,
                                        C.byref(rb_out.cstruct()), C.byref(fb.cstruct()), ap.caps,
                                        C.byref(ap_out.cstruct()), vhs, pool, dec, sp.caps,
                                        C.byref(state.cstruct()), rebuild.now_ns, refresh_flags, threads)
        if rc:
            raise RuntimeError(f"cdro_ndc_replicate_round rc={rc}")
        decs.append(dec)
        per_round.append((rb_out, ap_out))
    return state, vhs, pool, decs, per_round
