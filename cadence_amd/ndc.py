"""NDC replication with forked histories: branch management, conflict-resolution
rebuild and apply, over batches of workflows.

The flow restates nDCHistoryReplicator.applyNonStartEvents
(service/history/nDCHistoryReplicator.go:246-470) for one replication task per
workflow at a time:

1. ``branch``: nDCBranchMgr.prepareVersionHistory + nDCConflictResolver.prepareMutableState
   (ndc.hip ``k_ndc_branch``) decide per workflow: skip, apply to the current branch,
   rebuild the task's branch first, or backfill a non-current branch (VH only).
2. ``REBUILD`` workflows: nDCStateRebuilder.rebuild replays the branch's events 1..lastItem
   (the replay kernels, NDC builder, expected next event ID) and
   nDCConflictResolver.rebuild verifies the rebuilt VersionHistory and switches the
   current branch (``k_ndc_rebuild_verify``).
3. applyNonStartEventsToCurrentBranch: the task's events replay onto the current (or
   rebuilt) state (carry-in replay), and the replay's VersionHistory becomes the current
   branch's (``k_vhs_sync``).

The compute steps go through a backend (``GpuBackend`` here: the HIP kernels behind the
C ABI); this module is the host control flow between them.  After the rebuild the
reference keeps the rebuilt builder in memory; here the apply step reloads it (carry-in,
``mutableStateBuilder.Load`` semantics: currentVersion = EmptyVersion until the first
event of a running workflow sets it) — identical unless a closed workflow receives a
decision-failure event.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi, engine

ITEMS_CAP = 64  # version-history item slots per branch


def new_vhs(n: int, items_cap: int = ITEMS_CAP):
    """Empty VersionHistories for n workflows (items pool: MAX_BRANCHES x items_cap each)."""
    vhs = (abi.CdrVHS * max(1, n))()
    for w in range(n):
        vhs[w].items_cap = items_cap
        vhs[w].items_off = w * items_cap * abi.VHS_MAX_BRANCHES
    pool = (abi.CdrVHItem * max(1, n * items_cap * abi.VHS_MAX_BRANCHES))()
    return vhs, pool


def branch_items(vhs, pool, w: int, b: int):
    s = vhs[w]
    off = s.items_off + b * s.items_cap
    return [(pool[off + i].event_id, pool[off + i].version) for i in range(s.branch[b].n_items)]


TABLE_CAP = {"act": "act_cap", "timer": "timer_cap", "child": "child_cap", "cancel": "cancel_cap",
             "signal": "signal_cap", "vh": "vh_cap", "rp": "rp_cap", "sa": "sa_cap"}
TABLE_OFF = {t: c.replace("_cap", "_off") for t, c in TABLE_CAP.items()}


def gather_outputs(sources):
    """One Outputs holding, for entry w, the persisted state sources[w] = (Outputs, index)
    (None: an empty entry), with its own compact Plan — the loaded states of a carry-in."""
    n = len(sources)
    caps = (abi.CdrWfCaps * max(1, n))()
    tot = abi.CdrTotals()
    for w, src in enumerate(sources):
        if src is None:
            continue
        o, j = src
        r = o.result[j]
        for t, cname in TABLE_CAP.items():
            cnt = getattr(r, engine.TABLE_COUNT[t]) if r.code == abi.OK else 0
            setattr(caps[w], TABLE_OFF[t], getattr(tot, t))
            setattr(caps[w], cname, cnt)
            setattr(tot, t, getattr(tot, t) + cnt)
    pl = engine.Plan(caps=caps, totals=tot)

    class _B:  # the Outputs constructor only needs n_wfs
        pass
    b = _B()
    b.n_wfs = n
    out = engine.Outputs(b, pl)
    for w, src in enumerate(sources):
        if src is None:
            out.result[w].code = abi.E_HISTORY_EMPTY
            continue
        o, j = src
        C.memmove(C.byref(out.result[w]), C.byref(o.result[j]), C.sizeof(abi.CdrWfResult))
        C.memmove(C.byref(out.exec[w]), C.byref(o.exec[j]), C.sizeof(abi.CdrExecInfo))
        C.memmove(C.byref(out.repl[w]), C.byref(o.repl[j]), C.sizeof(abi.CdrReplState))
        if o.result[j].code != abi.OK:
            continue
        for t in engine.TABLES:
            cnt = getattr(caps[w], TABLE_CAP[t])
            if cnt:
                sz = C.sizeof(engine.TABLE_TYPES[t])
                src_off = getattr(o.plan.caps[j], TABLE_OFF[t])
                C.memmove(C.addressof(out.tables[t]) + getattr(caps[w], TABLE_OFF[t]) * sz,
                          C.addressof(o.tables[t]) + src_off * sz, cnt * sz)
    return out


def _masked(batch: engine.Batch, keep) -> engine.Batch:
    """The batch with the events of entries not in `keep` removed (ev_len 0)."""
    wfs = (abi.CdrWfDesc * batch.n_wfs)()
    C.memmove(wfs, batch.wfs, C.sizeof(wfs))
    for w in range(batch.n_wfs):
        if not keep[w]:
            wfs[w].ev_len = 0
    return engine._entry_batch(batch, wfs)


class GpuBackend:
    """The HIP path: replays through cdr_replay_batch, branch bookkeeping through the
    ndc.hip kernels (device buffers via the HIP runtime)."""

    def __init__(self, eng: engine.Engine):
        self.eng = eng

    def replay(self, batch: engine.Batch) -> engine.Outputs:
        return self.eng.replay(batch)

    def _run(self, fn, inputs, outputs):
        """Upload ctypes arrays, call fn(device pointers...), download `outputs`."""
        hip = engine._hip()
        ptrs = {}
        try:
            for k, a in {**inputs, **outputs}.items():
                p = C.c_void_p()
                nb = max(8, C.sizeof(a))
                if hip.hipMalloc(C.byref(p), C.c_size_t(nb)) != 0:
                    raise RuntimeError("hipMalloc failed")
                ptrs[k] = p
                if hip.hipMemcpy(p, C.addressof(a), C.c_size_t(C.sizeof(a)), 1) != 0:
                    raise RuntimeError("hipMemcpy H2D failed")
            rc = fn(ptrs)
            if rc:
                raise RuntimeError(f"ndc kernel rc={rc}")
            for k, a in outputs.items():  # hipMemcpy D2H synchronises the default stream
                if hip.hipMemcpy(C.addressof(a), ptrs[k], C.c_size_t(C.sizeof(a)), 2) != 0:
                    raise RuntimeError("hipMemcpy D2H failed")
        finally:
            for p in ptrs.values():
                hip.hipFree(p)

    def branch(self, tasks, items, vhs, pool, n):
        dec = (abi.CdrNdcDecision * max(1, n))()
        L = abi.lib()
        self._run(lambda p: L.cdr_ndc_branch_async(self.eng.ctx, p["tasks"], p["items"], n, p["vhs"], p["pool"],
                                                   p["dec"], None),
                  {"tasks": tasks, "items": items}, {"vhs": vhs, "pool": pool, "dec": dec})
        return dec

    def _out_dev(self, p, out: engine.Outputs):
        o = abi.CdrOut()
        o.result, o.exec, o.vh = p["result"], p["exec"], p["vh"]
        return o

    def rebuild_verify(self, dec, vhs, pool, out: engine.Outputs, n):
        L = abi.lib()

        def fn(p):
            o = self._out_dev(p, out)
            return L.cdr_ndc_rebuild_verify_async(self.eng.ctx, n, p["dec"], p["vhs"], p["pool"], p["caps"],
                                                  C.byref(o), None)
        self._run(fn, {"dec": dec, "pool": pool, "caps": out.plan.caps, "vh": out.tables["vh"]},
                  {"vhs": vhs, "result": out.result, "exec": out.exec})

    def vhs_sync(self, vhs, pool, out: engine.Outputs, n):
        L = abi.lib()

        def fn(p):
            o = self._out_dev(p, out)
            return L.cdr_vhs_sync_async(self.eng.ctx, n, p["vhs"], p["pool"], p["caps"], C.byref(o), None)
        self._run(fn, {"caps": out.plan.caps, "result": out.result, "exec": out.exec, "vh": out.tables["vh"]},
                  {"vhs": vhs, "pool": pool})


def replicate(be, base: engine.Batch, rebuild: engine.Batch, forks, items_cap: int = ITEMS_CAP):
    """Replicate every workflow's base branch from scratch, then each fork task in turn
    (forks = [(events batch, tasks, task items), ...], one task per workflow, entry order
    of `base`).  Returns (final state Outputs, vhs, pool, [decisions per fork],
    {"replayed_events": n})."""
    n = base.n_wfs
    out = be.replay(base)
    events = int(sum(base.wfs[w].ev_len for w in range(n)))
    state = [(out, w) for w in range(n)]
    vhs, pool = new_vhs(n, items_cap)
    be.vhs_sync(vhs, pool, out, n)
    decisions = []
    for fork_batch, tasks, items in forks:
        dec = be.branch(tasks, items, vhs, pool, n)
        decisions.append(dec)
        act = [dec[w].action if dec[w].code == abi.OK and state[w][0].result[state[w][1]].code == abi.OK else -1
               for w in range(n)]
        rb = None
        if any(a == abi.NDC_REBUILD for a in act):
            keep = [a == abi.NDC_REBUILD for a in act]
            rb = be.replay(_masked(rebuild, keep))
            events += int(sum(rebuild.wfs[w].ev_len for w in range(n) if keep[w]))
            be.rebuild_verify(dec, vhs, pool, rb, n)
        src, apply = [], []
        for w in range(n):
            if act[w] == abi.NDC_REBUILD:
                src.append((rb, w))
                apply.append(True)
            elif act[w] == abi.NDC_APPLY_CURRENT:
                src.append(state[w])
                apply.append(True)
            else:
                src.append(None)
                apply.append(False)
        if not any(apply):
            continue
        loaded = gather_outputs(src)
        ab = _masked(fork_batch, apply)
        ab.carry = engine.Carry(src=np.array([w if apply[w] else -1 for w in range(n)], np.int32), state=loaded)
        ap = be.replay(ab)
        events += int(sum(fork_batch.wfs[w].ev_len for w in range(n) if apply[w]))
        be.vhs_sync(vhs, pool, ap, n)
        for w in range(n):
            if apply[w]:
                state[w] = (ap, w)
            elif dec[w].code != abi.OK:
                state[w] = (_failed(dec[w].code), 0)
    final = gather_outputs(state)
    return final, vhs, pool, decisions, {"replayed_events": events}


_FAILED = {}


def _failed(code: int):
    """A one-entry Outputs carrying only a failed result (a task that errored)."""
    if code not in _FAILED:
        class _B:
            n_wfs = 1
        caps = (abi.CdrWfCaps * 1)()
        o = engine.Outputs(_B(), engine.Plan(caps=caps, totals=abi.CdrTotals()))
        o.result[0].code = code
        _FAILED[code] = o
    return _FAILED[code]


def synth_forked(config: int, n_wfs: int, seed: int, items_cap: int = ITEMS_CAP, **kw):
    """The parts of a synthetic forked population (config 5): (base, rebuild path,
    [(fork A batch, tasks, items), (fork B batch, tasks, items)])."""
    L = abi.lib()
    base = engine.synth_batch(config, n_wfs, seed, part=abi.SYNTH_PART_BASE, **kw)
    rebuild = engine.synth_batch(config, n_wfs, seed, part=abi.SYNTH_PART_REBUILD, **kw)
    forks = []
    for k, part in enumerate((abi.SYNTH_PART_FORK_A, abi.SYNTH_PART_FORK_B)):
        fb = engine.synth_batch(config, n_wfs, seed, part=part, **kw)
        p = abi.CdrSynthParams(config=config, n_wfs=n_wfs, seed=seed, builder=-1)
        for key in ("target_len", "max_len", "error_rate", "builder", "fault_kinds"):
            if key in kw:
                setattr(p, key, kw[key])
        im = kw.get("index_map")
        if im is not None:
            im = np.ascontiguousarray(im, dtype=np.uint32)
            p.index_map = im.ctypes.data
        tasks = (abi.CdrNdcTask * max(1, n_wfs))()
        items = (abi.CdrVHItem * max(1, n_wfs * items_cap))()
        rc = L.cdr_synth_ndc_tasks(C.byref(p), k, tasks, items, items_cap)
        if rc:
            raise RuntimeError(f"cdr_synth_ndc_tasks rc={rc}")
        forks.append((fb, tasks, items))
    return base, rebuild, forks
