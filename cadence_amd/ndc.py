"""NDC replication with forked histories over batches of workflows:
branch management, conflict-resolution rebuild and apply — nDCHistoryReplicator.applyNonStartEvents
(service/history/nDCHistoryReplicator.go:246-470) for one replication task per workflow per round.

``DeviceReplicator`` drives the device-resident pipeline behind the C ABI: the base branch
replayed into a state buffer, then one ``cdr_ndc_replicate_async`` call per round, which runs
on the device, with no host round trip and no allocation:

1. nDCBranchMgr.prepareVersionHistory + nDCConflictResolver.prepareMutableState
   (``k_ndc_branch``): skip, apply to the current branch, rebuild the task's branch first,
   or backfill a non-current branch (VH only);
2. ``REBUILD`` workflows: nDCStateRebuilder.rebuild (nDCStateRebuilder.go:92-160) replays the
   branch's events 1..lastItem (the replay kernels, the other workflows masked), then
   refreshTasks, then nDCConflictResolver.rebuild verifies the rebuilt VersionHistory and
   switches the current branch (nDCConflictResolver.go:117-184);
3. applyNonStartEventsToCurrentBranch (:330-398): the task's events replay onto the rebuilt
   state as the resolver hands it over — in memory, no Load (cdr_carry.in_memory) — or onto
   the loaded current state; the replay's VersionHistory becomes the current branch's.

This module is plumbing: planning, packing and device buffers (the HIP runtime the engine's
context uses).  The CPU restatement is ``oracle.ndc_replicate`` (replay_ref.cpp
cdro_ndc_replicate_round), which keeps each rebuilt MutableState itself in memory.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi, engine

ITEMS_CAP = 64  # version-history item slots per branch


def new_vhs(n: int, items_cap=ITEMS_CAP):
    """Empty VersionHistories for n workflows; items pool: MAX_BRANCHES x items_cap[w] slots
    for workflow w (items_cap: one capacity for all, or one per workflow)."""
    caps = np.broadcast_to(np.asarray(items_cap, dtype=np.int64), (n,)).astype(np.int64)
    offs = np.zeros(n + 1, np.int64)
    np.cumsum(caps * abi.VHS_MAX_BRANCHES, out=offs[1:])
    vhs = (abi.CdrVHS * max(1, n))()
    raw = np.frombuffer(vhs, dtype=np.uint8).reshape(max(1, n), C.sizeof(abi.CdrVHS))[:n]
    o_cap, o_off = abi.CdrVHS.items_cap.offset, abi.CdrVHS.items_off.offset
    raw[:, o_cap:o_cap + 4] = caps.astype(np.uint32).view(np.uint8).reshape(n, 4)
    raw[:, o_off:o_off + 8] = offs[:n].astype(np.uint64).view(np.uint8).reshape(n, 8)
    pool = (abi.CdrVHItem * max(1, int(offs[n])))()
    return vhs, pool


def items_cap_for(base: engine.Batch, rebuild: engine.Batch, forks) -> np.ndarray:
    """Per-workflow version-history item slots a replication run needs per branch: every
    branch holds at most the items of the state's whole history (the base's, the rebuilt
    branch's and every fork's version runs: state_caps_for's vh_cap), floor ITEMS_CAP."""
    sp = state_caps_for(base, rebuild, forks)
    n = base.n_wfs
    vh = np.frombuffer(sp.caps, dtype=np.uint8).reshape(max(1, n), C.sizeof(abi.CdrWfCaps))[:n]
    o = abi.CdrWfCaps.vh_cap.offset
    need = vh[:, o:o + 4].copy().view(np.uint32).ravel().astype(np.int64)
    return np.maximum(need, ITEMS_CAP)


def branch_items(vhs, pool, w: int, b: int):
    s = vhs[w]
    off = s.items_off + b * s.items_cap
    return [(pool[off + i].event_id, pool[off + i].version) for i in range(s.branch[b].n_items)]


TABLE_CAP = {"act": "act_cap", "timer": "timer_cap", "child": "child_cap", "cancel": "cancel_cap",
             "signal": "signal_cap", "vh": "vh_cap", "rp": "rp_cap", "sa": "sa_cap"}
TABLE_OFF = {t: c.replace("_cap", "_off") for t, c in TABLE_CAP.items()}
# peak live activities / user timers: a state the rounds leave holds at most the sum of its
# parts' peaks (the apply batches' working slots are sized by it, cdr_plan_ndc_apply)
TUPLE_LIVE = ("act_live", "timer_live")


class GpuBackend:
    """k_ndc_branch alone (the branch-kernel parity test): one cdr_ndc_branch_async call."""

    def __init__(self, eng: engine.Engine):
        self.eng = eng

    def branch(self, tasks, items, vhs, pool, n):
        dev = _Dev()
        try:
            dec = (abi.CdrNdcDecision * max(1, n))()
            pv, pp, pd = dev.up(vhs), dev.up(pool), dev.up(dec)
            rc = abi.lib().cdr_ndc_branch_async(self.eng.ctx, C.c_void_p(dev.up(tasks)), C.c_void_p(dev.up(items)),
                                                n, C.c_void_p(pv), C.c_void_p(pp), C.c_void_p(pd), None)
            if rc:
                raise RuntimeError(f"cdr_ndc_branch_async rc={rc}")
            dev.down(vhs, pv)
            dev.down(pool, pp)
            dev.down(dec, pd)
            return dec
        finally:
            dev.close()


# ------------------------------------------------------------ device-resident rounds
class _Dev:
    """Device buffers through the HIP runtime the engine's context already uses."""

    def __init__(self):
        self.hip = engine._hip()
        self.ptrs = []

    def alloc(self, nbytes: int, zero: bool = True) -> int:
        p = C.c_void_p()
        nb = max(8, int(nbytes))
        if self.hip.hipMalloc(C.byref(p), C.c_size_t(nb)) != 0:
            raise RuntimeError("hipMalloc failed")
        self.ptrs.append(p)
        if zero and self.hip.hipMemset(p, 0, C.c_size_t(nb)) != 0:
            raise RuntimeError("hipMemset failed")
        return p.value

    def up(self, x) -> int:
        if isinstance(x, np.ndarray):
            x = np.ascontiguousarray(x)
            nb, src = x.nbytes, x.ctypes.data
        else:
            nb, src = C.sizeof(x), C.addressof(x)
        p = self.alloc(nb, zero=False)
        if nb and self.hip.hipMemcpy(C.c_void_p(p), C.c_void_p(src), C.c_size_t(nb), 1) != 0:
            raise RuntimeError("hipMemcpy H2D failed")
        return p

    def down(self, dst, p: int, nbytes: int | None = None):
        nb = C.sizeof(dst) if nbytes is None else nbytes
        if nb and self.hip.hipMemcpy(C.c_void_p(C.addressof(dst)), C.c_void_p(p), C.c_size_t(nb), 2) != 0:
            raise RuntimeError("hipMemcpy D2H failed")

    def close(self):
        for p in self.ptrs:
            self.hip.hipFree(p)
        self.ptrs = []


def _plan_from(caps, totals) -> engine.Plan:
    return engine.Plan(caps=caps, totals=totals)


def offsets_from_caps(caps, n):
    """Re-derive every table's offsets (exclusive prefix of its capacities) and the totals."""
    tot = abi.CdrTotals()
    for w in range(n):
        for t, cname in TABLE_CAP.items():
            setattr(caps[w], TABLE_OFF[t], getattr(tot, t))
            setattr(tot, t, getattr(tot, t) + getattr(caps[w], cname))
        caps[w].xfer_off, caps[w].ttask_off = tot.xfer, tot.ttask
        tot.xfer += caps[w].xfer_cap
        tot.ttask += caps[w].ttask_cap
    return tot


def upload_batch(dev: _Dev, batch: engine.Batch, caps, mode: int = abi.PLAN_WAVE | abi.PLAN_PAR,
                 cls: bool = False) -> abi.CdrDevBatch:
    """Host planning + packing (cdr_plan_slices_ex / cdr_pack_slices / cdr_plan_scratch)
    of `batch` with capacities `caps`, uploaded: a device-resident cdr_dev_batch; `cls`:
    with the register-table slices' class-sorted blocks from the host packer (cdr_plan_cls /
    cdr_pack_cls), which k_replay_cls replays."""
    L = abi.lib()
    n = batch.n_wfs
    ns, rows, nw = C.c_uint32(), C.c_uint64(), C.c_uint32()
    rc = L.cdr_plan_slices_ex(batch.wfs, caps, n, mode, None, None, None, None, C.byref(ns), C.byref(rows),
                              C.byref(nw))
    if rc:
        raise RuntimeError(f"cdr_plan_slices_ex rc={rc}")
    lane = np.zeros(max(1, ns.value) * 64, np.int32)
    slen = np.zeros(max(1, ns.value), np.uint32)
    row0 = np.zeros(max(1, ns.value), np.uint64)
    flags = np.zeros(max(1, ns.value), np.uint32)
    L.cdr_plan_slices_ex(batch.wfs, caps, n, mode, lane.ctypes.data, slen.ctypes.data, row0.ctypes.data,
                         flags.ctypes.data, C.byref(ns), C.byref(rows), C.byref(nw))
    bs = batch.cstruct()
    aw = L.cdr_plan_arena_words(C.byref(bs))
    slab = np.zeros(max(1, int(rows.value)) * 64 * abi.EL_BYTES, np.uint8)
    arena = np.zeros(max(1, aw), np.uint64)
    s = abi.CdrSlices(n_slices=ns.value, n_rows=rows.value, arena_words=aw)
    s.slice_row0, s.slice_len, s.lane_wf = row0.ctypes.data, slen.ctypes.data, lane.ctypes.data
    s.slab, s.arena, s.slice_flags = slab.ctypes.data, arena.ctypes.data, flags.ctypes.data
    rc = L.cdr_pack_slices(C.byref(bs), C.byref(s), 0)
    if rc:
        raise RuntimeError(f"cdr_pack_slices rc={rc}")
    sc_off = np.zeros(max(1, ns.value), np.uint64)
    sc_act = np.zeros(max(1, ns.value), np.uint32)
    sc_tim = np.zeros(max(1, ns.value), np.uint32)
    words, nf = C.c_uint64(), C.c_uint32()
    rc = L.cdr_plan_scratch(caps, lane.ctypes.data, ns.value, sc_off.ctypes.data, sc_act.ctypes.data,
                            sc_tim.ctypes.data, flags.ctypes.data, C.byref(words), C.byref(nf))
    if rc:
        raise RuntimeError(f"cdr_plan_scratch rc={rc}")
    db = abi.CdrDevBatch()
    if cls and int(((flags[:ns.value] & abi.CLS_SLICES) != 0).sum()):
        crows = np.zeros(max(1, ns.value * 4), np.uint32)
        crow0 = np.zeros(ns.value + 1, np.uint64)
        rc = L.cdr_plan_cls(C.byref(s), C.cast(batch.wfs, C.c_void_p), crows.ctypes.data, crow0.ctypes.data)
        if rc:
            raise RuntimeError(f"cdr_plan_cls rc={rc}")
        cslab = np.empty(max(8, int(crow0[-1]) * abi.ROW_BYTES), np.uint8)
        rc = L.cdr_pack_cls(C.byref(s), C.cast(batch.wfs, C.c_void_p), crows.ctypes.data, crow0.ctypes.data,
                            cslab.ctypes.data, 0)
        if rc:
            raise RuntimeError(f"cdr_pack_cls rc={rc}")
        db.cls_slab, db.cls_row0, db.cls_rows = dev.up(cslab), dev.up(crow0), dev.up(crows)
    db.ev.n_slices, db.ev.n_rows, db.ev.arena_words = ns.value, rows.value, aw
    db.ev.slice_row0, db.ev.slice_len, db.ev.lane_wf = dev.up(row0), dev.up(slen), dev.up(lane)
    db.ev.slab, db.ev.arena = dev.up(slab), dev.up(arena)
    db.ev.slice_scratch_off, db.ev.slice_act_slots, db.ev.slice_tim_slots = dev.up(sc_off), dev.up(sc_act), dev.up(sc_tim)
    db.ev.slice_flags = dev.up(flags)
    db.scratch = dev.alloc(int(words.value) * 8)
    db.wfs, db.caps = dev.up(batch.wfs), dev.up(caps)
    db.kvs = dev.up(batch.kvs) if len(batch.kvs) else dev.alloc(8)
    db.rps = dev.up(batch.rps) if len(batch.rps) else dev.alloc(8)
    db.n_wfs = n
    db.empty_uuid, db.cluster, db.now_ns, db.uuid_seed = batch.empty_uuid, batch.cluster, batch.now_ns, batch.uuid_seed
    f = flags[:ns.value]
    db.n_fast_slices = nf.value
    db.n_wave_slices = int(((f & abi.SLICE_WAVE) != 0).sum())
    db.n_reg_slices = int(((f & abi.SLICE_REG) != 0).sum())
    db.n_reg2_slices = int(((f & abi.SLICE_REG2) != 0).sum())
    db.n_reg0_slices = int(((f & abi.SLICE_REG0) != 0).sum())
    db.n_par_slices = int(((f & abi.SLICE_PAR) != 0).sum())
    db.max_act_slots = int(sc_act[:ns.value].max()) if ns.value else 0
    db.max_tim_slots = int(sc_tim[:ns.value].max()) if ns.value else 0
    L.cdr_plan_class_ranges(flags.ctypes.data, ns.value, db.class_lo, db.class_hi)
    return db


def alloc_out(dev: _Dev, n: int, totals: abi.CdrTotals, tasks: bool = False) -> abi.CdrOut:
    o = abi.CdrOut()
    o.result = dev.alloc(max(1, n) * C.sizeof(abi.CdrWfResult))
    o.exec = dev.alloc(max(1, n) * C.sizeof(abi.CdrExecInfo))
    o.repl = dev.alloc(max(1, n) * C.sizeof(abi.CdrReplState))
    for t in engine.TABLES:
        setattr(o, t, dev.alloc(max(1, getattr(totals, t)) * C.sizeof(engine.TABLE_TYPES[t])))
    if tasks:
        o.transfer = dev.alloc(max(1, totals.xfer) * C.sizeof(abi.CdrTask))
        o.timer_tasks = dev.alloc(max(1, totals.ttask) * C.sizeof(abi.CdrTask))
        o.n_tasks = dev.alloc(2 * max(1, n) * 4)
    return o


def download_out(dev: _Dev, o: abi.CdrOut, n: int, pl: engine.Plan, tasks: bool = False) -> engine.Outputs:
    class _B:
        pass
    b = _B()
    b.n_wfs = n
    out = engine.Outputs(b, pl, tasks)
    dev.down(out.result, o.result)
    dev.down(out.exec, o.exec)
    dev.down(out.repl, o.repl)
    for t in engine.TABLES:
        dev.down(out.tables[t], getattr(o, t))
    if tasks:
        dev.down(out.tasks["xfer"], o.transfer)
        dev.down(out.tasks["ttask"], o.timer_tasks)
        dev.down(out.tasks["n"], o.n_tasks)
    return out


def state_caps_for(base: engine.Batch, rebuild: engine.Batch, forks, live_sum: bool = False):
    """Per-workflow capacities of the state buffer a replication run keeps: the base replay's
    flags, room for the largest state any round can leave (base or rebuilt rows + every
    fork's new rows).  live_sum: the peak live sets summed over the parts too (the bound an
    apply batch's working slots are sized by, cdr_plan_ndc_apply); else the base's own."""
    n = base.n_wfs
    bp = engine.plan(base)
    parts = [engine.plan(rebuild)] + [engine.plan(fb) for fb, _, _ in forks]
    caps = (abi.CdrWfCaps * max(1, n))()
    C.memmove(caps, bp.caps, C.sizeof(abi.CdrWfCaps) * n)
    for w in range(n):
        for cname in (TUPLE_LIVE if live_sum else ()) + tuple(TABLE_CAP.values()):
            setattr(caps[w], cname, getattr(bp.caps[w], cname) + sum(getattr(p.caps[w], cname) for p in parts))
    tot = offsets_from_caps(caps, n)
    return _plan_from(caps, tot)


class DeviceReplicator:
    """The device-resident replication run over a batch of workflows: the base branch
    replayed into the state buffer, then one cdr_ndc_replicate_async call per fork round —
    branch, rebuild + refresh + verify, apply onto the in-memory rebuilt or the loaded
    state, VH sync, adopt — with every buffer allocated up front."""

    def __init__(self, eng: engine.Engine, base: engine.Batch, rebuild: engine.Batch, forks, items_cap=None,
                 refresh_flags: int = abi.REFRESH_ADVANCED_VISIBILITY):
        n = base.n_wfs
        L = abi.lib()
        self.eng, self.n, self.dev = eng, n, _Dev()
        dev = self.dev
        self.state_plan = state_caps_for(base, rebuild, forks)
        live_bound = state_caps_for(base, rebuild, forks, live_sum=True).caps
        # the base and rebuild replays run the class-decomposed kernel (their class-sorted
        # blocks come from the host packer, like the rest of the setup)
        self.base_db = upload_batch(dev, base, self.state_plan.caps, cls=True)
        self.state = alloc_out(dev, n, self.state_plan.totals)
        self.state_caps_d = self.base_db.caps  # the state's capacities (the base batch was planned with them)
        self.rebuild_plan = engine.plan(rebuild)
        self.rebuild_db = upload_batch(dev, rebuild, self.rebuild_plan.caps, cls=True)
        self.rebuild_out = alloc_out(dev, n, self.rebuild_plan.totals, tasks=True)
        self.rounds = []
        for fb, tasks, items in forks:
            caps = (abi.CdrWfCaps * max(1, n))()
            tot = abi.CdrTotals()
            rc = L.cdr_plan_ndc_apply(C.byref(fb.cstruct()), live_bound, caps, C.byref(tot))
            if rc:
                raise RuntimeError(f"cdr_plan_ndc_apply rc={rc}")
            pl = _plan_from(caps, tot)
            r = abi.CdrNdcRound()
            r.tasks, r.task_items = dev.up(tasks), dev.up(items)
            r.rebuild, r.rebuild_out = self.rebuild_db, self.rebuild_out
            r.apply = upload_batch(dev, fb, caps, 0)
            r.apply_out = alloc_out(dev, n, tot)
            r.dec = dev.alloc(max(1, n) * C.sizeof(abi.CdrNdcDecision))
            r.refresh_now = rebuild.now_ns
            r.refresh_flags = refresh_flags
            self.rounds.append((r, pl))
        self.vhs_h, self.pool_h = new_vhs(n, items_cap_for(base, rebuild, forks) if items_cap is None else items_cap)
        self.vhs, self.pool = dev.up(self.vhs_h), dev.up(self.pool_h)
        self.vhs_fresh = dev.up(self.vhs_h)  # NewVersionHistories for every workflow (reset())
        self.events = [int(sum(base.wfs[w].ev_len for w in range(n)))] + [
            int(sum(fb.wfs[w].ev_len for w in range(n))) for fb, _, _ in forks]

    def reset(self, stream=None):
        """A fresh run: every workflow's VersionHistories back to empty (the base replay
        re-creates the state buffer itself); a device-to-device copy on the stream."""
        hip = self.dev.hip
        if hip.hipMemcpyAsync(C.c_void_p(self.vhs), C.c_void_p(self.vhs_fresh),
                              C.c_size_t(C.sizeof(self.vhs_h)), 3, C.c_void_p(stream)) != 0:
            raise RuntimeError("hipMemcpyAsync D2D failed")

    def base_replay(self, stream=None):
        L = abi.lib()
        rc = L.cdr_replay_sliced_async(self.eng.ctx, C.byref(self.base_db), C.byref(self.state), C.c_void_p(stream))
        if rc:
            raise RuntimeError(f"cdr_replay_sliced_async rc={rc}")
        rc = L.cdr_vhs_sync_async(self.eng.ctx, self.n, C.c_void_p(self.vhs), C.c_void_p(self.pool),
                                  C.c_void_p(self.state_caps_d), C.byref(self.state), C.c_void_p(stream))
        if rc:
            raise RuntimeError(f"cdr_vhs_sync_async rc={rc}")

    def round(self, k: int, stream=None):
        r, _ = self.rounds[k]
        rc = abi.lib().cdr_ndc_replicate_async(self.eng.ctx, self.n, C.byref(r), C.c_void_p(self.vhs),
                                               C.c_void_p(self.pool), C.c_void_p(self.state_caps_d),
                                               C.byref(self.state), C.c_void_p(stream))
        if rc:
            raise RuntimeError(f"cdr_ndc_replicate_async rc={rc}")

    def run(self):
        """Base replay + every round; returns (state Outputs, vhs, pool, [decisions],
        [(rebuild Outputs, apply Outputs) per round])."""
        self.reset()
        self.base_replay()
        per_round, decs = [], []
        for k, (r, pl) in enumerate(self.rounds):
            self.round(k)
            dec = (abi.CdrNdcDecision * max(1, self.n))()
            self.dev.down(dec, r.dec)
            decs.append(dec)
            per_round.append((download_out(self.dev, self.rebuild_out, self.n, self.rebuild_plan, tasks=True),
                              download_out(self.dev, r.apply_out, self.n, pl)))
        self.dev.down(self.vhs_h, self.vhs)
        self.dev.down(self.pool_h, self.pool)
        state = download_out(self.dev, self.state, self.n, self.state_plan)
        return state, self.vhs_h, self.pool_h, decs, per_round

    def close(self):
        self.dev.close()


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
