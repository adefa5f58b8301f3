"""Host-side engine API over libcdr (the MI355X replay engine's C ABI).

``Batch`` is a decoded history batch in the ABI's natural order (one record per
HistoryEvent, workflows contiguous); ``Outputs`` are the persisted mutable states
(include/cdr/schema.h).  ``replay(batch)`` runs the HIP path through
``cdr_replay_batch``; there is no CPU fallback — without the in-tree libcdr.so or a
GPU it raises.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import abi

TABLES = ("act", "timer", "child", "cancel", "signal", "vh", "rp", "sa")
TABLE_TYPES = {
    "act": abi.CdrActivityInfo, "timer": abi.CdrTimerInfo, "child": abi.CdrChildInfo,
    "cancel": abi.CdrCancelInfo, "signal": abi.CdrSignalInfo, "vh": abi.CdrVHItem, "rp": abi.CdrResetPoint,
    "sa": abi.CdrKV,
}
TABLE_COUNT = {"act": "n_activity", "timer": "n_timer", "child": "n_child", "cancel": "n_cancel",
               "signal": "n_signal", "vh": "n_vh", "rp": "n_reset_points", "sa": "n_search_attr"}


@dataclass
class Batch:
    events: C.Array
    wfs: C.Array
    kvs: C.Array
    rps: C.Array
    cluster: abi.CdrClusterMeta
    now_ns: int = 1_700_000_000_000_000_000
    uuid_seed: int = 1
    empty_uuid: int = 1
    strings: list = field(default_factory=list)  # handle -> string (fixture batches)
    carry: "Carry | None" = None  # loaded mutable states (cdr_carry), None = fresh builders

    @property
    def n_wfs(self):
        return len(self.wfs)

    def cstruct(self) -> abi.CdrBatch:
        b = abi.CdrBatch()
        b.events = C.cast(self.events, C.POINTER(abi.CdrEvent))
        b.n_events = len(self.events)
        b.wfs = C.cast(self.wfs, C.POINTER(abi.CdrWfDesc))
        b.n_wfs = len(self.wfs)
        b.empty_uuid = self.empty_uuid
        b.kvs = C.cast(self.kvs, C.POINTER(abi.CdrKV))
        b.n_kvs = len(self.kvs)
        b.rps = C.cast(self.rps, C.POINTER(abi.CdrResetPoint))
        b.n_rps = len(self.rps)
        b.cluster = self.cluster
        b.now_ns = self.now_ns
        b.uuid_seed = self.uuid_seed
        if self.carry is not None:
            b.carry = C.addressof(self.carry.cstruct())
        self._keep = b
        return b


@dataclass
class Carry:
    """Loaded mutable states for a batch (cdr_carry): entry w replays onto record
    src[w] of `state` (the Outputs of an earlier replay), -1 = fresh builder — the
    mutableStateBuilder.Load + applyEvents path (mutableStateBuilder.go:272-295)."""
    src: np.ndarray
    state: "Outputs"
    in_memory: "np.ndarray | None" = None  # uint8 per entry: continue an in-memory builder (cdr_carry.in_memory)

    def cstruct(self) -> abi.CdrCarry:
        self.src = np.ascontiguousarray(self.src, dtype=np.int32)
        c = abi.CdrCarry()
        c.src = self.src.ctypes.data
        if self.in_memory is not None:
            self.in_memory = np.ascontiguousarray(self.in_memory, dtype=np.uint8)
            c.in_memory = self.in_memory.ctypes.data
        c.caps = C.addressof(self.state.plan.caps)
        c.n_src = self.state.n_wfs
        c.totals = self.state.plan.totals
        c.state = self.state.cstruct()
        self._keep = c
        return c


def _calls(batch: Batch, w: int) -> list:
    """Event offsets (within entry w) where each applyEvents call starts."""
    d = batch.wfs[w]
    return [k for k in range(d.ev_len) if k == 0 or batch.events[d.ev_off + k].flags & abi.EVF_BATCH_FIRST]


def _entry_batch(batch: Batch, wfs, carry=None) -> Batch:
    return Batch(events=batch.events, wfs=wfs, kvs=batch.kvs, rps=batch.rps, cluster=batch.cluster,
                 now_ns=batch.now_ns, uuid_seed=batch.uuid_seed, empty_uuid=batch.empty_uuid,
                 strings=batch.strings, carry=carry)


def split_batch(batch: Batch, seed: int = 1):
    """Cut every top-level entry with two or more calls after a random number of its
    calls (before its continue-as-new call, if any).  Returns (prefix batch, cut) where
    cut[w] is the event offset of the cut (0 = entry not split; its prefix is the whole
    entry).  suffix_batch() builds the rest as a carry-in batch."""
    rng = np.random.default_rng(seed)
    wfs = (abi.CdrWfDesc * batch.n_wfs)()
    C.memmove(wfs, batch.wfs, C.sizeof(wfs))
    cut = np.zeros(batch.n_wfs, np.int64)
    for w in range(batch.n_wfs):
        d = wfs[w]
        if d.parent >= 0:
            continue
        calls = _calls(batch, w)
        hi = len(calls) - 1
        if d.newrun >= 0:
            hi = min(hi, d.newrun_call)
        if hi < 1:
            continue
        c = int(rng.integers(1, hi + 1))
        cut[w] = calls[c]
        d.ev_len = calls[c]  # the prefix never reaches a newrun call: its new run is not applied
    return _entry_batch(batch, wfs), cut


def split_half(batch: Batch) -> np.ndarray:
    """The call boundary nearest after the middle of every top-level entry without a
    continue-as-new (vectorised over the events' flag words, for full-size batches):
    cut[w] = event offset of that call's first event within entry w, 0 = not split (one
    call, or a new-run link).  The prefix [0, cut) and the suffix [cut, len) are the two
    applyEvents sequences a loaded-state replay splits the history into."""
    n = batch.n_wfs
    words = C.sizeof(abi.CdrEvent) // 4
    ev = np.frombuffer(batch.events, dtype=np.uint32).reshape(-1, words) if len(batch.events) else \
        np.zeros((0, words), np.uint32)
    bf = np.nonzero(ev[:, abi.CdrEvent.flags.offset // 4] & abi.EVF_BATCH_FIRST)[0].astype(np.int64)
    wf = np.frombuffer(batch.wfs, dtype=np.uint8).reshape(n, C.sizeof(abi.CdrWfDesc))

    def col(name, dt):
        o = getattr(abi.CdrWfDesc, name).offset
        return wf[:, o:o + np.dtype(dt).itemsize].copy().view(dt).ravel()
    off, ln = col("ev_off", np.uint64).astype(np.int64), col("ev_len", np.uint64).astype(np.int64)
    top = (col("parent", np.int32) < 0) & (col("newrun", np.int32) < 0)
    i = np.searchsorted(bf, off + ln // 2)
    pos = np.where(i < len(bf), bf[np.minimum(i, max(0, len(bf) - 1))] if len(bf) else 0, -1)
    ok = top & (pos > off) & (pos < off + ln)
    return np.where(ok, pos - off, 0)


def cut_batches(batch: Batch, cut) -> tuple:
    """(prefix wfs, suffix wfs) descriptor arrays of a split: entry w's events [0, cut[w])
    and [cut[w], len) (cut 0: the prefix is the whole entry and the suffix replays it again
    on a fresh builder — its carry src is -1)."""
    n = batch.n_wfs
    pre = (abi.CdrWfDesc * n)()
    suf = (abi.CdrWfDesc * n)()
    C.memmove(pre, batch.wfs, C.sizeof(pre))
    C.memmove(suf, batch.wfs, C.sizeof(suf))
    for w in np.nonzero(np.asarray(cut) > 0)[0]:
        c = int(cut[w])
        pre[w].ev_len = c
        suf[w].ev_off += c
        suf[w].ev_len -= c
    return _entry_batch(batch, pre), _entry_batch(batch, suf)


def suffix_batch(batch: Batch, cut, prefix: Batch, prefix_out: "Outputs") -> Batch:
    """The remainder of split_batch's cut as a batch replaying onto the prefix's
    persisted states; entries whose prefix failed (or were not cut) replay whole on a
    fresh builder."""
    wfs = (abi.CdrWfDesc * batch.n_wfs)()
    C.memmove(wfs, batch.wfs, C.sizeof(wfs))
    src = np.full(batch.n_wfs, -1, np.int32)
    for w in range(batch.n_wfs):
        c = int(cut[w])
        if c == 0 or prefix_out.result[w].code != abi.OK:
            continue
        d = wfs[w]
        calls_before = len(_calls(prefix, w))
        d.ev_off += c
        d.ev_len -= c
        if d.newrun >= 0:
            d.newrun_call -= calls_before
        src[w] = w
    return _entry_batch(batch, wfs, Carry(src=src, state=prefix_out))


def default_cluster() -> abi.CdrClusterMeta:
    c = abi.CdrClusterMeta()
    c.failover_version_increment = 10
    c.current_cluster = 0
    c.n_clusters = 3
    for i, v in enumerate((1, 2, 3)):
        c.initial_version[i] = v
    return c


class SynthBuffers:
    """Host buffers reused across synth_batch calls (chunked full-size generation):
    grown on demand, never zero-filled (cdr_synth_fill writes every byte it hands out)."""

    def __init__(self):
        self._b = {}

    def get(self, name: str, ty, n: int):
        need = max(1, n) * C.sizeof(ty)
        buf = self._b.get(name)
        if buf is None or buf.nbytes < need:
            buf = np.empty(int(need * 1.25) if name in self._b else need, np.uint8)
            self._b[name] = buf
        return (ty * max(1, n)).from_buffer(buf)


def synth_batch(config: int, n_wfs: int, seed: int, target_len: int = 0, max_len: int = 0,
                error_rate: float = 0.0, builder: int = -1, rebuild: bool = False, fault_kinds: int = 0,
                index_map=None, buffers: "SynthBuffers | None" = None, part: int = 0, long_stride: int = 0) -> Batch:
    """Deterministic synthetic batch (cadence_amd/csrc/synth.cpp) in natural order.
    `index_map` (uint32 array of n_wfs global workflow indices) generates a shard's
    share of a larger population: workflow i of the batch is global workflow
    index_map[i], identical to what the whole-population batch holds at that index.
    `buffers`: reuse these host buffers (the batch is valid until the next call with
    the same buffers).  `part` (config 5): which part of the forked histories
    (abi.SYNTH_PART_*: base, rebuild path, fork A, fork B)."""
    L = abi.lib()
    p = abi.CdrSynthParams(config=config, n_wfs=n_wfs, seed=seed, target_len=target_len, max_len=max_len,
                           error_rate=error_rate, builder=builder, rebuild=1 if rebuild else 0,
                           fault_kinds=fault_kinds, ndc_part=part, long_stride=long_stride)
    if index_map is not None:
        index_map = np.ascontiguousarray(index_map, dtype=np.uint32)
        assert len(index_map) == n_wfs
        p.index_map = index_map.ctypes.data
    sz = abi.CdrSynthSizes()
    rc = L.cdr_synth_size(C.byref(p), C.byref(sz))
    if rc:
        raise RuntimeError(f"cdr_synth_size rc={rc}")
    if buffers is not None:
        ev = buffers.get("ev", abi.CdrEvent, sz.n_events)
        wfs = buffers.get("wfs", abi.CdrWfDesc, sz.n_entries)
        kvs = buffers.get("kvs", abi.CdrKV, sz.n_kvs)
        rps = buffers.get("rps", abi.CdrResetPoint, sz.n_rps)
    else:
        ev = (abi.CdrEvent * max(1, sz.n_events))()
        wfs = (abi.CdrWfDesc * sz.n_entries)()
        kvs = (abi.CdrKV * max(1, sz.n_kvs))()
        rps = (abi.CdrResetPoint * max(1, sz.n_rps))()
    cb = abi.CdrBatch()
    rc = L.cdr_synth_fill(C.byref(p), ev, wfs, kvs, rps, C.byref(cb))
    if rc:
        raise RuntimeError(f"cdr_synth_fill rc={rc}")
    ev = (abi.CdrEvent * sz.n_events).from_buffer(ev) if sz.n_events else (abi.CdrEvent * 0)()
    wfs = (abi.CdrWfDesc * sz.n_entries).from_buffer(wfs)
    kvs = (abi.CdrKV * sz.n_kvs).from_buffer(kvs) if sz.n_kvs else (abi.CdrKV * 0)()
    rps = (abi.CdrResetPoint * sz.n_rps).from_buffer(rps) if sz.n_rps else (abi.CdrResetPoint * 0)()
    return Batch(events=ev, wfs=wfs, kvs=kvs, rps=rps, cluster=cb.cluster, now_ns=cb.now_ns,
                 uuid_seed=cb.uuid_seed, empty_uuid=cb.empty_uuid)


@dataclass
class Plan:
    caps: C.Array
    totals: abi.CdrTotals


def slice_kinds(batch: Batch, pl: "Plan | None" = None, mode: int = abi.PLAN_WAVE) -> tuple:
    """(fast-path slices, wave slices, slices) of the batch's slice plan (host planner only)."""
    L = abi.lib()
    pl = pl or plan(batch)
    ns, rows, nw = C.c_uint32(), C.c_uint64(), C.c_uint32()
    L.cdr_plan_slices_ex(batch.wfs, pl.caps, batch.n_wfs, mode, None, None, None, None, C.byref(ns), C.byref(rows),
                         C.byref(nw))
    lane = np.zeros(max(1, ns.value) * 64, np.int32)
    flags = np.zeros(max(1, ns.value), np.uint32)
    L.cdr_plan_slices_ex(batch.wfs, pl.caps, batch.n_wfs, mode, lane.ctypes.data, None, None, flags.ctypes.data,
                         C.byref(ns), C.byref(rows), C.byref(nw))
    words, nf = C.c_uint64(), C.c_uint32()
    L.cdr_plan_scratch(pl.caps, lane.ctypes.data, ns.value, None, None, None, flags.ctypes.data, C.byref(words),
                       C.byref(nf))
    return nf.value, nw.value, ns.value


def fast_slices(batch: Batch, pl: "Plan | None" = None) -> tuple:
    """(fast-path slices, slices) of the batch's lane-slice plan (no wave slices)."""
    nf, _, ns = slice_kinds(batch, pl, 0)
    return nf, ns


def plan(batch: Batch) -> Plan:
    L = abi.lib()
    caps = (abi.CdrWfCaps * max(1, batch.n_wfs))()
    tot = abi.CdrTotals()
    rc = L.cdr_plan_caps(C.byref(batch.cstruct()), caps, C.byref(tot))
    if rc:
        raise RuntimeError(f"cdr_plan_caps rc={rc}")
    return Plan(caps=caps, totals=tot)


class Outputs:
    """Host buffers for one batch's persisted mutable states (zero-initialised)."""

    def __init__(self, batch: Batch, pl: Plan, tasks: bool = False):
        n = max(1, batch.n_wfs)
        self.n_wfs = batch.n_wfs
        self.plan = pl
        self.result = (abi.CdrWfResult * n)()
        self.exec = (abi.CdrExecInfo * n)()
        self.repl = (abi.CdrReplState * n)()
        self.tables = {t: (TABLE_TYPES[t] * max(1, getattr(pl.totals, t)))() for t in TABLES}
        self.last_decision = (abi.CdrLastDecision * n)()  # applyEvents' lastDecision per entry
        self.tasks = None
        if tasks:  # stateBuilder transfer / timer task lists (cdr_task)
            self.alloc_tasks(pl)

    def alloc_tasks(self, pl: Plan):
        """(Re)allocate zeroed task lists (cdr_task) sized by the plan's totals."""
        self.tasks = {"xfer": (abi.CdrTask * max(1, pl.totals.xfer))(),
                      "ttask": (abi.CdrTask * max(1, pl.totals.ttask))(),
                      "n": (C.c_uint32 * (2 * max(1, self.n_wfs)))()}

    def cstruct(self) -> abi.CdrOut:
        o = abi.CdrOut()
        o.result = C.addressof(self.result)
        o.exec = C.addressof(self.exec)
        o.repl = C.addressof(self.repl)
        for t in TABLES:
            setattr(o, t, C.addressof(self.tables[t]))
        o.last_decision = C.addressof(self.last_decision)
        if self.tasks is not None:
            o.transfer = C.addressof(self.tasks["xfer"])
            o.timer_tasks = C.addressof(self.tasks["ttask"])
            o.n_tasks = C.addressof(self.tasks["n"])
        self._keep = o
        return o

    def task_rows(self, w: int, kind: str):
        """Transfer ("xfer") or timer ("ttask") tasks of entry w, in generation order."""
        c = self.plan.caps[w]
        off = c.xfer_off if kind == "xfer" else c.ttask_off
        n = self.tasks["n"][2 * w + (0 if kind == "xfer" else 1)]
        return [self.tasks[kind][off + j] for j in range(n)]

    # ---- per-workflow accessors
    def rows(self, w: int, table: str):
        r = self.result[w]
        c = self.plan.caps[w]
        off = getattr(c, {"act": "act_off", "timer": "timer_off", "child": "child_off", "cancel": "cancel_off",
                          "signal": "signal_off", "vh": "vh_off", "rp": "rp_off", "sa": "sa_off"}[table])
        n = getattr(r, TABLE_COUNT[table])
        return [self.tables[table][off + j] for j in range(n)]


_hip_lib = None


def _hip():
    """The HIP runtime (device buffers for small host-driven calls; no torch)."""
    global _hip_lib
    if _hip_lib is None:
        # the runtime libcdr.so is bound to: by soname, after libcdr.so is loaded (with torch
        # loaded first that is torch's copy, whose soname is the same; a plain
        # "libamdhip64.so" would load a second runtime beside it)
        abi.lib()
        L = C.CDLL("libamdhip64.so.7")
        L.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
        L.hipFree.argtypes = [C.c_void_p]
        L.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        L.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
        L.hipMemset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
        L.hipStreamCreate.argtypes = [C.POINTER(C.c_void_p)]
        L.hipStreamDestroy.argtypes = [C.c_void_p]
        L.hipMemGetInfo.argtypes = [C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]
        _hip_lib = L
    return _hip_lib


class Engine:
    """One device context (the analogue of one stateBuilder provider)."""

    def __init__(self, device: int = 0, fast_path: bool = True, wave: bool = True):
        L = abi.lib()
        opts = abi.CdrOpts()
        L.cdr_opts_default(C.byref(opts))
        opts.fast_path = 1 if fast_path else 0
        opts.plan_mode = (abi.PLAN_WAVE | abi.PLAN_PAR) if wave else 0
        self.ctx = L.cdr_create(device, C.byref(opts))
        if not self.ctx:
            raise RuntimeError("cdr_create failed: no usable HIP device (the engine has no CPU fallback)")

    def set_wave(self, enable: bool) -> bool:
        """Plan divergent histories into wave slices (one wavefront per workflow,
        replay_wave.inc; default) or into lane slices of the general kernel; returns
        the previous setting."""
        return bool(abi.lib().cdr_set_plan_mode(self.ctx, (abi.PLAN_WAVE | abi.PLAN_PAR) if enable else 0))

    def set_plan_mode(self, mode: int) -> int:
        """CDR_PLAN_* bits of cdr_replay_batch's slicing; returns the previous mode."""
        return int(abi.lib().cdr_set_plan_mode(self.ctx, mode))

    def set_cls(self, mode) -> int:
        """Class-decomposed replay of the register-table slices (k_replay_cls,
        cdr_set_cls_path): True / abi.CLS_BUILD — cdr_replay_batch packs their class-sorted
        blocks and replays them with k_replay_cls; False / abi.CLS_OFF — k_replay_reg alone;
        abi.CLS_ON (the context default) — class blocks only for device-resident batches
        that carry them; abi.CLS_ALONE (tests) — k_replay_cls without the k_replay_reg pass
        for the entries it hands on (result code CLS_RETRY).  Returns the previous mode."""
        if mode is True:
            mode = abi.CLS_BUILD
        elif mode is False:
            mode = abi.CLS_OFF
        return int(abi.lib().cdr_set_cls_path(self.ctx, int(mode)))

    def set_fast_path(self, enable: bool) -> bool:
        """Route sequential-activity slices to the fast-path kernel (default) or replay
        everything with the general kernel; returns the previous setting."""
        return bool(abi.lib().cdr_set_fast_path(self.ctx, 1 if enable else 0))

    def close(self):
        if self.ctx:
            abi.lib().cdr_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def replay(self, batch: Batch, pl: Plan | None = None, tasks: bool = False) -> Outputs:
        """Replay through cdr_replay_batch; `tasks` also emits the transfer / timer
        task lists (the kernels' TASKS instantiations; no wave / PAR slices)."""
        pl = pl or plan(batch)
        out = Outputs(batch, pl, tasks)
        rc = abi.lib().cdr_replay_batch(self.ctx, C.byref(batch.cstruct()), pl.caps, C.byref(pl.totals),
                                       C.byref(out.cstruct()), None)
        if rc:
            raise RuntimeError(f"cdr_replay_batch rc={rc}")
        return out

    def replay_one(self, batch: Batch) -> Outputs:
        """One workflow through cdr_replay_one (the applyEvents shim's call): `batch`
        holds its entry and, if it continues as new, the new run's (n_wfs 1 or 2).  The
        context's view is copied into an Outputs."""
        L = abi.lib()
        view, caps = C.c_void_p(), C.c_void_p()
        rc = L.cdr_replay_one(self.ctx, C.byref(batch.cstruct()), C.byref(view), C.byref(caps), None)
        if rc:
            raise RuntimeError(f"cdr_replay_one rc={rc}")
        v = abi.CdrOut.from_address(view.value)
        n = batch.n_wfs
        cp = (abi.CdrWfCaps * n).from_address(caps.value)
        pl = Plan((abi.CdrWfCaps * n)(), abi.CdrTotals())
        C.memmove(pl.caps, cp, C.sizeof(pl.caps))
        for t in TABLES:  # totals: the end of the last entry's slice of each table
            setattr(pl.totals, t, max(getattr(c, t + "_off") + getattr(c, t + "_cap") for c in pl.caps))
        out = Outputs(batch, pl)
        for name, dst in (("result", out.result), ("exec", out.exec), ("repl", out.repl),
                          ("last_decision", out.last_decision)):
            C.memmove(dst, getattr(v, name), C.sizeof(dst))
        for t in TABLES:
            C.memmove(out.tables[t], getattr(v, t), C.sizeof(TABLE_TYPES[t]) * getattr(pl.totals, t))
        return out

    def encode_rows(self, batch: Batch, out: Outputs, table: str) -> bytes:
        """sqlblobs row blobs of one pending table ("timer" or "cancel") of replayed
        outputs through cdr_encode_rows_async (the records go to HBM, the blobs come
        back): blob of row r in the slot at r * CDR_BLOB_*_STRIDE, returned as
        {row: blob bytes} for the rows of OK entries.  Device memory through the HIP
        runtime directly (the context this engine already initialised)."""
        tid, size, stride = {"timer": (1, 45, 48), "cancel": (3, 66, 80)}[table]
        hip = _hip()
        pl = out.plan
        ptrs = []

        def dalloc(nbytes):
            p = C.c_void_p()
            if hip.hipMalloc(C.byref(p), C.c_size_t(max(8, nbytes))) != 0:
                raise RuntimeError("hipMalloc failed")
            ptrs.append(p)
            return p

        def up(x):
            nb = C.sizeof(x)
            p = dalloc(nb)
            if hip.hipMemcpy(p, C.addressof(x), C.c_size_t(nb), 1) != 0:  # hipMemcpyHostToDevice
                raise RuntimeError("hipMemcpy H2D failed")
            return p
        try:
            n_rows = max(1, getattr(pl.totals, table))
            db = abi.CdrDevBatch()
            db.n_wfs = batch.n_wfs
            db.caps = up(pl.caps)
            o = abi.CdrOut()
            o.result = up(out.result)
            setattr(o, table, up(out.tables[table]))
            blobs = dalloc(n_rows * stride)
            hip.hipMemset(blobs, 0, C.c_size_t(n_rows * stride))
            rc = abi.lib().cdr_encode_rows_async(self.ctx, tid, C.byref(db), C.byref(o), blobs, None)
            if rc:
                raise RuntimeError(f"cdr_encode_rows_async rc={rc}")
            host = (C.c_uint8 * (n_rows * stride))()
            if hip.hipMemcpy(host, blobs, C.c_size_t(n_rows * stride), 2) != 0:  # DeviceToHost (synchronises)
                raise RuntimeError("hipMemcpy D2H failed")
            raw = bytes(host)
            off = {"timer": "timer_off", "cancel": "cancel_off"}[table]
            cnt = {"timer": "n_timer", "cancel": "n_cancel"}[table]
            blobs_out = {}
            for w in range(batch.n_wfs):
                if out.result[w].code == abi.OK:
                    base = getattr(pl.caps[w], off)
                    for j in range(getattr(out.result[w], cnt)):
                        r = base + j
                        blobs_out[r] = raw[r * stride:r * stride + size]
                        assert raw[r * stride + size:(r + 1) * stride] == bytes(stride - size), "slot padding"
            return blobs_out
        finally:
            for p in ptrs:
                hip.hipFree(p)

    def encode_blobs(self, batch: Batch, out: Outputs, table: str, strings: list, persist=None,
                     cluster_names=None, form: str = "sql"):
        """Variable-size sqlblobs row blobs through cdr_encode_blobs_async (size pass +
        scan, then the write pass) for table "act", "child", "signal" or "exec", with
        `strings[h]` (bytes) the string table: ({row: blob}, {row: CDR_BLOB_* status}) for
        the rows of OK entries (exec: row = entry).  `persist` is a cdr_exec_persist array
        and `cluster_names` a list of handles (table "exec").  form="cql": the Cassandra
        form instead (cdr_encode_cql_async: each row's CQL bound values), tables "act",
        "timer", "child", "cancel", "signal", "exec"."""
        tid = {"act": 0, "timer": 1, "child": 2, "cancel": 3, "signal": 4, "exec": 5}[table]
        fn = "cdr_encode_cql_async" if form == "cql" else "cdr_encode_blobs_async"
        hip = _hip()
        pl = out.plan
        ptrs = []

        def dalloc(nbytes):
            p = C.c_void_p()
            if hip.hipMalloc(C.byref(p), C.c_size_t(max(8, nbytes))) != 0:
                raise RuntimeError("hipMalloc failed")
            ptrs.append(p)
            return p

        def up(x, nb=None):
            nb = C.sizeof(x) if nb is None else nb
            p = dalloc(nb)
            if nb and hip.hipMemcpy(p, x if isinstance(x, int) else C.addressof(x), C.c_size_t(nb), 1) != 0:
                raise RuntimeError("hipMemcpy H2D failed")
            return p

        def down(p, nb):
            host = (C.c_uint8 * max(1, nb))()
            if nb and hip.hipMemcpy(host, p, C.c_size_t(nb), 2) != 0:
                raise RuntimeError("hipMemcpy D2H failed")
            return bytes(host)[:nb]
        try:
            lens = np.array([len(s) for s in strings], np.uint64)
            off = np.zeros(len(strings) + 1, np.uint64)
            np.cumsum(lens, out=off[1:])
            blob = np.frombuffer(b"".join(strings) or b"\0", np.uint8)
            st = abi.CdrStrtab(n=len(strings))
            st.bytes = up(blob.ctypes.data, blob.nbytes).value
            st.off = up(off.ctypes.data, off.nbytes).value
            db = abi.CdrDevBatch()
            db.n_wfs = batch.n_wfs
            db.caps = up(pl.caps)
            db.wfs = up(batch.wfs)
            db.cluster = batch.cluster
            o = abi.CdrOut()
            o.result = up(out.result)
            for t in ("exec", "repl"):
                setattr(o, t, up(getattr(out, t)))
            for t in ("act", "timer", "child", "cancel", "signal", "vh", "rp", "sa"):
                setattr(o, t, up(out.tables[t]))
            n_rows = batch.n_wfs if table == "exec" else max(1, getattr(pl.totals, table))
            pp = up(persist) if persist is not None else None
            cn = up((C.c_uint32 * max(1, len(cluster_names or [])))(*(cluster_names or [])))
            row_off = dalloc(8 * (n_rows + 1))
            status = dalloc(4 * n_rows)
            L = abi.lib()
            rc = getattr(L, fn)(self.ctx, tid, C.byref(db), C.byref(o), C.byref(st), pp, cn, n_rows,
                                row_off, None, status, None)
            if rc:
                raise RuntimeError(f"{fn} (sizes) rc={rc}")
            offs = np.frombuffer(down(row_off, 8 * (n_rows + 1)), np.uint64)
            total = int(offs[-1])
            blobs = dalloc(total)
            rc = getattr(L, fn)(self.ctx, tid, C.byref(db), C.byref(o), C.byref(st), pp, cn, n_rows,
                                row_off, blobs, status, None)
            if rc:
                raise RuntimeError(f"{fn} (write) rc={rc}")
            raw = down(blobs, total)
            stat = np.frombuffer(down(status, 4 * n_rows), np.int32)
            got, codes = {}, {}
            cnt = {"act": "n_activity", "timer": "n_timer", "child": "n_child", "cancel": "n_cancel",
                   "signal": "n_signal"}.get(table)
            for w in range(batch.n_wfs):
                if out.result[w].code != abi.OK:
                    continue
                rows = [w] if table == "exec" else [getattr(pl.caps[w], table + "_off") + j
                                                     for j in range(getattr(out.result[w], cnt))]
                for r in rows:
                    got[r] = raw[int(offs[r]):int(offs[r + 1])]
                    codes[r] = int(stat[r])
            return got, codes
        finally:
            for p in ptrs:
                hip.hipFree(p)

    def rebuild(self, batch: Batch, pl: Plan | None = None, advanced_visibility: bool = True, snapshot: bool = False) -> Outputs:
        """nDCStateRebuilder.rebuild's device half through cdr_rebuild_batch: replay
        (every kernel) then refreshTasks (refresh.hip) with now = batch.now_ns; the
        task lists are the refresher's."""
        pl = pl or plan(batch)
        out = Outputs(batch, pl, tasks=True)
        flags = (abi.REFRESH_ADVANCED_VISIBILITY if advanced_visibility else 0) | (
        abi.REFRESH_SNAPSHOT_PASSIVE if snapshot else 0)
        rc = abi.lib().cdr_rebuild_batch(self.ctx, C.byref(batch.cstruct()), pl.caps, C.byref(pl.totals),
                                        C.byref(out.cstruct()), flags, None)
        if rc:
            raise RuntimeError(f"cdr_rebuild_batch rc={rc}")
        return out


# ------------------------------------------------------------------ comparison
def _bytes(x) -> bytes:
    return bytes(memoryview(x).cast("B"))


def compare(batch: Batch, a: Outputs, b: Outputs, limit: int = 10, last_decision: bool = True):
    """Field-by-field comparison of two output sets (result of every workflow; the
    persisted state of every OK workflow; applyEvents' lastDecision unless
    last_decision=False).  Returns a list of mismatch strings."""
    bad = []
    for w in range(batch.n_wfs):
        ra, rb = a.result[w], b.result[w]
        ka = _bytes(ra)
        kb = _bytes(rb)
        if ka != kb:
            bad.append(f"wf {w}: result {_rec(ra, None)} != {_rec(rb, None)}")
        elif ra.code == abi.OK:
            if _bytes(a.exec[w]) != _bytes(b.exec[w]):
                diffs = [f for f, _ in abi.CdrExecInfo._fields_
                         if getattr(a.exec[w], f) != getattr(b.exec[w], f)]
                bad.append(f"wf {w}: exec differs in {diffs}")
            if batch.wfs[w].builder == abi.BUILDER_2DC and _bytes(a.repl[w]) != _bytes(b.repl[w]):
                bad.append(f"wf {w}: replication state differs")
            la, lb = a.last_decision[w], b.last_decision[w]
            if last_decision and _bytes(la) != _bytes(lb):
                bad.append(f"wf {w}: lastDecision differs in "
                           f"{[f for f, _ in abi.CdrLastDecision._fields_ if getattr(la, f) != getattr(lb, f)]}")
            for t in TABLES:
                na, nb = getattr(ra, TABLE_COUNT[t]), getattr(rb, TABLE_COUNT[t])
                if na != nb:
                    bad.append(f"wf {w}: {t} count {na} != {nb}")
                    continue
                xa = b"".join(_bytes(r) for r in a.rows(w, t))
                xb = b"".join(_bytes(r) for r in b.rows(w, t))
                if xa != xb:
                    rows_a, rows_b = a.rows(w, t), b.rows(w, t)  # noqa: F841
                    for j, (p, q) in enumerate(zip(rows_a, rows_b)):
                        fd = [f for f, _ in type(p)._fields_ if _bytes(p) != _bytes(q) and
                              getattr(p, f) != getattr(q, f)]
                        if fd:
                            bad.append(f"wf {w}: {t}[{j}] differs in {fd}")
                            break
        if len(bad) >= limit:
            break
    return bad


def compare_tasks(batch: Batch, a: Outputs, b: Outputs, limit: int = 10):
    """Task lists of every entry that is OK in both outputs, field by field."""
    bad = []
    for w in range(batch.n_wfs):
        if a.result[w].code != abi.OK or b.result[w].code != abi.OK:
            continue
        for kind in ("xfer", "ttask"):
            ra, rb = a.task_rows(w, kind), b.task_rows(w, kind)
            if len(ra) != len(rb):
                bad.append(f"wf {w}: {kind} count {len(ra)} != {len(rb)}")
                continue
            for j, (p, q) in enumerate(zip(ra, rb)):
                if _bytes(p) != _bytes(q):
                    bad.append(f"wf {w}: {kind}[{j}] {_rec(p, None)} != {_rec(q, None)}")
                    break
        if len(bad) >= limit:
            break
    return bad


def status_histogram(out: Outputs) -> dict:
    codes = np.array([out.result[w].code for w in range(out.n_wfs)], dtype=np.int64)
    vals, cnt = np.unique(codes, return_counts=True)
    return {abi.STATUS.get(int(v), str(int(v))): int(c) for v, c in zip(vals, cnt)}


# ------------------------------------------------------------------ export
_HANDLE_FIELDS = {
    "domain_id", "workflow_id", "run_id", "create_request_id", "parent_domain_id", "parent_workflow_id",
    "parent_run_id", "task_list", "workflow_type", "decision_request_id", "cron_schedule", "memo", "nonretriable",
    "branch_tree_id", "activity_id", "request_id", "timer_id", "started_workflow_id", "started_run_id",
    "domain_name", "signal_name", "input", "control", "binary_checksum", "key", "value",
}


def _rec(x, strings):
    d = {}
    for f, ty in type(x)._fields_:
        if f.startswith("_pad"):
            continue
        v = getattr(x, f)
        if hasattr(v, "__len__") and not isinstance(v, (bytes, str)):
            v = list(v)
        elif strings and f in _HANDLE_FIELDS:
            v = strings[v] if v < len(strings) else v
        elif isinstance(v, float):
            v = float.hex(v)  # bit-exact float in JSON
        d[f] = v
    return d


def export_state(batch: Batch, out: Outputs, w: int) -> dict:
    """JSON-able persisted state of workflow `w` (handles mapped to strings when the
    batch carries its string table)."""
    s = batch.strings or None
    r = out.result[w]
    d = {"result": _rec(r, None)}
    d["result"]["status"] = abi.STATUS.get(r.code, str(r.code))
    if r.code == abi.OK:
        d["exec"] = _rec(out.exec[w], s)
        if batch.wfs[w].builder == abi.BUILDER_2DC:
            d["repl"] = _rec(out.repl[w], s)
        for t in TABLES:
            d[t] = [_rec(x, s) for x in out.rows(w, t)]
    return d


def state_digest(batch: Batch, out: Outputs) -> str:
    """sha256 over the exported states of every workflow (golden-fixture pin)."""
    import hashlib
    import json
    h = hashlib.sha256()
    for w in range(batch.n_wfs):
        h.update(json.dumps(export_state(batch, out, w), sort_keys=True).encode())
    return h.hexdigest()
