"""Synthetic device-resident batches (benchmark and full-size parity plumbing).

``DeviceBatch`` generates a deterministic synthetic population (csrc/synth.cpp, the
SURVEY §8(d) config shapes) straight into the sliced SELL-64 layout on the host,
uploads it to HBM with torch (device memory only: torch is plumbing here) and keeps
device output buffers sized by the host planner.  Entry order is the natural order of
``engine.synth_batch`` over the same ``index_map`` (each workflow followed by its
continue-as-new run), so per-entry digests line up with the CPU restatement's.
"""
from __future__ import annotations

import ctypes as C
import os
import time

import numpy as np

from . import abi

# SURVEY §8(d) canonical algorithmic bytes: 48 B core per event + A[type]
A_TYPE = np.zeros(256, np.int64)
for _name, _b in (("WorkflowExecutionStarted", 96), ("ActivityTaskScheduled", 48), ("DecisionTaskScheduled", 12),
                  ("DecisionTaskCompleted", 12), ("TimerStarted", 8), ("StartChildWorkflowExecutionInitiated", 16),
                  ("SignalExternalWorkflowExecutionInitiated", 12), ("DecisionTaskStarted", 4),
                  ("ActivityTaskStarted", 4), ("DecisionTaskTimedOut", 4), ("ChildWorkflowExecutionStarted", 4),
                  ("WorkflowExecutionContinuedAsNew", 4), ("UpsertWorkflowSearchAttributes", 8)):
    A_TYPE[abi.EV[_name]] = _b
def encoded_event_bytes(tf) -> int:
    """Bytes of the packed input the fast kernel must read for these events (type_flags
    column `tf`, padding cells excluded): the 4-B type word, event_id / version unless the
    packer's delta bits imply them (CDR_SEF_ID_NEXT / VER_SAME), the operand columns the
    type's need bits name, and the arena record of WorkflowExecutionStarted /
    ActivityTaskScheduled.  The canonical SURVEY §8(d) price (48 + A[type]) assumes every
    core column is read; this is what the encoding leaves to read."""
    tf = np.asarray(tf)
    ty = tf & 0xFF
    real = ty < abi.EV["UpsertWorkflowSearchAttributes"] + 1
    b = np.full(tf.shape, 4, np.int64)
    b += np.where(tf & abi.SEF_ID_NEXT, 0, 8) + np.where(tf & abi.SEF_VER_SAME, 0, 8)
    for bit, w in ((1 << 16, 8), (1 << 17, 8), (1 << 18, 8), (1 << 19, 4), (1 << 20, 4)):  # CDR_SEF_NEED_*
        b += np.where(tf & bit, w, 0)
    b += np.where(ty == abi.EV["WorkflowExecutionStarted"], C.sizeof(abi.AttrStarted), 0)
    b += np.where(ty == abi.EV["ActivityTaskScheduled"], C.sizeof(abi.AttrATSched), 0)
    return int(b[real].sum())


ROW_BYTES = {"n_activity": 128, "n_timer": 32, "n_child": 48, "n_cancel": 24, "n_signal": 40}
RESULT_DTYPE = np.dtype([("code", "<i4"), ("flags", "<u4"), ("fid", "<i8"), ("fix", "<i8"),
                         ("n_activity", "<u4"), ("n_timer", "<u4"), ("n_child", "<u4"), ("n_cancel", "<u4"),
                         ("n_signal", "<u4"), ("n_vh", "<u4"), ("n_rp", "<u4"), ("n_sa", "<u4")])


class DeviceBatch:
    """Synthetic batch generated straight into the sliced layout, uploaded to HBM."""

    def __init__(self, torch, config, index_map, seed, target_len=0, plan_mode=abi.PLAN_WAVE | abi.PLAN_PAR, ctx_for_cls=None,
                 cls="host", long_stride=0, tasks=False):
        """cls: where the register-table slices' class-sorted blocks (replay_cls.inc) come
        from — "host": the packer emits them beside the slab (cdr_plan_cls / cdr_pack_cls,
        host packing time `cls_pack_s`, uploaded with the slab); "device": built on the
        device after the upload (cdr_cls_plan_async / cdr_cls_pack_async on ctx_for_cls,
        `cls_s`); None: no blocks (k_replay_reg alone).  tasks: also the stateBuilder's
        transfer / timer task lists (cdr_out.transfer / timer_tasks / n_tasks, sized by the
        synthetic plan's task capacities)."""
        if cls not in ("host", "device", None):
            raise ValueError(f"cls={cls!r}")
        if cls == "device" and not ctx_for_cls:
            raise ValueError("cls='device' needs ctx_for_cls")
        L = abi.lib()
        self.torch = torch
        self.index_map = index_map
        p = abi.CdrSynthParams(config=config, n_wfs=len(index_map), seed=seed, target_len=target_len, max_len=0,
                               error_rate=0.0, builder=-1, rebuild=0, index_map=index_map.ctypes.data,
                               plan_mode=plan_mode, long_stride=long_stride)
        self.params = p
        t0 = time.perf_counter()
        info = abi.CdrSynthPlanInfo()
        assert L.cdr_synth_sliced_plan(C.byref(p), C.byref(info)) == 0
        self.info = info
        self.h_slab = np.empty(info.n_rows * 64 * abi.EL_BYTES, np.uint8)
        self.h_lane = np.empty(info.n_slices * 64, np.int32)
        self.h_slen = np.empty(info.n_slices, np.uint32)
        self.h_row0 = np.empty(info.n_slices, np.uint64)
        self.h_sc_off = np.zeros(info.n_slices, np.uint64)
        self.h_sc_act = np.zeros(info.n_slices, np.uint32)
        self.h_sc_tim = np.zeros(info.n_slices, np.uint32)
        self.h_sflags = np.zeros(info.n_slices, np.uint32)
        self.h_arena = np.empty(max(1, info.arena_words), np.uint64)
        self.h_wfs = (abi.CdrWfDesc * info.n_entries)()
        self.h_caps = (abi.CdrWfCaps * info.n_entries)()
        self.h_kvs = np.zeros(max(1, info.n_kvs) * 2, np.uint32)
        self.h_rps = (abi.CdrResetPoint * max(1, info.n_rps))()
        s = abi.CdrSlices(n_slices=info.n_slices, n_rows=info.n_rows, arena_words=info.arena_words)
        s.slice_row0, s.slice_len, s.lane_wf = self.h_row0.ctypes.data, self.h_slen.ctypes.data, \
            self.h_lane.ctypes.data
        s.slab = self.h_slab.ctypes.data
        s.arena = self.h_arena.ctypes.data
        s.slice_scratch_off, s.slice_act_slots, s.slice_tim_slots = (
            self.h_sc_off.ctypes.data, self.h_sc_act.ctypes.data, self.h_sc_tim.ctypes.data)
        s.slice_flags = self.h_sflags.ctypes.data
        meta = abi.CdrBatch()
        threads = min(32, os.cpu_count() or 8)
        rc = L.cdr_synth_sliced_fill(C.byref(p), C.byref(s), self.h_wfs, self.h_caps, self.h_kvs.ctypes.data,
                                     self.h_rps, C.byref(meta), threads)
        assert rc == 0, rc
        self.meta = meta
        self.pack_s = time.perf_counter() - t0
        # ---- class-sorted blocks from the host packer (a second copy of the register-table
        # slices' events, regrouped per lane by entity class)
        self.cls_pack_s = 0.0
        h_cls = None
        n_cls_slices = int(((self.h_sflags & abi.CLS_SLICES) != 0).sum())
        if cls == "host" and n_cls_slices:
            t0 = time.perf_counter()
            h_cls_rows = np.zeros(max(1, info.n_slices * 4), np.uint32)
            h_cls_row0 = np.zeros(info.n_slices + 1, np.uint64)
            rc = L.cdr_plan_cls(C.byref(s), C.cast(self.h_wfs, C.c_void_p), h_cls_rows.ctypes.data,
                                h_cls_row0.ctypes.data)
            assert rc == 0, rc
            h_cls = np.empty(max(8, int(h_cls_row0[-1]) * abi.ROW_BYTES), np.uint8)
            rc = L.cdr_pack_cls(C.byref(s), C.cast(self.h_wfs, C.c_void_p), h_cls_rows.ctypes.data,
                                h_cls_row0.ctypes.data, h_cls.ctypes.data, threads)
            assert rc == 0, rc
            self.cls_pack_s = time.perf_counter() - t0
        # ---- upload (H2D timed separately)
        dev = torch.device("cuda", torch.cuda.current_device())
        t0 = time.perf_counter()
        self.keep = []

        def up(a):
            t = torch.from_numpy(np.ascontiguousarray(a).view(np.uint8)).to(dev)
            self.keep.append(t)
            return t.data_ptr()

        def up_ct(a):
            return up(np.frombuffer(a, np.uint8))

        db = abi.CdrDevBatch()
        db.ev.n_slices, db.ev.n_rows, db.ev.arena_words = info.n_slices, info.n_rows, info.arena_words
        db.ev.slice_row0, db.ev.slice_len, db.ev.lane_wf = up(self.h_row0), up(self.h_slen), up(self.h_lane)
        db.ev.slab = up(self.h_slab)
        db.ev.arena = up(self.h_arena)
        db.ev.slice_scratch_off = up(self.h_sc_off)
        db.ev.slice_act_slots = up(self.h_sc_act)
        db.ev.slice_tim_slots = up(self.h_sc_tim)
        db.ev.slice_flags = up(self.h_sflags)
        L.cdr_plan_scratch(self.h_caps, self.h_lane.ctypes.data, info.n_slices, None, None, None, None,
                           C.byref(sc_words := C.c_uint64()), None)
        self.scratch_t = torch.zeros(max(8, sc_words.value * 8), dtype=torch.uint8, device=dev)
        db.scratch = self.scratch_t.data_ptr()
        db.wfs, db.caps = up_ct(self.h_wfs), up_ct(self.h_caps)
        db.kvs, db.rps = up(self.h_kvs), up_ct(self.h_rps)
        db.n_wfs = info.n_entries
        db.max_act_slots = int(self.h_sc_act.max()) if len(self.h_sc_act) else 0
        db.max_tim_slots = int(self.h_sc_tim.max()) if len(self.h_sc_tim) else 0
        self.n_fast = int(((self.h_sflags & abi.SLICE_FAST) != 0).sum())
        self.n_wave = int(((self.h_sflags & abi.SLICE_WAVE) != 0).sum())
        self.n_reg = int(((self.h_sflags & abi.SLICE_REG) != 0).sum())
        db.n_fast_slices = self.n_fast
        db.n_wave_slices = self.n_wave
        db.n_reg_slices = self.n_reg
        self.n_reg2 = int(((self.h_sflags & abi.SLICE_REG2) != 0).sum())
        db.n_reg2_slices = self.n_reg2
        self.n_reg0 = int(((self.h_sflags & abi.SLICE_REG0) != 0).sum())
        db.n_reg0_slices = self.n_reg0
        self.n_par = int(((self.h_sflags & abi.SLICE_PAR) != 0).sum())
        db.n_par_slices = self.n_par
        L.cdr_plan_class_ranges(self.h_sflags.ctypes.data, len(self.h_sflags), db.class_lo, db.class_hi)
        db.empty_uuid = meta.empty_uuid
        db.cluster = meta.cluster
        db.now_ns = meta.now_ns
        db.uuid_seed = meta.uuid_seed
        self.db = db
        self.cls_s = 0.0
        self.cls_rows = 0
        self.cls_where = None
        self.cls_bytes = 0
        if h_cls is not None:
            db.cls_rows, db.cls_row0, db.cls_slab = up(h_cls_rows), up(h_cls_row0), up(h_cls)
            self.cls_dev = tuple(self.keep[-3:])  # (rows, row0, block) device tensors
            self.cls_rows = int(h_cls_row0[-1])
            self.cls_where = "host"
            self.cls_bytes = h_cls.nbytes
            del h_cls  # the device copy is the one replayed
        elif cls == "device" and n_cls_slices:
            self.build_cls(ctx_for_cls)
            self.cls_where = "device"
        tot = info.totals
        out = abi.CdrOut()
        sizes = {"result": info.n_entries * C.sizeof(abi.CdrWfResult),
                 "exec": info.n_entries * C.sizeof(abi.CdrExecInfo),
                 "repl": info.n_entries * C.sizeof(abi.CdrReplState),
                 "vh": tot.vh * C.sizeof(abi.CdrVHItem), "act": tot.act * C.sizeof(abi.CdrActivityInfo),
                 "timer": tot.timer * C.sizeof(abi.CdrTimerInfo), "child": tot.child * C.sizeof(abi.CdrChildInfo),
                 "cancel": tot.cancel * C.sizeof(abi.CdrCancelInfo),
                 "signal": tot.signal * C.sizeof(abi.CdrSignalInfo),
                 "rp": tot.rp * C.sizeof(abi.CdrResetPoint), "sa": tot.sa * C.sizeof(abi.CdrKV)}
        if tasks:
            sizes.update({"transfer": tot.xfer * C.sizeof(abi.CdrTask), "timer_tasks": tot.ttask * C.sizeof(abi.CdrTask),
                          "n_tasks": 2 * info.n_entries * 4})
            db.task_rows = tot.xfer + tot.ttask
        self.out_bytes = sum(sizes.values())
        self.out_t = {}
        for k, nb in sizes.items():
            t = torch.zeros(max(8, nb), dtype=torch.uint8, device=dev)
            self.out_t[k] = t
            setattr(out, k, t.data_ptr())
        self.out = out
        torch.cuda.synchronize()
        self.h2d_s = time.perf_counter() - t0
        self.in_bytes = self.h_slab.nbytes + self.h_arena.nbytes + self.cls_bytes  # uploaded
        tf = abi.slab_columns(self.h_slab, self.h_row0, self.h_slen, ("type_flags",))["type_flags"]
        types = tf & 0xFF
        self.type_counts = np.bincount(types, minlength=256)
        self.encoded_event_bytes = encoded_event_bytes(tf)
        del tf
        self.n_events = int(self.type_counts[:abi.EV["UpsertWorkflowSearchAttributes"] + 1].sum())

    def build_cls(self, ctx):
        """Class-sorted blocks of the register-table slices (cdr_cls_plan_async +
        cdr_cls_pack_async, replay_cls.inc): a packing step, done once per batch and timed
        apart from the replay (cls_s)."""
        torch, L, db = self.torch, abi.lib(), self.db
        ns = self.info.n_slices
        stream = torch.cuda.current_stream().cuda_stream
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rows_t = torch.zeros(max(1, ns * 4) * 4, dtype=torch.uint8, device="cuda")
        row0_t = torch.zeros((ns + 1) * 8, dtype=torch.uint8, device="cuda")
        rc = L.cdr_cls_plan_async(ctx, C.byref(db), C.c_void_p(rows_t.data_ptr()), C.c_void_p(row0_t.data_ptr()),
                                  C.c_void_p(stream))
        if rc:
            raise RuntimeError(f"cdr_cls_plan_async rc={rc}")
        total = int(row0_t.view(torch.int64)[ns].item())
        slab_t = torch.empty(max(8, total * 64 * abi.EL_BYTES), dtype=torch.uint8, device="cuda")
        db.cls_slab, db.cls_row0, db.cls_rows = slab_t.data_ptr(), row0_t.data_ptr(), rows_t.data_ptr()
        rc = L.cdr_cls_pack_async(ctx, C.byref(db), C.c_void_p(stream))
        if rc:
            raise RuntimeError(f"cdr_cls_pack_async rc={rc}")
        torch.cuda.synchronize()
        self.cls_s = time.perf_counter() - t0
        self.cls_rows = total
        self.keep += [rows_t, row0_t, slab_t]
        self.cls_dev = (rows_t, row0_t, slab_t)

    def builders(self) -> np.ndarray:
        """cdr_wf_desc.builder of every entry."""
        raw = np.frombuffer(self.h_wfs, dtype=np.uint8).reshape(len(self.h_wfs), -1)
        boff = abi.CdrWfDesc.builder.offset
        return raw[:, boff:boff + 4].copy().view(np.uint32)[:, 0]

    def digests(self, ctx, stream) -> tuple:
        """(per-entry output digests as uint64[n_entries], their wrapping sum) of the
        last replay, through cdr_entry_digests_async (k_digest) on `stream`."""
        torch = self.torch
        n = self.info.n_entries
        per = torch.zeros(max(1, n), dtype=torch.int64, device="cuda")
        tot = torch.zeros(1, dtype=torch.int64, device="cuda")
        rc = abi.lib().cdr_entry_digests_async(ctx, C.byref(self.db), C.byref(self.out), C.c_void_p(per.data_ptr()),
                                               C.c_void_p(tot.data_ptr()), C.c_void_p(stream))
        if rc:
            raise RuntimeError(f"cdr_entry_digests_async rc={rc}")
        torch.cuda.synchronize()
        return per[:n].cpu().numpy().view(np.uint64).copy(), int(tot.item()) & 0xFFFFFFFFFFFFFFFF

    def results(self):
        n = self.info.n_entries
        raw = self.out_t["result"][: n * C.sizeof(abi.CdrWfResult)].cpu().numpy().copy()
        return (abi.CdrWfResult * n).from_buffer(raw)

    def task_counts(self):
        """(transfer, timer) tasks emitted by the last replay (cdr_out.n_tasks, 2 per entry)."""
        if "n_tasks" not in self.out_t:
            return 0, 0
        n = self.out_t["n_tasks"][: 2 * self.info.n_entries * 4].view(self.torch.int32).view(-1, 2).to(self.torch.int64)
        t = n.sum(0).tolist()
        return int(t[0]), int(t[1])

    def algorithmic_bytes(self, res):
        ev_bytes = int((self.type_counts[:42] * (48 + A_TYPE[:42])).sum())
        n_ok, vh, rows, repl = 0, 0, 0, 0
        arr = np.frombuffer(res, dtype=RESULT_DTYPE)
        ok = arr["code"] == 0
        n_ok = int(ok.sum())
        vh = int(arr["n_vh"][ok].sum())
        for f, b in ROW_BYTES.items():
            rows += int(arr[f][ok].sum()) * b
        bld = self.builders()
        repl = int(((bld == abi.BUILDER_2DC) & ok).sum()) * 32
        wf_bytes = len(arr) * (256 + 8) + 16 * vh + repl
        return ev_bytes + wf_bytes + rows, n_ok, ev_bytes, wf_bytes, rows

    def encoded_bytes(self, res):
        """encoded_event_bytes + the same per-workflow and pending-row output bytes as
        algorithmic_bytes: the bytes one fast-kernel launch cannot avoid moving."""
        _, _, _, wf_bytes, rows = self.algorithmic_bytes(res)
        return self.encoded_event_bytes + wf_bytes + rows
