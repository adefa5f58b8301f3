"""Host packer of the class-sorted blocks (cdr_plan_cls / cdr_pack_cls, host.cpp) vs a
numpy restatement of the layout cdr.h documents: per register-table lane, its W /
activity / timer / external events in four regions aligned across the slice, each in
history order, annotated with (history index, index within its call, event_id -
NextEventID at its call).  The regrouping is the per-event type switch of
stateBuilder.go:157-600 sorted by entity class.  CPU only."""
import ctypes as C

import numpy as np
import pytest

from cadence_amd import abi, engine

PAD = 0xFF
SEF_BATCH_FIRST = 1 << 8
ID_NEXT, VER_SAME = 1 << 21, 1 << 22


def _tb(*names):
    return sum(1 << abi.EV[n] for n in names)


A_T = _tb("ActivityTaskScheduled", "ActivityTaskStarted", "ActivityTaskCompleted", "ActivityTaskFailed",
          "ActivityTaskTimedOut", "ActivityTaskCanceled", "ActivityTaskCancelRequested")
T_T = _tb("TimerStarted", "TimerFired", "TimerCanceled")
X_T = _tb(*[n for n in abi.EV if "Workflow" in n and ("Child" in n or "External" in n)])
DROP_T = _tb("MarkerRecorded", "CancelTimerFailed", "RequestCancelActivityTaskFailed")
NEED_ID = _tb("WorkflowExecutionStarted", "DecisionTaskScheduled", "DecisionTaskStarted", "DecisionTaskTimedOut",
              "DecisionTaskFailed", "ActivityTaskScheduled", "TimerStarted", "StartChildWorkflowExecutionInitiated",
              "RequestCancelExternalWorkflowExecutionInitiated", "SignalExternalWorkflowExecutionInitiated")


def cls_of(t):
    if t >= 64:
        return 0
    b = 1 << t
    return 1 if b & A_T else 2 if b & T_T else 3 if b & X_T else 4 if b & DROP_T else 0


def _packed(cfg, n, seed, mode=abi.PLAN_WAVE | abi.PLAN_PAR):
    b = engine.synth_batch(cfg, n, seed=seed)
    pl = engine.plan(b)
    L = abi.lib()
    ns, rows, nw = C.c_uint32(), C.c_uint64(), C.c_uint32()
    L.cdr_plan_slices_ex(b.wfs, pl.caps, b.n_wfs, mode, None, None, None, None, C.byref(ns), C.byref(rows),
                         C.byref(nw))
    lane = np.zeros(ns.value * 64, np.int32)
    slen = np.zeros(ns.value, np.uint32)
    row0 = np.zeros(ns.value, np.uint64)
    flags = np.zeros(ns.value, np.uint32)
    L.cdr_plan_slices_ex(b.wfs, pl.caps, b.n_wfs, mode, lane.ctypes.data, slen.ctypes.data, row0.ctypes.data,
                         flags.ctypes.data, C.byref(ns), C.byref(rows), C.byref(nw))
    words = C.c_uint64()
    L.cdr_plan_scratch(pl.caps, lane.ctypes.data, ns.value, None, None, None, flags.ctypes.data, C.byref(words), None)
    aw = L.cdr_plan_arena_words(C.byref(b.cstruct()))
    slab = np.zeros(int(rows.value) * 64 * abi.EL_BYTES, np.uint8)
    arena = np.zeros(max(1, aw), np.uint64)
    s = abi.CdrSlices(n_slices=ns.value, n_rows=rows.value, arena_words=aw)
    s.slice_row0, s.slice_len, s.lane_wf = row0.ctypes.data, slen.ctypes.data, lane.ctypes.data
    s.slab, s.arena, s.slice_flags = slab.ctypes.data, arena.ctypes.data, flags.ctypes.data
    assert L.cdr_pack_slices(C.byref(b.cstruct()), C.byref(s), 2) == 0
    keep = (lane, slen, row0, flags, slab, arena)
    return b, s, keep


def _host_cls(b, s, threads=3):
    L = abi.lib()
    ns = s.n_slices
    rows = np.zeros(max(1, ns * 4), np.uint32)
    row0 = np.zeros(ns + 1, np.uint64)
    assert L.cdr_plan_cls(C.byref(s), C.cast(b.wfs, C.c_void_p), rows.ctypes.data, row0.ctypes.data) == 0
    blk = np.zeros(max(8, int(row0[-1]) * abi.ROW_BYTES), np.uint8)
    assert L.cdr_pack_cls(C.byref(s), C.cast(b.wfs, C.c_void_p), rows.ctypes.data, row0.ctypes.data,
                          blk.ctypes.data, threads) == 0
    return rows.reshape(-1, 4) if ns else rows[:0].reshape(0, 4), row0, blk


@pytest.mark.parametrize("cfg,n", [(3, 400), (4, 3000), (5, 300)])
def test_host_class_blocks_match_restatement(cfg, n):
    b, s, keep = _packed(cfg, n, seed=0x5EED0C00 + cfg)
    lane, slen, row0, flags, slab, _ = keep
    rows, crow0, blk = _host_cls(b, s)
    reg = (flags & abi.CLS_SLICES) != 0
    assert reg.any()
    assert (rows[~reg] == 0).all()
    src = abi.slab_columns(slab)
    dst = abi.slab_columns(blk)
    lane = lane.reshape(-1, 64)
    for sl in np.nonzero(reg)[0][:: max(1, int(reg.sum()) // 40)]:
        r0 = int(row0[sl])
        base = int(crow0[sl])
        M = rows[sl].tolist()
        off = np.concatenate([[0], np.cumsum(M)[:-1]])
        assert int(crow0[sl + 1]) - base == sum(M)
        cnt_max = [0, 0, 0, 0]
        for ln in range(64):
            w = int(lane[sl, ln])
            ev_len = int(b.wfs[w].ev_len) if w >= 0 else 0
            pos = [0, 0, 0, 0]
            x_next, prev_id, k0, wver, any_w = 1, 0, 0, 0, False
            for k in range(ev_len):
                e = (r0 + k) * 64 + ln
                tf = int(src["type_flags"][e])
                eid, ver = int(src["event_id"][e]), int(src["version"][e])
                bf = (tf & SEF_BATCH_FIRST) or k == 0
                if bf and k > 0:
                    x_next = prev_id + 1
                if bf:
                    k0 = k
                prev_id = eid
                t = tf & 0xFF
                c = cls_of(t)
                if c == 4:
                    continue
                d = ((base + int(off[c]) + pos[c]) * 64) + ln
                pos[c] += 1
                need = t < 64 and (1 << t) & NEED_ID
                same_v = c != 0 or (any_w and ver == wver)
                if c == 0:
                    wver, any_w = ver, True
                want_tf = (tf & ~(ID_NEXT | VER_SAME)) | (0 if need else ID_NEXT) | (VER_SAME if same_v else 0)
                assert int(dst["type_flags"][d]) == want_tf, (sl, ln, k)
                xd = eid - x_next if 0 <= eid - x_next < 0xFFFFFFFF else 0xFFFFFFFF
                ann = k | (((k - k0) & 0xFFF) << 20) | (xd << 32)
                assert int(dst["task_id"][d]) & 0xFFFFFFFFFFFFFFFF == ann
                for col in ("event_id", "version", "timestamp", "key", "aux", "h", "n"):
                    assert int(dst[col][d]) == int(src[col][e]), (col, sl, ln, k)
            for c in range(4):
                cnt_max[c] = max(cnt_max[c], pos[c])
                for p in range(pos[c], M[c]):  # padding
                    d = (base + int(off[c]) + p) * 64 + ln
                    assert int(dst["type_flags"][d]) == PAD | ID_NEXT | VER_SAME
        assert cnt_max == M  # each region is exactly as tall as its fullest lane


def test_host_class_blocks_reject_foreign_plan():
    """A row plan that does not belong to the slab (a region too short) is refused, not
    overrun."""
    b, s, keep = _packed(3, 200, seed=5)
    L = abi.lib()
    ns = s.n_slices
    rows = np.zeros(ns * 4, np.uint32)
    row0 = np.zeros(ns + 1, np.uint64)
    assert L.cdr_plan_cls(C.byref(s), C.cast(b.wfs, C.c_void_p), rows.ctypes.data, row0.ctypes.data) == 0
    sl = int(np.nonzero(rows.reshape(-1, 4)[:, 1])[0][0])
    rows[4 * sl + 1] -= 1
    rows[4 * sl + 0] += 1  # same total rows, a short activity region
    blk = np.zeros(int(row0[-1]) * abi.ROW_BYTES, np.uint8)
    assert L.cdr_pack_cls(C.byref(s), C.cast(b.wfs, C.c_void_p), rows.ctypes.data, row0.ctypes.data,
                          blk.ctypes.data, 2) == -1  # CDR_API_EINVAL
