#!/usr/bin/env python3
"""Where k_replay_cls's slab reads go, counted on the host (no GPU): the synthetic population
is packed exactly as bench.py packs it (cdr_synth_sliced_* + cdr_plan_cls / cdr_pack_cls), then
every load the lane-form loops issue is replayed at 128-B line granularity — the unit the
memory side fetches (tools/calib.hip: one TCC_EA0_RDREQ per 128 B, FETCH_SIZE x 2).  A line is
fetched once per (row, column, line) if any lane of its group loads it (8-B columns: 16 lanes
per line, 4-B columns: 32).  Prints per loop: rows, lines fetched, bytes, bytes per event.

usage: tools/cls_traffic.py [config] [workflows]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cadence_amd import abi  # noqa: E402

ROW = abi.ROW_BYTES
PAD = 0xFF  # CDR_EV_PAD
NEED = {"ts": 1 << 16, "key": 1 << 17, "aux": 1 << 18, "h": 1 << 19, "n": 1 << 20}
COLS8 = {"id": 0, "ver": 1, "ts": 2, "task": 3, "key": 4, "aux": 5}
COLS4 = {"tf": 6, "h": 7, "n": 8}


def col_off(c):
    return 64 * (8 * c if c <= 6 else 48 + 4 * (c - 6))


def lines(mask, width):
    """128-B lines fetched for one column of one row: mask = lanes that load (bool[64])."""
    g = 128 // width
    return int(mask.reshape(64 // g, g).any(axis=1).sum())


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    nw = int(sys.argv[2]) if len(sys.argv) > 2 else 50000
    L = abi.lib()
    idx = np.arange(nw, dtype=np.uint32)
    p = abi.CdrSynthParams(config=cfg, n_wfs=nw, seed=0x5EED0000 + cfg, target_len=0, max_len=0, error_rate=0.0,
                           builder=-1, rebuild=0, index_map=idx.ctypes.data, plan_mode=abi.PLAN_WAVE | abi.PLAN_PAR,
                           long_stride=0)
    info = abi.CdrSynthPlanInfo()
    assert L.cdr_synth_sliced_plan(C.byref(p), C.byref(info)) == 0
    slab = np.zeros(info.n_rows * ROW, np.uint8)
    lane = np.empty(info.n_slices * 64, np.int32)
    slen = np.empty(info.n_slices, np.uint32)
    row0 = np.empty(info.n_slices, np.uint64)
    scz = [np.zeros(info.n_slices, t) for t in (np.uint64, np.uint32, np.uint32)]
    sfl = np.zeros(info.n_slices, np.uint32)
    arena = np.empty(max(1, info.arena_words), np.uint64)
    wfs = (abi.CdrWfDesc * info.n_entries)()
    caps = (abi.CdrWfCaps * info.n_entries)()
    kvs = np.zeros(max(1, info.n_kvs) * 2, np.uint32)
    rps = (abi.CdrResetPoint * max(1, info.n_rps))()
    s = abi.CdrSlices(n_slices=info.n_slices, n_rows=info.n_rows, arena_words=info.arena_words)
    s.slice_row0, s.slice_len, s.lane_wf = row0.ctypes.data, slen.ctypes.data, lane.ctypes.data
    s.slab, s.arena = slab.ctypes.data, arena.ctypes.data
    s.slice_scratch_off, s.slice_act_slots, s.slice_tim_slots = (a.ctypes.data for a in scz)
    s.slice_flags = sfl.ctypes.data
    meta = abi.CdrBatch()
    assert L.cdr_synth_sliced_fill(C.byref(p), C.byref(s), wfs, caps, kvs.ctypes.data, rps, C.byref(meta), 8) == 0
    crows = np.zeros(info.n_slices * 4, np.uint32)
    crow0 = np.zeros(info.n_slices + 1, np.uint64)
    assert L.cdr_plan_cls(C.byref(s), C.cast(wfs, C.c_void_p), crows.ctypes.data, crow0.ctypes.data) == 0
    cls = np.zeros(max(8, int(crow0[-1]) * ROW), np.uint8)
    assert L.cdr_pack_cls(C.byref(s), C.cast(wfs, C.c_void_p), crows.ctypes.data, crow0.ctypes.data,
                          cls.ctypes.data, 8) == 0
    ev_len = np.array([wfs[w].ev_len for w in range(info.n_entries)], np.int64)
    slab = slab.reshape(-1, ROW)
    cls = cls.reshape(-1, ROW)

    def c32(blk, r, c):
        o = col_off(c)
        return blk[r, o:o + 256].view(np.uint32)

    tot = {k: 0 for k in ("P", "W", "A", "T", "X")}
    per_col = {}
    rows_n = {k: 0 for k in tot}
    n_events = 0
    cls_sl = np.nonzero((sfl & abi.CLS_SLICES) != 0)[0]
    par = (sfl & abi.SLICE_PAR) != 0
    for si in cls_sl:
        if par[si]:
            continue  # PAR slices read in scan form (not modelled here)
        lw = lane[si * 64:(si + 1) * 64]
        ln = np.where(lw >= 0, ev_len[np.maximum(lw, 0)], 0)
        n_events += int(ln.sum())
        r0 = int(row0[si])
        for k in range(int(slen[si])):
            valid = k < ln
            if not valid.any():
                break
            tf = c32(slab, r0 + k, 6)
            b = lines(valid, 4) * 128
            per_col["P.tf"] = per_col.get("P.tf", 0) + b
            bi = lines(valid & ((tf & abi.SEF_ID_NEXT) == 0), 8) * 128
            bv = lines(valid & ((tf & abi.SEF_VER_SAME) == 0), 8) * 128
            per_col["P.id"] = per_col.get("P.id", 0) + bi
            per_col["P.ver"] = per_col.get("P.ver", 0) + bv
            tot["P"] += b + bi + bv
            rows_n["P"] += 1
        c0 = int(crow0[si])
        off = 0
        for j, name in enumerate("WATX"):
            m = int(crows[si * 4 + j])
            for pp in range(m):
                r = c0 + off + pp
                tf = c32(cls, r, 6)
                ty = tf & 0xFF
                live = lw >= 0
                act = live & (ty != PAD)
                loads = {"tf": live, "task": act, "id": act & ((tf & (1 << 21)) == 0),
                         "ver": act & ((tf & (1 << 22)) == 0)}
                for nm, bit in NEED.items():
                    loads[nm] = act & ((tf & bit) != 0)
                for nm, msk in loads.items():
                    b = lines(msk, 4 if nm in COLS4 else 8) * 128
                    per_col[f"{name}.{nm}"] = per_col.get(f"{name}.{nm}", 0) + b
                    tot[name] += b
                rows_n[name] += 1
            off += m
    allb = sum(tot.values())
    print(f"config {cfg}, {nw} workflows, {n_events} events on lane class slices "
          f"({len(cls_sl) - int(par[cls_sl].sum())} slices)")
    for k, v in tot.items():
        print(f"{k}: rows {rows_n[k]:9d}  bytes {v / 1e6:10.1f} MB  {v / max(1, n_events):6.1f} B/event")
    print(f"all loops: {allb / 1e6:.1f} MB, {allb / max(1, n_events):.1f} B/event")
    for k, v in sorted(per_col.items(), key=lambda x: -x[1])[:20]:
        print(f"   {k:10s} {v / max(1, n_events):6.1f} B/event")


if __name__ == "__main__":
    main()
