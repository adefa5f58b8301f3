#!/usr/bin/env python3
"""Throughput of the on-device ingest (cdr_ingest_decode + cdr_ingest_plan) against the
host path (cdr_plan_caps + cdr_pack_slices + H2D) on the same synthetic population,
blobs already resident in HBM for the device path.
usage: python tools/ingest_bench.py [--config 2] [--wfs 100000] [--reps 3]"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from cadence_amd import abi, engine, ingest, ndc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--wfs", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cls", action="store_true",
                    help="the plan also builds the class-sorted blocks on the device (CDR_CLS_BUILD): class kernels replay")
    ap.add_argument("--par", action="store_true", help="plan with CDR_PLAN_PAR (long histories on PAR slices)")
    args = ap.parse_args()
    L = abi.lib()
    hip = engine._hip()
    eng = engine.Engine(0)
    if args.cls:
        L.cdr_set_cls_path(eng.ctx, abi.CLS_BUILD)
    pmode = abi.PLAN_WAVE | (abi.PLAN_PAR if args.par else 0)
    b = engine.synth_batch(args.config, args.wfs, seed=0x5EED0000 + args.config)
    n_ev = len(b.events)
    enc = ingest.encode_batch(b, threads=16)
    sb, so = ingest._table(enc.seeds)
    dm = np.array(enc.domain_map, np.uint32).reshape(-1) if enc.domain_map else np.zeros(2, np.uint32)
    ptrs = []

    def up(a):
        a = np.ascontiguousarray(a)
        p = C.c_void_p()
        assert hip.hipMalloc(C.byref(p), C.c_size_t(max(8, a.nbytes))) == 0
        ptrs.append(p)
        assert hip.hipMemcpy(p, a.ctypes.data, C.c_size_t(a.nbytes), 1) == 0
        return p.value
    t0 = time.perf_counter()
    inp = abi.CdrIngestIn()
    inp.blob_bytes, inp.blob_off, inp.entry_blob0 = up(enc.blob_bytes), up(enc.blob_off), up(enc.entry_blob0)
    h2d_s = time.perf_counter() - t0
    inp.seed_bytes, inp.seed_off, inp.domain_map = up(sb), up(so), up(dm)
    inp.n_blobs, inp.n_entries = len(enc.blob_off) - 1, len(enc.entry_blob0) - 1
    inp.n_seeds, inp.n_domains = len(enc.seeds), len(enc.domain_map)
    meta = None
    dec_t, plan_t = [], []
    for rep in range(args.reps + 1):
        out = abi.CdrIngestOut()
        t0 = time.perf_counter()
        assert L.cdr_ingest_decode(eng.ctx, C.byref(inp), C.byref(out), None) == 0
        t1 = time.perf_counter()
        if meta is None:  # host entries (strings re-pointed at the seeds)
            wfs = (abi.CdrWfDesc * b.n_wfs)()
            C.memmove(wfs, b.wfs, C.sizeof(wfs))
            for w in range(b.n_wfs):
                for f in ("domain_id", "workflow_id", "run_id", "request_id"):
                    setattr(wfs[w], f, enc.seed_of.get(getattr(wfs[w], f), 0))
            mb = abi.CdrBatch()
            mb.wfs = C.cast(wfs, C.POINTER(abi.CdrWfDesc))
            mb.n_wfs = b.n_wfs
            mb.empty_uuid = 1
            mb.cluster, mb.now_ns, mb.uuid_seed = b.cluster, b.now_ns, b.uuid_seed
            meta = (mb, wfs)
        caps = (abi.CdrWfCaps * b.n_wfs)()
        tot = abi.CdrTotals()
        db = abi.CdrDevBatch()
        t2 = time.perf_counter()
        assert L.cdr_ingest_plan(eng.ctx, C.byref(out), C.byref(meta[0]), pmode, C.byref(db), caps,
                                 C.byref(tot), None) == 0
        t3 = time.perf_counter()
        if rep:  # the first round grows the workspace
            dec_t.append(t1 - t0)
            plan_t.append(t3 - t2)
    # end to end: the planned device batch replayed (decode + plan + pack + replay); the
    # output buffers are allocated once (sized by the plan's totals), outside the timing
    dev = ndc._Dev()
    o = ndc.alloc_out(dev, b.n_wfs, tot)
    rep_t = []
    for rep in range(args.reps + 1):
        assert hip.hipDeviceSynchronize() == 0
        t0 = time.perf_counter()
        assert L.cdr_replay_sliced_async(eng.ctx, C.byref(db), C.byref(o), None) == 0
        assert hip.hipDeviceSynchronize() == 0
        if rep:
            rep_t.append(time.perf_counter() - t0)
    res = (abi.CdrWfResult * b.n_wfs)()
    dev.down(res, o.result)
    n_ok = int(sum(1 for w in range(b.n_wfs) if res[w].code == 0))
    dev.close()
    # the host path on the same batch: cdr_plan_caps + slices + cdr_pack_slices (+ H2D of the slab)
    t0 = time.perf_counter()
    pl = engine.plan(b)
    ns, rows, nw = C.c_uint32(), C.c_uint64(), C.c_uint32()
    L.cdr_plan_slices_ex(b.wfs, pl.caps, b.n_wfs, abi.PLAN_WAVE, None, None, None, None, C.byref(ns),
                         C.byref(rows), C.byref(nw))
    lane = np.zeros(ns.value * 64, np.int32)
    slen = np.zeros(ns.value, np.uint32)
    row0 = np.zeros(ns.value, np.uint64)
    fl = np.zeros(ns.value, np.uint32)
    L.cdr_plan_slices_ex(b.wfs, pl.caps, b.n_wfs, abi.PLAN_WAVE, lane.ctypes.data, slen.ctypes.data,
                         row0.ctypes.data, fl.ctypes.data, C.byref(ns), C.byref(rows), C.byref(nw))
    aw = L.cdr_plan_arena_words(C.byref(b.cstruct()))
    slab = np.zeros(int(rows.value) * 64 * abi.EL_BYTES, np.uint8)
    arena = np.zeros(max(1, aw), np.uint64)
    s_ = abi.CdrSlices(n_slices=ns.value, n_rows=rows.value, arena_words=aw)
    s_.slice_row0, s_.slice_len, s_.lane_wf = row0.ctypes.data, slen.ctypes.data, lane.ctypes.data
    s_.slab, s_.arena, s_.slice_flags = slab.ctypes.data, arena.ctypes.data, fl.ctypes.data
    assert L.cdr_pack_slices(C.byref(b.cstruct()), C.byref(s_), 16) == 0
    host_pack_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    up(slab)
    host_h2d_s = time.perf_counter() - t0
    for p in ptrs:
        hip.hipFree(p)
    dec_s, plan_s, rep_s = float(np.median(dec_t)), float(np.median(plan_t)), float(np.median(rep_t))
    print(json.dumps({
        "config": args.config, "workflows": args.wfs, "events": n_ev, "blobs": int(inp.n_blobs),
        "class_blocks": bool(args.cls), "plan_par": bool(args.par),
        "blob_bytes": int(enc.blob_bytes.nbytes), "blob_h2d_s": h2d_s,
        "device_decode_s": dec_s, "device_plan_pack_s": plan_s,
        "device_events_per_s": n_ev / (dec_s + plan_s), "decode_gbs": enc.blob_bytes.nbytes / dec_s / 1e9,
        "device_replay_s": rep_s, "device_e2e_events_per_s": n_ev / (dec_s + plan_s + rep_s),
        "replay_ok_workflows": n_ok,
        "host_plan_pack_s": host_pack_s, "host_slab_h2d_s": host_h2d_s,
        "host_events_per_s": n_ev / (host_pack_s + host_h2d_s),
        "note": "device: blobs resident in HBM, decode + caps/plan/pack timed wall-clock incl. its host syncs; "
                "e2e adds the replay of the planned batch (cdr_replay_sliced_async, wall-clock); "
                "host: cdr_plan_caps + cdr_plan_slices_ex + cdr_pack_slices(16 threads) + slab H2D from cdr_event records"}))


if __name__ == "__main__":
    main()
