#!/usr/bin/env python3
"""A/B timing of libcdr kernel variants on one device-resident batch (interleaved
rounds in one process, cdr_timing ring = HIP events on the launch stream).
usage: python tools/perf.py [--config 2] [--wfs 1000000] [--rounds 5] variants/libcdr_a.so ..."""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from cadence_amd import abi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--wfs", type=int, default=1_000_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--no-wave", action="store_true", help="plan divergent histories into lane slices")
    ap.add_argument("--wave-all", action="store_true", help="every divergent history on a wave slice")
    ap.add_argument("--no-reg", action="store_true", help="register-table slices on the general kernel")
    ap.add_argument("--no-long", action="store_true", help="long lane-capable histories stay in lane slices")
    ap.add_argument("--no-par", action="store_true", help="long register-table histories on wave slices, not PAR slices")
    ap.add_argument("--par-subset", type=int, default=0,
                    help="replay only the histories of the full batch's first N PAR slices (PAR kernel alone)")
    ap.add_argument("--tasks", action="store_true", help="with the stateBuilder task lists (bench.py --tasks's batch)")
    ap.add_argument("--tasks-no-cls", action="store_true", help="--tasks without class blocks (k_replay_reg<TASKS>)")
    ap.add_argument("--tasks-par", action="store_true", help="--tasks with bench.py's task plan (long histories on PAR slices, one each)")
    ap.add_argument("--ab-cls", action="store_true",
                    help="each lib twice: class-decomposed register slices (k_replay_cls) on, then off")
    args = ap.parse_args()
    import torch
    from cadence_amd.synth import DeviceBatch
    torch.cuda.set_device(0)
    idx = np.arange(args.wfs, dtype=np.uint32)
    bctx = abi.lib().cdr_create(0, None)
    if args.par_subset:
        full = DeviceBatch(torch, args.config, idx, 0x5EED0000 + args.config, cls=None)
        par = np.nonzero(full.h_sflags & abi.SLICE_PAR)[0][:args.par_subset]
        lanes = full.h_lane.reshape(-1, 64)[par].ravel()
        idx = np.sort(idx[lanes[(lanes >= 0) & (lanes < len(idx))]])
        del full
        torch.cuda.empty_cache()
    db = DeviceBatch(torch, args.config, idx, 0x5EED0000 + args.config,
                     plan_mode=0 if args.no_wave else abi.PLAN_WAVE | (abi.PLAN_WAVE_ALL if args.wave_all else 0)
                     | (abi.PLAN_NO_LONG if args.no_long else 0) | (0 if args.no_par else abi.PLAN_PAR),
                     ctx_for_cls=bctx) if not args.tasks else \
        DeviceBatch(torch, args.config, idx, 0x5EED0000 + args.config,
                    plan_mode=abi.PLAN_WAVE | abi.PLAN_PAR | abi.PLAN_PAR_SOLO if args.tasks_par else 0,
                    cls=None if args.tasks_no_cls else "host", tasks=True)
    print(json.dumps({"cls_pack_s": round(db.cls_pack_s, 4), "cls_rows": db.cls_rows, "rows": db.info.n_rows}),
          flush=True)
    stream = torch.cuda.current_stream().cuda_stream
    libs = [(p, abi.load(p)) for p in args.libs]
    if args.ab_cls:
        libs = [(p + tag, L) for p, L in libs for tag in ("", "#nocls")]
    ctxs = [L.cdr_create(0, None) for _, L in libs]
    for (p, L), c in zip(libs, ctxs):
        if p.endswith("#nocls"):
            L.cdr_set_cls_path(c, 0)
    if args.no_reg:
        for (_, L), c in zip(libs, ctxs):
            L.cdr_set_reg_path(c, 0)
    times = {p: [] for p, _ in libs}
    sums = {}
    for rnd in range(args.rounds):
        for (p, L), ctx in zip(libs, ctxs):
            L.cdr_replay_sliced_async(ctx, C.byref(db.db), C.byref(db.out), C.c_void_p(stream))
            L.cdr_timing_begin(ctx, args.reps)
            for _ in range(args.reps):
                L.cdr_replay_sliced_async(ctx, C.byref(db.db), C.byref(db.out), C.c_void_p(stream))
            ms = (C.c_float * args.reps)()
            n = C.c_uint32(args.reps)
            L.cdr_timing_read(ctx, ms, C.byref(n))
            times[p] += list(ms)[: n.value]
            if rnd == 0:
                cs = torch.zeros(1, dtype=torch.int64, device="cuda")
                L.cdr_checksum_async(ctx, C.byref(db.db), C.byref(db.out), C.c_void_p(cs.data_ptr()),
                                     C.c_void_p(stream))
                torch.cuda.synchronize()
                sums[p] = int(cs.item())
    base = None
    for p, _ in libs:
        t = np.array(times[p])
        med = float(np.median(t))
        base = base or med
        print(json.dumps({"lib": os.path.basename(p), "median_ms": round(med, 4), "min_ms": round(float(t.min()), 4),
                          "events_per_s": db.n_events / (med / 1e3), "rel": round(med / base, 4),
                          "checksum": sums[p] & 0xFFFFFFFFFFFFFFFF}), flush=True)
    if len(set(sums.values())) != 1:
        print("CHECKSUM MISMATCH between variants", file=sys.stderr)
        sys.exit(1)


if __name__ == "__main__":
    main()
