"""Per-wave loop times of the PAR slices (variant build with -DCDR_PAR_PROF: the result's
fail_event_id holds the P+T, W, A and X waves' times to their final barrier, us) on a
full-size synthetic batch, with the slices' class rows: which loop sets the PAR kernel's
critical path.  usage: python tools/par_prof.py variants/libcdr_prof.so --config 4"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cadence_amd import abi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("lib")
ap.add_argument("--config", type=int, default=4)
ap.add_argument("--wfs", type=int, default=1_000_000)
ap.add_argument("--top", type=int, default=8)
ap.add_argument("--alone", action="store_true", help="replay only the PAR slices' histories")
ap.add_argument("--long-stride", type=int, default=0, help="bench.py --long-stride (histories at the count limit)")
args = ap.parse_args()
import torch  # noqa: E402
from cadence_amd.synth import DeviceBatch, RESULT_DTYPE  # noqa: E402
torch.cuda.init()
idx = np.arange(args.wfs, dtype=np.uint32)
bctx = abi.lib().cdr_create(0, None)
db = DeviceBatch(torch, args.config, idx, 0x5EED0000 + args.config, ctx_for_cls=bctx, long_stride=args.long_stride)
Lv = abi.load(args.lib)
ctx = Lv.cdr_create(0, None)
stream = torch.cuda.current_stream().cuda_stream
for _ in range(3):
    Lv.cdr_replay_sliced_async(ctx, C.byref(db.db), C.byref(db.out), C.c_void_p(stream))
torch.cuda.synchronize()
res = np.frombuffer(db.results(), dtype=RESULT_DTYPE)
rows = db.cls_dev[0].view(torch.int32).cpu().numpy()[:db.info.n_slices * 4].reshape(-1, 4) if hasattr(db, "cls_dev") else None
lane = db.h_lane.reshape(-1, 64)
par = np.nonzero(db.h_sflags & abi.SLICE_PAR)[0]
out = []
for s in par:
    ws = [w for w in lane[s] if 0 <= w < len(res)]
    if not ws:
        continue
    f = int(res["fid"][ws[0]])
    t = [(f >> (16 * j)) & 0xFFFF for j in range(4)]
    out.append({"slice": int(s), "len": int(db.h_slen[s]), "n": len(ws), "us_PT_W_A_X": t,
                "start_us": int(res["fix"][ws[0]]) & 0xFFFFFFFF,
                "rows_WATX": rows[s].tolist() if rows is not None else None})
t0 = min(d["start_us"] for d in out)
for d in out:
    d["start_us"] -= t0
    d["end_us"] = d["start_us"] + max(d["us_PT_W_A_X"])
starts = np.array([d["start_us"] for d in out])
out.sort(key=lambda d: -d["end_us"])
crit = np.array([d["us_PT_W_A_X"] for d in out])
print(json.dumps({"config": args.config, "par_slices": len(out), "max_us_PT_W_A_X": crit.max(0).tolist(),
                  "max_end_us": max(d["end_us"] for d in out),
                  "start_us_pctl_50_90_100": np.percentile(starts, [50, 90, 100]).tolist(),
                  "top": out[:args.top]}))
