"""Entries the class kernels hand on (CLS_RETRY) on a full-size synthetic batch: the class
kernels alone (cdr_set_cls_path CLS_ALONE, no k_replay_reg pass), counted per slice class,
with the type histogram of the handed-on entries' histories and the first few entries'
event types.  usage: python tools/cls_handon.py [--config 3] [--wfs N] [--lib path]"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cadence_amd import abi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=3)
ap.add_argument("--wfs", type=int, default=1_000_000)
ap.add_argument("--lib", default=None)
ap.add_argument("--show", type=int, default=3)
args = ap.parse_args()
import torch  # noqa: E402
from cadence_amd.synth import DeviceBatch, RESULT_DTYPE  # noqa: E402
torch.cuda.init()
idx = np.arange(args.wfs, dtype=np.uint32)
L = abi.load(args.lib) if args.lib else abi.lib()
db = DeviceBatch(torch, args.config, idx, 0x5EED0000 + args.config)
ctx = L.cdr_create(0, None)
assert L.cdr_set_cls_path(ctx, abi.CLS_ALONE) >= 0
stream = torch.cuda.current_stream().cuda_stream
for _ in range(2):
    assert L.cdr_replay_sliced_async(ctx, C.byref(db.db), C.byref(db.out), C.c_void_p(stream)) == 0
torch.cuda.synchronize()
res = np.frombuffer(db.results(), dtype=RESULT_DTYPE)
lane = db.h_lane.reshape(-1, 64)
names = {abi.SLICE_REG0: "REG0", abi.SLICE_REG: "REG", abi.SLICE_REG2: "REG2", abi.SLICE_PAR: "PAR"}
out = {"config": args.config, "wfs": args.wfs, "per_class": {}}
bad = []
for s in range(len(db.h_sflags)):
    f = int(db.h_sflags[s])
    nm = next((v for k, v in names.items() if f & k), None)
    if nm is None:
        continue
    ws = [int(w) for w in lane[s] if w >= 0]
    r = [w for w in ws if res["code"][w] == abi.CLS_RETRY]
    d = out["per_class"].setdefault(nm, {"slices": 0, "entries": 0, "handed_on": 0, "slices_with": 0})
    d["slices"] += 1
    d["entries"] += len(ws)
    d["handed_on"] += len(r)
    d["slices_with"] += 1 if r else 0
    bad += [(nm, s, w, int(res["fix"][w])) for w in r]
cols = abi.slab_columns(db.h_slab, db.h_row0, db.h_slen, ("type_flags",))["type_flags"] & 0xFF
out["examples"] = []
for nm, s, w, fix in bad[:args.show]:
    l = list(lane[s]).index(w)
    n = int(db.h_wfs[w].ev_len) if hasattr(db, "h_wfs") else 0
    t = [int(cols[(int(db.h_row0[s]) + k) * 64 + l]) for k in range(min(n, int(db.h_slen[s])))]
    out["examples"].append({"class": nm, "slice": s, "wf": w, "fail_index": fix, "len": n,
                            "types": [abi.EVENT_TYPES[x] if x < len(abi.EVENT_TYPES) else x for x in t]})
print(json.dumps(out))
