"""Which entries the class kernel hands on (CLS_RETRY) on a full-size synthetic batch, and
why: the class kernel runs alone (cdr_set_cls_path mode 2) and the PAR variant writes the
checks that handed an entry on into the result's fail_index (W scan bits 0-7: bad type,
Started not first, Started checks, transient without NextEventID, DecisionTaskStarted
schedule ID, reset-point cap, continue-as-new, close transition; 0x100 P, 0x200 A, 0x400 T,
0x800 X).  usage: python tools/cls_retry.py --config 4"""
import argparse
import collections
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cadence_amd import abi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=4)
ap.add_argument("--wfs", type=int, default=1_000_000)
args = ap.parse_args()
import torch  # noqa: E402
from cadence_amd.synth import DeviceBatch, RESULT_DTYPE  # noqa: E402
torch.cuda.init()
L = abi.lib()
ctx = L.cdr_create(0, None)
db = DeviceBatch(torch, args.config, np.arange(args.wfs, dtype=np.uint32), 0x5EED0000 + args.config, ctx_for_cls=ctx)
L.cdr_set_cls_path(ctx, 2)
stream = torch.cuda.current_stream().cuda_stream
L.cdr_replay_sliced_async(ctx, C.byref(db.db), C.byref(db.out), C.c_void_p(stream))
torch.cuda.synchronize()
res = np.frombuffer(db.results(), dtype=RESULT_DTYPE)
rt = np.nonzero(res["code"] == abi.CLS_RETRY)[0]
lane = db.h_lane.reshape(-1, 64)
fl = db.h_sflags
slice_of = np.full(len(res), -1, np.int64)
for s in range(lane.shape[0]):
    for w in lane[s]:
        if 0 <= w < len(res):
            slice_of[w] = s
names = {abi.SLICE_PAR: "par", abi.SLICE_REG: "reg", abi.SLICE_REG0: "reg0", abi.SLICE_REG2: "reg2"}
out = {"config": args.config, "retried": int(len(rt)), "by_class": {}, "by_reason": {}}
cls = collections.Counter()
why = collections.Counter()
for w in rt:
    f = int(fl[slice_of[w]]) if slice_of[w] >= 0 else 0
    cls["+".join(n for b, n in names.items() if f & b) or "other"] += 1
    why[hex(int(res["fix"][w]))] += 1
out["by_class"] = dict(cls)
out["by_reason"] = dict(why.most_common(20))
print(json.dumps(out))
