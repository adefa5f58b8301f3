"""Per-slice class-row counts (W, A, T, X) of a synthetic batch's register-table and PAR
slices, longest first: which loop sets a slice's critical path (GPU)."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cadence_amd import abi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=4)
ap.add_argument("--wfs", type=int, default=1_000_000)
ap.add_argument("--top", type=int, default=6)
args = ap.parse_args()
import torch  # noqa: E402
from cadence_amd.synth import DeviceBatch  # noqa: E402
torch.cuda.init()
idx = np.arange(args.wfs, dtype=np.uint32)
ctx = abi.lib().cdr_create(0, None)
db = DeviceBatch(torch, args.config, idx, 0x5EED0000 + args.config, ctx_for_cls=ctx, cls="device")
rows = db.cls_dev[0].view(torch.int32).cpu().numpy()[:db.info.n_slices * 4].reshape(-1, 4)
fl, sl = db.h_sflags, db.h_slen
out = {"config": args.config}
for name, bit in (("par", abi.SLICE_PAR), ("reg0", abi.SLICE_REG0), ("reg", abi.SLICE_REG), ("reg2", abi.SLICE_REG2)):
    s = np.nonzero(fl & bit)[0]
    if not len(s):
        continue
    tot = rows[s].sum(1)
    top = s[np.argsort(-tot, kind="stable")[:args.top]]
    out[name] = {"slices": int(len(s)), "events_rows": int(sl[s].sum()), "class_rows": rows[s].sum(0).tolist(),
                 "top": [[int(sl[t])] + rows[t].tolist() for t in top]}
print(json.dumps(out))
