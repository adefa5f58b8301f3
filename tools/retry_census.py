#!/usr/bin/env python3
"""Which entries k_replay_cls hands on to k_replay_reg (CLS_RETRY), per slice class: the
class kernels alone (cdr_set_cls_path CLS_ALONE) over a synthetic batch, then the handed-on
entries' history lengths and planner capacities.
usage: tools/retry_census.py [config] [workflows]"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cadence_amd import abi  # noqa: E402


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    nw = int(sys.argv[2]) if len(sys.argv) > 2 else 200000
    import torch
    from cadence_amd.synth import DeviceBatch
    torch.cuda.set_device(0)
    L = abi.lib()
    ctx = L.cdr_create(0, None)
    db = DeviceBatch(torch, cfg, np.arange(nw, dtype=np.uint32), 0x5EED0000 + cfg, ctx_for_cls=ctx)
    L.cdr_set_cls_path(ctx, abi.CLS_ALONE)
    stream = torch.cuda.current_stream().cuda_stream
    assert L.cdr_replay_sliced_async(ctx, C.byref(db.db), C.byref(db.out), C.c_void_p(stream)) == 0
    torch.cuda.synchronize()
    res = db.results()
    codes = np.array([r.code for r in res])
    lane = db.h_lane.reshape(-1, 64)
    out = {}
    for name, flag in (("reg0", abi.SLICE_REG0), ("reg", abi.SLICE_REG), ("reg2", abi.SLICE_REG2), ("par", abi.SLICE_PAR)):
        sl = np.nonzero(db.h_sflags & flag)[0]
        ws = lane[sl].ravel()
        ws = ws[(ws >= 0) & (ws < len(codes))]
        rt = ws[codes[ws] == abi.CLS_RETRY]
        caps = db.h_caps
        lens = np.array([int(db.h_wfs[w].ev_len) for w in rt[:2000]]) if len(rt) else np.array([0])
        out[name] = {"entries": int(len(ws)), "handed_on": int(len(rt)),
                     "handed_on_len_median": float(np.median(lens)),
                     "fail_index_sample": [int(res[w].fail_index) for w in rt[:8]],
                     "act_live_sample": [int(caps[w].act_live) for w in rt[:8]],
                     "rp_cap_sample": [int(caps[w].rp_cap) for w in rt[:8]],
                     "sa_cap_sample": [int(caps[w].sa_cap) for w in rt[:8]]}
    print(json.dumps(out, indent=1))
    L.cdr_destroy(ctx)


if __name__ == "__main__":
    main()
