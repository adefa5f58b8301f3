"""Refresh on the bench's sliced synthetic batch (GPU): result-code histogram after
replay and after refresh, and for failing entries whether their slab event IDs ascend.
usage: python tools/refresh_check.py [config] [wfs]"""
import ctypes as C
import os
import sys
from collections import Counter

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from cadence_amd import abi  # noqa: E402


def codes(db):
    return Counter(int(r.code) for r in db.results())


def main():
    import torch
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    torch.cuda.set_device(0)
    L = abi.lib()
    ctx = L.cdr_create(0, None)
    idx = np.arange(n, dtype=np.uint32)
    db = bench.DeviceBatch(torch, cfg, idx, 0x5EED0002)
    stream = torch.cuda.current_stream().cuda_stream
    assert L.cdr_replay_sliced_async(ctx, C.byref(db.db), C.byref(db.out), C.c_void_p(stream)) == 0
    torch.cuda.synchronize()
    print("after replay ", codes(db))
    bench.refresh_measure(torch, L, ctx, db, stream, 1)
    res = db.results()
    print("after refresh", codes(db))
    cols = abi.slab_columns(db.h_slab, db.h_row0, db.h_slen, ("event_id",))
    lane = db.h_lane
    bad = [w for w in range(len(res)) if res[w].code != 0][:5]
    for w in bad:
        i = int(np.nonzero(lane == w)[0][0])
        s, l = divmod(i, 64)
        d = db.h_wfs[w]
        print(f"wf {w}: code {res[w].code} slice {s} lane {l} ev_len {d.ev_len} slice_len {db.h_slen[s]} "
              f"flags {db.h_sflags[s]:#x} counts act {res[w].n_activity} timer {res[w].n_timer} "
              f"child {res[w].n_child} cancel {res[w].n_cancel} signal {res[w].n_signal}")
        if not db.h_sflags[s] & abi.SLICE_WAVE:
            ids = cols["event_id"].reshape(-1, 64)[int(db.h_row0[s]):int(db.h_row0[s]) + int(d.ev_len), l]
            print("   ids ascending:", bool(np.all(np.diff(ids) > 0)), ids[:8])
    L.cdr_destroy(ctx)


if __name__ == "__main__":
    main()
