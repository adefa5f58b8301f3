#!/usr/bin/env python3
"""CPU baseline per configuration (BASELINE.md asks for one on each of C1-C5): the
oracle restatement (oracle/, "port") on the host's cores over a bounded sample of each
config, the same measurement bench.py's cpu_baseline leg makes for the bench config.
usage: python tools/cpu_baselines.py [--configs 1 2 3 4 5] [--wfs 20000] [--seconds 8] [--out FILE]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", type=int, nargs="+", default=[1, 2, 3, 4, 5])
    ap.add_argument("--wfs", type=int, default=20000)
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    rows = {}
    for c in args.configs:
        t0 = time.perf_counter()
        # C1 (configs[0]) is the reference's CPU case at its own size: 10k echo workflows
        n = args.wfs if c != 1 else 10000
        r = bench.cpu_baseline(c, n, 0x5EED0000 + c, min_seconds=args.seconds)
        r["wall_s"] = time.perf_counter() - t0
        rows[f"C{c}"] = r
        print(json.dumps({f"C{c}": r}), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"source": "tools/cpu_baselines.py", "host_cpus": os.cpu_count(),
                       "cores_used": bench.host_cores(), "configs": rows}, f, indent=1)


if __name__ == "__main__":
    main()
