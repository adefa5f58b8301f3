#!/usr/bin/env python3
"""Summarise `tools/gpu.sh calib` (gpurun_out/calib/) into profiles/<name>.json + .txt:
per calibration kernel, the known bytes it moves (tools/calib.hip, printed by the plain run)
against FETCH_SIZE / WRITE_SIZE (KiB) and the EA request counters of the rocprofv3 --pmc
passes, averaged over the kernel's dispatches.  The ratio counter_bytes / known_bytes is the
factor tools/traffic.py divides by for each access width.
usage: tools/calib.py [gpurun_out/calib] [profile name]"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "calib")
    name = sys.argv[2] if len(sys.argv) > 2 else "r5_pmc_calibration"
    known, gbs = {}, collections.defaultdict(list)
    for ln in open(os.path.join(d, "plain.log")):
        p = ln.split()
        if len(p) == 4 and p[0].startswith("k_cal"):
            known[p[0]] = float(p[1])
            gbs[p[0]].append(float(p[3]))
    agg = {}
    for sub in ("fetch", "write", "rdreq", "wrreq"):
        for k, cs in counters(os.path.join(d, sub)).items():
            for c, v in cs.items():
                agg.setdefault(k, {})[c] = sum(v) / len(v)
    rows, out = [], {}
    for k, b in known.items():
        # the CSV kernel names carry template arguments in their demangled form
        m = next((v for kk, v in agg.items() if kk.replace(" ", "") == k.replace(" ", "")), None)
        if m is None:
            m = next((v for kk, v in agg.items() if kk.split("<")[0] == k.split("<")[0] and
                      kk.replace(" ", "").endswith(k.split("<", 1)[-1].replace(" ", "")) if "<" in k), {})
        e = {"known_bytes": b, "gbs_best": max(gbs[k])}
        if "FETCH_SIZE" in m:
            e["fetch_size_bytes"] = m["FETCH_SIZE"] * 1024
            e["fetch_ratio"] = e["fetch_size_bytes"] / b
        if "WRITE_SIZE" in m:
            e["write_size_bytes"] = m["WRITE_SIZE"] * 1024
            e["write_ratio"] = e["write_size_bytes"] / b
        for c in ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum"):
            if c in m:
                e[c] = m[c]
                e[c + "_per_known_128B"] = m[c] / (b / 128)
        out[k] = e
        rows.append(f"{k:22s} known {b / 2**30:7.3f} GiB  {e['gbs_best']:7.0f} GB/s  "
                    f"FETCH/known {e.get('fetch_ratio', float('nan')):.3f}  WRITE/known {e.get('write_ratio', float('nan')):.3f}"
                    + "".join(f"  {c.replace('TCC_EA0_', '')}/128B {e[c + '_per_known_128B']:.3f}"
                              for c in ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_WRREQ_sum",
                                        "TCC_EA0_WRREQ_64B_sum") if c in e))
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    json.dump({"source": "tools/calib.hip under rocprofv3 --pmc (tools/gpu.sh calib)", "kernels": out},
              open(os.path.join(ROOT, "profiles", name + ".json"), "w"), indent=1)
    open(os.path.join(ROOT, "profiles", name + ".txt"), "w").write("\n".join(rows) + "\n")
    print("\n".join(rows))


if __name__ == "__main__":
    main()
