#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc counter CSVs under a directory.
usage: tools/pmcsum.py <dir> [kernel-substring]"""
import collections
import csv
import glob
import os
import re
import sys

d = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(float)
nd = collections.defaultdict(set)
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if kern not in r["Kernel_Name"]:
            continue
        m = re.search(r"(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
        k = (m.group(1) if m else r["Kernel_Name"].split("(")[0], r["Counter_Name"])
        agg[k] += float(r["Counter_Value"])
        nd[k].add(r["Dispatch_Id"])
waves = {}
for (kn, c), v in sorted(agg.items()):
    a = v / len(nd[(kn, c)])
    if c == "SQ_WAVES":
        waves[kn] = a
    print(f"{kn[-40:]:40s} {c:22s} {a:.6g}")
for (kn, c), v in sorted(agg.items()):
    if c.startswith("SQ_INSTS") and waves.get(kn):
        print(f"{kn[-40:]:40s} {c:22s} per wave {v / len(nd[(kn, c)]) / waves[kn]:.1f}")
