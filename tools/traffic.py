#!/usr/bin/env python3
"""Summarise a tools/pmc.sh run (gpurun_out/<tag>_pmc) for the replay kernel into
profiles/<name>_pmc.txt and profiles/traffic_latest.json (read by bench.py).

HBM bytes per launch follow /opt/skills/guides/MI355X_MICROARCH.md (HBM section):
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of
a coalesced streaming read (128-B requests tallied at 64 B), so it is doubled;
WRITE_SIZE is taken as is.  Calibrated for the replay kernels' own access widths
(tools/calib.hip, profiles/r5_pmc_calibration.txt): FETCH_SIZE = 0.500 x the bytes for
4-, 8- and 16-B-per-lane loads and for the slab's column-per-row pattern (one
TCC_EA0_RDREQ per 128 B), so x2 holds for every read here; WRITE_SIZE = 1.000 x the bytes
for 4-, 8- and 16-B streaming stores, while a record written 8 B per store from lanes 256 B
apart costs one 64-B write request per store (WRITE_SIZE = 8.1 x the record bytes, 548 GB/s
of records) — real write traffic, not a miscount.  Counters are averaged over the profiled dispatches — or, with
an anchor kernel (a multi-kernel step: C3-C5 run several replay kernels per step), summed
over every matching dispatch and divided by the anchor's dispatch count (one per step).
Writes profiles/traffic_<workload>.json (and traffic_latest.json).
usage: tools/traffic.py <tag> <workload> <profile-name> [kernel-substring] [anchor-kernel] [anchors per step]
env TRAFFIC_AFTER=<regex>: count only the dispatches from the first one whose kernel name matches
(a bench line whose setup replays first: the carry line's prefix); TRAFFIC_EXCLUDE=<substring>:
leave out matching kernels (the NDC line's closing k_digest)."""
import collections
import re
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag, workload, name = sys.argv[1:4]
    kern = sys.argv[4] if len(sys.argv) > 4 else "k_replay"
    anchor = sys.argv[5] if len(sys.argv) > 5 else None
    per_step = float(sys.argv[6]) if len(sys.argv) > 6 else 1.0  # anchor dispatches per step
    agg = collections.defaultdict(float)
    nd = collections.defaultdict(set)
    steps = collections.defaultdict(set)  # per counter pass: the anchor's dispatches
    kernels = collections.defaultdict(set)
    after = re.compile(os.environ["TRAFFIC_AFTER"]) if os.environ.get("TRAFFIC_AFTER") else None
    excl = os.environ.get("TRAFFIC_EXCLUDE")
    for f in glob.glob(os.path.join(ROOT, "gpurun_out", f"{tag}_pmc", "*", "*counter_collection.csv")):
        rows = list(csv.DictReader(open(f)))
        if after:  # this pass's first dispatch of the timed kernels (dispatch ids are per process)
            ids = [int(r["Dispatch_Id"]) for r in rows if after.search(r["Kernel_Name"])]
            first = min(ids) if ids else 1 << 62
            rows = [r for r in rows if int(r["Dispatch_Id"]) >= first]
        if excl:
            rows = [r for r in rows if excl not in r["Kernel_Name"]]
        for r in rows:
            if anchor and anchor in r["Kernel_Name"]:
                steps[r["Counter_Name"]].add(r["Dispatch_Id"])
            if kern not in r["Kernel_Name"]:
                continue
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            nd[r["Counter_Name"]].add(r["Dispatch_Id"])
            kernels[r["Kernel_Name"].split("(")[0]].add(r["Dispatch_Id"])
    if anchor:
        avg = {c: v / max(1, len(steps[c])) * per_step for c, v in agg.items()}
    else:
        avg = {c: v / len(nd[c]) for c, v in agg.items()}
    lines = [f"{c:24s} {v:.6g}" for c, v in sorted(avg.items())]
    waves = avg.get("SQ_WAVES", 0)
    out = {"workload": workload, "kernel": kern, "source": f"rocprofv3 --pmc passes, tools/pmc.sh ({tag})",
           "per": f"step (sum over the matching kernels / {anchor} dispatches)" if anchor else "dispatch",
           "kernels": sorted(kernels), "counters": avg}
    sha = os.path.join(ROOT, "gpurun_out", f"{tag}_pmc", "lib_sha1")
    if os.path.exists(sha):
        out["lib_sha1"] = open(sha).read().strip()
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        rd = avg["FETCH_SIZE"] * 1024 * 2
        wr = avg["WRITE_SIZE"] * 1024
        out.update({"read_bytes_per_launch": rd, "write_bytes_per_launch": wr, "bytes_per_launch": rd + wr,
                    "correction": "FETCH_SIZE KiB x 1024 x 2 (gfx950 half-count), WRITE_SIZE KiB x 1024"})
        lines.append(f"HBM read  bytes/launch  {rd:.4g} (FETCH_SIZE x 2 KiB)")
        lines.append(f"HBM write bytes/launch  {wr:.4g}")
    if waves:
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_BRANCH", "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS"):
            if c in avg:
                lines.append(f"{c} per wave            {avg[c] / waves:.1f}")
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    open(os.path.join(ROOT, "profiles", f"{name}_pmc.txt"), "w").write("\n".join(lines) + "\n")
    json.dump(out, open(os.path.join(ROOT, "profiles", f"traffic_{workload}.json"), "w"), indent=1)
    json.dump(out, open(os.path.join(ROOT, "profiles", "traffic_latest.json"), "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
