"""The kernel-stats summary of a rocprofv3 results database (its top_kernels view) as the
CSV rocprofv3 --stats writes: Name, Calls, TotalDurationNs, AverageNs, Percentage.
usage: tools/db_stats.py <run_results.db> <out.csv>"""
import csv
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
cur = c.execute("select * from top_kernels")
cols = [d[0] for d in cur.description]
with open(sys.argv[2], "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "source_columns:" + "|".join(cols)])
    for name, calls, tot, avg, pct in cur:
        w.writerow([name, calls, int(round(tot * 1e3)), round(avg * 1e3, 1), round(pct, 3)])
