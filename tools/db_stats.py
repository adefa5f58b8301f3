"""The kernel-stats summary of a rocprofv3 results database as the CSV rocprofv3 --stats writes
(Name, Calls, TotalDurationNs, AverageNs, Percentage), one row per kernel AND grid size: a run
that launches one kernel over two batches (bench.py's timed 1M-workflow launches, then a smaller
host-path batch) gets a row for each, so the timed launches' average is the one to compare with
the bench line's live kernel_ms.
usage: tools/db_stats.py <run_results.db> <out.csv>"""
import csv
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, grid_x, count(*), sum(end - start), avg(end - start) from kernels "
                 "group by name, grid_x order by sum(end - start) desc").fetchall()
total = sum(r[3] for r in rows) or 1
with open(sys.argv[2], "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Grid", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
    for name, grid, calls, tot, avg in rows:
        w.writerow([name, grid, calls, int(tot), round(avg, 1), round(100.0 * tot / total, 3)])
