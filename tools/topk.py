"""Per-kernel totals from a rocprofv3 results database (its top_kernels view): name,
calls, total ms, average us, percent.  usage: tools/topk.py <run_results.db> [n]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
for name, calls, tot, avg, pct in c.execute(f"select * from top_kernels limit {n}"):
    print(f"{calls:6d} {tot / 1e3:9.2f} ms {avg / 1e3:9.3f} ms/call {pct:5.1f}%  {name[:110]}")
