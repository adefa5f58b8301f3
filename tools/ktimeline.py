"""Kernel timeline of the last N dispatches from a rocprofv3 results database (its kernels
view): start offset, duration (us), queue/stream, name.  usage: tools/ktimeline.py <db> [n] [filter]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
flt = sys.argv[3] if len(sys.argv) > 3 else ""
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
q = "select name, start, end, queue_id, stream_id from kernels order by start"
rows = [r for r in c.execute(q) if flt in r[0]][-n:]
t0 = rows[0][1]
for name, s, e, qid, sid in rows:
    print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:9.1f} q{qid} s{sid}  {name[:90]}")
