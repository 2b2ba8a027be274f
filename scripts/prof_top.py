"""Top kernels by total time from a rocprofv3 results database (rocpd sqlite).

usage: python scripts/prof_top.py <results.db> [rows]
"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 30
q = ("select name, count(*), sum(duration), avg(duration) from kernels group by name "
     "order by sum(duration) desc")
res = db.execute(q).fetchall()
tot = sum(r[2] for r in res)
print(f"total kernel time {tot / 1e6:.3f} ms over {sum(r[1] for r in res)} launches")
for name, n, s, a in res[:rows]:
    print(f"{s / 1e6:10.3f} ms {n:6d} x {a / 1e3:9.2f} us {100 * s / tot:5.1f}%  {name[:120]}")
