"""Per-launch kernel durations from a rocprofv3 results database (rocpd sqlite), in launch
order, grouped into runs of the same kernel and grid: name, grid, launches, durations (us).

usage: python scripts/prof_launches.py <results.db> [name-substring]
"""
import itertools
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
sub = sys.argv[2] if len(sys.argv) > 2 else ""
rows = db.execute("select name, duration, grid_x, scratch_size, vgpr_count, lds_size from kernels "
                  "order by start").fetchall()
rows = [r for r in rows if sub in r[0]]
for (name, grid), grp in itertools.groupby(rows, key=lambda r: (r[0].split("(")[0][:60], r[2])):
    g = list(grp)
    d = [r[1] / 1e3 for r in g]
    s = sorted(d)
    print(f"{name:60s} grid {grid:7d} n {len(g):4d} scratch {g[0][3]} vgpr {g[0][4]} lds {g[0][5]} "
          f"median {s[len(s) // 2]:9.2f} us  first {[round(x, 1) for x in d[:6]]}")
