"""Per-kernel statistics from a rocprofv3 rocpd SQLite database (rocprofv3 7.x default output):
    python tools/prof_db_stats.py run_results.db [--skip N]   -> name, calls, avg/min/max us, total us."""
import sqlite3
import sys
from collections import defaultdict

db = sqlite3.connect(sys.argv[1])
rows = db.execute("select * from kernels").fetchall()
cols = [d[0] for d in db.execute("select * from kernels").description]
ix = {c: i for i, c in enumerate(cols)}
name_col = "kernel_name" if "kernel_name" in ix else "name"
stat = defaultdict(list)
for r in rows:
    stat[r[ix[name_col]]].append((r[ix["end"]] - r[ix["start"]]) / 1e3)
tot = sum(sum(v) for v in stat.values())
for k, v in sorted(stat.items(), key=lambda kv: -sum(kv[1])):
    print(f"{sum(v):10.1f} us {100 * sum(v) / tot:5.1f}%  n={len(v):5d} avg={sum(v) / len(v):8.2f} min={min(v):8.2f}  {k[:110]}")
