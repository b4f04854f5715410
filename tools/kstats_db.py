"""Per-step kernel table from a rocprofv3 rocpd database (sqlite; the default output format of
ROCm 7): python tools/kstats_db.py run_results.db [steps] [top]."""
import sqlite3
import sys

db = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 4.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "name" if "name" in cols else "kernel_name"
rows = c.execute(f"select {name}, count(*), sum(end - start) from kernels group by {name} "
                 f"order by sum(end - start) desc").fetchall()
tot = sum(r[2] for r in rows)
for n, k, t in rows[:top]:
    print(f"{t / steps / 1e3:9.1f} us/step {k / steps:7.1f}/step  {n[:90]}")
print(f"total {tot / steps / 1e3:.1f} us/step over {sum(r[1] for r in rows) / steps:.0f} launches/step")
