"""Per-step kernel table from a rocprofv3 rocpd database (sqlite; the default output format of
ROCm 7): python tools/kstats_db.py run_results.db [steps] [top] [--median] [--marker NAME --last K].

--median: per step = median duration x calls / steps (robust to the few launches that queue
behind the copy stream's H2D blit under the profiler); otherwise total duration / steps.
--marker NAME --last K: only the launches from the K-th-from-last launch of kernel NAME (one per
step, e.g. k_nl_count) to the end of the trace -- the last K steps, without the set-up copies,
fills and library uploads that otherwise inflate the launch count per step; steps = K.
--timeline (with --marker): also print one whole step (between the last two marker launches):
each kernel's start offset from the marker, duration and queue, to read the step's critical path."""
import sqlite3
import statistics
import sys


def opt(name, default=None):
    return sys.argv[sys.argv.index(name) + 1] if name in sys.argv else default


flags = {"--marker", "--last"}
args = []
skip = False
for a in sys.argv[1:]:
    if skip:
        skip = False
        continue
    if a in flags:
        skip = True
        continue
    if not a.startswith("--"):
        args.append(a)
median = "--median" in sys.argv
db = args[0]
steps = float(args[1]) if len(args) > 1 else 4.0
top = int(args[2]) if len(args) > 2 else 25
marker, last = opt("--marker"), opt("--last")
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "name" if "name" in cols else "kernel_name"
rows_all = c.execute(f"select {name}, start, end from kernels order by start").fetchall()
if marker and "--timeline" in sys.argv:
    marks = [s for n, s, e in rows_all if marker in n]
    if len(marks) >= 2:
        a, b = marks[-2], marks[-1]
        step_rows = [r for r in rows_all if a <= r[1] < b]
        print(f"one step: {len(step_rows)} launches, marker to last kernel end "
              f"{(max(e for _, _, e in step_rows) - a) / 1e3:.1f} us, marker period {(b - a) / 1e3:.1f} us")
        for n, s_, e in step_rows:
            print(f"  +{(s_ - a) / 1e3:8.1f} us  {(e - s_) / 1e3:8.1f} us  {n[:80]}")
        print()
if marker and last:
    marks = [s for n, s, e in rows_all if marker in n]
    k = int(last)
    if len(marks) >= k:
        t0 = marks[-k]
        rows_all = [r for r in rows_all if r[1] >= t0]
        steps = float(k)
durs = {}
for n, s, e in rows_all:
    durs.setdefault(n, []).append(e - s)
rows = []
for n, d in durs.items():
    t = statistics.median(d) * len(d) if median else sum(d)
    rows.append((n, len(d), t, statistics.median(d)))
rows.sort(key=lambda r: -r[2])
tot = sum(r[2] for r in rows)
for n, k, t, m in rows[:top]:
    print(f"{t / steps / 1e3:9.1f} us/step {k / steps:7.1f}/step  med {m / 1e3:8.1f}  {n[:90]}")
print(f"total {tot / steps / 1e3:.1f} us/step over {sum(r[1] for r in rows) / steps:.0f} launches/step"
      + (" (median-based)" if median else ""))
