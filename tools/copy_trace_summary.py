"""List the copy records of a rocprofv3 rocpd database in time order: blit kernels
(``__amd_rocclr_copy*``, with duration) and memory-copy records (size, duration, engine fields
when present). python tools/copy_trace_summary.py run_results.db"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
tables = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
print("tables:", ", ".join(t for t in tables if "copy" in t.lower() or "kernel" in t.lower()))
rows = []
kcols = [r[1] for r in c.execute("pragma table_info(kernels)")]
kname = "name" if "name" in kcols else "kernel_name"
for n, s, e in c.execute(f"select {kname}, start, end from kernels"):
    if "rocclr_copy" in n or "rocclr_fill" in n:
        rows.append((s, e, "kernel " + n[:40], ""))
for t in tables:
    if t.lower() in ("memory_copies", "memory_copy", "rocpd_memory_copy") or t.lower().startswith("memory_cop"):
        cols = [r[1] for r in c.execute(f"pragma table_info({t})")]
        print(t, "columns:", cols)
        want = [x for x in cols if x in ("start", "end", "size", "name", "src_agent_id", "dst_agent_id",
                                           "src_agent_abs_index", "dst_agent_abs_index", "queue_id", "stream_id")]
        for r in c.execute(f"select {', '.join(want)} from {t}"):
            d = dict(zip(want, r))
            rows.append((d.get("start", 0), d.get("end", 0), "copy " + str(d.get("name", "")),
                         " ".join(f"{k}={v}" for k, v in d.items() if k not in ("start", "end", "name"))))
        break
rows.sort()
t0 = rows[0][0] if rows else 0
for s, e, what, extra in rows:
    if (e - s) < 20_000 and what.startswith("kernel"):
        continue                                       # small fills/copies of set-up
    print(f"+{(s - t0) / 1e6:10.3f} ms  {(e - s) / 1e3:10.1f} us  {what}  {extra}")
