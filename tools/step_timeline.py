"""Timeline of one bulk step from a rocprofv3 kernel trace (rocpd sqlite): every kernel / copy of
the median step in start order with its duration and the idle gap before it, plus per-step totals
(span, busy = union of kernel intervals, idle gaps). Steps are delimited by a marker kernel that
runs once per step (default k_nl_count); the first --skip steps are ignored (warm-up).

    python tools/step_timeline.py run_results.db [--marker k_nl_count] [--skip 2]

Answers "where does the step's device time go": kernel time vs gaps where the GPU waits for the
host (the mid-step count read, launch overhead of the post-match chain)."""
import argparse
import sqlite3
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="k_nl_count")
    ap.add_argument("--skip", type=int, default=2)
    ap.add_argument("--gap-us", type=float, default=20.0, help="list gaps longer than this")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else "kernel_name"
    ev = [(s, e, n) for n, s, e in c.execute(f"select {name}, start, end from kernels")]
    try:
        ev += [(s, e, "<copy>") for s, e in c.execute("select start, end from memory_copies")]
    except sqlite3.Error:
        pass
    ev.sort()
    marks = [s for s, e, n in ev if a.marker in n]
    steps = []
    for x, y in zip(marks, marks[1:]):
        steps.append([t for t in ev if x <= t[0] < y and t[2] != "<copy>"])
    steps = steps[a.skip:]
    if not steps:
        raise SystemExit("no complete steps after --skip")
    stats = []
    for st in steps:
        # the marker kernel's start may wait behind the ingest copy: measure from its END
        t0 = st[0][1]
        body = st[1:]
        end = max(e for _, e, _ in st)
        busy, cur_s, cur_e = 0, None, None
        for s, e, _ in body:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            busy += cur_e - cur_s
        stats.append(((end - t0) / 1e3, busy / 1e3, len(st)))
    med = sorted(range(len(stats)), key=lambda i: stats[i][0])[len(stats) // 2]
    print(f"steps {len(stats)}: span (after the marker) med {statistics.median(s[0] for s in stats):.1f} us, "
          f"busy med {statistics.median(s[1] for s in stats):.1f} us, launches med "
          f"{statistics.median(s[2] for s in stats)}")
    st = steps[med]
    t0 = st[0][1]
    prev = t0
    print(f"timeline of step {med + a.skip}: offset_us dur_us gap_us name (gaps > {a.gap_us} us flagged *)")
    for s, e, n in st[1:]:
        gap = max(0.0, (s - prev) / 1e3)
        flag = "*" if gap > a.gap_us else " "
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {gap:8.1f}{flag} {n[:70]}")
        prev = max(prev, e)


if __name__ == "__main__":
    main()
