#!/usr/bin/env python3
"""Is a request's GPU chain bound by the host's launches? Reads a
``rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv`` run of tools/request_trace.py and
joins every kernel with the HIP API call that launched it (Correlation_Id): per kernel name, the
median time from the launch call's END (the kernel is in the queue) to the kernel's START, and from
the previous kernel's end to its start. A kernel that starts right after its launch call returned,
with an idle GPU before it, waited for the host -- not for the GPU.

    python tools/launch_lag.py gpurun_out/lag --requests 200
"""
import argparse
import csv
import glob
import json
import os
import statistics


def _rows(d, pat):
    out = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        with open(f, newline="") as fh:
            out.extend(csv.DictReader(fh))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--requests", type=int, default=200)
    ap.add_argument("--marker", default="k_freq_evict", help="one launch per request (request boundary)")
    a = ap.parse_args()
    ks = _rows(a.dir, "*kernel_trace.csv")
    api = _rows(a.dir, "*hip_api_trace.csv")
    launch = {}
    for r in api:
        if "Launch" in r.get("Function", "") or "launch" in r.get("Function", ""):
            launch[r["Correlation_Id"]] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"])
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Correlation_Id"]) for r in ks)
    marks = [i for i, x in enumerate(ev) if a.marker in x[2]]
    groups = [ev[i:j] for i, j in zip(marks, marks[1:])][-a.requests:]
    per = {}
    rows_med = None
    for g in groups:
        prev_end = None
        rows = []
        for s, e, name, cid in g:
            l = launch.get(cid)
            lag = (s - l[1]) / 1e3 if l else float("nan")         # queued -> started
            idle = (s - prev_end) / 1e3 if prev_end is not None else 0.0
            per.setdefault(name[:60], []).append((lag, idle, (e - s) / 1e3))
            rows.append((name[:60], (s - g[0][0]) / 1e3, (e - s) / 1e3, idle, lag,
                         (l[1] - g[0][0]) / 1e3 if l else float("nan")))
            prev_end = e if prev_end is None else max(prev_end, e)
        rows_med = rows_med or rows
    print(json.dumps({"requests": len(groups), "launch_calls": len(launch), "kernels": len(ev)}))
    print("median per kernel: queued->start us, idle-before us, duration us, name")
    for name, v in sorted(per.items(), key=lambda kv: -statistics.median(x[2] for x in kv[1])):
        print(f"{statistics.median(x[0] for x in v):8.1f} {statistics.median(x[1] for x in v):8.1f} "
              f"{statistics.median(x[2] for x in v):8.1f}  {name}")
    if groups:
        g = groups[len(groups) // 2]
        print("one request: offset_us dur_us idle_before_us queued_to_start_us launch_returned_at_us name")
        prev_end = None
        for s, e, name, cid in g:
            l = launch.get(cid)
            idle = (s - prev_end) / 1e3 if prev_end is not None else 0.0
            print(f"{(s - g[0][0]) / 1e3:8.1f} {(e - s) / 1e3:7.1f} {idle:7.1f} "
                  f"{((s - l[1]) / 1e3) if l else float('nan'):8.1f} {((l[1] - g[0][0]) / 1e3) if l else float('nan'):8.1f}"
                  f"  {name[:60]}")
            prev_end = e if prev_end is None else max(prev_end, e)
        # every HIP API call of that request's host thread(s), from the first kernel's launch
        t0 = g[0][0]
        lo = launch[g[0][3]][0] if g[0][3] in launch else t0
        hi = g[-1][1]
        calls = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in api
                       if lo <= int(r["Start_Timestamp"]) <= hi)
        print("API calls of that request: start_us (rel. first kernel start) dur_us function")
        for s, e, f in calls:
            print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {f}")
        # median host cost per API function over all requests' windows
        per_f = {}
        for g2 in groups:
            lo2 = launch[g2[0][3]][0] if g2[0][3] in launch else g2[0][0]
            for r in api:
                s2 = int(r["Start_Timestamp"])
                if lo2 <= s2 <= g2[-1][1]:
                    per_f.setdefault(r["Function"], []).append((int(r["End_Timestamp"]) - s2) / 1e3)
        print("per function: calls/request, median us, total us/request")
        n = len(groups)
        for f, v in sorted(per_f.items(), key=lambda kv: -sum(kv[1])):
            print(f"{len(v) / n:6.1f} {statistics.median(v):7.2f} {sum(v) / n:8.1f}  {f}")


if __name__ == "__main__":
    main()
