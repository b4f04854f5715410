"""Per-step kernel table from a rocprofv3 --stats CSV (bench.py --steps 3 --warmup 1 = 4 steps)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_stats.csv")))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 4.0
for r in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 10]:
    print(f"{float(r['TotalDurationNs']) / steps / 1e3:9.1f} us/step {int(r['Calls']) / steps:6.1f}/step  {r['Name'][:80]}")
print(f"total {sum(float(r['TotalDurationNs']) for r in rows) / steps / 1e3:.1f} us/step")
