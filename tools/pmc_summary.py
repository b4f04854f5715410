#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc/p*/run_counter_collection.csv) per kernel.

Prints a markdown table: for each of our kernels (lp::*), dispatch count, mean duration, VGPRs,
LDS, and the mean per-dispatch value of every collected counter, plus derived ratios
(LDS bank-conflict cycles per LDS instruction, VALU instructions per wave, MFMA share)."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
vals = defaultdict(lambda: defaultdict(list))
meta = {}
for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if not k.startswith(("lp::", "void lp::")):
            continue
        name = k.replace("void ", "").split("(")[0]
        vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        m = meta.setdefault(name, {"vgpr": r["VGPR_Count"], "agpr": r["Accum_VGPR_Count"], "lds": r["LDS_Block_Size"],
                                   "wg": r["Workgroup_Size"], "dur": []})
        m["dur"].append(dur)

counters = sorted({c for v in vals.values() for c in v})
print("| kernel | VGPR/AGPR | LDS B | WG | " + " | ".join(counters) + " | derived |")
print("|" + "---|" * (len(counters) + 5))
for name in sorted(vals, key=lambda n: -sum(meta[n]["dur"])):
    v = vals[name]
    mean = {c: (sum(x) / len(x)) for c, x in v.items()}
    d = []
    if mean.get("SQ_INSTS_LDS"):
        if "SQ_LDS_BANK_CONFLICT" in mean:
            d.append(f"bankconf/LDS-inst={mean['SQ_LDS_BANK_CONFLICT'] / mean['SQ_INSTS_LDS']:.2f}")
    if mean.get("SQ_WAVES") and "SQ_INSTS_VALU" in mean:
        d.append(f"VALU/wave={mean['SQ_INSTS_VALU'] / mean['SQ_WAVES']:.0f}")
    if mean.get("SQ_INSTS_MFMA") and mean.get("SQ_INSTS_VALU"):
        d.append(f"MFMA/VALU={mean['SQ_INSTS_MFMA'] / mean['SQ_INSTS_VALU']:.3f}")
    if mean.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in mean:
        d.append(f"MFMA-busy/GUI={mean['SQ_VALU_MFMA_BUSY_CYCLES'] / mean['GRBM_GUI_ACTIVE']:.3f}")
    m = meta[name]
    row = [name, f"{m['vgpr']}/{m['agpr']}", m["lds"], m["wg"]] + [f"{mean[c]:.4g}" if c in mean else "" for c in counters]
    print("| " + " | ".join(str(x) for x in row) + " | " + "; ".join(d) + " |")
