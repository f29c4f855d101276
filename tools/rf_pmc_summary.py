#!/usr/bin/env python3
"""Per-kernel summary of tools/rf_pmc.sh output: counters summed over dispatches of the last fit's
big kernels (rf_init_rows, rf_partition), per-wave and per-cycle ratios.
usage: tools/rf_pmc_summary.py [gpurun_out/rfpmc]"""
import collections
import csv
import glob
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/rfpmc"
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob(f"{d}/set*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        if "rf_" not in n:
            continue
        acc[n][r["Counter_Name"]] += float(r["Counter_Value"])
for n, c in acc.items():
    w = c.get("SQ_WAVES", 0) or 1
    print(f"{n}")
    for k in sorted(c):
        print(f"  {k:24s} {c[k]:16.4g}   per-wave {c[k] / w:10.1f}")
    if c.get("SQ_BUSY_CYCLES"):
        print(f"  LDS active / wave-cycles  {c.get('SQ_ACTIVE_INST_LDS', 0) / max(c.get('SQ_WAVE_CYCLES', 1), 1):.3f}")
        print(f"  bank conflict / LDS-active cycles {c.get('SQ_LDS_BANK_CONFLICT', 0) / max(c.get('SQ_LDS_IDX_ACTIVE', 1), 1):.3f}")
