#!/usr/bin/env python3
"""Summarise tools/gpu_pmc.sh output: per-counter average over the trace kernel's dispatches."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "trace_kernel"
agg = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "p*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
avg = {k: sum(v) / len(v) for k, v in agg.items()}
for k in sorted(avg):
    print(f"{k:28s} {avg[k]:.6g}  (n={len(agg[k])})")
if "SQ_THREAD_CYCLES_VALU" in avg and "SQ_ACTIVE_INST_VALU" in avg:
    print("VALU lane utilisation       %.3f" % (avg["SQ_THREAD_CYCLES_VALU"] / (avg["SQ_ACTIVE_INST_VALU"] * 64)))
if "FETCH_SIZE" in avg:
    print("HBM read  (FETCH_SIZE x2, gfx950 correction) %.1f MB" % (avg["FETCH_SIZE"] * 2 * 1024 / 1e6))
if "WRITE_SIZE" in avg:
    print("HBM write (WRITE_SIZE)                       %.1f MB" % (avg["WRITE_SIZE"] * 1024 / 1e6))
