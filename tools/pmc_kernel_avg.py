#!/usr/bin/env python3
"""tools/pmc_kernel_avg.py DIR [BENCH_JSON] — per-launch averages of every PMC
counter a rocprofv3 --pmc run under DIR collected for the trace kernel
(trace_samples_*), plus the bench line's kernel time and parity flag."""
import collections
import csv
import glob
import json
import sys

d = sys.argv[1]
tot = collections.defaultdict(float)
n = collections.Counter()
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "trace_samples" not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        n[r["Counter_Name"]] += 1
for k in sorted(tot):
    print("%-24s %.4g per launch (n=%d)" % (k, tot[k] / n[k], n[k]))
if "SQC_DCACHE_HITS" in tot and "SQC_DCACHE_MISSES" in tot:
    h, m = tot["SQC_DCACHE_HITS"], tot["SQC_DCACHE_MISSES"]
    print("scalar-cache miss rate   %.3f" % (m / (h + m)))
if len(sys.argv) > 2:
    line = [x for x in open(sys.argv[2]).read().splitlines() if x.startswith("{")][-1]
    b = json.loads(line)
    print("kernel_ms", b.get("kernel_ms"), "bit_exact", b.get("parity", {}).get("bit_exact"))
