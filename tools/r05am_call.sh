#!/usr/bin/env bash
# r05am: diagnostic: every BVH query reads node copy 0 (one eighth of the node footprint, worse child order) vs its octant's copy: C5 A/B and scalar-cache PMC
# a contiguous eighth of the frame; GPU tests; C5 A/B; SQC scalar-cache PMC
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05am; mkdir -p $O

STEPS=5 bash tools/ab_bench.sh -r 3 -c c5 ab/librtg_base.so ab/librtg_oct0.so > $O/ab_c5_oct0.log 2>&1 || exit 1
cat $O/ab_c5_oct0.log
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 180 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_DCACHE_HITS SQC_DCACHE_MISSES \
    --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_c5 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c5 --steps 1 --warmup 1 \
    --no-cpu-baseline --no-work-count --no-e2e > $GRAFT_REPO_ROOT/$O/b_c5.json 2> $GRAFT_REPO_ROOT/$O/b_c5.err ) || exit 1
python3 - <<PY | tee $O/sqc.txt
import csv, glob, collections
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob("$O/pmc_c5/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "trace_samples" not in r["Kernel_Name"]: continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(tot): print("c5 oct0", k, "%.4g" % (tot[k] / n[k]), "per launch (n=%d)" % n[k])
PY
