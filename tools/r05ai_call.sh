#!/usr/bin/env bash
# r05ai: instruction- and scalar-data-cache hits/misses (SQC) of the C5 and C3
# trace kernels, one PMC pass each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$GRAFT_REPO_ROOT/gpurun_out/r05ai; mkdir -p $O
for c in c5 c3; do
  steps=3; [ $c = c5 ] && steps=1
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 180 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_DCACHE_HITS SQC_DCACHE_MISSES \
      --output-format csv -d $O/pmc_$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps $steps --warmup 1 \
      --no-cpu-baseline --no-work-count --no-e2e > $O/b_$c.json 2> $O/b_$c.err ) || exit 1
  python3 - <<PY | tee -a $O/sqc.txt
import csv, glob, collections
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob("$O/pmc_$c/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "trace_samples" not in r["Kernel_Name"]: continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(tot): print("$c", k, "%.4g" % (tot[k] / n[k]), "per launch (n=%d)" % n[k])
PY
done
