#!/usr/bin/env bash
# r05ao: where C5's scalar-cache misses are: SQC hits/misses of the shipped
# build and of a diagnostic build whose queries all take the BVH (no sphere
# lists), with the SMEM instruction count; both frames timed
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$GRAFT_REPO_ROOT/gpurun_out/r05ao; mkdir -p $O
for L in base nolists; do
  ( cd /tmp && export TMPDIR=/tmp && RTG_LIB=$GRAFT_REPO_ROOT/ab/librtg_$L.so timeout -s KILL 240 rocprofv3 --pmc SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_INSTS_SMEM SQ_INSTS_VALU \
      --output-format csv -d $O/pmc_$L -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c5 --steps 1 --warmup 1 \
      --no-cpu-baseline --no-work-count --no-e2e > $O/b_$L.json 2> $O/b_$L.err ) || exit 1
  python3 - <<PY | tee -a $O/sqc.txt
import csv, glob, collections, json
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob("$O/pmc_$L/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "trace_samples" not in r["Kernel_Name"]: continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
d = json.loads(open("$O/b_$L.json").read().strip().splitlines()[-1])
for k in sorted(tot): print("c5 $L", k, "%.4g" % (tot[k] / n[k]), "per launch (n=%d)" % n[k])
print("c5 $L kernel_ms", d["kernel_ms"], "bit_exact", d["parity"].get("bit_exact"))
PY
done
