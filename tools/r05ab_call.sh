#!/usr/bin/env bash
# r05ab: the cull pass loads a group's previous cost before its sphere tests
# (latency overlapped) vs after; A/B C3/C2 and rocprof cull times
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05ab; mkdir -p $O
STEPS=30 bash tools/ab_bench.sh -r 3 -c c3 ab/librtg_base.so ab/librtg_early.so > $O/ab_c3_early.log 2>&1 &&
STEPS=40 bash tools/ab_bench.sh -r 3 -c c2 ab/librtg_base.so ab/librtg_early.so > $O/ab_c2_early.log 2>&1 || exit 1
cat $O/ab_*.log
for L in base early; do
  for c in c3 c2; do
  ( cd /tmp && export TMPDIR=/tmp && RTG_LIB=$GRAFT_REPO_ROOT/ab/librtg_$L.so timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $GRAFT_REPO_ROOT/$O/prof_${L}_$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 20 --warmup 3 \
      --no-cpu-baseline --no-work-count --no-e2e > $GRAFT_REPO_ROOT/$O/b_${L}_$c.json 2> $GRAFT_REPO_ROOT/$O/b_${L}_$c.err ) || exit 1
  python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$O/prof_${L}_$c/**/run_kernel_stats.csv',recursive=True)[0])):
    if 'cull' in r['Name']: print('$L $c', r['Name'][:30], r['AverageNs'], r['Calls'])
" | tee -a $O/cull_prof.txt
  done
done
