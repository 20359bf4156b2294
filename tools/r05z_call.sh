#!/usr/bin/env bash
# r05z: list partitions 8 / 16 / 32 on C3: frame A/B and rocprof kernel times
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05z; mkdir -p $O
STEPS=30 bash tools/ab_bench.sh -r 3 -c c3 ab/librtg_p8.so ab/librtg_base.so ab/librtg_p32.so > $O/ab_c3_parts.log 2>&1 || exit 1
cat $O/ab_c3_parts.log
for L in p8 base p32; do
  ( cd /tmp && export TMPDIR=/tmp && RTG_LIB=$GRAFT_REPO_ROOT/ab/librtg_$L.so timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $GRAFT_REPO_ROOT/$O/prof_$L -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c3 --steps 20 --warmup 3 \
      --no-cpu-baseline --no-work-count --no-e2e > $GRAFT_REPO_ROOT/$O/b_$L.json 2> $GRAFT_REPO_ROOT/$O/b_$L.err ) || exit 1
  python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$O/prof_$L/**/run_kernel_stats.csv',recursive=True)[0])):
    if 'cull' in r['Name'] or 'trace_samples' in r['Name']: print('$L c3', r['Name'][:40], r['AverageNs'], r['Calls'])
" | tee -a $O/parts_prof.txt
done
