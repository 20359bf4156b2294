#!/usr/bin/env bash
# r05n: cull pass and trace kernel times with kernel arguments forced into
# device memory / host memory (HIP_FORCE_DEV_KERNARG), same library
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05n; mkdir -p $O
for K in unset 0 1; do
  for c in c2 c3; do
    ( cd /tmp && export TMPDIR=/tmp && if [ $K != unset ]; then export HIP_FORCE_DEV_KERNARG=$K; fi &&
      timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv \
        -d $GRAFT_REPO_ROOT/$O/prof_k${K}_$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 20 --warmup 3 \
        --no-cpu-baseline --no-work-count --no-e2e > $GRAFT_REPO_ROOT/$O/b_k${K}_$c.json 2> $GRAFT_REPO_ROOT/$O/b_k${K}_$c.err ) || exit 1
    python3 -c "
import csv,glob,json
d=json.loads(open('$O/b_k${K}_$c.json').read().strip().splitlines()[-1])
for r in csv.DictReader(open(glob.glob('$O/prof_k${K}_$c/**/run_kernel_stats.csv',recursive=True)[0])):
    if 'cull' in r['Name'] or 'trace_samples' in r['Name']: print('kernarg=$K $c', r['Name'][:40], r['AverageNs'], r['Calls'], 'bench ms', d['ms_per_step'])
" | tee -a $O/kernarg_times.txt
  done
done
