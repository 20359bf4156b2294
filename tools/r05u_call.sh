#!/usr/bin/env bash
# r05u: cull-pass rounds per lane (RTG_CULL_ROUNDS 1 / 2 / 4) now that the
# partitioned list's atomics no longer serialise: bench frame time, and the
# cull pass's time under rocprof for C3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05u; mkdir -p $O
for c in c2 c3 c4; do
  for r in 1 2 3; do
    for R in 1 2 4; do
      RTG_LIB=$PWD/ab/librtg_rounds.so RTG_CULL_ROUNDS=$R timeout -k 10 200 python bench.py --config $c --steps 30 --warmup 3 --no-cpu-baseline \
          --no-work-count --no-e2e 2>>$O/err.log \
        | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$c', 'rounds $R', d['kernel_ms'], d['parity'].get('bit_exact'), flush=True)" | tee -a $O/cull_rounds.log || exit 1
    done
  done
done
for R in 1 2 4; do
  for c in c3 c2; do
  ( cd /tmp && export TMPDIR=/tmp && RTG_LIB=$GRAFT_REPO_ROOT/ab/librtg_rounds.so RTG_CULL_ROUNDS=$R timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $GRAFT_REPO_ROOT/$O/prof_${R}_$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 20 --warmup 3 \
      --no-cpu-baseline --no-work-count --no-e2e > $GRAFT_REPO_ROOT/$O/b_${R}_$c.json 2> $GRAFT_REPO_ROOT/$O/b_${R}_$c.err ) || exit 1
  python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$O/prof_${R}_$c/**/run_kernel_stats.csv',recursive=True)[0])):
    if 'cull' in r['Name'] or 'trace_samples' in r['Name']: print('rounds $R $c', r['Name'][:40], r['AverageNs'], r['Calls'])
" | tee -a $O/cull_rounds_prof.txt
  done
done
