#!/usr/bin/env bash
# r05l: GPU tests on one-event launches; A/B against the two-event base;
# cull pass timing of diagnostic builds (no zero-fill / no sphere test / neither)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05l; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
STEPS=40 bash tools/ab_bench.sh -r 4 -c c2 ab/librtg_ev0.so ab/librtg_cb.so > $O/ab_c2_one_event.log 2>&1 &&
STEPS=40 bash tools/ab_bench.sh -r 3 -c c3 ab/librtg_ev0.so ab/librtg_cb.so > $O/ab_c3_one_event.log 2>&1 || exit 1
cat $O/ab_*.log
for L in cb cnf cns cnn; do
  for c in c2 c3; do
    ( cd /tmp && export TMPDIR=/tmp && RTG_LIB=$GRAFT_REPO_ROOT/ab/librtg_$L.so timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv \
        -d $GRAFT_REPO_ROOT/$O/prof_${L}_$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 20 --warmup 3 \
        --no-cpu-baseline --no-work-count --no-e2e > $GRAFT_REPO_ROOT/$O/b_${L}_$c.json 2> $GRAFT_REPO_ROOT/$O/b_${L}_$c.err ) || exit 1
    python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$O/prof_${L}_$c/**/run_kernel_stats.csv',recursive=True)[0])):
    if 'cull' in r['Name'] or 'trace_samples' in r['Name']: print('$L $c', r['Name'][:40], r['AverageNs'], r['Calls'])
" | tee -a $O/cull_times.txt
  done
done
