#!/usr/bin/env bash
# r05p: GPU tests on the partitioned group list; A/B against one-list build (cb);
# cull pass time of the partitioned build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05p; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
STEPS=40 bash tools/ab_bench.sh -r 4 -c c2 ab/librtg_cb.so ab/librtg_part.so > $O/ab_c2_parts.log 2>&1 &&
STEPS=40 bash tools/ab_bench.sh -r 3 -c c3 ab/librtg_cb.so ab/librtg_part.so > $O/ab_c3_parts.log 2>&1 &&
STEPS=10 bash tools/ab_bench.sh -r 2 -c c4 ab/librtg_cb.so ab/librtg_part.so > $O/ab_c4_parts.log 2>&1 || exit 1
cat $O/ab_*.log
for c in c2 c3; do
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $GRAFT_REPO_ROOT/$O/prof_$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 20 --warmup 3 \
      --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/bench_prof_$c.json 2> $GRAFT_REPO_ROOT/$O/bench_prof_$c.err ) &&
  python tools/timed_stats.py $O/prof_$c $O/bench_prof_$c.json $O/timed_stats_$c | tail -1 || exit 1
done
