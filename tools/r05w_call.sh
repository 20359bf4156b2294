#!/usr/bin/env bash
# r05w: the cull pass zero-fills only the empty groups' pixels (the trace
# kernel writes the live ones) vs every group's; GPU tests on the former
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05w; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
STEPS=30 bash tools/ab_bench.sh -r 3 -c c3 ab/librtg_allfill.so ab/librtg_deadfill.so > $O/ab_c3_deadfill.log 2>&1 &&
STEPS=40 bash tools/ab_bench.sh -r 3 -c c2 ab/librtg_allfill.so ab/librtg_deadfill.so > $O/ab_c2_deadfill.log 2>&1 &&
STEPS=10 bash tools/ab_bench.sh -r 2 -c c4 ab/librtg_allfill.so ab/librtg_deadfill.so > $O/ab_c4_deadfill.log 2>&1 || exit 1
cat $O/ab_*.log
