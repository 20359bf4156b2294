#!/usr/bin/env bash
# r05v: GPU tests on the one-group-per-lane cull pass; A/B against the
# rounds-per-lane policy it replaces (librtg_rounds.so without RTG_CULL_ROUNDS)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05v; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
STEPS=30 bash tools/ab_bench.sh -r 3 -c c3 ab/librtg_rounds.so ab/librtg_r1.so > $O/ab_c3_r1.log 2>&1 &&
STEPS=10 bash tools/ab_bench.sh -r 2 -c c4 ab/librtg_rounds.so ab/librtg_r1.so > $O/ab_c4_r1.log 2>&1 &&
STEPS=40 bash tools/ab_bench.sh -r 3 -c c2 ab/librtg_rounds.so ab/librtg_r1.so > $O/ab_c2_r1.log 2>&1 || exit 1
cat $O/ab_*.log
