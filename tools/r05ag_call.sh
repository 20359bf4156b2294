#!/usr/bin/env bash
# r05ag: octant-ordered slab tests for waves whose rays all point into the node
# copy's octant (11 VALU per box instead of 17) vs the general form; GPU tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05ag; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
STEPS=5 bash tools/ab_bench.sh -r 3 -c c5 ab/librtg_base.so ab/librtg_ord.so > $O/ab_c5_ord.log 2>&1; rc=$?
cat $O/ab_c5_ord.log; exit $rc
