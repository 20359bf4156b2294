#!/usr/bin/env bash
# r05aa: list partitions spread over XCDs and shader engines (runs of 32
# indices per partition), 16 and 32 partitions, vs one partition per wave
# index mod 16 (base); GPU tests on the spread build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05aa; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
STEPS=30 bash tools/ab_bench.sh -r 3 -c c3 ab/librtg_base.so ab/librtg_spread.so ab/librtg_spread32.so > $O/ab_c3_spread.log 2>&1 &&
STEPS=40 bash tools/ab_bench.sh -r 3 -c c2 ab/librtg_base.so ab/librtg_spread.so ab/librtg_spread32.so > $O/ab_c2_spread.log 2>&1 &&
STEPS=10 bash tools/ab_bench.sh -r 2 -c c4 ab/librtg_base.so ab/librtg_spread.so ab/librtg_spread32.so > $O/ab_c4_spread.log 2>&1 || exit 1
cat $O/ab_*.log
