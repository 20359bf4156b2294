#!/usr/bin/env bash
# r05y: 32 list partitions vs 16 (C2, C3)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05y; mkdir -p $O
STEPS=40 bash tools/ab_bench.sh -r 4 -c c2 ab/librtg_base.so ab/librtg_p32.so > $O/ab_c2_p32.log 2>&1 &&
STEPS=30 bash tools/ab_bench.sh -r 3 -c c3 ab/librtg_base.so ab/librtg_p32.so > $O/ab_c3_p32.log 2>&1; rc=$?
cat $O/ab_*.log; exit $rc
