#!/usr/bin/env bash
# r05i: same-box A/B of the round-4 head against the round-5 head on C3 and C2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05i
STEPS=40 bash tools/ab_bench.sh -r 4 -c c3 ab/librtg_r04.so ab/librtg_r05.so > gpurun_out/r05i/ab_c3_r04_r05.log 2>&1 &&
STEPS=40 bash tools/ab_bench.sh -r 4 -c c2 ab/librtg_r04.so ab/librtg_r05.so > gpurun_out/r05i/ab_c2_r04_r05.log 2>&1
rc=$?; cat gpurun_out/r05i/*.log; exit $rc
