#!/usr/bin/env bash
# r05k: same-box A/B of the compacted launch's stream events (base / no events / no system fence / no system fence + same-stream waits skipped)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05k
STEPS=40 bash tools/ab_bench.sh -r 4 -c c2 ab/librtg_ev0.so ab/librtg_ev1.so ab/librtg_ev3.so ab/librtg_ev4.so > gpurun_out/r05k/ab_c2_events.log 2>&1 &&
STEPS=40 bash tools/ab_bench.sh -r 3 -c c3 ab/librtg_ev0.so ab/librtg_ev1.so ab/librtg_ev3.so ab/librtg_ev4.so > gpurun_out/r05k/ab_c3_events.log 2>&1
rc=$?; cat gpurun_out/r05k/*.log; exit $rc
