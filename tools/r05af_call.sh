#!/usr/bin/env bash
# r05af: cull-pass workgroups of 512 and 1024 threads vs 256 (C2, C3, C4)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05af; mkdir -p $O
STEPS=40 bash tools/ab_bench.sh -r 3 -c c2 ab/librtg_base.so ab/librtg_t512.so ab/librtg_t1024.so > $O/ab_c2_cullwg.log 2>&1 &&
STEPS=30 bash tools/ab_bench.sh -r 3 -c c3 ab/librtg_base.so ab/librtg_t512.so ab/librtg_t1024.so > $O/ab_c3_cullwg.log 2>&1 &&
STEPS=10 bash tools/ab_bench.sh -r 2 -c c4 ab/librtg_base.so ab/librtg_t512.so ab/librtg_t1024.so > $O/ab_c4_cullwg.log 2>&1 || exit 1
cat $O/ab_*.log
