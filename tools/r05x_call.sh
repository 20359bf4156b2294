#!/usr/bin/env bash
# r05x: the BVH node record as three scalar loads issued together (64 + 32 +
# 16 bytes; the containment radii only where used) vs two 64-byte loads that
# the register allocator serialised (overlapping SGPR ranges): C5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05x; mkdir -p $O
STEPS=5 bash tools/ab_bench.sh -r 3 -c c5 ab/librtg_base.so ab/librtg_load3.so > $O/ab_c5_load3.log 2>&1; rc=$?
cat $O/ab_c5_load3.log; exit $rc
