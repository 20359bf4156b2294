#!/usr/bin/env bash
# tools/r03_aabb_ab.sh — GPU tests on the in-tree build, then same-box A/B of
# the sphere-bound BVH (ab/librtg_top.so) against the box BVH
# (ab/librtg_aabb.so) on C5, then the scratch-traffic A/B
# (tools/r03_scratch_ab.sh).  Each GPU step has its own time limit; the chain
# stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-aabb_ab}
mkdir -p $OUT
echo "== pytest -m gpu" &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== A/B c5" &&
STEPS=5 bash tools/ab_bench.sh -r 3 -c c5 $PWD/ab/librtg_top.so $PWD/ab/librtg_aabb.so | tee $OUT/ab_c5.log || exit 1
[ -n "$SKIP_SCRATCH" ] || TAG=${TAG:-aabb_ab}_scratch bash tools/r03_scratch_ab.sh
