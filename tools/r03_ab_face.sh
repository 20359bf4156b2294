#!/usr/bin/env bash
# tools/r03_ab_face.sh — GPU tests on the in-tree build, then the A/B of the
# lights' facing-away pre-test (ab/librtg_face2.so) against the previous
# build (ab/librtg_head.so) on C3, C4 and C5.  Each GPU step has its own time
# limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab_face}
mkdir -p $OUT
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== A/B c3"
STEPS=20 bash tools/ab_bench.sh -r 3 -c c3 $PWD/ab/librtg_head.so $PWD/ab/librtg_face2.so | tee $OUT/ab_c3.log || exit 1
echo "== A/B c4"
STEPS=10 bash tools/ab_bench.sh -r 2 -c c4 $PWD/ab/librtg_head.so $PWD/ab/librtg_face2.so | tee $OUT/ab_c4.log || exit 1
echo "== A/B c5"
STEPS=5 bash tools/ab_bench.sh -r 2 -c c5 $PWD/ab/librtg_head.so $PWD/ab/librtg_face2.so | tee $OUT/ab_c5.log || exit 1
echo "== done"
