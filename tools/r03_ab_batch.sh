#!/usr/bin/env bash
# tools/r03_ab_batch.sh — one GPU call: GPU tests on the in-tree build, the
# launch-order A/B (tools/order_ab.sh, ROUNDS rounds), the C5 A/B of the BVH
# and list changes, and the C3/C4 A/B of the internal-reflection enter path.
# Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-order_ab}
mkdir -p $OUT
ROUNDS=${ROUNDS:-2} bash tools/order_ab.sh || exit 1
echo "== A/B c5"
STEPS=5 bash tools/ab_bench.sh -r 2 -c c5 $PWD/ab/librtg_fb.so $PWD/ab/librtg_ik.so $PWD/ab/librtg_rr.so $PWD/ab/librtg_ie.so | tee $OUT/ab_c5.log || exit 1
echo "== A/B c3"
STEPS=20 bash tools/ab_bench.sh -r 3 -c c3 $PWD/ab/librtg_rr.so $PWD/ab/librtg_ie.so | tee $OUT/ab_c3.log || exit 1
echo "== A/B c4"
STEPS=10 bash tools/ab_bench.sh -r 2 -c c4 $PWD/ab/librtg_rr.so $PWD/ab/librtg_ie.so | tee $OUT/ab_c4.log || exit 1
echo "== done"
