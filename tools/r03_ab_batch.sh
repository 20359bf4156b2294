#!/usr/bin/env bash
# tools/r03_ab_batch.sh — one GPU call: GPU tests on the in-tree build, the
# launch-order A/B (tools/order_ab.sh, ROUNDS rounds: ab/librtg_base.so, the
# feedback build ab/librtg_fb2.so with feedback and with the popcount order)
# and the C5 A/B of the list/key changes (ab/librtg_ik.so) against it.
# Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-order_ab}
mkdir -p $OUT
ROUNDS=${ROUNDS:-2} bash tools/order_ab.sh || exit 1
echo "== A/B c5"
STEPS=5 bash tools/ab_bench.sh -r 2 -c c5 $PWD/ab/librtg_ik.so $PWD/ab/librtg_fb2.so | tee $OUT/ab_c5.log || exit 1
echo "== done"
