#!/usr/bin/env bash
# tools/order_ab.sh — GPU tests on the in-tree build, then the launch-order
# A/B (tools/order_ab.py) interleaved over ROUNDS rounds: the previous
# library (ab/librtg_base.so), the feedback build (ab/librtg_fb2.so) with
# feedback and with RTG_LAUNCH_ORDER=popcount, on C3 and C4.  Each GPU step
# has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-order_ab}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  echo "== pytest -m gpu"
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq ${ROUNDS:-3}); do
  for c in ${CONFIGS:-c3 c4}; do
    RTG_LIB=$PWD/ab/librtg_base.so timeout -k 10 300 python tools/order_ab.py --config $c | tee -a $OUT/ab.jsonl || exit 1
    RTG_LIB=$PWD/ab/librtg_fb2.so timeout -k 10 300 python tools/order_ab.py --config $c | tee -a $OUT/ab.jsonl || exit 1
    RTG_LAUNCH_ORDER=popcount RTG_LIB=$PWD/ab/librtg_fb2.so timeout -k 10 300 python tools/order_ab.py --config $c | tee -a $OUT/ab.jsonl || exit 1
  done
done
echo "== done"
