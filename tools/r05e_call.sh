# round-5 GPU call: GPU tests on the per-sphere list waterfall build
# (blocked_cap_lanes / container_lanes), then a same-box A/B against the
# previous sources on C5 (and C4, unaffected: masked kernel).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r05e; mkdir -p $OUT
echo "== pytest -m gpu" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== A/B c5 list waterfalls" &&
STEPS=8 bash tools/ab_bench.sh -r 3 -c c5 ab/librtg_cur.so ab/librtg_lanes.so > $OUT/ab_c5_lanes.log 2>&1; rc=$?; cat $OUT/ab_c5_lanes.log; [ $rc -eq 0 ] || exit $rc
echo "== counters c5" &&
TAG=r05e SKIP_TESTS=1 COUNT_CONFIGS=c5 bash tools/r05_probe.sh 2>&1 | tail -14 || exit 1
echo "== done"
