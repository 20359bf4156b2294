# round-5 GPU call: GPU tests on the list-waterfall sources, then the walk
# budget (kListWalks 3 / 4 / 5 / 6) A/B on C5.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r05g; mkdir -p $OUT
echo "== pytest -m gpu" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== A/B c5 walks" &&
STEPS=8 bash tools/ab_bench.sh -r 3 -c c5 ab/librtg_k4.so ab/librtg_k3.so ab/librtg_k5.so ab/librtg_k6.so > $OUT/ab_c5_walks.log 2>&1; rc=$?; cat $OUT/ab_c5_walks.log; [ $rc -eq 0 ] || exit $rc
echo "== counters c5" &&
TAG=r05g SKIP_TESTS=1 COUNT_CONFIGS=c5 bash tools/r05_probe.sh 2>&1 | tail -14 || exit 1
echo "== done"
