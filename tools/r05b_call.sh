set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r05b; mkdir -p $OUT
echo "== pytest -m gpu" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== A/B c5 any-hit" &&
STEPS=8 bash tools/ab_bench.sh -r 3 -c c5 ab/librtg_base.so ab/librtg_anyhit.so > $OUT/ab_c5_anyhit.log 2>&1; rc=$?; cat $OUT/ab_c5_anyhit.log; [ $rc -eq 0 ] || exit $rc
echo "== counters c5" &&
TAG=r05b SKIP_TESTS=1 COUNT_CONFIGS=c5 bash tools/r05_probe.sh 2>&1 | tail -14 || exit 1
echo "== cold probe" &&
timeout -k 10 300 python tools/cold_probe.py --config c3 --json $OUT/cold_c3.json > $OUT/cold_c3.txt 2>&1; rc=$?; cat $OUT/cold_c3.txt | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/cold_probe.py --config c2 --json $OUT/cold_c2.json > $OUT/cold_c2.txt 2>&1; rc=$?; cat $OUT/cold_c2.txt | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
echo "== done"
