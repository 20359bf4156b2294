# round-5 GPU call: GPU tests on the BVH-scene internal-reflection build
# (in-tree), then a same-box A/B against the previous sources on C5.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r05h; mkdir -p $OUT
echo "== pytest -m gpu" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== A/B c5 internal reflections" &&
STEPS=8 bash tools/ab_bench.sh -r 3 -c c5 ab/librtg_k4.so ab/librtg_inref.so ab/librtg_k5.so > $OUT/ab_c5_inref.log 2>&1; rc=$?; cat $OUT/ab_c5_inref.log; [ $rc -eq 0 ] || exit $rc
echo "== done"
