# round-5 GPU call: GPU tests on the cleaned-up sources, then a same-box A/B
# of the BVH kernel at 7 waves per SIMD (ab/librtg_w7.so) against them on C5.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r05c; mkdir -p $OUT
echo "== pytest -m gpu" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== A/B c5 7 waves" &&
STEPS=8 bash tools/ab_bench.sh -r 3 -c c5 ab/librtg_cur.so ab/librtg_w7.so > $OUT/ab_c5_w7.log 2>&1; rc=$?; cat $OUT/ab_c5_w7.log; [ $rc -eq 0 ] || exit $rc
echo "== done"
