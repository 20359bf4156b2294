# round-5 GPU call: same-box A/B of the entering-ray list waterfall
# (lanes2) and its walk budget (2 / 4 / 8) against the shadow + containment
# waterfall (lanes) on C5.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r05f; mkdir -p $OUT
echo "== A/B c5" &&
STEPS=8 bash tools/ab_bench.sh -r 3 -c c5 ab/librtg_lanes.so ab/librtg_lanes2.so ab/librtg_lanes2_k2.so ab/librtg_lanes2_k8.so > $OUT/ab_c5_enter_walks.log 2>&1; rc=$?; cat $OUT/ab_c5_enter_walks.log; [ $rc -eq 0 ] || exit $rc
echo "== done"
