# round-5 GPU call: PMC SQ_INSTS_VALU per scene for the unit-cost calibration on the final sources, bench configs at full size
# (tools/calib_units.py), in its own rocprofv3 pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05ac; mkdir -p $OUT
echo "== calibration PMC" &&
( cd /tmp && export TMPDIR=/tmp &&
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU --output-format csv -d $OUT/calib -o run \
    -- python3 $GRAFT_REPO_ROOT/tools/calib_units.py --collect $OUT/calib > $OUT/calib.log 2>&1 ); rc=$?; tail -3 $OUT/calib.log; [ $rc -eq 0 ] || exit $rc
python3 tools/calib_units.py --fit $OUT/calib > $OUT/fit.txt 2>&1; tail -50 $OUT/fit.txt
echo "== done"
