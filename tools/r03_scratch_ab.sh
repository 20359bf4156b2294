#!/usr/bin/env bash
# tools/r03_scratch_ab.sh — does the reflection-child scratch traffic cost
# time?  Interleaved same-box A/B of three builds of one revision:
#   top  the default (every reflection child ray in private memory)
#   fr0  RTG_FR0_REGS=1: level 0's child ray in VGPRs (less traffic)
#   x2   RTG_SCRATCH_X2=1: every child ray written and read twice (2x traffic)
# on C3 and C4, then the HBM traffic (FETCH_SIZE / WRITE_SIZE passes) of each
# build on C3.  Each GPU step has its own time limit; the chain stops at the
# first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-scratch_ab}
mkdir -p $OUT
LIBS=${LIBS:-"$PWD/ab/librtg_top.so $PWD/ab/librtg_fr0.so $PWD/ab/librtg_x2.so"}
echo "== A/B c3" &&
STEPS=20 bash tools/ab_bench.sh -r ${ROUNDS:-4} -c c3 $LIBS | tee $OUT/ab_c3.log &&
echo "== A/B c4" &&
STEPS=10 bash tools/ab_bench.sh -r 3 -c c4 $LIBS | tee $OUT/ab_c4.log || exit 1
for b in top fr0 x2; do
  echo "== traffic $b" &&
  RTG_LIB=$PWD/ab/librtg_$b.so TAG=${TAG:-scratch_ab}_$b PMC_GROUPS="FETCH_SIZE|WRITE_SIZE|SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
    bash tools/gpu_pmc.sh > $OUT/pmc_$b.log 2>&1 || { tail -5 $OUT/pmc_$b.log; exit 1; }
  grep -E "HBM|SQ_WAIT|SQ_WAVE_CYCLES" $OUT/pmc_$b.log
done
echo "== done"
