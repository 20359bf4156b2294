#!/usr/bin/env bash
# tools/gpu_pmc.sh — PMC passes (one counter group per rocprofv3 run, kernel
# trace only, as MI355X_MICROARCH.md prescribes) over a short bench run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
TAG=${TAG:-r01}
CFG=${CFG:-c3}
ARGS=${ARGS:-"--config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-work-count --no-e2e"}
mkdir -p $OUT/pmc_$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/pmc_$TAG/counters_list.txt 2>&1 || true
i=0
PMC_GROUPS=${PMC_GROUPS:-"FETCH_SIZE|WRITE_SIZE|SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE|SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA"}
IFS='|' read -ra GRPS <<< "$PMC_GROUPS"
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/pmc_$TAG/p$i -o run \
     -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/pmc_$TAG/p$i.json 2> $OUT/pmc_$TAG/p$i.err || { echo "pass $i failed"; tail -5 $OUT/pmc_$TAG/p$i.err; exit 1; }
done
echo "== done"
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $OUT/pmc_$TAG --config $CFG --json $OUT/pmc_$TAG/pmc_$CFG.json > $OUT/pmc_$TAG/summary.txt && cat $OUT/pmc_$TAG/summary.txt
