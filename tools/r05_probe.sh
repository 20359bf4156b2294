#!/usr/bin/env bash
# tools/r05_probe.sh — round-5 measurement call: GPU tests (optional), the
# executed-work counters of the bench configs (stage-0 insignificant queries,
# VERDICT r04 item 3), and PMC memory passes (TCC hit/miss, EA requests;
# item 6).  Every GPU step has its own time limit; the chain stops at the
# first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r05a}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  echo "== pytest -m gpu" &&
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
for c in ${COUNT_CONFIGS:-c3 c5}; do
  echo "== counters $c"
  timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --no-e2e > $OUT/count_$c.json 2> $OUT/count_$c.err || { tail -5 $OUT/count_$c.err; exit 1; }
  python - $OUT/count_$c.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
c, u = r.get("counters", {}), r.get("units", {})
for k in ("D.insig", "D.insigAll", "D.shdSame", "D.enterAll", "D.enterSame"):
    print(k, "[waves, lanes]", c.get(k))
for k in ("U.node", "U.bvhNode", "U.bvhSlot", "U.bvhExact", "U.capIter", "U.ovIter", "U.selExact"):
    print(k, u.get(k))
print("ms", d["ms_per_step"], "first", d.get("first_launch_ms"), "frac", r.get("frac"))
PY
done
if [ -n "$COST_DUMP" ]; then
  for c in $COST_DUMP; do
    echo "== cost dump $c" &&
    timeout -k 10 300 python tools/cost_study.py --dump --config $c --out $OUT/cost_$c.npz > $OUT/cost_$c.txt 2>&1; rc=$?; tail -2 $OUT/cost_$c.txt; [ $rc -eq 0 ] || exit $rc
  done
fi
if [ -n "$MEM_PMC" ]; then
  echo "== memory PMC c3" &&
  TAG=${TAG}_mem CFG=c3 PMC_GROUPS="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum|TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum|FETCH_SIZE|WRITE_SIZE|SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE|SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA" bash tools/gpu_pmc.sh > $OUT/pmc_mem.log 2>&1; rc=$?; tail -30 $OUT/pmc_mem.log; [ $rc -eq 0 ] || exit $rc
fi
echo "== all done"
