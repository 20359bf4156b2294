#!/usr/bin/env bash
# tools/r03_evidence.sh — one GPU call for the round's evidence set: an
# optional same-box A/B (AB_LIBS, AB_CONFIG), the GPU tests and smoke, the
# C3/C5 PMC passes (copied to profiles/ for the bench's `traffic`), the bench
# line of every one-GPU config (roofline from executed work, E2E, CPU
# baseline), the rocprofv3 kernel trace of the C3 bench and the
# shard-balance rehearsals.  Every GPU step has its own time limit;
# the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$AB_LIBS" ]; then
  echo "== A/B $AB_CONFIG" &&
  STEPS=${AB_STEPS:-10} bash tools/ab_bench.sh -r ${AB_ROUNDS:-3} -c ${AB_CONFIG:-c3} $AB_LIBS > $OUT/ab.log 2>&1; cat $OUT/ab.log
fi
if [ -z "$SKIP_TESTS" ]; then
  echo "== pytest -m gpu" &&
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log || exit 1
fi
# PMC passes first, so that the bench lines below carry `traffic` (bench.py
# reads profiles/pmc_<config>.json when its source hash matches these sources)
if [ -z "$NO_PMC" ]; then
  echo "== PMC c3" &&
  TAG=${TAG}_c3 bash tools/gpu_pmc.sh > $OUT/pmc_c3.log 2>&1 && tail -6 $OUT/pmc_c3.log &&
  cp gpurun_out/pmc_${TAG}_c3/pmc_c3.json profiles/pmc_c3.json &&
  echo "== PMC c5" &&
  TAG=${TAG}_c5 CFG=c5 ARGS="--config c5 --steps 1 --warmup 1 --no-cpu-baseline --no-work-count --no-e2e" bash tools/gpu_pmc.sh > $OUT/pmc_c5.log 2>&1 && tail -6 $OUT/pmc_c5.log &&
  cp gpurun_out/pmc_${TAG}_c5/pmc_c5.json profiles/pmc_c5.json || exit 1
fi
for c in ${CONFIGS:-c3 c2 c4 c5}; do
  echo "== bench $c" &&
  timeout -k 10 600 python bench.py --config $c --steps ${STEPS:-20} --warmup 3 > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -5 $OUT/bench_$c.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/bench_$c.json').read().strip().splitlines()[-1]);r=d['roofline'] or {};print('$c', d['value'], d['unit'], d['ms_per_step'], 'frac', r.get('frac'), 'cpu', (d['cpu_baseline'] or {}).get('value'), 'bit_exact', d['parity'].get('bit_exact'), 'e2e', (d['e2e'] or {}).get('e2e_ms'))"
done
[ -n "$NO_PROFILES" ] && exit 0
echo "== rocprofv3 kernel trace (c3 bench)" &&
( cd /tmp && export TMPDIR=/tmp &&
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof_c3" -o run \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline \
    > "$GRAFT_REPO_ROOT/$OUT/bench_prof_c3.json" 2> "$GRAFT_REPO_ROOT/$OUT/bench_prof_c3.err" ) &&
echo "== shard balance" &&
timeout -k 10 600 python tools/shard_balance.py --config c4 --blocks 8,16 --json $OUT/shard_balance_c4.json > $OUT/shard_balance_c4.log 2>&1 &&
timeout -k 10 600 python tools/shard_balance.py --config c3 --blocks 4,8 --json $OUT/shard_balance_c3.json > $OUT/shard_balance_c3.log 2>&1 &&
tail -3 $OUT/shard_balance_c3.log &&
echo "== profiles done" || exit 1
echo "== chunk rehearsal (rank 0's part of the N > 1 step)" &&
timeout -k 10 300 python tools/chunk_rehearsal.py --config c3 --ranks 2,4,8 --chunks 2,3,4 --last-frac 0.15 --json $OUT/chunks_c3_last15.json > /dev/null &&
timeout -k 10 300 python tools/chunk_rehearsal.py --config c3 --ranks 2,4,8 --chunks 1,2,4 --json $OUT/chunks_c3_even.json > /dev/null &&
echo "== 2-rank rehearsal (gloo gather, both ranks on this GPU)" &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --steps 5 --warmup 1 --dist-backend gloo > $OUT/bench2_gloo.json 2> $OUT/bench2_gloo.err &&
echo "== timeline c3" &&
timeout -k 10 300 python tools/timeline.py --config c3 --waves-per-block 1 --json $OUT/timeline_c3.json > /dev/null &&
echo "== all done"
