#!/usr/bin/env bash
# round-3 diagnostics: GPU tests, C5 bench with unit counters, C5 PMC passes,
# the C4 shard-balance rehearsal.  Each GPU step has its own time limit; the
# chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03b}
mkdir -p $OUT
echo "== pytest -m gpu" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== bench c5 (counts)" &&
timeout -k 10 600 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err &&
echo "== shard balance c4" &&
timeout -k 10 600 python tools/shard_balance.py --config c4 --blocks 8,16 --json $OUT/shard_balance_c4.json > $OUT/shard_balance_c4.log 2>&1 &&
tail -8 $OUT/shard_balance_c4.log &&
echo "== PMC c5" &&
TAG=${TAG:-r03b}_c5 ARGS="--config c5 --steps 1 --warmup 1 --no-cpu-baseline --no-work-count --no-e2e" bash tools/gpu_pmc.sh > $OUT/pmc_c5.log 2>&1; tail -25 $OUT/pmc_c5.log
