#!/usr/bin/env bash
# tools/r03_check.sh — round-3 GPU sequence: parity tests, smoke, and the bench
# line of every one-GPU config (roofline from executed work, E2E, CPU
# baseline).  Every GPU step has its own time limit; the chain stops at the
# first failure.  OUT=gpurun_out/$TAG.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03}
OUT=gpurun_out/$TAG
mkdir -p $OUT
CONFIGS=${CONFIGS:-"c3 c2 c4 c5"}
if [ -z "$SKIP_TESTS" ]; then
  echo "== pytest -m gpu" &&
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
      > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -4 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  echo "== smoke" &&
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
  tail -2 $OUT/smoke.log || exit 1
fi
for c in $CONFIGS; do
  echo "== bench $c" &&
  timeout -k 10 600 python bench.py --config $c --steps ${STEPS:-20} --warmup 3 $BENCH_ARGS \
      > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -5 $OUT/bench_$c.err; exit 1; }
  python -c "import json,sys;d=json.loads(open('$OUT/bench_$c.json').read().strip().splitlines()[-1]);r=d['roofline'] or {};print('$c', d['value'], d['unit'], d['ms_per_step'], 'frac', r.get('frac'), 'cpu', (d['cpu_baseline'] or {}).get('value'), 'bit_exact', d['parity'].get('bit_exact'), 'e2e', (d['e2e'] or {}).get('e2e_ms'))"
done
echo "== done"
