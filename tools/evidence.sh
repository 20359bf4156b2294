#!/usr/bin/env bash
# tools/evidence.sh — a round's evidence set in one GPU call (TAG, default
# r06), on the final sources: GPU tests + smoke, the PMC passes of C3, C2, C4
# and C5 (their
# records go to profiles/pmc_<config>.json, which bench.py matches by source
# hash), the bench line of every config (C1 as the CPU-only line), and the
# rocprofv3 kernel trace of the C3 / C2 / C5 bench commands cut to their timed
# launches (tools/timed_stats.py).  Every GPU step has its own time limit; the
# chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  echo "== pytest -m gpu" &&
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log || exit 1
fi
if [ -z "$NO_PMC" ]; then
  for c in ${PMC_CONFIGS:-c3 c2 c4 c5}; do
    steps=3; [ "$c" = c5 ] && steps=1
    echo "== PMC $c" &&
    TAG=${TAG}_$c CFG=$c ARGS="--config $c --steps $steps --warmup 1 --no-cpu-baseline --no-work-count --no-e2e" \
      bash tools/gpu_pmc.sh > $OUT/pmc_$c.log 2>&1 && tail -6 $OUT/pmc_$c.log &&
    cp gpurun_out/pmc_${TAG}_$c/pmc_$c.json profiles/pmc_$c.json || exit 1
  done
fi
for c in ${CONFIGS:-c3 c2 c4 c5 c1cpu}; do
  echo "== bench $c"
  if [ "$c" = c1cpu ]; then
    timeout -k 10 300 python bench.py --cpu-only --config c1 --steps 5 --ppm-out $OUT/c1_cpu.ppm > $OUT/bench_c1_cpu.json 2> $OUT/bench_c1_cpu.err || { tail -5 $OUT/bench_c1_cpu.err; exit 1; }
    tail -c 300 $OUT/bench_c1_cpu.json; echo
    continue
  fi
  timeout -k 10 600 python bench.py --config $c --steps ${STEPS:-20} --warmup 3 ${BENCH_ARGS:-} > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -5 $OUT/bench_$c.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/bench_$c.json').read().strip().splitlines()[-1]);r=d['roofline'] or {};print('$c', d['value'], d['unit'], d['ms_per_step'], 'first', d.get('first_launch_ms'), 'warm-first', d.get('first_launch_warm_gpu_ms'), 'frac', r.get('frac'), 'frac_pmc', r.get('frac_pmc'), 'model/pmc', r.get('model_vs_pmc_valu'), 'traffic', r.get('traffic'), 'cpu', (d['cpu_baseline'] or {}).get('value'), 'bit_exact', d['parity'].get('bit_exact'), 'fb', d['parity'].get('fb_md5_match'), 'ppm', d['parity'].get('ppm_md5_match'))"
done
[ -n "$NO_PROFILES" ] && exit 0
for c in ${PROF_CONFIGS:-c3 c2 c5}; do
  steps=20; [ "$c" = c5 ] && steps=5
  echo "== rocprofv3 kernel trace ($c bench)" &&
  ( cd /tmp && export TMPDIR=/tmp &&
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof_$c" -o run \
      -- python3 "$GRAFT_REPO_ROOT/bench.py" --config $c --steps $steps --warmup 3 --no-cpu-baseline \
      > "$GRAFT_REPO_ROOT/$OUT/bench_prof_$c.json" 2> "$GRAFT_REPO_ROOT/$OUT/bench_prof_$c.err" ) &&
  python tools/timed_stats.py $OUT/prof_$c $OUT/bench_prof_$c.json $OUT/timed_stats_$c || exit 1
done
echo "== all done"
