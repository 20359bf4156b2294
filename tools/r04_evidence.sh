#!/usr/bin/env bash
# tools/r04_evidence.sh — one GPU call of round 4: optional same-box A/B
# (AB_LIBS, AB_CONFIG), the GPU tests and smoke, the PMC passes (NO_PMC=1
# skips), the bench line of every config in CONFIGS (default c3 c2 c4 c5, C1
# as the CPU-only line), and the rocprofv3 kernel trace of the C3 bench with
# its timed-launch summary (tools/timed_stats.py).  Every GPU step has its
# own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$AB_LIBS" ]; then
  echo "== A/B $AB_CONFIG" &&
  STEPS=${AB_STEPS:-10} bash tools/ab_bench.sh -r ${AB_ROUNDS:-3} -c ${AB_CONFIG:-c3} $AB_LIBS > $OUT/ab.log 2>&1; cat $OUT/ab.log
fi
if [ -z "$SKIP_TESTS" ]; then
  echo "== pytest -m gpu" &&
  timeout -k 10 1200 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log || exit 1
fi
if [ -z "$NO_PMC" ]; then
  echo "== PMC c3" &&
  TAG=${TAG}_c3 bash tools/gpu_pmc.sh > $OUT/pmc_c3.log 2>&1 && tail -6 $OUT/pmc_c3.log &&
  cp gpurun_out/pmc_${TAG}_c3/pmc_c3.json profiles/pmc_c3.json &&
  echo "== PMC c5" &&
  TAG=${TAG}_c5 CFG=c5 ARGS="--config c5 --steps 1 --warmup 1 --no-cpu-baseline --no-work-count --no-e2e" bash tools/gpu_pmc.sh > $OUT/pmc_c5.log 2>&1 && tail -6 $OUT/pmc_c5.log &&
  cp gpurun_out/pmc_${TAG}_c5/pmc_c5.json profiles/pmc_c5.json || exit 1
fi
for c in ${CONFIGS:-c3 c2 c4 c5 c1cpu}; do
  echo "== bench $c"
  if [ "$c" = c1cpu ]; then
    timeout -k 10 300 python bench.py --cpu-only --config c1 --steps 5 --ppm-out $OUT/c1_cpu.ppm > $OUT/bench_c1_cpu.json 2> $OUT/bench_c1_cpu.err || { tail -5 $OUT/bench_c1_cpu.err; exit 1; }
    tail -c 400 $OUT/bench_c1_cpu.json; echo
    continue
  fi
  timeout -k 10 600 python bench.py --config $c --steps ${STEPS:-20} --warmup 3 ${BENCH_ARGS:-} > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -5 $OUT/bench_$c.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/bench_$c.json').read().strip().splitlines()[-1]);r=d['roofline'] or {};print('$c', d['value'], d['unit'], d['ms_per_step'], 'first', d.get('first_launch_ms'), 'frac', r.get('frac'), 'cpu', (d['cpu_baseline'] or {}).get('value'), 'bit_exact', d['parity'].get('bit_exact'), 'fb', d['parity'].get('fb_md5_match'), 'ppm', d['parity'].get('ppm_md5_match'), 'e2e', (d['e2e'] or {}).get('e2e_ms'))"
done
if [ -n "$CHUNKS" ]; then
  echo "== chunk rehearsal c3/c4 (8-GPU prediction inputs)" &&
  timeout -k 10 300 python tools/chunk_rehearsal.py --config c3 --ranks 2,4,8 --chunks 1,3,4 --last-frac 0.15 --json $OUT/chunks_c3.json > $OUT/chunks_c3.txt 2>&1 && tail -8 $OUT/chunks_c3.txt &&
  timeout -k 10 300 python tools/chunk_rehearsal.py --config c4 --ranks 8 --chunks 1,3 --last-frac 0.15 --json $OUT/chunks_c4.json > $OUT/chunks_c4.txt 2>&1 && tail -4 $OUT/chunks_c4.txt || exit 1
fi
[ -n "$NO_PROFILES" ] && exit 0
echo "== rocprofv3 kernel trace (c3 bench)" &&
( cd /tmp && export TMPDIR=/tmp &&
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof_c3" -o run \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline \
    > "$GRAFT_REPO_ROOT/$OUT/bench_prof_c3.json" 2> "$GRAFT_REPO_ROOT/$OUT/bench_prof_c3.err" ) &&
python tools/timed_stats.py $OUT/prof_c3 $OUT/bench_prof_c3.json $OUT/timed_stats_c3 &&
echo "== all done"
