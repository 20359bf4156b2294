#!/usr/bin/env bash
# r05ad: bench lines of C3, C2, C5 with the refitted unit prices (model/PMC)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05ad; mkdir -p $O
for c in c3 c2 c5; do
  timeout -k 10 600 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { tail -5 $O/bench_$c.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_$c.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$c', d['ms_per_step'], 'frac', r.get('frac'), 'frac_model', r.get('frac_model'), 'model/pmc', r.get('model_vs_pmc_valu'), 'traffic', r.get('traffic'))"
done
