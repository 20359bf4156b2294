#!/usr/bin/env bash
# r05t: cold launch order (no launch-order feedback yet) policies, RTG_COLD_ORDER:
# 0 popcount >= 2 first (current), 1 popcount 3+/2/1, 2 material-weighted
# estimate in four runs, 3 image order; the first three launches of a fresh
# frame geometry on a warm GPU (bench.py fresh_geometry_launches_warm_ms)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05t; mkdir -p $O
for c in c3 c2 c4; do
  for r in 1 2 3; do
    for p in 0 1 2 3; do
      RTG_LIB=$PWD/ab/librtg_cold.so RTG_COLD_ORDER=$p timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline \
          --no-work-count --no-e2e 2>>$O/err.log \
        | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$c', 'policy $p', 'fresh', d['fresh_geometry_launches_warm_ms'], 'first', d['first_launch_ms'], 'steady', d['kernel_ms'], d['parity'].get('bit_exact'), flush=True)" | tee -a $O/cold_order.log || exit 1
    done
  done
done
