#!/usr/bin/env bash
# tools/r03_check_mg.sh — GPU tests on the in-tree build, the 2- and 3-rank
# gloo rehearsals of bench.py's N > 1 path (all ranks on this GPU), and the
# C3/C4 one-GPU bench lines (E2E with the host scene preparation).  Each GPU
# step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-mg}
mkdir -p $OUT
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== 2-rank rehearsal"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 3 --dist-backend gloo > $OUT/b2.json 2> $OUT/b2.err || { tail -20 $OUT/b2.err; exit 1; }
tail -1 $OUT/b2.json | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['multi_gpu'], d['parity'])"
echo "== 3-rank rehearsal (c2)"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 3 --steps 3 --warmup 2 --dist-backend gloo --config c2 > $OUT/b3.json 2> $OUT/b3.err || { tail -20 $OUT/b3.err; exit 1; }
tail -1 $OUT/b3.json | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['multi_gpu'], d['parity'])"
for c in c3 c4; do
  echo "== bench $c"
  timeout -k 10 600 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -5 $OUT/bench_$c.err; exit 1; }
  tail -1 $OUT/bench_$c.json | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$c', d['value'], d['ms_per_step'], d['e2e'])"
done
echo "== done"
