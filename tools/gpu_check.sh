#!/usr/bin/env bash
# tools/gpu_check.sh — the GPU-box sequence: parity tests, smoke, bench, rocprof.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-r01}
STEPS=${STEPS:-20}
echo "== pytest -m gpu" &&
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu_$TAG.log 2>&1 &&
tail -3 $OUT/pytest_gpu_$TAG.log &&
echo "== smoke" &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 &&
cat $OUT/smoke_$TAG.log &&
echo "== bench" &&
timeout -k 10 600 python bench.py --steps $STEPS --warmup 3 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err &&
cat $OUT/bench_$TAG.json &&
echo "== 2-rank rehearsal (gloo gather, both ranks on this GPU)" &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --steps 5 --warmup 1 --dist-backend gloo > $OUT/bench2_$TAG.json 2> $OUT/bench2_$TAG.err &&
python -c "import json;l=[x for x in open('$OUT/bench2_$TAG.json') if x.startswith('{')][-1];print('2-rank parity', json.loads(l)['parity'])" &&
echo "== rocprofv3 kernel trace" &&
( cd /tmp && export TMPDIR=/tmp &&
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof_$TAG" -o run \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps $STEPS --warmup 3 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/bench_prof_$TAG.json" 2> "$GRAFT_REPO_ROOT/$OUT/bench_prof_$TAG.err" ) &&
echo "== done"
