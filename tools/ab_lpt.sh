set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/lpt
for r in 1 2 3; do for v in 2 65 3; do
  RTG_LPT_MIN=$v timeout -k 10 200 python bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --no-work-count --no-e2e 2>/dev/null | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('c3 lpt$v', d['kernel_ms'], d['parity'].get('bit_exact'), flush=True)" || exit 1
  RTG_LPT_MIN=$v timeout -k 10 200 python tools/shard_balance.py --config c3 --blocks 8 --ranks 8 --reps 3 2>/dev/null | python3 -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);print('c3/8 lpt$v', max(d['shard_ms']), d['shard_ms'], flush=True)" || exit 1
done; done
