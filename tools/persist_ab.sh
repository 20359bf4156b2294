set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  for p in 0 28 56 112; do
    RTG_PERSIST_PER_CU=$p timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('persist', $p, d['kernel_ms'], d['parity'].get('fb_md5_match'), flush=True)" || exit 1
  done
done
