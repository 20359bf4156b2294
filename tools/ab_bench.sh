#!/usr/bin/env bash
# tools/ab_bench.sh LIB_A LIB_B [ROUNDS] [CONFIG] — interleaved same-box A/B of two
# librtg.so builds on a bench config (kernel ms from HIP events per run).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A=$1; B=$2; N=${3:-4}; C=${4:-c3}
for r in $(seq $N); do
  for L in "$A" "$B"; do
    RTG_LIB=$L timeout -k 10 200 python bench.py --config $C --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null \
      | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$(basename $L)', d['kernel_ms'], d['parity'].get('fb_md5_match'))" || exit 1
  done
done
