#!/usr/bin/env bash
# tools/ab_bench.sh [-r ROUNDS] [-c CONFIG] LIB... — interleaved same-box A/B of
# librtg.so builds on a bench config (kernel ms from HIP events per run, and
# whether the frame's md5 matches the golden one).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=4
C=c3
while getopts "r:c:" o; do
  case $o in
    r) N=$OPTARG ;;
    c) C=$OPTARG ;;
    *) exit 2 ;;
  esac
done
shift $((OPTIND - 1))
for r in $(seq "$N"); do
  for L in "$@"; do
    RTG_LIB=$L timeout -k 10 200 python bench.py --config "$C" --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline \
        --no-work-count --no-e2e 2>>gpurun_out/ab_bench.err \
      | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$C', '$(basename "$L")', d['kernel_ms'], d['parity'].get('bit_exact'), flush=True)" || exit 1
  done
done
