#!/usr/bin/env bash
# tools/final_check.sh [LIB...] — one GPU call: an optional same-box A/B of
# librtg builds (C3), the GPU parity tests, smoke() and the round evidence set
# (tools/round_profiles.sh).  Every GPU step has its own time limit; the chain
# stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ $# -gt 0 ]; then
  bash tools/ab_bench.sh -r 3 -c c3 "$@" > gpurun_out/ab_final_c3.log 2>&1 && cat gpurun_out/ab_final_c3.log || exit 1
fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1 && tail -2 gpurun_out/pytest_gpu_final.log &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 && tail -3 gpurun_out/smoke_final.log &&
TAG=r02 bash tools/round_profiles.sh
