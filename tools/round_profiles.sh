#!/usr/bin/env bash
# tools/round_profiles.sh — the evidence set of a round on one GPU box:
# bench lines of every config, the rocprofv3 kernel-trace summary of the C3
# bench, the PMC passes (tools/gpu_pmc.sh) and the wave timeline.  Every GPU
# step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r02}
OUT=gpurun_out/$TAG
mkdir -p $OUT
echo "== bench c3 (default line)" &&
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > $OUT/bench_c3.json 2> $OUT/bench_c3.err &&
for c in c2 c4 c5; do
  echo "== bench $c" &&
  timeout -k 10 600 python bench.py --config $c --steps ${STEPS_OTHER:-5} --warmup 1 --no-cpu-baseline \
      > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit 1
done &&
echo "== rocprofv3 kernel trace (c3 bench)" &&
( cd /tmp && export TMPDIR=/tmp &&
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof_c3" -o run \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline \
    > "$GRAFT_REPO_ROOT/$OUT/bench_prof_c3.json" 2> "$GRAFT_REPO_ROOT/$OUT/bench_prof_c3.err" ) &&
echo "== timeline" &&
timeout -k 10 300 python tools/timeline.py --config c3 --waves-per-block 1 --json $OUT/timeline_c3.json > /dev/null &&
echo "== PMC" &&
TAG=$TAG bash tools/gpu_pmc.sh > $OUT/pmc.log 2>&1 &&
tail -8 $OUT/pmc.log &&
echo "== done"
