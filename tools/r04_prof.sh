#!/usr/bin/env bash
# tools/r04_prof.sh — rocprofv3 kernel traces of the bench command for the
# configs in CONFIGS (default c2 c5), each cut to its timed launches by
# tools/timed_stats.py.  One GPU step per config, each with its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04p}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for c in ${CONFIGS:-c2 c5}; do
  echo "== rocprofv3 kernel trace ($c bench)"
  ( cd /tmp && export TMPDIR=/tmp &&
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof_$c" -o run \
      -- python3 "$GRAFT_REPO_ROOT/bench.py" --config $c --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline \
      > "$GRAFT_REPO_ROOT/$OUT/bench_prof_$c.json" 2> "$GRAFT_REPO_ROOT/$OUT/bench_prof_$c.err" ) || exit 1
  python tools/timed_stats.py $OUT/prof_$c $OUT/bench_prof_$c.json $OUT/timed_stats_$c || exit 1
done
echo "== all done"
