#!/usr/bin/env bash
# tools/r03_ab_memset.sh — GPU tests on the in-tree build, then the A/B of
# one memset per compacted launch (ab/librtg_z.so: the trace kernel zeroes
# the next launch's cost sum) against the previous build (ab/librtg_head.so)
# on the C3/C4 frames and 1/8 shards (tools/order_ab.py), and C3 shard
# timelines.  Each GPU step has its own time limit; the chain stops at the
# first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab_memset}
mkdir -p $OUT
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for c in c3 c4; do
    for L in head z; do
      RTG_LIB=$PWD/ab/librtg_$L.so timeout -k 10 300 python tools/order_ab.py --config $c | tee -a $OUT/ab.jsonl || exit 1
    done
  done
done
timeout -k 10 200 python tools/timeline.py --config c3 --waves-per-block 1 --shard 0 --shards 8 --json $OUT/c3_s0of8.json --raw $OUT/c3_s0of8.npz > /dev/null || exit 1
echo "== done"
