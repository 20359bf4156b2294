#!/usr/bin/env bash
# tools/r04_probe.sh — round-4 diagnostics in one GPU call: the facing-away
# A/B (>= 4 interleaved rounds), the C5 probe-build cycle
# shares (variant 110, an AB=1 library), the C2 wave timeline and C2 PMC.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04d}
mkdir -p $OUT
echo "== A/B facing c3" && STEPS=20 bash tools/ab_bench.sh -r 5 -c c3 ab/librtg_head.so ab/librtg_noface.so > $OUT/ab_face_c3.log 2>&1; cat $OUT/ab_face_c3.log
echo "== A/B facing c4" && STEPS=5 bash tools/ab_bench.sh -r 4 -c c4 ab/librtg_head.so ab/librtg_noface.so > $OUT/ab_face_c4.log 2>&1; cat $OUT/ab_face_c4.log
echo "== C5 probe shares" &&
RTG_LIB=$PWD/ab/librtg_abv.so timeout -k 10 300 python bench.py --config c5 --steps 2 --warmup 1 --diag 110 --no-cpu-baseline --no-e2e --no-work-count > $OUT/diag_c5.json 2> $OUT/diag_c5.err; grep diag $OUT/diag_c5.err | tail -2
echo "== C3 probe shares" &&
RTG_LIB=$PWD/ab/librtg_abv.so timeout -k 10 300 python bench.py --config c3 --steps 5 --warmup 1 --diag 110 --no-cpu-baseline --no-e2e --no-work-count > $OUT/diag_c3.json 2> $OUT/diag_c3.err; grep diag $OUT/diag_c3.err | tail -2
echo "== C2 timeline" &&
timeout -k 10 300 python tools/timeline.py --config c2 --waves-per-block 1 --json $OUT/timeline_c2.json > $OUT/timeline_c2.log 2>&1; tail -12 $OUT/timeline_c2.log
echo "== C2 PMC" &&
TAG=${TAG:-r04d}_c2 CFG=c2 ARGS="--config c2 --steps 3 --warmup 1 --no-cpu-baseline --no-work-count --no-e2e" bash tools/gpu_pmc.sh > $OUT/pmc_c2.log 2>&1; tail -12 $OUT/pmc_c2.log
echo "== done"
