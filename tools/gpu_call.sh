#!/usr/bin/env bash
# tools/gpu_call.sh TAG STEP... — one gpurun call's worth of GPU steps, each
# under its own time limit, stopping at the first failure.  Output goes to
# gpurun_out/TAG/.  Steps (run in the order given):
#   ab:CFG:ROUNDS:LIB1,LIB2,...   interleaved same-box A/B (tools/ab_bench.sh)
#   pmc:CFG[:LIB]                 PMC passes (tools/gpu_pmc.sh), optional library
#   sqc:CFG[:LIB]                 scalar-cache hit/miss pass
#   tests                         the GPU test tier
#   bench:CFG[:EXTRA_ARGS]        one default bench line (the shipped library)
#   prof:CFG                      rocprofv3 --kernel-trace --stats of a bench run
#   calib                         unit-cost calibration data (tools/calib_units.py --collect)
#   chunks:CFG[:RANKS[:CHUNKS]]   one rank's chunked shard (tools/chunk_rehearsal.py)
# Replaces round 5's per-call wrappers (tools/r05*_call.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
TAG=${1:?tag}
shift
O=$ROOT/gpurun_out/$TAG
mkdir -p "$O"
lib_path() { case $1 in /*) echo "$1" ;; *) echo "$ROOT/ab/librtg_$1.so" ;; esac; }
for step in "$@"; do
  IFS=':' read -r kind a b c <<< "$step"
  echo "== $step $(date +%T)"
  case $kind in
    ab)
      libs=()
      IFS=',' read -ra names <<< "$c"
      for n in "${names[@]}"; do libs+=("$(lib_path "$n")"); done
      STEPS=${STEPS:-10} bash tools/ab_bench.sh -r "$b" -c "$a" "${libs[@]}" > "$O/ab_$a.log" 2>&1 || { cat "$O/ab_$a.log"; exit 1; }
      cat "$O/ab_$a.log" ;;
    pmc)
      lib=""; [ -n "$b" ] && lib=$(lib_path "$b")
      RTG_LIB=$lib TAG="$TAG/pmc_${a}_${b:-shipped}" CFG=$a bash tools/gpu_pmc.sh > "$O/pmc_${a}_${b:-shipped}.log" 2>&1 || { tail -20 "$O/pmc_${a}_${b:-shipped}.log"; exit 1; }
      tail -25 "$O/pmc_${a}_${b:-shipped}.log" ;;
    sqc)
      lib=""; [ -n "$b" ] && lib=$(lib_path "$b")
      d=$O/sqc_${a}_${b:-shipped}
      ( cd /tmp && export TMPDIR=/tmp && RTG_LIB=$lib timeout -s KILL 240 rocprofv3 --pmc SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_INSTS_SMEM SQ_INSTS_VMEM \
          --output-format csv -d "$d" -o run -- python3 "$ROOT/bench.py" --config "$a" --steps 1 --warmup 1 \
          --no-cpu-baseline --no-work-count --no-e2e > "$d.json" 2> "$d.err" ) || { tail -5 "$d.err"; exit 1; }
      python3 tools/pmc_kernel_avg.py "$d" "$d.json" | tee "$d.txt" ;;
    calib)
      # tools/calib_units.py --collect under the SQ_INSTS_VALU counter
      ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 600 rocprofv3 --pmc SQ_INSTS_VALU --output-format csv \
          -d "$O/calib" -o run -- python3 "$ROOT/tools/calib_units.py" --collect "$O/calib" > "$O/calib.log" 2>&1 ) \
        || { tail -20 "$O/calib.log"; exit 1; }
      tail -3 "$O/calib.log" ;;
    chunks)
      timeout -k 10 300 python tools/chunk_rehearsal.py --config "$a" --ranks "${b:-8,4,2}" --chunks "${c:-1,3,4}" \
        --last-frac 0.15 --steps 20 --json "$O/chunks_$a.json" > "$O/chunks_$a.txt" 2>&1 || { tail -5 "$O/chunks_$a.txt"; exit 1; }
      cat "$O/chunks_$a.txt" | grep config ;;
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
      tail -5 "$O/pytest_gpu.log" ;;
    bench)
      timeout -k 10 600 python bench.py --config "$a" ${b:-} > "$O/bench_$a.json" 2> "$O/bench_$a.err" || { tail -20 "$O/bench_$a.err"; exit 1; }
      cat "$O/bench_$a.json" ;;
    prof)
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$O/prof_$a" -o run -- python3 "$ROOT/bench.py" --config "$a" > "$O/prof_bench_$a.json" 2> "$O/prof_bench_$a.err" ) \
        || { tail -20 "$O/prof_bench_$a.err"; exit 1; }
      python3 tools/timed_stats.py "$O/prof_$a" "$O/prof_bench_$a.json" "$O/timed_stats_$a" > "$O/timed_stats_$a.txt" 2>&1 || true
      cat "$O/timed_stats_$a.txt" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== all steps done $(date +%T)"
