#!/usr/bin/env bash
# r05ae: short launches (one rank's shard of a 4- and 8-way frame in chunks,
# tools/chunk_rehearsal.py) with the group list in 16 partitions vs one
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05ae; mkdir -p $O
for r in 1 2; do
  for L in p1 base; do
    for c in c3 c4; do
      RTG_LIB=$PWD/ab/librtg_$L.so timeout -k 10 300 python tools/chunk_rehearsal.py --config $c --ranks 4,8 --chunks 3 --last-frac 0.15 --steps 10 \
        > $O/chunks_${L}_${c}_$r.txt 2>> $O/err.log || exit 1
      echo "== $L $c round $r"; tail -4 $O/chunks_${L}_${c}_$r.txt
    done
  done
done
