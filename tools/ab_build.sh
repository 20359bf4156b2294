#!/usr/bin/env bash
# tools/ab_build.sh REV — build librtg.so of git revision REV into
# ab/librtg_REV.so (a scratch git worktree under /tmp), for same-box A/B runs:
#   RTG_LIB=$PWD/ab/librtg_REV.so python bench.py ...
set -euo pipefail
REV=${1:?revision}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=/tmp/rtg_ab_$REV
rm -rf "$WT"
git -C "$ROOT" worktree prune
git -C "$ROOT" worktree add --detach "$WT" "$REV" > /dev/null
make -s -j"${JOBS:-8}" -C "$WT/raytracer-gamma_amd" ARCH=gfx950 librtg.so
mkdir -p "$ROOT/ab"
cp "$WT/raytracer-gamma_amd/librtg.so" "$ROOT/ab/librtg_$REV.so"
git -C "$ROOT" worktree remove --force "$WT"
echo "built $ROOT/ab/librtg_$REV.so"
