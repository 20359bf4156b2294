#!/usr/bin/env bash
# tools/ab_build.sh REV [NAME] — build librtg.so of git revision REV into
# ab/librtg_NAME.so (NAME defaults to REV; a scratch git worktree under /tmp),
# for same-box A/B runs:   RTG_LIB=$PWD/ab/librtg_NAME.so python bench.py ...
# Compiler-setting trials: EXTRA="-O2" tools/ab_build.sh HEAD o2 (EXTRA is
# appended to the Makefile's HIPFLAGS).
set -euo pipefail
REV=${1:?revision}
NAME=${2:-$REV}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=/tmp/rtg_ab_$NAME
rm -rf "$WT"
git -C "$ROOT" worktree prune
git -C "$ROOT" worktree add --detach "$WT" "$REV" > /dev/null
make -s -j"${JOBS:-8}" -C "$WT/raytracer-gamma_amd" ARCH=gfx950 AB="${AB:-0}" EXTRA="${EXTRA:-}" librtg.so
mkdir -p "$ROOT/ab"
cp "$WT/raytracer-gamma_amd/librtg.so" "$ROOT/ab/librtg_$NAME.so"
git -C "$ROOT" worktree remove --force "$WT"
echo "built $ROOT/ab/librtg_$NAME.so"
