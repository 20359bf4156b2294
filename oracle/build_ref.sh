#!/usr/bin/env bash
# oracle/build_ref.sh — TEST INFRASTRUCTURE: build the reference CPU raytracer
# (raytracer.h, in place under /root/reference) into oracle/_ref/.
#
# Output: oracle/_ref/librtgref_S<S>.so for S in $STACKS (default 1..16).
# S = RTSTACK_MAXSIZE (raytraceStack.h:10) = depth + 1.
#   * S=6 is the reference as shipped: compiled straight from
#     /root/reference/raytracer_gamma with nothing changed.
#   * S!=6: raytraceStack.h hard-codes the capacity, so a copy of that ONE
#     header with the single `#define RTSTACK_MAXSIZE` line changed is written
#     to a scratch dir under /tmp and included ahead of raytracer.h (its include
#     guard then turns raytracer.h's own #include into a no-op); every other
#     file still comes from /root/reference.  Nothing is copied into the repo.
# Nothing here runs on the GPU box (no /root/reference there); the built .so
# files travel with the snapshot (oracle/_ref is git-ignored, not gpurun-ignored).
set -euo pipefail
REF=${RTG_REFERENCE:-/root/reference/raytracer_gamma}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT="$HERE/_ref"
CXX=${CXX_REF:-/opt/rocm/lib/llvm/bin/clang++}
STACKS=${STACKS:-"1 2 3 4 5 6 7 8 9 10 11 12 13 14 15 16"}
if [ ! -f "$REF/raytracer.h" ]; then
  echo "build_ref: reference not present at $REF (expected on the GPU box); skipping" >&2
  exit 0
fi
mkdir -p "$OUT"
FLAGS="-O2 -ffp-contract=off -ftrivial-auto-var-init=zero -DRSIZE_MAX=0x7FFFFFFF \
  -fPIC -shared -pthread -w -std=c++14"
for S in $STACKS; do
  lib="$OUT/librtgref_S$S.so"
  if [ -f "$lib" ] && [ "$lib" -nt "$HERE/ref_harness.cpp" ] && [ "$lib" -nt "$0" ]; then
    continue
  fi
  INC="-I$REF"
  if [ "$S" != "6" ]; then
    tmp=$(mktemp -d /tmp/rtgref_S$S.XXXX)
    sed "s/^#define RTSTACK_MAXSIZE 6\$/#define RTSTACK_MAXSIZE $S/" \
      "$REF/raytraceStack.h" > "$tmp/raytraceStack.h"
    grep -q "^#define RTSTACK_MAXSIZE $S\$" "$tmp/raytraceStack.h"
    INC="-I$REF -DRTG_STACK_HEADER=\"$tmp/raytraceStack.h\""
  fi
  $CXX $FLAGS $INC "$HERE/ref_harness.cpp" -o "$lib"
  [ "$S" != "6" ] && rm -rf "$tmp"
  echo "built $lib"
done
