#!/usr/bin/env bash
# oracle/build_ref_cl.sh — TEST INFRASTRUCTURE: compile the reference's own
# OpenCL kernel (raytrace_kernel.cl, in place under /root/reference) for
# gfx950 with clang's OpenCL C front end and the ROCm device libraries, through
# the harness oracle/ref_cl_harness.cl, into oracle/_ref/rtg_ref_cl.hsaco.
# The tests load it as a HIP module (tests/clref.py) and check the
# OpenCL-semantics oracle and the kernel's kCL mode against it bit for bit.
#
# Arithmetic contract: IEEE f32 with correctly rounded division and square
# root (-cl-fp32-correctly-rounded-divide-sqrt) and no contraction
# (-ffp-contract=off): the strict instantiation of the kernel's source.
# Deterministic recipe: the kernel reads bgMaterial.opacity uninitialised,
# as the CPU path does (raytrace_kernel.cl:939-942 and :518-521 set matte,
# gloss and the index only); -ftrivial-auto-var-init=zero makes it 0, the
# same recipe as build_ref.sh's CPU build.  (The
# image the author's GPU produced, testPPM.ppm, used OpenCL's default relaxed
# division / sqrt and contraction; that one is not reproducible bit for bit.)
# Nothing here runs on the GPU box (no /root/reference there); the code
# object travels with the snapshot (oracle/_ref is git-ignored, not
# gpurun-ignored).
set -euo pipefail
REF=${RTG_REFERENCE:-/root/reference/raytracer_gamma}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT="$HERE/_ref"
CLANG=${CLANG_CL:-/opt/rocm/llvm/bin/clang}
if [ ! -f "$REF/raytrace_kernel.cl" ]; then
  echo "build_ref_cl: reference not present at $REF (expected on the GPU box); skipping" >&2
  exit 0
fi
mkdir -p "$OUT"
co="$OUT/rtg_ref_cl.hsaco"
if [ -f "$co" ] && [ "$co" -nt "$HERE/ref_cl_harness.cl" ] && [ "$co" -nt "$0" ]; then
  exit 0
fi
$CLANG -x cl -cl-std=CL1.2 -Xclang -finclude-default-header -target amdgcn-amd-amdhsa \
  -mcpu=gfx950 -O2 -cl-fp32-correctly-rounded-divide-sqrt -ffp-contract=off \
  -ftrivial-auto-var-init=zero -w -I"$REF" "$HERE/ref_cl_harness.cl" -o "$co"
echo "built $co"
