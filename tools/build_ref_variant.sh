#!/bin/bash
# Build libforma_rt from the kernel sources of a git revision, for A/B timing against the
# working tree (tools/ab_bench.py):
#   tools/build_ref_variant.sh REV NAME [DEFS]  ->  fo-rma_amd/build/ab/libforma_rt_NAME.so (shipped to the GPU box; delete after the A/B session)
# REV "." takes the working tree's sources (for -D variants of uncommitted code).
# The host objects (scene, JSON, BVH, post) come from the working tree's build; the ABI of
# REV must match the working tree's include/forma_rt.h.
set -e
rev=$1; name=$2; defs=${3:-}
root="$(cd "$(dirname "$0")/.." && pwd)"
tmp=$(mktemp -d)
trap 'rm -rf "$tmp"' EXIT
mkdir -p "$tmp/fo-rma_amd/csrc" "$tmp/include"
if [ "$rev" = "." ]; then
  cp -r "$root/fo-rma_amd/csrc" "$tmp/fo-rma_amd/" && cp -r "$root/include" "$tmp/"
else
  git -C "$root" archive "$rev" fo-rma_amd/csrc include | tar -x -C "$tmp"
fi
make -C "$root/fo-rma_amd" -s build/scene.o build/json_min.o build/bvh.o build/post.o build/jit_cache.o
mkdir -p "$root/fo-rma_amd/build/ab"
# the scene-specialised kernel is compiled at run time from the sources embedded in jit.o:
# embed REV's trace_kernel.h (and what it includes), so the A/B covers the hiprtc kernel too
c="$tmp/fo-rma_amd/csrc"
mkdir -p "$tmp/fo-rma_amd/build"
python3 "$c/embed_sources.py" "$tmp/fo-rma_amd/build/jit_sources.inc" trace_kernel.h="$c/trace_kernel.h" \
  rt_core.h="$c/rt_core.h" bvh.h="$c/bvh.h" forma_rt.h="$tmp/include/forma_rt.h"
g++ -O2 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function $defs -D__HIP_PLATFORM_AMD__ \
  -I/opt/rocm/include -c "$c/jit.cpp" -o "$tmp/jit.o"
FP="-ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $FP -fno-slp-vectorize $defs \
  -c "$tmp/fo-rma_amd/csrc/render.hip" -o "$tmp/render.o"
objs="$tmp/render.o"
if [ -f "$tmp/fo-rma_amd/csrc/sum.hip" ]; then  # sum_kernel's own unit (round 4 on)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $FP -fno-slp-vectorize $defs \
    -c "$tmp/fo-rma_amd/csrc/sum.hip" -o "$tmp/sum.o"
  objs="$objs $tmp/sum.o"
fi
b="$root/fo-rma_amd/build"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$b/ab/libforma_rt_$name.so" $objs \
  "$b/scene.o" "$b/json_min.o" "$b/bvh.o" "$b/post.o" "$b/jit_cache.o" "$tmp/jit.o" -L/opt/rocm/lib -lhiprtc -Wl,-rpath,/opt/rocm/lib
echo "$b/ab/libforma_rt_$name.so"
