#!/bin/bash
# Build the kernel library of another git revision as an A/B variant:
#   tools/build_rev.sh <rev> <variant> [EXTRA flags]  ->  simple-raytracer_amd/lib_<variant>/
set -eu
cd "$(dirname "$0")/.."
rev=$1; var=$2; shift 2
d=$(mktemp -d /tmp/rtrev.XXXXXX)
git archive "$rev" simple-raytracer_amd/csrc include | tar -x -C "$d"
c="$d/simple-raytracer_amd/csrc"
if [ -f "$c/rt_accel.cpp" ]; then
  make -C simple-raytracer_amd VARIANT="$var" SRC="$c" INC="$d/include" EXTRA="${*:-}" -B -j8 >/dev/null
elif [ -f "$c/rt_scene.cpp" ]; then   # before the host BVH build moved to rt_accel.cpp (round 4)
  make -C simple-raytracer_amd VARIANT="$var" SRC="$c" INC="$d/include" KSRC="$c/rt_kernels.hip $c/rt_scene.cpp" \
       KDEPS="$c/rt_kernels.hip $c/rt_scene.cpp $c/rt_device.h $c/rt_bvh.h" EXTRA="${*:-}" -B -j8 >/dev/null
else   # before the host side moved out of rt_kernels.hip
  make -C simple-raytracer_amd VARIANT="$var" SRC="$d/simple-raytracer_amd/csrc" KSRC="$d/simple-raytracer_amd/csrc/rt_kernels.hip" \
       KDEPS="$d/simple-raytracer_amd/csrc/rt_kernels.hip" INC="$d/include" EXTRA="${*:-}" -B -j8 >/dev/null
fi
rm -rf "$d"
echo "built simple-raytracer_amd/lib_$var from $rev"
