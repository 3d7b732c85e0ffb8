#!/bin/bash
# Build the kernel library of another git revision as an A/B variant:
#   tools/build_rev.sh <rev> <variant> [EXTRA flags]  ->  simple-raytracer_amd/lib_<variant>/
set -eu
cd "$(dirname "$0")/.."
rev=$1; var=$2; shift 2
d=$(mktemp -d /tmp/rtrev.XXXXXX)
git show "$rev:simple-raytracer_amd/csrc/rt_kernels.hip" > "$d/rt_kernels.hip"
git show "$rev:simple-raytracer_amd/csrc/rt_bvh.h" > "$d/rt_bvh.h"
make -C simple-raytracer_amd VARIANT="$var" KSRC="$d/rt_kernels.hip" EXTRA="${*:-}" -B -j8 >/dev/null
rm -rf "$d"
echo "built simple-raytracer_amd/lib_$var from $rev"
