#!/bin/bash
# Round-4 GPU session 13: no hold of reflection / refraction searches once a
# wave's work is drained (lib_gd0) -- C3, C5 and the N=8 C3 share.
set -e
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s13
O=gpurun_out/s13
timeout -k 10 400 python -u tools/ab.py --rounds 3 --steps 20 --config C3 def: gd0:lib_gd0: > $O/ab_C3.txt 2>&1
timeout -k 10 300 python -u tools/ab.py --rounds 2 --steps 3 --config C5 def: gd0:lib_gd0: > $O/ab_C5.txt 2>&1
timeout -k 10 150 python -u tools/rank_balance.py C3 --ns 1,8 --rank-only 0 > $O/rb8_def.txt 2>&1
RTAMD_LIB_DIR=$PWD/simple-raytracer_amd/lib_gd0 timeout -k 10 150 python -u tools/rank_balance.py C3 --ns 1,8 --rank-only 0 > $O/rb8_gd0.txt 2>&1
timeout -k 10 150 python -u tools/rank_balance.py C3 --ns 1,8 --rank-only 3 > $O/rb8_def_r3.txt 2>&1
RTAMD_LIB_DIR=$PWD/simple-raytracer_amd/lib_gd0 timeout -k 10 150 python -u tools/rank_balance.py C3 --ns 1,8 --rank-only 3 > $O/rb8_gd0_r3.txt 2>&1
