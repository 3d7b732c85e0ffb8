#!/bin/bash
# Round-4 GPU session 3: which part of the work-band change costs C3 --
# bands + static first batch (lib), static only (work_parts=1), bands only
# (lib_nostatic), neither (lib_nostatic work_parts=1), round-4 HEAD before
# them (lib_nb); C2 and the N=8 C3 share likewise.
set -e
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s3
O=gpurun_out/s3
timeout -k 10 420 python -u tools/ab.py --rounds 3 --steps 100 --config C3 both: static::work_parts=1 bands:lib_nostatic neither:lib_nostatic:work_parts=1 nb:lib_nb > $O/ab_C3.txt 2>&1
timeout -k 10 300 python -u tools/ab.py --rounds 2 --steps 300 --config C2 both: static::work_parts=1 bands:lib_nostatic neither:lib_nostatic:work_parts=1 > $O/ab_C2.txt 2>&1
timeout -k 10 200 python -u tools/rank_balance.py C3 --ns 8 > $O/bal8_both.txt 2>&1
timeout -k 10 200 python -u tools/rank_balance.py C3 --ns 8 --option work_parts=1 > $O/bal8_static.txt 2>&1
RTAMD_LIB_DIR=$PWD/simple-raytracer_amd/lib_nostatic timeout -k 10 200 python -u tools/rank_balance.py C3 --ns 8 --option work_parts=1 > $O/bal8_neither.txt 2>&1
RTAMD_LIB_DIR=$PWD/simple-raytracer_amd/lib_nb timeout -k 10 200 python -u tools/rank_balance.py C3 --ns 8 > $O/bal8_nb.txt 2>&1
