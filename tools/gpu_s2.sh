#!/bin/bash
# Round-4 GPU session 2: per-XCD work bands + static first batch (lib) against
# the same library without them (lib_nb, HEAD) and round 3's (lib_r3).
set -e
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s2
O=gpurun_out/s2
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "refill or row_blocks or c2_full or render_pixels or origin_leaf or frames_in_flight or multi_rank" --timeout 240 --timeout-method thread > $O/pytest_sel.log 2>&1
timeout -k 10 300 python -u tools/ab.py --rounds 3 --steps 300 --config C2 bands: nb:lib_nb r3:lib_r3 bands1::work_parts=1 > $O/ab_C2.txt 2>&1
timeout -k 10 300 python -u tools/ab.py --rounds 3 --steps 100 --config C3 bands: nb:lib_nb r3:lib_r3 > $O/ab_C3.txt 2>&1
timeout -k 10 300 python -u tools/rank_balance.py C3 --ns 1,8 > $O/bal_C3_bands.txt 2>&1
RTAMD_LIB_DIR=$PWD/simple-raytracer_amd/lib_nb timeout -k 10 300 python -u tools/rank_balance.py C3 --ns 1,8 > $O/bal_C3_nb.txt 2>&1
timeout -k 10 300 python -u tools/rank_balance.py C4 --ns 1,8 > $O/bal_C4_bands.txt 2>&1
RTAMD_LIB_DIR=$PWD/simple-raytracer_amd/lib_prof timeout -k 10 120 python -u tools/timeline.py C2 > $O/tl_C2.txt 2>&1
RTAMD_LIB_DIR=$PWD/simple-raytracer_amd/lib_prof timeout -k 10 120 python -u tools/timeline.py C3 --rows 8:0 > $O/tl_C3_r8.txt 2>&1
timeout -k 10 400 python -u tools/ab.py --rounds 2 --steps 4 --config C5 bands: nb:lib_nb > $O/ab_C5.txt 2>&1
timeout -k 10 300 python -u tools/ab.py --rounds 2 --steps 30 --config C4 bands: nb:lib_nb > $O/ab_C4.txt 2>&1
