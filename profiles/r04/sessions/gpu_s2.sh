#!/bin/bash
# Round-4 GPU session 2: per-XCD work bands + static first batch + scalar
# shadow mask (lib) against the library before them (lib_nb) and round 3's
# (lib_r3); the shadow-ray helpers (lib_help, RT_SHADOW_HELP=1).
set -e
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s2
O=gpurun_out/s2
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "refill or row_blocks or c2_full or render_pixels or origin_leaf or frames_in_flight or multi_rank" --timeout 240 --timeout-method thread > $O/pytest_sel.log 2>&1
rc=0
RTAMD_LIB_DIR=$PWD/simple-raytracer_amd/lib_help timeout -k 10 300 python -u -m pytest tests/test_float_goldens.py tests/test_gpu_parity.py -x -q -m gpu -k "reference_floats or refill or render_pixels or directional or special or test7" --timeout 240 --timeout-method thread > $O/pytest_help.log 2>&1 || rc=$?
# test failures (1) are results; anything else (a fault, an abort, a time limit) ends the session
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/ab.py --rounds 2 --steps 300 --config C2 bands: nb:lib_nb bands1::work_parts=1 > $O/ab_C2.txt 2>&1
timeout -k 10 360 python -u tools/ab.py --rounds 3 --steps 100 --config C3 bands: nb:lib_nb help:lib_help > $O/ab_C3.txt 2>&1
timeout -k 10 300 python -u tools/rank_balance.py C3 --ns 1,8 > $O/bal_C3_bands.txt 2>&1
RTAMD_LIB_DIR=$PWD/simple-raytracer_amd/lib_prof timeout -k 10 120 python -u tools/timeline.py C2 > $O/tl_C2.txt 2>&1
