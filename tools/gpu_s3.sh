#!/bin/bash
# Round-4 GPU session 3: shadow-ray helpers (lib_help: RT_SHADOW_HELP=1) --
# parity against the reference's floats and the oracle, then A/B speed.
set -e
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s3
O=gpurun_out/s3
H=$PWD/simple-raytracer_amd/lib_help
RTAMD_LIB_DIR=$H timeout -k 10 400 python -u -m pytest tests/test_float_goldens.py tests/test_gpu_parity.py -x -q -m gpu -k "reference_floats or c3 or C3 or test7 or depth or special or many_lights or directional or c2_full" --timeout 240 --timeout-method thread > $O/pytest_help.log 2>&1 || rc=$?
# test failures (1) are results; anything else (a fault, an abort, a time limit) ends the session
if [ "${rc:-0}" -ne 0 ] && [ "${rc:-0}" -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/ab.py --rounds 3 --steps 100 --config C3 bands: help:lib_help > $O/ab_C3.txt 2>&1
timeout -k 10 300 python -u tools/ab.py --rounds 2 --steps 50 --config C3D bands: help:lib_help > $O/ab_C3D.txt 2>&1
timeout -k 10 300 python -u tools/ab.py --rounds 2 --steps 30 --config C4 bands: help:lib_help > $O/ab_C4.txt 2>&1
timeout -k 10 400 python -u tools/ab.py --rounds 2 --steps 4 --config C5 bands: help:lib_help > $O/ab_C5.txt 2>&1
