#!/bin/bash
# Round-4 GPU session 10: the last light's zero-Phong skip (lib_ll1 vs
# lib_ll0) -- GPU suite on lib_ll1, A/B on C3 / C4 / C5; the work bands after
# the exit-counter fix (work_parts=1 against auto) on C2 / C3 / C4.
set -e
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s10
O=gpurun_out/s10
RTAMD_LIB_DIR=$PWD/simple-raytracer_amd/lib_ll1 timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/pytest_ll1.log 2>&1
timeout -k 10 500 python -u tools/ab.py --rounds 3 --steps 20 --config C3 ll0:lib_ll0: ll1:lib_ll1: ll0p1:lib_ll0:work_parts=1 > $O/ab_C3.txt 2>&1
timeout -k 10 400 python -u tools/ab.py --rounds 3 --steps 20 --config C4 ll0:lib_ll0: ll1:lib_ll1: ll0p1:lib_ll0:work_parts=1 > $O/ab_C4.txt 2>&1
timeout -k 10 300 python -u tools/ab.py --rounds 2 --steps 3 --config C5 ll0:lib_ll0: ll1:lib_ll1: > $O/ab_C5.txt 2>&1
timeout -k 10 200 python -u tools/ab.py --rounds 3 --steps 300 --config C2 ll0:lib_ll0: ll0p1:lib_ll0:work_parts=1 > $O/ab_C2.txt 2>&1
