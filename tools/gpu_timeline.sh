#!/bin/bash
# Round-4 first GPU session: per-wave launch timelines (RT_PROF library) of
# C2, the N=8 shares of C3 / C4 and full C3; the GPU suite on the refactored
# library; a C3 bench line; the one-shot CLI runs (tools/e2e.py).
set -e
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export RTAMD_LIB_DIR=$PWD/simple-raytracer_amd/lib_prof
timeout -k 10 240 python -u tools/timeline.py C2 > gpurun_out/tl_C2.txt 2>&1
timeout -k 10 120 python -u tools/timeline.py C2 grid=256 > gpurun_out/tl_C2_g256.txt 2>&1
timeout -k 10 120 python -u tools/timeline.py C3 --rows 8:0 > gpurun_out/tl_C3_r8.txt 2>&1
timeout -k 10 120 python -u tools/timeline.py C3 > gpurun_out/tl_C3.txt 2>&1
timeout -k 10 120 python -u tools/timeline.py C4 --rows 8:0 > gpurun_out/tl_C4_r8.txt 2>&1
unset RTAMD_LIB_DIR
timeout -k 10 200 python -u bench.py --steps 20 --cpu-baseline off > gpurun_out/bench_C3_new.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 600 python -u tools/e2e.py C3 C4 C5 > gpurun_out/e2e.txt 2>&1
