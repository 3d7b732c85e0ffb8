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
# A/B: this library against round 3's final kernel (lib_r3, tools/build_rev.sh 268f298 r3)
timeout -k 10 300 python -u tools/ab.py --rounds 3 --steps 100 --config C3 head: r3:lib_r3 > gpurun_out/ab_r4_vs_r3_C3.txt 2>&1
timeout -k 10 300 python -u tools/ab.py --rounds 3 --steps 200 --config C2 head: r3:lib_r3 chunk256::chunk=256 chunk1024::chunk=1024 > gpurun_out/ab_C2_chunk.txt 2>&1
timeout -k 10 400 python -u tools/ab.py --rounds 2 --steps 4 --config C5 head: r3:lib_r3 > gpurun_out/ab_r4_vs_r3_C5.txt 2>&1
