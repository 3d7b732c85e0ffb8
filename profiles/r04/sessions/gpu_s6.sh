#!/bin/bash
# Round-4 GPU session 6: the exit-time stats atomics (probe library without
# them), suspended searches (options suspend_active / suspend_done).
set -e
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s6
O=gpurun_out/s6
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "suspend_bit_identical" > $O/pytest.log 2>&1
timeout -k 10 300 python -u tools/ab.py --rounds 2 --steps 300 --config C2 def: nostats:lib_nostats: copies:lib_copies: s8::suspend_active=8,suspend_done=32 > $O/ab_C2.txt 2>&1
timeout -k 10 500 python -u tools/ab.py --rounds 3 --steps 20 --config C3 def: nostats:lib_nostats: copies:lib_copies: s4::suspend_active=4,suspend_done=16 s8::suspend_active=8,suspend_done=32 s16::suspend_active=16,suspend_done=32 s8d16::suspend_active=8,suspend_done=16 s24::suspend_active=24,suspend_done=24 > $O/ab_C3.txt 2>&1
timeout -k 10 300 python -u tools/ab.py --rounds 2 --steps 3 --config C5 def: nostats:lib_nostats: copies:lib_copies: s8::suspend_active=8,suspend_done=32 > $O/ab_C5.txt 2>&1
RTAMD_LIB_DIR=$PWD/simple-raytracer_amd/lib_prof timeout -k 10 200 python -u tools/prof_phases.py C3 > $O/ph_C3.txt 2>&1
RTAMD_LIB_DIR=$PWD/simple-raytracer_amd/lib_prof timeout -k 10 200 python -u tools/prof_phases.py C3 suspend_active=8 suspend_done=32 > $O/ph_C3_s8.txt 2>&1
