#!/bin/bash
# Round-4 GPU session 8: segment order (option order: costliest segments
# first) -- GPU suite, A/B on C3 / C5, the executed-test counters' cost,
# timelines of the ordered frame, N=8 rank shares.
set -e
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s8
O=gpurun_out/s8
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1
timeout -k 10 500 python -u tools/ab.py --rounds 3 --steps 20 --config C3 def: o0::order=0 nt:lib_notests: ns:lib_nostats:order=0 base:lib_base: > $O/ab_C3.txt 2>&1
timeout -k 10 300 python -u tools/ab.py --rounds 2 --steps 3 --config C5 def: o0::order=0 > $O/ab_C5.txt 2>&1
timeout -k 10 200 python -u tools/ab.py --rounds 2 --steps 300 --config C2 def: base:lib_base: > $O/ab_C2.txt 2>&1
export RTAMD_LIB_DIR=$PWD/simple-raytracer_amd/lib_prof
timeout -k 10 120 python -u tools/timeline.py C3 > $O/tl_C3.txt 2>&1
timeout -k 10 120 python -u tools/timeline.py C3 --rows 8:0 > $O/tl_C3_r8.txt 2>&1
timeout -k 10 120 python -u tools/timeline.py C3 --rows 8:0 order=0 > $O/tl_C3_r8_o0.txt 2>&1
unset RTAMD_LIB_DIR
timeout -k 10 200 python -u tools/rank_balance.py C3 > $O/rb_C3.txt 2>&1
timeout -k 10 200 python -u tools/rank_balance.py C3 --option order=0 > $O/rb_C3_o0.txt 2>&1
timeout -k 10 200 python -u tools/rank_balance.py C4 > $O/rb_C4.txt 2>&1
