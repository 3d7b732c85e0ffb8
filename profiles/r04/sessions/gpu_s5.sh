#!/bin/bash
# Round-4 GPU session 5: hot copies of the BVH's top (option hot_copies) --
# bit identity, then A/B on C2 / C3 / C5 and the N=8 C3 rank share.
set -e
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s5
O=gpurun_out/s5
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "bands_and_hot or refill_options or lds_stack" > $O/pytest.log 2>&1
timeout -k 10 300 python -u tools/ab.py --rounds 2 --steps 300 --config C2 def: h4::hot_copies=4 h16::hot_copies=16 h64::hot_copies=64 h16p1::hot_copies=16,work_parts=1 > $O/ab_C2.txt 2>&1
timeout -k 10 400 python -u tools/ab.py --rounds 3 --steps 20 --config C3 def: h16::hot_copies=16 h64::hot_copies=64 p1::work_parts=1 h16p1::hot_copies=16,work_parts=1 > $O/ab_C3.txt 2>&1
timeout -k 10 300 python -u tools/ab.py --rounds 2 --steps 3 --config C5 def: h16::hot_copies=16 > $O/ab_C5.txt 2>&1
timeout -k 10 200 python -u tools/rank_balance.py C3 --option hot_copies=16 > $O/rb_C3_h16.txt 2>&1
timeout -k 10 200 python -u tools/rank_balance.py C3 --option hot_copies=16 --option work_parts=1 > $O/rb_C3_h16p1.txt 2>&1
