#!/bin/bash
# Round-4 GPU session 10: all counters behind the counting instantiation
# (option counters; bench times the one without) -- GPU suite; the last
# light's zero-Phong skip (lib = on, lib_ll0 = off) on C3 / C4 / C5; the
# work bands after the exit-counter fix; the N=8 C3 share.
set -e
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s10
O=gpurun_out/s10
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1
timeout -k 10 500 python -u tools/ab.py --rounds 3 --steps 20 --config C3 ll1: ll0:lib_ll0: p1::work_parts=1 > $O/ab_C3.txt 2>&1
timeout -k 10 400 python -u tools/ab.py --rounds 3 --steps 20 --config C4 ll1: ll0:lib_ll0: p1::work_parts=1 > $O/ab_C4.txt 2>&1
timeout -k 10 300 python -u tools/ab.py --rounds 2 --steps 3 --config C5 ll1: ll0:lib_ll0: > $O/ab_C5.txt 2>&1
timeout -k 10 200 python -u tools/ab.py --rounds 3 --steps 300 --config C2 ll1: p1::work_parts=1 > $O/ab_C2.txt 2>&1
timeout -k 10 300 python -u tools/rank_balance.py C3 > $O/rb_C3.txt 2>&1
