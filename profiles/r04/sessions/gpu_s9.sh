#!/bin/bash
# Round-4 GPU session 9: the executed-test counters as a separate kernel
# instantiation (option count_tests, default off) -- GPU suite, A/B of the
# counting / non-counting / no-counter (nostats probe) kernels, a bench line.
set -e
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s9
O=gpurun_out/s9
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1
timeout -k 10 500 python -u tools/ab.py --rounds 3 --steps 20 --config C3 def: ct1::count_tests=1 ns:lib_nostats: > $O/ab_C3.txt 2>&1
timeout -k 10 300 python -u tools/ab.py --rounds 2 --steps 3 --config C5 def: ct1::count_tests=1 ns:lib_nostats: > $O/ab_C5.txt 2>&1
timeout -k 10 300 python -u tools/ab.py --rounds 2 --steps 20 --config C4 def: ct1::count_tests=1 ns:lib_nostats: > $O/ab_C4.txt 2>&1
timeout -k 10 200 python -u bench.py --steps 20 > $O/bench_C3.json 2> $O/bench_C3.err
timeout -k 10 300 python -u tools/rank_balance.py C3 > $O/rb_C3.txt 2>&1
timeout -k 10 300 python -u tools/rank_balance.py C4 > $O/rb_C4.txt 2>&1
