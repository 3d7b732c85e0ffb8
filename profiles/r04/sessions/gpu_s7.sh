#!/bin/bash
# Round-4 GPU session 7: the exit counters spread over 16 copies (one memory
# channel each) -- GPU suite, then A/B against the previous library (base), a
# probe without exit counters (nostats) and the spill count by atomics (spillat).
set -e
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s7
O=gpurun_out/s7
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1
timeout -k 10 300 python -u tools/ab.py --rounds 2 --steps 300 --config C2 def: base:lib_base: nostats:lib_nostats: spillat:lib_spillat: > $O/ab_C2.txt 2>&1
timeout -k 10 400 python -u tools/ab.py --rounds 3 --steps 20 --config C3 def: base:lib_base: nostats:lib_nostats: spillat:lib_spillat: > $O/ab_C3.txt 2>&1
timeout -k 10 300 python -u tools/ab.py --rounds 2 --steps 3 --config C5 def: base:lib_base: spillat:lib_spillat: > $O/ab_C5.txt 2>&1
