#!/bin/bash
# Round-4 GPU session 12: the batching / leaf-postponement knobs re-swept on
# the kernel without counters (C3, C4).
set -e
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s12
O=gpurun_out/s12
timeout -k 10 600 python -u tools/ab.py --rounds 3 --steps 20 --config C3 def: lw1:lib_lw1: lw4:lib_lw4: rm24::refill_min=24 rm40::refill_min=40 gx24::gate_x=24 gx40::gate_x=40 > $O/ab_C3.txt 2>&1
timeout -k 10 300 python -u tools/ab.py --rounds 2 --steps 20 --config C4 def: lw1:lib_lw1: lw4:lib_lw4: > $O/ab_C4.txt 2>&1
