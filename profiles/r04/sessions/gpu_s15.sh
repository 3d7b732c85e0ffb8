#!/bin/bash
# Round-4 GPU session 15: leaf postponement threshold of the depth > 4
# instantiation (C5) re-swept on the kernel without counters.
set -e
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s15
O=gpurun_out/s15
timeout -k 10 500 python -u tools/ab.py --rounds 2 --steps 3 --config C5 def: lwd8:lib_lwd8: lwd20:lib_lwd20: > $O/ab_C5.txt 2>&1
