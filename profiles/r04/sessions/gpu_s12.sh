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
# the N=8 C3 share, pipelined: frames in flight, reserved slots, hardware queues
for f in 4 8; do for r in 0 8; do
  timeout -k 10 120 python -u tools/rank_balance.py C3 --ns 1,8 --rank-only 0 --inflight $f --reserve $r > $O/rb8_C3_f${f}_r${r}.txt 2>&1
done; done
for q in 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python -u tools/rank_balance.py C3 --ns 1,8 --rank-only 0 --inflight 8 --reserve 8 > $O/rb8_C3_q$q.txt 2>&1
done
