#!/bin/bash
# Round-4 GPU session 11: non-temporal frame / spill stores (lib_nt) against
# the default library on C5 and C3 -- speed, and C5's memory-side bytes
# (FETCH_SIZE / WRITE_SIZE, TCC hit rate, DRAM share of the requests).
set -e
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/s11
O=$R/gpurun_out/s11
timeout -k 10 300 python -u tools/ab.py --rounds 2 --steps 3 --config C5 def: nt:lib_nt: > $O/ab_C5.txt 2>&1
timeout -k 10 300 python -u tools/ab.py --rounds 3 --steps 20 --config C3 def: nt:lib_nt: > $O/ab_C3.txt 2>&1
cd /tmp
for v in lib lib_nt; do
  for ctr in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"; do
    n=$(echo $ctr | cut -d' ' -f1)
    RTAMD_LIB_DIR=$R/simple-raytracer_amd/$v timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr -d $O/pmc_C5_$v/p_$n -o run --output-format csv -- python3 $R/bench.py --config C5 --cpu-baseline off --steps 1 --warmup 0 --inflight 1 --count-render off > $O/pmc_C5_${v}_$n.log 2>&1
  done
done
cd $R
for v in lib lib_nt; do RTAMD_LIB_DIR=$R/simple-raytracer_amd/$v RENDERS=2 python3 tools/pmc_summary.py $O/pmc_C5_$v > $O/C5_pmc_$v.json; done
# the N=8 C3 share, pipelined: frames in flight and reserved slots
for f in 4 8; do for r in 0 8; do
  timeout -k 10 120 python -u tools/rank_balance.py C3 --ns 1,8 --rank-only 0 --inflight $f --reserve $r > $O/rb8_C3_f${f}_r${r}.txt 2>&1
done; done
for q in 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python -u tools/rank_balance.py C3 --ns 1,8 --rank-only 0 --inflight 8 --reserve 8 > $O/rb8_C3_q$q.txt 2>&1
done
