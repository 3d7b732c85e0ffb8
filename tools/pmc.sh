#!/bin/bash
# PMC passes over one bench render (separate rocprofv3 runs, counters only
# with --kernel-trace, never combined with tracing domains).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
ARGS="--cpu-baseline off --steps 1 --warmup 0 ${BENCH_ARGS:-}"
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
while read -r pass; do
  [ -z "$pass" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $pass -d $OUT/p$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc: $pass"
  [ $rc -eq 0 ] || exit $rc
done <<PASSES
${PASSES:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU
SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum
TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum
TCP_TOTAL_READ_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_WRITE_sum
TA_BUSY_avr TCP_TCC_READ_REQ_LATENCY_sum}
PASSES
