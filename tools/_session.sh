cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_gpu.log; \
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1; echo "bench rc=$?"; tail -1 gpurun_out/bench.log | cut -c1-600; \
PASSES="FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU
SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD
TA_BUSY_avr TCP_TCC_READ_REQ_LATENCY_sum" timeout -k 10 400 bash tools/pmc.sh > gpurun_out/pmc.log 2>&1; echo "pmc rc=$?"; RENDERS=2 python tools/pmc_summary.py > gpurun_out/pmc_new.json; grep -E "hbm_|l2_hit|kernel_ns|wait|lane_util|active" gpurun_out/pmc_new.json; \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --cpu-baseline off --steps 10 --inflight 1 > gpurun_out/prof.log 2>&1; echo "prof rc=$?"
