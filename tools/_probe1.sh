set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_round.sh
PASSES='FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU
SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY
TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum
GRBM_GUI_ACTIVE GRBM_COUNT' BENCH_ARGS="--inflight 1" bash tools/pmc.sh
RENDERS=2 python tools/pmc_summary.py > gpurun_out/pmc_summary.json
for c in C2 C4 C5; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --cpu-baseline off > gpurun_out/bench_$c.json
  python -c "import json;d=json.load(open('gpurun_out/bench_$c.json'));print('$c', d['value'], d['ms_per_step'], d['frame_latency_ms'], d['roofline']['frac'])"
done
timeout -k 10 120 python tools/overlap_probe.py C3 --rows 8:0 --frames 10 --slots > gpurun_out/ovl8s.json
cat gpurun_out/ovl8s.json
RTAMD_LIB_DIR=simple-raytracer_amd/lib_prof timeout -k 10 120 python tools/prof_phases.py C3 > gpurun_out/ph_full.json
RTAMD_LIB_DIR=simple-raytracer_amd/lib_prof timeout -k 10 120 python tools/prof_phases.py C3 --rows 8:0 > gpurun_out/ph_8.json
timeout -k 10 200 python tools/strip_balance.py C3 > gpurun_out/balance.txt
tail -1 gpurun_out/balance.txt
