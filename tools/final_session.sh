#!/bin/bash
# End-of-round evidence on one GPU box (all outputs under gpurun_out/final/;
# round 4: copied to profiles/r04/final_*):
# smoke, the GPU test suite, one bench line per config, a rocprofv3 kernel
# trace of the default bench at one frame in flight and at two, the PMC
# passes whose FETCH_SIZE / WRITE_SIZE give profiles/pmc_traffic.json
# (tools/pmc_traffic.py; recorded with the library's sha), the projected
# N-GPU balance (tools/rank_balance.py), the one-shot CLI phases
# (tools/e2e.py) and a wave timeline of C2.  Every GPU step has its own time
# limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export TMPDIR=/tmp
O=$R/gpurun_out/final
mkdir -p $O
step() { echo "== $1"; shift; "$@"; rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
PART=${PART:-all}
if [ "$PART" = all ] || [ "$PART" = a ]; then
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
step tests bash -c "timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=\$?; tail -2 $O/pytest_gpu.log; exit \$rc"
step bench_C3 bash -c "timeout -k 10 600 python bench.py > $O/C3_bench.json 2> $O/C3_bench.err"
for c in C2 C3D C3G; do
  step bench_$c bash -c "timeout -k 10 600 python bench.py --config $c --cpu-baseline off --steps 100 > $O/${c}_bench.json 2> $O/${c}_bench.err"
done
for c in C4 C5; do
  step bench_$c bash -c "timeout -k 10 600 python bench.py --config $c --cpu-baseline off --steps 8 --warmup 2 > $O/${c}_bench.json 2> $O/${c}_bench.err"
done
step e2e bash -c "timeout -k 10 600 python -u tools/e2e.py C3 C4 C5 > $O/e2e.txt 2>&1"
for c in C3 C4; do
  step bal_$c bash -c "timeout -k 10 600 python -u tools/rank_balance.py $c --ns 1,2,4,8 > $O/${c}_row_balance.txt 2>&1"
done
step bal_C5 bash -c "timeout -k 10 600 python -u tools/rank_balance.py C5 --ns 1,8 --frames 8 > $O/C5_row_balance.txt 2>&1"
fi
if [ "$PART" = all ] || [ "$PART" = c ]; then
step tests_cli bash -c "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -k 'cli or seam or binding or smoke' > $O/pytest_gpu_cli.log 2>&1; rc=\$?; tail -2 $O/pytest_gpu_cli.log; exit \$rc"
step e2e_c bash -c "timeout -k 10 600 python -u tools/e2e.py C3 C4 C5 > $O/e2e.txt 2>&1"
# this round's kernel against round 3's (lib_r3: tools/build_rev.sh 268f298 r3), interleaved
step ab_r3_C3 bash -c "timeout -k 10 400 python -u tools/ab.py --rounds 3 --steps 100 --config C3 r4: r3:lib_r3 > $O/ab_r4_vs_r3_C3.txt 2>&1"
step ab_r3_C2 bash -c "timeout -k 10 300 python -u tools/ab.py --rounds 3 --steps 300 --config C2 r4: r3:lib_r3 > $O/ab_r4_vs_r3_C2.txt 2>&1"
step ab_r3_C4 bash -c "timeout -k 10 300 python -u tools/ab.py --rounds 2 --steps 20 --config C4 r4: r3:lib_r3 > $O/ab_r4_vs_r3_C4.txt 2>&1"
step ab_r3_C5 bash -c "timeout -k 10 400 python -u tools/ab.py --rounds 2 --steps 3 --config C5 r4: r3:lib_r3 > $O/ab_r4_vs_r3_C5.txt 2>&1"
# the C3 line again, now that profiles/pmc_traffic.json holds this library's PMC bytes
step bench_C3_traffic bash -c "timeout -k 10 600 python bench.py > $O/C3_bench_traffic.json 2> $O/C3_bench_traffic.err"
fi
if [ "$PART" = all ] || [ "$PART" = b ]; then
cd /tmp
step prof timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --cpu-baseline off --steps 5 --inflight 1
step prof2 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_inflight2 -o run --output-format csv -- python3 $R/bench.py --cpu-baseline off --steps 20 --inflight 2
for c in C2 C4 C5; do
  step prof_$c timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o run --output-format csv -- python3 $R/bench.py --config $c --cpu-baseline off --steps 3 --warmup 1 --inflight 1
done
i=0
while read -r pass; do
  [ -z "$pass" ] && continue
  i=$((i+1))
  step pmc_$i timeout -k 10 300 rocprofv3 --kernel-trace --pmc $pass -d $O/pmc/p$i -o run --output-format csv -- python3 $R/bench.py --cpu-baseline off --steps 1 --warmup 0 --inflight 1 --count-render off
done <<PASSES
FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU
SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_THREAD_CYCLES_VALU TA_BUSY_avr
TCC_HIT_sum TCC_MISS_sum
TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum
PASSES
cd $R
RENDERS=2 python3 tools/pmc_summary.py $O/pmc > $O/C3_pmc.json
cd /tmp
for c in C4 C5; do
  for ctr in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"; do
    n=$(echo $ctr | cut -d' ' -f1)
    step pmc_${c}_$n timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr -d $O/pmc_$c/p_$n -o run --output-format csv -- python3 $R/bench.py --config $c --cpu-baseline off --steps 1 --warmup 0 --inflight 1 --count-render off
  done
done
cd $R
for c in C4 C5; do RENDERS=2 python3 tools/pmc_summary.py $O/pmc_$c > $O/${c}_pmc.json; done
step timeline bash -c "RTAMD_LIB_DIR=$R/simple-raytracer_amd/lib_prof timeout -k 10 200 python -u tools/timeline.py C2 > $O/tl_C2.txt 2>&1"
step timeline_C3r8 bash -c "RTAMD_LIB_DIR=$R/simple-raytracer_amd/lib_prof timeout -k 10 200 python -u tools/timeline.py C3 --rows 8:0 > $O/tl_C3_r8.txt 2>&1"
step phases_C3 bash -c "RTAMD_LIB_DIR=$R/simple-raytracer_amd/lib_prof timeout -k 10 200 python -u tools/prof_phases.py C3 > $O/phases_C3.txt 2>&1"
step phases_C3_nc bash -c "RTAMD_LIB_DIR=$R/simple-raytracer_amd/lib_prof timeout -k 10 200 python -u tools/prof_phases.py C3 counters=0 > $O/phases_C3_nocount.txt 2>&1"
step phases_C5 bash -c "RTAMD_LIB_DIR=$R/simple-raytracer_amd/lib_prof timeout -k 10 300 python -u tools/prof_phases.py C5 > $O/phases_C5.txt 2>&1"
fi
echo done
