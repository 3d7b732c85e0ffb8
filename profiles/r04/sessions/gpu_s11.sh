#!/bin/bash
# Round-4 GPU session 11: the MAXF = 1 instantiation (scenes with no
# reflecting / refracting material: C2, C4) -- GPU suite, the last light's
# zero-Phong skip there (lib vs lib_ll0); non-temporal frame / spill stores
# (lib_nt) on C5 and C3 with C5's memory-side bytes.
set -e
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/s11
O=$R/gpurun_out/s11
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1
timeout -k 10 300 python -u tools/ab.py --rounds 3 --steps 20 --config C4 def: ll0:lib_ll0: > $O/ab_C4.txt 2>&1
timeout -k 10 200 python -u tools/ab.py --rounds 3 --steps 300 --config C2 def: ll0:lib_ll0: > $O/ab_C2.txt 2>&1
timeout -k 10 300 python -u tools/ab.py --rounds 2 --steps 3 --config C5 def: nt:lib_nt: > $O/ab_C5.txt 2>&1
timeout -k 10 300 python -u tools/ab.py --rounds 3 --steps 20 --config C3 def: nt:lib_nt: > $O/ab_C3.txt 2>&1
cd /tmp
for v in lib lib_nt; do
  for ctr in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"; do
    n=$(echo $ctr | cut -d' ' -f1)
    RTAMD_LIB_DIR=$R/simple-raytracer_amd/$v timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr -d $O/pmc_C5_$v/p_$n -o run --output-format csv -- python3 $R/bench.py --config C5 --cpu-baseline off --steps 1 --warmup 0 --inflight 1 --count-render off > $O/pmc_C5_${v}_$n.log 2>&1
  done
done
cd $R
for v in lib lib_nt; do RTAMD_LIB_DIR=$R/simple-raytracer_amd/$v RENDERS=2 python3 tools/pmc_summary.py $O/pmc_C5_$v > $O/C5_pmc_$v.json; done
