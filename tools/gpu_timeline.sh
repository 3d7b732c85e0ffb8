set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
export RTAMD_LIB_DIR=$PWD/simple-raytracer_amd/lib_prof
timeout -k 10 240 python -u tools/timeline.py C2 > gpurun_out/tl_C2.txt 2>&1
timeout -k 10 120 python -u tools/timeline.py C2 grid=256 > gpurun_out/tl_C2_g256.txt 2>&1
timeout -k 10 120 python -u tools/timeline.py C3 --rows 8:0 > gpurun_out/tl_C3_r8.txt 2>&1
timeout -k 10 120 python -u tools/timeline.py C3 > gpurun_out/tl_C3.txt 2>&1
timeout -k 10 120 python -u tools/timeline.py C4 --rows 8:0 > gpurun_out/tl_C4_r8.txt 2>&1
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_c2 -o run -- python3 $GRAFT_REPO_ROOT/tools/timeline.py C2 --frames 10 > $GRAFT_REPO_ROOT/gpurun_out/tl_C2_prof.txt 2>&1
cd $GRAFT_REPO_ROOT
unset RTAMD_LIB_DIR
timeout -k 10 200 python -u bench.py --steps 20 --cpu-baseline off > gpurun_out/bench_C3_new.txt 2>&1
