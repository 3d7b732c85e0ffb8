set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in lib lib_tour lib lib_tour; do
  RTAMD_LIB_DIR=simple-raytracer_amd/$v timeout -k 10 120 python bench.py --cpu-baseline off --steps 10 > gpurun_out/ab.json
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['tests_per_launch'])"
done
RTAMD_LIB_DIR=simple-raytracer_amd/lib_tour timeout -k 10 300 python -m pytest tests -m gpu -x -q -k "parity_forced or depth_knob or c3_full" > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
