set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for v in base cur base cur; do
  if [ $v = base ]; then L=simple-raytracer_amd/lib_base; else L=simple-raytracer_amd/lib; fi
  RTAMD_LIB_DIR=$L timeout -k 10 120 python bench.py --cpu-baseline off --steps 10 > gpurun_out/ab.json
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
