set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for o in "chain=0" "chain=1" "chain=0" "chain=1"; do
  timeout -k 10 120 python bench.py --cpu-baseline off --steps 10 --option $o > gpurun_out/sw.json
  python -c "import json;d=json.load(open('gpurun_out/sw.json'));r=d['roofline'];print('$o', d['value'], d['ms_per_step'], r['kernel_ms'], r['tests_per_launch'], d['ray_counts']['shadow'])"
done
