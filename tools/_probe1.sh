set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for w in 0 1; do
timeout -k 10 200 python bench.py --steps 5 --warmup $w --cpu-baseline off > gpurun_out/w.json
python -c "import json;d=json.load(open('gpurun_out/w.json'));print('warmup $w', d['value'], d['ms_per_step'])"
done
timeout -k 10 200 python bench.py --config C2 --steps 3 --warmup 0 --cpu-baseline off > gpurun_out/w.json
python -c "import json;d=json.load(open('gpurun_out/w.json'));print('C2 warmup 0', d['value'], d['ms_per_step'])"
