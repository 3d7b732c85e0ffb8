set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 120 python tools/overlap_probe.py C3 --rows 8:0 --frames 10 --slots > gpurun_out/ovl8s.json
cat gpurun_out/ovl8s.json
for v in base cur; do
  if [ $v = base ]; then L=simple-raytracer_amd/lib_base; else L=simple-raytracer_amd/lib; fi
  RTAMD_LIB_DIR=$L timeout -k 10 120 python bench.py --cpu-baseline off --inflight 1 --steps 10 > gpurun_out/b_$v.json
  python -c "import json;d=json.load(open('gpurun_out/b_$v.json'));print('$v inflight1', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
timeout -k 10 120 python bench.py --cpu-baseline off --inflight 2 --steps 10 > gpurun_out/b_cur2.json
python -c "import json;d=json.load(open('gpurun_out/b_cur2.json'));print('cur inflight2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['frame_latency_ms'])"
RTAMD_LIB_DIR=simple-raytracer_amd/lib_base timeout -k 10 120 python bench.py --cpu-baseline off --inflight 1 --steps 10 > gpurun_out/b_base2.json
python -c "import json;d=json.load(open('gpurun_out/b_base2.json'));print('base inflight1 again', d['value'], d['ms_per_step'])"
