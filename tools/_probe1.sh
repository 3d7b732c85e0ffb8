set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in lib lib_b64 lib_b128 lib lib_b64 lib_b128; do
  RTAMD_LIB_DIR=simple-raytracer_amd/$v timeout -k 10 120 python bench.py --cpu-baseline off --steps 10 > gpurun_out/ab.json
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['frame_latency_ms'])"
done
RTAMD_LIB_DIR=simple-raytracer_amd/lib_b64 timeout -k 10 120 python tools/overlap_probe.py C3 --rows 8:0 --frames 10 --slots
timeout -k 10 120 python tools/overlap_probe.py C3 --rows 8:0 --frames 10 --slots
