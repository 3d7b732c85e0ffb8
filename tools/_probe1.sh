set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for a in "--config C2 --steps 3" "--config C2 --steps 20" "--config C2 --steps 20 --inflight 1" "--steps 5" "--steps 20"; do
  timeout -k 10 300 python bench.py $a --cpu-baseline off > gpurun_out/b.json
  python -c "import json;d=json.load(open('gpurun_out/b.json'));print('$a', d['value'], d['ms_per_step'], d['frame_latency_ms'], d['roofline']['kernel_ms'])"
done
