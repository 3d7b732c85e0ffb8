set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --steps 10 --cpu-baseline off --verify > gpurun_out/v1.json
python -c "import json;d=json.load(open('gpurun_out/v1.json'));print(1, d['value'], d['verified'], d['config']['frames_in_flight'], d['roofline']['kernel_ms'])"
for n in 2 4; do
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2953$n bench.py --gpus $n --steps 6 --warmup 1 --dist-backend gloo --verify --cpu-baseline off > gpurun_out/v$n.json 2> gpurun_out/v$n.err
python -c "import json;d=json.loads(open('gpurun_out/v$n.json').read().strip().splitlines()[-1]);print($n, d['value'], d['verified'], d['config']['frames_in_flight'], d['config']['reserved_block_slots'], d['roofline']['kernel_ms'])"
done
