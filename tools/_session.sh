cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
for c in C2 C5; do s=20; [ $c = C5 ] && s=4; timeout -k 10 600 python bench.py --config $c --cpu-baseline off --steps $s --warmup 1 > gpurun_out/bench_$c.log 2>&1; echo "bench $c rc=$?"; python -c "
import json; j=json.loads(open('gpurun_out/bench_$c.log').read().strip().splitlines()[-1]); print('$c', j['value'], j['ms_per_step'], j['work'], j['config']['launch'], j['one_frame'])"; done
