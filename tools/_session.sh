cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -5 gpurun_out/pytest_gpu.log; \
for c in C3 C3D C3G C4; do timeout -k 10 300 python bench.py --config $c --cpu-baseline off --steps 20 > gpurun_out/bench_$c.log 2>&1; echo "bench $c rc=$?"; python -c "
import json; j=json.loads(open('gpurun_out/bench_$c.log').read().strip().splitlines()[-1]); print('$c', j['value'], j['ms_per_step'], j['work']['bf_queries'], j['work']['stack_spills'], j['roofline']['tests_per_launch'])"; done; \
RTAMD_LIB_DIR=$GRAFT_REPO_ROOT/simple-raytracer_amd/lib_base timeout -k 10 300 python bench.py --config C4 --cpu-baseline off --steps 20 > gpurun_out/bench_base_C4.log 2>&1; echo "base C4 rc=$?"; tail -1 gpurun_out/bench_base_C4.log | cut -c1-160
timeout -k 5 60 ./tools/tex_probe > gpurun_out/tex_probe.txt 2>&1; echo "probe rc=$?"; head -3 gpurun_out/tex_probe.txt
