cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rf --timeout 200 --timeout-method thread -k "packets" > gpurun_out/pytest_pk.log 2>&1; echo "pytest rc=$?"; tail -1 gpurun_out/pytest_pk.log; \
grep -q " passed" gpurun_out/pytest_pk.log && ! grep -q "failed\|error" gpurun_out/pytest_pk.log && \
timeout -k 10 500 python tools/ab.py --rounds 3 --steps 20 base:lib_base pk: nopk::primary_pass=0 > gpurun_out/ab_pk.log 2>&1; echo "ab rc=$?"; tail -4 gpurun_out/ab_pk.log; \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pkprof -o run --output-format csv -- python3 bench.py --cpu-baseline off --steps 3 --warmup 1 --inflight 1 > gpurun_out/pkprof.log 2>&1; echo "prof rc=$?"
