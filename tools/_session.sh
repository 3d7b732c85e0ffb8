cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/wr && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rf --timeout 200 --timeout-method thread -k "scene_parity or special or depth or c5 or glass or deep or nan or float_golden or c3_full" > gpurun_out/pytest_root.log 2>&1; echo "pytest rc=$?"; tail -1 gpurun_out/pytest_root.log; \
grep -q " passed" gpurun_out/pytest_root.log && ! grep -q "failed\|error" gpurun_out/pytest_root.log && \
RTAMD_LIB_DIR=$GRAFT_REPO_ROOT/simple-raytracer_amd/lib_base timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/wr/base -o run --output-format csv -- python3 bench.py --cpu-baseline off --steps 1 --warmup 0 --inflight 1 > gpurun_out/wr/base.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/wr/new -o run --output-format csv -- python3 bench.py --cpu-baseline off --steps 1 --warmup 0 --inflight 1 > gpurun_out/wr/new.log 2>&1 && \
echo "pmc rc=$?"; \
timeout -k 10 500 python tools/ab.py --rounds 3 --steps 20 base:lib_base new: > gpurun_out/ab_root.log 2>&1; echo "ab rc=$?"; tail -3 gpurun_out/ab_root.log
