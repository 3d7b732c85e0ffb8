cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_gpu.log; \
timeout -k 10 1100 python tools/ab.py --rounds 4 --steps 20 w2: w0:lib_w0 w5:lib_w5 > gpurun_out/ab_w.log 2>&1; echo "ab rc=$?"; tail -5 gpurun_out/ab_w.log
