cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -1 gpurun_out/pytest_gpu.log; \
grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q "failed\|error" gpurun_out/pytest_gpu.log && \
timeout -k 10 500 python tools/ab.py --rounds 3 --steps 20 base:lib_base hg:lib_hg > gpurun_out/ab_hg.log 2>&1; echo "ab rc=$?"; tail -3 gpurun_out/ab_hg.log
