cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rf --timeout 200 --timeout-method thread -k "deep_stack or lds_stack" > gpurun_out/pytest_deep.log 2>&1; echo "pytest rc=$?"; tail -1 gpurun_out/pytest_deep.log; \
grep -q " passed" gpurun_out/pytest_deep.log && ! grep -q "failed\|error" gpurun_out/pytest_deep.log && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -1 gpurun_out/pytest_gpu.log; \
grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q "failed\|error" gpurun_out/pytest_gpu.log && \
timeout -k 10 600 python tools/ab.py --rounds 3 --steps 20 base:lib_base new: pad19:lib_pad19 > gpurun_out/ab_ovf.log 2>&1; echo "ab rc=$?"; tail -4 gpurun_out/ab_ovf.log
