cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rf --timeout 200 --timeout-method thread -k "scene_parity or special or collapse or depth or c5" > gpurun_out/pytest_l.log 2>&1; echo "pytest rc=$?"; tail -1 gpurun_out/pytest_l.log; \
grep -q " passed" gpurun_out/pytest_l.log && ! grep -q "failed\|error" gpurun_out/pytest_l.log && \
timeout -k 10 500 python tools/ab.py --config C5 --rounds 2 --steps 3 base:lib_base new: > gpurun_out/ab_lazy_c5.log 2>&1; echo "ab rc=$?"; tail -3 gpurun_out/ab_lazy_c5.log; \
timeout -k 10 500 python tools/ab.py --rounds 3 --steps 20 base:lib_base new: > gpurun_out/ab_lazy.log 2>&1; echo "ab rc=$?"; tail -3 gpurun_out/ab_lazy.log
