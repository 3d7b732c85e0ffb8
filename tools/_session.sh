cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rf --timeout 200 --timeout-method thread -k "nan_rays" > gpurun_out/pytest_nan2.log 2>&1; echo "pytest rc=$?"; tail -1 gpurun_out/pytest_nan2.log; \
RTAMD_LIB_DIR=simple-raytracer_amd/lib_prof timeout -k 10 300 python tools/prof_phases.py C5 > gpurun_out/phases_C5.json 2>gpurun_out/phases.err; echo "rc=$?"; \
RTAMD_LIB_DIR=simple-raytracer_amd/lib_prof timeout -k 10 300 python tools/prof_phases.py C3 > gpurun_out/phases_C3.json 2>>gpurun_out/phases.err; echo "rc=$?"
