cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_gpu.log; \
timeout -k 10 900 python tools/ab.py --rounds 3 --steps 20 head:lib_head new: > gpurun_out/ab_rec.log 2>&1; echo "ab rc=$?"; tail -3 gpurun_out/ab_rec.log; \
PASSES="FETCH_SIZE
WRITE_SIZE" timeout -k 10 300 bash tools/pmc.sh > gpurun_out/pmc.log 2>&1; echo "pmc rc=$?"; RENDERS=2 python tools/pmc_summary.py > gpurun_out/pmc_rec.json; grep -E "hbm_" gpurun_out/pmc_rec.json; \
RTAMD_LIB_DIR=$GRAFT_REPO_ROOT/simple-raytracer_amd/lib_head PASSES="FETCH_SIZE
WRITE_SIZE" timeout -k 10 300 bash tools/pmc.sh > gpurun_out/pmc_h.log 2>&1; echo "pmc head rc=$?"; RENDERS=2 python tools/pmc_summary.py > gpurun_out/pmc_head.json; grep -E "hbm_" gpurun_out/pmc_head.json
