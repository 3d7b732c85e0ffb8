cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 600 python tools/ab.py --rounds 3 --steps 20 cur: shade_load1:lib_sm > gpurun_out/ab_probe3.log 2>&1; echo "ab rc=$?"; tail -3 gpurun_out/ab_probe3.log
