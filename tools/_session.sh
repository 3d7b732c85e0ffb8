cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 1100 python tools/ab.py --rounds 5 --steps 20 cur: t1:lib_t1 t2:lib_t2 t3:lib_t3 > gpurun_out/ab_t.log 2>&1; echo "ab rc=$?"; tail -5 gpurun_out/ab_t.log
