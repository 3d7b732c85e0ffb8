cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 900 python tools/ab.py --rounds 3 --steps 20 cur: pk:lib_pk > gpurun_out/ab_pk.log 2>&1; echo "ab rc=$?"; tail -4 gpurun_out/ab_pk.log
