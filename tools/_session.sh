cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 900 python tools/ab.py --rounds 3 --steps 20 --config C4 bytes:lib_tex0 tiled: > gpurun_out/ab_c4.log 2>&1; echo "ab rc=$?"; tail -4 gpurun_out/ab_c4.log
