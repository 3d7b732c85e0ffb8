cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 700 python tools/ab.py --rounds 3 --steps 20 h: n21s14::lds_nodes=21 n25s14dp::lds_nodes=25,bvh_collapse=1,bvh_node=500 n21s14dp::lds_nodes=21,bvh_collapse=1,bvh_node=500 > gpurun_out/ab_half3.log 2>&1; echo "ab rc=$?"; tail -6 gpurun_out/ab_half3.log; \
timeout -k 10 500 python tools/ab.py --config C5 --rounds 2 --steps 3 h: n21s14::lds_nodes=21 n25s14dp::lds_nodes=25,bvh_collapse=1,bvh_node=500 > gpurun_out/ab_half3_c5.log 2>&1; echo "ab rc=$?"; tail -5 gpurun_out/ab_half3_c5.log
