#!/bin/bash
# Round-4 GPU session 18: C4 (10 000 triangles, primary + shadow rays only):
# refill batch and BVH build knobs.
set -e
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s18
O=gpurun_out/s18
timeout -k 10 600 python -u tools/ab.py --rounds 2 --steps 20 --config C4 def: rm48::refill_min=48 rm56::refill_min=56 leaf4::bvh_leaf=4 leaf6::bvh_leaf=6 leaf12::bvh_leaf=12 node250::bvh_node=250 node1000::bvh_node=1000 > $O/ab_C4.txt 2>&1
