#!/bin/bash
# Round-4 GPU session 17: where C4's time goes (MAXF = 1 kernel): phase split
# and wave timeline of the profiling build.
set -e
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s17
O=gpurun_out/s17
export RTAMD_LIB_DIR=$PWD/simple-raytracer_amd/lib_prof
timeout -k 10 200 python -u tools/prof_phases.py C4 counters=0 > $O/ph_C4.txt 2>&1
timeout -k 10 200 python -u tools/prof_phases.py C4 > $O/ph_C4_count.txt 2>&1
timeout -k 10 200 python -u tools/timeline.py C4 counters=0 > $O/tl_C4.txt 2>&1
