#!/bin/bash
# Round-4 GPU session 4: where a C2 step's time goes (RT_PROF cycle split with
# the work-counter wait; a probe without framebuffer stores), grid sizes.
set -e
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s4
O=gpurun_out/s4
P=$PWD/simple-raytracer_amd/lib_prof
RTAMD_LIB_DIR=$P timeout -k 10 200 python -u tools/prof_phases.py C2 > $O/ph_C2.txt 2>&1
RTAMD_LIB_DIR=$P timeout -k 10 200 python -u tools/prof_phases.py C2 work_parts=1 > $O/ph_C2_p1.txt 2>&1
RTAMD_LIB_DIR=$P timeout -k 10 200 python -u tools/prof_phases.py C3 > $O/ph_C3.txt 2>&1
RTAMD_LIB_DIR=$P timeout -k 10 200 python -u tools/prof_phases.py C3 work_parts=1 > $O/ph_C3_p1.txt 2>&1
RTAMD_LIB_DIR=$P timeout -k 10 200 python -u tools/prof_phases.py C3 --rows 8:0 > $O/ph_C3_r8.txt 2>&1
timeout -k 10 300 python -u tools/ab.py --rounds 2 --steps 300 --config C2 both: nostore:lib_nostore p1::work_parts=1 nostore_p1:lib_nostore:work_parts=1 g2560::grid=2560 g640::grid=640 g256::grid=256 > $O/ab_C2.txt 2>&1
