#!/bin/bash
# Parity subset of the -m gpu suite on a kernel library variant (A/B builds
# under simple-raytracer_amd/lib_<variant>/): the golden fixtures, the
# reference's own floats, the depth knob, the option bit-identity tests and
# the full-size C3 rows.   tools/lib_parity.sh lib_pair4
set -o pipefail
lib=$1; shift
export RTAMD_LIB_DIR=${GRAFT_REPO_ROOT:-$(pwd)}/simple-raytracer_amd/$lib
exec python -m pytest tests/test_gpu_parity.py tests/test_float_goldens.py -m gpu -q -p no:cacheprovider --maxfail=${MAXFAIL:-12} \
  --timeout 300 --timeout-method thread \
  -k "${K:-golden or reference_floats or depth_knob or bit_identical or c3_full or c3_variants or lds_stack}" "$@"
