#!/bin/bash
# Round-4 GPU session 14: the CLI's overlapped device->host copy and P3
# write (stream_ppm) -- the CLI / seam tests, then the one-shot phases.
set -e
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s14
O=gpurun_out/s14
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ -k "cli or seam or binding or smoke or e2e" > $O/pytest.log 2>&1
timeout -k 10 600 python -u tools/e2e.py C3 C4 C5 > $O/e2e.txt 2>&1
