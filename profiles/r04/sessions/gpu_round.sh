#!/bin/bash
# One GPU-box session: smoke -> gpu tests -> bench -> rocprof kernel trace.
# Every GPU step has its own time limit; any failure stops the script (a GPU
# fault inside pytest surfaces as an ordinary test failure, rc 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ]; }
STEPS="${STEPS:-smoke tests bench prof}"
for s in $STEPS; do
  case $s in
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?;;
    tests) timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1; rc=$?;;
    bench) timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1; rc=$?;;
    prof)  timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --cpu-baseline off --steps 3 --inflight 1 ${BENCH_ARGS:-} > $OUT/prof.log 2>&1; rc=$?;;
    *) echo "unknown step $s"; rc=2;;
  esac
  echo "step $s rc=$rc"
  tail -3 $OUT/$s*.log 2>/dev/null
  ok $rc || { echo "stopping after $s (rc=$rc)"; exit $rc; }
done
