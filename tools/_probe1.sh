set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json
cat gpurun_out/bench_default.json
