#!/bin/bash
# HBM bytes of one config's launch against the recursion depth (option depth):
# for each depth, a FETCH_SIZE pass and a WRITE_SIZE pass (rocprofv3 --pmc, one
# counter group per run, never with tracing) and one bench line with the
# counting render (rays by kind), so that the bytes can be set against the
# secondary rays and child opens each depth adds (where C5's
# bytes go).  Usage (on the GPU box, from the repo root):
#   bash tools/depth_traffic.sh C5 0,1,2,4,8 gpurun_out/depth
set -o pipefail
cfg=$1; depths=$2; out=$3
R=$GRAFT_REPO_ROOT
mkdir -p "$out"
for d in ${depths//,/ }; do
  i=0
  for pass in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    (cd /tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $pass -d "$R/$out/d$d/p$i" -o run \
      --output-format csv -- python3 "$R/bench.py" --config "$cfg" --cpu-baseline off --steps 1 --warmup 0 \
      --inflight 1 --count-render off --option depth=$d) > "$out/d${d}_p$i.log" 2>&1 || { tail -20 "$out/d${d}_p$i.log"; exit 1; }
  done
  RENDERS=2 python3 tools/pmc_summary.py "$out/d$d" > "$out/d${d}_pmc.json" || exit 1
  timeout -k 10 300 python3 bench.py --config "$cfg" --cpu-baseline off --steps 2 --warmup 1 --option depth=$d \
    --out-json "$out/d${d}_bench.json" > "$out/d${d}_bench.log" 2>&1 || { tail -20 "$out/d${d}_bench.log"; exit 1; }
  echo "depth $d done $(date +%T)"
done
