#!/bin/bash
# One GPU session on the box (gpurun): every step under its own time limit,
# chained so that the first failure ends the session (no GPU step after a
# fault or a timeout).  Usage:
#   gpurun -- 'bash tools/gpu_session.sh NAME STEP [STEP ...]'
# STEP: tests | bench[:CONFIG] | ab:CONFIG:ROUNDS:STEPS:SPEC,SPEC,... |
#       prof:CONFIG | overlap:CONFIG | pmc:CONFIG[:LIBDIR] | e2e | phases:CONFIG[:OPTS] | balance:CONFIG[:NS] | cmd:NAME:CMD
set -o pipefail
name=$1; shift
out=gpurun_out/$name
mkdir -p "$out"
export TMPDIR=/tmp
for step in "$@"; do
  IFS=: read -r kind a b c d <<< "$step"
  echo "[session $name] $step $(date +%T)"
  case $kind in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        -p no:cacheprovider > "$out/pytest.log" 2>&1 || { tail -30 "$out/pytest.log"; exit 1; } ;;
    bench)
      timeout -k 10 400 python bench.py --config "${a:-C3}" --steps 20 --warmup 5 \
        --out-json "$out/bench_${a:-C3}.json" > "$out/bench_${a:-C3}.log" 2>&1 || { tail -20 "$out/bench_${a:-C3}.log"; exit 1; } ;;
    ab)
      timeout -k 10 900 python tools/ab.py --config "$a" --rounds "$b" --steps "$c" ${d//,/ } \
        > "$out/ab_$a.txt" 2>&1 || { tail -20 "$out/ab_$a.txt"; exit 1; } ;;
    prof)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof_$a" \
        -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --config "$a" --steps 10 --warmup 2 --inflight 1 \
        --cpu-baseline off) > "$out/prof_$a.log" 2>&1 || { tail -20 "$out/prof_$a.log"; exit 1; } ;;
    overlap)
      # two frames in flight (bench.py's N = 1 setting) under a kernel trace:
      # the dispatches' overlap and the period between their ends (the step)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$out/overlap_$a" \
        -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --config "$a" --steps 20 --warmup 3 \
        --inflight 2 --cpu-baseline off --count-render off) > "$out/overlap_$a.log" 2>&1 || { tail -20 "$out/overlap_$a.log"; exit 1; }
      python3 tools/overlap_trace.py $(find "$out/overlap_$a" -name '*kernel_trace.csv' | head -1) --steps 20 \
        > "$out/overlap_$a.json" 2>&1 || { tail -20 "$out/overlap_$a.json"; exit 1; } ;;
    pmc)
      # FETCH / WRITE bytes and the SQ/TA/TCC counters of one frame, one
      # rocprofv3 pass per counter group (never combined with tracing);
      # b: a library variant's directory under simple-raytracer_amd/ (lib_base)
      i=0; tag=$a${b:+_$b}
      if [ -n "$b" ]; then export RTAMD_LIB_DIR=$GRAFT_REPO_ROOT/simple-raytracer_amd/$b; else unset RTAMD_LIB_DIR; fi
      for pass in "FETCH_SIZE" "WRITE_SIZE" \
          "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU" \
          "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_THREAD_CYCLES_VALU TA_BUSY_avr" \
          "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"; do
        i=$((i+1))
        (cd /tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $pass -d "$GRAFT_REPO_ROOT/$out/pmc_$tag/p$i" \
          -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --config "$a" --cpu-baseline off \
          --steps 1 --warmup 0 --inflight 1 --count-render off) > "$out/pmc_${tag}_p$i.log" 2>&1 \
          || { tail -20 "$out/pmc_${tag}_p$i.log"; exit 1; }
      done
      RENDERS=2 python3 tools/pmc_summary.py "$out/pmc_$tag" > "$out/${tag}_pmc.json"
      unset RTAMD_LIB_DIR ;;
    e2e)
      # a: extra flags (floats: the float writer, RT_PPM_FLOATS)
      timeout -k 10 600 python -u tools/e2e.py C3 C4 C5 ${a:+--$a} > "$out/e2e$a.txt" 2>&1 || { tail -20 "$out/e2e$a.txt"; exit 1; } ;;
    phases)
      # RT_PROF build (make VARIANT=prof EXTRA=-DRT_PROF=1); b: extra options (counters=0)
      RTAMD_LIB_DIR=$GRAFT_REPO_ROOT/simple-raytracer_amd/lib_prof timeout -k 10 300 python -u tools/prof_phases.py \
        "$a" $b > "$out/phases_$a$b.txt" 2>&1 || { tail -20 "$out/phases_$a$b.txt"; exit 1; } ;;
    balance)
      timeout -k 10 600 python -u tools/rank_balance.py "$a" --ns "${b:-1,8}" > "$out/${a}_row_balance.txt" 2>&1 \
        || { tail -20 "$out/${a}_row_balance.txt"; exit 1; } ;;
    cmd)
      # an arbitrary command line (a = its log name), e.g. cmd:x:'python tools/foo.py';
      # the command keeps its own colons (pytest -p no:cacheprovider)
      rest=${step#cmd:}; a=${rest%%:*}; b=${rest#*:}
      timeout -k 10 600 bash -c "$b" > "$out/$a.log" 2>&1 || { tail -20 "$out/$a.log"; exit 1; } ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[session $name] done $(date +%T)"
