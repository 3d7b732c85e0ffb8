#!/usr/bin/env python3
"""A/B timing of kernel variants on one GPU: interleaved rounds, one bench.py
subprocess per (library variant, runtime options) pair.

  python tools/ab.py --rounds 2 --config C3 base: w4:lib_w4 leaf4::bvh_leaf=4 ...

Each spec is  name:libdir:opt=v,opt=v[:--arg=v,--arg=v]  (libdir relative
to simple-raytracer_amd/, empty = lib; the last field: extra bench.py
arguments, e.g. --inflight=3).  Results -> gpurun_out/ab.jsonl + a summary
table on stdout."""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--timeout", type=int, default=300)
    ap.add_argument("specs", nargs="+")
    a = ap.parse_args()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    out = open(os.path.join(ROOT, "gpurun_out", "ab.jsonl"), "a")
    res: dict[str, list] = {}
    for r in range(a.rounds):
        for spec in a.specs:
            name, lib, opts, bargs = (spec.split(":") + ["", "", ""])[:4]
            env = dict(os.environ)
            if lib:
                env["RTAMD_LIB_DIR"] = os.path.join(ROOT, "simple-raytracer_amd", lib)
            cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--cpu-baseline", "off", "--steps",
                   str(a.steps), "--config", a.config]
            for o in filter(None, opts.split(",")):
                cmd += ["--option", o]
            cmd += [x for x in bargs.split(",") if x]
            p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=a.timeout)
            line = next((l for l in p.stdout.splitlines() if l.startswith("{")), None)
            if p.returncode != 0 or line is None:
                # any failure may be a GPU fault: stop using the GPU in this call
                print(f"{name}: FAILED rc={p.returncode}\n{p.stderr[-2000:]}", flush=True)
                sys.exit(1)
            j = json.loads(line)
            j["ab_name"], j["ab_round"] = name, r
            out.write(json.dumps(j) + "\n")
            out.flush()
            res.setdefault(name, []).append(j)
            rl = j["roofline"]
            print(f"r{r} {name:14s} {j['value']:9.1f} Mrays/s  kernel {rl['kernel_ms']:8.2f} ms  "
                  f"frac {rl['frac']:.4f}  tests {rl.get('tests_per_launch')}", flush=True)
    print("\nsummary (median over rounds)")
    for name, js in res.items():
        v = statistics.median(x["value"] for x in js)
        k = statistics.median(x["roofline"]["kernel_ms"] for x in js)
        print(f"  {name:14s} {v:9.1f} Mrays/s  {k:8.2f} ms")


if __name__ == "__main__":
    main()
