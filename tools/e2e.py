#!/usr/bin/env python3
"""One-shot drop-in runs: scene file -> PPM with the CLI (simple-raytracer_amd/
lib/rt, the SimpleRayTracer replacement), its --stats-json phase breakdown
(parse, scene upload, BVH build, render, device->host copy, quantise + P3
write) per config, at N = 1:

  python tools/e2e.py C3 C4 C5 [--keep]

Scenes are the seeded benchmark scenes (rtamd/scenes.py) written under
$TMPDIR; the PPM goes next to the scene (the reference's contract,
main.cpp:613-617) and is deleted afterwards unless --keep.  Results ->
gpurun_out/e2e_<cfg>.json and one summary line per config on stdout."""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "simple-raytracer_amd"))


def main():
    from rtamd import scenes as gen
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    keep = "--keep" in sys.argv
    # --floats: the P3 file from the float image (RT_PPM_FLOATS), for an A/B
    # against the default byte path (device-quantised, 3 B per pixel)
    floats = "--floats" in sys.argv
    tag = "_floats" if floats else ""
    cli = os.path.join(ROOT, "simple-raytracer_amd", "lib", "rt")
    od = os.path.join(ROOT, "gpurun_out")
    os.makedirs(od, exist_ok=True)
    for cfg in args or ["C3", "C4", "C5"]:
        d = tempfile.mkdtemp(prefix=f"rte2e_{cfg}_")
        path = gen.write_scene(d, cfg)
        js = os.path.join(d, "stats.json")
        cmd = [cli, path, "--depth", str(gen.CONFIGS[cfg]["depth"]), "--stats-json", js]
        t0 = time.perf_counter()
        # RT_TIMING: the library's own step times (scene creation, BVH upload,
        # first launch) on stderr, kept in the record
        r = subprocess.run(cmd, cwd=d, capture_output=True, text=True, timeout=600,
                           env={**os.environ, "RT_TIMING": "1", **({"RT_PPM_FLOATS": "1"} if floats else {})})
        wall = time.perf_counter() - t0
        if r.returncode != 0:
            print(f"{cfg}: rt failed rc={r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-2000:]}", flush=True)
            sys.exit(1)
        j = json.load(open(js))
        j["config"] = cfg
        j["rt_timing"] = [l[len("[rt timing] "):] for l in r.stderr.splitlines() if l.startswith("[rt timing] ")]
        j["process_wall_ms"] = round(wall * 1e3, 1)
        j["note"] = ("phases on the host clock inside one `rt scene.txt` run (N=1); process_wall_ms adds process "
                     "start, HIP runtime initialisation and exit")
        ppm = os.path.splitext(path)[0] + ".ppm"
        if not keep and os.path.exists(ppm):
            os.remove(ppm)
        with open(os.path.join(od, f"e2e_{cfg}{tag}.json"), "w") as f:
            json.dump(j, f, indent=1)
        print(json.dumps(j), flush=True)


if __name__ == "__main__":
    main()
