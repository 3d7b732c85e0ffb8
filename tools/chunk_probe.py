#!/usr/bin/env python3
"""Refill-chunk sensitivity per scene property (one GPU): renders variants of
a config with the `chunk` option at several values and prints the median
kernel time of each.

  python tools/chunk_probe.py C4 [chunk ...]

Variants: the config as is, untextured, with two point lights, at half
resolution -- which property makes a wave's 8x8-tile refill slower than
taking the idle lanes' count from the counter."""
from __future__ import annotations

import json
import os
import statistics
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "simple-raytracer_amd"))


def main():
    import torch
    import rtamd
    from rtamd import scenes as gen

    name = sys.argv[1]
    chunks = [int(c) for c in sys.argv[2:]] or [0, 64]
    base = dict(gen.CONFIGS[name])
    variants = {"as_is": {}, "untextured": {"textured": False}, "point2": {"lights": "point2"},
                "half_res": {"w": base["w"] // 2, "h": base["h"] // 2}}
    d = tempfile.mkdtemp()
    for vname, over in variants.items():
        gen.CONFIGS["_probe"] = dict(base, **over)
        path = gen.write_scene(d, "_probe", tag=f"probe_{vname}")
        hs = rtamd.HostScene(path, cwd=d)
        hs.set_depth(base["depth"])
        W, H = hs.width, hs.height
        cam = hs.camera()
        out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
        row = {"variant": vname}
        for c in chunks:
            gs = rtamd.GpuScene(hs, device=0)
            gs.set_option("chunk", c)
            gs.prepare(cam, W, H)
            ms = []
            for _ in range(4):
                gs.render_rows_async(cam, W, H, 0, H, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
                torch.cuda.synchronize()
                ms.append(gs.last_stats().kernel_ms)
            row[f"c{c}_ms"] = round(statistics.median(ms[1:]), 3)
            gs.close()
        print(json.dumps(row), flush=True)
        hs.close()


if __name__ == "__main__":
    main()
