#!/usr/bin/env python3
"""The face pre-split (rt_accel.cpp presplit) on other seeds of a config's
generator: the kernel time of one whole frame (kernel without counters, the
best of `reps`) and the executed box tests (one counted frame) with the
option bvh_presplit at each value, per seed -- is the benched seed's gain a
property of the scene kind or of one tree?

  python tools/presplit_seeds.py C4 --seeds 1234,1,2,3 --values 0,2"""
import argparse
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "simple-raytracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("--seeds", default="1234,1,2,3")
    ap.add_argument("--values", default="0,2")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    import rtamd
    from rtamd import scenes as gen
    d = tempfile.mkdtemp(prefix="rtps_")
    cfg = gen.CONFIGS[a.config]
    for seed in (int(s) for s in a.seeds.split(",")):
        path = os.path.join(d, f"{a.config}_{seed}.txt")
        with open(path, "w") as f:
            f.write(gen.scene_text(a.config, seed=seed))
        if cfg["textured"]:
            gen.write_scene(d, a.config)            # (the texture file beside it)
        hs = rtamd.HostScene(path, cwd=d)
        hs.set_depth(cfg["depth"])
        W, H = hs.width, hs.height
        cam = hs.camera()
        out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
        row = {"seed": seed}
        for v in (int(x) for x in a.values.split(",")):
            g = rtamd.GpuScene(hs)
            g.set_option("bvh_presplit", v)
            g.render_row_blocks_async(cam, W, H, 0, H, H, H, out.data_ptr())
            box = g.last_stats().box_tests
            g.set_option("counters", 0)
            best = 1e30
            for _ in range(a.reps):
                g.render_row_blocks_async(cam, W, H, 0, H, H, H, out.data_ptr())
                best = min(best, g.last_stats().kernel_ms)
            row[f"ps{v}"] = dict(kernel_ms=round(best, 3), box_tests=int(box))
            g.close()
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
