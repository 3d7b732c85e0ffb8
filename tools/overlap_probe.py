#!/usr/bin/env python3
"""How much of a launch's tail do two frames in flight recover?

  python tools/overlap_probe.py [C3] [--rows N:r] [--frames K]

Renders K frames of one rank's row set (--rows 8:0 = rank 0 of 8, the N=8
share) back to back on one stream, then with two scenes (each with its own
work counter and frame buffer) alternating over two streams, and prints the
ms per frame of both."""
from __future__ import annotations

import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "simple-raytracer_amd"))


def main():
    import torch
    import rtamd
    from rtamd import scenes as gen
    from rtamd.dist import row_set

    args = sys.argv[1:]
    rows, frames = (1, 0), 10
    if "--rows" in args:
        i = args.index("--rows")
        rows = tuple(int(v) for v in args[i + 1].split(":"))
        del args[i:i + 2]
    for flag in ("--own-streams", "--slots"):
        if flag in args:
            args.remove(flag)
    if "--frames" in args:
        i = args.index("--frames")
        frames = int(args[i + 1])
        del args[i:i + 2]
    cfg = args[0] if args else "C3"
    d = tempfile.mkdtemp(prefix="rtovl_")
    path = gen.write_scene(d, cfg)
    hs = rtamd.HostScene(path, cwd=d)
    hs.set_depth(gen.CONFIGS[cfg]["depth"])
    W, H = hs.width, hs.height
    cam = hs.camera()
    y0, b, step, nr, _ = row_set(H, rows[0], rows[1])
    slots = "--slots" in sys.argv          # one scene, option inflight=F (render slots)
    F = int(os.environ.get("INFLIGHT", "2"))
    if slots:
        g = rtamd.GpuScene(hs)
        g.set_option("inflight", F)
        if "RESERVE" in os.environ:
            g.set_option("reserve", int(os.environ["RESERVE"]))
        scenes = [g] * F
    else:
        F = 2
        scenes = [rtamd.GpuScene(hs), rtamd.GpuScene(hs)]
    outs = [torch.empty((nr, W, 3), dtype=torch.float32, device="cuda") for _ in range(F)]
    streams = [torch.cuda.Stream() for _ in range(F)]
    for s_ in streams:
        with torch.cuda.stream(s_):
            outs[0][:1].zero_()
    torch.cuda.synchronize()

    own = "--own-streams" in sys.argv       # the scenes' own rt_scene streams

    def run(nflight):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(frames):
            j = k % nflight
            scenes[j].render_row_blocks_async(cam, W, H, y0, b, step, nr, outs[j].data_ptr(),
                                              None if own else streams[j].cuda_stream)
        for sc in scenes[:nflight]:
            sc.last_stats()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / frames

    res = {"config": cfg, "rows": rows, "frames": frames, "mode": "slots" if slots else
           ("own-streams" if own else "two scenes, torch streams")}
    for nflight in (1, F, 1, F):
        run(nflight)                       # warm
        res[f"ms_per_frame_{nflight}"] = round(run(nflight), 3)
    st = scenes[0].last_stats()
    res["single_kernel_ms"] = round(st.kernel_ms, 3)
    res["rays"] = st.rays()
    for o in outs[1:]:
        torch.testing.assert_close(outs[0], o, rtol=0, atol=0, equal_nan=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
