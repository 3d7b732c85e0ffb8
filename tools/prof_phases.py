#!/usr/bin/env python3
"""Where the render kernel's time goes, from an RT_PROF build
(make VARIANT=prof EXTRA=-DRT_PROF=1):

  RTAMD_LIB_DIR=simple-raytracer_amd/lib_prof python tools/prof_phases.py C3 [opt=v ...]

Prints the per-wave cycle split (shading state machine + refill / BVH
traversal / brute-force fallback), the lane occupancy of the trace calls and
the traversal loop's SIMD efficiency (lane trips / (64 x wave trips))."""
from __future__ import annotations

import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "simple-raytracer_amd"))


def main():
    import torch  # noqa: F401  (torch's HIP runtime first)
    import rtamd
    from rtamd import scenes as gen

    cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
    opts = dict(a.split("=") for a in sys.argv[2:])
    d = tempfile.mkdtemp(prefix="rtprof_")
    path = gen.write_scene(d, cfg)
    hs = rtamd.HostScene(path, cwd=d)
    gs = rtamd.GpuScene(hs)
    for k, v in opts.items():
        gs.set_option(k, int(v))
    W, H = hs.width, hs.height
    cam = hs.camera()
    out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    for _ in range(2):
        gs.render_rows_async(cam, W, H, 0, H, out.data_ptr())
        st = gs.last_stats()
    c = gs.debug_counters()
    shade, trace, bf, iters, lanes, wtrips, ltrips = c[9:16]
    tot = shade + trace + bf
    res = {
        "config": cfg, "options": opts, "kernel_ms": st.kernel_ms,
        "cycles_split": {"shade_refill": shade / tot, "trace": trace / tot, "bf_scan": bf / tot} if tot else None,
        "outer_iterations": iters,
        "trace_lane_occupancy": lanes / (64 * iters) if iters else None,
        "traversal_simd_eff": ltrips / (64 * wtrips) if wtrips else None,
        "lane_trips_per_trace_lane": ltrips / lanes if lanes else None,
        "wave_trips_per_iter": wtrips / iters if iters else None,
        "launch": dict(zip(["mode", "blocks_per_cu", "grid", "lds_bytes", "bvh_nodes", "bvh_depth",
                            "bvh_stack", "cus"], c[16:24])),
        "raw": c,
    }
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
