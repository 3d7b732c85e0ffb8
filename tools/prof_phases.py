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

    args = sys.argv[1:]
    rows = None                       # --rows N:r -> rank r's row set of N (multi-GPU share)
    if "--rows" in args:
        i = args.index("--rows")
        rows = tuple(int(v) for v in args[i + 1].split(":"))
        del args[i:i + 2]
    kw = {}                           # --objects S,T -> override sphere / triangle counts
    if "--objects" in args:
        i = args.index("--objects")
        sp, tr = (int(v) for v in args[i + 1].split(","))
        kw = dict(n_spheres=sp, n_tris=tr, tag=f"obj{sp}_{tr}")
        del args[i:i + 2]
    cfg = args[0] if args else "C3"
    opts = dict(a.split("=") for a in args[1:])
    d = tempfile.mkdtemp(prefix="rtprof_")
    path = gen.write_scene(d, cfg, **kw)
    hs = rtamd.HostScene(path, cwd=d)
    hs.set_depth(gen.CONFIGS[cfg]["depth"])          # the config's depth (C5: 8), as bench.py
    gs = rtamd.GpuScene(hs)
    for k, v in opts.items():
        gs.set_option(k, int(v))
    W, H = hs.width, hs.height
    cam = hs.camera()
    out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    from rtamd.dist import row_set
    for _ in range(2):
        if rows:
            y0, b, step, nr, _ = row_set(H, rows[0], rows[1])
            gs.render_row_blocks_async(cam, W, H, y0, b, step, nr, out.data_ptr())
        else:
            gs.render_rows_async(cam, W, H, 0, H, out.data_ptr())
        st = gs.last_stats()
    c = gs.debug_counters()
    shade, trace, bf, iters, lanes, wtrips, ltrips = c[9:16]
    tot = shade + trace + bf
    res = {
        "config": cfg, "objects": kw, "rows": rows, "options": opts, "kernel_ms": st.kernel_ms,
        "cycles_split": {"shade_refill": shade / tot, "trace": trace / tot, "bf_scan": bf / tot} if tot else None,
        # of shade_refill: waiting for the work counter's atomic (RT_PROF, round 4)
        "work_counter_wait_frac": c[46] / tot if tot else None,
        "work_counter_wait_cycles_per_refill": c[46] / c[47] if c[47] else None,
        "outer_iterations": iters,
        "trace_lane_occupancy": lanes / (64 * iters) if iters else None,
        # the lanes that sit a step out, by reason (fractions of 64 x steps)
        "idle_lanes_by_reason": {"no_pixel": c[50] / (64 * iters), "held_secondary": c[51] / (64 * iters),
                                 "known_shadow": c[52] / (64 * iters)} if iters and len(c) > 52 else None,
        "traversal_simd_eff": ltrips / (64 * wtrips) if wtrips else None,
        "lane_trips_per_trace_lane": ltrips / lanes if lanes else None,
        "wave_trips_per_iter": wtrips / iters if iters else None,
        "launch": dict(zip(["mode", "blocks_per_cu", "grid", "lds_bytes", "bvh_nodes", "bvh_depth",
                            "bvh_stack", "cus"], c[16:24])),
        "timeline_us": ({"kernel": (c[26] - c[24]) / 100.0, "drain": (c[25] - c[24]) / 100.0,
                         "tail": (c[26] - c[25]) / 100.0, "mean_wave_tail": c[27] / max(1, c[29]) / 100.0,
                         "mean_wave_life": c[28] / max(1, c[29]) / 100.0, "waves": c[29]}
                        if c[29] else None),
        "inner_trip_cycles": ({"fetch": c[30] / max(1, c[6] // 4), "trip": c[31] / max(1, c[6] // 4)}
                              if c[31] else None),
        "lane_trips_by_kind": dict(zip(["primary", "shadow", "refr_refl"], c[36:39])),
        "mixed_step_frac": c[39] / iters if iters else None,   # steps with primary and other searches together
        "raw": c,
    }
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
