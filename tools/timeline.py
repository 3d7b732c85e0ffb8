#!/usr/bin/env python3
"""Per-wave launch timeline of one render, from an RT_PROF build
(make VARIANT=prof EXTRA=-DRT_PROF=1):

  RTAMD_LIB_DIR=simple-raytracer_amd/lib_prof python tools/timeline.py C2 [--rows 8:0] [opt=v ...]

Decomposes a frame on the kernel's own 100 MHz clock (s_memrealtime): when
the waves start (the dispatch ramp), how long the prologue takes, when the
work counter runs dry, and how the waves end (the tail), overall and per XCD;
next to the host-visible time of the same launch (torch events around it,
which add the dispatch and the counter resets).  One frame alone on the GPU
(synchronised before and after), the last of --frames."""
from __future__ import annotations

import json
import os
import statistics
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "simple-raytracer_amd"))


def q(v, fr):
    v = sorted(v)
    return v[min(len(v) - 1, int(fr * (len(v) - 1) + 0.5))]


def summary(vals):
    return {"min": round(min(vals), 2), "p10": round(q(vals, 0.1), 2), "p50": round(q(vals, 0.5), 2),
            "p90": round(q(vals, 0.9), 2), "max": round(max(vals), 2)}


def main():
    import torch
    import rtamd
    from rtamd import scenes as gen
    from rtamd.dist import row_set

    args = sys.argv[1:]
    rows = None
    if "--rows" in args:
        i = args.index("--rows")
        rows = tuple(int(v) for v in args[i + 1].split(":"))
        del args[i:i + 2]
    frames = 5
    if "--frames" in args:
        i = args.index("--frames")
        frames = int(args[i + 1])
        del args[i:i + 2]
    cfg = args[0] if args else "C2"
    opts = dict(a.split("=") for a in args[1:])
    d = tempfile.mkdtemp(prefix="rttl_")
    path = gen.write_scene(d, cfg)
    hs = rtamd.HostScene(path, cwd=d)
    hs.set_depth(gen.CONFIGS[cfg]["depth"])
    gs = rtamd.GpuScene(hs)
    for k, v in opts.items():
        gs.set_option(k, int(v))
    W, H = hs.width, hs.height
    cam = hs.camera()
    out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    gs.prepare(cam, W, H)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    host_ms = []
    kern_ms = []
    for _ in range(frames):
        torch.cuda.synchronize()
        e0.record()
        if rows:
            y0, b, step, nr, _ = row_set(H, rows[0], rows[1])
            gs.render_row_blocks_async(cam, W, H, y0, b, step, nr, out.data_ptr())
        else:
            gs.render_rows_async(cam, W, H, 0, H, out.data_ptr())
        e1.record()
        torch.cuda.synchronize()
        host_ms.append(e0.elapsed_time(e1))
        kern_ms.append(gs.last_stats().kernel_ms)
    wl = gs.debug_wavelog()
    if wl is None:
        sys.exit("not an RT_PROF library (RTAMD_LIB_DIR=.../lib_prof)")
    c = gs.debug_counters()
    st = gs.last_stats()
    t0 = min(w[0] for w in wl)
    us = lambda t: (t - t0) / 100.0      # noqa: E731  (100 MHz ticks -> us)
    start = [us(w[0]) for w in wl]
    prologue = [(w[1] - w[0]) / 100.0 for w in wl]
    first_step = [(w[4] - w[1]) / 100.0 for w in wl if w[4]]
    end = [us(w[3]) for w in wl]
    drained = [us(w[2]) for w in wl if w[2]]
    tail = [(w[3] - w[2]) / 100.0 for w in wl if w[2]]
    life = [(w[3] - w[0]) / 100.0 for w in wl]
    iters = [w[6] for w in wl]
    refills = [w[7] for w in wl]
    kernel_us = max(end)
    # waves alive over the launch, in 20 slices
    nb = 20
    alive = []
    for b in range(nb):
        t = kernel_us * (b + 0.5) / nb
        alive.append(sum(1 for s, e in zip(start, end) if s <= t < e))
    per_xcd = {}
    for w, s, e in zip(wl, start, end):
        x = int(w[5]) & 0xF           # XCC_ID
        per_xcd.setdefault(x, []).append((s, e, w[2] and us(w[2])))
    xcd = {str(x): {"waves": len(v), "start_p50": round(q([a for a, _, _ in v], 0.5), 2),
                    "start_max": round(max(a for a, _, _ in v), 2),
                    "end_p50": round(q([b for _, b, _ in v], 0.5), 2), "end_max": round(max(b for _, b, _ in v), 2)}
           for x, v in sorted(per_xcd.items())}
    res = {
        "config": cfg, "rows": rows, "options": opts, "imsize": [W, H],
        "rays": st.primary + st.shadow + st.refraction + st.reflection,
        "host_event_ms": [round(v, 4) for v in host_ms],
        "kernel_clock_ms": [round(v, 4) for v in kern_ms],
        "waves": len(wl), "grid": c[18], "blocks_per_cu": c[17],
        "timeline_us": {
            "kernel": round(kernel_us, 2),
            "wave_start": summary(start),
            "prologue": summary(prologue),
            "first_trace_step": summary(first_step) if first_step else None,
            "work_drained": summary(drained) if drained else None,
            "wave_tail_after_drain": summary(tail) if tail else None,
            "wave_end": summary(end),
            "wave_life": summary(life),
        },
        "iterations_per_wave": summary(iters),
        "mean_step_us": round(sum((w[3] - w[4]) / 100.0 for w in wl if w[4]) / max(1, sum(max(0, w[6] - 1) for w in wl)), 3),
        "refills_per_wave": summary(refills),
        "alive_waves_by_twentieth": alive,
        "per_xcd": xcd,
        "note": "kernel-clock timestamps relative to the first wave's start; host_event_ms adds the "
                "dispatch and the three counter resets before the launch",
    }
    print(json.dumps(res, indent=1))
    od = os.path.join(ROOT, "gpurun_out")
    os.makedirs(od, exist_ok=True)
    tag = f"{cfg}" + (f"_rows{rows[0]}_{rows[1]}" if rows else "") + "".join(f"_{k}{v}" for k, v in opts.items())
    with open(os.path.join(od, f"timeline_{tag}.json"), "w") as f:
        json.dump(dict(res, raw=wl), f)


if __name__ == "__main__":
    main()
