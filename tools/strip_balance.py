#!/usr/bin/env python3
"""Per-strip render time on one GPU: how balanced are N contiguous row strips
of the C3 image (the multi-GPU partition)?  Prints kernel ms per strip."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "simple-raytracer_amd"))
import torch  # noqa: F401,E402  (one HIP runtime: torch's)
import rtamd  # noqa: E402
from rtamd import scenes as gen  # noqa: E402
from rtamd.dist import row_set  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
d = os.path.join(os.environ.get("TMPDIR", "/tmp"), "rtamd_balance")
path = gen.write_scene(d, cfg)
hs = rtamd.HostScene(path, cwd=d)
W, H = hs.width, hs.height
cam = hs.camera()
gs = rtamd.GpuScene(hs)
buf = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
out = {}
for n in (1, 2, 4, 8):
    times = []
    for r in range(n):
        y0, b, step, nr, _ = row_set(H, n, r)
        for _ in range(2):
            gs.render_row_blocks_async(cam, W, H, y0, b, step, nr, buf.data_ptr())
            st = gs.last_stats()
        times.append(round(st.kernel_ms, 3))
    out[n] = dict(ms=times, max=max(times), mean=round(sum(times) / n, 3),
                  efficiency=round(sum(times) / n / max(times), 3))
    print(n, out[n], flush=True)
print(json.dumps(out))
