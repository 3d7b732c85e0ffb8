"""Diagnostic: render C3_64x64 with a given suspend / lds_stack and report."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "simple-raytracer_amd"))
import numpy as np
import rtamd
sus, lds = int(sys.argv[1]), int(sys.argv[2])
scn = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "scenes")
hs = rtamd.HostScene("C3_64x64.txt", cwd=scn)
W, H = hs.width, hs.height
cam = hs.camera()
g0 = rtamd.GpuScene(hs)
g0.set_option("suspend", 0)
ref, st = g0.render_rows(cam, W, H, 0, H)
gs = rtamd.GpuScene(hs)
gs.set_option("suspend", sus)
if lds:
    gs.set_option("lds_stack", lds)
try:
    img, st2 = gs.render_rows(cam, W, H, 0, H)
    print("ok", sus, lds, "pauses", gs.debug_counters()[35], "equal", np.array_equal(np.nan_to_num(img, nan=-9), np.nan_to_num(ref, nan=-9)), flush=True)
except Exception as e:
    print("ERR", sus, lds, e, "dbg", gs.debug_counters()[16:24], flush=True)
