"""bench.py's CPU baseline leg (the oracle port timed on the host, SURVEY.md
§8d): it loads each config's seeded scene from the directory the generator
wrote it to -- C4 names its texture relative to that directory (round 5:
loading it from the working directory failed and the unchecked handle
crashed bench.py --config C4) -- and a scene the oracle cannot load raises
instead of reaching the C library with no scene."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "simple-raytracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


@pytest.mark.parametrize("config", ["C3", "C4"])
def test_cpu_port_baseline_loads_config_scene(config):
    import bench
    r = bench.cpu_port_baseline(config, 16, target_s=0.05, threads=2)
    assert r["kind"] == "port" and r["cores"] == 2
    assert r["value"] > 0
    side = int(r["sample"].split(" scene at ")[1].split("x")[0])
    assert 8 <= side <= 16 and side % 8 == 0, r["sample"]      # (the cap: sample 16)


def test_sized_run_bounds_the_sample():
    """sized_run doubles a cheap probe until it takes 1/16 of the target, then
    sizes one render for the target, never above the cap; an expensive probe
    (a 100 000-sphere scene) stays small."""
    import bench
    cost = {}

    def run(side, per_px=1e-6):
        dt = side * side * per_px
        cost[side] = dt
        return side * side, dt
    r, dt, side = bench.sized_run(run, 1.0, 4096)
    assert side == 1000 and abs(dt - 1.0) < 0.01
    r, dt, side = bench.sized_run(lambda s: run(s, 1e-6), 1.0, 256)
    assert side == 256
    r, dt, side = bench.sized_run(lambda s: run(s, 0.1), 10.0, 4096)      # 6.4 s for the 8x8 probe
    assert side == 8


def test_oracle_scene_unloaded_raises(tmp_path):
    from oracle_py import OracleScene
    o = OracleScene(str(tmp_path / "missing.txt"))
    assert o.rc != 0
    with pytest.raises(RuntimeError):
        o.set_depth(4)
    with pytest.raises(RuntimeError):
        o.render(threads=1)
