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
    assert f"{config} scene at 16x16" in r["sample"]


def test_oracle_scene_unloaded_raises(tmp_path):
    from oracle_py import OracleScene
    o = OracleScene(str(tmp_path / "missing.txt"))
    assert o.rc != 0
    with pytest.raises(RuntimeError):
        o.set_depth(4)
    with pytest.raises(RuntimeError):
        o.render(threads=1)
