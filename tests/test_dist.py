"""Multi-rank sharding + gather (bench.py's N>1 data path) on CPU with gloo.

Each rank renders its row strip -- here with the CPU oracle standing in for
the GPU renderer, since this test runs without a GPU -- and rank 0 must
reassemble exactly the full-image render."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import SCENES
from rtamd.dist import ImageGather, image_rows, row_set


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, scene, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle_py import OracleScene
    sc = OracleScene(scene, cwd=SCENES)
    W, H = sc.width, sc.height
    rows = image_rows(H, world, rank)
    g = ImageGather(H, W, world, rank, "cpu", torch)
    if rows:
        img, _ = sc.render(rows=np.array(rows))
        g.strip[: len(rows)] = torch.from_numpy(img)
    for _ in range(2):                    # buffers are reused frame after frame
        full = g.gather(dist)
    if rank == 0:
        out_q.put(full.numpy().copy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 5])
def test_gather_reassembles_image(world):
    scene = "test7_s.txt"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, scene, q)) for r in range(world)]
    for p in procs:
        p.start()
    full = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    from oracle_py import OracleScene
    ref, _ = OracleScene(scene, cwd=SCENES).render()
    assert np.array_equal(np.nan_to_num(full, nan=-9), np.nan_to_num(ref, nan=-9))


def test_row_sets_cover_image():
    for H in (1, 7, 64, 100, 4096, 4097):
        for world in (1, 2, 3, 8):
            rows = []
            for r in range(world):
                y0, b, step, n, per = row_set(H, world, r)
                assert 0 <= n <= per
                rr = image_rows(H, world, r)
                assert len(rr) == n and all(0 <= y < H for y in rr)
                rows += rr
            assert sorted(rows) == list(range(H))


@pytest.mark.parametrize("H", [1, 7, 8, 9, 64, 67, 1080, 4096])
@pytest.mark.parametrize("world", [1, 2, 3, 5, 8])
def test_cli_row_set_matches_dist(H, world):
    """The C++ CLI's multi-device row mapping (rth_row_set, librt_host) is the
    one the Python bench uses (rtamd.dist.row_set): every image row exactly
    once, equal-size gather buffers."""
    import ctypes as C
    import rtamd
    from rtamd.dist import row_set
    L = rtamd.host_lib()
    seen = []
    for r in range(world):
        y0, step, n, per = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        assert L.rth_row_set(H, world, r, 8, C.byref(y0), C.byref(step), C.byref(n), C.byref(per)) == 0
        py = row_set(H, world, r)
        assert (y0.value, 8, step.value, n.value, per.value) == py
        seen += [y0.value + (k // 8) * step.value + k % 8 for k in range(n.value)]
    assert sorted(seen) == list(range(H))
    y = C.c_int()
    assert L.rth_row_set(H, world, world, 8, C.byref(y), C.byref(y), C.byref(y), C.byref(y)) == -1
