#!/usr/bin/env python3
"""Benchmark: Mrays/s of the MI355X ray-trace hot path (BASELINE.json metric).

  python bench.py [--gpus N --steps K --warmup W] [--config C3]

One step = one render of the whole image of the workload (every primary,
shadow, refraction and reflection ray of the reference's TraceRay count,
SURVEY.md §8a).  Workload (N=1 and the default): config C3 of BASELINE.json,
4096x4096, 1000 spheres + 1000 triangles, reflection/refraction depth 4,
seeded synthetic scene (simple-raytracer_amd/rtamd/scenes.py).

Multi-GPU (torchrun, one process per GPU): the image's rows are dealt to the
ranks in 8-row blocks, round robin (strong scaling: the image is fixed); each
rank renders its rows into HBM and the row sets are gathered to rank 0 over
RCCL (torch.distributed "nccl") and put back in image order.  Timed region: barrier + synchronize on both
sides, K steps, max over ranks.  Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "simple-raytracer_amd"))

PEAK_FP32_TFLOPS = 157.3        # MI355X vector FP32 (MI355X_MICROARCH.md, chip table)
PEAK_HBM_GBPS = 8000.0          # HBM3E spec
FLOP_SPHERE, FLOP_TRI = 20, 42  # algorithmic FLOPs per ray-primitive test
# ray-box test as the kernel executes it per child box: 6 plane
# distances by FMA (12 FLOP), entry = max of 3 near distances and tmin (3),
# exit = min of 3 far distances and tmax (3), entry <= exit (1) -- the octant
# selects near/far planes without per-axis min/max; the binary16 bounds are
# converted inside the FMA (v_fma_mix_f32), so there is nothing else to count
FLOP_BOX = 19

WORKLOADS = {
    "C2": "C2: 1024x1024, 100 spheres, 2 point lights, no reflection/refraction",
    "C3": "C3: 4096x4096, 1000 spheres + 1000 triangles, reflection+refraction depth 4, 2 point lights",
    "C4": "C4: 8192x8192, 10k textured triangles, 1 directional + 1 point light (hard shadows)",
    "C5": "C5: 16384x16384, 100k spheres, reflection+refraction depth 8",
    "C3D": "C3 with a directional light (1,-1,-1) + a point light: unnormalised directional shadow rays "
           "against spheres (main.cpp:895)",
    "C3G": "C3 with 10% glass triangles: face-incident refraction, SKIP_TRANS (main.cpp:1000-1002)",
}


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="C3", choices=sorted(WORKLOADS))
    ap.add_argument("--cpu-baseline", default="auto", choices=["auto", "off"])
    ap.add_argument("--cpu-sample", type=int, default=256,
                    help="CPU legs: the reference renders the same scene at up to NxN (the port at up to "
                         "8N x 8N), sized for ~15 s / ~10 s (sized_run)")
    ap.add_argument("--option", action="append", default=[],
                    help="kernel option key=value (rt_scene_set_option)")
    ap.add_argument("--inflight", type=int, default=0,
                    help="frames in flight: step k renders on stream k mod F (rt_scene option "
                         "'inflight'), so one frame's tail overlaps the next frame's work; "
                         "0 = 2 at N=1 (3 or 4: no gain), 8 at N>1 (a rank's short frame leaves a long tail: "
                         "8 in flight take C3's N=8 share from 2.36 to 2.25 ms, profiles/r03/inflight_n8.txt)")
    ap.add_argument("--reserve", type=int, default=-1,
                    help="block slots the persistent render leaves free (rt_scene option 'reserve'); "
                         "-1 = 0 at N=1, 8 at N>1 (room for the RCCL gather beside the next frame)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend for N>1: nccl (= RCCL over xGMI), gloo only to rehearse "
                         "the multi-rank data path on one GPU (ranks share device 0)")
    ap.add_argument("--verify", action="store_true",
                    help="rank 0 checks the last gathered image bit for bit against one whole-image render")
    ap.add_argument("--gather-format", default="auto", choices=["auto", "f32", "u8"],
                    help="N>1: what rank 0 gathers -- f32 rows (12 B per pixel) or the P3 writer's "
                         "pixel values as bytes (3 B, quantised on each rank's GPU; exact for values "
                         "0..255). auto = u8 unless the warm-up frame has a value outside 0..255")
    ap.add_argument("--count-render", default="on", choices=["on", "off"],
                    help="after the timed region, one more render by the kernel instantiation with "
                         "counters (rays by kind for value, executed tests for the roofline; the timed "
                         "frames run without them); off for PMC passes that divide a run's counters by "
                         "its renders (the line's value is then 0)")
    ap.add_argument("--out-json", default=None)
    return ap.parse_args()


def scene_dir() -> str:
    d = os.path.join(os.environ.get("TMPDIR", tempfile.gettempdir()), "rtamd_bench_scenes")
    os.makedirs(d, exist_ok=True)
    return d


def sized_run(run, target_s: float, cap: int, side: int = 8):
    """A CPU leg's bounded sample: square renders of the config's scene from
    side x side, doubling while one takes under 1/16 of target_s, then one
    render sized for ~target_s seconds (at most cap x cap).  A 100 000-sphere
    scene renders a few hundred rays per second on one core, so a fixed
    sample would take minutes there and milliseconds on C2.  Each render is
    logged to stderr (a GPU lease kills a run that is silent for minutes).
    run(side) -> (rays, seconds); returns (rays, seconds, side)."""
    def timed(n):
        r, dt = run(n)
        print(f"[bench] cpu leg: {n}x{n}, {r} rays, {dt:.2f} s", file=sys.stderr, flush=True)
        return r, dt
    r, dt = timed(side)
    while dt < target_s / 16 and side * 2 <= cap:
        side *= 2
        r, dt = timed(side)
    new = int(min(cap, side * (target_s / max(dt, 1e-3)) ** 0.5)) // 8 * 8
    if new > side:
        side = new
        r, dt = timed(side)
    return r, dt, side


def cpu_baseline(config: str, sample: int, gpu_rays_fn, target_s: float = 15.0) -> dict | None:
    """The REAL reference (oracle/_ref/SimpleRayTracer, compiled from the
    reference's own sources by oracle/Makefile) timed on this host's cores on a
    bounded sample: the same seeded scene at side x side pixels (the whole
    field of view), side <= sample chosen for ~target_s seconds (sized_run).
    Rays of the sample are counted by the GPU path on the same scene file
    (counts are parity-tested equal to the reference's TraceRay calls)."""
    from rtamd import scenes as gen
    ref = os.path.join(ROOT, "oracle", "_ref", "SimpleRayTracer")
    if not os.path.exists(ref):
        return None                          # (cpu_port_baseline times this repo's port beside it)

    def run(side: int):
        d = tempfile.mkdtemp(prefix="rtamd_cpu_")
        path = gen.write_scene(d, config, w=side, h=side, tag=f"{config}_{side}")
        rays = gpu_rays_fn(path)
        t0 = time.perf_counter()
        subprocess.run([ref, os.path.basename(path)], cwd=d, check=True, stdout=subprocess.DEVNULL)
        return rays, time.perf_counter() - t0

    rays, dt, side = sized_run(run, target_s, sample)
    return {"value": rays / dt / 1e6, "unit": "Mrays/s", "cores": 1, "kind": "reference", "host": host_cores(),
            "sample": f"{config} scene at {side}x{side} (full field of view), {rays} rays, "
                      f"{dt:.1f} s, single-threaded reference binary"}


def cpu_port_baseline(config: str, sample: int, target_s: float = 10.0, threads: int | None = None) -> dict:
    """SURVEY.md §8d's CPU path: this repo's C restatement of the reference
    (oracle/rt_oracle.c: the same brute-force TraceRay/ShadeRay), OpenMP over
    rows on every core this process may run on (its affinity: all the node's
    CPUs the lease gives it, not the lease's OMP_NUM_THREADS share), timed on
    a render of the same seeded scene at a size chosen for ~target_s seconds
    (sized_run; at most sample x sample and the config's own image).  A
    reported baseline, not the product (the product path has no CPU
    fallback)."""
    from rtamd import scenes as gen
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_py import OracleScene
    host = host_cores()
    threads = threads or host["affinity"]

    def run(side: int):
        d = tempfile.mkdtemp(prefix="rtamd_port_")
        path = gen.write_scene(d, config, w=side, h=side, tag=f"{config}_{side}_port")
        o = OracleScene(path, cwd=d)         # (a textured scene names its texture relative to d)
        if o.rc:
            raise RuntimeError(f"oracle could not load {path}: {o.msg}")
        o.set_depth(gen.CONFIGS[config]["depth"])
        t0 = time.perf_counter()
        _, cnt = o.render(threads=threads)
        dt = time.perf_counter() - t0
        return sum(cnt[k] for k in ("primary", "shadow", "refraction", "reflection")), dt

    r, dt, side = sized_run(run, target_s, min(sample, gen.CONFIGS[config]["w"]))
    return {"value": r / dt / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port", "host": host,
            "sample": f"{config} scene at {side}x{side} (full field of view), {r} rays, {dt:.1f} s, "
                      f"C restatement (oracle/rt_oracle.c), OpenMP over rows on {threads} threads"
                      + (" (the process's affinity)" if threads == host["affinity"] else "")}


def host_cores() -> dict:
    """What the CPU legs may use: the machine's CPUs (nproc of the node), the
    ones this process may run on (its affinity), OMP_NUM_THREADS (0 when
    unset) and the cgroup's CPU quota in CPUs (cpu.max; None when unlimited or
    unreadable) -- a GPU lease can see every CPU of the node yet get the time
    of only a share of them."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count()
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"nproc": os.cpu_count(), "affinity": aff,
            "omp_num_threads": int(os.environ.get("OMP_NUM_THREADS", "0") or 0), "cgroup_cpus": quota}


def lib_sha16() -> str:
    """sha256 (first 16 hex) of the librt_hip.so this process loads."""
    import hashlib
    import rtamd
    with open(os.path.join(rtamd.LIB_DIR, "librt_hip.so"), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def load_pmc_traffic(config: str, lib: str):
    """HBM bytes per launch from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, tools/pmc_traffic.py), only when it was
    measured on this very library (its lib_sha16): (bytes or None, note)."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            e = json.load(f).get(config)
    except (OSError, ValueError):
        return None, "no profiles/pmc_traffic.json"
    if not e:
        return None, f"no PMC summary for {config}"
    if e.get("lib_sha16") != lib:
        return None, (f"the PMC summary ({e.get('source')}) was measured on librt_hip.so {e.get('lib_sha16')}, "
                      f"this run loads {lib}: traffic not reported")
    return e.get("hbm_bytes_per_launch"), f"PMC summary {e.get('source')} of this library"


def main() -> None:
    args = parse_args()
    import numpy as np
    import torch
    import torch.distributed as dist

    import rtamd
    from rtamd import scenes as gen

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and not (world == 1 and args.gpus == 1):
        if world == 1:
            raise SystemExit("bench.py --gpus N>1 must be launched with torchrun (one process per GPU)")
    dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group("gloo")

    cfg = gen.CONFIGS[args.config]
    sd = os.path.join(scene_dir(), f"rank{rank}")
    path = gen.write_scene(sd, args.config)
    hs = rtamd.HostScene(path, cwd=sd)
    hs.set_depth(cfg["depth"])
    W, H = hs.width, hs.height
    cam = hs.camera()
    gs = rtamd.GpuScene(hs, device=dev)
    for kv in args.option:
        k, v = kv.split("=")
        gs.set_option(k, int(v))

    # strong scaling: block-interleaved row sets (rtamd/dist.py), equal-size
    # buffers for the gather
    from rtamd.dist import ImageGather, row_set
    ry0, rblock, rstep, nrows, _ = row_set(H, world, rank)
    # F frames in flight: frame k renders into buffer k mod F, ordered on
    # stream k mod F (the render on a library stream of its own, the gather
    # after it); frame k+1 on the next stream overlaps frame k's tail.
    F = max(1, min(8, args.inflight if args.inflight > 0 else (2 if world == 1 else 8)))
    reserve = args.reserve if args.reserve >= 0 else (0 if world == 1 else 8)
    if reserve:
        gs.set_option("reserve", reserve)
    # the timed frames run the kernel instantiation without counters (rays by
    # kind, events, executed tests: registers live across the whole loop,
    # ~4 %); one render with them after the timed region gives the counts,
    # identical every frame (option counters; an --option counters=1 keeps them)
    counting = not any(kv.startswith("counters=") for kv in args.option)
    if counting:
        try:
            gs.set_option("counters", 0)
        except rtamd.RTError:     # a library before the option (A/B baselines): it always counts
            counting = False
    if F > 1:
        gs.set_option("inflight", F)
    gs.prepare(cam, W, H)                 # BVH + every slot's frame buffer, before any step
    fmt = "f32" if world == 1 or args.gather_format == "f32" else "u8"
    gathers = [ImageGather(H, W, world, rank, "cuda", torch, fmt) for _ in range(F)]
    streams = [torch.cuda.Stream() for _ in range(F)]
    for s in streams:                     # bind each stream to its hardware queue before timing
        with torch.cuda.stream(s):
            gathers[0].strip[:1].zero_()
    torch.cuda.synchronize()

    def step(k):
        s, g = streams[k % F], gathers[k % F]
        with torch.cuda.stream(s):
            if nrows > 0:
                gs.render_row_blocks_async(cam, W, H, ry0, rblock, rstep, nrows, g.strip.data_ptr(),
                                           s.cuda_stream)
            return g.gather(dist)

    def any_flag() -> bool:
        # a value outside 0..255 on any rank (u8 gathers): the bytes are not the writer's
        f = torch.zeros(1, dtype=torch.int32, device="cuda")
        for g in gathers:
            if g.flag is not None:
                f |= g.flag
        if world > 1:
            ff = f if args.dist_backend == "nccl" else f.cpu()
            dist.all_reduce(ff, op=dist.ReduceOp.MAX)
            f = ff
        return bool(int(f.item()))

    for k in range(args.warmup if fmt == "f32" else max(1, args.warmup)):
        step(k)
    torch.cuda.synchronize()
    if fmt == "u8" and any_flag():
        if args.gather_format == "u8":
            raise SystemExit("--gather-format u8: the image has values outside 0..255")
        fmt = "f32"
        gathers = [ImageGather(H, W, world, rank, "cuda", torch, fmt) for _ in range(F)]
        for k in range(max(1, args.warmup)):
            step(k)
        torch.cuda.synchronize()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        last_img = step(k)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if fmt == "u8" and any_flag():     # the frames are identical: cannot differ from the warm-up's
        raise SystemExit("u8 gather: a timed frame had values outside 0..255")
    verified = None
    if args.verify and rank == 0:
        # the last timed step's image (all ranks' rows, gathered and put back in
        # image order) against one whole-image render on this device
        ref = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
        vs = rtamd.GpuScene(hs, device=dev)
        vs.render_rows_async(cam, W, H, 0, H, ref.data_ptr(), torch.cuda.current_stream().cuda_stream)
        vs.last_stats()
        if fmt == "u8":                   # the gathered bytes against the whole render's
            from rtamd.dist import quantize_u8_device
            ref8 = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")
            flag = torch.zeros(1, dtype=torch.int32, device="cuda")
            quantize_u8_device(rtamd, torch, ref, ref8, flag)
            ref = ref8
        torch.cuda.synchronize()
        a, b = torch.nan_to_num(last_img.float(), nan=-9.0), torch.nan_to_num(ref.float(), nan=-9.0)
        verified = bool(torch.equal(a, b))
        vs.close()
        if not verified:
            raise SystemExit(f"verify: gathered image differs from the whole-image render in "
                             f"{int((a != b).any(dim=-1).sum())} pixels")
    # the last timed frame's image (this rank's rows, as the kernel without
    # counters rendered them), kept before the frames below reuse the buffers
    timed_rows = gathers[(args.steps - 1) % F].strip.clone() if nrows > 0 and args.steps > 0 else None
    # single-frame latency (nothing else in flight), after the timed region
    torch.cuda.synchronize()
    lat0 = time.perf_counter()
    step(0)
    torch.cuda.synchronize()
    latency_ms = (time.perf_counter() - lat0) * 1e3
    st_time = gs.last_stats()     # that render's clock
    dbg = gs.debug_counters()
    # device time of one launch with no other frame on the CUs (first wave start
    # .. last wave end on the kernel's own clock; what rocprofv3 reports per
    # dispatch at --inflight 1)
    kernel_ms = [st_time.kernel_ms]
    # the counts (rays by kind for `value`, known-zero shadow rays, executed
    # tests for the roofline) from one more render by the counting
    # instantiation; the roofline divides its tests by the uncounted launch's
    # time above
    st = st_time
    verified_rows = None
    if args.count_render == "on":
        # the counting render writes a buffer of its own; the timed frame must
        # equal it bit for bit (NaN for NaN) on every rank: the benched
        # instantiation is checked on the very frame the line times, against
        # the instantiation every parity test pins to the oracle
        if counting:
            gs.set_option("counters", 1)
        cnt_rows = torch.empty_like(gathers[0].strip)
        s0 = torch.cuda.current_stream()
        if nrows > 0:
            gs.render_row_blocks_async(cam, W, H, ry0, rblock, rstep, nrows, cnt_rows.data_ptr(), s0.cuda_stream)
        torch.cuda.synchronize()
        st = gs.last_stats()
        if counting:
            gs.set_option("counters", 0)
        same = True
        if timed_rows is not None:
            a = torch.nan_to_num(timed_rows[:nrows], nan=-9.0)
            b = torch.nan_to_num(cnt_rows[:nrows], nan=-9.0)
            same = bool(torch.equal(a, b))
        ok = torch.tensor([1 if same else 0], dtype=torch.int32,
                          device="cuda" if args.dist_backend == "nccl" else "cpu")
        if world > 1:
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        verified_rows = bool(int(ok.item()))
        del cnt_rows
        if not verified_rows:
            raise SystemExit("verify: the last timed frame differs from the counting render of the same rows")
    st_tests = st
    my_rays = st.rays()

    t = torch.tensor([elapsed, float(my_rays), float(np.mean(kernel_ms)), latency_ms], dtype=torch.float64,
                     device="cuda" if args.dist_backend == "nccl" else "cpu")
    if world > 1:
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = t.clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        elapsed, rays_total, kmax, latency_ms = float(tmax[0]), float(tsum[1]), float(tmax[2]), float(tmax[3])
    else:
        rays_total, kmax = float(my_rays), float(np.mean(kernel_ms))

    if rank == 0:
        value = rays_total * args.steps / elapsed / 1e6
        # rays actually searched: shadow rays whose cumulative mask was already
        # 0 are TraceRay calls of the reference (so in `value`) but are not
        # searched (their result is known); rank 0's share scaled to the job
        known = float(st.shadow_known) * (rays_total / my_rays if my_rays else 0.0)
        value_traced = (rays_total - known) * args.steps / elapsed / 1e6
        ns, nt = cfg["spheres"], cfg["tris"]
        bf_flop_per_ray = FLOP_SPHERE * ns + FLOP_TRI * nt
        # dominant kernel = render_kernel; per launch on rank 0 (its strip).
        # achieved = FLOPs of the tests the launch executed (ray-box + ray-face +
        # ray-sphere, counted by the kernel) / its average launch time.
        k_s = float(np.mean(kernel_ms)) / 1e3
        flops = st_tests.box_tests * FLOP_BOX + st_tests.face_tests * FLOP_TRI + st_tests.sphere_tests * FLOP_SPHERE
        achieved = flops / k_s / 1e12
        bf_equiv = my_rays * bf_flop_per_ray / k_s / 1e12
        px = nrows * W
        scene_bytes = 80 * nt + 16 * ns + 52 * (ns + nt)
        alg_bytes = 12 * px + scene_bytes
        # PMC bytes were collected for a whole-image launch: only the N=1 line's
        # launch is that launch (a rank's strip at N>1 is not measured)
        lib = lib_sha16()
        traffic, traffic_note = load_pmc_traffic(args.config, lib) if world == 1 else (None, "N = 1 only")
        cpu = cpu_port = None
        if args.cpu_baseline == "auto" and world == 1:
            def gpu_rays(p):
                _, s = rtamd.render_scene(p, cwd=os.path.dirname(p), depth=cfg["depth"], device=local)
                return s.rays()
            try:
                cpu = cpu_baseline(args.config, args.cpu_sample, gpu_rays)
            except Exception as e:  # never lose the GPU line to the CPU leg
                cpu = {"error": repr(e)}
            try:
                # every core the process may run on (its affinity) -- and, when
                # the lease's OMP_NUM_THREADS share is smaller, that share too:
                # a lease whose cgroup gives it the time of only some of the CPUs
                # it sees runs the oversubscribed affinity count slower.  The
                # baseline is the faster of the two (the port on
                # every core the host actually delivers)
                runs = [cpu_port_baseline(args.config, 8 * args.cpu_sample)]
                h = runs[0]["host"]
                share = h["omp_num_threads"] or (int(h["cgroup_cpus"]) if h["cgroup_cpus"] else 0)
                if 0 < share < h["affinity"]:
                    runs.append(cpu_port_baseline(args.config, 8 * args.cpu_sample, threads=share))
                cpu_port = dict(max(runs, key=lambda r: r["value"]))
                cpu_port["runs"] = [{k: r[k] for k in ("value", "cores", "sample")} for r in runs]
                cpu_port["note"] = ("the faster of the port on every affinity CPU and on the lease's "
                                    "OMP_NUM_THREADS / cgroup share (runs: both)")
            except Exception as e:
                cpu_port = {"error": repr(e)}
        line = {
            "metric": "Mrays/s (primary+secondary)",
            "value": round(value, 3),
            "unit": "Mrays/s",
            "value_traced": round(value_traced, 3),
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "frame_latency_ms": round(latency_ms, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded scene generator, rtamd/scenes.py)",
            "config": {"workload": WORKLOADS[args.config], "imsize": [W, H], "spheres": ns,
                       "triangles": nt, "depth": cfg["depth"], "lights": 2,
                       "rays_per_step": int(rays_total), "parallelism": f"interleaved 8-row blocks x{world}"
                       + ((" + RCCL gather" if args.dist_backend == "nccl" else " + gloo gather (rehearsal, one GPU)")
                          if world > 1 else ""), "frames_in_flight": F,
                       "gather_format": (fmt + (" (the P3 writer's values, 3 B/pixel)" if fmt == "u8" else
                                                " (12 B/pixel)")) if world > 1 else None,
                       "reserved_block_slots": reserve,
                       "launch": {"blocks_per_cu": int(dbg[17]), "grid": int(dbg[18]),
                                  "lds_bytes_per_block": int(dbg[19]), "bvh_nodes": int(dbg[20]),
                                  "lds_stack": int(dbg[42]), "lights_in_lds": int(dbg[43]),
                                  "org_first": int(dbg[40]), "scene_density": round(dbg[41] / 1000, 2)}},
            "one_frame": {"Mrays_per_s": round(my_rays / k_s / 1e6, 3) if world == 1 else None,
                          "Mrays_per_s_traced": round((my_rays - st.shadow_known) / k_s / 1e6, 3)
                          if world == 1 else None,
                          "kernel_ms": round(float(np.mean(kernel_ms)), 3),
                          "note": "one frame alone on the GPU (kernel clock); value pipelines "
                                  f"{F} frames in flight"},
            "work": {"shadow_known_zero": int(st.shadow_known), "traced_rays": int(my_rays - st.shadow_known),
                     "bf_queries": int(st.bf_queries),
                     "stack_spills": int(st.stack_spills), "bvh_build_ms": round(st.bvh_build_ms, 2),
                     "note": "shadow_known_zero: shadow rays counted in value whose cumulative mask was "
                             "already 0 (result known, not searched; value_traced leaves them out); "
                             "bvh_build_ms: host build before the timed region, not in value"},
            "roofline": {"bound": "valu", "achieved": round(achieved, 3), "peak": PEAK_FP32_TFLOPS,
                         "basis": "FLOPs of the ray-box/face/sphere tests the launch executed (kernel "
                                  "counters x flop_per_test) / kernel_ms; replaces SURVEY 8(d)'s brute-force "
                                  "basis, which exceeds peak once the BVH skips ~98% of the tests "
                                  "(brute_force_equivalent)",
                         "unit": "TFLOP/s", "frac": round(achieved / PEAK_FP32_TFLOPS, 4),
                         "traffic": traffic, "traffic_note": traffic_note, "lib_sha16": lib,
                         "kernel": "render_kernel",
                         "kernel_ms": round(float(np.mean(kernel_ms)), 3),
                         "per_step": {"achieved": round(flops / (elapsed / args.steps) / 1e12, 3),
                                      "frac": round(flops / (elapsed / args.steps) / 1e12
                                                    / PEAK_FP32_TFLOPS, 4)},
                         "rays_per_launch": my_rays,
                         "tests_per_launch": {"box": st_tests.box_tests, "face": st_tests.face_tests,
                                              "sphere": st_tests.sphere_tests},
                         "flop_per_test": {"box": FLOP_BOX, "face": FLOP_TRI, "sphere": FLOP_SPHERE},
                         "brute_force_equivalent": {"flop_per_ray": bf_flop_per_ray,
                                                    "TFLOPs": round(bf_equiv, 3),
                                                    "frac": round(bf_equiv / PEAK_FP32_TFLOPS, 4)},
                         "hbm": {"alg_bytes_per_launch": alg_bytes,
                                 "achieved_GBps": round(alg_bytes / k_s / 1e9, 3),
                                 "peak_GBps": PEAK_HBM_GBPS,
                                 "frac": round(alg_bytes / k_s / 1e9 / PEAK_HBM_GBPS, 7)}},
            # the baseline is the C restatement on the host's
            # cores (kind "port"); the real reference binary on one core is the
            # anchor beside it (kind "reference")
            "cpu_baseline": cpu_port if cpu_port is not None and "error" not in cpu_port else cpu,
            "cpu_reference_anchor": cpu,
            "verified": (None if verified_rows is None and verified is None
                         else all(v for v in (verified_rows, verified) if v is not None)),
            "verified_rows": verified_rows,
            "verified_gather": verified,
            "verified_note": "verified_rows: every rank's rows of the last timed frame (render_kernel without "
                             "counters) equal bit for bit (NaN for NaN) the counting instantiation's render "
                             "of the same rows, which the parity tests pin to the oracle; verified_gather "
                             "(--verify, rank 0): the gathered image equals one whole-image render; "
                             "verified: every check that ran passed",
            "ray_counts": {k: int(getattr(st, k)) for k in ("primary", "shadow", "refraction",
                                                             "reflection", "skip_trans", "ub_back")},
        }
        s = json.dumps(line)
        print(s, flush=True)
        if args.out_json:
            with open(args.out_json, "w") as f:
                f.write(s + "\n")
    gs.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
