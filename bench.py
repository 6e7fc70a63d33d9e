#!/usr/bin/env python3
"""Benchmark of the MI355X grid-indexed point-in-polygon join (BASELINE.json metric).

Workload (BASELINE.json configs[1], "C2"): 100M synthetic points per GPU, uniform in
the NYC taxi-zone bounding box, joined against the 263 NYC taxi zones
(python/test/data/NYC_Taxi_Zones.geojson, committed as tests/golden/nyc_taxi_zones.npz)
tessellated at H3 resolution 9.  One step = one join (cell id -> chip probe -> is_core OR
st_contains -> ordered pair output) over the GPU's resident points.

Multi-GPU (one process per GPU): `--gpus N` under torchrun (WORLD_SIZE set) runs as that
rank; without WORLD_SIZE and N > 1 it starts the N ranks itself (child processes, before
anything touches a GPU) and exits with their status -- never a 1-GPU line for N GPUs.
Points are sharded by contiguous id range (weak scaling: the per-GPU point count is
fixed), the chip table is built on rank 0 and replicated with one RCCL broadcast; every
timed step ends with the RCCL all-gather of the per-rank pair counts (this rank's slice of
the globally ordered output) -- both through the C ABI (mgpu_comm_init,
mgpu_chips_broadcast, mgpu_pair_offsets; mosaic_amd/csrc/comm.cpp).  torch.distributed
(gloo) is only the control plane: the RCCL unique id, the barriers and the max over
ranks of the barrier-bracketed K steps.

A step is one mgpu_pip_join call, whichever of the library's three pipelines its planner
picks for the chip table: split (C2, C5: classify_pair_kernel over every
point by its pixel, pip_mixed_kernel for the mixed ones, split_emit_kernel), binned (C3:
bin_hist / bin_scatter, pip_binned_kernel over the binned points, bin_gather /
bin_emit) or fused (C4: pip_join_kernel, pip_fix_kernel, tile_scan_kernel,
pair_emit_kernel).  Every step ends with the ordered (point_id, polygon_id) pairs.

Also reported: the dominant kernel's achieved bandwidth against the HBM roofline --
algorithmic bytes per launch (classify 18 B/point; binned join 24 B/point;
fused join 16 B/point + 8 B/pair + 12 B/tile) over its average duration measured with HIP
events on the launch stream -- the HBM bytes the PMC counters saw for that kernel
(profiles/pmc_join_traffic*.json, when measured on this workload and kernel), the
PCIe-inclusive rate (points in pinned host memory, pairs back to it; never `value`), and
a CPU baseline: the oracle's multithreaded C restatement of the reference path on a
bounded sample (rank 0, N=1 only).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

NYC_BBOX = (-74.25559136315209, 40.496115395170364, -73.7000090639354, 40.91553277700258)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
METRIC = "PIP-join points/sec (H3 res 9) at 1/2/4/8 GPUs + achieved HBM GB/s"


def log(msg):
    """Progress to stderr (setup of the large configs takes a minute)."""
    print("[bench %.1fs] %s" % (time.perf_counter() - T_START, msg), file=sys.stderr, flush=True)


T_START = time.perf_counter()


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--points", type=int, default=None, help="points per GPU (default 1e8; c3: 1.25e8)")
    ap.add_argument("--config", default="c2", choices=["c2", "c3", "c4", "c5"],
                    help="BASELINE.json config: c2 (default, the headline), c3 (74k tracts, res 10), "
                         "c4 (BNG), c5 (skewed)")
    ap.add_argument("--res", type=int, default=None, help="default: 9 (c2, c5), 10 (c3), 4 (c4)")
    ap.add_argument("--seed", type=int, default=0x20250314)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pcie", action="store_true", help="skip the PCIe-inclusive measurement")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample duration")
    ap.add_argument("--option", action="append", default=[], metavar="KEY=VALUE",
                    help="context option (mgpu_ctx_set_option, include/mosaic_gpu.h) set before the chip table "
                         "is uploaded, e.g. raster_bng=1 or pipeline=0; repeatable")
    return ap.parse_args()


def gen_points(n, begin, seed, dev):
    """Uniform points in the NYC bbox; the shard starting at global index `begin` is
    generated from its own seeded stream so any world size sees the same workload shape."""
    g = torch.Generator(device=dev)
    g.manual_seed(seed * 1000003 + begin)
    x = torch.rand(n, dtype=torch.float64, device=dev, generator=g)
    y = torch.rand(n, dtype=torch.float64, device=dev, generator=g)
    x.mul_(NYC_BBOX[2] - NYC_BBOX[0]).add_(NYC_BBOX[0])
    y.mul_(NYC_BBOX[3] - NYC_BBOX[1]).add_(NYC_BBOX[1])
    return x, y


def cpu_baseline(chips, isys, res, wl, seed, target_s):
    """Oracle (CPU restatement of the reference path) on a bounded sample: points/s.
    Chunks of up to 20M points until ~target_s seconds of join time are spent."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    threads = max(1, min(threads, 64))
    chunk_seed = [seed]

    def run(n):
        chunk_seed[0] += 1
        x, y = wl["points_np"](n, chunk_seed[0])
        t = time.perf_counter()
        O.pip_join(isys.code, res, x, y, chips.cell, chips.polygon_id, chips.is_core, chips.wkb_offsets, chips.wkb,
                   threads=threads)
        return time.perf_counter() - t

    n0 = 200_000
    dt0 = run(n0)
    rate = n0 / max(dt0, 1e-6)
    total_n, total_t = 0, 0.0
    while total_t < target_s:
        n = int(min(20_000_000, max(n0, rate * min(target_s - total_t, 5.0))))
        total_t += run(n)
        total_n += n
    return {"value": total_n / total_t, "unit": "points/s", "cores": threads, "kind": "port",
            "sample": "%d points (chunks of <= 20M) of the same workload, %s res %d, oracle pip_join "
                      "(C restatement of the reference's cell id + hash join on cell + JTS PointLocator with "
                      "per-candidate WKB re-parse, as its JVM path does), %d threads, %.1f s"
                      % (total_n, isys.name, res, threads, total_t)}


def pcie_inclusive(x, y, chips, res, isys, begin, cap, M, reps=3):
    """The same join with its points starting in (pinned) host memory and its pairs
    ending there: H2D copy + join + D2H copy of the pairs, on one stream (SURVEY §8d's
    second number; never `value`)."""
    dev = x.device
    hx = torch.empty(x.numel(), dtype=torch.float64, pin_memory=True)
    hy = torch.empty(y.numel(), dtype=torch.float64, pin_memory=True)
    hx.copy_(x)
    hy.copy_(y)
    hp = torch.empty(cap, dtype=torch.int64, pin_memory=True)
    hq = torch.empty(cap, dtype=torch.int32, pin_memory=True)
    dx, dy = torch.empty_like(x), torch.empty_like(y)
    dp = torch.empty(cap, dtype=torch.int64, device=dev)
    dq = torch.empty(cap, dtype=torch.int32, device=dev)
    ts = []
    for _ in range(reps + 1):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        dx.copy_(hx, non_blocking=True)
        dy.copy_(hy, non_blocking=True)
        r = M.pip_join(dx, dy, chips, res, index_system=isys, point_id_base=begin, out=(dp, dq), capacity=cap)
        m = len(r)
        hp[:m].copy_(dp[:m], non_blocking=True)
        hq[:m].copy_(dq[:m], non_blocking=True)
        torch.cuda.synchronize(dev)
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts[1:]))
    n = x.numel()
    return {"value": n / t, "unit": "points/s", "ms_per_step": t * 1e3,
            "bytes_over_pcie": 16 * n + 12 * m,
            "note": "points in pinned host memory, H2D copy + join + D2H copy of the pairs, median of %d" % reps}


def workload(a, W, M):
    """The config's polygons, index system and point generators (bench_workloads.py)."""
    if a.config == "c3":
        a.res = 10 if a.res is None else a.res
        a.points = 125_000_000 if a.points is None else a.points
        E = W.TRACT_EXTENT
        return {"isys": M.H3IndexSystem(), "polygons": W.tract_polygons(),
                "points": lambda n, begin, dev: W.extent_points(E, n, a.seed * 1000003 + begin, dev),
                "points_np": lambda n, sd: W.extent_points(E, n, sd),
                "pairs_per_point": 1.05, "keep_core": False,
                "workload": "C3: %d points/GPU uniform in lon [-77.5, -73.5] x lat [39.5, 42.5] x 74,000 "
                            "census-tract-like polygons (seeded Voronoi, jittered shared edges, 17-337 vertices), "
                            "H3 res %d; chips from grid_tessellateexplode(keepCoreGeometries=false)",
                "data": "synthetic (uniform points; seeded tract-like Voronoi partition of the extent)"}
    if a.config == "c4":
        a.res = 4 if a.res is None else a.res
        a.points = 100_000_000 if a.points is None else a.points
        return {"isys": M.BNGIndexSystem(), "polygons": W.london_districts(),
                "points": lambda n, begin, dev: W.london_points(n, a.seed * 1000003 + begin, dev),
                "points_np": lambda n, sd: W.london_points(n, sd),
                "pairs_per_point": 1.1,
                "workload": "C4: %d points/GPU uniform in the London BNG extent (0.01 m) x 180 UK-style districts "
                            "(seeded Voronoi partition, jittered edges), BNG res %d",
                "data": "synthetic (UPRN-like points; Voronoi districts covering the extent)"}
    if a.config == "c5":
        a.res = 9 if a.res is None else a.res
        a.points = 100_000_000 if a.points is None else a.points
        P = W.skewed_polygons()
        return {"isys": M.H3IndexSystem(), "polygons": P,
                "points": lambda n, begin, dev: W.boundary_points(P, n, a.seed * 1000003 + begin, 0.003, dev),
                "points_np": lambda n, sd: W.boundary_points(P, n, sd, 0.003),
                "pairs_per_point": 0.7,
                "workload": "C5: %d points/GPU, 90%% Gaussian (sigma 0.003 deg) around the boundaries of 4 "
                            "fractal polygons of 49k vertices, H3 res %d",
                "data": "synthetic (skewed points near polygon edges; seeded fractal polygons)"}
    a.res = 9 if a.res is None else a.res
    a.points = 100_000_000 if a.points is None else a.points
    return {"isys": M.H3IndexSystem(), "polygons": W.nyc_zones(),
            "points": lambda n, begin, dev: gen_points(n, begin, a.seed, dev),
            "points_np": lambda n, sd: (np.random.default_rng(sd).uniform(NYC_BBOX[0], NYC_BBOX[2], n),
                                        np.random.default_rng(sd + 7).uniform(NYC_BBOX[1], NYC_BBOX[3], n)),
            "pairs_per_point": 0.5,
            "workload": "C2: %d points/GPU uniform in NYC bbox x 263 NYC taxi zones, H3 res %d",
            "data": "synthetic (uniform points in the NYC zone bbox; real NYC taxi-zone polygons from the reference)"}


def spawn_ranks(a):
    """`--gpus N` without a launcher: start N ranks of this script (one per GPU, the
    torchrun environment variables set, rendezvous on 127.0.0.1) and return the first
    failing rank's status (the others are then stopped).  Nothing here touches a GPU:
    counting devices does not initialise one on this stack."""
    import socket
    import subprocess
    have = torch.cuda.device_count()
    if have < a.gpus and os.environ.get("MGPU_DIST_BACKEND", "rccl") != "gloo":
        print("--gpus %d: only %d GPUs visible" % (a.gpus, have), file=sys.stderr)
        return 2
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus), LOCAL_WORLD_SIZE=str(a.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    while procs:
        for p in list(procs):
            st = p.poll()
            if st is None:
                continue
            procs.remove(p)
            if st != 0 and rc == 0:
                rc = st
                for q in procs:
                    q.terminate()
        time.sleep(0.05)
    return rc


def traffic_key(options, info):
    """What a PMC traffic profile (profiles/pmc_join_traffic*.json, tools/traffic_summary.py)
    must share with a bench line to be attached to it: the context options, the uploaded
    table (chips, blob bytes) and the kernels' source."""
    import hashlib
    src = os.path.join(ROOT, "mosaic_amd", "csrc", "kernels.hip")
    return {"options": dict(sorted(kv.split("=", 1) for kv in options)), "chips": int(info["chips"]),
            "blob_bytes": int(info.get("bytes") or 0),
            "kernels_sha16": hashlib.sha256(open(src, "rb").read()).hexdigest()[:16]}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "0"))
    if world == 0 and a.gpus > 1:
        sys.exit(spawn_ranks(a))
    world = max(world, 1)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus != world:
        raise SystemExit("--gpus %d but WORLD_SIZE %d" % (a.gpus, world))
    import mosaic_amd as M
    from mosaic_amd import dist as D
    # MGPU_DIST_BACKEND=gloo and more ranks than GPUs: a protocol rehearsal on a
    # 1-GPU box (never a measurement: the chip blob and the counts travel over gloo);
    # the real run is RCCL through the C ABI, one rank per GPU
    rehearsal = os.environ.get("MGPU_DIST_BACKEND", "rccl") == "gloo"
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")  # control plane only
    ctx = M.default_context(dev)
    for kv in a.option:
        k, v = kv.split("=", 1)
        ctx.set_option(k, int(v))
    if world > 1 and not rehearsal:
        D.init_comm(ctx)
    import bench_workloads as W
    wl = workload(a, W, M)
    isys, zones = wl["isys"], wl["polygons"]
    log("config %s: %d polygons" % (a.config, len(zones)))
    table = None
    setup = {"tessellate_s": 0.0, "upload_s": 0.0, "broadcast_s": 0.0}
    if rank == 0:
        # setup (grid_tessellateexplode's chip table, built once per polygon
        # set): the host tessellator, the blob build + upload, the replication
        t = time.perf_counter()
        table = M.tessellate(zones, isys, a.res, keep_core_geometries=wl.get("keep_core", True))
        setup["tessellate_s"] = time.perf_counter() - t
        log("tessellated: %d chips (%.2f s)" % (len(table), setup["tessellate_s"]))
        t = time.perf_counter()
        chips = table.upload(ctx)
        torch.cuda.synchronize(dev)
        setup["upload_s"] = time.perf_counter() - t
        log("chip table uploaded (%.2f s)" % setup["upload_s"])
    else:
        chips = None
    if world > 1:
        dist.barrier()
        t = time.perf_counter()
        if not rehearsal:
            chips = D.broadcast_chips(chips, ctx)
        else:
            blob = D.broadcast_host_blob(D.host_blob(table) if rank == 0 else None, 0)
            chips = chips if rank == 0 else D.upload_host_blob(blob, ctx)
        torch.cuda.synchronize(dev)
        tb = torch.tensor([time.perf_counter() - t], dtype=torch.float64)
        dist.all_reduce(tb, op=dist.ReduceOp.MAX)
        setup["broadcast_s"] = float(tb.item())
    info = chips.info()

    n = a.points
    begin = rank * n
    x, y = wl["points"](n, begin, dev)
    cap = int(n * wl["pairs_per_point"]) + 1024
    out_p = torch.empty(cap, dtype=torch.int64, device=dev)
    out_q = torch.empty(cap, dtype=torch.int32, device=dev)
    ctx.reserve(n)

    def step():
        r = M.pip_join(x, y, chips, a.res, index_system=isys, point_id_base=begin, out=(out_p, out_q),
                       capacity=cap)
        # N > 1: this rank's slice of the globally ordered output (RCCL all-gather of the
        # per-rank pair counts, mgpu_pair_offsets), part of every step
        if world > 1:
            r.offsets = D.gather_offsets_host(len(r)) if rehearsal else D.global_offsets(len(r), ctx)
        return r

    log("points generated; warmup")
    for _ in range(a.warmup):
        r = step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    kms, sms = [], []
    pairs = 0
    ties = 0
    mms, ems = [], []
    for _ in range(a.steps):
        r = step()
        kms.append(r.stats["kernel_ms"])
        sms.append(r.stats["stream_kernel_ms"])
        mms.append(r.stats["mixed_kernel_ms"])
        ems.append(r.stats["emit_kernel_ms"])
        pairs = len(r)
        ties = r.stats["n_near_ties"]
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        off, total_pairs, _ = r.offsets
    else:
        total_pairs = pairs

    ms_step = elapsed / a.steps * 1e3
    pipeline_ms = float(np.mean(kms))
    stream_ms = float(np.mean(sms))
    split = r.stats["pipeline"] == M._native.MGPU_PIPELINE_SPLIT
    binned = r.stats["pipeline"] == M._native.MGPU_PIPELINE_BINNED
    if binned:
        # the binned pipeline: the dominant kernel is pip_binned_kernel, the
        # join over the binned points: 16 B read + its 8-byte answer written per point
        kernel = "pip_binned_kernel<%s>" % isys.name
        alg_bytes = 24.0 * n
    elif split:
        # the split pipeline: the dominant kernel is the classify pass over every
        # point: 16 B read + its code (2 B H3 / 4 B BNG) written per point --
        # classify_pair_kernel (two points per lane, 16-byte loads) when both coordinate
        # arrays are 16-byte aligned, as torch's allocations are, else classify_wave_kernel
        pair = x.data_ptr() % 16 == 0 and y.data_ptr() % 16 == 0
        kernel = "%s<%s>" % ("classify_pair_kernel" if pair else "classify_wave_kernel", isys.name)
        alg_bytes = (16.0 + (2.0 if isys.code == M._native.MGPU_H3 else 4.0)) * n
    else:
        kernel = "pip_join_kernel<%s>" % isys.name
        tp = M._native.lib().mgpu_join_tile_points()
        tiles = (n + tp - 1) // tp
        alg_bytes = 16.0 * n + 8.0 * pairs + 12.0 * tiles
    achieved = alg_bytes / (stream_ms * 1e-3) / 1e9
    out = {
        "metric": METRIC,
        "value": world * n / (elapsed / a.steps),
        "unit": "points/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": wl["data"],
        "config": {"workload": wl["workload"] % (n, a.res),
                   "points_per_gpu": n, "polygons": len(zones.poly_part_off) - 1, "chips": info["chips"],
                   "chip_cells": info["cells"], "index_system": isys.name, "resolution": a.res,
                   **({"options": dict(kv.split("=", 1) for kv in a.option)} if a.option else {}),
                   "parallelism": ("points sharded x%d, chip table replicated (%s)"
                                   % (world, "gloo host blob: a protocol rehearsal, not a measurement" if rehearsal
                                      else "RCCL broadcast") if world > 1 else "one GPU")},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "kernel": kernel, "kernel_ms": stream_ms,
                     "alg_bytes_per_launch": alg_bytes, "pipeline_ms": pipeline_ms,
                     # the whole call: 16 B per point in, 12 B per (point_id, polygon_id) pair out
                     "pipeline_GBps": (16.0 * n + 12.0 * pairs) / (pipeline_ms * 1e-3) / 1e9,
                     "pipeline_frac": (16.0 * n + 12.0 * pairs) / (pipeline_ms * 1e-3) / 1e9 / HBM_PEAK_GBS},
        "pipeline": "split" if split else ("binned" if binned else "fused"),
        "kernels_ms": ({"classify": stream_ms, "mixed": float(np.mean(mms)), "emit": float(np.mean(ems))} if split
                       else {"bin": float(np.mean(mms)), "pip_binned": stream_ms, "emit": float(np.mean(ems))} if binned
                       else {"pip_join": stream_ms, "rest": pipeline_ms - stream_ms}),
        # once per chip table, outside the timed steps (rank 0 builds, every rank receives)
        "setup_s": dict(setup, total_s=sum(setup.values()),
                        core_rule="mosaicfill", chip_stats=(table.core_stats if table is not None else None),
                        blob_bytes=info.get("bytes")),
        "pairs_per_gpu": pairs,
        "pairs_total": total_pairs,
        "near_ties": ties,
        "libm_overrides": r.stats["libm_overrides"],
        "candidates_per_point": float(r.stats["n_candidates"]) / n,
    }
    default_res = {"c2": 9, "c3": 10, "c4": 4, "c5": 9}[a.config]
    name = ("pmc_join_traffic" if a.config == "c2" else "pmc_join_traffic_%s" % a.config) + \
        ("" if a.res == default_res else "_r%d" % a.res) + ".json"
    prof = os.path.join(ROOT, "profiles", name)
    if os.path.exists(prof):
        try:
            p = json.load(open(prof))
            # (only a profile of the kernel this run's pipeline made dominant)
            same_kernel = p.get("kernel", "pip_join_kernel").split("<")[0] == kernel.split("<")[0]
            # (and only one measured on this build of the kernels, this table and these options:
            # a stale profile attaches nothing)
            if (p.get("res") == a.res and p.get("config", "c2") == a.config and p.get("points") and same_kernel
                    and p.get("key") == traffic_key(a.option, info)):
                # measured per launch on p["points"] points of this workload (rocprofv3 PMC
                # passes, tools/gpu.sh traffic); scaled to this launch's size if it differs
                out["roofline"]["traffic"] = p["hbm_bytes_per_launch"] * n / p["points"]
                out["roofline"]["traffic_source"] = "profiles/%s (%s%s)" % (
                    name, p.get("round", "?"), "" if p["points"] == n else ", measured on %d points, scaled" % p["points"])
        except (ValueError, KeyError):
            pass
    # VALU issue: the kernel's VALU wave-instructions per point (rocprofv3 SQ_INSTS_VALU of
    # the same workload, profiles/pmc_valu.json) over this run's kernel time: each wave64
    # VALU instruction occupies a SIMD-32 for 2 cycles (FP64 FMAs 4: a lower bound), 1024
    # SIMDs at 2.4 GHz.  When it exceeds the HBM fraction the kernel is issue-bound.
    vprof = os.path.join(ROOT, "profiles", "pmc_valu.json")
    if os.path.exists(vprof):
        try:
            v = json.load(open(vprof)).get("%s_r%d" % (a.config, a.res))
            if v and v["kernel"].split("<")[0] == kernel.split("<")[0] and v.get("key") == traffic_key(a.option, info):
                valu = v["valu_insts_per_point"] * n * 2.0 / (1024 * 2.4e9 * stream_ms * 1e-3)
                out["roofline"]["valu_issue_frac"] = valu
                out["roofline"]["salu_insts_per_point"] = v["salu_insts_per_point"]
                out["roofline"]["valu_source"] = "profiles/pmc_valu.json (%s)" % v["round"]
                if valu > out["roofline"]["frac"]:
                    out["roofline"]["bound"] = "valu"
        except (ValueError, KeyError):
            pass
    if rank == 0 and world == 1 and not a.no_pcie:
        out["pcie_inclusive"] = pcie_inclusive(x, y, chips, a.res, isys, begin, cap, M)
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        if table is None:
            table = M.tessellate(zones, isys, a.res, keep_core_geometries=wl.get("keep_core", True))
        log("timed; cpu baseline")
        out["cpu_baseline"] = cpu_baseline(table, isys, a.res, wl, a.seed, a.cpu_seconds)
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
