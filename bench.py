#!/usr/bin/env python3
"""Headline benchmark: ray-bounces/s on models/room.stl (BASELINE.json configs[1], "K2").

One step = one pass of the hot path over one synthetic isotropic burst of 1M rays per GPU, one
rt_trace_cir call (one launch on room.stl's brute-force mesh):
  trace kernel (trace_paths_kernel, kernel.py:38-98: ray generation, 3 bounces of closest hit vs
              receiver + environment, reflect, full reference output contract: traced_paths,
              received_paths, row_mask -- tracer.py:70-72), whose last block to finish does the
              compaction + CIR (tracer.py:87-117: received rows in ray order -> delay bins ->
              impulse response, zeroed and accumulated in ray order)
  RCCL all-reduce of the impulse response (N > 1: the job's CIR is the sum over ray shards).
Rays are sharded by global ray id (rank r traces ids [r*N, (r+1)*N)): per-GPU work is fixed as
GPUs are added ("weak").  Inputs (mesh tables) are resident in HBM before the timed region.

Side legs (each its own JSON object in the line): K1 (almost_empty.stl, 10k rays, 1 bounce: the
reference's CPU plumbing config), K3 coverage (room, 256^2 cells), K4 (terrain
stand-in, 5 bounces, ray shards) and K5 coverage (terrain, 1024^2 cells), each with the roofline of
its dominant kernel from HIP events recorded by the library (rt_coverage_profile / rt_profile), and
CPU baselines (the oracle, -O3 -march=native, built and timed on this host).

    python bench.py [--gpus N --steps K --warmup W] [--legs k1,k2,k3,k4,k5]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU, RCCL)

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
VALU_PEAK_GWI = 1024 * 2.4 / 2  # 256 CUs x 4 SIMDs, one wave64 VALU instruction per 2 cycles


def d4_bytes(B):
    """algorithmic bytes per ray-bounce = the reference kernel's per-ray buffer
    contract (traced + received rows of 12 (B+1) B, row_mask 4 B) over its B bounces."""
    return (24 * (B + 1) + 4) / B


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--settle-steps", type=int, default=250,
                    help="untimed steps before the warmup (~40 ms of K2): the GPU clock ramps up over the "
                         "first tens of ms of load (K2 trace kernel 148 -> 141 us); the same count on every rank")
    ap.add_argument("--profile-every", type=int, default=8,
                    help="K2: every k-th launch of the timed loop carries the start/stop events the kernel "
                         "time comes from (each such launch costs the stream a few us; 1 = all)")
    ap.add_argument("--legs", default="k1,k2,k3,k4,k5", help="comma list of k1, k2 (always run), k3, k4, k5")
    ap.add_argument("--rays", type=int, default=1_000_000, help="rays per GPU per step (K2: 1M)")
    ap.add_argument("--bounces", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-runs", type=int, default=5, help="timed CPU-baseline runs (median), after 1 warm-up")
    ap.add_argument("--cpu-rays", type=int, default=8_000_000, help="rays per CPU-baseline run (all threads)")
    ap.add_argument("--cpu-cells", type=int, default=8,
                    help="K3 / K5 cells per coverage CPU-baseline run (SURVEY 8(d) D5: median of 5 after a warm-up)")
    ap.add_argument("--cpu-cells-1thread", type=int, default=1,
                    help="K3 / K5 cells per run of the one-thread coverage leg (the first of the seeded cells)")
    ap.add_argument("--no-coverage", action="store_true", help="skip K3 (same as leaving it out of --legs)")
    ap.add_argument("--coverage-grid", type=int, default=256, help="K3: n x n receiver cells at z=5 on room.stl")
    ap.add_argument("--coverage-rays", type=int, default=1_000_000)
    ap.add_argument("--coverage-runs", type=int, default=3)
    ap.add_argument("--coverage-shard", choices=("sectors", "rays", "cells"), default="sectors",
                    help="N>1 coverage decomposition: ray shards by initial azimuth (four interleaved wedges per "
                         "GPU) or by ray-id range, each with a record all-to-all, or x-column cell shards")
    ap.add_argument("--no-validate", action="store_true",
                    help="N>1: skip rank 0's one-GPU reference map (the N-rank map is compared with it bit for bit)")
    ap.add_argument("--debug-unordered-rows", action="store_true",
                    help="test hook: ray-sharded coverage (also at N=1), with two received rows of each owner's first "
                         "segment swapped -- the owner stage must flag it and the bench exit non-zero")
    ap.add_argument("--no-k4", action="store_true", help="skip the terrain (apollo stand-in) legs K4/K5")
    ap.add_argument("--k4-rays", type=int, default=2_097_152, help="rays per GPU (K4: 16.7M over 8 GPUs)")
    ap.add_argument("--k5-grid", type=int, default=1024)
    ap.add_argument("--k5-rays", type=int, default=1_000_000)
    ap.add_argument("--k5-runs", type=int, default=2)
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic_k2.json"),
                    help="per-launch HBM bytes measured by rocprofv3 PMC (profiles/)")
    a = ap.parse_args()
    legs = set(x.strip() for x in a.legs.split(",") if x.strip()) | {"k2"}
    if a.no_coverage:
        legs.discard("k3")
    if a.no_k4:
        legs -= {"k4", "k5"}
    a.legs = legs
    return a


# ------------------------------------------------------------------ CPU baselines (rank 0, N=1)
def host_info():
    model = ""
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                model = line.split(":", 1)[1].strip()
    except (OSError, subprocess.SubprocessError):
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    # the box gives one GPU's job a share of the host (OMP_NUM_THREADS, 16 there); use all of it
    share = int(os.environ.get("OMP_NUM_THREADS") or aff or 1)
    quota = None  # the cgroup's CPU bandwidth limit in CPUs (cpu.max "quota period"), if any
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
            quota = None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    return {"lscpu_model": model, "os_cpu_count": os.cpu_count(), "affinity_cpus": aff, "threads_used": share,
            "cgroup_cpu_quota": quota}


def native_oracle():
    """Build the oracle -O3 -march=native on this host (the prebuilt one is -march=x86-64-v3)."""
    from oracle import oracle as orc
    path = os.path.join(tempfile.mkdtemp(prefix="rfrt_oracle_"), "librt_oracle_native.so")
    try:
        orc.build_native(path)
        orc.load(path)
        return "gcc -O3 -march=native -ffp-contract=off -fopenmp (built on this host)"
    except (OSError, subprocess.CalledProcessError):
        orc.load(os.path.join(REPO, "oracle", "_build", "librt_oracle.so"))
        return "gcc -O3 -march=x86-64-v3 -ffp-contract=off -fopenmp (prebuilt; native build failed)"


_CPU = {}


def cpu_setup():
    """(host info, oracle build description), built once per process (rank 0, N=1 only)."""
    if not _CPU:
        _CPU["info"] = host_info()
        _CPU["build"] = native_oracle()
    return _CPU["info"], _CPU["build"]


def _median_runs(fn, runs):
    fn()  # warm-up
    ts = []
    for _ in range(runs):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), ts


def cpu_baseline_k2(args, B, tx, rx, info, build):
    """The oracle (C restatement of kernel.py + tracer.py host tail) on the host cores: one run =
    trace of `rays` rays of the K2 burst + clean + CIR (tracer.py:84-117), median of cpu_runs."""
    from oracle import oracle as orc
    from rf_ray_tracing_warp_amd.mesh import load_stl, sphere

    env = load_stl(os.path.join(REPO, "models", "room.stl"))
    rxm = sphere(rx, 0.1, 1)
    E, R = orc.Mesh(env.vertices, env.faces), orc.Mesh(rxm.vertices, rxm.faces)
    out = {}
    for label, threads, rays in (("all", info["threads_used"], args.cpu_rays),
                                 ("1thread", 1, max(args.cpu_rays // 16, 50_000)),
                                 ("all_cores", info["affinity_cpus"], args.cpu_rays)):
        def run():
            o = orc.trace(E, R, tx, B, 0, rays, want_traced=True, nthreads=threads)
            orc.cir_from_paths(orc.clean_paths(o["received"], o["mask"]), 1, rays, 2.998e8, 100e9, 100e-9)
        med, ts = _median_runs(run, args.cpu_runs)
        out[label] = {"value": rays * B / med, "unit": "ray-bounces/s", "cores": threads, "kind": "port",
                      "sample": f"ray ids 0..{rays - 1} of the K2 room.stl burst ({rays} rays x {B} bounces): "
                                f"trace (traced + received + row_mask) + host CIR, oracle/rt_oracle.c, "
                                f"median of {args.cpu_runs} runs after 1 warm-up ({', '.join(f'{t:.2f}' for t in ts)} s)",
                      "build": build, "host": info}
    return out


def cpu_baseline_k3(args, info):
    """coverage.py:38-57 literally on the host for a seeded sample of K3 cells (full 1M-ray trace
    with the cell's icosphere, the per-path host CIR of tracer.py:84-117, np.convolve power):
    cells/s over the sample, median of cpu_runs, on all threads and (the first cpu_cells_1thread
    cells) on one thread.  Also the reference's np.convolve step alone."""
    from oracle import oracle as orc
    from rf_ray_tracing_warp_amd.coverage import CoverageGrid
    from rf_ray_tracing_warp_amd.mesh import load_stl, sphere

    env = load_stl(os.path.join(REPO, "models", "room.stl"))
    E = orc.Mesh(env.vertices, env.faces)
    grid = CoverageGrid.square(args.coverage_grid, 15.0, 5.0)
    cells = np.random.default_rng(2).choice(grid.num_cells, args.cpu_cells, replace=False)
    cen = grid.centers().reshape(-1, 3)[cells]
    N, B, tx = args.coverage_rays, args.bounces, (10.0, 0.0, 5.0)

    def leg(sel, threads):
        def run():
            for c in cen[:sel]:
                rxm = sphere(c, 0.1, 1)
                o = orc.trace(E, orc.Mesh(rxm.vertices, rxm.faces), tx, B, 0, N, want_traced=False, nthreads=threads)
                ir = orc.cir_from_paths(orc.clean_paths(o["received"], o["mask"]), 1, N, 2.998e8, 100e9, 100e-9)
                orc.signal_power(ir, 100e-9)
        med, ts = _median_runs(run, args.cpu_runs)
        return {"value": sel / med, "unit": "cells/s", "cores": threads, "kind": "port",
                "sample": f"{sel} seeded K3 cells ({', '.join(str(int(c)) for c in cells[:sel])}), each the reference "
                          f"loop body: {N}-ray trace with its icosphere + host CIR + np.convolve power; median of "
                          f"{len(ts)} runs after 1 warm-up ({', '.join(f'{t:.2f}' for t in ts)} s)", "host": info}
    ir = np.zeros(10000)
    ir[[3000, 5000, 7000]] = 1e-6
    conv, _ = _median_runs(lambda: orc.signal_power(ir, 100e-9), 5)
    out = {"all": leg(len(cells), info["threads_used"]), "1thread": leg(args.cpu_cells_1thread, 1),
           "all_cores": leg(len(cells), info["affinity_cpus"])}
    out["all"]["np_convolve_power_ms_per_cell"] = conv * 1e3
    return out


def cpu_baseline_k1(args, info, build):
    """K1 (BASELINE.json configs[0], the reference's CPU-only plumbing case): almost_empty.stl,
    tx (1,0,1), rx (41,0,1) r=0.1 (main.py:25-27), 10k rays, 1 bounce, 20000 bins (main.py:15-17):
    trace + host CIR per burst.  A burst is ~1 ms of CPU work, so one timed run repeats it."""
    from oracle import oracle as orc
    from rf_ray_tracing_warp_amd.mesh import load_stl, sphere

    env = load_stl(os.path.join(REPO, "models", "almost_empty.stl"))
    rxm = sphere((41.0, 0.0, 1.0), 0.1, 1)
    E, R = orc.Mesh(env.vertices, env.faces), orc.Mesh(rxm.vertices, rxm.faces)
    n, B, reps = 10_000, 1, 50
    out = {}
    for label, threads in (("all", info["threads_used"]), ("1thread", 1), ("all_cores", info["affinity_cpus"])):
        def run():
            for _ in range(reps):
                o = orc.trace(E, R, (1.0, 0.0, 1.0), B, 0, n, want_traced=True, nthreads=threads)
                orc.cir_from_paths(orc.clean_paths(o["received"], o["mask"]), 1, n, 2.998e8, 100e9, 200e-9)
        med, ts = _median_runs(run, args.cpu_runs)
        out[label] = {"value": reps * n * B / med, "unit": "ray-bounces/s", "cores": threads, "kind": "port",
                      "sample": f"{reps} K1 bursts (ray ids 0..{n - 1}, {B} bounce, almost_empty.stl): trace "
                                f"(traced + received + row_mask) + host CIR each, oracle/rt_oracle.c, median of "
                                f"{args.cpu_runs} runs after 1 warm-up ({', '.join(f'{t:.3f}' for t in ts)} s)",
                      "build": build, "host": info}
    return out


def cpu_baseline_k4(args, terr, info, build):
    """K4 on the host: the oracle's BVH path (its own median-split tree over the 2.09M-face terrain)
    for a contiguous sample of the burst's ray ids, trace + host CIR; extrapolated as ray-bounces/s."""
    from oracle import oracle as orc
    from rf_ray_tracing_warp_amd.mesh import sphere

    t0 = time.perf_counter()
    E = orc.Mesh(terr.vertices, terr.faces)
    t_tree = time.perf_counter() - t0
    rxm = sphere((-10.125, 0.0, 4.8), 0.1, 1)
    R = orc.Mesh(rxm.vertices, rxm.faces)
    B = 5
    out = {}
    for label, threads, rays in (("all", info["threads_used"], 1_000_000), ("1thread", 1, 50_000),
                                 ("all_cores", info["affinity_cpus"], 1_000_000)):
        def run():
            o = orc.trace(E, R, (10.0, 0.0, 4.5), B, 0, rays, want_traced=True, nthreads=threads)
            orc.cir_from_paths(orc.clean_paths(o["received"], o["mask"]), 1, rays, 2.998e8, 100e9, 200e-9)
        med, ts = _median_runs(run, args.cpu_runs)
        out[label] = {"value": rays * B / med, "unit": "ray-bounces/s", "cores": threads, "kind": "port",
                      "sample": f"ray ids 0..{rays - 1} of the K4 burst ({rays} of 16,777,216 rays x {B} bounces) "
                                f"on the terrain stand-in: trace (traced + received + row_mask) + host CIR, "
                                f"oracle/rt_oracle.c BVH path (tree built once, {t_tree:.2f} s, not timed), median "
                                f"of {args.cpu_runs} runs after 1 warm-up ({', '.join(f'{t:.2f}' for t in ts)} s)",
                      "build": build, "host": info}
    return out


def cpu_baseline_k5(args, terr, info):
    """coverage.py:38-57 literally on the host for seeded K5 cells of the terrain map: per cell a
    1M-ray trace with its icosphere (oracle BVH path), host CIR, np.convolve power; all threads and
    (the first cpu_cells_1thread cells) one thread."""
    from oracle import oracle as orc
    from rf_ray_tracing_warp_amd.coverage import CoverageGrid
    from rf_ray_tracing_warp_amd.mesh import sphere

    E = orc.Mesh(terr.vertices, terr.faces)
    grid = CoverageGrid.square(args.k5_grid, 50.0, 2.0)
    ids = np.random.default_rng(5).choice(grid.num_cells, args.cpu_cells, replace=False)
    cen = grid.centers().reshape(-1, 3)[ids]
    N, B, tx = args.k5_rays, 3, (10.0, 0.0, 4.5)

    def leg(sel, threads):
        def run():
            for c in cen[:sel]:
                rxm = sphere(c, 0.1, 1)
                o = orc.trace(E, orc.Mesh(rxm.vertices, rxm.faces), tx, B, 0, N, want_traced=False, nthreads=threads)
                ir = orc.cir_from_paths(orc.clean_paths(o["received"], o["mask"]), 1, N, 2.998e8, 100e9, 200e-9)
                orc.signal_power(ir, 200e-9)
        med, ts = _median_runs(run, args.cpu_runs)
        return {"value": sel / med, "unit": "cells/s", "cores": threads, "kind": "port",
                "sample": f"{sel} seeded K5 cells ({', '.join(str(int(c)) for c in ids[:sel])}), each the reference "
                          f"loop body: {N}-ray trace over the terrain stand-in with its icosphere (oracle BVH path) + "
                          f"host CIR + np.convolve power; median of {len(ts)} runs after 1 warm-up "
                          f"({', '.join(f'{t:.2f}' for t in ts)} s)", "host": info}
    return {"all": leg(len(ids), info["threads_used"]), "1thread": leg(args.cpu_cells_1thread, 1),
            "all_cores": leg(len(ids), info["affinity_cpus"])}


# ------------------------------------------------------------------ coverage legs
def shard_desc(mode, world):
    if world == 1:
        return "1 GPU"
    if mode in ("rays", "sectors"):
        how = "four interleaved wedges of initial azimuth" if mode == "sectors" else "a ray-id range"
        return (f"rays sharded x{world} (1/{world} of every cell's rays per GPU: {how}), (cell, bin, amplitude) "
                f"records to the cells' owners (ix % {world}) by one RCCL all-to-all, RCCL gather of the power map")
    return f"cells sharded by x column (ix % {world}), every GPU traces all rays, RCCL sum of the power map"


def _leg_traffic(kernel):
    """HBM bytes per launch of `kernel` at the bench's default leg sizes, from the last PMC passes
    (profiles/traffic_legs.json, tools/summarize_r2.py): a property of the code and the input."""
    try:
        with open(os.path.join(REPO, "profiles", "traffic_legs.json")) as fh:
            t = json.load(fh).get(kernel)
        return (t["hbm_bytes_per_launch"], t.get("l2_hit_rate"), t.get("source")) if t else (None, None, None)
    except (OSError, ValueError, KeyError):
        return None, None, None


def _roofline(kernel, ms, work, B, note, default_size=True):
    if not (ms and ms > 0 and work):
        return None
    bpb = d4_bytes(B)
    ach = work * bpb / (ms * 1e-3) / 1e9
    traffic, l2, src = _leg_traffic(kernel) if default_size else (None, None, None)
    return {"bound": "hbm", "kernel": kernel, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": ach / HBM_PEAK_GBS, "traffic": traffic, "l2_hit_rate": l2, "traffic_source": src,
            "kernel_ms": ms, "ray_bounces": int(work), "bytes_per_ray_bounce": bpb,
            "ray_bounces_per_s": work / (ms * 1e-3), "note": note}


def _swap_first_rows(cov):
    """--debug-unordered-rows: break the owner stage's precondition (each received segment strictly
    ascending by key) by swapping two rows of the first segment that has two."""
    orig = cov.power_from_rows

    def broken(rows, counts=None):
        if counts is not None:
            off = 0
            for c in counts:
                if c >= 2:
                    rows = rows.clone()
                    rows[[off, off + 1]] = rows[[off + 1, off]]
                    break
                off += c
        return orig(rows, counts)
    cov.power_from_rows = broken


def coverage_mode(args, world):
    if args.debug_unordered_rows:
        return "rays"
    return args.coverage_shard if world > 1 else "cells"


def run_coverage(cov, tx, runs, world, dist, local):
    """Time `runs` maps (profiling off), then one profiled map for the stage breakdown.  After the
    timed maps (outside the timed region) the plan's device-side error report is checked
    (Coverage.check: a look-back wait that gave up or an owner-stage segment out of key order means
    that map is wrong): RfrtError, and the bench exits non-zero."""
    import torch

    from rf_ray_tracing_warp_amd.dist import gather_power_map

    def one():
        p = cov.run_device(tx, 1)
        if world > 1:  # the sum-reduce of the owners' disjoint x columns, as an all-gather
            p = gather_power_map(p, cov.grid.nx)
        return p

    one()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(runs):
        p = one()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = (time.perf_counter() - t0) / runs
    cov.check()  # raises on a device-flagged error of the timed maps (outside the timed region)
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t[0])
    pm = p.cpu().numpy()
    cov.profile(True)
    one()
    prof = cov.last_profile()
    cov.profile(False)
    cov.check()
    return dt, pm, prof


def one_gpu_reference(make_plan, tx, pm, rank, world):
    """N>1 validation (outside the timed region): rank 0 computes the same map with a one-GPU plan
    and compares it with the gathered N-rank map bit for bit (the per-bin sums are exact fixed point,
    so the decomposition must not move a single bit).  Returns (equal, sha256 of the N-rank map,
    sha256 of the one-GPU map) on rank 0, None elsewhere or at N=1."""
    import hashlib
    if world == 1 or rank != 0:
        return None
    ref = make_plan()
    r = ref.run_device(tx, 1).cpu().numpy()
    ref.check()
    ref.close()
    a, b = hashlib.sha256(pm.tobytes()).hexdigest(), hashlib.sha256(r.tobytes()).hexdigest()
    return a == b, a, b


def coverage_block(name, cov, grid, dt, pm, prof, B, val, workload, world, mode, bvh, default_size):
    t = "true" if bvh else "false"
    traj = _roofline(f"k_traj<{t}>", prof["traj_ms"], prof["traced_ray_bounces"], B,
                     "trajectory pass, D4 bytes over the actually traced ray-bounces (rays x segments)",
                     default_size and world == 1)
    if traj:
        traj["active_ray_bounces"] = int(prof["traced_ray_bounces"])
        traj["nominal_ray_bounces"] = int(cov.ray_count) * B
    rep = _roofline(f"k_replay<{t}>", prof["replay_ms"], prof["replayed_ray_bounces"], B,
                    "first-win replay, D4 bytes over its ray-bounces (sum of B - k0 over first-win records)",
                    default_size and world == 1)
    return {"metric": "coverage cells/sec", "value": grid.num_cells / dt, "unit": "cells/s", "ms_per_map": dt * 1e3,
            "workload": workload + f"; {shard_desc(mode, world)}", "scaling": "strong",
            "cells_receiving": int(np.isfinite(pm).sum()), "candidates": int(prof["candidates"]),
            "first_win_records": int(prof["records"]),
            "stage_ms": {k: prof[k] for k in ("traj_ms", "candidates_ms", "win_ms", "replay_ms", "reduce_power_ms",
                                                "total_ms")},
            "roofline": traj, "roofline_replay": rep,
            # N>1: the gathered map against rank 0's one-GPU map, bit for bit (null at N=1)
            "map_equals_one_gpu": None if val is None else bool(val[0]),
            "map_sha256": None if val is None else val[1],
            "algorithm": "exact shared-trajectory (csrc/coverage.hip)", "name": name}


def coverage_leg(args, env_m, env, local, rank, world, dist):
    """K3: coverage.py on room.stl, n x n cells at z = 5, tx (10,0,5), 1M rays per cell, 3 bounces."""
    from rf_ray_tracing_warp_amd.coverage import Coverage, CoverageGrid

    grid = CoverageGrid.square(args.coverage_grid, 15.0, 5.0)
    mode = coverage_mode(args, world)
    cov = Coverage(env_m, 2.998e8, 100e9, 100e-9, args.bounces, args.coverage_rays, grid, 0.1, device=local,
                   shard_index=rank, shard_count=world, env_mesh=env, shard_mode=mode)
    if args.debug_unordered_rows:
        _swap_first_rows(cov)
    dt, pm, prof = run_coverage(cov, (10.0, 0.0, 5.0), args.coverage_runs, world, dist, local)
    cov.close()
    val = None if args.no_validate else one_gpu_reference(
        lambda: Coverage(env_m, 2.998e8, 100e9, 100e-9, args.bounces, args.coverage_rays, grid, 0.1, device=local,
                         env_mesh=env), (10.0, 0.0, 5.0), pm, rank, world)
    return coverage_block("K3", cov, grid, dt, pm, prof, args.bounces, val,
                          f"K3: room.stl, {grid.nx}x{grid.ny} receivers at z=5 (centres -15+(i+1/2)*30/{grid.nx}), "
                          f"tx (10,0,5), {args.coverage_rays} rays per cell, {args.bounces} bounces, 10000 bins, "
                          f"signal power per cell", world, mode, False,
                          args.coverage_grid == 256 and args.coverage_rays == 1_000_000 and args.bounces == 3)


def k1_leg(args, local, rank, world, dist):
    """K1 (BASELINE.json configs[0]): almost_empty.stl, tx (1,0,1), rx (41,0,1) r=0.1 (main.py:25-27),
    10k rays, 1 bounce, 20000 bins -- the reference's CPU-only plumbing case, run here as one
    rt_trace_cir per step on the GPU (launch-latency bound: a 10k-ray burst is 40 waves)."""
    import torch
    from rf_ray_tracing_warp_amd._lib import DeviceMesh, check, lib, ptr
    from rf_ray_tracing_warp_amd.mesh import load_stl, sphere
    from rf_ray_tracing_warp_amd.tracer import cir_flags

    dev = f"cuda:{local}"
    N, B, nb = 10_000, 1, 20_000
    m = load_stl(os.path.join(REPO, "models", "almost_empty.stl"))
    env = DeviceMesh(m.vertices, m.faces, local)
    rxm = sphere((41.0, 0.0, 1.0), 0.1, 1)
    rx = DeviceMesh(rxm.vertices, rxm.faces, local)
    tx = np.asarray((1.0, 0.0, 1.0), np.float32)
    traced = torch.empty((N, B + 1, 3), dtype=torch.float32, device=dev)
    received = torch.empty_like(traced)
    mask = torch.empty(N, dtype=torch.int32, device=dev)
    index = torch.empty(N, dtype=torch.int64, device=dev)
    count = torch.empty(1, dtype=torch.int64, device=dev)
    ir = torch.empty(nb, dtype=torch.float64, device=dev)
    L = lib()
    ws = torch.zeros(int(L.rt_trace_cir_workspace_bytes(N)), dtype=torch.uint8, device=dev)
    sh = torch.cuda.current_stream().cuda_stream
    flags = cir_flags(2.998e8, 100e9)

    def step():
        check(L.rt_trace_cir(env.handle, tx.ctypes.data, rx.handle, B, rank * N, N, ptr(traced), ptr(received),
                             ptr(mask), 1.0 / (N * world), 2.998e8, 100e9, flags, nb, ptr(ir), ptr(index), ptr(count),
                             ptr(ws), ws.numel(), sh), "rt_trace_cir")

    for _ in range(50):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    steps = 500
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt[0])
    rows = int(count.item())
    env.close()
    rx.close()
    return {"metric": "ray-bounces/sec", "value": world * N * B / dt, "unit": "ray-bounces/s", "ms_per_step": dt * 1e3,
            "workload": f"K1 (BASELINE configs[0]): almost_empty.stl, tx (1,0,1), rx (41,0,1) r=0.1, {N} rays/GPU x "
                        f"{world}, {B} bounce, {nb} bins, rt_trace_cir per step ({steps} steps)",
            "scaling": "weak", "received_rows_last_step": rows}


def terrain_legs(args, local, rank, world, dist):
    """K4/K5 on the declared apollo stand-in (mesh.synthetic_terrain: 1024^2 vertices, 2.09M faces, BVH):
    K4 = TX (10,0,4.5), RX (-10.125,0,4.8) r=0.1 (main.py:22-23), 5 bounces, 16.7M rays / 8 GPUs
    sharded by ray id; K5 = coverage of k5_grid^2 cells 1 m above the terrain's mean level."""
    import torch
    from rf_ray_tracing_warp_amd._lib import DeviceMesh, check, lib, ptr
    from rf_ray_tracing_warp_amd.coverage import Coverage, CoverageGrid
    from rf_ray_tracing_warp_amd.mesh import sphere, synthetic_terrain

    dev = f"cuda:{local}"
    t_build = time.perf_counter()
    terr = synthetic_terrain(1024, 50.0)
    env = DeviceMesh(terr.vertices, terr.faces, local)
    t_build = time.perf_counter() - t_build
    k4 = k5 = None
    L = lib()
    if "k4" in args.legs:
        B, N = 5, args.k4_rays
        P = B + 1
        rxm = sphere((-10.125, 0.0, 4.8), 0.1, 1)
        rx = DeviceMesh(rxm.vertices, rxm.faces, local)
        tx = np.asarray((10.0, 0.0, 4.5), np.float32)
        traced = torch.empty((N, P, 3), dtype=torch.float32, device=dev)
        received = torch.empty((N, P, 3), dtype=torch.float32, device=dev)
        mask = torch.empty(N, dtype=torch.int32, device=dev)
        sh = torch.cuda.current_stream().cuda_stream

        def step(kind=None):
            check(L.rt_trace(env.handle, tx.ctypes.data, rx.handle, B, rank * N, N, ptr(traced), ptr(received),
                             ptr(mask), ptr(kind), None, sh), "rt_trace")

        step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = (time.perf_counter() - t0) / reps
        if world > 1:
            tt = torch.tensor([dt], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            dt = float(tt[0])
        # one profiled launch (kernel and ray-order sort on HIP events), then the active ray-bounces
        L.rt_profile(1)
        step()
        pr = np.zeros(2, np.float64)
        check(L.rt_trace_last_profile(pr.ctypes.data, 2), "rt_trace_last_profile")
        L.rt_profile(0)
        kind = torch.empty((N, B), dtype=torch.int32, device=dev)
        step(kind)
        # iterations that issued a query: every env / RX hit plus each ray's first miss
        active = int((kind != 0).sum().item()) + int((kind == 0).any(dim=1).sum().item())
        roof = _roofline("k_trace_bvh<5>", float(pr[0]), N * B, B, "nominal N x B ray-bounces (D4); kernel_ms spans "
                         "the coalesced NaN / 0 fill of received and row_mask (k_fill_received) and the trace kernel, "
                         "which stores only the received rows (the ray-order sort is sort_ms); traffic: both launches, "
                         "BVH node/leaf gathers (16-B lanes, FETCH_SIZE x2 not calibrated for gathers: the true bytes "
                         "lie between traffic/2 and traffic)",
                         N == 2_097_152 and world == 1)
        if roof:
            roof["sort_ms"] = float(pr[1])
            roof["active_ray_bounces"] = active
        k4 = {"metric": "ray-bounces/sec", "value": world * N * B / dt, "unit": "ray-bounces/s",
              "ms_per_step": dt * 1e3,
              "workload": f"K4 on the declared apollo stand-in (synthetic terrain 1024^2 vertices, {len(terr.faces)} "
                          f"faces, BVH), {N} rays/GPU x {world}, {B} bounces, traced+received+row_mask",
              "scaling": "weak", "mesh_build_s": t_build, "roofline": roof}
        del traced, received, mask, kind
        rx.close()
    if "k5" in args.legs:
        grid = CoverageGrid.square(args.k5_grid, 50.0, 2.0)
        mode = coverage_mode(args, world)
        cov = Coverage(terr, 2.998e8, 100e9, 200e-9, 3, args.k5_rays, grid, 0.1, device=local, shard_index=rank,
                       shard_count=world, env_mesh=env, shard_mode=mode)
        if args.debug_unordered_rows:
            _swap_first_rows(cov)
        dt, pm, prof = run_coverage(cov, (10.0, 0.0, 4.5), args.k5_runs, world, dist, local)
        cov.close()
        val = None if args.no_validate else one_gpu_reference(
            lambda: Coverage(terr, 2.998e8, 100e9, 200e-9, 3, args.k5_rays, grid, 0.1, device=local, env_mesh=env),
            (10.0, 0.0, 4.5), pm, rank, world)
        k5 = coverage_block("K5", cov, grid, dt, pm, prof, 3, val,
                            f"K5 on the terrain stand-in: {grid.nx}x{grid.ny} receivers at z=2 over +-50 m, "
                            f"tx (10,0,4.5), {args.k5_rays} rays per cell, 3 bounces, 20000 bins", world, mode,
                            True, args.k5_grid == 1024 and args.k5_rays == 1_000_000)
    env.close()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        info, build = cpu_setup()
        if k4 is not None:
            cb = cpu_baseline_k4(args, terr, info, build)
            k4["cpu_baseline"], k4["cpu_baseline_1thread"] = cb["all"], cb["1thread"]
            k4["cpu_baseline_all_cores"] = cb["all_cores"]
        if k5 is not None:
            cb = cpu_baseline_k5(args, terr, info)
            k5["cpu_baseline"], k5["cpu_baseline_1thread"] = cb["all"], cb["1thread"]
            k5["cpu_baseline_all_cores"] = cb["all_cores"]
    return k4, k5


def summary(out):
    """Every leg's headline figures in one compact block (printed last in the line)."""
    def r(x, nd=4):
        return None if x is None else float(f"{x:.{nd}g}")

    def roof(leg):
        rf = (leg or {}).get("roofline") or {}
        return r(rf.get("frac"), 3), r(rf.get("kernel_ms"), 4)

    s = {"k2": {"value": r(out["value"]), "ms_per_step": r(out["ms_per_step"]),
                "roofline_frac": r(out["roofline"]["frac"], 3), "kernel_ms": r(out["roofline"]["kernel_ms"]),
                "cpu": r((out.get("cpu_baseline") or {}).get("value")),
                "cpu_1t": r((out.get("cpu_baseline_1thread") or {}).get("value"))}}
    for key, name in (("k1_plumbing", "k1"), ("k4_terrain", "k4")):
        leg = out.get(key)
        if leg:
            f, k = roof(leg)
            s[name] = {"value": r(leg["value"]), "ms_per_step": r(leg["ms_per_step"]), "roofline_frac": f,
                       "kernel_ms": k, "cpu": r((leg.get("cpu_baseline") or {}).get("value")),
                       "cpu_1t": r((leg.get("cpu_baseline_1thread") or {}).get("value"))}
    for key, name in (("coverage", "k3"), ("k5_terrain_coverage", "k5")):
        leg = out.get(key)
        if leg:
            f, k = roof(leg)
            s[name] = {"value": r(leg["value"]), "ms_per_map": r(leg["ms_per_map"]), "roofline_frac": f,
                       "traj_ms": k, "replay_ms": r((leg.get("stage_ms") or {}).get("replay_ms")),
                       "map_equals_one_gpu": leg.get("map_equals_one_gpu"),
                       "cpu": r((leg.get("cpu_baseline") or {}).get("value")),
                       "cpu_1t": r((leg.get("cpu_baseline_1thread") or {}).get("value"))}
    return s


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N>1 path on a one-GPU box: every rank on cuda:0, gloo instead of RCCL
    # (RFRT_BENCH_ONE_GPU=1; never used for reported numbers)
    one_gpu = os.environ.get("RFRT_BENCH_ONE_GPU") == "1"
    if one_gpu:
        local = 0
    torch.cuda.set_device(local)
    dev = f"cuda:{local}"
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if one_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device(dev))

    from rf_ray_tracing_warp_amd._lib import DeviceMesh, check, lib, ptr
    from rf_ray_tracing_warp_amd.mesh import load_stl, sphere
    from rf_ray_tracing_warp_amd.tracer import cir_flags

    N, B = args.rays, args.bounces
    P = B + 1
    tx, rx, r_rx = (10.0, 0.0, 5.0), (-10.0, 0.0, 5.0), 0.1  # main.py:29-31 (room scene)
    c, fs, win, tx_power = 2.998e8, 100e9, 100e-9, 1
    n_bins = int(win * fs)
    env_m = load_stl(os.path.join(REPO, "models", "room.stl"))
    env = DeviceMesh(env_m.vertices, env_m.faces, local)
    rxm = sphere(rx, r_rx, 1)
    rxd = DeviceMesh(rxm.vertices, rxm.faces, local)
    tx32 = np.asarray(tx, np.float32)

    traced = torch.empty((N, P, 3), dtype=torch.float32, device=dev)
    received = torch.empty((N, P, 3), dtype=torch.float32, device=dev)
    mask = torch.empty(N, dtype=torch.int32, device=dev)
    index = torch.empty(N, dtype=torch.int64, device=dev)
    count = torch.empty(1, dtype=torch.int64, device=dev)
    # rt_trace_cir's workspace: zero-filled once, left ready by every call
    ws = torch.zeros(int(lib().rt_trace_cir_workspace_bytes(N)), dtype=torch.uint8, device=dev)
    # two impulse-response buffers: step i's RCCL all-reduce (on RCCL's own stream) overlaps step
    # i+1's trace; a buffer is reused only once the all-reduce issued on it two steps earlier is done
    irs = [torch.zeros(n_bins, dtype=torch.float64, device=dev) for _ in range(2)]
    pending = [None, None]
    amp0 = tx_power / (N * world)
    ray_offset = rank * N
    flags = cir_flags(c, fs)
    L = lib()
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream

    def drain():
        for j in range(2):
            if pending[j] is not None:
                pending[j].wait()  # the current stream waits for that all-reduce
                pending[j] = None

    def step(i):
        # the whole hot path of one burst: trace (traced + received + row_mask, kernel.py:38-98),
        # then one fused launch for the ordered compaction and the impulse response (overwritten;
        # tracer.py:87-117) -- rt_trace_cir
        ir = irs[i % 2]
        if pending[i % 2] is not None:
            pending[i % 2].wait()
            pending[i % 2] = None
        check(L.rt_trace_cir(env.handle, tx32.ctypes.data, rxd.handle, B, ray_offset, N, ptr(traced), ptr(received),
                             ptr(mask), amp0, c, fs, flags, n_bins, ptr(ir), ptr(index), ptr(count), ptr(ws),
                             ws.numel(), sh), "rt_trace_cir")
        if world > 1:
            pending[i % 2] = dist.all_reduce(ir, async_op=True)

    settle = max(0, args.settle_steps)
    for i in range(settle):
        step(i)
        if i % 32 == 31:
            drain()
            torch.cuda.synchronize()
    for i in range(args.warmup):
        step(i)
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # trace-kernel time from the events its own dispatch packets carry (no marker packets in the
    # timed stream; rt_trace_profile_stats after the loop)
    L.rt_profile(args.profile_every)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    L.rt_profile(0)
    pst = np.zeros(4, np.float64)
    check(L.rt_trace_profile_stats(pst.ctypes.data, 4), "rt_trace_profile_stats")
    kern_ms = float(pst[1])
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
    received_rows = int(count.item())
    # active ray-bounces: the bounce iterations that issue a query -- every env / RX
    # hit plus each ray's first miss (later iterations of a missed ray repeat it, kernel.py:57-98)
    kind = torch.empty((N, B), dtype=torch.int32, device=dev)
    check(L.rt_trace(env.handle, tx32.ctypes.data, rxd.handle, B, ray_offset, N, ptr(traced), ptr(received), ptr(mask),
                     ptr(kind), None, sh), "rt_trace")
    active = int((kind != 0).sum().item()) + int((kind == 0).any(dim=1).sum().item())
    del traced, received, kind

    k1_out = k1_leg(args, local, rank, world, dist) if "k1" in args.legs else None
    cov_out = coverage_leg(args, env_m, env, local, rank, world, dist) if "k3" in args.legs else None
    k4_out = k5_out = None
    if args.legs & {"k4", "k5"}:
        k4_out, k5_out = terrain_legs(args, local, rank, world, dist)

    if rank == 0:
        bounces = world * N * B * args.steps
        value = bounces / elapsed
        bytes_per_launch = N * (24 * P + 4)  # traced + received rows + row_mask
        achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
        traffic = traffic_parts = None
        try:
            with open(args.traffic_json) as fh:
                tj = json.load(fh)
            if tj.get("rays") == N and tj.get("bounces") == B:
                # both launches of the step's timed span: the coalesced NaN / 0 fill of received and
                # row_mask (k_fill_received) and the trace kernel
                traffic = tj.get("hbm_bytes_per_launch")
                traffic_parts = {"k_fill_received": tj.get("fill_bytes_per_launch"),
                                 f"k_trace_bf<{B}>": tj.get("trace_kernel_bytes_per_launch"), "source": tj.get("tag")}
        except (OSError, ValueError):
            pass
        # the binding resource of the brute-force LDS kernel is the VALU issue rate: VALU
        # instructions per launch come from a PMC pass (profiles/, a property of the code and the
        # input), the time from the live HIP events above
        valu = None
        try:
            with open(os.path.join(REPO, "profiles", "k2_sq_counters.json")) as fh:
                sq = json.load(fh)
            if N == 1_000_000 and B == 3:
                rate = sq["SQ_INSTS_VALU"] / (kern_ms * 1e-3) / 1e9  # wave-instructions / ns
                valu = {"bound": "valu", "achieved": rate, "peak": VALU_PEAK_GWI, "unit": "G wave-instr/s",
                        "frac": rate / VALU_PEAK_GWI, "valu_instr_per_launch": sq["SQ_INSTS_VALU"],
                        "source": sq.get("source"),
                        "note": "peak = 1024 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU instruction"}
        except (OSError, ValueError, KeyError):
            pass
        gpus = f"{world} GPU" + ("s" if world > 1 else "")
        out = {
            "metric": f"ray-bounces/sec on room.stl ({gpus}, K2); coverage cells/sec ({gpus}) in 'coverage' (K3) "
                      f"and 'k5_terrain_coverage' (K5)",
            "value": value,
            "unit": "ray-bounces/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "models/room.stl (reference mesh) + synthetic isotropic burst (PCG ray ids, kernel.py:51-52)",
            "config": {"workload": "K2: room.stl, 1 TX (10,0,5), RX (-10,0,5) r=0.1, 1M rays/GPU, 3 bounces, "
                                   "traced+received+row_mask + ordered compaction + CIR (10000 bins), rt_trace_cir",
                       "rays_per_gpu": N, "bounces": B, "rays_total": N * world, "settle_steps": settle,
                       "parallelism": f"ray-id shards x{world}, RCCL all-reduce of the CIR"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_parts": traffic_parts,
                         "kernel": f"k_fill_received + k_trace_bf<{B}>", "kernel_ms": kern_ms,
                         "kernel_ms_span": "HIP events carried by the fill's and the trace kernel's dispatch packets "
                                           "(fill start to trace end)",
                         "launches_timed": int(pst[0]), "launch_sampling": f"every {args.profile_every}",
                         "algorithmic_bytes_per_launch": bytes_per_launch, "ray_bounces": N * B,
                         "active_ray_bounces": active},
            "compute_roofline": valu,
            "received_rows_last_step": received_rows,
        }
        if cov_out is not None:
            out["coverage"] = cov_out
        if k4_out is not None:
            out["k4_terrain"] = k4_out
        if k5_out is not None:
            out["k5_terrain_coverage"] = k5_out
        if k1_out is not None:
            out["k1_plumbing"] = k1_out
        if world == 1 and not args.no_cpu_baseline:
            info, build = cpu_setup()
            cb = cpu_baseline_k2(args, B, tx, rx, info, build)
            out["cpu_baseline"] = cb["all"]
            # Warp's CPU launch is serial: the same restatement on one thread
            out["cpu_baseline_1thread"] = cb["1thread"]
            # every CPU the process may run on (affinity), beside the box's thread share;
            # host.cgroup_cpu_quota says how many of them the box's scheduler lets run at once
            out["cpu_baseline_all_cores"] = cb["all_cores"]
            if cov_out is not None:
                cb3 = cpu_baseline_k3(args, info)
                out["coverage"]["cpu_baseline"], out["coverage"]["cpu_baseline_1thread"] = cb3["all"], cb3["1thread"]
                out["coverage"]["cpu_baseline_all_cores"] = cb3["all_cores"]
            if k1_out is not None:
                cb1 = cpu_baseline_k1(args, info, build)
                k1_out["cpu_baseline"], k1_out["cpu_baseline_1thread"] = cb1["all"], cb1["1thread"]
                k1_out["cpu_baseline_all_cores"] = cb1["all_cores"]
        out["summary"] = summary(out)  # last key: survives a truncated tail of the line
        print(json.dumps(out), flush=True)
        bad = [k for k in ("coverage", "k5_terrain_coverage") if (out.get(k) or {}).get("map_equals_one_gpu") is False]
    else:
        bad = []
    if world > 1:
        dist.destroy_process_group()
    if bad:
        print(f"bench: the {world}-rank map of {', '.join(bad)} differs from the one-GPU map", file=sys.stderr,
              flush=True)
        sys.exit(3)


if __name__ == "__main__":
    main()
