#!/usr/bin/env python3
"""Headline benchmark: ray-bounces/s on models/room.stl (BASELINE.json configs[1], "K2").

One step = one pass of the hot path over one synthetic isotropic burst of 1M rays per GPU:
  rt_trace   (trace_paths_kernel, kernel.py:38-98: ray generation, 3 bounces of closest hit vs
              receiver + environment, reflect, full reference output contract: traced_paths,
              received_paths, row_mask -- tracer.py:70-72)
  rt_compact + rt_cir (tracer.py:87-117: received rows -> delay bins -> impulse response)
  RCCL all-reduce of the impulse response (N > 1: the job's CIR is the sum over ray shards).
Rays are sharded by global ray id (rank r traces ids [r*N, (r+1)*N)): per-GPU work is fixed as
GPUs are added ("weak").  Inputs (mesh tables) are resident in HBM before the timed region.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU, RCCL)

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "ray-bounces/sec on room.stl (1 GPU) + coverage cells/sec at 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
VALU_PEAK_GWI = 1024 * 2.4 / 2  # 256 CUs x 4 SIMDs, one wave64 VALU instruction per 2 cycles


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rays", type=int, default=1_000_000, help="rays per GPU per step (K2: 1M)")
    ap.add_argument("--bounces", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=1_000_000, help="rays per CPU-baseline chunk (~10 s total)")
    ap.add_argument("--no-coverage", action="store_true")
    ap.add_argument("--coverage-grid", type=int, default=256, help="K3: n x n receiver cells at z=5 on room.stl")
    ap.add_argument("--coverage-rays", type=int, default=1_000_000)
    ap.add_argument("--coverage-runs", type=int, default=3)
    ap.add_argument("--coverage-shard", choices=("rays", "cells"), default="rays",
                    help="N>1 coverage decomposition: ray shards + record all-to-all, or x-column cell shards")
    ap.add_argument("--no-k4", action="store_true", help="skip the terrain (apollo stand-in) legs K4/K5")
    ap.add_argument("--k4-rays", type=int, default=2_097_152, help="rays per GPU (K4: 16.7M over 8 GPUs)")
    ap.add_argument("--k5-grid", type=int, default=1024)
    ap.add_argument("--k5-rays", type=int, default=1_000_000)
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic_k2.json"),
                    help="per-launch HBM bytes measured by rocprofv3 PMC (profiles/)")
    return ap.parse_args()


def cpu_baseline(sample_rays, B, tx, rx, min_s=10.0, max_rays=400_000_000, threads=None):
    """The oracle (C restatement of kernel.py + tracer.py host tail) on the host cores."""
    from oracle import oracle as orc
    from rf_ray_tracing_warp_amd.mesh import load_stl, sphere

    env = load_stl(os.path.join(REPO, "models", "room.stl"))
    rxm = sphere(rx, 0.1, 1)
    E, R = orc.Mesh(env.vertices, env.faces), orc.Mesh(rxm.vertices, rxm.faces)
    threads = threads or min(16, os.cpu_count() or 1)
    orc.trace(E, R, tx, B, 0, 2000, nthreads=threads)  # warm
    # bounded sample: consecutive chunks of the same burst (ray ids 0, 1, 2, ...) until ~min_s of CPU work
    t0 = time.perf_counter()
    done = 0
    while True:
        o = orc.trace(E, R, tx, B, done, sample_rays, want_traced=True, nthreads=threads)
        paths = orc.clean_paths(o["received"], o["mask"])
        orc.cir_from_paths(paths, 1, sample_rays, 2.998e8, 100e9, 100e-9)
        done += sample_rays
        dt = time.perf_counter() - t0
        if dt >= min_s or done >= max_rays:
            break
    return {"value": done * B / dt, "unit": "ray-bounces/s", "cores": threads, "kind": "port",
            "sample": f"{done} rays x {B} bounces (ray ids 0..{done - 1}, chunks of {sample_rays}) of the K2 "
                      f"room.stl burst: trace + host CIR by oracle/rt_oracle.c (OpenMP, {threads} threads), "
                      f"{dt:.1f} s"}


def shard_desc(mode, world):
    if world == 1:
        return "1 GPU"
    if mode == "rays":
        return (f"rays sharded x{world} (1/{world} of every cell's rays per GPU), (cell, bin, amplitude) records "
                f"to the cells' owners (ix % {world}) by one RCCL all-to-all, RCCL sum of the power map")
    return f"cells sharded by x column (ix % {world}), every GPU traces all rays, RCCL sum of the power map"


def coverage_leg(args, env_m, env, local, rank, world, dist):
    """K3: coverage.py on room.stl, n x n cells at z = 5, tx (10,0,5), 1M rays per cell, 3 bounces.
    N > 1: each rank traces 1/N of every cell's rays and sends its (cell, bin, amplitude) records to
    the cells' owners (x columns, ix % world) in one RCCL all-to-all, or (--coverage-shard cells)
    each rank computes its x columns from all rays; the power map is sum-reduced (RCCL)."""
    import torch
    from rf_ray_tracing_warp_amd.coverage import Coverage, CoverageGrid

    grid = CoverageGrid.square(args.coverage_grid, 15.0, 5.0)
    mode = args.coverage_shard if world > 1 else "cells"
    cov = Coverage(env_m, 2.998e8, 100e9, 100e-9, args.bounces, args.coverage_rays, grid, 0.1, device=local,
                   shard_index=rank, shard_count=world, env_mesh=env, shard_mode=mode)
    tx = (10.0, 0.0, 5.0)

    def one():
        p = cov.run_device(tx, 1)
        if world > 1:
            dist.all_reduce(p)
        return p

    one()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.coverage_runs):
        p = one()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = (time.perf_counter() - t0) / args.coverage_runs
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t[0])
    pm = p.cpu().numpy()
    cand = torch.tensor([float(cov.last_candidates)], dtype=torch.float64, device=f"cuda:{local}")
    if world > 1:
        dist.all_reduce(cand)
    cov.close()
    return {"metric": "coverage cells/sec", "value": grid.num_cells / dt, "unit": "cells/s", "ms_per_map": dt * 1e3,
            "workload": f"K3: room.stl, {grid.nx}x{grid.ny} receivers at z=5 (centres -15+(i+1/2)*30/{grid.nx}), "
                        f"tx (10,0,5), {args.coverage_rays} rays per cell, {args.bounces} bounces, 10000 bins, "
                        f"signal power per cell; {shard_desc(mode, world)}",
            "scaling": "strong", "cells_receiving": int(np.isfinite(pm).sum()),
            "candidates": int(cand.item()), "algorithm": "exact shared-trajectory (csrc/coverage.hip)"}


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
    B, N = 5, args.k4_rays
    P = B + 1
    rxm = sphere((-10.125, 0.0, 4.8), 0.1, 1)
    rx = DeviceMesh(rxm.vertices, rxm.faces, local)
    tx = np.asarray((10.0, 0.0, 4.5), np.float32)
    traced = torch.empty((N, P, 3), dtype=torch.float32, device=dev)
    received = torch.empty((N, P, 3), dtype=torch.float32, device=dev)
    mask = torch.empty(N, dtype=torch.int32, device=dev)
    sh = torch.cuda.current_stream().cuda_stream
    L = lib()

    def step():
        check(L.rt_trace(env.handle, tx.ctypes.data, rx.handle, B, rank * N, N, ptr(traced), ptr(received), ptr(mask),
                         None, None, sh), "rt_trace")

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
    k4 = {"metric": "ray-bounces/sec", "value": world * N * B / dt, "unit": "ray-bounces/s", "ms_per_step": dt * 1e3,
          "workload": f"K4 on the declared apollo stand-in (synthetic terrain 1024^2 vertices, {len(terr.faces)} faces, "
                      f"BVH), {N} rays/GPU x {world}, {B} bounces, traced+received+row_mask",
          "scaling": "weak", "mesh_build_s": t_build}
    del traced, received, mask
    grid = CoverageGrid.square(args.k5_grid, 50.0, 2.0)
    mode = args.coverage_shard if world > 1 else "cells"
    cov = Coverage(terr, 2.998e8, 100e9, 200e-9, 3, args.k5_rays, grid, 0.1, device=local, shard_index=rank,
                   shard_count=world, env_mesh=env, shard_mode=mode)

    def one():
        p = cov.run_device((10.0, 0.0, 4.5), 1)
        if world > 1:
            dist.all_reduce(p)
        return p

    one()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    p = one()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt[0])
    pm = p.cpu().numpy()
    k5 = {"metric": "coverage cells/sec", "value": grid.num_cells / dt, "unit": "cells/s", "ms_per_map": dt * 1e3,
          "workload": f"K5 on the terrain stand-in: {grid.nx}x{grid.ny} receivers at z=2 over +-50 m, tx (10,0,4.5), "
                      f"{args.k5_rays} rays per cell, 3 bounces, 20000 bins; {shard_desc(mode, world)}",
          "scaling": "strong", "cells_receiving": int(np.isfinite(pm).sum()), "candidates": int(cov.last_candidates)}
    cov.close()
    return k4, k5


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

    from rf_ray_tracing_warp_amd import _lib
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
    ws = torch.empty(int(lib().rt_compact_workspace_bytes(N)), dtype=torch.uint8, device=dev)
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
    ev = []

    def drain():
        for j in range(2):
            if pending[j] is not None:
                pending[j].wait()  # the current stream waits for that all-reduce
                pending[j] = None

    def step(i, timed):
        ir = irs[i % 2]
        if pending[i % 2] is not None:
            pending[i % 2].wait()
            pending[i % 2] = None
        ir.zero_()
        if timed:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        check(L.rt_trace(env.handle, tx32.ctypes.data, rxd.handle, B, ray_offset, N, ptr(traced), ptr(received),
                         ptr(mask), None, None, sh), "rt_trace")
        if timed:
            e1.record(stream)
            ev.append((e0, e1))
        check(L.rt_compact(ptr(mask), N, ptr(ws), ws.numel(), ptr(index), ptr(count), sh), "rt_compact")
        check(L.rt_cir(ptr(received), ptr(index), ptr(count), N, B, amp0, c, fs, flags, n_bins, ptr(ir), None, None,
                       sh), "rt_cir")
        if world > 1:
            pending[i % 2] = dist.all_reduce(ir, async_op=True)

    for i in range(args.warmup):
        step(i, False)
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i, True)
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
    received_rows = int(count.item())

    cov_out = None
    if not args.no_coverage:
        cov_out = coverage_leg(args, env_m, env, local, rank, world, dist)
    k4_out = k5_out = None
    if not args.no_k4:
        k4_out, k5_out = terrain_legs(args, local, rank, world, dist)

    if rank == 0:
        bounces = world * N * B * args.steps
        value = bounces / elapsed
        bytes_per_launch = N * (24 * P + 4)  # traced + received rows + row_mask
        achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
        traffic = None
        try:
            with open(args.traffic_json) as fh:
                tj = json.load(fh)
            if tj.get("rays") == N and tj.get("bounces") == B:
                traffic = tj.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            pass
        # the binding resource of the brute-force LDS kernel is the VALU issue rate: VALU
        # instructions per launch come from a PMC pass (profiles/r1_k2_sq_counters.json, a
        # property of the code and the input), the time from the live HIP events above
        valu = None
        try:
            with open(os.path.join(REPO, "profiles", "r1_k2_sq_counters.json")) as fh:
                sq = json.load(fh)
            if N == 1_000_000 and B == 3:
                rate = sq["SQ_INSTS_VALU"] / (kern_ms * 1e-3) / 1e9  # wave-instructions / ns
                peak = VALU_PEAK_GWI
                valu = {"bound": "valu", "achieved": rate, "peak": peak, "unit": "G wave-instr/s", "frac": rate / peak,
                        "valu_instr_per_launch": sq["SQ_INSTS_VALU"],
                        "note": "peak = 1024 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU instruction"}
        except (OSError, ValueError, KeyError):
            pass
        out = {
            "metric": METRIC,
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
                                   "traced+received+row_mask + CIR (10000 bins)",
                       "rays_per_gpu": N, "bounces": B, "rays_total": N * world,
                       "parallelism": f"ray-id shards x{world}, RCCL all-reduce of the CIR"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "k_trace_bf<3>", "kernel_ms": kern_ms,
                         "algorithmic_bytes_per_launch": bytes_per_launch},
            "compute_roofline": valu,
            "received_rows_last_step": received_rows,
        }
        if cov_out is not None:
            out["coverage"] = cov_out
        if k4_out is not None:
            out["k4_terrain"] = k4_out
        if k5_out is not None:
            out["k5_terrain_coverage"] = k5_out
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.cpu_sample, B, tx, rx)
            # Warp's CPU launch is serial: the same restatement on one thread
            out["cpu_baseline_1thread"] = cpu_baseline(args.cpu_sample // 4, B, tx, rx, min_s=3.0, threads=1)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
