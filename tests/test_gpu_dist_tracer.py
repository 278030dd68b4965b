"""Ray-sharded Tracer on one GPU: 2 ranks (gloo), each tracing half of the global
ray ids, must return the single-process compute_cir result: the same received paths in ray-id
order (bit-exact) and the same impulse response (bins exactly, amplitudes to f64 summation order)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
mp = pytest.importorskip("torch.multiprocessing")

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, B = 200_000, 3


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _scene():
    from rf_ray_tracing_warp_amd.mesh import load_stl
    return load_stl(os.path.join(REPO, "models", "room.stl"))


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rf_ray_tracing_warp_amd import Tracer
    t = Tracer(_scene(), 2.998e8, 100e9, 100e-9, B, N, device=0)
    paths, ir = t.compute_cir_distributed((10.0, 0.0, 5.0), 1, (6.0, 2.0, 5.0), 0.1)
    if rank == 0:
        q.put(([p.tolist() for p in paths], ir))
    dist.barrier()
    dist.destroy_process_group()


def test_ray_sharded_compute_cir_equals_single(require_gpu):
    from rf_ray_tracing_warp_amd import Tracer
    t = Tracer(_scene(), 2.998e8, 100e9, 100e-9, B, N, device=0)
    ref_paths, ref_ir = t.compute_cir((10.0, 0.0, 5.0), 1, (6.0, 2.0, 5.0), 0.1)
    del t
    q = mp.get_context("spawn").SimpleQueue()
    pc = mp.spawn(_worker, args=(2, _port(), q), nprocs=2, join=False)
    paths, ir = q.get()
    pc.join()
    assert len(paths) == len(ref_paths) and len(ref_paths) > 0
    for a, b in zip(paths, ref_paths):
        np.testing.assert_array_equal(np.asarray(a, np.float32), b)
    np.testing.assert_array_equal(np.nonzero(ir)[0], np.nonzero(ref_ir)[0])
    np.testing.assert_allclose(ir, ref_ir, rtol=1e-12, atol=0)


def _cov_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rf_ray_tracing_warp_amd.coverage import CoverageGrid, coverage_map
    grid = CoverageGrid(8.0, -2.5, 4.6, 0.37, 0.41, 0.4, 13, 12, 2)
    p = coverage_map(_scene(), (10.0, 0.0, 5.0), grid, max_bounces=3, tx_num_rays=60_000, device=0)
    if rank == 0:
        q.put(p)
    dist.barrier()
    dist.destroy_process_group()


def test_ray_sharded_coverage_map_equals_single(require_gpu):
    """coverage_map under a 2-rank process group (ray shards, record all-to-all, map all-reduce)."""
    from rf_ray_tracing_warp_amd.coverage import CoverageGrid, coverage_map
    grid = CoverageGrid(8.0, -2.5, 4.6, 0.37, 0.41, 0.4, 13, 12, 2)
    ref = coverage_map(_scene(), (10.0, 0.0, 5.0), grid, max_bounces=3, tx_num_rays=60_000, device=0)
    q = mp.get_context("spawn").SimpleQueue()
    pc = mp.spawn(_cov_worker, args=(2, _port(), q), nprocs=2, join=False)
    got = q.get()
    pc.join()
    np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
    ok = ~np.isnan(ref)
    assert ok.sum() >= 20
    np.testing.assert_allclose(got[ok], ref[ok], rtol=1e-12)


def _device_worker(rank, world, port, q):
    """compute_cir_distributed and Coverage.run must issue every collective with the plan's GPU
    current (RCCL uses the current device), and must leave the caller's current device alone."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rf_ray_tracing_warp_amd import Tracer
    from rf_ray_tracing_warp_amd.coverage import Coverage, CoverageGrid
    seen = []
    real = {name: getattr(dist, name) for name in ("all_reduce", "all_gather", "all_to_all_single")}

    def spy(name):
        def f(*a, **k):
            seen.append((name, torch.cuda.current_device()))
            return real[name](*a, **k)
        return f

    for name in real:
        setattr(dist, name, spy(name))
    dev = torch.cuda.device_count() - 1  # the last GPU (cuda:0 on a one-GPU box)
    t = Tracer(_scene(), 2.998e8, 100e9, 100e-9, B, 50_000, device=dev)
    t.compute_cir_distributed((10.0, 0.0, 5.0), 1, (6.0, 2.0, 5.0), 0.1)
    grid = CoverageGrid(8.0, -2.5, 4.6, 0.37, 0.41, 0.4, 6, 5, 1)
    cov = Coverage(_scene(), 2.998e8, 100e9, 100e-9, B, 20_000, grid, device=dev, shard_index=rank,
                   shard_count=world, shard_mode="rays")
    cov.run((10.0, 0.0, 5.0), 1)
    cov.close()
    q.put((rank, dev, seen, torch.cuda.current_device()))
    dist.barrier()
    dist.destroy_process_group()


def test_collectives_run_on_the_plan_device(require_gpu):
    q = mp.get_context("spawn").SimpleQueue()
    pc = mp.spawn(_device_worker, args=(2, _port(), q), nprocs=2, join=False)
    got = [q.get() for _ in range(2)]
    pc.join()
    for rank, dev, seen, cur_after in got:
        names = {n for n, _ in seen}
        assert {"all_reduce", "all_gather", "all_to_all_single"} <= names, names
        assert all(d == dev for _, d in seen), seen
        assert cur_after == 0  # the caller's current device is untouched


def _nccl_worker(q, port):
    """world_size 1 under the "nccl" backend (RCCL): the only RCCL process group a one-GPU box can
    form (RCCL refuses two ranks on one GPU).  Runs the RCCL code paths end to end."""
    import torch.distributed as dist
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda:0"))
    from rf_ray_tracing_warp_amd import Tracer
    from rf_ray_tracing_warp_amd import dist as rdist
    from rf_ray_tracing_warp_amd.coverage import Coverage, CoverageGrid
    t = Tracer(_scene(), 2.998e8, 100e9, 100e-9, B, N, device=0)
    paths, ir = t.compute_cir_distributed((10.0, 0.0, 5.0), 1, (6.0, 2.0, 5.0), 0.1)
    grid = CoverageGrid(8.0, -2.5, 4.6, 0.37, 0.41, 0.4, 13, 12, 2)
    cov = Coverage(_scene(), 2.998e8, 100e9, 100e-9, B, 60_000, grid, device=0, shard_mode="rays")
    rows, counts = cov.trace_rows((10.0, 0.0, 5.0), 1)
    rows = rows.clone()
    r2, c2 = rdist.exchange_rows(rows, counts)  # RCCL all-to-all (world 1)
    p = cov.power_from_rows(r2, c2)
    cov.check()
    dist.all_reduce(p)
    q.put(([pp.tolist() for pp in paths], ir, p.cpu().numpy(), bool(torch.equal(r2, rows))))
    dist.destroy_process_group()


def test_rccl_world1_paths(require_gpu):
    from rf_ray_tracing_warp_amd import Tracer
    from rf_ray_tracing_warp_amd.coverage import CoverageGrid, coverage_map
    t = Tracer(_scene(), 2.998e8, 100e9, 100e-9, B, N, device=0)
    ref_paths, ref_ir = t.compute_cir((10.0, 0.0, 5.0), 1, (6.0, 2.0, 5.0), 0.1)
    grid = CoverageGrid(8.0, -2.5, 4.6, 0.37, 0.41, 0.4, 13, 12, 2)
    ref_map = coverage_map(_scene(), (10.0, 0.0, 5.0), grid, max_bounces=3, tx_num_rays=60_000, device=0)
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    p = ctx.Process(target=_nccl_worker, args=(q, _port()))
    p.start()
    paths, ir, pm, same_keys = q.get()
    p.join(timeout=120)
    assert p.exitcode == 0
    assert same_keys
    assert len(paths) == len(ref_paths) > 0
    for a, b in zip(paths, ref_paths):
        np.testing.assert_array_equal(np.asarray(a, np.float32), b)
    np.testing.assert_array_equal(ir, ref_ir)
    pm = pm.reshape(ref_map.shape)
    np.testing.assert_array_equal(np.isnan(pm), np.isnan(ref_map))
    ok = ~np.isnan(ref_map)
    np.testing.assert_allclose(pm[ok], ref_map[ok], rtol=1e-12)
