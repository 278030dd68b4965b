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
