"""World-size-2 runs of the multi-rank logic on CPU (gloo): ray shards and cell shards reduce to
the single-process result.  The per-rank compute is the CPU oracle here (no GPU); on the GPU the
same dist.py functions carry the HIP results over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle import oracle as orc
from rf_ray_tracing_warp_amd import dist as rdist
from rf_ray_tracing_warp_amd.mesh import load_stl, sphere

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TX, RX, B, N_PER = (10.0, 0.0, 5.0), (5.0, 3.0, 4.0), 3, 40_000


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ray_worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    env = load_stl(os.path.join(REPO, "models", "room.stl"))
    rxm = sphere(RX, 0.1, 1)
    off, n = rdist.ray_shard(rank, world, N_PER)
    o = orc.trace(orc.Mesh(env.vertices, env.faces), orc.Mesh(rxm.vertices, rxm.faces), TX, B, off, n,
                  want_traced=False, nthreads=2)
    paths = orc.clean_paths(o["received"], o["mask"])
    ir = torch.from_numpy(orc.cir_from_paths(paths, 1, N_PER * world, 2.998e8, 100e9, 100e-9))
    rdist.reduce_sum(ir)
    if rank == 0:
        out.put(ir.numpy())
    dist.destroy_process_group()


def test_ray_shards_sum_to_single_process():
    world = 2
    q = mp.get_context("spawn").SimpleQueue()
    pc = mp.spawn(_ray_worker, args=(world, _port(), q), nprocs=world, join=False)
    got = q.get()  # read before join: the child's queue feeder must drain first
    pc.join()
    env = load_stl(os.path.join(REPO, "models", "room.stl"))
    rxm = sphere(RX, 0.1, 1)
    o = orc.trace(orc.Mesh(env.vertices, env.faces), orc.Mesh(rxm.vertices, rxm.faces), TX, B, 0, N_PER * world,
                  want_traced=False)
    ref = orc.cir_from_paths(orc.clean_paths(o["received"], o["mask"]), 1, N_PER * world, 2.998e8, 100e9, 100e-9)
    assert np.count_nonzero(ref) > 0
    np.testing.assert_array_equal(np.nonzero(got)[0], np.nonzero(ref)[0])
    np.testing.assert_allclose(got, ref, rtol=1e-12)


def _cell_worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    env = load_stl(os.path.join(REPO, "models", "room.stl"))
    E = orc.Mesh(env.vertices, env.faces)
    centers = np.array([[x, y, 5.0] for x in (6.0, 8.0, 9.5) for y in (-1.0, 0.5, 2.0)])
    pm = np.zeros(len(centers))
    mine = [c for c in range(len(centers)) if rdist.owns_cell(c, rank, world, 3)]
    p, _ = orc.coverage_loop(E, TX, centers[mine], B, 20_000, nthreads=2)
    pm[mine] = p
    t = torch.from_numpy(pm)
    rdist.reduce_sum(t)
    if rank == 0:
        out.put(t.numpy())
    dist.destroy_process_group()


def test_cell_shards_sum_to_single_process():
    world = 2
    q = mp.get_context("spawn").SimpleQueue()
    pc = mp.spawn(_cell_worker, args=(world, _port(), q), nprocs=world, join=False)
    got = q.get()
    pc.join()
    env = load_stl(os.path.join(REPO, "models", "room.stl"))
    centers = np.array([[x, y, 5.0] for x in (6.0, 8.0, 9.5) for y in (-1.0, 0.5, 2.0)])
    ref, _ = orc.coverage_loop(orc.Mesh(env.vertices, env.faces), TX, centers, B, 20_000)
    np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
    ok = ~np.isnan(ref)
    assert ok.sum() >= 3
    np.testing.assert_array_equal(got[ok], ref[ok])


def test_shard_helpers():
    assert rdist.ray_shard(3, 8, 1000) == (3000, 1000)
    owners = [sum(rdist.owns_cell(c, r, 8, 10) for r in range(8)) for c in range(100)]
    assert owners == [1] * 100
    # a whole x column belongs to one rank
    assert all(rdist.owns_cell(c, (c % 10) % 8, 8, 10) for c in range(100))


def _a2a_worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # rank r sends (r + d + 1) rows to rank d: key = r*1000 + d*100 + i, sum words (key, 3 key, -key)
    counts = [rank + d + 1 for d in range(world)]
    keys = torch.tensor([rank * 1000 + d * 100 + i for d in range(world) for i in range(counts[d])], dtype=torch.int64)
    rows = torch.stack([keys, keys, keys * 3, -keys], dim=1)  # Coverage.trace_rows' (n, 4) int64 layout
    r4, rc = rdist.exchange_rows(rows, counts)
    assert r4.shape == (sum(rc), 4) and rc == [r + rank + 1 for r in range(world)]
    assert (r4[:, 1] == r4[:, 0]).all() and (r4[:, 2] == 3 * r4[:, 0]).all() and (r4[:, 3] == -r4[:, 0]).all()
    out.put((rank, r4[:, 0].tolist(), rc))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_rows_routes_in_source_rank_order(world):
    """dist.exchange_rows (ray-sharded coverage): every owner receives its rows from rank 0, then
    rank 1, ... -- one ascending segment per source, the owner stage's merge precondition -- with
    every word intact, and the per-source counts."""
    q = mp.get_context("spawn").SimpleQueue()
    pc = mp.spawn(_a2a_worker, args=(world, _port(), q), nprocs=world, join=False)
    got = dict((r, (k, c)) for r, k, c in (q.get() for _ in range(world)))
    pc.join()
    for d in range(world):
        want = [r * 1000 + d * 100 + i for r in range(world) for i in range(r + d + 1)]
        assert got[d][0] == want
        assert got[d][1] == [r + d + 1 for r in range(world)]


def test_ray_range_partitions_the_burst():
    for n, w in [(1_000_000, 8), (7, 3), (16_777_216, 8), (5, 5)]:
        parts = [rdist.ray_range(r, w, n) for r in range(w)]
        assert parts[0][0] == 0 and sum(c for _, c in parts) == n
        for (o1, c1), (o2, _) in zip(parts, parts[1:]):
            assert o1 + c1 == o2


def _gather_worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # rank r holds r*2 rows (rank 0: none) of shape (4, 3), values r*100 + row
    rows = np.stack([np.full((4, 3), rank * 100 + i, np.float32) for i in range(rank * 2)]) if rank else \
        np.zeros((0, 4, 3), np.float32)
    parts = rdist.gather_rows(rows, None, 0)
    out.put((rank, [p.tolist() for p in parts]))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_rows_variable_counts(world):
    """dist.gather_rows (Tracer.compute_cir_distributed's path gather): counts all-gather + one padded
    tensor all-gather; every rank gets every rank's rows in rank order, empty blocks included."""
    q = mp.get_context("spawn").SimpleQueue()
    pc = mp.spawn(_gather_worker, args=(world, _port(), q), nprocs=world, join=False)
    got = dict(q.get() for _ in range(world))
    pc.join()
    for r in range(world):
        assert len(got[r]) == world
        for src in range(world):
            blk = np.asarray(got[r][src], np.float32).reshape(-1, 4, 3)
            assert blk.shape[0] == src * 2
            for i in range(src * 2):
                assert (blk[i] == src * 100 + i).all()


def _a2a_empty_worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # rank 0 sends nothing at all (a ray share with no first-win record); the others send 2 per owner
    counts = [0] * world if rank == 0 else [2] * world
    n = sum(counts)
    keys = torch.tensor([rank * 100 + d * 10 + i for d in range(world) for i in range(counts[d])], dtype=torch.int64)
    rows = torch.stack([keys, keys + 1, keys + 2, keys + 3], dim=1) if n else torch.empty((0, 4), dtype=torch.int64)
    r4, rc = rdist.exchange_rows(rows, counts)
    assert rc == [0] + [2] * (world - 1)
    out.put((rank, r4.tolist()))
    dist.destroy_process_group()


def test_exchange_rows_with_an_empty_sender():
    """a rank whose send counts are all zero must not break the row all-to-all."""
    world = 3
    q = mp.get_context("spawn").Queue()
    pc = mp.spawn(_a2a_empty_worker, args=(world, _port(), q), nprocs=world, join=False)
    got = dict(q.get(timeout=120) for _ in range(world))
    pc.join()
    for d in range(world):
        want = [r * 100 + d * 10 + i for r in range(1, world) for i in range(2)]
        assert got[d] == [[x, x + 1, x + 2, x + 3] for x in want]


def _gather_map_worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rows, nx = 6, 7  # nx not a multiple of the world size
    full = torch.arange(rows * nx, dtype=torch.float64) * 1.25 + 0.5
    full[3] = float("nan")  # an owner's NaN (a cell that receives nothing)
    ix = torch.arange(rows * nx) % nx
    mine = torch.where(ix % world == rank, full, torch.zeros_like(full))
    g = rdist.gather_power_map(mine.clone(), nx)
    r = mine.clone()
    dist.all_reduce(r)
    out.put((rank, g.tolist(), r.tolist(), full.tolist()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_power_map_equals_the_sum_reduce(world):
    """The owners' disjoint x columns gathered equal the sum-reduce of their maps, bit for bit."""
    q = mp.get_context("spawn").Queue()
    pc = mp.spawn(_gather_map_worker, args=(world, _port(), q), nprocs=world, join=False)
    got = [q.get(timeout=120) for _ in range(world)]
    pc.join()
    for _, g, r, full in got:
        a, b, f = np.array(g), np.array(r), np.array(full)
        assert a.tobytes() == b.tobytes() and a.tobytes() == f.tobytes()
