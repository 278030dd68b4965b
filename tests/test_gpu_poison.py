"""Read-before-write audit (VERDICT r1 "What's weak" #2): every coverage plan buffer, and a 256 MB
block of the default memory pool that the stream-ordered sort workspaces come from, is filled with
a poison byte before each run (rt_debug_poison).  A kernel that read memory the run did not write
-- stale records of an earlier run, an unwritten key slot, an uninitialised sort workspace -- would
make the result depend on the byte.  Maps, sparse impulse responses and trace outputs must be
bit-identical for every byte, on a fresh plan and on a re-used one, and equal to the oracle.

The receiver-first replay order (environment query culled at the receiver hit) is checked the same
way in a child process (RFRT_COV_RXFIRST=1): it must give the default order's bits."""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from oracle import oracle as orc  # noqa: E402
from rf_ray_tracing_warp_amd._lib import DeviceMesh, check, lib, ptr  # noqa: E402
from rf_ray_tracing_warp_amd.coverage import Coverage, CoverageGrid  # noqa: E402
from rf_ray_tracing_warp_amd.mesh import load_stl, sphere, synthetic_terrain  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BYTES = (0x00, 0xFF, 0x7F, 0xA5)


@pytest.fixture(scope="module", autouse=True)
def _gpu(require_gpu):
    lib()
    yield
    lib().rt_debug_poison(-1)


def _poison(b):
    check(lib().rt_debug_poison(b), "rt_debug_poison")


def _scenes():
    room = load_stl(os.path.join(REPO, "models", "room.stl"))
    terr = synthetic_terrain(256, 50.0)
    return {
        "room": (room, CoverageGrid.square(48, 15.0, 5.0), (10.0, 0.0, 5.0), 100e-9, 200_000),
        "terrain": (terr, CoverageGrid(-20.0, -20.0, 2.0, 0.8, 0.8, 1.0, 50, 50, 1), (10.0, 0.0, 4.5), 200e-9, 200_000),
    }


def _run(cov, tx):
    p = cov.run(tx, 1).reshape(-1)
    c, b, a = cov.impulse_responses()
    return p, c, b, a


def _digest(p, c, b, a):
    return hashlib.sha256(p.tobytes() + c.tobytes() + b.tobytes() + a.tobytes()).hexdigest()


@pytest.mark.parametrize("scene", ["room", "terrain"])
def test_poisoned_buffers_do_not_change_coverage(scene):
    mesh, grid, tx, win, N = _scenes()[scene]
    env = DeviceMesh(mesh.vertices, mesh.faces, 0)
    _poison(-1)
    cov = Coverage(mesh, 2.998e8, 100e9, win, 3, N, grid, 0.1, device=0, env_mesh=env)
    ref = _run(cov, tx)
    assert np.isfinite(ref[0]).sum() >= 10
    want = _digest(*ref)
    for byte in BYTES:
        _poison(byte)
        fresh = Coverage(mesh, 2.998e8, 100e9, win, 3, N, grid, 0.1, device=0, env_mesh=env)
        assert _digest(*_run(fresh, tx)) == want, f"fresh plan, poison {byte:#x}"
        assert _digest(*_run(fresh, tx)) == want, f"re-used plan, poison {byte:#x}"
        fresh.close()
        assert _digest(*_run(cov, tx)) == want, f"first plan re-run, poison {byte:#x}"
    _poison(-1)
    # and the poisoned result is the reference's: a few cells by the literal per-cell loop
    p, cells, bins, amps = ref
    nb = np.bincount(cells, minlength=grid.num_cells)
    pick = list(np.argsort(-nb)[:3]) + list(np.nonzero(nb == 1)[0][:2])
    E = orc.Mesh(mesh.vertices, mesh.faces)
    cen = grid.centers().reshape(-1, 3)
    for c in pick:
        r = orc.coverage_cell(E, tx, cen[c], 3, N, win=win)
        np.testing.assert_array_equal(bins[cells == c], np.nonzero(r["ir"])[0])
        np.testing.assert_allclose(p[c], r["power_cr"], rtol=1e-9)
    cov.close()
    env.close()


def test_poisoned_buffers_do_not_change_ray_sharded_coverage():
    mesh, grid, tx, win, N = _scenes()["terrain"]
    env = DeviceMesh(mesh.vertices, mesh.faces, 0)

    def sharded(W=3):
        plans = [Coverage(mesh, 2.998e8, 100e9, win, 3, N, grid, 0.1, device=0, env_mesh=env, shard_index=r,
                          shard_count=W, shard_mode="rays") for r in range(W)]
        sent = []
        for pl in plans:
            rows, counts = pl.trace_rows(tx, 1)
            o = np.concatenate([[0], np.cumsum(counts)])
            sent.append([rows[o[d]:o[d + 1]].clone() for d in range(W)])
        tot = torch.zeros(grid.num_cells, dtype=torch.float64, device="cuda:0")
        for d, pl in enumerate(plans):
            tot += pl.power_from_rows(torch.cat([sent[r][d] for r in range(W)]), [len(sent[r][d]) for r in range(W)])
            pl.check()
            pl.close()
        return tot.cpu().numpy()

    _poison(-1)
    ref = sharded()
    for byte in (0xFF, 0x00):
        _poison(byte)
        got = sharded()
        assert got.tobytes() == ref.tobytes(), f"poison {byte:#x}"
    _poison(-1)
    env.close()


def test_poisoned_overflowing_first_run_of_a_rank_plan():
    """A K3 rank plan of 8 (125k of 1M rays, 256^2 cells) overflows its first candidate capacity (8
    per ray) on its first run while the early window replay is queued: that attempt must test
    nothing (the keys past the capacity have holes -- poison here) and the rerun must give the
    unpoisoned plan's records bit for bit."""
    room = load_stl(os.path.join(REPO, "models", "room.stl"))
    grid = CoverageGrid.square(256, 15.0, 5.0)
    tx, win, W, r = (10.0, 0.0, 5.0), 100e-9, 8, 3

    def records():
        pl = Coverage(room, 2.998e8, 100e9, win, 3, 1_000_000, grid, 0.1, device=0, shard_index=r, shard_count=W,
                      shard_mode="rays")
        rows, counts = pl.trace_rows(tx, 1)
        out = (rows[:, 0].cpu().numpy().copy(), rows[:, 1:].cpu().numpy().copy(), list(counts), pl.last_candidates)
        pl.close()
        return out

    _poison(-1)
    ref = records()
    assert ref[3] > 8 * (1_000_000 // W)  # the first attempt overflowed
    for byte in (0xFF, 0xA5):
        _poison(byte)
        got = records()
        assert got[2] == ref[2], f"poison {byte:#x}"
        assert got[0].tobytes() == ref[0].tobytes() and got[1].tobytes() == ref[1].tobytes(), f"poison {byte:#x}"
    _poison(-1)


def test_poisoned_pool_does_not_change_bvh_trace():
    """rt_trace on a BVH mesh sorts its rows by direction in a stream-ordered pool workspace."""
    terr = synthetic_terrain(256, 50.0)
    env = DeviceMesh(terr.vertices, terr.faces, 0)
    rxm = sphere((-10.125, 0.0, 4.8), 0.1, 1)
    rx = DeviceMesh(rxm.vertices, rxm.faces, 0)
    N, B = 1 << 17, 5
    tx = np.asarray((10.0, 0.0, 4.5), np.float32)
    s = torch.cuda.current_stream().cuda_stream

    def trace(fill):
        tr = torch.full((N, B + 1, 3), fill, dtype=torch.float32, device="cuda:0")
        rc = torch.full((N, B + 1, 3), fill, dtype=torch.float32, device="cuda:0")
        m = torch.full((N,), 7, dtype=torch.int32, device="cuda:0")
        kind = torch.full((N, B), 9, dtype=torch.int32, device="cuda:0")
        face = torch.full((N, B), 9, dtype=torch.int32, device="cuda:0")
        check(lib().rt_trace(env.handle, tx.ctypes.data, rx.handle, B, 0, N, ptr(tr), ptr(rc), ptr(m), ptr(kind),
                             ptr(face), s), "rt_trace")
        return [x.cpu().numpy().tobytes() for x in (tr, rc, m, kind, face)]

    _poison(-1)
    ref = trace(0.0)
    for byte, fill in ((0xFF, float("nan")), (0x00, 1e30), (0xA5, -3.0)):
        _poison(byte)
        assert trace(fill) == ref, f"poison {byte:#x}"
    _poison(-1)
    o = orc.trace(orc.Mesh(terr.vertices, terr.faces), orc.Mesh(rxm.vertices, rxm.faces), tx, B, 0, 4096)
    got = np.frombuffer(ref[3], np.int32).reshape(N, B)[:4096]
    np.testing.assert_array_equal(got, o["hit_kind"])
    env.close()
    rx.close()


_CHILD = r"""
import hashlib, json, os, sys
sys.path.insert(0, os.environ["REPO"])
import numpy as np
from rf_ray_tracing_warp_amd._lib import lib
from rf_ray_tracing_warp_amd.coverage import Coverage, CoverageGrid
from rf_ray_tracing_warp_amd.mesh import synthetic_terrain
lib().rt_debug_poison(int(os.environ["POISON"]))
terr = synthetic_terrain(256, 50.0)
grid = CoverageGrid(-20.0, -20.0, 2.0, 0.8, 0.8, 1.0, 50, 50, 1)
cov = Coverage(terr, 2.998e8, 100e9, 200e-9, 3, 200_000, grid, 0.1, device=0)
out = []
for _ in range(3):
    p = cov.run((10.0, 0.0, 4.5), 1).reshape(-1)
    c, b, a = cov.impulse_responses()
    out.append(hashlib.sha256(p.tobytes() + c.tobytes() + b.tobytes() + a.tobytes()).hexdigest())
print(json.dumps(out))
"""


def test_receiver_first_replay_is_bit_identical():
    """The replay variant DESIGN.md r1 dropped as nondeterministic: receiver query first, BVH query
    culled at the receiver's t.  Same bits as the default order, run after run, under poison."""
    res = {}
    for rxfirst, poison in (("0", "-1"), ("1", "-1"), ("1", "255"), ("1", "165")):
        env = dict(os.environ, REPO=REPO, RFRT_COV_RXFIRST=rxfirst, POISON=poison)
        r = subprocess.run([sys.executable, "-c", _CHILD], env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        res[(rxfirst, poison)] = json.loads(r.stdout.strip().splitlines()[-1])
    want = res[("0", "-1")][0]
    for k, hs in res.items():
        assert hs == [want] * 3, k
