"""HIP path vs the CPU oracle, through the C ABI (needs an MI355X).

Bar: bit-exact for everything the kernel computes (directions, hit t, hit face ids, bounce
kinds, every path point, row_mask); impulse response within 1e-5 relative (north_star) with
bins identical.  Every row is compared, at the bench sizes too (K2's 1M rays, K4-shaped 1M-ray
bursts): the brute-force kernels skip faces and receivers by conservative float bounds (wave cones,
bundle boxes, reach tests; csrc/trace.hip), and an under-margin would show as a missing candidate on
any single ray, so no sampled-row comparison is left.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from oracle import oracle as orc  # noqa: E402
from rf_ray_tracing_warp_amd import _lib  # noqa: E402
from rf_ray_tracing_warp_amd._lib import DeviceMesh, check, lib, ptr  # noqa: E402
from rf_ray_tracing_warp_amd.mesh import load_stl, sphere  # noqa: E402
from rf_ray_tracing_warp_amd.tracer import Tracer  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
DEV = "cuda:0"


def _stream():
    return torch.cuda.current_stream().cuda_stream


@pytest.fixture(scope="module", autouse=True)
def _gpu(require_gpu):
    lib()


@pytest.fixture(scope="module")
def room():
    return load_stl(os.path.join(REPO, "models", "room.stl"))


@pytest.fixture(scope="module")
def empty():
    return load_stl(os.path.join(REPO, "models", "almost_empty.stl"))


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


@pytest.mark.parametrize("op,gen", [
    (0, lambda r: np.abs(r.standard_normal(1 << 20)).astype(np.float32) * np.float32(1e3)),
    (1, lambda r: (r.standard_normal(1 << 20) * 10).astype(np.float32)),
    (2, lambda r: r.uniform(0, 2 * np.pi, 1 << 20).astype(np.float32)),
    (3, lambda r: r.uniform(0, 2 * np.pi, 1 << 20).astype(np.float32)),
    (4, lambda r: r.uniform(-1, 1, 1 << 20).astype(np.float32)),
])
def test_math_bitexact(op, gen):
    x = gen(np.random.default_rng(op))
    if op == 4:
        x[:5] = [-1.0, 1.0, 0.5, -0.5, 0.0]
    xt = torch.from_numpy(x).to(DEV)
    out = torch.empty_like(xt)
    check(lib().rt_selftest_math(ptr(xt), x.size, ptr(out), op, _stream()))
    got = out.cpu().numpy()
    if op == 0:
        ref = np.sqrt(x)
    elif op == 1:
        ref = (np.float32(1.0) / x).astype(np.float32)
    elif op in (2, 3):
        s, c = orc.sincosf(x)
        ref = s if op == 2 else c
    else:
        ref = orc.acosf(x)
    np.testing.assert_array_equal(_bits(got), _bits(ref))


@pytest.mark.parametrize("offset,n", [(0, 1 << 20), (79_000_000, 1 << 18), ((1 << 31) - 100, 100)])
def test_ray_dirs_bitexact(offset, n):
    out = torch.empty((n, 3), dtype=torch.float32, device=DEV)
    check(lib().rt_ray_dirs(offset, n, ptr(out), _stream()))
    np.testing.assert_array_equal(_bits(out.cpu().numpy()), _bits(orc.ray_dirs(offset, n)))


def _random_rays(rng, n, lo, hi):
    o = rng.uniform(lo, hi, (n, 3)).astype(np.float32)
    d = rng.standard_normal((n, 3))
    d /= np.linalg.norm(d, axis=1)[:, None]
    return o, d.astype(np.float32)


@pytest.mark.parametrize("which", ["room", "rx1", "rx3"])
def test_query_bitexact(which, room):
    rng = np.random.default_rng(7)
    if which == "room":
        v, f = room.vertices, room.faces
        o, d = _random_rays(rng, 200_000, -16, 16)
    else:
        m = sphere((-10.0, 0.0, 5.0), 0.1, 1 if which == "rx1" else 3)
        v, f = m.vertices, m.faces
        o, d = _random_rays(rng, 200_000, -0.2, 0.2)
        o += np.array([-10.0, 0.0, 5.0], np.float32)  # origins around the sphere (inside and out)
    dm = DeviceMesh(v, f)
    ot, dt = torch.from_numpy(o).to(DEV), torch.from_numpy(d).to(DEV)
    t = torch.empty(len(o), dtype=torch.float32, device=DEV)
    face = torch.empty(len(o), dtype=torch.int32, device=DEV)
    check(lib().rt_query(dm.handle, ptr(ot), ptr(dt), len(o), ptr(t), ptr(face), _stream()))
    rt, rf, _ = orc.Mesh(v, f).query(o, d)
    np.testing.assert_array_equal(face.cpu().numpy(), rf)
    np.testing.assert_array_equal(_bits(t.cpu().numpy()), _bits(rt))
    assert (rf >= 0).mean() > 0.05


def _gpu_trace(env, rxm, tx, B, off, n, want_traced=True, builder="sah", reps=1):
    """rt_trace on fresh device meshes; reps > 1 launches again on the same meshes (the cached ray
    order and, from the second launch on, the longest-first chunk schedule) and asserts every
    launch's outputs equal the first's bit for bit."""
    e = DeviceMesh(env.vertices, env.faces, builder=builder)
    r = DeviceMesh(rxm.vertices, rxm.faces) if rxm is not None else None
    P = B + 1
    out = {
        "traced": torch.empty((n, P, 3), dtype=torch.float32, device=DEV) if want_traced else None,
        "received": torch.empty((n, P, 3), dtype=torch.float32, device=DEV),
        "mask": torch.empty(n, dtype=torch.int32, device=DEV),
        "hit_kind": torch.empty((n, B), dtype=torch.int32, device=DEV),
        "hit_face": torch.empty((n, B), dtype=torch.int32, device=DEV),
    }
    tx32 = np.asarray(tx, np.float32)
    first = None
    for _ in range(reps):
        for v in out.values():
            if v is not None:
                v.fill_(7)  # a stale buffer must not pass for a result
        check(lib().rt_trace(e.handle, tx32.ctypes.data, r.handle if r else None, B, off, n, ptr(out["traced"]),
                             ptr(out["received"]), ptr(out["mask"]), ptr(out["hit_kind"]), ptr(out["hit_face"]),
                             _stream()))
        torch.cuda.synchronize()
        got = {k: (v.cpu().numpy() if v is not None else None) for k, v in out.items()}
        if first is None:
            first = got
        else:
            for k, v in got.items():
                if v is not None:
                    np.testing.assert_array_equal(_bits(v) if v.dtype == np.float32 else v,
                                                  _bits(first[k]) if v.dtype == np.float32 else first[k], err_msg=k)
    return first


def _assert_trace_equal(g, o, rows=None):
    for k in ("traced", "received"):
        if g[k] is None or o[k] is None:
            continue
        a = g[k] if rows is None else g[k][rows]
        np.testing.assert_array_equal(_bits(a), _bits(o[k]), err_msg=k)
    for k in ("hit_kind", "hit_face"):
        a = g[k] if rows is None else g[k][rows]
        np.testing.assert_array_equal(a, o[k], err_msg=k)
    a = g["mask"] if rows is None else g["mask"][rows]
    np.testing.assert_array_equal(a.astype(np.uint32), o["mask"])


@pytest.mark.parametrize("cfg", [
    # K1: almost_empty, tx (1,0,1), rx (41,0,1), 10k rays, 1 bounce (main.py:25-27)
    ("almost_empty", (1, 0, 1), (41, 0, 1), 1, 0, 10_000),
    ("room", (10, 0, 5), (-10, 0, 5), 3, 0, 60_000),
    ("room", (10, 0, 5), (5, 3, 4), 3, 1_000_000, 60_000),
    ("room", (10, 0, 5), (-10, 8, 5), 5, 3, 40_000),
    ("room", (0, 5, 7), (10, 0.5, 5), 8, 17, 20_000),
    ("room", (10, 0, 5), (9.95, 0.02, 5.01), 4, 0, 20_000),  # tx inside the receiver ball
])
def test_trace_bitexact_small(cfg, room, empty):
    name, tx, rx, B, off, n = cfg
    env = room if name == "room" else empty
    rxm = sphere(rx, 0.1, 1)
    g = _gpu_trace(env, rxm, tx, B, off, n)
    o = orc.trace(orc.Mesh(env.vertices, env.faces), orc.Mesh(rxm.vertices, rxm.faces), tx, B, off, n)
    _assert_trace_equal(g, o)


def test_trace_generic_b12(room):
    rxm = sphere((5, 3, 4), 0.1, 1)
    g = _gpu_trace(room, rxm, (10, 0, 5), 12, 5, 8_000)
    o = orc.trace(orc.Mesh(room.vertices, room.faces), orc.Mesh(rxm.vertices, rxm.faces), (10, 0, 5), 12, 5, 8_000)
    _assert_trace_equal(g, o)


@pytest.mark.parametrize("rx", [(-10, 8, 5), (-10, 0, 5)])  # K2's receiver (main.py:29-31) and one in LOS
def test_trace_k2_full_size(room, rx):
    """K2: room.stl, 1M rays, 3 bounces -- every row of traced / received / row_mask / hit kinds /
    hit faces bit-exact against the oracle's trace of the same 1M rays (~0.1 s on 16 host threads)."""
    n, B, tx = 1_000_000, 3, (10, 0, 5)
    rxm = sphere(rx, 0.1, 1)
    g = _gpu_trace(room, rxm, tx, B, 0, n, reps=3)
    E, R = orc.Mesh(room.vertices, room.faces), orc.Mesh(rxm.vertices, rxm.faces)
    o = orc.trace(E, R, tx, B, 0, n)
    _assert_trace_equal(g, o)
    # invariants over all rows: received is a prefix of traced; mask <-> any RX hit
    tr, rc, hk = g["traced"], g["received"], g["hit_kind"]
    has_rx = (hk == 2).any(axis=1)
    np.testing.assert_array_equal(g["mask"].astype(bool), has_rx)
    fin = ~np.isnan(rc[..., 0])
    np.testing.assert_array_equal(rc[fin], tr[fin])


@pytest.mark.parametrize("tx,rx,rad,B,off", [
    ((10, 0, 5), (6, 1, 5), 1.0, 3, 0),          # a large receiver near the TX: many bounce-0 waves reach it
    ((10, 0, 5), (10.3, 0.2, 5.1), 0.5, 3, 7),   # TX inside the (padded) receiver ball
    ((-3, 4, 2), (12, -6, 8), 0.8, 5, 123_457),  # receiver near a corner, reached after reflections
    ((0, 5, 7), (10, 0.5, 5), 0.3, 8, 99),
    ((10, 0, 5), (6, 1, 5), 1.0, 1, 5),           # k_trace_bf<1>: bounce 0 only
    ((10, 0, 5), (-4, 3, 6), 0.6, 2, 77),
    ((2, -6, 3), (-8, 8, 9), 0.9, 4, 31_337),
    ((-12, 12, 13), (9, -9, 2), 0.9, 7, 4_242),
])
def test_trace_sorted_bursts(room, tx, rx, rad, B, off):
    """Direction-sorted brute-force bursts (n >= 2^16): bounce-0 wave cones, the bounce >= 1 bundle
    boxes and the receiver's wave tests -- every row bit-exact."""
    n = 100_000
    rxm = sphere(rx, rad, 1)
    g = _gpu_trace(room, rxm, tx, B, off, n, reps=3)
    assert g["mask"].sum() > 0
    E, R = orc.Mesh(room.vertices, room.faces), orc.Mesh(rxm.vertices, rxm.faces)
    o = orc.trace(E, R, tx, B, off, n)
    _assert_trace_equal(g, o)


def _cluttered_room(room, extra, seed):
    """room.stl plus `extra` small random triangles inside it (face counts around the 64-face
    limit of the bounce-0 cones and the bounce >= 1 bundle boxes, whose slot nf < 64 holds the receiver)."""
    from rf_ray_tracing_warp_amd.mesh import TriMesh
    rng = np.random.default_rng(seed)
    v = np.asarray(room.vertices, np.float64)
    f = np.asarray(room.faces, np.int64)
    c = rng.uniform((-12, -12, 1), (12, 12, 12), (extra, 1, 3))
    tri = c + rng.uniform(-1.5, 1.5, (extra, 3, 3))
    v2 = np.concatenate([v, tri.reshape(-1, 3)])
    f2 = np.concatenate([f, len(v) + np.arange(3 * extra).reshape(extra, 3)])
    return TriMesh(v2, f2)


@pytest.mark.parametrize("extra", [19, 20, 21])  # 63, 64, 65 faces
def test_trace_sorted_bursts_face_limits(room, extra):
    env = _cluttered_room(room, extra, seed=extra)
    assert len(env.faces) == 44 + extra
    n, B, tx, rx, off = 80_000, 3, (10, 0, 5), (4, 2, 5), 11
    rxm = sphere(rx, 0.7, 1)
    g = _gpu_trace(env, rxm, tx, B, off, n, reps=2)
    assert g["mask"].sum() > 0
    E, R = orc.Mesh(env.vertices, env.faces), orc.Mesh(rxm.vertices, rxm.faces)
    o = orc.trace(E, R, tx, B, off, n)
    _assert_trace_equal(g, o)


def test_artifact_scene_html_gpu(empty):
    """The reference artifact's 119 received rays (tests/golden/scene_html.npz) on the GPU."""
    g = np.load(os.path.join(HERE, "golden", "scene_html.npz"))
    rxm = sphere(g["rx"], 0.1, 3)
    ids = np.sort(g["cone_ids"])
    ids = ids[ids <= g["ray_ids"].max()]
    got = []
    for i in ids:
        r = _gpu_trace(empty, rxm, g["tx"], 3, int(i), 1, want_traced=False)
        if r["mask"][0]:
            got.append(int(i))
            k = int(np.nonzero(g["ray_ids"] == i)[0][0])
            assert np.abs(r["received"][0][1] - g["paths"][k][1]).max() < 4e-6
    assert sorted(got) == sorted(g["ray_ids"].tolist())


# ---------------------------------------------------------------------------- CIR
def _device_cir(received, mask, B, c, fs, win, txp, N):
    rec = torch.from_numpy(np.ascontiguousarray(received)).to(DEV)
    m = torch.from_numpy(mask.astype(np.int32)).to(DEV)
    n = len(received)
    ws = torch.empty(int(lib().rt_compact_workspace_bytes(n)), dtype=torch.uint8, device=DEV)
    idx = torch.empty(max(n, 1), dtype=torch.int64, device=DEV)
    cnt = torch.empty(1, dtype=torch.int64, device=DEV)
    check(lib().rt_compact(ptr(m), n, ptr(ws), ws.numel(), ptr(idx), ptr(cnt), _stream()))
    nb = int(win * fs)
    ir = torch.zeros(nb, dtype=torch.float64, device=DEV)
    bins = torch.full((max(n, 1),), -1, dtype=torch.int32, device=DEV)
    amps = torch.zeros(max(n, 1), dtype=torch.float64, device=DEV)
    check(lib().rt_cir(ptr(rec), ptr(idx), ptr(cnt), n, B, txp / N, c, fs, 0, nb, ptr(ir), ptr(bins), ptr(amps),
                       _stream()))
    k = int(cnt.item())
    return ir.cpu().numpy(), idx[:k].cpu().numpy(), bins[:k].cpu().numpy(), amps[:k].cpu().numpy()


@pytest.mark.parametrize("n", [0, 1, 2047, 2048, 2049, 1_000_000, 2048 * 1024, 2048 * 1024 + 1, 5_000_000])
@pytest.mark.parametrize("density", [0.0, 1e-6, 0.01, 0.5, 1.0])
def test_compact_ordered(n, density):
    """rt_compact == np.nonzero(row_mask) (tracer.py:87), through both launch paths (the scan folded
    into the scatter up to 1024 tiles, a separate scan above), from no row set to every row set."""
    rng = np.random.default_rng(n + int(density * 1000))
    mask = (rng.random(n) < density).astype(np.int32)
    if n and density == 1e-6:
        mask[n - 1] = 1  # last row of the last tile
    m = torch.from_numpy(mask).to(DEV)
    ws = torch.empty(int(lib().rt_compact_workspace_bytes(n)), dtype=torch.uint8, device=DEV)
    idx = torch.full((max(n, 1),), -1, dtype=torch.int64, device=DEV)
    cnt = torch.full((1,), -1, dtype=torch.int64, device=DEV)
    check(lib().rt_compact(ptr(m), n, ptr(ws), ws.numel(), ptr(idx), ptr(cnt), _stream()))
    k = int(cnt.item())
    ref = np.nonzero(mask)[0]
    assert k == len(ref)
    np.testing.assert_array_equal(idx[:k].cpu().numpy(), ref)


@pytest.mark.parametrize("case", ["edge", "room0", "room1", "room2"])
def test_cir_matches_reference_golden(case):
    h = np.load(os.path.join(HERE, "golden", "host_cir.npz"))
    rec, mask = h[f"{case}_received"], h[f"{case}_mask"]
    c, fs, win, txp = h[f"{case}_params"]
    ir, idx, bins, amps = _device_cir(rec, mask, rec.shape[1] - 1, float(c), float(fs), float(win), float(txp),
                                      len(rec))
    np.testing.assert_array_equal(idx, np.nonzero(mask)[0])
    ref = h[f"{case}_ir"]
    np.testing.assert_array_equal(np.nonzero(ir)[0], np.nonzero(ref)[0])
    np.testing.assert_allclose(ir, ref, rtol=1e-5, atol=0)
    paths = orc.clean_paths(rec, mask)
    for p, b, a in zip(paths, bins, amps):
        rb, ra = orc.path_bin_amp(p, float(txp), len(rec), float(c), float(fs))
        assert b == rb
        assert abs(a - ra) <= 1e-5 * abs(ra)


def test_compute_cir_end_to_end(room):
    """Tracer.compute_cir == oracle trace + reference host CIR (K2-shaped, 200k rays)."""
    N, B, tx, rx = 200_000, 3, (10, 0, 5), (5, 3, 4)
    t = Tracer(room, 2.998e8, 100e9, 100e-9, B, N)
    paths, ir = t.compute_cir(np.array(tx), 1, np.array(rx), 0.1)
    rxm = sphere(rx, 0.1, 1)
    o = orc.trace(orc.Mesh(room.vertices, room.faces), orc.Mesh(rxm.vertices, rxm.faces), tx, B, 0, N,
                  want_traced=False)
    ref_paths = orc.clean_paths(o["received"], o["mask"])
    assert len(paths) == len(ref_paths) > 0
    for a, b in zip(paths, ref_paths):
        np.testing.assert_array_equal(a, b)
    ref_ir = orc.cir_from_paths(ref_paths, 1, N, 2.998e8, 100e9, 100e-9)
    np.testing.assert_array_equal(np.nonzero(ir)[0], np.nonzero(ref_ir)[0])
    np.testing.assert_allclose(ir, ref_ir, rtol=1e-5, atol=0)


# ---------------------------------------------------------------------------- BVH (large meshes)
@pytest.fixture(scope="module")
def terrain256():
    from rf_ray_tracing_warp_amd.mesh import synthetic_terrain
    return synthetic_terrain(256, 50.0)


@pytest.mark.parametrize("builder", ["sah", "gpu"])
def test_bvh_query_bitexact(terrain256, builder):
    t = terrain256
    rng = np.random.default_rng(11)
    n = 300_000
    o = np.c_[rng.uniform(-50, 50, (n, 2)), rng.uniform(-2, 8, n)].astype(np.float32)
    d = rng.standard_normal((n, 3))
    d[:, 2] -= 0.3
    d = (d / np.linalg.norm(d, axis=1)[:, None]).astype(np.float32)
    om = orc.Mesh(t.vertices, t.faces)
    tb, fb, _ = om.query(o, d)
    hit = fb >= 0
    o = np.concatenate([o, (o[hit] + d[hit] * tb[hit][:, None]).astype(np.float32)])  # rays leaving the surface
    d = np.concatenate([d, d[hit]])
    dm = DeviceMesh(t.vertices, t.faces, builder=builder)
    info = dm.bvh_info()
    assert info["nodes"] > 0 and 0 < info["depth"] <= 60 and info["max_leaf"] <= 4
    ot, dt = torch.from_numpy(o).to(DEV), torch.from_numpy(d).to(DEV)
    tt = torch.empty(len(o), dtype=torch.float32, device=DEV)
    ff = torch.empty(len(o), dtype=torch.int32, device=DEV)
    check(lib().rt_query(dm.handle, ptr(ot), ptr(dt), len(o), ptr(tt), ptr(ff), _stream()))
    rt_, rf_, _ = om.query(o, d)
    np.testing.assert_array_equal(ff.cpu().numpy(), rf_)
    np.testing.assert_array_equal(_bits(tt.cpu().numpy()), _bits(rt_))


@pytest.mark.parametrize("B,off,n,builder", [(5, 0, 60_000, "sah"), (3, 5_000_000, 40_000, "sah"),
                                             (12, 7, 10_000, "sah"), (5, 0, 80_000, "gpu")])
def test_trace_bvh_bitexact(terrain256, B, off, n, builder):
    tx, rx = (10.0, 0.0, 4.5), (-10.125, 0.0, 4.8)  # main.py:22-23
    rxm = sphere(rx, 0.1, 1)
    g = _gpu_trace(terrain256, rxm, tx, B, off, n, builder=builder, reps=2)
    o = orc.trace(orc.Mesh(terrain256.vertices, terrain256.faces), orc.Mesh(rxm.vertices, rxm.faces), tx, B, off, n)
    _assert_trace_equal(g, o)
    assert (g["hit_kind"] == 1).sum() > n // 4


def test_receiver_too_large_rejected(terrain256):
    """Receivers are queried by brute force: a mesh beyond 65536 faces is refused before launch."""
    from rf_ray_tracing_warp_amd._lib import RfrtError
    from rf_ray_tracing_warp_amd.mesh import icosphere
    v, f = icosphere(6)  # 81920 faces
    big = DeviceMesh(v * 0.1, f)
    env = DeviceMesh(terrain256.vertices, terrain256.faces)
    n = 1024
    rec = torch.empty((n, 4, 3), dtype=torch.float32, device=DEV)
    mask = torch.empty(n, dtype=torch.int32, device=DEV)
    tx = np.asarray((0.0, 0.0, 5.0), np.float32)
    rc = lib().rt_trace(env.handle, tx.ctypes.data, big.handle, 3, 0, n, None, ptr(rec), ptr(mask), None, None,
                        _stream())
    assert rc != 0 and b"receiver mesh too large" in lib().rt_last_error()
    with pytest.raises(RfrtError):
        check(rc, "rt_trace")


def test_gpu_bvh_build_k4_mesh():
    """the device LBVH builds the 2.09M-face K4 mesh in well under the host SAH time,
    and traces on it equal the oracle (every row of a 200k-ray, 5-bounce burst)."""
    import time
    from rf_ray_tracing_warp_amd.mesh import synthetic_terrain
    t = synthetic_terrain(1024, 50.0)
    t0 = time.perf_counter()
    dm = DeviceMesh(t.vertices, t.faces, builder="gpu")
    t_gpu = time.perf_counter() - t0
    info = dm.bvh_info()
    dm.close()
    t0 = time.perf_counter()
    DeviceMesh(t.vertices, t.faces, builder="sah").close()
    t_sah = time.perf_counter() - t0
    print(f"mesh create: gpu LBVH {t_gpu:.3f} s, host SAH {t_sah:.3f} s, {info}")
    assert t_gpu < t_sah and info["depth"] <= 60
    n, B, tx, rx = 200_000, 5, (10.0, 0.0, 4.5), (-10.125, 0.0, 4.8)
    rxm = sphere(rx, 0.1, 1)
    g = _gpu_trace(t, rxm, tx, B, 0, n, builder="gpu")
    o = orc.trace(orc.Mesh(t.vertices, t.faces), orc.Mesh(rxm.vertices, rxm.faces), tx, B, 0, n)
    _assert_trace_equal(g, o)


def test_trace_k4_terrain_full_mesh():
    """K4 shape on one GPU: the 2.09M-triangle terrain, 1M rays, 5 bounces; every row bit-exact."""
    from rf_ray_tracing_warp_amd.mesh import synthetic_terrain
    t = synthetic_terrain(1024, 50.0)
    n, B, tx, rx = 1_000_000, 5, (10.0, 0.0, 4.5), (-10.125, 0.0, 4.8)
    rxm = sphere(rx, 0.1, 1)
    g = _gpu_trace(t, rxm, tx, B, 3_000_000, n, want_traced=True, reps=2)
    o = orc.trace(orc.Mesh(t.vertices, t.faces), orc.Mesh(rxm.vertices, rxm.faces), tx, B, 3_000_000, n)
    _assert_trace_equal(g, o)


def test_release_caches_between_traces(room):
    """rt_release_caches frees the cached ray orders and chunk schedules: the next
    launch recomputes them and every output bit is the same; destroying a mesh drops its own
    schedules (keyed by the mesh's process-unique id, not its address)."""
    rxm = sphere((6, 1, 5), 1.0, 1)
    a = _gpu_trace(room, rxm, (10, 0, 5), 3, 0, 100_000, reps=2)
    check(lib().rt_release_caches())
    b = _gpu_trace(room, rxm, (10, 0, 5), 3, 0, 100_000, reps=2)
    for k in a:
        if a[k] is not None:
            assert a[k].tobytes() == b[k].tobytes(), k
