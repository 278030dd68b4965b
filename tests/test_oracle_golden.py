"""The CPU oracle against the reference's own outputs (CPU only).

host_cir.npz   -- produced by running the reference's tracer.py (stub-warp harness,
                  tests/golden/make_golden.py).  Pins tracer.py:84-117 and :34-61.
scene_html.npz -- extracted from the reference artifact web/scene.html
                  (tests/golden/extract_scene_html.py).  Pins ray generation (kernel.py:51-52),
                  the receiver icosphere (tracer.py:27) and the watertight closest hit
                  (kernel.py:71) on the artifact's almost_empty.stl run.
"""
import os

import numpy as np
import pytest

from oracle import oracle as orc
from rf_ray_tracing_warp_amd.mesh import icosphere, load_stl, sphere

HERE = os.path.dirname(os.path.abspath(__file__))
G = os.path.join(HERE, "golden")


@pytest.fixture(scope="module")
def host():
    return np.load(os.path.join(G, "host_cir.npz"))


@pytest.fixture(scope="module")
def scene():
    return np.load(os.path.join(G, "scene_html.npz"))


CASES = ["edge", "room0", "room1", "room2"]


@pytest.mark.parametrize("case", CASES)
def test_host_cir_matches_reference(host, case):
    rec, mask = host[f"{case}_received"], host[f"{case}_mask"]
    c, fs, win, txp = host[f"{case}_params"]
    paths = orc.clean_paths(rec, mask)
    assert [len(p) for p in paths] == host[f"{case}_lengths"].tolist()
    if paths:
        np.testing.assert_array_equal(np.concatenate(paths), host[f"{case}_paths"])
    ir = orc.cir_from_paths(paths, int(txp), len(rec), float(c), float(fs), float(win))
    np.testing.assert_array_equal(ir, host[f"{case}_ir"])  # bit-exact: same NumPy ops


def test_bounce_amplitude_matches_reference(host):
    a = host["amp_angles32"]
    got32 = np.array([float(orc.bounce_amplitude(x)) for x in a])
    got64 = np.array([float(orc.bounce_amplitude(float(x))) for x in a])
    np.testing.assert_array_equal(got32, host["amp_f32"])
    np.testing.assert_array_equal(got64, host["amp_f64"])


def test_icosphere_matches_artifact(scene):
    v, f = icosphere(3)
    np.testing.assert_array_equal(f, scene["sphere_f"].astype(np.int64))
    np.testing.assert_array_equal((v * 0.5 + scene["tx"]).astype(np.float32), scene["sphere_v"])
    np.testing.assert_array_equal((v * 0.5 + scene["rx"]).astype(np.float32), scene["rx_sphere_v"])


def test_ray_generation_matches_artifact(scene):
    ids, paths = scene["ray_ids"], scene["paths"]
    assert len(set(ids.tolist())) == len(ids) == 119
    d = orc.ray_dirs(0, 1)  # warm
    d = np.array([orc.ray_dirs(int(i), 1)[0] for i in ids]).astype(np.float64)
    d /= np.linalg.norm(d, axis=1)[:, None]
    u = (paths[:, 1] - paths[:, 0]).astype(np.float64)
    u /= np.linalg.norm(u, axis=1)[:, None]
    ang = np.arccos(np.clip((d * u).sum(1), -1, 1))
    assert ang.max() < 5e-8, ang.max()


def _merge(pts, tol=1e-5):
    out = [pts[0]]
    for p in pts[1:]:
        if np.linalg.norm(p - out[-1]) > tol:
            out.append(p)
    return np.array(out)


def test_trace_matches_artifact(scene, repo):
    env = load_stl(os.path.join(repo, "models", "almost_empty.stl"))
    rxm = sphere(scene["rx"], 0.1, 3)  # that run used trimesh's default subdivisions=3
    E, R = orc.Mesh(env.vertices, env.faces), orc.Mesh(rxm.vertices, rxm.faces)
    cands = np.sort(scene["cone_ids"])
    cands = cands[cands <= scene["ray_ids"].max()]
    received, rows = [], {}
    for i in cands:
        o = orc.trace(E, R, scene["tx"], 3, int(i), 1, nthreads=1)
        if o["mask"][0]:
            received.append(int(i))
            rows[int(i)] = o["received"][0]
    # the same 119 rays are received, and no other ray of the candidate cone
    assert sorted(received) == sorted(scene["ray_ids"].tolist())
    exact_first, structure = 0, 0
    for k, i in enumerate(scene["ray_ids"]):
        r = rows[int(i)]
        r = r[~np.isnan(r[:, 0])]
        ref = scene["paths"][k][: scene["lengths"][k]]
        assert np.abs(r[1] - ref[1]).max() < 4e-6
        exact_first += np.array_equal(r[1], ref[1])
        m = _merge(r)  # trimesh.load_path merges near-duplicate vertices in the artifact
        if len(m) == len(ref):
            structure += 1
            assert np.abs(m - ref).max() < 4e-6
    assert exact_first >= 117, exact_first
    assert structure >= 118, structure


@pytest.mark.parametrize("case", CASES)
def test_vectorised_host_cir_matches_reference(host, case):
    """orc.cir_from_rows (the per-path loop vectorised, used for cells that receive every ray) on the
    reference-generated goldens: bins exact, amplitudes to libm ulps (math.sin vs np.sin)."""
    rec, mask = host[f"{case}_received"], host[f"{case}_mask"]
    c, fs, win, txp = host[f"{case}_params"]
    ir, _, _ = orc.cir_from_rows(rec, mask, int(txp), len(rec), float(c), float(fs), float(win))
    ref = host[f"{case}_ir"]
    np.testing.assert_array_equal(np.nonzero(ir)[0], np.nonzero(ref)[0])
    np.testing.assert_allclose(ir, ref, rtol=1e-13, atol=0)


def test_vectorised_host_cir_matches_loop_on_dense_paths():
    """A cell whose receiver contains the transmitter receives every ray (paths of every length,
    RX self-hits with NaN angles): the vectorised CIR equals the literal loop, both arccos forms."""
    from rf_ray_tracing_warp_amd.mesh import load_stl, sphere
    env = load_stl(os.path.join(os.path.dirname(HERE), "models", "room.stl"))
    tx, N, B = (10.0, 0.0, 5.0), 20_000, 3
    rxm = sphere((10.02, 0.05, 5.0), 0.1, 1)
    o = orc.trace(orc.Mesh(env.vertices, env.faces), orc.Mesh(rxm.vertices, rxm.faces), tx, B, 0, N,
                  want_traced=False, nthreads=4)
    assert o["mask"].sum() == N
    paths = orc.clean_paths(o["received"], o["mask"])
    assert len({len(p) for p in paths}) >= 2
    for arc_loop, arc_vec in ((np.arccos, np.arccos), (orc._arccos_cr, orc.arccos_cr_vec)):
        ref = orc.cir_from_paths(paths, 1, N, 2.998e8, 100e9, 100e-9, arccos=arc_loop)
        ir, _, _ = orc.cir_from_rows(o["received"], o["mask"], 1, N, 2.998e8, 100e9, 100e-9, arccos=arc_vec)
        np.testing.assert_array_equal(np.nonzero(ir)[0], np.nonzero(ref)[0])
        np.testing.assert_allclose(ir, ref, rtol=1e-12, atol=0)
