"""The oracle's BVH (used for large meshes) returns exactly what its brute force returns (CPU)."""
import numpy as np

from oracle import oracle as orc
from rf_ray_tracing_warp_amd.mesh import synthetic_terrain


def test_terrain_shape():
    t = synthetic_terrain(64, 50.0)
    assert t.faces.shape == (2 * 63 * 63, 3)
    z = t.vertices[:, 2]
    assert z.min() > -3 and z.max() < 1.5


def test_oracle_bvh_equals_brute_force():
    t = synthetic_terrain(48, 20.0, seed=3)
    bvh = orc.Mesh(t.vertices, t.faces, bvh_min=16)
    brute = orc.Mesh(t.vertices, t.faces, bvh_min=1 << 40)
    rng = np.random.default_rng(0)
    n = 20_000
    o = np.c_[rng.uniform(-20, 20, (n, 2)), rng.uniform(-1, 6, n)].astype(np.float32)
    d = rng.standard_normal((n, 3))
    d[:, 2] -= 0.5
    d = (d / np.linalg.norm(d, axis=1)[:, None]).astype(np.float32)
    # include rays starting exactly on the surface (self-hit quirk Q3)
    tb, fb, _ = brute.query(o, d)
    hit = fb >= 0
    o2 = (o[hit] + d[hit] * tb[hit][:, None]).astype(np.float32)
    o = np.concatenate([o, o2])
    d = np.concatenate([d, d[hit]])
    t1, f1, _ = bvh.query(o, d)
    t2, f2, _ = brute.query(o, d)
    np.testing.assert_array_equal(f1, f2)
    np.testing.assert_array_equal(t1.view(np.uint32), t2.view(np.uint32))
    assert (f2 >= 0).mean() > 0.3
