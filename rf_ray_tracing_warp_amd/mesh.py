"""Mesh I/O and the receiver icosphere.

The reference gets both from trimesh (``tm.load_mesh``, ``main.py:21``; ``tm.primitives.Sphere``,
``tracer.py:27``).  trimesh is not installed on this image, so both are restated here:

* :func:`load_stl` reads binary and ASCII STL.  Vertices are merged (exact float equality),
  faces keep STL order, which is what ``Tracer.__init__`` uploads (``tracer.py:22-23``).
* :func:`icosphere` / :func:`sphere` restate ``trimesh.creation.icosphere`` and
  ``trimesh.primitives.Sphere``.  Their f32 vertices and face order are pinned bit-exactly by
  the two 642-vertex spheres embedded in the reference artifact ``web/scene.html``
  (``tests/golden/scene_html.npz``, test ``test_icosphere_matches_artifact``).

Any object with ``.vertices`` (V,3) and ``.faces`` (F,3) is accepted by :class:`Tracer`
(``tracer.py:22-23``), so a real ``trimesh.Trimesh`` works unchanged.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass

import numpy as np

__all__ = ["TriMesh", "load_stl", "load_mesh", "icosahedron", "icosphere", "sphere", "synthetic_terrain"]


@dataclass
class TriMesh:
    """Minimal stand-in for ``trimesh.Trimesh``: float64 vertices, int64 faces."""

    vertices: np.ndarray
    faces: np.ndarray

    def __post_init__(self):
        self.vertices = np.ascontiguousarray(self.vertices, dtype=np.float64).reshape(-1, 3)
        self.faces = np.ascontiguousarray(self.faces, dtype=np.int64).reshape(-1, 3)

    @property
    def triangles(self) -> np.ndarray:
        return self.vertices[self.faces]

    @property
    def bounds(self) -> np.ndarray:
        return np.stack([self.vertices.min(0), self.vertices.max(0)])


def _merge(tri: np.ndarray) -> TriMesh:
    """Merge exactly-equal corner positions; faces keep triangle order."""
    flat = np.ascontiguousarray(tri.reshape(-1, 3), dtype=np.float32)
    uniq, first, inverse = np.unique(flat.view(np.dtype((np.void, 12))).ravel(),
                                     return_index=True, return_inverse=True)
    # number vertices by first appearance (stable, like trimesh's merge on a fresh load)
    order = np.argsort(first, kind="stable")
    rank = np.empty_like(order)
    rank[order] = np.arange(len(order))
    verts = flat[first[order]].astype(np.float64)
    faces = rank[inverse.ravel()].reshape(-1, 3)
    return TriMesh(verts, faces)


def load_stl(path) -> TriMesh:
    """Load a binary or ASCII STL file."""
    with open(path, "rb") as fh:
        data = fh.read()
    if len(data) >= 84:
        (n,) = struct.unpack("<I", data[80:84])
        if 84 + 50 * n == len(data):
            rec = np.frombuffer(data[84:84 + 50 * n],
                                dtype=np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")]))
            return _merge(np.asarray(rec["v"]))
    text = data.decode("ascii", errors="replace")
    if "facet" not in text:
        raise ValueError(f"{path}: not a binary or ASCII STL file")
    verts = []
    for line in text.splitlines():
        parts = line.split()
        if len(parts) == 4 and parts[0] == "vertex":
            verts.append([float(x) for x in parts[1:]])
    if len(verts) % 3:
        raise ValueError(f"{path}: ASCII STL with {len(verts)} vertices (not a multiple of 3)")
    return _merge(np.asarray(verts, dtype=np.float32).reshape(-1, 3, 3))


def load_mesh(path) -> TriMesh:
    """``tm.load_mesh`` stand-in (``main.py:21``); STL only."""
    return load_stl(path)


def icosahedron():
    """Unit icosahedron, vertex and face order as trimesh.creation.icosahedron."""
    t = (1.0 + 5.0 ** 0.5) / 2.0
    v = np.array([-1, t, 0, 1, t, 0, -1, -t, 0, 1, -t, 0, 0, -1, t, 0, 1, t,
                  0, -1, -t, 0, 1, -t, t, 0, -1, t, 0, 1, -t, 0, -1, -t, 0, 1],
                 dtype=np.float64).reshape(-1, 3)
    f = np.array([0, 11, 5, 0, 5, 1, 0, 1, 7, 0, 7, 10, 0, 10, 11,
                  1, 5, 9, 5, 11, 4, 11, 10, 2, 10, 7, 6, 7, 1, 8,
                  3, 9, 4, 3, 4, 2, 3, 2, 6, 3, 6, 8, 3, 8, 9,
                  4, 9, 5, 2, 4, 11, 6, 2, 10, 8, 6, 7, 9, 8, 1], dtype=np.int64).reshape(-1, 3)
    return v / np.sqrt(2.0 + t), f


def _subdivide(v: np.ndarray, f: np.ndarray):
    """One midpoint subdivision with trimesh.remesh.subdivide's vertex/face ordering."""
    edges = np.sort(f[:, [0, 1, 1, 2, 2, 0]].reshape(-1, 2), axis=1)
    key = edges[:, 0].astype(np.int64) | (edges[:, 1].astype(np.int64) << 32)
    _, unique, inverse = np.unique(key, return_index=True, return_inverse=True)
    mid = v[edges[unique]].mean(axis=1)
    mid_idx = inverse.reshape(-1, 3) + len(v)
    nf = np.column_stack([f[:, 0], mid_idx[:, 0], mid_idx[:, 2],
                          mid_idx[:, 0], f[:, 1], mid_idx[:, 1],
                          mid_idx[:, 2], mid_idx[:, 1], f[:, 2],
                          mid_idx[:, 0], mid_idx[:, 1], mid_idx[:, 2]]).reshape(-1, 3)
    faces = np.vstack((f, nf[len(f):]))
    faces[: len(f)] = nf[: len(f)]
    return np.vstack((v, mid)), faces


def icosphere(subdivisions: int = 3, radius: float = 1.0):
    """(vertices float64, faces int64) of trimesh.creation.icosphere."""
    v, f = icosahedron()
    for _ in range(subdivisions):
        v, f = _subdivide(v, f)
        scalar = np.sqrt(np.dot(v ** 2, [1, 1, 1]))
        unit = v / scalar.reshape(-1, 1)
        v = v + unit * (radius - scalar).reshape(-1, 1)
    return v, f


def sphere(center, radius: float, subdivisions: int = 1) -> TriMesh:
    """``tm.primitives.Sphere(center=, radius=, subdivisions=)`` (``tracer.py:27``)."""
    v, f = icosphere(subdivisions)
    return TriMesh(v * float(radius) + np.asarray(center, dtype=np.float64), f)


def synthetic_terrain(n: int = 1024, half_extent: float = 50.0, seed: int = 17, craters: int = 80) -> TriMesh:
    """Declared stand-in for models/apollo_17_landing_site.stl (absent: .MISSING_LARGE_BLOBS:1).

    An n x n vertex heightfield over [-h, h]^2 (2*(n-1)^2 triangles; n=1024 -> 2.09M)
    with gentle undulation and seeded bowl craters with raised rims, heights within about
    [-2, 1] m so the reference scene's TX (10, 0, 4.5) and RX (-10.125, 0, 4.8) (main.py:22-23) sit
    above the ground.  Deterministic for a given (n, half_extent, seed, craters) on one machine.
    """
    rng = np.random.default_rng(seed)
    xs = np.linspace(-half_extent, half_extent, n)
    X, Y = np.meshgrid(xs, xs, indexing="xy")
    Z = 0.25 * np.sin(0.13 * X) * np.cos(0.11 * Y) + 0.15 * np.sin(0.05 * (X + Y))
    cx = rng.uniform(-half_extent, half_extent, craters)
    cy = rng.uniform(-half_extent, half_extent, craters)
    cr = rng.uniform(1.0, 8.0, craters)
    for x0, y0, r in zip(cx, cy, cr):
        d2 = ((X - x0) ** 2 + (Y - y0) ** 2) / (r * r)
        depth = 0.25 * r / 8.0 * 2.0
        Z -= depth * np.clip(1.0 - d2, 0.0, None)
        Z += 0.15 * depth * np.exp(-((np.sqrt(d2) - 1.0) / 0.3) ** 2)
    verts = np.stack([X.ravel(), Y.ravel(), Z.ravel()], axis=1)
    i = np.arange(n - 1)
    a = (i[None, :] + n * i[:, None]).ravel()  # lower-left corner of each quad
    b, c, d = a + 1, a + n, a + n + 1
    faces = np.empty((2 * len(a), 3), dtype=np.int64)
    faces[0::2] = np.stack([a, b, d], axis=1)
    faces[1::2] = np.stack([a, d, c], axis=1)
    return TriMesh(verts, faces)
