"""Scene export for inspecting traced paths (reference ``viz/visualization.py``).

The reference builds a trimesh ``Scene`` -- the environment mesh in grey, TX / RX spheres in red /
green, the received paths as polylines, optional point clouds and coloured marker spheres --,
writes it with trimesh's three.js viewer to ``viz/scene.html`` and serves it on port 8000
(``viz/visualization.py:6-50``).  trimesh is not installed here, so this module writes the same
scene itself:

* :class:`Scene` holds the geometries and writes a binary glTF 2.0 file (GLB) laid out as trimesh
  lays out its own: one node per geometry under a ``world`` root; triangle meshes as indexed
  ``mode 4`` primitives with float32 ``POSITION``, uint32 indices and normalised uint8 ``COLOR_0``
  per vertex; paths as ``mode 1`` (line segment pairs) and point clouds as ``mode 0``.  The TX
  sphere and the paths of the reference's own artifact (``web/scene.html``) are reproduced
  array for array (``tests/test_scene_export.py``).
* :func:`scene_to_html` wraps a GLB in a small three.js page (GLTFLoader + OrbitControls loaded
  from a CDN by an import map; the reference inlines its copy of three.js instead).
* :func:`visualize` keeps the reference's signature and behaviour: write ``viz/scene.html``, then
  serve it on port 8000 (``serve=False`` writes the file only).

Presentation only: nothing here touches the GPU path.
"""
from __future__ import annotations

import base64
import json
import os
import struct

import numpy as np

from .mesh import sphere

__all__ = ["Scene", "scene_to_html", "visualize", "read_glb"]

GREY = (100, 100, 100, 255)
RED = (255, 0, 0, 255)
GREEN = (0, 255, 0, 255)
PATH_GREY = (200, 200, 200, 255)
WHITE = (255, 255, 255, 255)


def _rgba(color, n):
    c = np.asarray(color, dtype=np.float64).reshape(-1)
    if c.size == 3:
        c = np.append(c, 255)
    if c.max() <= 1.0 and c.dtype.kind == "f" and np.any(c % 1):  # [0, 1] floats
        c = c * 255.0
    return np.tile(np.clip(np.round(c), 0, 255).astype(np.uint8), (n, 1))


def _dedupe_consecutive(points):
    """Consecutive equal vertices collapse to one (trimesh.load_path merges equal vertices; a
    polyline that revisits a point keeps both visits)."""
    p = np.ascontiguousarray(points, dtype=np.float64).reshape(-1, 3)
    if len(p) < 2:
        return p
    keep = np.ones(len(p), bool)
    keep[1:] = np.any(p[1:] != p[:-1], axis=1)
    return p[keep]


class Scene:
    """Geometries of one visualisation; ``to_glb()`` / ``to_html()`` write it."""

    def __init__(self):
        self._geoms = []  # dicts: name, mode, pos (n,3) f32, idx (m,) u32 or None, col (n,4) u8

    def add_mesh(self, vertices, faces, color=GREY, name=None):
        v = np.ascontiguousarray(vertices, dtype=np.float32).reshape(-1, 3)
        f = np.ascontiguousarray(faces, dtype=np.uint32).reshape(-1)
        self._geoms.append({"name": name or f"geometry_{len(self._geoms)}", "mode": 4, "pos": v, "idx": f,
                            "col": _rgba(color, len(v))})
        return self

    def add_sphere(self, center, radius, color, subdivisions=3, name=None):
        """trimesh.primitives.Sphere(radius, center): the unit icosphere (subdivisions 3) scaled and
        moved in float64 (mesh.sphere), then stored as float32."""
        m = sphere(center, radius, subdivisions)
        return self.add_mesh(m.vertices, m.faces, color, name)

    def add_path(self, points, color=PATH_GREY, name=None):
        """A polyline (trimesh.load_path of an (n, 3) array) as line segments p0-p1, p1-p2, ..."""
        p = _dedupe_consecutive(points)
        if len(p) < 2:
            return self
        seg = np.empty((2 * (len(p) - 1), 3), np.float64)
        seg[0::2] = p[:-1]
        seg[1::2] = p[1:]
        seg = seg.astype(np.float32)
        self._geoms.append({"name": name or f"geometry_{len(self._geoms)}", "mode": 1, "pos": seg, "idx": None,
                            "col": _rgba(color, len(seg))})
        return self

    def add_points(self, points, colors=WHITE, name=None):
        p = np.ascontiguousarray(points, dtype=np.float32).reshape(-1, 3)
        col = np.asarray(colors)
        col = _rgba(colors, len(p)) if col.ndim < 2 else np.asarray(
            [_rgba(c, 1)[0] for c in col], np.uint8).reshape(len(p), 4)
        self._geoms.append({"name": name or f"geometry_{len(self._geoms)}", "mode": 0, "pos": p, "idx": None,
                            "col": col})
        return self

    def __len__(self):
        return len(self._geoms)

    def to_glb(self) -> bytes:
        blob = bytearray()
        views, accessors, meshes, nodes = [], [], [], [{"name": "world", "children": []}]
        line_material = False

        def put(arr, comp, typ, count, minmax=True, normalized=False):
            while len(blob) % 4:
                blob.append(0)
            raw = np.ascontiguousarray(arr).tobytes()
            views.append({"buffer": 0, "byteOffset": len(blob), "byteLength": len(raw)})
            blob.extend(raw)
            acc = {"componentType": comp, "type": typ, "bufferView": len(views) - 1, "count": int(count)}
            if typ != "SCALAR":
                acc["byteOffset"] = 0
            if normalized:
                acc["normalized"] = True
            if minmax and count:
                a = np.asarray(arr).reshape(count, -1)
                acc["max"] = [x.item() for x in a.max(0)]
                acc["min"] = [x.item() for x in a.min(0)]
            accessors.append(acc)
            return len(accessors) - 1

        for g in self._geoms:
            prim = {"attributes": {}, "mode": g["mode"]}
            if g["idx"] is not None:
                prim["indices"] = put(g["idx"], 5125, "SCALAR", len(g["idx"]))
            prim["attributes"]["POSITION"] = put(g["pos"], 5126, "VEC3", len(g["pos"]))
            prim["attributes"]["COLOR_0"] = put(g["col"], 5121, "VEC4", len(g["col"]), normalized=True)
            if g["mode"] != 4:
                prim["material"] = 0
                line_material = True
            meshes.append({"name": g["name"], "primitives": [prim]})
            nodes[0]["children"].append(len(nodes))
            nodes.append({"name": g["name"], "mesh": len(meshes) - 1})
        while len(blob) % 4:
            blob.append(0)
        gltf = {"scene": 0, "scenes": [{"nodes": [0]}],
                "asset": {"version": "2.0", "generator": "rf_ray_tracing_warp_amd.scene"},
                "accessors": accessors, "meshes": meshes, "nodes": nodes,
                "buffers": [{"byteLength": len(blob)}], "bufferViews": views}
        if line_material:
            gltf["materials"] = [{"pbrMetallicRoughness": {"baseColorFactor": [1, 1, 1, 1], "metallicFactor": 0,
                                                            "roughnessFactor": 0}}]
        js = json.dumps(gltf, separators=(",", ":")).encode()
        js += b" " * (-len(js) % 4)
        total = 12 + 8 + len(js) + 8 + len(blob)
        return b"".join([struct.pack("<4sII", b"glTF", 2, total), struct.pack("<I4s", len(js), b"JSON"), js,
                         struct.pack("<I4s", len(blob), b"BIN\x00"), bytes(blob)])

    def to_html(self) -> str:
        return scene_to_html(self.to_glb())


def read_glb(data: bytes):
    """(gltf JSON dict, binary chunk) of a GLB; accessor(i) helpers are left to the caller."""
    magic, version, total = struct.unpack("<4sII", data[:12])
    if magic != b"glTF" or version != 2 or total != len(data):
        raise ValueError("not a glTF 2.0 binary")
    off, chunks = 12, []
    while off < len(data):
        clen, _ = struct.unpack("<I4s", data[off:off + 8])
        chunks.append(data[off + 8:off + 8 + clen])
        off += 8 + clen
    return json.loads(chunks[0]), chunks[1] if len(chunks) > 1 else b""


_HTML = """<!DOCTYPE html>
<html>
<head>
<meta charset="utf-8">
<title>rf_ray_tracing_warp_amd scene</title>
<style>html, body {{ margin: 0; height: 100%; overflow: hidden; background: #202020; }}</style>
<script type="importmap">
{{"imports": {{"three": "https://unpkg.com/three@0.160.0/build/three.module.js",
  "three/addons/": "https://unpkg.com/three@0.160.0/examples/jsm/"}}}}
</script>
</head>
<body>
<div id="scene-glb" data-glb="{glb}"></div>
<script type="module">
import * as THREE from "three";
import {{ GLTFLoader }} from "three/addons/loaders/GLTFLoader.js";
import {{ OrbitControls }} from "three/addons/controls/OrbitControls.js";
const b64 = document.getElementById("scene-glb").dataset.glb;
const bytes = Uint8Array.from(atob(b64), c => c.charCodeAt(0));
const renderer = new THREE.WebGLRenderer({{ antialias: true }});
renderer.setSize(window.innerWidth, window.innerHeight);
document.body.appendChild(renderer.domElement);
const scene = new THREE.Scene();
scene.add(new THREE.AmbientLight(0xffffff, 0.6));
const sun = new THREE.DirectionalLight(0xffffff, 0.8);
sun.position.set(1, 2, 3);
scene.add(sun);
const camera = new THREE.PerspectiveCamera(60, window.innerWidth / window.innerHeight, 0.01, 1e5);
const controls = new OrbitControls(camera, renderer.domElement);
new GLTFLoader().parse(bytes.buffer, "", gltf => {{
  scene.add(gltf.scene);
  const box = new THREE.Box3().setFromObject(gltf.scene);
  const c = box.getCenter(new THREE.Vector3()), r = box.getSize(new THREE.Vector3()).length() || 1;
  camera.position.set(c.x + r, c.y + r, c.z + r);
  controls.target.copy(c);
  controls.update();
}});
window.addEventListener("resize", () => {{
  camera.aspect = window.innerWidth / window.innerHeight;
  camera.updateProjectionMatrix();
  renderer.setSize(window.innerWidth, window.innerHeight);
}});
(function loop() {{ requestAnimationFrame(loop); renderer.render(scene, camera); }})();
</script>
</body>
</html>
"""


def scene_to_html(glb: bytes) -> str:
    """A standalone page showing the GLB (base64 in the ``data-glb`` attribute of ``#scene-glb``)."""
    return _HTML.format(glb=base64.b64encode(glb).decode("ascii"))


def glb_from_html(html: str) -> bytes:
    i = html.index('data-glb="') + len('data-glb="')
    return base64.b64decode(html[i:html.index('"', i)])


def visualize(mesh=None, tx_pos=None, rx_pos=None, paths=None, points=None, point_color_pairs=None,
              out_path="viz/scene.html", serve=True, port=8000, host="127.0.0.1"):
    """viz/visualization.py:6-50: the scene of a trace as ``viz/scene.html``, then an HTTP server on
    ``host:port`` answering ``/`` and ``/index.html`` with it and 404 for everything else (blocks,
    as the reference does).  host defaults to the loopback interface; pass "" for all interfaces."""
    sc = Scene()
    if mesh is not None:
        sc.add_mesh(mesh.vertices, mesh.faces, GREY, name=getattr(mesh, "name", None))
    if tx_pos is not None:
        sc.add_sphere(tx_pos, 0.25, RED)
    if rx_pos is not None:
        sc.add_sphere(rx_pos, 0.25, GREEN)
    if points is not None:
        sc.add_points(points, WHITE)
    if paths is not None:
        print(f"Adding {len(paths)} paths to the scene...")
        for path in paths:
            sc.add_path(path, PATH_GREY)
    if point_color_pairs is not None:
        for point, color in point_color_pairs:
            sc.add_sphere(point, 0.1, color)
    d = os.path.dirname(out_path)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(out_path, "w") as f:
        f.write(sc.to_html())
    if serve:
        import http.server

        httpd = http.server.HTTPServer((host, port), _page_handler(out_path))
        print(f"Serving visualization at {host or 'localhost'}:{port}")
        httpd.serve_forever()
    return sc


def _page_handler(out_path):
    """HTTP handler that answers only / and /index.html, with the page at out_path (the
    reference's handler, viz/visualization.py:43-47, serves nothing else either); every other path
    is a 404, so the working directory is never listed or served."""
    import http.server

    class Handler(http.server.BaseHTTPRequestHandler):
        def do_GET(self):
            if self.path not in ("/", "/index.html"):
                self.send_error(404)
                return
            with open(out_path, "rb") as f:
                body = f.read()
            self.send_response(200)
            self.send_header("Content-Type", "text/html; charset=utf-8")
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def log_message(self, *args):
            pass

    return Handler
