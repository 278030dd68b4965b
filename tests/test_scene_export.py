"""Scene export (reference viz/visualization.py): the GLB that rf_ray_tracing_warp_amd.scene
writes reproduces the reference artifact web/scene.html (a trimesh export of a main.py run) array
for array -- the TX / RX spheres and the 119 received paths, whose arrays are the golden fixture
tests/golden/scene_html.npz -- and round-trips through the HTML page.  CPU only."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from rf_ray_tracing_warp_amd.mesh import load_stl  # noqa: E402
from rf_ray_tracing_warp_amd.scene import GREEN, RED, Scene, glb_from_html, read_glb, visualize  # noqa: E402


@pytest.fixture(scope="module")
def golden():
    return np.load(os.path.join(HERE, "golden", "scene_html.npz"))


def _acc(js, binb, i):
    a = js["accessors"][i]
    bv = js["bufferViews"][a["bufferView"]]
    dt = {5126: np.float32, 5125: np.uint32, 5121: np.uint8}[a["componentType"]]
    nc = {"SCALAR": 1, "VEC3": 3, "VEC4": 4}[a["type"]]
    o = bv.get("byteOffset", 0) + a.get("byteOffset", 0)
    assert o % 4 == 0
    return np.frombuffer(binb, dtype=dt, count=a["count"] * nc, offset=o).reshape(a["count"], nc)


def _artifact_scene(golden):
    env = load_stl(os.path.join(os.path.dirname(HERE), "models", "almost_empty.stl"))
    sc = Scene().add_mesh(env.vertices, env.faces, name="almost_empty.stl")
    sc.add_sphere(golden["tx"], 0.5, RED).add_sphere(golden["rx"], 0.5, GREEN)  # that run's radius
    for p, n in zip(golden["paths"], golden["lengths"]):
        sc.add_path(p[:n])
    return sc


def test_glb_reproduces_the_artifact_geometry(golden):
    js, binb = read_glb(_artifact_scene(golden).to_glb())
    meshes = js["meshes"]
    assert len(meshes) == 3 + 119
    assert js["nodes"][0]["name"] == "world" and js["nodes"][0]["children"] == list(range(1, len(meshes) + 1))
    tx = meshes[1]["primitives"][0]
    assert tx["mode"] == 4
    np.testing.assert_array_equal(_acc(js, binb, tx["attributes"]["POSITION"]), golden["sphere_v"])
    np.testing.assert_array_equal(_acc(js, binb, tx["indices"]).reshape(-1, 3), golden["sphere_f"])
    np.testing.assert_array_equal(_acc(js, binb, tx["attributes"]["COLOR_0"]), np.tile([255, 0, 0, 255], (642, 1)))
    rx = meshes[2]["primitives"][0]
    np.testing.assert_array_equal(_acc(js, binb, rx["attributes"]["POSITION"]), golden["rx_sphere_v"])
    for m, p, n in zip(meshes[3:], golden["paths"], golden["lengths"]):
        prim = m["primitives"][0]
        assert prim["mode"] == 1 and prim["material"] == 0
        seg = _acc(js, binb, prim["attributes"]["POSITION"])
        pts = p[:n]
        np.testing.assert_array_equal(seg[0::2], pts[:-1])
        np.testing.assert_array_equal(seg[1::2], pts[1:])
    # accessor bounds are what a glTF loader checks
    a = js["accessors"][tx["attributes"]["POSITION"]]
    np.testing.assert_array_equal(a["min"], golden["sphere_v"].min(0).astype(np.float64))
    np.testing.assert_array_equal(a["max"], golden["sphere_v"].max(0).astype(np.float64))


def test_paths_collapse_repeated_points():
    """A receiver self-hit at t=0 repeats a path point; the polyline keeps one copy."""
    p = np.array([[0, 0, 0], [1, 0, 0], [1, 0, 0], [1, 1, 0]], np.float32)
    js, binb = read_glb(Scene().add_path(p).to_glb())
    seg = _acc(js, binb, js["meshes"][0]["primitives"][0]["attributes"]["POSITION"])
    np.testing.assert_array_equal(seg, np.array([[0, 0, 0], [1, 0, 0], [1, 0, 0], [1, 1, 0]], np.float32))


def test_visualize_writes_a_page_that_round_trips(tmp_path, golden):
    env = load_stl(os.path.join(os.path.dirname(HERE), "models", "almost_empty.stl"))
    out = tmp_path / "viz" / "scene.html"
    sc = visualize(env, golden["tx"], golden["rx"], [p[:n] for p, n in zip(golden["paths"], golden["lengths"])],
                   points=np.zeros((5, 3)), point_color_pairs=[((0, 0, 1), (0, 0, 255, 255))], out_path=str(out),
                   serve=False)
    html = out.read_text()
    assert "GLTFLoader" in html
    js, binb = read_glb(glb_from_html(html))
    assert glb_from_html(html) == sc.to_glb()
    # grey mesh, red TX (r 0.25), green RX, white points (mode 0), 119 paths, one blue marker
    modes = [m["primitives"][0]["mode"] for m in js["meshes"]]
    assert modes == [4, 4, 4, 0] + [1] * 119 + [4]
    tx = _acc(js, binb, js["meshes"][1]["primitives"][0]["attributes"]["POSITION"]).astype(np.float64)
    assert abs(np.linalg.norm(tx - golden["tx"], axis=1).max() - 0.25) < 1e-6
    col = _acc(js, binb, js["meshes"][-1]["primitives"][0]["attributes"]["COLOR_0"])
    assert (col == [0, 0, 255, 255]).all()


def test_page_handler_serves_only_the_page(tmp_path):
    """the viewer answers / and /index.html only (viz/visualization.py:43-47), never
    other files of the working directory."""
    import http.client
    import http.server
    import threading

    from rf_ray_tracing_warp_amd.scene import _page_handler
    page = tmp_path / "scene.html"
    page.write_text("<html>scene</html>")
    (tmp_path / "secret.txt").write_text("no")
    httpd = http.server.HTTPServer(("127.0.0.1", 0), _page_handler(str(page)))
    th = threading.Thread(target=httpd.serve_forever, daemon=True)
    th.start()
    try:
        port = httpd.server_address[1]
        got = {}
        for path in ("/", "/index.html", "/secret.txt", "/scene.html", "/../", "/tests/"):
            c = http.client.HTTPConnection("127.0.0.1", port, timeout=10)
            c.request("GET", path)
            r = c.getresponse()
            got[path] = (r.status, r.read())
            c.close()
        assert got["/"] == (200, b"<html>scene</html>") and got["/index.html"] == got["/"]
        for path in ("/secret.txt", "/scene.html", "/../", "/tests/"):
            assert got[path][0] == 404
    finally:
        httpd.shutdown()
        httpd.server_close()
