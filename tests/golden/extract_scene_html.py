"""Extract golden vectors from the reference artifact web/scene.html (run in the dev container only).

scene.html (reference web/scene.html:1242) embeds a trimesh GLB of an older run of main.py on
models/almost_empty.stl: TX and RX visualisation spheres (trimesh icosphere, subdivisions=3,
radius 0.5) and the 119 received paths returned by Tracer.compute_cir.  This script stores them
as plain arrays (data, not source) in tests/golden/scene_html.npz:

  tx, rx              sphere centres (means of the two 642-vertex meshes)
  sphere_v, sphere_f  the TX sphere's f32 vertices (642,3) and faces (1280,3), as exported
  rx_sphere_v         the RX sphere's f32 vertices
  paths               (119, 4, 3) f32, NaN padded; lengths (119,)
  ray_ids             the ray ids whose generated direction matches each path's first segment
                      (found by scanning ids 0..2^28 with the PCG restatement)

Usage: python tests/golden/extract_scene_html.py [path/to/scene.html]
"""
import base64
import json
import os
import re
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def glb_from_html(path):
    s = open(path).read()
    b = base64.b64decode(re.search(r'base64_data="([A-Za-z0-9+/=]+)"', s).group(1))
    off, chunks = 12, []
    while off < len(b):
        clen, ctype = struct.unpack("<II", b[off:off + 8])
        chunks.append(b[off + 8:off + 8 + clen])
        off += 8 + clen
    return json.loads(chunks[0]), chunks[1]


def main(path):
    js, binb = glb_from_html(path)

    def acc(i):
        a = js["accessors"][i]
        bv = js["bufferViews"][a["bufferView"]]
        dt = {5126: np.float32, 5125: np.uint32}[a["componentType"]]
        nc = {"SCALAR": 1, "VEC3": 3}[a["type"]]
        o = bv.get("byteOffset", 0) + a.get("byteOffset", 0)
        return np.frombuffer(binb, dtype=dt, count=a["count"] * nc, offset=o).reshape(a["count"], nc).copy()

    meshes = js["meshes"]
    tx_v = acc(meshes[1]["primitives"][0]["attributes"]["POSITION"])
    tx_f = acc(meshes[1]["primitives"][0]["indices"]).reshape(-1, 3)
    rx_v = acc(meshes[2]["primitives"][0]["attributes"]["POSITION"])
    paths, lengths = [], []
    for m in meshes[3:]:
        seg = acc(m["primitives"][0]["attributes"]["POSITION"])  # GL_LINES: point pairs
        pts = np.array([seg[0]] + [seg[i] for i in range(1, len(seg), 2)], np.float32)
        lengths.append(len(pts))
        paths.append(np.pad(pts, ((0, 4 - len(pts)), (0, 0)), constant_values=np.nan))
    paths = np.array(paths, np.float32)
    tx = np.round(tx_v.astype(np.float64).mean(0), 4)
    rx = np.round(rx_v.astype(np.float64).mean(0), 4)

    # find the ray id of every path with the PCG/sphere-sampling restatement (oracle)
    sys.path.insert(0, os.path.join(HERE, "..", ".."))
    from oracle import oracle as orc
    axis = (rx - tx) / np.linalg.norm(rx - tx)
    ids, dirs = [], []
    step = 1 << 22
    for start in range(0, 1 << 27, step):
        d = orc.ray_dirs(start, step).astype(np.float64)
        d /= np.linalg.norm(d, axis=1)[:, None]  # f32 norm error ~1e-7 ~ 1-cos(3e-4)
        sel = np.nonzero(d @ axis > np.cos(0.004))[0]
        ids.extend(start + sel)
        dirs.extend(d[sel])
    ids, dirs = np.array(ids), np.array(dirs)
    ray_ids = []
    for p in paths:
        u = (p[1] - p[0]).astype(np.float64)
        u /= np.linalg.norm(u)
        ray_ids.append(int(ids[np.argmax(dirs @ u)]))
    np.savez_compressed(os.path.join(HERE, "scene_html.npz"), tx=tx, rx=rx, sphere_v=tx_v, sphere_f=tx_f,
                        rx_sphere_v=rx_v, paths=paths, lengths=np.array(lengths), ray_ids=np.array(ray_ids),
                        cone_ids=ids)
    print("stored", len(paths), "paths; ray ids", min(ray_ids), "..", max(ray_ids), "; cone candidates", len(ids))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/web/scene.html")
