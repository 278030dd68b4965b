"""Diagnostic: BVH traversal steps per ray-bounce of the K5 trajectory pass on the terrain stand-in
(sequential per-lane traversal vs a simulated G-wide group traversal), and the per-wave maximum
in direction-sorted order -- what bounds a latency-bound traversal kernel.  GPU box only."""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from rf_ray_tracing_warp_amd import _lib
    from rf_ray_tracing_warp_amd._lib import DeviceMesh, lib, ptr
    from rf_ray_tracing_warp_amd.mesh import synthetic_terrain
    so = os.path.join(ROOT, "tools", "libbvh_steps.so")
    if not os.path.exists(so):
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-fPIC", "-shared", "--offload-arch=gfx950",
                               "-ffp-contract=off", "-o", so, os.path.join(ROOT, "tools", "bvh_steps.hip")])
    T = ctypes.CDLL(so)
    t = synthetic_terrain(1024, 50.0)
    env = DeviceMesh(t.vertices, t.faces, 0, builder=os.environ.get("BUILDER", "sah"))
    print(json.dumps({"bvh": env.bvh_info()}), flush=True)
    N, B = int(os.environ.get("N", "125000")), 3
    tx = np.asarray((10.0, 0.0, 4.5), np.float32)
    dirs = torch.empty((N, 3), dtype=torch.float32, device="cuda")
    lib().rt_ray_dirs(0, N, ptr(dirs), None)
    d = dirs.cpu().numpy()
    for G in [int(g) for g in os.environ.get("GS", "8").split(",")]:
        its = torch.empty(N * B, dtype=torch.int32, device="cuda")
        lvs = torch.empty(N * B, dtype=torch.int32, device="cuda")
        itg = torch.empty(N * B, dtype=torch.int32, device="cuda")
        mm = torch.zeros(1, dtype=torch.int32, device="cuda")
        T.bvh_steps(env.handle, ctypes.c_void_p(tx.ctypes.data), ctypes.c_int64(0), ctypes.c_int64(N), B, G,
                    ctypes.c_void_p(ptr(its)), ctypes.c_void_p(ptr(lvs)), ctypes.c_void_p(ptr(itg)),
                    ctypes.c_void_p(ptr(mm)))
        a = its.cpu().numpy().reshape(N, B)
        lv = lvs.cpu().numpy().reshape(N, B)
        g = itg.cpu().numpy().reshape(N, B)
        # per-ray serial chain = sum over bounces; direction-sorted order (octahedral 256^2 cell)
        sa = np.where(a < 0, 0, a).sum(1)
        sg = np.where(g < 0, 0, g).sum(1)
        x, y, z = d[:, 0], d[:, 1], d[:, 2]
        s = np.abs(x) + np.abs(y) + np.abs(z)
        u, v = x / s, y / s
        neg = z < 0
        u2 = np.where(neg, (1 - np.abs(v)) * np.sign(u), u)
        v2 = np.where(neg, (1 - np.abs(u)) * np.sign(v), v)
        key = (np.clip(((v2 + 1) * 128).astype(int), 0, 255) * 256 + np.clip(((u2 + 1) * 128).astype(int), 0, 255))
        o = np.argsort(key, kind="stable")
        nw = N // 64
        wmax = sa[o][:nw * 64].reshape(nw, 64).max(1)
        wmaxg = sg[o][:nw * 64].reshape(nw, 64).max(1)

        def pct(v):
            return {p: int(np.percentile(v, p)) for p in (50, 90, 99, 99.9)} | {"max": int(v.max()), "mean": float(v.mean())}
        print(json.dumps({"G": G, "mismatch": int(mm.item()),
                          "per_bounce_seq_mean": [float(np.mean(a[:, k][a[:, k] >= 0])) for k in range(B)],
                          "per_bounce_leaves_mean": [float(np.mean(lv[:, k][lv[:, k] >= 0])) for k in range(B)],
                          "ray_seq": pct(sa), "ray_grp": pct(sg), "wave_max_seq": pct(wmax), "wave_max_grp": pct(wmaxg),
                          "total_seq": int(sa.sum()), "total_grp_iters": int(sg.sum())}), flush=True)
        if G == 8:
            T.bvh_time.restype = ctypes.c_float
            out = torch.empty(1_000_000, dtype=torch.float32, device="cuda")
            of = torch.empty(1_000_000, dtype=torch.int32, device="cuda")
            worst = int(np.argmax(wmax))
            sets = {"sorted125k": o, "worst_wave": o[worst * 64:(worst + 1) * 64], "unsorted1M": np.arange(1_000_000)}
            ref = {}
            for mode, block in [(0, 256), (1, 256), (2, 256), (3, 256), (3, 64), (2, 64)]:
                res = {"mode": mode, "block": block}
                for name, ids in sets.items():
                    idt = torch.from_numpy(np.ascontiguousarray(ids, dtype=np.int64)).cuda()
                    ms = float(T.bvh_time(env.handle, ctypes.c_void_p(tx.ctypes.data), ctypes.c_void_p(ptr(idt)),
                                          ctypes.c_int64(len(ids)), B, 5, mode, block, ctypes.c_void_p(ptr(out)),
                                          ctypes.c_void_p(ptr(of))))
                    chk = (out[:len(ids)].cpu().numpy().copy(), of[:len(ids)].cpu().numpy().copy())
                    if mode == 0 and block == 256:
                        ref[name] = chk
                    res[name + "_ms"] = round(ms, 4)
                    res[name + "_same"] = bool(np.array_equal(chk[0], ref[name][0]) and np.array_equal(chk[1], ref[name][1]))
                print(json.dumps(res), flush=True)

if __name__ == "__main__":
    main()
