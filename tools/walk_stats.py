"""BVH walk statistics of the K4 burst (terrain stand-in, 2,097,152 rays, B=5) from a diagnostic
library built with RT_COUNT_STEPS=1:

    python tools/build_variants.py steps="-DRT_COUNT_STEPS=1"
    RFRT_LIB_PATH=tools/_var/lib_steps.so python tools/walk_stats.py

Prints one JSON line: queries, walk steps per query (mean, max), wave loop iterations, and the
SIMD utilisation of the walk loop (lane steps / (64 x wave iterations)).  Counting adds atomics
per query, so the line carries no time."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from rf_ray_tracing_warp_amd._lib import DeviceMesh, check, lib, ptr
    from rf_ray_tracing_warp_amd.mesh import sphere, synthetic_terrain
    n, B = 2_097_152, 5
    m = synthetic_terrain(1024, 50.0)
    env = DeviceMesh(m.vertices, m.faces, 0)
    rs = sphere((-10.125, 0.0, 4.8), 0.1, 1)
    rx = DeviceMesh(rs.vertices, rs.faces, 0)
    mk = torch.empty(n, dtype=torch.int32, device="cuda")
    tx = np.asarray((10.0, 0.0, 4.5), np.float32)
    st = torch.cuda.current_stream()
    L = lib()
    f = L.rt_debug_walk_stats
    f.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int]
    out = (ctypes.c_double * 4)()
    res = {"lib": os.path.basename(os.environ.get("RFRT_LIB_PATH", "librfrt.so")), "case": "k4", "rays": n, "B": B}
    for name, (t, r) in (("mask", (None, None)),):
        check(L.rt_trace(env.handle, tx.ctypes.data, rx.handle, B, 0, n, ptr(t), ptr(r), ptr(mk), None, None,
                         st.cuda_stream), "rt_trace")
        torch.cuda.synchronize()
        check(f(out, 1), "walk stats")  # reset after the warm-up launch
        check(L.rt_trace(env.handle, tx.ctypes.data, rx.handle, B, 0, n, ptr(t), ptr(r), ptr(mk), None, None,
                         st.cuda_stream), "rt_trace")
        torch.cuda.synchronize()
        check(f(out, 1), "walk stats")
        steps, iters, q, mx = list(out)
        res.update({"queries": q, "steps_per_query": steps / q, "max_steps": mx,
                    "wave_iterations": iters, "simd_utilisation": steps / (64.0 * iters)})
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
