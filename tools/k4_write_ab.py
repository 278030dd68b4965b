"""K4 write-traffic A/B: rt_trace on the K4 burst (terrain stand-in, 2,097,152
rays, B=5, main.py:22-23) three times per output set, in this order: traced + received + row_mask,
received + row_mask, row_mask only.  Under `rocprofv3 --pmc WRITE_SIZE --kernel-trace` the
k_trace_bvh<5> dispatches then split the kernel's written bytes into row stores and the rest (the
walk stack's scratch write-back).  RFRT_LIB_PATH selects a variant library.  Prints one JSON line
with the HIP-event time per set."""
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
    tr = torch.empty((n, B + 1, 3), dtype=torch.float32, device="cuda")
    rc = torch.empty_like(tr)
    mk = torch.empty(n, dtype=torch.int32, device="cuda")
    tx = np.asarray((10.0, 0.0, 4.5), np.float32)
    st = torch.cuda.current_stream()
    L = lib()
    out = {"lib": os.path.basename(os.environ.get("RFRT_LIB_PATH", "librfrt.so")), "us": {}}
    for name, t, r in (("traced+received+mask", tr, rc), ("received+mask", None, rc), ("mask", None, None)):
        def go():
            check(L.rt_trace(env.handle, tx.ctypes.data, rx.handle, B, 0, n, ptr(t), ptr(r), ptr(mk), None, None,
                             st.cuda_stream), "rt_trace")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(3):
            go()
        e1.record(st)
        torch.cuda.synchronize()
        out["us"][name] = e0.elapsed_time(e1) * 1e3 / 3
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
