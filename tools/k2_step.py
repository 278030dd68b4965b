"""K2 step wall time (rt_trace_cir, 1M rays, room.stl) with the library's trace profiling off and
on (dispatch-packet events), to see what the measurement itself costs.  GPU box only."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from rf_ray_tracing_warp_amd._lib import DeviceMesh, check, lib, ptr
    from rf_ray_tracing_warp_amd.mesh import load_stl, sphere
    from rf_ray_tracing_warp_amd.tracer import cir_flags
    room = load_stl(os.path.join(ROOT, "models", "room.stl"))
    env = DeviceMesh(room.vertices, room.faces, 0)
    m = sphere((-10.0, 0.0, 5.0), 0.1, 1)
    rx = DeviceMesh(m.vertices, m.faces, 0)
    N, B, P = 1_000_000, 3, 4
    tx = np.asarray((10.0, 0.0, 5.0), np.float32)
    tr = torch.empty((N, P, 3), dtype=torch.float32, device="cuda")
    rc = torch.empty_like(tr)
    mk = torch.empty(N, dtype=torch.int32, device="cuda")
    idx = torch.empty(N, dtype=torch.int64, device="cuda")
    cnt = torch.empty(1, dtype=torch.int64, device="cuda")
    ir = torch.empty(10000, dtype=torch.float64, device="cuda")
    L = lib()
    ws = torch.zeros(int(L.rt_trace_cir_workspace_bytes(N)), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream

    def step():
        check(L.rt_trace_cir(env.handle, tx.ctypes.data, rx.handle, B, 0, N, ptr(tr), ptr(rc), ptr(mk), 1e-6, 2.998e8,
                             100e9, cir_flags(2.998e8, 100e9), 10000, ptr(ir), ptr(idx), ptr(cnt), ptr(ws), ws.numel(),
                             s), "rt_trace_cir")
    for _ in range(250):  # settle the clock
        step()
    torch.cuda.synchronize()
    for prof in (0, 1, 8, 0, 1, 8):
        for _ in range(5):
            step()
        torch.cuda.synchronize()
        L.rt_profile(prof)
        t0 = time.perf_counter()
        for _ in range(200):
            step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 200
        st = np.zeros(4)
        L.rt_trace_profile_stats(st.ctypes.data, 4)
        L.rt_profile(0)
        print(f"profile={prof}: {dt * 1e6:.1f} us/step, {int(st[0]) if prof else 0} launches timed, "
              f"kernel {st[1] * 1e3 if prof else float('nan'):.1f} us", flush=True)


if __name__ == "__main__":
    main()
