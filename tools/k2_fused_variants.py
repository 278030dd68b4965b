"""K2 step time per library (LIBS="a.so b.so ...", one child process each, RFRT_LIB_PATH): the
rt_trace_cir step and the bare rt_trace launch, HIP events over REPS back-to-back calls after a
clock-settling run, plus a hash of the step's outputs (index list, count, impulse response).
GPU box only.

    LIBS="rf_ray_tracing_warp_amd/librfrt.so tools/_libs/x.so" python tools/k2_fused_variants.py
"""
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(reps):
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch
    from rf_ray_tracing_warp_amd._lib import DeviceMesh, check, lib, ptr
    from rf_ray_tracing_warp_amd.mesh import load_stl, sphere
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
    st = torch.cuda.current_stream().cuda_stream

    def step():
        check(L.rt_trace_cir(env.handle, tx.ctypes.data, rx.handle, B, 0, N, ptr(tr), ptr(rc), ptr(mk), 1e-6,
                             2.998e8, 1e9, 0, 10000, ptr(ir), ptr(idx), ptr(cnt), ptr(ws), ws.numel(), st),
              "rt_trace_cir")

    def trace():
        check(L.rt_trace(env.handle, tx.ctypes.data, rx.handle, B, 0, N, ptr(tr), ptr(rc), ptr(mk), None, None, st),
              "rt_trace")

    out = {"lib": os.path.basename(os.environ.get("RFRT_LIB_PATH", "librfrt.so"))}
    for name, fn in (("step_us", step), ("trace_us", trace), ("step_us_2", step)):
        for _ in range(250):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[name] = e0.elapsed_time(e1) * 1e3 / reps
    step()
    torch.cuda.synchronize()
    c = int(cnt.item())
    h = hashlib.sha256(idx[:c].cpu().numpy().tobytes() + ir.cpu().numpy().tobytes()).hexdigest()
    out.update(count=c, hash=h[:16])
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        child(int(sys.argv[2]))
        sys.exit(0)
    reps = int(os.environ.get("REPS", "400"))
    for so in os.environ["LIBS"].split():
        env = dict(os.environ, RFRT_LIB_PATH=os.path.abspath(so))
        r = subprocess.run([sys.executable, __file__, "child", str(reps)], env=env, timeout=300)
        if r.returncode != 0:
            sys.exit(r.returncode)
