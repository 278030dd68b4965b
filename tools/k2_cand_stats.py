"""Candidate faces per wave and bounce on the K2 burst, from a diagnostics build of trace.hip
(RT_DIAG_CAND=1: hit_face holds the wave's candidate count | rx_wave << 8 | alive << 9).

    RFRT_BUILD_DIR=/tmp/diag RFRT_LIB_OUT=rf_ray_tracing_warp_amd/_diag.so \\
        RFRT_EXTRA_CFLAGS=-DRT_DIAG_CAND=1 python -m rf_ray_tracing_warp_amd.build
    RFRT_LIB_PATH=rf_ray_tracing_warp_amd/_diag.so python tools/k2_cand_stats.py     (GPU)
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from rf_ray_tracing_warp_amd._lib import DeviceMesh, check, lib, ptr
    from rf_ray_tracing_warp_amd.mesh import load_stl, sphere
    n, B = 1_000_000, 3
    m = load_stl(os.path.join(ROOT, "models/room.stl"))
    env = DeviceMesh(m.vertices, m.faces, 0)
    rs = sphere((-10.0, 0.0, 5.0), 0.1, 1)
    rx = DeviceMesh(rs.vertices, rs.faces, 0)
    tr = torch.empty((n, B + 1, 3), dtype=torch.float32, device="cuda")
    hk = torch.empty((n, B), dtype=torch.int32, device="cuda")
    hf = torch.empty((n, B), dtype=torch.int32, device="cuda")
    tx = np.asarray((10.0, 0.0, 5.0), np.float32)
    check(lib().rt_trace(env.handle, tx.ctypes.data, rx.handle, B, 0, n, ptr(tr), None, None, ptr(hk), ptr(hf),
                         torch.cuda.current_stream().cuda_stream), "rt_trace")
    torch.cuda.synchronize()
    d = hf.cpu().numpy()
    out = {}
    for b in range(B):
        c, rxw, alive = d[:, b] & 255, (d[:, b] >> 8) & 1, (d[:, b] >> 9) & 1
        out[f"bounce{b}"] = {"cand_mean_per_ray": float(c.mean()), "cand_p50": float(np.median(c)),
                             "cand_p90": float(np.percentile(c, 90)), "cand_max": int(c.max()),
                             "rx_wave_frac": float(rxw.mean()), "alive_frac": float(alive.mean()),
                             "hist": np.bincount(c, minlength=45)[:45].tolist()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
