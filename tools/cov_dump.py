"""Dump one coverage map (power, sparse impulse responses) to gpurun_out/<tag>.npz for offline
comparison of two library variants:  RFRT_LIB_PATH=... python tools/cov_dump.py k3|k5 <tag>"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(case, tag):
    from rf_ray_tracing_warp_amd.coverage import Coverage, CoverageGrid
    from rf_ray_tracing_warp_amd.mesh import load_stl, synthetic_terrain
    if case == "k3":
        m = load_stl(os.path.join(ROOT, "models/room.stl"))
        grid, tx, win = CoverageGrid.square(256, 15.0, 5.0), (10.0, 0.0, 5.0), 100e-9
    else:
        m = synthetic_terrain(1024, 50.0)
        grid, tx, win = CoverageGrid.square(1024, 50.0, 2.0), (10.0, 0.0, 4.5), 200e-9
    cov = Coverage(m, 2.998e8, 100e9, win, 3, 1_000_000, grid, 0.1, device=0)
    p = cov.run(tx, 1).reshape(-1)
    c, b, a = cov.impulse_responses()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"{tag}.npz"), power=p, cells=c, bins=b, amps=a)
    print(tag, int(np.isfinite(p).sum()), len(c))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
