"""Child process of tests/test_gpu_switches.py: the library's A/B switches are read once per
process (RFRT_K2_BOX, RFRT_K2_LPT, RFRT_TRAJ_SPLIT_MAX), so their non-default paths run here, in a
process started with them set, and must give the default paths' bits: a direction-sorted
brute-force burst against the oracle (every row), traced twice (the second launch would take a
chunk schedule), and a rank plan of a ray-sharded terrain map against the whole map."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    from oracle import oracle as orc
    from rf_ray_tracing_warp_amd._lib import DeviceMesh, check, lib, ptr
    from rf_ray_tracing_warp_amd.coverage import Coverage, CoverageGrid
    from rf_ray_tracing_warp_amd.mesh import load_stl, sphere, synthetic_terrain

    room = load_stl(os.path.join(REPO, "models", "room.stl"))
    n, B, tx, rx, off = 100_000, 3, (10.0, 0.0, 5.0), (6.0, 1.0, 5.0), 7
    rxm = sphere(rx, 1.0, 1)
    e, r = DeviceMesh(room.vertices, room.faces), DeviceMesh(rxm.vertices, rxm.faces)
    out = [torch.empty(s, dtype=torch.float32, device="cuda") for s in ((n, B + 1, 3), (n, B + 1, 3))]
    mask = torch.empty(n, dtype=torch.int32, device="cuda")
    kind = torch.empty((n, B), dtype=torch.int32, device="cuda")
    face = torch.empty((n, B), dtype=torch.int32, device="cuda")
    o = orc.trace(orc.Mesh(room.vertices, room.faces), orc.Mesh(rxm.vertices, rxm.faces), tx, B, off, n)
    t32 = np.asarray(tx, np.float32)
    for _ in range(2):
        check(lib().rt_trace(e.handle, t32.ctypes.data, r.handle, B, off, n, ptr(out[0]), ptr(out[1]), ptr(mask),
                             ptr(kind), ptr(face), torch.cuda.current_stream().cuda_stream), "rt_trace")
        torch.cuda.synchronize()
        assert out[0].cpu().numpy().tobytes() == o["traced"].tobytes()
        assert out[1].cpu().numpy().tobytes() == o["received"].tobytes()
        assert (mask.cpu().numpy().astype(np.uint32) == o["mask"]).all() and o["mask"].sum() > 0
        assert (kind.cpu().numpy() == o["hit_kind"]).all() and (face.cpu().numpy() == o["hit_face"]).all()
    t = synthetic_terrain(256, 50.0)
    env = DeviceMesh(t.vertices, t.faces, 0)
    grid, ttx, N = CoverageGrid(4.0, -6.0, 2.0, 0.9, 0.8, 1.0, 16, 16, 1), (10.0, 0.0, 4.5), 40_000
    whole = Coverage(t, 2.998e8, 100e9, 200e-9, B, N, grid, env_mesh=env)
    ref = whole.run_device(ttx).cpu().numpy()
    whole.close()
    W = 4
    plans = [Coverage(t, 2.998e8, 100e9, 200e-9, B, N, grid, shard_index=k, shard_count=W, shard_mode="rays",
                      env_mesh=env) for k in range(W)]
    sent = [(lambda rc: (rc[0].clone(), rc[1]))(p.trace_rows(ttx, 1)) for p in plans]
    total = torch.zeros(grid.num_cells, dtype=torch.float64, device="cuda")
    for d, p in enumerate(plans):
        parts = [rows[sum(c[:d]):sum(c[:d]) + c[d]] for rows, c in sent]
        total += p.power_from_rows(torch.cat(parts), [c[d] for _, c in sent])
        p.check()
        p.close()
    assert (~np.isnan(ref)).sum() >= 10
    assert total.cpu().numpy().tobytes() == ref.tobytes()
    print("switch paths ok", {k: os.environ.get(k) for k in ("RFRT_K2_BOX", "RFRT_K2_LPT", "RFRT_TRAJ_SPLIT_MAX")})


if __name__ == "__main__":
    main()
