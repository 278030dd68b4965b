"""Coverage timing per configuration, for rocprofv3 --kernel-trace and for strong-scaling
estimates: K3 (room, 256^2) and K5 (terrain stand-in, 1024^2), each as the whole map and as
rank 0 of an S-way cell shard (the per-rank work of an S-GPU run).  Prints one JSON line per case."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from rf_ray_tracing_warp_amd._lib import DeviceMesh
    from rf_ray_tracing_warp_amd.coverage import Coverage, CoverageGrid
    from rf_ray_tracing_warp_amd.mesh import load_stl, synthetic_terrain
    cases = os.environ.get("CASES", "k3,k5").split(",")
    shards = [int(s) for s in os.environ.get("SHARDS", "1,8").split(",")]
    reps = int(os.environ.get("REPS", "3"))
    for case in cases:
        if case == "k3":
            m = load_stl(os.path.join(ROOT, "models/room.stl"))
            grid, tx, win, B = CoverageGrid.square(256, 15.0, 5.0), (10.0, 0.0, 5.0), 100e-9, 3
        else:
            m = synthetic_terrain(1024, 50.0)
            grid, tx, win, B = CoverageGrid.square(1024, 50.0, 2.0), (10.0, 0.0, 4.5), 200e-9, 3
        env = DeviceMesh(m.vertices, m.faces, 0)
        for S in shards:
            cov = Coverage(m, 2.998e8, 100e9, win, B, 1_000_000, grid, 0.1, device=0, shard_index=0, shard_count=S,
                           env_mesh=env)
            cov.run_device(tx)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                cov.run_device(tx)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / reps
            print(json.dumps({"case": case, "shards": S, "ms_per_map_rank0": dt * 1e3,
                              "candidates_rank0": cov.last_candidates}), flush=True)
            cov.close()
        env.close()


if __name__ == "__main__":
    main()
