"""Coverage A/B: time K3 (room, 256^2) and K5 (terrain stand-in, 1024^2) maps on one GPU and hash
their outputs (power map + sparse impulse responses), once per library in LIBS (RFRT_LIB_PATH
per child process).  The hashes check that every variant is bit-identical to the first."""
import hashlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(cases, reps):
    sys.path.insert(0, ROOT)
    import torch
    from rf_ray_tracing_warp_amd._lib import DeviceMesh
    from rf_ray_tracing_warp_amd.coverage import Coverage, CoverageGrid
    from rf_ray_tracing_warp_amd.mesh import load_stl, synthetic_terrain
    out = {"lib": os.path.basename(os.environ.get("RFRT_LIB_PATH", "librfrt.so")),
           "rxfirst": os.environ.get("RFRT_COV_RXFIRST", "1")}
    for case in cases:
        if case == "k3":
            m = load_stl(os.path.join(ROOT, "models/room.stl"))
            grid, tx, win = CoverageGrid.square(256, 15.0, 5.0), (10.0, 0.0, 5.0), 100e-9
        else:
            m = synthetic_terrain(1024, 50.0)
            grid, tx, win = CoverageGrid.square(1024, 50.0, 2.0), (10.0, 0.0, 4.5), 200e-9
        env = DeviceMesh(m.vertices, m.faces, 0)
        cov = Coverage(m, 2.998e8, 100e9, win, 3, 1_000_000, grid, 0.1, device=0, env_mesh=env)
        p = cov.run_device(tx)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            p = cov.run_device(tx)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        c, b, a = cov.impulse_responses()
        h = hashlib.sha256(p.cpu().numpy().tobytes() + c.tobytes() + b.tobytes() + a.tobytes()).hexdigest()[:16]
        cov.profile(True)
        cov.run_device(tx)
        pr = cov.last_profile()
        cov.profile(False)
        out[case] = {"ms": round(dt * 1e3, 3), "hash": h,
                     "stages": {k: round(v, 3) for k, v in pr.items() if k.endswith("_ms")}}
        cov.close()
        env.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        child(sys.argv[2].split(","), int(sys.argv[3]))
        sys.exit(0)
    libs = os.environ["LIBS"].split()
    cases = os.environ.get("CASES", "k3,k5")
    reps = os.environ.get("REPS", "3")
    res = []
    for spec in libs:  # path[@VAR=value,...]: per-variant environment (e.g. @RFRT_COV_RXFIRST=0)
        lib, _, extra = spec.partition("@")
        env = dict(os.environ, RFRT_LIB_PATH=os.path.abspath(lib))
        env.update(kv.split("=", 1) for kv in extra.split(",") if kv)
        r = subprocess.run([sys.executable, __file__, "child", cases, reps], env=env, capture_output=True, text=True,
                           timeout=600)
        if r.returncode != 0:
            print(r.stderr[-3000:])
            sys.exit(r.returncode)
        res.append(json.loads(r.stdout.strip().splitlines()[-1]))
        print(json.dumps(res[-1]), flush=True)
    same = all(all(x[c]["hash"] == res[0][c]["hash"] for c in cases.split(",")) for x in res)
    print("bit-identical outputs across variants:", same)
    sys.exit(0 if same else 3)
