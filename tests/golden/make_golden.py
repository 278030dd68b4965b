"""Generate host-side golden vectors by running the reference's own tracer.py (dev container only).

warp-lang and trimesh are not installed here, so this script inserts small
stand-ins for both into sys.modules, imports /root/reference/tracer.py (and kernel.py, which only
needs the decorators), and runs ``Tracer.compute_cir`` end to end.  The stand-in ``wp.launch``
does not trace anything: it copies a prepared ``received_paths`` / ``row_mask`` pair into the
arrays tracer.py allocated.  Everything after the launch -- readback, mask filter, NaN strip,
Fresnel factor, float32 distance/delay, impulse-response accumulation (tracer.py:84-117) -- is the
reference's code running on this container's NumPy 2.2.

Inputs come from two sources:
  * realistic received paths from the CPU oracle's trace of models/room.stl (oracle/rt_oracle.c);
  * hand-made edge cases (LOS, RX pass-through, zero-length segment -> NaN amplitude, cos>1,
    out-of-window delay, empty mask).

Output: tests/golden/host_cir.npz (inputs + the reference's outputs; data only).
Run:    python tests/golden/make_golden.py
"""
import contextlib
import io
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
REF = "/root/reference"


class _FakeArray:
    def __init__(self, data=None, dtype=None):
        if data is None:  # used as a type annotation in kernel.py:44-46
            self._a = None
            return
        a = np.asarray(data)
        if dtype == "vec3":
            a = a.astype(np.float32)
        elif dtype == "uint32":
            a = a.astype(np.uint32)
        elif dtype == "int32":
            a = a.astype(np.int32)
        self._a = np.ascontiguousarray(a)

    def numpy(self):
        return self._a


_PENDING = {}


def _install_fakes():
    wp = types.ModuleType("warp")
    wp.vec3 = "vec3"
    wp.uint32 = "uint32"
    wp.int32 = "int32"
    wp.uint64 = "uint64"
    wp.float32 = "float32"
    wp.init = lambda: None
    wp.build = types.SimpleNamespace(clear_kernel_cache=lambda: None)
    wp.array = _FakeArray
    wp.array2d = lambda dtype=None: None
    wp.func = lambda f: f
    wp.kernel = lambda f: f

    class Mesh:
        def __init__(self, points=None, velocities=None, indices=None):
            self.id = id(self)

    wp.Mesh = Mesh

    def launch(kernel, dim, inputs):
        received, row_mask = inputs[5], inputs[6]
        received._a[...] = _PENDING["received"]
        row_mask._a[...] = _PENDING["mask"]

    wp.launch = launch
    wp.synchronize_device = lambda: None
    sys.modules["warp"] = wp

    tm = types.ModuleType("trimesh")
    sys.path.insert(0, REPO)
    from rf_ray_tracing_warp_amd.mesh import sphere

    tm.primitives = types.SimpleNamespace(Sphere=lambda center, radius, subdivisions: sphere(center, radius, subdivisions))
    tm.viewer = types.ModuleType("trimesh.viewer")
    sys.modules["trimesh"] = tm
    sys.modules["trimesh.viewer"] = tm.viewer


def _reference_tracer():
    _install_fakes()
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import tracer  # noqa: E402  (the reference's tracer.py)

    return tracer


def run_reference(tracer_mod, received, mask, params, tx_power):
    n, P, _ = received.shape
    t = tracer_mod.Tracer(types.SimpleNamespace(vertices=np.zeros((3, 3)), faces=np.zeros((1, 3), int)),
                          params["c"], params["fs"], params["win"], P - 1, n)
    _PENDING["received"] = received
    _PENDING["mask"] = mask
    with contextlib.redirect_stdout(io.StringIO()):
        paths, ir = t.compute_cir(np.array([0.0, 0.0, 0.0]), tx_power, np.array([0.0, 0.0, 0.0]), 0.1)
    return paths, ir


def edge_cases():
    nan = np.nan
    P = 4
    rows = []
    # LOS tx->rx front
    rows.append([[10, 0, 5], [-9.9, 0, 5], [nan] * 3, [nan] * 3])
    # pass-through front -> back (angle 0)
    rows.append([[10, 0, 5], [-9.9, 0, 5], [-10.1, 0, 5], [nan] * 3])
    # long one-bounce path outside a 100 ns window
    rows.append([[10, 0, 5], [14.9, 3, 5], [-9.9, 0.05, 5.02], [nan] * 3])
    # zero-length segment (RX self-hit duplicate) -> 0/0 -> NaN angle -> amplitude 0
    rows.append([[10, 0, 5], [-9.9, 0, 5], [-9.9, 0, 5], [-10.1, 0, 5]])
    # env bounce then rx
    rows.append([[10, 0, 5], [0.4, 1.0, 5.5], [-9.95, 0.01, 5.0], [-10.05, 0.01, 5.0]])
    # near-collinear segments (cos rounding at/above 1 possible)
    rows.append([[10, 0, 5], [-9.90001, 1e-7, 5], [-10.0999, 2e-7, 5.0000001], [nan] * 3])
    # grazing reflection
    rows.append([[10, 0, 5], [0, 0, 0.0001], [-9.92, 0.0, 4.99], [nan] * 3])
    rec = np.array(rows, np.float32).reshape(-1, P, 3)
    mask = np.ones(len(rec), np.uint32)
    # padding rows that are not received
    pad = np.full((5, P, 3), np.nan, np.float32)
    pad[:, 0] = [10, 0, 5]
    return np.concatenate([rec, pad]), np.concatenate([mask, np.zeros(5, np.uint32)])


def oracle_cases():
    sys.path.insert(0, REPO)
    from oracle import oracle as orc
    from rf_ray_tracing_warp_amd.mesh import load_stl, sphere

    env = load_stl(os.path.join(REPO, "models", "room.stl"))
    out = []
    for (rx, B, n, off) in [((5, 3, 4), 3, 400_000, 0), ((-10, 8, 5), 5, 300_000, 7_000_000),
                            ((3, -12, 2), 4, 300_000, 123_456)]:
        rxm = sphere(rx, 0.1, 1)
        r = orc.trace(orc.Mesh(env.vertices, env.faces), orc.Mesh(rxm.vertices, rxm.faces), (10, 0, 5), B, off, n,
                      want_traced=False)
        keep = np.nonzero(r["mask"])[0]
        # keep the received rows plus a sprinkle of unreceived ones (the reference filters them)
        idx = np.union1d(keep, np.arange(0, n, max(1, n // 50)))
        out.append((r["received"][idx], r["mask"][idx], int(len(keep))))
    return out


def main():
    tr = _reference_tracer()
    cases = []
    params_room = {"c": 2.998e8, "fs": 100e9, "win": 100e-9}
    rec, mask = edge_cases()
    cases.append(("edge", rec, mask, params_room, 1))
    for k, (rec, mask, nrec) in enumerate(oracle_cases()):
        cases.append((f"room{k}", rec, mask, {"c": 2.998e8, "fs": 100e9, "win": 200e-9 if k == 1 else 100e-9}, 1))
    store = {}
    for name, rec, mask, prm, txp in cases:
        paths, ir = run_reference(tr, rec, mask, prm, txp)
        store[f"{name}_received"] = rec
        store[f"{name}_mask"] = mask
        store[f"{name}_params"] = np.array([prm["c"], prm["fs"], prm["win"], txp], np.float64)
        store[f"{name}_ir"] = ir
        store[f"{name}_lengths"] = np.array([len(p) for p in paths], np.int64)
        store[f"{name}_paths"] = (np.concatenate(paths).astype(np.float32) if paths else np.zeros((0, 3), np.float32))
        print(name, "received", len(paths), "nonzero bins", int(np.count_nonzero(ir)), "sum", ir.sum())
    # _bounce_amplitude on f32 and Python-float angles (tracer.py:34-61)
    t = tr.Tracer(types.SimpleNamespace(vertices=np.zeros((3, 3)), faces=np.zeros((1, 3), int)), 2.998e8, 100e9,
                  100e-9, 1, 1)
    angles32 = np.concatenate([np.linspace(0, np.pi, 2001, dtype=np.float32),
                               np.array([0.0, 1e-7, 0.5, np.pi / 2, 3.0, np.float32(np.pi), np.nan], np.float32)])
    with contextlib.redirect_stdout(io.StringIO()):
        amp32 = np.array([float(t._bounce_amplitude(a)) for a in angles32])
        amp64 = np.array([float(t._bounce_amplitude(float(a))) for a in angles32])
    store["amp_angles32"] = angles32
    store["amp_f32"] = amp32
    store["amp_f64"] = amp64
    np.savez_compressed(os.path.join(HERE, "host_cir.npz"), **store)
    print("wrote", os.path.join(HERE, "host_cir.npz"))


if __name__ == "__main__":
    main()
