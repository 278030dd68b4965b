"""ctypes front end of the CPU oracle (oracle/rt_oracle.c) + the host-side CIR restatement.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg -- never by the product package.

``cir_from_received`` restates ``Tracer.compute_cir``'s host tail (``tracer.py:84-117``) and
``Tracer._bounce_amplitude`` (``tracer.py:34-61``) with the same NumPy calls, so it inherits
NumPy 2's float32 semantics (NEP 50) exactly; it is pinned against goldens produced by the
reference's own ``tracer.py`` (tests/golden/make_golden.py).  ``signal_power`` restates
``coverage.py:45-55`` / ``main.py:46-55``.
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "librt_oracle.so")
_lib = None

_f32p = ctypes.POINTER(ctypes.c_float)
_i32p = ctypes.POINTER(ctypes.c_int32)
_u32p = ctypes.POINTER(ctypes.c_uint32)


def build():
    """Compile the oracle (make, in-tree)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def build_native(out_path):
    """-O3 -march=native build for the CPU baseline, on the machine that times it."""
    subprocess.run(["make", "-s", "-C", _HERE, "native", f"OUT={out_path}"], check=True)
    return out_path


def load(path):
    """Use the oracle library at ``path`` (e.g. build_native's) for every later call."""
    global _lib, _LIB_PATH
    _lib, _LIB_PATH = None, path
    return lib()


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.orc_mesh_create.restype = ctypes.c_void_p
        L.orc_mesh_create.argtypes = [_f32p, ctypes.c_int64, _i32p, ctypes.c_int64]
        L.orc_mesh_destroy.argtypes = [ctypes.c_void_p]
        L.orc_trace.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _f32p, ctypes.c_int, ctypes.c_int64,
                                ctypes.c_int64, _f32p, _f32p, _u32p, _i32p, _i32p, ctypes.c_int]
        L.orc_trace_ids.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _f32p, ctypes.c_int, ctypes.c_int64,
                                    ctypes.POINTER(ctypes.c_int64), ctypes.c_int64, _f32p, _f32p, _u32p, _i32p, _i32p,
                                    ctypes.c_int]
        L.orc_ray_dirs.argtypes = [ctypes.c_int64, ctypes.c_int64, _f32p]
        L.orc_sincosf_bulk.argtypes = [_f32p, ctypes.c_int64, _f32p, _f32p]
        L.orc_acosf_bulk.argtypes = [_f32p, ctypes.c_int64, _f32p]
        L.orc_query_bulk.restype = ctypes.c_int
        L.orc_query_bulk.argtypes = [ctypes.c_void_p, _f32p, _f32p, ctypes.c_int64, ctypes.c_float,
                                     _f32p, _i32p, _f32p]
        L.orc_set_bvh_min.argtypes = [ctypes.c_int64]
        L.orc_pcg.restype = ctypes.c_uint32
        L.orc_pcg.argtypes = [ctypes.c_uint32]
        _lib = L
    return _lib


def _p(a, t):
    return None if a is None else a.ctypes.data_as(t)


class Mesh:
    """A prepared triangle mesh inside the oracle (median-split BVH above ``bvh_min`` faces)."""

    def __init__(self, vertices, faces, bvh_min=2048):
        self.v = np.ascontiguousarray(np.asarray(vertices, dtype=np.float64).astype(np.float32)).reshape(-1, 3)
        self.f = np.ascontiguousarray(np.asarray(faces).astype(np.int32)).reshape(-1, 3)
        lib().orc_set_bvh_min(int(bvh_min))
        self.h = lib().orc_mesh_create(_p(self.v, _f32p), len(self.v), _p(self.f, _i32p), len(self.f))
        lib().orc_set_bvh_min(2048)

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_mesh_destroy(self.h)
            self.h = None

    def query(self, o, d, max_t=1.0e6):
        o = np.ascontiguousarray(o, dtype=np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(d, dtype=np.float32).reshape(-1, 3)
        n = len(o)
        t = np.empty(n, np.float32)
        f = np.empty(n, np.int32)
        nr = np.empty((n, 3), np.float32)
        lib().orc_query_bulk(self.h, _p(o, _f32p), _p(d, _f32p), n, max_t, _p(t, _f32p), _p(f, _i32p),
                             _p(nr, _f32p))
        return t, f, nr


def trace(env: Mesh, rx: Mesh, tx, B, ray_offset, n, want_traced=True, nthreads=None):
    """Run the trace_paths_kernel restatement. Returns dict of numpy arrays."""
    P = B + 1
    tx = np.ascontiguousarray(np.asarray(tx, dtype=np.float64).astype(np.float32))
    out = {
        "traced": np.empty((n, P, 3), np.float32) if want_traced else None,
        "received": np.empty((n, P, 3), np.float32),
        "mask": np.empty(n, np.uint32),
        "hit_kind": np.empty((n, B), np.int32),
        "hit_face": np.empty((n, B), np.int32),
    }
    if nthreads is None:
        nthreads = min(16, os.cpu_count() or 1)
    lib().orc_trace(env.h, rx.h, _p(tx, _f32p), B, ray_offset, n, _p(out["traced"], _f32p),
                    _p(out["received"], _f32p), _p(out["mask"], _u32p), _p(out["hit_kind"], _i32p),
                    _p(out["hit_face"], _i32p), int(nthreads))
    return out


def trace_ids(env: Mesh, rx: Mesh, tx, B, ids, want_traced=True, nthreads=None):
    """trace() for an explicit list of ray ids (rows follow ``ids``)."""
    ids = np.ascontiguousarray(ids, dtype=np.int64)
    n, P = len(ids), B + 1
    tx = np.ascontiguousarray(np.asarray(tx, dtype=np.float64).astype(np.float32))
    out = {
        "traced": np.empty((n, P, 3), np.float32) if want_traced else None,
        "received": np.empty((n, P, 3), np.float32),
        "mask": np.empty(n, np.uint32),
        "hit_kind": np.empty((n, B), np.int32),
        "hit_face": np.empty((n, B), np.int32),
    }
    if nthreads is None:
        nthreads = min(16, os.cpu_count() or 1)
    lib().orc_trace_ids(env.h, rx.h, _p(tx, _f32p), B, 0, ids.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), n,
                        _p(out["traced"], _f32p), _p(out["received"], _f32p), _p(out["mask"], _u32p),
                        _p(out["hit_kind"], _i32p), _p(out["hit_face"], _i32p), int(nthreads))
    return out


def ray_dirs(ray_offset, n):
    out = np.empty((n, 3), np.float32)
    lib().orc_ray_dirs(ray_offset, n, _p(out, _f32p))
    return out


def sincosf(x):
    x = np.ascontiguousarray(x, dtype=np.float32)
    s = np.empty_like(x)
    c = np.empty_like(x)
    lib().orc_sincosf_bulk(_p(x, _f32p), x.size, _p(s, _f32p), _p(c, _f32p))
    return s, c


def acosf(x):
    x = np.ascontiguousarray(x, dtype=np.float32)
    o = np.empty_like(x)
    lib().orc_acosf_bulk(_p(x, _f32p), x.size, _p(o, _f32p))
    return o


# --------------------------------------------------------------------------------------------
# host tail of Tracer.compute_cir (tracer.py:84-117), NumPy semantics kept op for op
# --------------------------------------------------------------------------------------------
def bounce_amplitude(angle_between):
    """tracer.py:34-61 without the prints."""
    if math.isnan(angle_between):
        return 0
    theta = (math.pi / 2) - (angle_between / 2)
    n_1 = 5.0
    n_2 = 1.0
    theta_i = math.asin((n_2 * math.sin(theta)) / n_1)
    num = n_2 * math.cos(theta_i) - n_1 * math.cos(theta)
    denom = n_2 * math.cos(theta_i) + n_1 * math.cos(theta)
    amp = -(num / denom) ** 2
    if amp < -1:
        amp = -1
    if math.isnan(amp):
        return 0
    return -amp


def clean_paths(received, mask):
    """tracer.py:87-97: keep masked rows (ray order), cut each at its first NaN point."""
    paths = received[mask != 0, :, :]
    cleaned = []
    for path in paths:
        new_path = []
        for i in range(path.shape[0]):
            if np.isnan(path[i]).any():
                break
            new_path.append(path[i])
        cleaned.append(np.array(new_path))
    return cleaned


def _arccos_cr(x):
    """float32 arccos rounded once from double: the device's choice (NumPy's SIMD float32 arccos is
    a few ulp off; used only to separate that rounding from other differences in the tests)."""
    return np.float32(math.acos(float(x))) if abs(float(x)) <= 1.0 else np.float32("nan")


def cir_from_paths(cleaned_paths, tx_power, tx_num_rays, light_speed_mps, sample_rate_hz, sample_window_s,
                   arccos=np.arccos):
    """tracer.py:101-117 (``arccos`` replaceable only for the conditioning checks of the tests)."""
    with np.errstate(all="ignore"):
        impulse_response = np.zeros(int(sample_window_s * sample_rate_hz))
        for path in cleaned_paths:
            amplitude = tx_power / tx_num_rays
            distance = 0.0
            for p1, p2, p3 in zip(path[:-2], path[1:-1], path[2:]):
                seg1 = p2 - p1
                seg2 = p3 - p2
                seg1_len = np.linalg.norm(seg1)
                angle_between = arccos(np.dot(seg1, seg2) / (seg1_len * np.linalg.norm(seg2)))
                amplitude *= bounce_amplitude(angle_between)
                distance += seg1_len
            distance += np.linalg.norm(path[-2] - path[-1])
            delay_samples = int((distance / light_speed_mps) * sample_rate_hz)
            if delay_samples < impulse_response.shape[0]:
                impulse_response[delay_samples] += amplitude
    return impulse_response


def path_bin_amp(path, tx_power, tx_num_rays, light_speed_mps, sample_rate_hz):
    """(delay bin, amplitude) of one cleaned path -- the per-path body of tracer.py:101-117."""
    with np.errstate(all="ignore"):
        amplitude = tx_power / tx_num_rays
        distance = 0.0
        for p1, p2, p3 in zip(path[:-2], path[1:-1], path[2:]):
            seg1 = p2 - p1
            seg2 = p3 - p2
            seg1_len = np.linalg.norm(seg1)
            angle_between = np.arccos(np.dot(seg1, seg2) / (seg1_len * np.linalg.norm(seg2)))
            amplitude *= bounce_amplitude(angle_between)
            distance += seg1_len
        distance += np.linalg.norm(path[-2] - path[-1])
        return int((distance / light_speed_mps) * sample_rate_hz), amplitude


def signal_power(impulse_response, sample_window_s):
    """coverage.py:45-52 / main.py:39-52: mean-square of the nonzero samples of ir (*) sin."""
    with np.errstate(all="ignore"):
        time = np.linspace(0, sample_window_s, impulse_response.shape[0])
        signal_tx = np.sin(2 * np.pi * 2.4e9 * time)
        signal_rx = np.convolve(impulse_response, signal_tx, mode="same")
        r = np.nonzero(signal_rx)[:10000]
        signal_rx = signal_rx[r]
        return np.sum(signal_rx ** 2) / signal_rx.shape[0]


def to_dbm(power):
    """main.py:12-13."""
    with np.errstate(all="ignore"):
        return 10 * np.log10(power / 1e-3)


def coverage_loop(env: Mesh, tx, centers, B, n_rays, c=2.998e8, fs=100e9, win=100e-9, tx_power=1, rx_radius=0.1,
                  nthreads=None, with_cr=False):
    """coverage.py:38-57 literally: for every receiver centre a full trace (kernel.py) with that
    cell's icosphere (tracer.py:27), the host CIR (tracer.py:84-117) and the signal power
    (coverage.py:45-52).  Returns (power per cell, list of impulse responses)."""
    import sys as _sys
    _sys.path.insert(0, os.path.dirname(_HERE))
    from rf_ray_tracing_warp_amd.mesh import sphere

    powers, irs, powers_cr = [], [], []
    for cen in np.asarray(centers, dtype=np.float64).reshape(-1, 3):
        rxm = sphere(cen, rx_radius, 1)
        o = trace(env, Mesh(rxm.vertices, rxm.faces), tx, B, 0, n_rays, want_traced=False, nthreads=nthreads)
        paths = clean_paths(o["received"], o["mask"])
        ir = cir_from_paths(paths, tx_power, n_rays, c, fs, win)
        irs.append(ir)
        powers.append(signal_power(ir, win))
        if with_cr:
            powers_cr.append(signal_power(cir_from_paths(paths, tx_power, n_rays, c, fs, win, arccos=_arccos_cr), win))
    if with_cr:
        return np.array(powers), irs, np.array(powers_cr)
    return np.array(powers), irs


# --------------------------------------------------------------------------------------------
# the same host tail, vectorised over paths (cells whose receiver contains the transmitter receive
# every ray: a million paths, too many for the literal per-path loop above)
# --------------------------------------------------------------------------------------------
def _dot32(a, b):
    """np.dot of float32 3-vectors, row-wise: f32 products summed left to right in f64, rounded once
    (equal to np.dot on 200k random vectors)."""
    p = (a * b).astype(np.float64)
    return ((p[:, 0] + p[:, 1]) + p[:, 2]).astype(np.float32)


def _bounce_amplitude_vec(angle):
    """tracer.py:34-61 element-wise: theta in float32 (NEP 50: math.pi / 2 - float32), the rest in
    float64 with NumPy's sin/cos/arcsin instead of math's (equal up to libm ulps)."""
    with np.errstate(all="ignore"):
        theta = np.float32(math.pi / 2) - angle / np.float32(2)
        th = theta.astype(np.float64)
        ti = np.arcsin((1.0 * np.sin(th)) / 5.0)
        num = 1.0 * np.cos(ti) - 5.0 * np.cos(th)
        den = 1.0 * np.cos(ti) + 5.0 * np.cos(th)
        amp = -(num / den) ** 2
        amp = np.where(amp < -1, -1.0, amp)
        out = -amp
        out = np.where(np.isnan(angle) | np.isnan(amp), 0.0, out)
    return out


def cir_from_rows(received, mask, tx_power, tx_num_rays, light_speed_mps, sample_rate_hz, sample_window_s,
                  arccos=np.arccos):
    """clean_paths + cir_from_paths (tracer.py:87-117) vectorised over the received rows: the same
    float32/float64 operations in the same order per path, accumulated with np.add.at in ray order
    (sequential, like the loop).  ``arccos`` acts on float32 arrays; pass ``arccos_cr_vec`` for the
    rounded-once variant.  Returns (impulse_response, per-path delay bins, per-path amplitudes)."""
    rows = received[mask != 0]
    n, P = rows.shape[0], rows.shape[1]
    bad = np.isnan(rows).any(axis=2)
    length = np.where(bad.any(axis=1), np.argmax(bad, axis=1), P)
    amp = np.full(n, tx_power / tx_num_rays, dtype=np.float64)
    dist = np.zeros(n, dtype=np.float32)
    with np.errstate(all="ignore"):
        for i in range(P - 2):  # vertex i+1 is interior where i + 2 < length
            act = i + 2 < length
            if not act.any():
                break
            p1, p2, p3 = rows[act, i], rows[act, i + 1], rows[act, i + 2]
            s1, s2 = p2 - p1, p3 - p2
            l1 = np.sqrt(_dot32(s1, s1))
            cosv = _dot32(s1, s2) / (l1 * np.sqrt(_dot32(s2, s2)))
            amp[act] = amp[act] * _bounce_amplitude_vec(arccos(cosv).astype(np.float32))
            dist[act] = dist[act] + l1
        idx = np.arange(n)
        last = rows[idx, length - 2] - rows[idx, length - 1]
        dist = dist + np.sqrt(_dot32(last, last))
        delay = ((dist / light_speed_mps) * sample_rate_hz).astype(np.int64)
    ir = np.zeros(int(sample_window_s * sample_rate_hz))
    keep = delay < ir.shape[0]
    np.add.at(ir, delay[keep], amp[keep])
    return ir, delay, amp


def arccos_cr_vec(x):
    """float32 arccos rounded once from float64 (the device's choice), element-wise."""
    with np.errstate(all="ignore"):
        return np.arccos(np.asarray(x, np.float64)).astype(np.float32)


def coverage_cell(env: Mesh, tx, center, B, n_rays, c=2.998e8, fs=100e9, win=100e-9, tx_power=1, rx_radius=0.1,
                  nthreads=None):
    """One iteration of coverage.py:38-57 for one receiver centre, at full burst size: the trace
    restatement, the vectorised host CIR (NumPy arccos and the rounded-once arccos) and the power.
    Returns dict(ir, ir_cr, power, power_cr, paths)."""
    import sys as _sys
    _sys.path.insert(0, os.path.dirname(_HERE))
    from rf_ray_tracing_warp_amd.mesh import sphere

    rxm = sphere(np.asarray(center, np.float64), rx_radius, 1)
    o = trace(env, Mesh(rxm.vertices, rxm.faces), tx, B, 0, n_rays, want_traced=False, nthreads=nthreads)
    ir, _, _ = cir_from_rows(o["received"], o["mask"], tx_power, n_rays, c, fs, win)
    ir_cr, _, _ = cir_from_rows(o["received"], o["mask"], tx_power, n_rays, c, fs, win, arccos=arccos_cr_vec)
    return {"ir": ir, "ir_cr": ir_cr, "power": signal_power(ir, win), "power_cr": signal_power(ir_cr, win),
            "paths": int(np.count_nonzero(o["mask"]))}
