"""ctypes binding of librfrt.so (include/rfrt.h).

There is no fallback: if the library is missing or fails to load, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RFRT_LIB_PATH") or os.path.join(_PKG, "librfrt.so")

RT_MESH_BVH_GPU = 1
RT_CIR_C_F64 = 1
RT_CIR_FS_F64 = 2

_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_int = ctypes.c_int
_lib = None


class RfrtError(RuntimeError):
    pass


def lib():
    """Load librfrt.so once (raises RfrtError if it is not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RfrtError(f"{LIB_PATH} is not built: run `python -m rf_ray_tracing_warp_amd.build` "
                        "(the HIP path has no CPU fallback)")
    # PyTorch ships its own HIP/HSA runtime libraries under the same sonames as /opt/rocm's.  Load
    # torch first so librfrt binds to the runtime torch uses: loaded the other way round, the
    # process ends up with two HSA runtimes and librfrt's sees no device (GPU box, r2a).
    import torch  # noqa: F401
    L = ctypes.CDLL(LIB_PATH)
    L.rt_last_error.restype = ctypes.c_char_p
    L.rt_version.restype = _int
    L.rt_mesh_create.argtypes = [_int, _vp, _i64, _vp, _i64, ctypes.POINTER(_vp)]
    L.rt_mesh_create_ex.argtypes = [_int, _vp, _i64, _vp, _i64, _int, ctypes.POINTER(_vp)]
    L.rt_mesh_destroy.argtypes = [_vp]
    L.rt_mesh_info.argtypes = [_vp, _vp, _vp, _vp]
    L.rt_bvh_info.argtypes = [_vp, _vp]
    L.rt_trace.argtypes = [_vp, _vp, _vp, _int, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp]
    L.rt_compact_workspace_bytes.restype = _i64
    L.rt_compact_workspace_bytes.argtypes = [_i64]
    L.rt_compact.argtypes = [_vp, _i64, _vp, _i64, _vp, _vp, _vp]
    L.rt_trace_cir_workspace_bytes.restype = _i64
    L.rt_trace_cir_workspace_bytes.argtypes = [_i64]
    L.rt_trace_cir.argtypes = [_vp, _vp, _vp, _int, _i64, _i64, _vp, _vp, _vp, ctypes.c_double, ctypes.c_double,
                               ctypes.c_double, _int, _i64, _vp, _vp, _vp, _vp, _i64, _vp]
    L.rt_cir.argtypes = [_vp, _vp, _vp, _i64, _int, ctypes.c_double, ctypes.c_double, ctypes.c_double, _int, _i64,
                         _vp, _vp, _vp, _vp]
    L.rt_coverage_create.argtypes = [_int, _vp, _int, _i64, _i64, _vp, ctypes.c_double, _int, _int,
                                     ctypes.POINTER(_vp)]
    L.rt_coverage_destroy.argtypes = [_vp]
    L.rt_coverage_run.argtypes = [_vp, _vp, ctypes.c_double, ctypes.c_double, ctypes.c_double, _int, _i64,
                                  ctypes.c_double, _vp, _vp, _vp]
    L.rt_coverage_create_rays.argtypes = [_int, _vp, _int, _i64, _i64, _i64, _vp, ctypes.c_double, _int, _int,
                                          ctypes.POINTER(_vp)]
    L.rt_coverage_create_sectors.argtypes = [_int, _vp, _int, _i64, _vp, ctypes.c_double, _int, _int, _vp]
    L.rt_coverage_records_packed.argtypes = [_vp, _vp, _i64, _vp]
    L.rt_coverage_power_rows.argtypes = [_vp, _vp, _i64, _i64, ctypes.c_double, _vp, _vp]
    L.rt_coverage_power_packed.argtypes = [_vp, _vp, _vp, _int, _i64, ctypes.c_double, _vp, _vp]
    L.rt_coverage_amps_to_sums.argtypes = [_vp, _i64, _vp, _vp]
    L.rt_coverage_received.argtypes = [_vp, _vp, _vp, _i64, ctypes.POINTER(_i64), _vp]
    L.rt_power_dense.argtypes = [_vp, _i64, _i64, ctypes.c_double, _vp, _i64, _vp, _vp]
    L.rt_coverage_profile.argtypes = [_vp, _int]
    L.rt_coverage_check.argtypes = [_vp, _vp, _vp]
    L.rt_coverage_trace_rows_async.argtypes = [_vp, _vp, ctypes.c_double, ctypes.c_double, ctypes.c_double, _int,
                                               _i64, _vp, _i64, _vp, _vp]
    L.rt_coverage_trace_rows_finish.argtypes = [_vp, _vp, _vp, _vp]
    L.rt_coverage_last_profile.argtypes = [_vp, _vp, _int]
    L.rt_debug_poison.argtypes = [_int]
    L.rt_release_caches.argtypes = []
    L.rt_debug_replay_window_max.argtypes = [_i64]
    L.rt_profile.argtypes = [_int]
    L.rt_trace_last_profile.argtypes = [_vp, _int]
    L.rt_trace_profile_stats.argtypes = [_vp, _int]
    L.rt_selftest_math.argtypes = [_vp, _i64, _vp, _int, _vp]
    L.rt_ray_dirs.argtypes = [_i64, _i64, _vp, _vp]
    L.rt_query.argtypes = [_vp, _vp, _vp, _i64, _vp, _vp, _vp]
    L.rt_selftest_fx.argtypes = [_vp, _vp, _i64, _int]
    for name in ("rt_mesh_create", "rt_mesh_create_ex", "rt_mesh_destroy", "rt_mesh_info", "rt_bvh_info", "rt_trace", "rt_compact", "rt_cir", "rt_trace_cir",
                 "rt_coverage_create", "rt_coverage_destroy", "rt_coverage_run", "rt_coverage_received",
                 "rt_coverage_create_rays", "rt_coverage_create_sectors",
                 "rt_coverage_records_packed",
                 "rt_coverage_power_rows",
                 "rt_coverage_power_packed", "rt_coverage_amps_to_sums", "rt_coverage_profile", "rt_coverage_check",
                 "rt_coverage_trace_rows_async", "rt_coverage_trace_rows_finish",
                 "rt_coverage_last_profile", "rt_debug_poison", "rt_debug_replay_window_max", "rt_release_caches",
                 "rt_profile", "rt_trace_last_profile", "rt_trace_profile_stats",
                 "rt_power_dense", "rt_selftest_math", "rt_ray_dirs", "rt_query", "rt_selftest_fx"):
        if hasattr(L, name):
            getattr(L, name).restype = _int
    _lib = L
    return L


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().rt_last_error().decode(errors="replace")
        raise RfrtError(f"{what or 'librfrt'} failed ({rc}): {msg}")


def ptr(t) -> int | None:
    """data_ptr() of a torch tensor (None -> NULL)."""
    return None if t is None else t.data_ptr()


def stream_handle(device) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream


class DeviceMesh:
    """A triangle mesh resident on one GPU (the wp.Mesh of tracer.py:24,30)."""

    def __init__(self, vertices, faces, device: int = 0, builder: str = "sah"):
        """builder: "sah" (host binned-SAH BVH, default) or "gpu" (device LBVH, RT_MESH_BVH_GPU);
        only meshes of more than 192 faces get a BVH, and results do not depend on it."""
        v = np.ascontiguousarray(np.asarray(vertices, dtype=np.float64).astype(np.float32)).reshape(-1, 3)
        f = np.ascontiguousarray(np.asarray(faces).astype(np.int32)).reshape(-1, 3)
        if builder not in ("sah", "gpu"):
            raise ValueError(f"builder must be 'sah' or 'gpu', not {builder!r}")
        self.device = int(device)
        self.num_faces = len(f)
        self._h = _vp()
        flags = RT_MESH_BVH_GPU if builder == "gpu" else 0
        check(lib().rt_mesh_create_ex(self.device, v.ctypes.data, len(v), f.ctypes.data, len(f), flags,
                                      ctypes.byref(self._h)), "rt_mesh_create_ex")

    @property
    def handle(self):
        return self._h

    def info(self):
        nf = ctypes.c_int64()
        b = np.zeros(6, np.float32)
        s = np.zeros(4, np.float32)
        check(lib().rt_mesh_info(self._h, ctypes.byref(nf), b.ctypes.data, s.ctypes.data), "rt_mesh_info")
        return int(nf.value), b, s

    def bvh_info(self):
        """{'nodes', 'leaves', 'depth', 'max_leaf'} of the BVH (all 0 for brute-force meshes)."""
        out = np.zeros(4, np.int64)
        check(lib().rt_bvh_info(self._h, out.ctypes.data), "rt_bvh_info")
        return dict(zip(("nodes", "leaves", "depth", "max_leaf"), (int(x) for x in out)))

    def close(self):
        if getattr(self, "_h", None) and self._h.value and _lib is not None:
            _lib.rt_mesh_destroy(self._h)
            self._h = _vp()

    def __del__(self):
        self.close()
