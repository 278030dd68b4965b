"""Drop-in ``Tracer`` for the reference's tracer.py, running on MI355X through librfrt.so.

Same constructor and ``compute_cir`` signature and return values as the reference
(``tracer.py:11-121``):

    tracer = Tracer(mesh, light_speed_mps, sample_rate_hz, sample_window_s, max_bounces, tx_num_rays)
    cleaned_paths, impulse_response = tracer.compute_cir(tx_pos, tx_power, rx_pos, rx_radius)

* ``mesh`` is any object with ``.vertices`` (V,3) and ``.faces`` (F,3) (a trimesh.Trimesh, or
  :class:`rf_ray_tracing_warp_amd.mesh.TriMesh` from :func:`load_mesh`).
* ``cleaned_paths``: list of float32 (L,3) arrays, received rays in ray-id order (tracer.py:87-97).
* ``impulse_response``: float64 (int(sample_window_s*sample_rate_hz),) (tracer.py:101-117).

Differences that are not semantic: buffers live in HBM as PyTorch tensors, only the received
rows cross PCIe (not the whole (N,B+1,3) array, tracer.py:84), the impulse response is
accumulated on the device, and nothing is printed unless ``verbose=True``.
"""
from __future__ import annotations

import math
import time

import numpy as np

from . import _lib
from . import dist as rdist
from ._lib import DeviceMesh, check, lib, ptr
from .mesh import sphere

__all__ = ["Tracer", "cir_flags"]


def _promotes_f32(x) -> bool:
    """Does ``np.float32 <op> x`` compute in float64 under NumPy 2 (NEP 50)?  Python int/float
    scalars are weak and keep float32; NumPy scalars and arrays are strong and follow
    np.result_type (float64, int32/int64/uint32/uint64 -> float64; float16, int8/int16 -> float32)."""
    if isinstance(x, (np.generic, np.ndarray)):
        return np.result_type(np.float32, np.asarray(x).dtype) != np.float32
    return False


def cir_flags(light_speed_mps, sample_rate_hz) -> int:
    """tracer.py:115 ``int((distance / light_speed_mps) * sample_rate_hz)`` with ``distance`` a
    np.float32: each operation is float32 unless NumPy's promotion makes it float64 (NEP 50)."""
    f = 0
    if _promotes_f32(light_speed_mps):
        f |= _lib.RT_CIR_C_F64
    if _promotes_f32(sample_rate_hz):
        f |= _lib.RT_CIR_FS_F64
    return f


class Tracer:
    """tracer.py:11 ``class Tracer`` -- same constructor arguments, plus ``device`` / ``verbose``."""

    # rt_trace_cir's per-call limit (its chunk tables, include/rfrt.h); larger bursts take rt_trace +
    # rt_compact + rt_cir, which have no cap (the reference's tracer.py has none either)
    TRACE_CIR_MAX_RAYS = 1 << 25

    def __init__(self, environment_trimesh, light_speed_mps, sample_rate_hz, sample_window_s, max_bounces,
                 tx_num_rays, device: int | None = None, verbose: bool = False):
        import torch

        if not torch.cuda.is_available():
            raise _lib.RfrtError("Tracer needs a ROCm GPU (librfrt has no CPU path)")
        # one process per GPU: LOCAL_RANK under torchrun, else the current device
        self.device = rdist.default_device() if device is None else int(device)
        self.light_speed_mps = light_speed_mps
        self.sample_rate_hz = sample_rate_hz
        self.sample_window_s = sample_window_s
        self.max_bounces = int(max_bounces)
        self.tx_num_rays = int(tx_num_rays)
        self.verbose = verbose
        lib()  # fail loudly now if the extension is missing
        self.env = DeviceMesh(environment_trimesh.vertices, environment_trimesh.faces, self.device)
        self._ws = None

    # tracer.py:26-30
    def _generate_rx_mesh(self, rx_pos, rx_radius):
        rx = sphere(rx_pos, rx_radius, subdivisions=1)
        return DeviceMesh(rx.vertices, rx.faces, self.device)

    # tracer.py:34-61 (host helper, kept for API parity; the device path uses the same formula)
    def _bounce_amplitude(self, angle_between):
        if math.isnan(angle_between):
            return 0
        theta = (math.pi / 2) - (angle_between / 2)
        n_1, n_2 = 5.0, 1.0
        theta_i = math.asin((n_2 * math.sin(theta)) / n_1)
        num = n_2 * math.cos(theta_i) - n_1 * math.cos(theta)
        denom = n_2 * math.cos(theta_i) + n_1 * math.cos(theta)
        amp = -(num / denom) ** 2
        if amp < -1:
            amp = -1
        if math.isnan(amp):
            return 0
        return -amp

    def _workspace(self, n):
        import torch

        need = int(lib().rt_compact_workspace_bytes(n))
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device=f"cuda:{self.device}")
        return self._ws

    def trace_device(self, tx_pos, rx_mesh, received, mask, traced=None, ray_offset=0, n=None, hit_kind=None,
                     hit_face=None):
        """The wp.launch of tracer.py:75-79 on caller-provided device tensors (asynchronous)."""
        tx = np.ascontiguousarray(np.asarray(tx_pos, dtype=np.float64).astype(np.float32))
        n = self.tx_num_rays if n is None else int(n)
        check(lib().rt_trace(self.env.handle, tx.ctypes.data, rx_mesh.handle if rx_mesh is not None else None,
                             self.max_bounces, int(ray_offset), n, ptr(traced), ptr(received), ptr(mask),
                             ptr(hit_kind), ptr(hit_face), _lib.stream_handle(self.device)), "rt_trace")

    def cir_device(self, received, mask, tx_power, impulse_response, n=None, index=None, count=None):
        """tracer.py:87-117 on the device: compaction + per-path amplitude/delay + accumulate.

        Returns (index, count) device tensors of the received rows (ray-id order)."""
        import torch

        n = self.tx_num_rays if n is None else int(n)
        dev = f"cuda:{self.device}"
        if index is None:
            index = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        if count is None:
            count = torch.empty(1, dtype=torch.int64, device=dev)
        ws = self._workspace(n)
        s = _lib.stream_handle(self.device)
        check(lib().rt_compact(ptr(mask), n, ptr(ws), ws.numel(), ptr(index), ptr(count), s), "rt_compact")
        amp0 = tx_power / self.tx_num_rays
        check(lib().rt_cir(ptr(received), ptr(index), ptr(count), n, self.max_bounces, float(amp0),
                           float(self.light_speed_mps), float(self.sample_rate_hz),
                           cir_flags(self.light_speed_mps, self.sample_rate_hz), impulse_response.numel(),
                           ptr(impulse_response), None, None, s), "rt_cir")
        return index, count

    def trace_cir_device(self, tx_pos, rx_mesh, received, mask, tx_power, impulse_response, traced=None,
                         ray_offset=0, n=None, index=None, count=None, amp_rays=None):
        """tracer.py:67-117 on the device in two launches (rt_trace_cir): the trace, then the ordered
        compaction + impulse response (overwritten).  amp_rays: the burst size of the amplitude
        tx_power / amp_rays (default tx_num_rays).  Returns (index, count) device tensors."""
        import torch

        n = self.tx_num_rays if n is None else int(n)
        dev = f"cuda:{self.device}"
        if index is None:
            index = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        if count is None:
            count = torch.empty(1, dtype=torch.int64, device=dev)
        need = int(lib().rt_trace_cir_workspace_bytes(n))
        if getattr(self, "_tc_ws", None) is None or self._tc_ws.numel() < need:
            self._tc_ws = torch.zeros(need, dtype=torch.uint8, device=dev)  # zeroed once, kept ready by the calls
        tx = np.ascontiguousarray(np.asarray(tx_pos, dtype=np.float64).astype(np.float32))
        amp0 = tx_power / (self.tx_num_rays if amp_rays is None else amp_rays)
        check(lib().rt_trace_cir(self.env.handle, tx.ctypes.data, rx_mesh.handle if rx_mesh is not None else None,
                                 self.max_bounces, int(ray_offset), n, ptr(traced), ptr(received), ptr(mask),
                                 float(amp0), float(self.light_speed_mps), float(self.sample_rate_hz),
                                 cir_flags(self.light_speed_mps, self.sample_rate_hz), impulse_response.numel(),
                                 ptr(impulse_response), ptr(index), ptr(count), ptr(self._tc_ws),
                                 self._tc_ws.numel(), _lib.stream_handle(self.device)), "rt_trace_cir")
        return index, count

    def _trace_and_cir(self, tx_pos, rx_mesh, received, mask, tx_power, ir, traced=None, ray_offset=0, n=None):
        """tracer.py:75-117 on the device for a burst of any size: the fused rt_trace_cir up to
        TRACE_CIR_MAX_RAYS rays, else rt_trace then rt_compact + rt_cir (ir must be zero; rt_cir adds
        the paths in ray order).  Returns (index, count) device tensors of the received rows."""
        n = self.tx_num_rays if n is None else int(n)
        if n <= self.TRACE_CIR_MAX_RAYS:
            return self.trace_cir_device(tx_pos, rx_mesh, received, mask, tx_power, ir, traced=traced,
                                         ray_offset=ray_offset, n=n)
        self.trace_device(tx_pos, rx_mesh, received, mask, traced=traced, ray_offset=ray_offset, n=n)
        return self.cir_device(received, mask, tx_power, ir, n=n)

    def n_bins(self) -> int:
        return int(self.sample_window_s * self.sample_rate_hz)  # tracer.py:101

    # tracer.py:63-121
    def compute_cir(self, tx_pos, tx_power, rx_pos, rx_radius):
        import torch

        start_time = time.perf_counter()
        dev = f"cuda:{self.device}"
        N, P = self.tx_num_rays, self.max_bounces + 1
        rx_mesh = self._generate_rx_mesh(rx_pos, rx_radius)
        received = torch.empty((N, P, 3), dtype=torch.float32, device=dev)
        mask = torch.empty(N, dtype=torch.int32, device=dev)  # uint32 row_mask bits
        ir = torch.zeros(self.n_bins(), dtype=torch.float64, device=dev)
        if self.max_bounces > 8:
            traced = torch.empty((N, P, 3), dtype=torch.float32, device=dev)
        else:
            traced = None  # scratch in the reference (Q6); kept in registers here
        index, count = self._trace_and_cir(tx_pos, rx_mesh, received, mask, tx_power, ir, traced=traced)
        k = int(count.item())  # synchronises (tracer.py:80)
        rows = received.index_select(0, index[:k]).cpu().numpy() if k else np.zeros((0, P, 3), np.float32)
        cleaned_paths = []
        for row in rows:  # tracer.py:90-97
            bad = np.isnan(row).any(axis=1)
            L = int(np.argmax(bad)) if bad.any() else P
            cleaned_paths.append(np.array(row[:L]))
        impulse_response = ir.cpu().numpy()
        if self.verbose:
            print(f"Traced {len(cleaned_paths)} paths in {time.perf_counter() - start_time} seconds")
        rx_mesh.close()
        return cleaned_paths, impulse_response

    def compute_cir_distributed(self, tx_pos, tx_power, rx_pos, rx_radius, group=None):
        """``compute_cir`` with the burst sharded over the ranks of ``group``.

        Rank r traces the global ray ids [N*r/world, N*(r+1)/world): ids are global (kernel.py:48-51),
        so every ray's path is the one the single-GPU call traces, and each path keeps amplitude
        tx_power / N.  The impulse responses are sum-reduced (RCCL on an "nccl" group, host tensors on
        gloo) and the received rows are gathered in rank order, which is ray-id order.  Every rank
        returns the same (cleaned_paths, impulse_response) as ``compute_cir`` (bins exactly; each
        bin's amplitude up to the order of its f64 sum).
        """
        import torch
        import torch.distributed as dist

        # collectives run with this tracer's GPU current: under "nccl" (RCCL) a collective uses
        # the current device, which must be the device of the tensors it moves
        with torch.cuda.device(self.device):
            return self._compute_cir_distributed(tx_pos, tx_power, rx_pos, rx_radius, group)

    def _compute_cir_distributed(self, tx_pos, tx_power, rx_pos, rx_radius, group):
        import torch
        import torch.distributed as dist

        rank, world = dist.get_rank(group), dist.get_world_size(group)
        dev = f"cuda:{self.device}"
        N, P = self.tx_num_rays, self.max_bounces + 1
        lo, hi = N * rank // world, N * (rank + 1) // world
        n = hi - lo
        rx_mesh = self._generate_rx_mesh(rx_pos, rx_radius)
        received = torch.empty((max(n, 1), P, 3), dtype=torch.float32, device=dev)
        mask = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        ir = torch.zeros(self.n_bins(), dtype=torch.float64, device=dev)
        traced = torch.empty((max(n, 1), P, 3), dtype=torch.float32, device=dev) if self.max_bounces > 8 else None
        k = 0
        rows = np.zeros((0, P, 3), np.float32)
        if n > 0:
            index, count = self._trace_and_cir(tx_pos, rx_mesh, received, mask, tx_power, ir, traced=traced,
                                               ray_offset=lo, n=n)
            k = int(count.item())
            if k:
                rows = received.index_select(0, index[:k]).cpu().numpy()
        wire = ir.to(rdist.wire_device(group, self.device))
        dist.all_reduce(wire, group=group)
        impulse_response = wire.cpu().numpy()
        parts = rdist.gather_rows(rows, group, self.device)
        cleaned_paths = []
        for part in parts:
            for row in part:  # tracer.py:90-97
                bad = np.isnan(row).any(axis=1)
                L = int(np.argmax(bad)) if bad.any() else P
                cleaned_paths.append(np.array(row[:L]))
        rx_mesh.close()
        return cleaned_paths, impulse_response

