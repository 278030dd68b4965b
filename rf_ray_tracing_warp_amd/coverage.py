"""Coverage map: the reference's coverage.py on the device.

coverage.py:38-57 loops over receiver positions, runs ``Tracer.compute_cir`` for each and turns the
impulse response into a received signal power (coverage.py:45-52), then dBm.  ``Coverage`` computes
the same per-cell power for a whole lattice of receivers in one shot (csrc/coverage.hip, exact
shared-trajectory algorithm).  Across ranks (one process per GPU) the work is split either by rays
(``shard_mode="rays"``: every rank traces its share of each cell's
rays, records go to the cells' owners in one sparse all-to-all) or by cells (``"cells"``: every
rank traces all rays for its x columns); "sectors" (the default of ``coverage_map``) is "rays" with
each rank's rays chosen as four interleaved wedges of initial azimuth instead of an id range.  The
power map is then gathered over the process group (RCCL over xGMI with the "nccl" backend).

    grid = CoverageGrid.from_ranges(range(-15, 16, 2), range(-15, 16, 2), range(0, 16, 2))  # coverage.py:38-40
    cov = Coverage(mesh, 2.998e8, 100e9, 100e-9, max_bounces=2, tx_num_rays=1_000_000, grid=grid)
    power = cov.run(tx_pos=(10, 0, 5), tx_power=1)        # (nz, ny, nx) float64 watts, NaN = no path
    dbm = to_dbm(power)
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib
from . import dist as rdist
from ._lib import DeviceMesh, check, lib, ptr
from .power import CARRIER_HZ, to_dbm
from .tracer import cir_flags

__all__ = ["CoverageGrid", "Coverage", "coverage_points", "phase_step"]


class _Grid(ctypes.Structure):
    _fields_ = [("x0", ctypes.c_double), ("y0", ctypes.c_double), ("z0", ctypes.c_double),
                ("dx", ctypes.c_double), ("dy", ctypes.c_double), ("dz", ctypes.c_double),
                ("nx", ctypes.c_int64), ("ny", ctypes.c_int64), ("nz", ctypes.c_int64)]


@dataclass(frozen=True)
class CoverageGrid:
    """Receiver lattice: cell (i,j,k) centre = (x0 + i*dx, y0 + j*dy, z0 + k*dz) in float64."""

    x0: float
    y0: float
    z0: float
    dx: float
    dy: float
    dz: float
    nx: int
    ny: int
    nz: int

    @classmethod
    def from_ranges(cls, xs, ys, zs):
        """From three arithmetic progressions (e.g. the range() loops of coverage.py:38-40)."""
        def ap(v):
            v = list(v)
            step = float(v[1] - v[0]) if len(v) > 1 else 1.0
            if any(abs((v[i] - v[0]) - i * step) > 1e-12 * max(1.0, abs(step) * len(v)) for i in range(len(v))):
                raise ValueError("coverage grid axes must be arithmetic progressions")
            return float(v[0]), step, len(v)
        (x0, dx, nx), (y0, dy, ny), (z0, dz, nz) = ap(xs), ap(ys), ap(zs)
        return cls(x0, y0, z0, dx, dy, dz, nx, ny, nz)

    @classmethod
    def square(cls, n, half_extent, z):
        """n x n cells covering [-h, h]^2 at height z, centres -h + (i + 1/2) * 2h/n."""
        d = 2.0 * half_extent / n
        return cls(-half_extent + 0.5 * d, -half_extent + 0.5 * d, float(z), d, d, 1.0, n, n, 1)

    @property
    def num_cells(self) -> int:
        return self.nx * self.ny * self.nz

    def centers(self) -> np.ndarray:
        """(nz, ny, nx, 3) float64 centres, the exact doubles the device uses."""
        i = np.arange(self.nx, dtype=np.float64)
        j = np.arange(self.ny, dtype=np.float64)
        k = np.arange(self.nz, dtype=np.float64)
        X = self.x0 + i * self.dx
        Y = self.y0 + j * self.dy
        Z = self.z0 + k * self.dz
        out = np.empty((self.nz, self.ny, self.nx, 3))
        out[..., 0] = X[None, None, :]
        out[..., 1] = Y[None, :, None]
        out[..., 2] = Z[:, None, None]
        return out

    def _c(self):
        return _Grid(self.x0, self.y0, self.z0, self.dx, self.dy, self.dz, self.nx, self.ny, self.nz)


def phase_step(sample_window_s, n_bins) -> float:
    """Phase of np.sin(2*np.pi*2.4e9*np.linspace(0, window, n)) per sample (coverage.py:45-46)."""
    return (2 * np.pi * CARRIER_HZ) * (sample_window_s / (n_bins - 1))


class Coverage:
    """All receiver cells of ``grid`` for one transmitter: coverage.py:38-57 in one device pass."""

    def __init__(self, environment_trimesh, light_speed_mps, sample_rate_hz, sample_window_s, max_bounces,
                 tx_num_rays, grid: CoverageGrid, rx_radius=0.1, device: int | None = None, shard_index: int = 0,
                 shard_count: int = 1, env_mesh: DeviceMesh | None = None, shard_mode: str = "cells"):
        """shard_index / shard_count: this rank of the job.  shard_mode "cells": this rank traces all
        tx_num_rays rays for the cells of its x columns (ix % shard_count == shard_index); "rays":
        it traces its contiguous share of the rays (dist.ray_range) for every cell and exchanges
        records with the other ranks in run() (dist.exchange_rows); "sectors": as "rays", with the
        rank's rays a wedge of initial azimuth (rt_coverage_create_sectors) instead of an id range."""
        import torch

        if not torch.cuda.is_available():
            raise _lib.RfrtError("Coverage needs a ROCm GPU (librfrt has no CPU path)")
        # one process per GPU: LOCAL_RANK under torchrun, else the current device
        self.device = rdist.default_device() if device is None else int(device)
        self.light_speed_mps = light_speed_mps
        self.sample_rate_hz = sample_rate_hz
        self.sample_window_s = sample_window_s
        self.max_bounces = int(max_bounces)
        self.tx_num_rays = int(tx_num_rays)
        self.grid = grid
        self.rx_radius = float(rx_radius)
        self.n_bins = int(sample_window_s * sample_rate_hz)
        self.shard_index, self.shard_count = int(shard_index), int(shard_count)
        if shard_mode not in ("cells", "rays", "sectors"):
            raise ValueError(f"shard_mode must be 'cells', 'rays' or 'sectors', not {shard_mode!r}")
        self.shard_mode = shard_mode
        self.env = env_mesh or DeviceMesh(environment_trimesh.vertices, environment_trimesh.faces, self.device)
        self._h = _lib._vp()
        g = grid._c()
        if shard_mode == "sectors":  # ray shards by initial azimuth (rt_coverage_create_sectors)
            self.ray_offset, self.ray_count = 0, rdist.ray_range(self.shard_index, self.shard_count, self.tx_num_rays)[1]
            check(lib().rt_coverage_create_sectors(self.device, self.env.handle, self.max_bounces, self.tx_num_rays,
                                                   ctypes.byref(g), self.rx_radius, self.shard_index, self.shard_count,
                                                   ctypes.byref(self._h)), "rt_coverage_create_sectors")
        elif shard_mode == "rays":
            self.ray_offset, self.ray_count = rdist.ray_range(self.shard_index, self.shard_count, self.tx_num_rays)
            check(lib().rt_coverage_create_rays(self.device, self.env.handle, self.max_bounces, self.tx_num_rays,
                                                self.ray_offset, self.ray_count, ctypes.byref(g), self.rx_radius,
                                                self.shard_index, self.shard_count, ctypes.byref(self._h)),
                  "rt_coverage_create_rays")
        else:
            self.ray_offset, self.ray_count = 0, self.tx_num_rays
            check(lib().rt_coverage_create(self.device, self.env.handle, self.max_bounces, self.tx_num_rays, 0,
                                           ctypes.byref(g), self.rx_radius, self.shard_index, self.shard_count,
                                           ctypes.byref(self._h)), "rt_coverage_create")
        self.power = torch.empty(grid.num_cells, dtype=torch.float64, device=f"cuda:{self.device}")
        self.last_candidates = 0
        self.last_first_wins = 0

    def trace_rows(self, tx_pos, tx_power=1):
        """Ray mode, stage 1: this rank's rays for every cell, as one (n, 4) int64 row per record
        (key = cell << 32 | bin, then the amplitudes summed per (cell, bin) over this rank's rays as
        exact fixed point: 192-bit unsigned, unit 2^-136, least significant word first;
        include/rfrt.h), grouped by owner rank -- the layout exchange_rows sends as it is and
        power_from_rows takes.  Returns (rows, counts), counts[d] rows for rank d; rows is a view of
        this plan's buffer, overwritten by its next call.  trace_rows_async + trace_rows_finish."""
        self.trace_rows_async(tx_pos, tx_power)
        return self.trace_rows_finish()

    def trace_rows_async(self, tx_pos, tx_power=1):
        """trace_rows without the host wait: queues the trace stage on the current stream and returns
        the device (world,) int64 send counts; trace_rows_finish() then waits once and returns
        (rows, counts) as trace_rows does.  Between the two a rank queues the all-to-all of the
        counts (run_device, "nccl"), so one host wait serves the send and the receive counts."""
        import torch

        if self.shard_mode not in ("rays", "sectors"):
            raise _lib.RfrtError("trace_rows_async needs shard_mode 'rays' or 'sectors'")
        tx = np.ascontiguousarray(np.asarray(tx_pos, dtype=np.float64).astype(np.float32))
        dev = f"cuda:{self.device}"
        if getattr(self, "_rows", None) is None:
            self._rows = torch.empty((max(self.ray_count * 2, 1 << 16), 4), dtype=torch.int64, device=dev)
        if getattr(self, "_send_counts", None) is None:
            self._send_counts = torch.empty(self.shard_count, dtype=torch.int64, device=dev)
        check(lib().rt_coverage_trace_rows_async(
            self._h, tx.ctypes.data, float(tx_power), float(self.light_speed_mps), float(self.sample_rate_hz),
            cir_flags(self.light_speed_mps, self.sample_rate_hz), self.n_bins, ptr(self._rows), self._rows.shape[0],
            ptr(self._send_counts), _lib.stream_handle(self.device)), "rt_coverage_trace_rows_async")
        return self._send_counts

    def trace_rows_finish(self):
        """The host half of trace_rows_async: waits for the current stream; (rows, counts)."""
        import torch

        counts = np.zeros(self.shard_count, np.int64)
        stats = np.zeros(3, np.int64)
        check(lib().rt_coverage_trace_rows_finish(self._h, counts.ctypes.data, stats.ctypes.data,
                                                  _lib.stream_handle(self.device)), "rt_coverage_trace_rows_finish")
        n = int(counts.sum())
        rows = self._rows
        if n and not stats[2]:
            self._rows = rows = torch.empty((n + n // 4 + 1024, 4), dtype=torch.int64, device=rows.device)
            check(lib().rt_coverage_records_packed(self._h, ptr(rows), rows.shape[0], _lib.stream_handle(self.device)),
                  "rt_coverage_records_packed")
        self.last_candidates = int(stats[0])
        self.last_first_wins = int(stats[1])
        return rows[:n], [int(c) for c in counts]

    def power_from_rows(self, rows, counts=None):
        """Ray mode, last stage: the power of this rank's cells from (n, 4) int64 rows of
        trace_rows' layout; the (num_cells,) float64 device map, 0 elsewhere.  counts: the rows
        arrive as consecutive segments, counts[t] from rank t (exchange_rows' output), each in
        trace_rows' order (strictly ascending keys): the segments are merged, not sorted
        (rt_coverage_power_packed).  The merge counts keys out of order, and check() (run() calls it)
        raises on them: that map is wrong.  Without counts the rows may come in any order, with
        repeated keys summed exactly (rt_coverage_power_rows: sorted)."""
        import torch
        n = int(rows.shape[0]) if rows.dim() == 2 else 0
        if n and (tuple(rows.shape) != (n, 4) or not rows.is_contiguous() or rows.dtype != torch.int64):
            raise ValueError(f"rows must be a contiguous (n, 4) int64 tensor, got {tuple(rows.shape)} {rows.dtype}")
        alpha = phase_step(self.sample_window_s, self.n_bins)
        s = _lib.stream_handle(self.device)
        if counts is None:
            check(lib().rt_coverage_power_rows(self._h, ptr(rows) if n else None, n, self.n_bins, alpha,
                                               ptr(self.power), s), "rt_coverage_power_rows")
            return self.power
        c = np.ascontiguousarray(np.asarray(counts, dtype=np.int64))
        if int(c.sum()) != n or (c < 0).any():
            raise ValueError(f"segment counts {c.tolist()} do not add up to the {n} rows")
        check(lib().rt_coverage_power_packed(self._h, ptr(rows) if n else None, c.ctypes.data, len(c), self.n_bins,
                                             alpha, ptr(self.power), s), "rt_coverage_power_packed")
        return self.power

    def power_from_amplitudes(self, keys, amps):
        """power_from_rows for (cell << 32 | bin) int64 keys with float64 amplitudes, in any order
        (e.g. per-cell impulse responses computed elsewhere): packed into rows with their exact
        fixed-point sums on the device first."""
        import torch
        n = int(keys.numel())
        rows = torch.empty((n, 4), dtype=torch.int64, device=keys.device)
        if n:
            rows[:, 0] = keys.reshape(-1).to(torch.int64)
            rows[:, 1:] = amps_to_sums(amps.reshape(-1))
        return self.power_from_rows(rows)

    def run_device(self, tx_pos, tx_power=1, process_group=None):
        """Launch; returns the (num_cells,) float64 device tensor (0 for cells of other shards).
        Ray mode with more than one shard exchanges records over ``process_group`` here."""
        import torch
        with torch.cuda.device(self.device):  # collectives (RCCL) use the current device
            return self._run_device(tx_pos, tx_power, process_group)

    def _run_device(self, tx_pos, tx_power, process_group):
        if self.shard_mode in ("rays", "sectors"):
            if self.shard_count > 1 and rdist.device_collectives(process_group):
                # RCCL: the counts' all-to-all is queued behind the trace stage, and one host wait
                # (trace_rows_finish) returns the send and the receive counts together
                sc = self.trace_rows_async(tx_pos, tx_power)
                rc = rdist.exchange_counts_async(sc, process_group)
                rows, counts = self.trace_rows_finish()
                rows, counts = rdist.exchange_rows(rows, counts, process_group, recv_counts=rc.tolist())
                return self.power_from_rows(rows, counts)
            rows, counts = self.trace_rows(tx_pos, tx_power)
            if self.shard_count > 1:
                rows, counts = rdist.exchange_rows(rows, counts, process_group)
            return self.power_from_rows(rows, counts)
        tx = np.ascontiguousarray(np.asarray(tx_pos, dtype=np.float64).astype(np.float32))
        stats = np.zeros(2, np.int64)
        check(lib().rt_coverage_run(self._h, tx.ctypes.data, float(tx_power), float(self.light_speed_mps),
                                    float(self.sample_rate_hz), cir_flags(self.light_speed_mps, self.sample_rate_hz),
                                    self.n_bins, phase_step(self.sample_window_s, self.n_bins), ptr(self.power),
                                    stats.ctypes.data, _lib.stream_handle(self.device)), "rt_coverage_run")
        self.last_candidates = int(stats[0])
        self.last_first_wins = int(stats[1])
        return self.power

    def check(self):
        """Raise if the device flagged this plan's earlier asynchronous stages (rt_coverage_check: a
        look-back wait that gave up, or an owner-stage segment out of key order -- those results
        are wrong).  Synchronizes the plan's stream; run() calls it after every map."""
        out = np.zeros(2, np.int64)
        check(lib().rt_coverage_check(self._h, out.ctypes.data, _lib.stream_handle(self.device)), "rt_coverage_check")

    def run(self, tx_pos, tx_power=1, process_group=None):
        """Power map (nz, ny, nx) float64 on the host; with a process group, sum-reduced over ranks."""
        import torch
        p = self.run_device(tx_pos, tx_power, process_group)
        self.check()
        if process_group is not None or self.shard_count > 1:
            import torch.distributed as dist
            with torch.cuda.device(self.device):
                if (dist.get_world_size(process_group), dist.get_rank(process_group)) == \
                        (self.shard_count, self.shard_index):
                    # owners hold disjoint x columns: the sum-reduce is an all-gather of them
                    p = rdist.gather_power_map(p, self.grid.nx, process_group)
                else:
                    wire = p.to(rdist.wire_device(process_group, self.device))
                    dist.all_reduce(wire, group=process_group)
                    p = wire
        g = self.grid
        return p.cpu().numpy().reshape(g.nz, g.ny, g.nx)

    def impulse_responses(self):
        """Sparse per-cell impulse responses of the last run: (cell, bin, amplitude) arrays."""
        import torch

        n = ctypes.c_int64()
        check(lib().rt_coverage_received(self._h, None, None, 0, ctypes.byref(n), _lib.stream_handle(self.device)),
              "rt_coverage_received")
        m = n.value
        dev = f"cuda:{self.device}"
        keys = torch.empty(max(m, 1), dtype=torch.int64, device=dev)
        amps = torch.empty(max(m, 1), dtype=torch.float64, device=dev)
        check(lib().rt_coverage_received(self._h, ptr(keys), ptr(amps), m, ctypes.byref(n),
                                         _lib.stream_handle(self.device)), "rt_coverage_received")
        k = keys[:m].cpu().numpy().view(np.uint64)
        return (k >> np.uint64(32)).astype(np.int64), (k & np.uint64(0xFFFFFFFF)).astype(np.int64), \
            amps[:m].cpu().numpy()

    PROFILE_KEYS = ("traj_ms", "candidates_ms", "win_ms", "replay_ms", "reduce_power_ms", "total_ms",
                    "traced_ray_bounces", "replayed_ray_bounces", "candidates", "records")

    def profile(self, enable=True):
        """Record HIP events around this plan's kernels on every later run (rt_coverage_profile)."""
        check(lib().rt_coverage_profile(self._h, 1 if enable else 0), "rt_coverage_profile")

    def last_profile(self):
        """Stage times (ms, GPU events) and work counts of the last run: PROFILE_KEYS -> value."""
        out = np.zeros(10, np.float64)
        check(lib().rt_coverage_last_profile(self._h, out.ctypes.data, 10), "rt_coverage_last_profile")
        return dict(zip(self.PROFILE_KEYS, (float(x) for x in out)))

    def close(self):
        if getattr(self, "_h", None) and self._h.value and _lib._lib is not None:
            _lib._lib.rt_coverage_destroy(self._h)
            self._h = _lib._vp()

    def __del__(self):
        self.close()


def amps_to_sums(amps):
    """float64 device amplitudes (finite, >= 0) -> (n, 3) int64 exact fixed-point sums
    (rt_coverage_amps_to_sums: 192-bit unsigned, unit 2^-136)."""
    import torch
    n = int(amps.numel())
    sums = torch.empty((max(n, 1), 3), dtype=torch.int64, device=amps.device)
    a = amps.contiguous().to(torch.float64)
    check(lib().rt_coverage_amps_to_sums(ptr(a) if n else None, n, ptr(sums) if n else None,
                                         _lib.stream_handle(amps.device.index)), "rt_coverage_amps_to_sums")
    return sums[:n]


def coverage_points(power_map, grid: CoverageGrid):
    """(rx_pos, dBm) pairs in coverage.py's loop order (x outer, then y, then z; coverage.py:38-57)."""
    c = grid.centers()
    out = []
    for i in range(grid.nx):
        for j in range(grid.ny):
            for k in range(grid.nz):
                out.append((c[k, j, i], float(to_dbm(power_map[k, j, i]))))
    return out


def _dist_shard():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def coverage_map(environment_trimesh, tx_pos, grid: CoverageGrid, light_speed_mps=2.998e8, sample_rate_hz=100e9,
                 sample_window_s=100e-9, max_bounces=2, tx_num_rays=1_000_000, tx_power=1, rx_radius=0.1,
                 device=None, shard_mode="sectors"):
    """coverage.py as a function.  Under torch.distributed the work is sharded over the ranks (by
    rays with a record all-to-all, or by x columns of cells) and the power map is all-reduced;
    every rank returns the full map."""
    rank, world = _dist_shard()
    cov = Coverage(environment_trimesh, light_speed_mps, sample_rate_hz, sample_window_s, max_bounces, tx_num_rays,
                   grid, rx_radius, device=device, shard_index=rank, shard_count=world,
                   shard_mode=shard_mode if world > 1 else "cells")
    try:
        return cov.run(tx_pos, tx_power)
    finally:
        cov.close()
