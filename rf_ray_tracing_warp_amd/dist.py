"""Multi-GPU plumbing: one process per GPU, torch.distributed ("nccl" = RCCL over xGMI on ROCm).

Decompositions:
* rays  -- rank r traces global ray ids [r*n, (r+1)*n) (Warp tid = global id, kernel.py:48-51, so
  every ray's path is independent of the shard); the impulse response is the sum over shards,
  amplitude tx_power / (n * world) per ray (tracer.py:103): ``reduce_sum``.
* cells -- coverage cells whose x column ix = cell % nx satisfies ix % world == rank belong to
  rank (x-column cyclic: a strip of constant ix is wholly one rank's, so the candidate passes
  shrink with the rank count); every other rank leaves 0 in its power map and the maps are
  sum-reduced: ``reduce_sum`` again (NaN of an owner survives).
* coverage rays -- rank r traces its share of every cell's rays (``ray_range``, or a wedge of
  initial azimuth for "sectors" plans), sums its first-win records per (cell, bin) and sends each
  record, one 32-B (key, exact sum) row, to the owner of its cell (the x-column rule above):
  ``exchange_rows``, one sparse all-to-all.  Owners sum what they receive (exact fixed point, so
  the order is irrelevant), compute their cells' power, and the maps are gathered
  (``gather_power_map``).
"""
from __future__ import annotations

import os


def default_device():
    """The GPU of this process: LOCAL_RANK under torchrun (one process per GPU), else the current
    device.  Never the global rank, which exceeds the local GPU count beyond one node."""
    import torch
    lr = os.environ.get("LOCAL_RANK")
    if lr is not None:
        return int(lr)
    return torch.cuda.current_device()


def wire_device(group, device):
    """Where tensors of a collective live: the process's GPU for "nccl" (RCCL), the host for gloo."""
    import torch
    import torch.distributed as dist
    if dist.get_backend(group) == "nccl":
        return torch.device(f"cuda:{int(device)}")
    return torch.device("cpu")


def gather_rows(rows, group=None, device=0):
    """All-gather of variable-length row blocks (numpy (k, ...) float32 arrays, one per rank):
    a counts all-gather, then one padded tensor all-gather.  Returns the list of every rank's rows
    in rank order.  Replaces dist.all_gather_object (which pickles, and under "nccl" stages the
    pickles on whatever device is current)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    wire = wire_device(group, device)
    rows = np.ascontiguousarray(rows, dtype=np.float32)
    shape = rows.shape[1:]
    cnt = torch.tensor([rows.shape[0]], dtype=torch.int64, device=wire)
    counts = [torch.empty_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt, group=group)
    counts = [int(c.item()) for c in counts]
    m = max(max(counts), 1)
    buf = torch.full((m,) + shape, float("nan"), dtype=torch.float32, device=wire)
    if rows.shape[0]:
        buf[:rows.shape[0]] = torch.from_numpy(rows).to(wire)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    return [p[:c].cpu().numpy() for p, c in zip(parts, counts)]


def rank_world(group=None):
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def ray_shard(rank: int, world: int, rays_per_rank: int):
    """(ray_offset, count) of this rank's global ray ids."""
    return rank * rays_per_rank, rays_per_rank


def ray_range(rank: int, world: int, n_total: int):
    """(ray_offset, count) of rank's share of one burst of n_total rays (contiguous, balanced)."""
    lo = rank * n_total // world
    return lo, (rank + 1) * n_total // world - lo


def owns_cell(cell: int, rank: int, world: int, nx: int) -> bool:
    """Cell ownership used by rt_coverage_run (csrc/coverage.hip: ix % nshard == shard, ix = cell % nx)."""
    return (cell % nx) % world == rank


def reduce_sum(t, group=None):
    """In-place sum over the ranks (CIR bins or a zero-padded power map)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def gather_power_map(p, nx: int, group=None):
    """The coverage power map on every rank from the ranks' owned x columns (ix % world == rank,
    zero elsewhere): the sum-reduce of such maps is an all-gather of the owned columns, half the
    bytes of an all-reduce (K5: 1 MB per rank instead of the 8-MB map through a reduce-scatter
    and an all-gather).  p: (num_cells,) float64, cell = row * nx + ix.  Returns a new tensor on
    p's device, equal bit for bit to all_reduce(p) (every cell has exactly one non-zero source;
    NaN of an owner survives)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if world == 1:
        return p
    home = p.device
    wire = wire_device(group, home.index if home.type == "cuda" else 0)
    rows = p.numel() // nx
    w = (nx + world - 1) // world  # owned columns per rank, padded
    full = p.reshape(rows, nx)
    if w * world != nx:
        full = torch.nn.functional.pad(full, (0, w * world - nx))
    mine = full.reshape(rows, w, world)[:, :, rank].contiguous().to(wire)  # column q of mine = ix q*world + rank
    out = torch.empty((world, rows, w), dtype=p.dtype, device=wire)
    if hasattr(dist, "all_gather_into_tensor") and dist.get_backend(group) != "gloo":
        dist.all_gather_into_tensor(out, mine, group=group)
    else:
        dist.all_gather(list(out.unbind(0)), mine, group=group)
    # full[row, q*world + d] = out[d, row, q]
    return out.to(home).permute(1, 2, 0).reshape(rows, w * world)[:, :nx].reshape(-1)


def reduce_max(value: float, device, group=None) -> float:
    """Max of a scalar over the ranks (bench timing: the slowest rank defines the step)."""
    import torch
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        t = torch.tensor([value], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        return float(t[0])
    return value


def device_collectives(group=None):
    """True when the group's collectives run on the GPU ("nccl" = RCCL): device tensors go in
    as they are and the collectives are queued on the stream (gloo stages through the host)."""
    import torch.distributed as dist
    return dist.get_backend(group) == "nccl"


def exchange_counts_async(send_counts_dev, group=None):
    """All-to-all of the per-destination send counts, queued on the device (RCCL) behind the trace
    stage that wrote them (Coverage.trace_rows_async).  Returns the receive counts in pinned host
    memory, filled once the current stream reaches this point: read them after the stream has
    been waited for (Coverage.trace_rows_finish does), so one host wait serves both counts."""
    import torch
    import torch.distributed as dist
    rc = torch.empty_like(send_counts_dev)
    dist.all_to_all_single(rc, send_counts_dev, group=group)
    host = torch.empty(rc.shape, dtype=rc.dtype, pin_memory=True)
    host.copy_(rc, non_blocking=True)
    return host


def exchange_rows(rows, send_counts, group=None, recv_counts=None):
    """Sparse all-to-all of packed coverage records: rows (n, w) int64 grouped by destination rank,
    send_counts[d] rows for rank d (Coverage.trace_rows).  One collective for the counts, one for
    the rows, nothing packed or unpacked around them.  Returns (received rows, in source-rank order;
    the number of rows from each rank).  recv_counts: the receive counts when the caller has them
    already (exchange_counts_async), so only the rows move here.
    The host needs the receive counts before the rows move: all_to_all_single takes its split sizes
    and the output's size on the host (there is no device-side split form), so either this
    function reads them (one blocking read) or the caller reads them in the same wait as its own
    send counts (run_device on "nccl")."""
    import torch
    import torch.distributed as dist
    home = rows.device
    wire = torch.device("cpu") if (home.type != "cpu" and dist.get_backend(group) == "gloo") else home
    send_counts = [int(c) for c in send_counts]
    n = sum(send_counts)
    w = int(rows.shape[1]) if rows.dim() == 2 else 4
    if recv_counts is None:
        sc = torch.tensor(send_counts, dtype=torch.int64, device=wire)
        rc = torch.empty_like(sc)
        dist.all_to_all_single(rc, sc, group=group)
        recv_counts = rc.tolist()
    recv_counts = [int(c) for c in recv_counts]
    out = torch.empty((sum(recv_counts), w), dtype=torch.int64, device=wire)
    dist.all_to_all_single(out, rows[:n].reshape(n, w).to(wire), recv_counts, send_counts, group=group)
    return out.to(home), recv_counts
