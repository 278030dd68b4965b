"""Multi-GPU plumbing: one process per GPU, torch.distributed ("nccl" = RCCL over xGMI on ROCm).

Two decompositions:
* rays  -- rank r traces global ray ids [r*n, (r+1)*n) (Warp tid = global id, kernel.py:48-51, so
  every ray's path is independent of the shard); the impulse response is the sum over shards,
  amplitude tx_power / (n * world) per ray (tracer.py:103): ``reduce_sum``.
* cells -- coverage cells whose x column ix = cell % nx satisfies ix % world == rank belong to
  rank (x-column cyclic: a strip of constant ix is wholly one rank's, so the candidate passes
  shrink with the rank count); every other rank leaves 0 in its power map and the maps are
  sum-reduced: ``reduce_sum`` again (NaN of an owner survives).
"""
from __future__ import annotations


def rank_world(group=None):
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def ray_shard(rank: int, world: int, rays_per_rank: int):
    """(ray_offset, count) of this rank's global ray ids."""
    return rank * rays_per_rank, rays_per_rank


def owns_cell(cell: int, rank: int, world: int, nx: int) -> bool:
    """Cell ownership used by rt_coverage_run (csrc/coverage.hip: ix % nshard == shard, ix = cell % nx)."""
    return (cell % nx) % world == rank


def reduce_sum(t, group=None):
    """In-place sum over the ranks (CIR bins or a zero-padded power map)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def reduce_max(value: float, device, group=None) -> float:
    """Max of a scalar over the ranks (bench timing: the slowest rank defines the step)."""
    import torch
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        t = torch.tensor([value], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        return float(t[0])
    return value
