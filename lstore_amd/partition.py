"""Static stripe partitioning across ranks (one process per GPU).

Stripes are independent units (each encode_block call touches one stripe's k+m chunks,
src/lio/segment/jerasure.c:1847), so G GPUs take G contiguous blocks of the stripe index
range and never exchange data.  The only collectives are for measurement: a barrier and a
max-over-ranks reduction of the elapsed time.
"""
from __future__ import annotations


def stripe_range(nstripes: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous block [s0, s1) of rank `rank`; sizes differ by at most one stripe."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(nstripes, world)
    s0 = rank * base + min(rank, extra)
    return s0, s0 + base + (1 if rank < extra else 0)


def max_over_ranks(value: float, device=None) -> float:
    """Max of a float over all ranks (identity when torch.distributed is not initialised)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device if device is not None else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value: int, device=None) -> int:
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.int64, device=device if device is not None else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())
