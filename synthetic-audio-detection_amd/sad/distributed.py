"""Multi-GPU sharding of batched segment inference.

Segments are independent: rank r of W takes the contiguous range
``shard_range(n, r, W)``; weights are replicated; the only exchange is ONE
all-gather of the per-segment logits (RCCL over xGMI with the "nccl" backend on
ROCm; gloo in the CPU tests).  Ragged shards are padded to the largest shard so
``all_gather_into_tensor`` moves equal-sized blocks, then trimmed in rank order,
which restores the global segment order exactly.

The reference has no torch.distributed at all (inference is single-device,
inference_runner.py:243); this replaces "run everything on one GPU".
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(n: int, rank: int, world: int):
    """Contiguous [start, stop) of n items for `rank`; sizes differ by <= 1."""
    base, rem = divmod(n, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def gather_rows(local: torch.Tensor, n_total: int, group=None) -> torch.Tensor:
    """All-gather each rank's rows (its shard_range of n_total) into [n_total, ...]
    on every rank."""
    world = dist.get_world_size(group)
    if world == 1:
        return local
    cap = -(-n_total // world)
    pad = torch.zeros((cap,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[:local.shape[0]] = local
    out = torch.empty((world * cap,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    if local.device.type == 'cuda' and dist.get_backend(group) == 'nccl':
        dist.all_gather_into_tensor(out, pad, group=group)
    else:
        dist.all_gather(list(out.chunk(world)), pad, group=group)
    pieces = []
    for r in range(world):
        s, e = shard_range(n_total, r, world)
        pieces.append(out[r * cap:r * cap + (e - s)])
    return torch.cat(pieces)


def infer_sharded(engine, n_total: int, make_pcm, chunk: int = 2048, group=None):
    """Run ``engine`` over this rank's shard of n_total segments and all-gather the
    merged logits.  ``make_pcm(first, count)`` returns int16 [count, 128000] on
    the engine's device for global segments first..first+count-1."""
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    s, e = shard_range(n_total, rank, world)
    outs = []
    for c in range(s, e, chunk):
        cnt = min(chunk, e - c)
        _, merged = engine.forward_pcm(make_pcm(c, cnt))
        outs.append(merged)
    local = torch.cat(outs) if outs else torch.zeros(0, engine.n_heads + 1, device=engine.device)
    return gather_rows(local, n_total, group) if world > 1 else local
