"""Data-parallel sharding for the caption path.

Videos are independent: rank r of W processes videos [r*B/W, (r+1)*B/W) with replicated weights,
one process per GPU.  The only exchange is ONE all-gather of the int32 token ids at the end
(RCCL over xGMI with backend "nccl"; list all_gather on gloo for CPU tests)."""
from __future__ import annotations

from typing import Tuple

import torch
import torch.distributed as dist


def shard_range(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, balanced split of n items over world ranks (first n % world ranks get one more)."""
    q, r = divmod(n, world)
    start = rank * q + min(rank, r)
    return start, start + q + (1 if rank < r else 0)


def gather_ids(local: torch.Tensor, world: int, group=None) -> torch.Tensor:
    """[B_local, L] int32 per rank -> [world * B_local, L] on every rank (equal B_local per rank)."""
    if world == 1:
        return local
    if dist.get_backend(group) == "nccl":
        out = torch.empty(world * local.shape[0], *local.shape[1:], dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(out, local.contiguous(), group=group)
        return out
    # gloo (CPU tests, one-GPU rehearsals): gather host copies
    host = local.detach().to("cpu").contiguous()
    parts = [torch.empty_like(host) for _ in range(world)]
    dist.all_gather(parts, host, group=group)
    return torch.cat(parts, dim=0).to(local.device)
