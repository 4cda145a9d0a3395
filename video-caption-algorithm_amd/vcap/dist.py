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
    """[B_local, L] int32 per rank -> [world * B_local, L] on every rank (equal B_local per rank).
    A single process without a process group returns `local`; an initialised group of one rank
    still runs the collective (the RCCL path of a one-GPU job)."""
    if world == 1 and not (dist.is_available() and dist.is_initialized()):
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


def caption_sharded(model, videos: torch.Tensor, prompt_ids, *, cfg=None, ln_scale: float = 0.6,
                    in_weight: float = 0.4, group=None, device=None) -> torch.Tensor:
    """Data-parallel captioning of a global batch (BASELINE configs[2]).

    Every rank holds (or can index) the same global `videos` [N, T, 3, H, W] (host or device); rank
    r encodes + decodes only its contiguous shard `shard_range(N, W, r)` with its replicated
    weights (`model.generate_ids`, HipVideoCaptionModel's fused encode + greedy decode graph), and
    ONE all-gather of the int32 ids (RCCL over xGMI on "nccl", gloo host copies otherwise) gives
    every rank the [N, max_new] ids in global order.  Uneven shards are padded to the largest
    shard for the gather and trimmed after it; no data-path collective exists besides that one."""
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    rank = dist.get_rank(group) if world > 1 else 0
    n = int(videos.shape[0])
    lo, hi = shard_range(n, world, rank)
    per = -(-n // world)                       # largest shard
    dev = torch.device(device) if device is not None else getattr(model, "device", videos.device)
    kw = {"ln_scale": ln_scale, "in_weight": in_weight}
    if cfg is not None:
        kw["cfg"] = cfg
    if hi > lo:
        ids = model.generate_ids(videos[lo:hi].to(dev), list(prompt_ids), **kw).to(torch.int32)
    else:                                       # more ranks than videos: an empty shard
        L = cfg.max_new_tokens if cfg is not None else 24
        ids = torch.empty(0, L, dtype=torch.int32, device=dev)
    local = torch.full((per, ids.shape[1]), -1, dtype=torch.int32, device=dev)
    local[:hi - lo] = ids
    full = gather_ids(local, world, group)      # [world * per, L]
    keep = torch.cat([torch.arange(*shard_range(n, world, r)) - shard_range(n, world, r)[0] + r * per
                      for r in range(world)]).to(full.device)
    return full.index_select(0, keep)
