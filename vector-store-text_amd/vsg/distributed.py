"""Row-range sharding across the GPUs of one node.

One process per GPU.  Rank r owns rows [r N/G, (r+1) N/G) in its own HBM
index; build needs no communication.  A query batch is searched on every shard,
the per-shard top-k (B x k keys + distances, ~80 KB per rank at B=1024, k=10)
is all-gathered over RCCL (xGMI) and k-way merged on every rank by the HIP merge
kernel.  Global keys are the caller's u64 keys, so no id translation is needed.

The gloo path (CPU tensors) exists for the multi-process CPU tests and for
rehearsing several ranks on one GPU; the merge of CPU-resident results is a
host-side (distance, key) lexicographic selection, the same order the HIP
kernel uses.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(n: int, rank: int, world: int):
    return rank * n // world, (rank + 1) * n // world


def gather_topk(keys: torch.Tensor, dists: torch.Tensor, group=None):
    """(nq, k) per rank -> (world, nq, k) on every rank."""
    world = dist.get_world_size(group)
    if world == 1:
        return keys.unsqueeze(0), dists.unsqueeze(0)
    if dist.get_backend(group) == "nccl":
        gk = torch.empty((world,) + tuple(keys.shape), dtype=keys.dtype, device=keys.device)
        gd = torch.empty((world,) + tuple(dists.shape), dtype=dists.dtype, device=dists.device)
        dist.all_gather_into_tensor(gk, keys.contiguous(), group=group)
        dist.all_gather_into_tensor(gd, dists.contiguous(), group=group)
        return gk, gd
    kc, dc = keys.cpu().contiguous(), dists.cpu().contiguous()
    lk = [torch.empty_like(kc) for _ in range(world)]
    ld = [torch.empty_like(dc) for _ in range(world)]
    dist.all_gather(lk, kc, group=group)
    dist.all_gather(ld, dc, group=group)
    return torch.stack(lk).to(keys.device), torch.stack(ld).to(dists.device)


def merge_topk(gk: torch.Tensor, gd: torch.Tensor, k: int, stream=None):
    """(parts, nq, k) -> (nq, k), ascending (distance, key); padding key = -1 (u64 max)."""
    if gk.is_cuda:
        from .index import merge_topk_device
        return merge_topk_device(gk.contiguous(), gd.contiguous(), k, stream=stream)
    parts, nq, kk = gk.shape
    keys = gk.permute(1, 0, 2).reshape(nq, parts * kk)
    d = gd.permute(1, 0, 2).reshape(nq, parts * kk).clone()
    if parts * kk < k:  # shards returned fewer candidates than k: pad
        keys = torch.cat([keys, torch.full((nq, k - parts * kk), -1, dtype=keys.dtype)], 1)
        d = torch.cat([d, torch.full((nq, k - parts * kk), float("inf"), dtype=d.dtype)], 1)
    pad = keys == -1
    d[pad] = float("inf")
    # lexicographic (distance, key): stable sort by key (as unsigned), then by distance
    ukey = torch.where(pad, torch.full_like(keys, torch.iinfo(torch.int64).max), keys)
    o1 = torch.argsort(ukey, dim=1, stable=True)
    d1 = torch.gather(d, 1, o1)
    o2 = torch.argsort(d1, dim=1, stable=True)
    order = torch.gather(o1, 1, o2)[:, :k]
    return torch.gather(keys, 1, order), torch.gather(d, 1, order)


def sharded_search(index, queries: torch.Tensor, k: int, ef: int = 0, exact: bool = False,
                   group=None, stream=None, k_shard: int = 0):
    """Search every shard, gather, merge.  `index` is this rank's vsg.Index.
    k_shard (<= k) candidates per shard suffice when the merged recall target
    allows it (each shard holds ~1/G of the true neighbours)."""
    ks = k_shard or k
    keys, dists = index.search_device(queries, ks, ef, stream=stream, exact=exact)
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return keys, dists
    gk, gd = gather_topk(keys, dists, group)
    return merge_topk(gk, gd, k, stream=stream)
