"""Node-ID range sharding across GPUs (north_star: "The index shards by node-ID
range across up to 8 MI355X GPUs with RCCL all-gather of per-shard top-k").

One process per GPU.  Rank r of W owns the contiguous key range
shard_range(n_total, W, r) and builds an independent sub-graph over it (no
collective during build).  A query batch is searched on every shard; each
rank's (distance, key) top-k lists are all-gathered (RCCL over xGMI when the
tensors live on the GPU: B*k*12 bytes per rank, ~120 KB for B=1024, k=10) and
merged per query by (distance, key) -- on the GPU with
mhnsw_merge_topk_device.  The reference has no distributed code;
this is the only exchange step on the path.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(n_total: int, world: int, rank: int):
    """Contiguous node-ID range [lo, hi) owned by `rank` (sizes differ by <= 1)."""
    base, rem = divmod(n_total, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def gather_topk(keys: torch.Tensor, dists: torch.Tensor, n: torch.Tensor, group=None):
    """All-gather per-shard top-k -> ([W,B,k] keys, [W,B,k] dists, [W,B] n)."""
    world = dist.get_world_size(group)
    if keys.is_cuda and dist.get_backend(group) == "gloo":
        # rehearsal path (several ranks on one device): stage through the host
        ak, ad, an = gather_topk(keys.cpu(), dists.cpu(), n.cpu(), group)
        return ak.to(keys.device), ad.to(keys.device), an.to(keys.device)
    if keys.is_cuda:
        ak = torch.empty((world,) + tuple(keys.shape), dtype=keys.dtype, device=keys.device)
        ad = torch.empty((world,) + tuple(dists.shape), dtype=dists.dtype, device=dists.device)
        an = torch.empty((world,) + tuple(n.shape), dtype=n.dtype, device=n.device)
        dist.all_gather_into_tensor(ak, keys.contiguous(), group=group)
        dist.all_gather_into_tensor(ad, dists.contiguous(), group=group)
        dist.all_gather_into_tensor(an, n.contiguous(), group=group)
        return ak, ad, an
    lk = [torch.empty_like(keys) for _ in range(world)]
    ld = [torch.empty_like(dists) for _ in range(world)]
    ln = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(lk, keys.contiguous(), group=group)
    dist.all_gather(ld, dists.contiguous(), group=group)
    dist.all_gather(ln, n.contiguous(), group=group)
    return torch.stack(lk), torch.stack(ld), torch.stack(ln)


def merge_topk(ak: torch.Tensor, ad: torch.Tensor, an: torch.Tensor, k: int):
    """Merge gathered shard lists on the GPU (k_merge via the C ABI)."""
    from .graph import merge_topk_device

    if not ak.is_cuda:
        raise RuntimeError("merge_topk runs on the GPU; gathered tensors must be on a HIP device")
    S, B = an.shape
    ok = torch.empty(B, k, dtype=torch.int64, device=ak.device)
    od = torch.empty(B, k, dtype=torch.float32, device=ak.device)
    on = torch.empty(B, dtype=torch.int32, device=ak.device)
    merge_topk_device(ak.data_ptr(), ad.data_ptr(), an.data_ptr(), S, B, k, ok.data_ptr(), od.data_ptr(),
                      on.data_ptr(), torch.cuda.current_stream().cuda_stream)
    return ok, od, on


def sharded_search(local_search, queries, k: int, group=None, merge=merge_topk):
    """Search every shard with the same queries and merge: local_search(queries)
    -> (keys[B,k] int64, dists[B,k] f32, n[B] i32) with global keys."""
    keys, dists, n = local_search(queries)
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        ak, ad, an = gather_topk(keys, dists, n, group)
        return merge(ak, ad, an, k)
    return keys, dists, n
