"""Node-ID range sharding across GPUs (north_star: "The index shards by node-ID
range across up to 8 MI355X GPUs with RCCL all-gather of per-shard top-k").

One process per GPU.  Rank r of W owns the contiguous key range
shard_range(n_total, W, r) and builds an independent sub-graph over it (no
collective during build).  A query batch is searched on every shard; each
rank's (distance, key) top-k lists are packed into one byte buffer and
all-gathered in a single collective (RCCL over xGMI when the tensors live on
the GPU: B*(12k+4) bytes per rank, ~127 KB for B=1024, k=10), then merged per
query by (distance, key) on the GPU with mhnsw_merge_topk_device.  The
reference has no distributed code; this is the only exchange step
on the path.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(n_total: int, world: int, rank: int):
    """Contiguous node-ID range [lo, hi) owned by `rank` (sizes differ by <= 1)."""
    base, rem = divmod(n_total, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def _layout(B: int, k: int):
    """byte offsets of keys | dists | n in one packed list; total padded to 8"""
    o_d = B * k * 8
    o_n = o_d + B * k * 4
    end = o_n + B * 4
    return o_d, o_n, end, (end + 7) // 8 * 8


def pack_topk(keys: torch.Tensor, dists: torch.Tensor, n: torch.Tensor) -> torch.Tensor:
    """(keys int64[B,k], dists f32[B,k], n i32[B]) -> one uint8 buffer"""
    B, k = keys.shape
    o_d, o_n, end, tot = _layout(B, k)
    buf = torch.zeros(tot, dtype=torch.uint8, device=keys.device)
    buf[:o_d].view(torch.int64).copy_(keys.reshape(-1))
    buf[o_d:o_n].view(torch.float32).copy_(dists.reshape(-1))
    buf[o_n:end].view(torch.int32).copy_(n.reshape(-1))
    return buf


def unpack_topk(g: torch.Tensor, B: int, k: int):
    """[W, bytes] gathered buffers -> ([W,B,k] keys, [W,B,k] dists, [W,B] n), contiguous"""
    W = g.shape[0]
    o_d, o_n, end, _ = _layout(B, k)
    ak = g[:, :o_d].contiguous().view(torch.int64).view(W, B, k)
    ad = g[:, o_d:o_n].contiguous().view(torch.float32).view(W, B, k)
    an = g[:, o_n:end].contiguous().view(torch.int32).view(W, B)
    return ak, ad, an


def gather_topk(keys: torch.Tensor, dists: torch.Tensor, n: torch.Tensor, group=None):
    """All-gather per-shard top-k in ONE collective -> ([W,B,k] keys, [W,B,k]
    dists, [W,B] n)."""
    world = dist.get_world_size(group)
    B, k = keys.shape
    buf = pack_topk(keys, dists, n)
    dev = buf.device
    if buf.is_cuda and dist.get_backend(group) == "gloo":
        buf = buf.cpu()  # rehearsal path (several ranks on one device): stage through the host
    out = torch.empty((world, buf.numel()), dtype=torch.uint8, device=buf.device)
    if buf.is_cuda:
        dist.all_gather_into_tensor(out, buf, group=group)
    else:
        dist.all_gather(list(out.unbind(0)), buf, group=group)
    return unpack_topk(out.to(dev), B, k)


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


def engine_local_search(g, k: int, mode: int, ef: int = 0):
    """local_search over a HIP engine handle (hnsw_amd.Graph) on device tensors:
    one mhnsw_search_device on torch's current stream, no host sync (a caller
    that needs the kernels' error word calls g.device_status())."""
    def run(q: torch.Tensor):
        B, d = q.shape
        keys = torch.empty(B, k, dtype=torch.int64, device=q.device)
        dists = torch.empty(B, k, dtype=torch.float32, device=q.device)
        n = torch.empty(B, dtype=torch.int32, device=q.device)
        g.search_device(q.data_ptr(), B, d, k, keys.data_ptr(), dists.data_ptr(), n.data_ptr(), mode=mode, ef=ef,
                        stream=torch.cuda.current_stream().cuda_stream)
        return keys, dists, n
    return run
