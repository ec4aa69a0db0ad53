"""Process-per-GPU sharding of the ray march.

Rays are independent, so inference shards with NO data-path collective: every
rank renders a contiguous range of frames (or of rays) from its own replica of
the MLPs and the latent, and writes its own output.  The only collectives are
control-plane ones: a barrier and an all_reduce(MAX) of the elapsed time for
benchmarking, and an optional gather for callers that want the whole result on
one rank.  This replaces the reference's single-process nn.DataParallel ray
scatter / gather to device 0 (nerf.py:367-371, train/multigpu.py:74).
"""
import os

import torch
import torch.distributed as dist

__all__ = ["shard_range", "env_rank", "init_from_env", "max_over_ranks", "render_sharded",
           "gather_to_rank0", "allreduce_grads"]

# xGMI is point-to-point (7 links x ~153 GB/s per GPU): RCCL's ring all-reduce is per-link
# bound, so a few large buckets beat many small ones.  The whole training gradient is
# ~60 MB; 32 MB buckets give two collectives per step.
BUCKET_BYTES = 32 << 20


def shard_range(n, rank, world):
    """Contiguous [start, end) of n items for `rank` (sizes differ by at most one)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world %d/%d" % (rank, world))
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def env_rank():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init_from_env(backend="nccl"):
    """torch.distributed over RCCL ("nccl" on ROCm) when WORLD_SIZE > 1.

    Diagnostics only: PNR_DIST_BACKEND overrides the backend and PNR_FORCE_DEVICE pins every
    rank to one device (rehearsing the multi-rank bench on a one-GPU box with gloo)."""
    rank, world, local = env_rank()
    backend = os.environ.get("PNR_DIST_BACKEND", backend)
    if "PNR_FORCE_DEVICE" in os.environ:
        local = int(os.environ["PNR_FORCE_DEVICE"])
    if world > 1 and not dist.is_initialized():
        dist.init_process_group(backend, init_method="env://")
    return rank, world, local


def max_over_ranks(value, device=None):
    """Max of a float over all ranks (the timing reduction of bench.py)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    if dist.get_backend() != "nccl":
        device = "cpu"   # gloo: host tensor
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def render_sharded(render_fn, rays, rank, world, chunk):
    """Render this rank's contiguous slice of `rays` (N, 8) in chunks of `chunk` rays
    with ``render_fn(rays_chunk (1, n, 8)) -> (rgb (1, n, 3), depth (1, n))`` (the
    gen_video.py:213-217 loop).  Returns (start, end, rgb (n, 3), depth (n))."""
    start, end = shard_range(rays.shape[0], rank, world)
    rgbs, depths = [], []
    for r in torch.split(rays[start:end], chunk, dim=0):
        rgb, depth = render_fn(r[None])
        rgbs.append(rgb[0])
        depths.append(depth[0])
    if not rgbs:
        dev = rays.device
        return start, end, torch.zeros(0, 3, device=dev), torch.zeros(0, device=dev)
    return start, end, torch.cat(rgbs), torch.cat(depths)


def gather_to_rank0(t, n_total, rank, world):
    """Assemble per-rank contiguous slices on rank 0 (optional, off the hot path)."""
    if world == 1:
        return t
    parts = [None] * world if rank == 0 else None
    dist.gather_object(t.cpu(), parts, dst=0)
    if rank != 0:
        return None
    out = torch.cat(parts)
    assert out.shape[0] == n_total
    return out


def allreduce_grads(params, world, bucket_bytes=BUCKET_BYTES):
    """Data-parallel gradient mean (the DDP all-reduce of the training step):
    the grads of `params` are packed into flat fp32 buckets of <= `bucket_bytes`, each
    bucket is all-reduced (SUM, RCCL over xGMI on ROCm; gloo on CPU) and scaled by
    1 / world, then unpacked in place.  Params without a grad are skipped (e.g. the
    encoder's unused layer4).  Returns the number of collectives issued."""
    if world == 1:
        return 0
    grads = [p.grad for p in params if p.grad is not None]
    n = 0
    i = 0
    while i < len(grads):
        bucket, size = [], 0
        while i < len(grads) and (not bucket or size + grads[i].numel() * 4 <= bucket_bytes):
            bucket.append(grads[i])
            size += grads[i].numel() * 4
            i += 1
        flat = torch.cat([g.reshape(-1).float() for g in bucket])
        dist.all_reduce(flat, op=dist.ReduceOp.SUM)
        flat.mul_(1.0 / world)
        o = 0
        for g in bucket:
            g.copy_(flat[o: o + g.numel()].view_as(g))
            o += g.numel()
        n += 1
    return n
