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
import torch.nn.functional as F
from torch import nn

__all__ = ["shard_range", "env_rank", "init_from_env", "max_over_ranks", "render_sharded",
           "gather_to_rank0", "allreduce_grads", "GradReducer", "SyncBatchNorm2d", "FrozenBatchNorm2d",
           "set_batchnorm_mode"]

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


class GradReducer:
    """The data-parallel gradient mean of ``allreduce_grads``, overlapped with the backward (what
    DDP's reducer does for the reference's DataParallel training).

    A post-accumulate-grad hook on every parameter appends it to the open bucket as its gradient
    lands. A bucket that reaches ``bucket_bytes`` is flattened and all-reduced (SUM) with
    ``async_op=True``. RCCL runs it on its own stream while autograd goes on, so the MLP buckets,
    which are ready first, reduce under the encoder's backward. ``finish()`` after ``backward()``
    launches the last bucket, waits, scales by 1 / world and unpacks in place.

    Autograd visits the graph in the same order on every rank, so every rank launches the same
    buckets in the same order. A parameter whose gradient accumulates again after its bucket was
    launched (a module used twice in one step) is reduced once more, whole, in ``finish()``.

    Usage per step: ``r.arm(); loss.backward(); r.finish()``. World size 1: no hooks, no work."""

    def __init__(self, params, world, bucket_bytes=BUCKET_BYTES):
        self.world = world
        self.bucket_bytes = bucket_bytes
        self.armed = False
        self._reset()
        self.hooks = []
        if world > 1:
            self.hooks = [p.register_post_accumulate_grad_hook(self._ready) for p in params if p.requires_grad]

    def _reset(self):
        self.open, self.open_bytes = [], 0
        self.flights = []      # (work, flat, params) of launched buckets
        self.launched = set()  # id() of params in launched buckets
        self.seen = set()      # id() of params in the open bucket
        self.late = []         # params accumulated again after their bucket was launched

    def _ready(self, p):
        if not self.armed or p.grad is None:
            # None: the engine runs post-accumulate hooks also for a parameter whose backward
            # returned no gradient; whoever sets .grad later runs the hook again
            return
        if id(p) in self.launched:
            if all(q is not p for q in self.late):
                self.late.append(p)
            return
        if id(p) in self.seen:
            return   # accumulated again while its bucket is still open: the bucket reads .grad at launch
        self.seen.add(id(p))
        self.open.append(p)
        self.open_bytes += p.grad.numel() * 4
        if self.open_bytes >= self.bucket_bytes:
            self._launch()

    def _launch(self):
        if not self.open:
            return
        ps, self.open, self.open_bytes = self.open, [], 0
        self.seen.clear()
        flat = torch.cat([p.grad.reshape(-1).float() for p in ps])
        self.flights.append((dist.all_reduce(flat, op=dist.ReduceOp.SUM, async_op=True), flat, ps))
        self.launched.update(id(p) for p in ps)

    def arm(self):
        """Before ``loss.backward()``."""
        self._reset()
        self.armed = self.world > 1

    def finish(self):
        """After ``loss.backward()``: the gradients are the mean over the ranks. Returns the
        number of collectives issued."""
        if not self.armed:
            return 0
        self._launch()
        n = len(self.flights)
        late = {id(p) for p in self.late}
        for work, flat, ps in self.flights:
            work.wait()
            flat.mul_(1.0 / self.world)
            o = 0
            for p in ps:
                k = p.grad.numel()
                if id(p) not in late:
                    p.grad.copy_(flat[o: o + k].view_as(p.grad))
                o += k
        if self.late:
            n += allreduce_grads(self.late, self.world, self.bucket_bytes)
        self.armed = False
        self._reset()
        return n

    def remove(self):
        for h in self.hooks:
            h.remove()
        self.hooks = []


# ---- encoder BatchNorm across ranks (SURVEY §8(e) "semantics difference to resolve") ------
# The reference encodes all SB objects of a step in ONE batch on device 0 (train.py:257-262)
# with the ResNet34's BatchNorm in train mode (encoder.py:28-53, trainer.py:194), so the
# statistics are over the whole SB x NS image batch.  One process per GPU with each rank
# encoding its own objects would normalise over that rank's share only, and the running
# statistics would drift apart between ranks.  SyncBatchNorm2d restores the reference's
# semantics: the per-channel sums of the batch are all-reduced (one collective per layer in
# the forward, one in the backward), so every rank normalises with the full batch's mean and
# biased variance and updates identical running statistics (unbiased variance, as torch's
# BatchNorm does).  FrozenBatchNorm2d is the other resolution SURVEY §8(e) names: the
# running statistics are used and never updated (eval-mode BN, what the reference's step 0
# runs because render_par is built .eval(), train.py:93).


class _SyncBNFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, eps, momentum, group):
        C = x.shape[1]
        dims = [0] + list(range(2, x.dim()))
        xd = x.double()
        n_local = x.numel() // C
        stats = torch.cat([xd.sum(dims), (xd * xd).sum(dims),
                           torch.full((1,), float(n_local), dtype=torch.float64, device=x.device)])
        dev_cpu = dist.get_backend(group) != "nccl" and x.device.type != "cpu"
        red = stats.cpu() if dev_cpu else stats   # gloo reduces host tensors
        dist.all_reduce(red, group=group)
        stats = red.to(x.device) if dev_cpu else red
        n = stats[-1]
        mean = stats[:C] / n
        var = (stats[C:2 * C] / n - mean * mean).clamp_min(0.0)   # biased, as BatchNorm normalises
        invstd = torch.rsqrt(var + eps)
        if running_mean is not None:
            with torch.no_grad():
                running_mean.mul_(1.0 - momentum).add_(mean.to(running_mean.dtype), alpha=momentum)
                # on the device: no host read of the count (a sync per layer)
                unbiased = torch.where(n > 1, var * n / (n - 1.0).clamp_min(1.0), var)
                running_var.mul_(1.0 - momentum).add_(unbiased.to(running_var.dtype), alpha=momentum)
        shape = [1, C] + [1] * (x.dim() - 2)
        mean_f = mean.to(x.dtype).view(shape)
        invstd_f = invstd.to(x.dtype).view(shape)
        xhat = (x - mean_f) * invstd_f
        ctx.save_for_backward(xhat, invstd_f, weight, n.reshape(1))
        ctx.group = group
        ctx.dev_cpu = dev_cpu
        return xhat * weight.view(shape) + bias.view(shape)

    @staticmethod
    def backward(ctx, dy):
        xhat, invstd, weight, n = ctx.saved_tensors
        C = xhat.shape[1]
        dims = [0] + list(range(2, xhat.dim()))
        shape = [1, C] + [1] * (xhat.dim() - 2)
        dy = dy.contiguous()
        sum_dy = dy.sum(dims)
        sum_dy_xhat = (dy * xhat).sum(dims)
        red = torch.cat([sum_dy, sum_dy_xhat]).double()
        red = red.cpu() if ctx.dev_cpu else red
        dist.all_reduce(red, group=ctx.group)
        red = red.to(dy.device) / n
        mean_dy = red[:C].to(dy.dtype).view(shape)
        mean_dy_xhat = red[C:].to(dy.dtype).view(shape)
        dx = (dy - mean_dy - xhat * mean_dy_xhat) * (invstd * weight.view(shape))
        # the affine parameters' gradients stay local: the data-parallel gradient mean
        # (allreduce_grads) sums them over ranks like every other parameter's
        return dx, sum_dy_xhat, sum_dy, None, None, None, None, None


class SyncBatchNorm2d(nn.BatchNorm2d):
    """nn.BatchNorm2d whose train-mode statistics span every rank of ``group`` (the
    reference's single-process batch, train.py:257-262).  Same parameters, buffers and
    state-dict keys as BatchNorm2d; eval mode and a one-rank world are plain BatchNorm2d."""

    group = None

    def forward(self, x):
        world = dist.get_world_size(self.group) if dist.is_available() and dist.is_initialized() else 1
        if not self.training or world == 1:
            return super().forward(x)
        if not self.affine or not self.track_running_stats or self.momentum is None:
            raise NotImplementedError("SyncBatchNorm2d: affine, tracked stats and a float momentum only")
        self.num_batches_tracked.add_(1)
        return _SyncBNFunction.apply(x, self.weight, self.bias, self.running_mean, self.running_var,
                                     self.eps, self.momentum, self.group)


class FrozenBatchNorm2d(nn.BatchNorm2d):
    """nn.BatchNorm2d that always normalises with its running statistics and never updates
    them (eval-mode BN inside a training step).  Same parameters and state-dict keys; the
    affine weight and bias still train."""

    def forward(self, x):
        return F.batch_norm(x, self.running_mean, self.running_var, self.weight, self.bias, False, 0.0, self.eps)


_BN_CLASSES = {"batch": nn.BatchNorm2d, "sync": SyncBatchNorm2d, "frozen": FrozenBatchNorm2d}


def set_batchnorm_mode(module, mode, group=None):
    """Switch every BatchNorm2d of ``module`` (e.g. a PixelNeRFNet's encoder) in place to
    ``mode``: "batch" (the reference: statistics of this process's batch), "sync" (statistics
    of the whole batch over the ranks of ``group``: the reference's semantics under one process
    per GPU), or "frozen" (running statistics, never updated).  Parameters, buffers and
    state-dict keys are unchanged.  Returns the number of layers switched."""
    cls = _BN_CLASSES[mode]
    n = 0
    for m in module.modules():
        if isinstance(m, nn.BatchNorm2d):
            m.__class__ = cls
            if cls is SyncBatchNorm2d:
                m.group = group
            n += 1
    return n
