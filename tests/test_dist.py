"""world_size-2 gloo tests of the process-per-GPU sharding (CPU).

Each rank renders its contiguous slice of a frame's rays with the CPU oracle as
the per-rank renderer (the HIP renderer needs a GPU); the assembled image must
equal the single-process render bit for bit, and the timing reduction must be
the max over ranks.
"""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pnr import dist as pdist
from pnr import synth


def test_shard_range_covers_exactly():
    for n in (0, 1, 7, 16384, 98304):
        for world in (1, 2, 3, 8):
            spans = [pdist.shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        pdist.shard_range(10, 2, 2)


def _scene():
    from oracle import ref_cpu

    sd = synth.pixelnerf_state(3, d_latent=64, d_hidden=64)
    sc = synth.scene_srn(seed=2, n_rays=40, channels=64, h_l=8, w_l=8, pick="hash")
    scene = ref_cpu.Scene(sc["latent"], sc["poses"], sc["focal"], 128, 128, None)
    return sd, scene, sc["rays"]


def _render_fn(sd, scene, rays_all):
    from oracle import ref_cpu

    streams_all = synth.rng_streams(4, rays_all.shape[0], 16, 16, 0)
    index = {}

    def fn(r):
        # streams follow the ray (global index), so sharding cannot change results
        n = r.shape[1]
        start = index.setdefault("pos", 0)
        index["pos"] = start + n
        st = tuple(s[start:start + n] if s.shape[1] else s[:n] for s in streams_all)
        with torch.no_grad():
            out = ref_cpu.render(lambda p, c, d: ref_cpu.pixelnerf_forward(
                sd, scene, p, c, d, d_latent=64), r, 16, 16, 0, st, True)
        return out["fine"]["rgb"], out["fine"]["depth"]

    return fn, index


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    r, w, _ = pdist.init_from_env("gloo")
    sd, scene, rays = _scene()
    fn, index = _render_fn(sd, scene, rays)
    start, end = pdist.shard_range(rays.shape[0], r, w)
    index["pos"] = start
    s, e, rgb, depth = pdist.render_sharded(fn, rays, r, w, chunk=8)
    full = pdist.gather_to_rank0(rgb, rays.shape[0], r, w)
    tmax = pdist.max_over_ranks(float(r + 1))
    dist.barrier()
    if r == 0:
        q.put((full, tmax))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_gloo_render_equals_single_process():
    sd, scene, rays = _scene()
    fn, index = _render_fn(sd, scene, rays)
    _, _, ref_rgb, _ = pdist.render_sharded(fn, rays, 0, 1, chunk=40)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    full, tmax = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert tmax == 2.0
    assert torch.equal(full, ref_rgb)


# ---- data-parallel training: the gradient all-reduce -------------------
def _train_grads(objs, before_backward=None):
    """Oracle training-step grads (tests/golden/train_step.npz inputs) over the objects
    `objs` only: rays, streams, target, camera and latent rows of those objects.
    ``before_backward(params)`` runs between the forward and ``loss.backward()``."""
    import fixtures
    from oracle import ref_cpu

    cfg, arr = fixtures.load("train_step")
    per = arr["rays"].shape[1]
    rows = torch.cat([torch.arange(o * per, (o + 1) * per) for o in objs])
    sd = synth.pixelnerf_state(cfg["seed"], d_latent=cfg["d_latent"], d_hidden=cfg["d_hidden"])
    params = {k: v.clone().requires_grad_(True) for k, v in sd.items() if k.startswith("mlp_")}
    sd.update(params)
    latent = arr["latent"][objs].clone().requires_grad_(True)
    scene = ref_cpu.Scene(latent, arr["poses"][objs], arr["focal"][objs], cfg["width"], cfg["height"],
                          arr["c"][objs])

    def model_fn(pts, coarse, dirs):
        return ref_cpu.pixelnerf_forward(sd, scene, pts, coarse, dirs, d_latent=cfg["d_latent"])

    streams = tuple(arr[k][rows] for k in ("u_coarse", "u_fine", "u_fine_jit", "n_depth"))
    out = ref_cpu.render(model_fn, arr["rays"][objs], cfg["n_coarse"], cfg["n_fine"], cfg["n_fine_depth"],
                         streams, cfg["white_bkgd"], depth_std=cfg["depth_std"])
    mse = torch.nn.functional.mse_loss
    loss = mse(out["coarse"]["rgb"], arr["target"][objs]) + mse(out["fine"]["rgb"], arr["target"][objs])
    if before_backward is not None:
        before_backward(params)
    loss.backward()
    return params


def _train_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    torch.set_num_threads(1)
    r, w, _ = pdist.init_from_env("gloo")
    params = _train_grads([r])
    n = pdist.allreduce_grads(list(params.values()), w, bucket_bytes=64 << 10)
    if r == 0:
        q.put(({k: p.grad.numpy().copy() for k, p in params.items()}, n))   # by value
    dist.barrier()
    dist.destroy_process_group()


def _overlap_worker(rank, world, port, q):
    """The overlapped reducer (pnr.dist.GradReducer): buckets all-reduced from the backward's
    grad hooks, with a parameter accumulated twice (a second, scaled use of one MLP weight
    through a leaf-sharing term) to exercise the late re-reduction."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    torch.set_num_threads(1)
    r, w, _ = pdist.init_from_env("gloo")
    state = {}

    def arm(params):
        state["red"] = pdist.GradReducer(list(params.values()), w, bucket_bytes=64 << 10)
        state["red"].arm()

    params = _train_grads([r], arm)
    red = state["red"]
    n_hooked = len(red.flights)
    # a second backward through one parameter after its bucket went out: the late path
    k0 = next(k for k in params if k.endswith("lin_in.weight"))
    red.armed = True
    (params[k0] * float(r + 1)).sum().backward()
    n = red.finish()
    if r == 0:
        q.put(({k: p.grad.numpy().copy() for k, p in params.items()}, n, n_hooked, k0))
    red.remove()
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_overlapped_reducer_equals_full_batch():
    """pnr.dist.GradReducer (bench.py's training step): buckets launched from the backward's
    grad hooks give the same mean gradient as the single-process whole-batch backward; a
    parameter accumulated again after its bucket was launched is reduced whole."""
    ref = _train_grads([0, 1])
    k0 = next(k for k in ref if k.endswith("lin_in.weight"))
    ref[k0].grad += (1.0 + 2.0) / 2.0   # the extra term: mean over ranks of (r + 1)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_overlap_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, n_coll, n_hooked, k_late = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert k_late == k0
    assert n_hooked >= 2          # buckets went out during the backward
    assert n_coll >= n_hooked + 1  # + the last bucket / the late re-reduction
    for k, p in ref.items():
        torch.testing.assert_close(torch.from_numpy(got[k]), p.grad, atol=1e-6, rtol=1e-4, msg=k)


def test_two_rank_gloo_gradient_allreduce_equals_full_batch():
    """Each rank trains on its own object; the bucketed all-reduce (mean) of the rank
    gradients equals the single-process gradient of the whole batch (equal shards)."""
    ref = _train_grads([0, 1])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_train_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, n_coll = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert n_coll >= 2   # several buckets
    for k, p in ref.items():
        torch.testing.assert_close(torch.from_numpy(got[k]), p.grad, atol=1e-6, rtol=1e-4, msg=k)


# ---- encoder BatchNorm across ranks (train.py:257-262, encoder.py:28-53) -----
def _encoder_step(images, weights, mode, world=1):
    """One training-mode encoder pass of `images` (n, 3, H, W) through the ResNet34 trunk +
    latent concat (pnr.encoder.SpatialEncoder), loss = mean over ranks of
    sum(latent * weights): returns (latent, grads by name, running stats by name)."""
    from pnr.encoder import SpatialEncoder

    torch.manual_seed(0)
    enc = SpatialEncoder(pretrained=False, use_first_pool=False).double()
    pdist.set_batchnorm_mode(enc, mode)
    enc.train()
    enc.latent = torch.empty(1, 1, 1, 1, dtype=torch.float64)
    lat = enc(images)
    loss = (lat * weights).sum()
    loss.backward()
    params = [p for _, p in enc.named_parameters()]
    pdist.allreduce_grads(params, world)
    grads = {k: p.grad.clone() for k, p in enc.named_parameters() if p.grad is not None}
    stats = {k: v.clone() for k, v in enc.state_dict().items() if "running" in k or "num_batches" in k}
    return lat.detach(), grads, stats


def _bn_inputs():
    g = torch.Generator().manual_seed(7)
    images = torch.rand(4, 3, 32, 32, generator=g, dtype=torch.float64) * 2 - 1
    weights = torch.randn(4, 512, 16, 16, generator=g, dtype=torch.float64)
    return images, weights


def _bn_worker(rank, world, port, mode, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    r, w, _ = pdist.init_from_env("gloo")
    images, weights = _bn_inputs()
    s, e = pdist.shard_range(images.shape[0], r, w)
    # rank r's loss is its share of the full-batch loss x world (mean over ranks = full loss)
    lat, grads, stats = _encoder_step(images[s:e], weights[s:e] * w, mode, w)
    q.put((r, lat.numpy(), {k: v.numpy() for k, v in grads.items()}, {k: v.numpy() for k, v in stats.items()}))
    dist.barrier()
    dist.destroy_process_group()


def _run_bn(mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bn_worker, args=(r, 2, port, mode, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict((r, (lat, g, st)) for r, lat, g, st in (q.get(timeout=300) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


def test_two_rank_sync_batchnorm_encode_equals_one_rank_full_batch():
    """SyncBatchNorm2d: a 2-rank train-mode encode of split objects (2 images per rank) equals
    the 1-rank encode of all 4 (the reference's one-batch encode): latents, every encoder
    gradient after the data-parallel mean, and both ranks' running statistics."""
    images, weights = _bn_inputs()
    ref_lat, ref_g, ref_st = _encoder_step(images, weights, "batch")
    got = _run_bn("sync")
    lat = torch.cat([torch.from_numpy(got[r][0]) for r in (0, 1)])
    torch.testing.assert_close(lat, ref_lat, atol=1e-9, rtol=1e-9)
    for r in (0, 1):
        for k, v in ref_g.items():
            # fp64 sums over a different association (per-rank partial sums, sum / sum-of-squares
            # variance) through ~30 normalised layers: agreement to ~1e-7 of the gradient's scale
            torch.testing.assert_close(torch.from_numpy(got[r][1][k]), v, atol=1e-7 * float(v.abs().max()),
                                       rtol=1e-6, msg=k)
        for k, v in ref_st.items():
            torch.testing.assert_close(torch.from_numpy(got[r][2][k]), v, atol=1e-9, rtol=1e-9, msg=k)


def test_two_rank_local_batchnorm_differs_and_frozen_matches_eval():
    """Without the sync each rank normalises over its own share (the semantic gap SURVEY §8(e)
    names): its latent differs from the full-batch encode.  FrozenBatchNorm2d uses the running
    statistics, so its train-mode encode equals an eval-mode encode and leaves them untouched."""
    from pnr.encoder import SpatialEncoder

    images, weights = _bn_inputs()
    ref_lat, _, _ = _encoder_step(images, weights, "batch")
    got = _run_bn("batch")
    lat = torch.cat([torch.from_numpy(got[r][0]) for r in (0, 1)])
    assert float((lat - ref_lat).abs().max()) > 1e-3
    lat_f, _, st_f = _encoder_step(images, weights, "frozen")
    torch.manual_seed(0)
    enc = SpatialEncoder(pretrained=False, use_first_pool=False).double().eval()
    enc.latent = torch.empty(1, 1, 1, 1, dtype=torch.float64)
    with torch.no_grad():
        ev = enc(images)
    torch.testing.assert_close(lat_f, ev, atol=1e-12, rtol=1e-12)
    for k, v in st_f.items():
        if "running_mean" in k:
            assert float(v.abs().max()) == 0.0, k
