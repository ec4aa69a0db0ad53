"""world_size-2 gloo tests of the process-per-GPU sharding (CPU).

Each rank renders its contiguous slice of a frame's rays with the CPU oracle as
the per-rank renderer (the HIP renderer needs a GPU); the assembled image must
equal the single-process render bit for bit, and the timing reduction must be
the max over ranks.
"""
import os
import socket

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
