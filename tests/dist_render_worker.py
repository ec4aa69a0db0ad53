"""Worker of tests/test_gpu_dist.py (not collected by pytest): one rank of a 2-rank HIP
render of the cfg3 NMR batch shape on ONE device (gloo control plane; the driver's N-GPU
runs put one rank per GPU over RCCL).

Each rank renders its contiguous ray range (pnr.dist.shard_range, the reference's ray
scatter nerf.py:367-371) with the HIP renderer and injected random streams sliced by the
global ray index, so sharding cannot change a ray's draws.  Rank 0 gathers the shards
(pnr.dist.gather_to_rank0), renders the whole batch once more in one process, and writes
{"equal": bool, ...} to argv[1].
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "pixel-nerf_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from pnr import dist as pdist  # noqa: E402
from pnr import synth, util  # noqa: E402
from pnr.models import PixelNeRFNet  # noqa: E402
from pnr.renderer import NeRFRenderer  # noqa: E402

N_FRAMES, SIZE, KC, KF = 3, 64, 64, 64


def conf():
    mlp = dict(type="resnet", n_blocks=5, d_hidden=512, combine_layer=3, combine_type="average")
    return dict(use_encoder=True, use_xyz=True, use_code=True,
                code=dict(num_freqs=6, freq_factor=1.5, include_input=True), use_viewdirs=True,
                use_code_viewdirs=False, mlp_coarse=mlp, mlp_fine=mlp,
                encoder=dict(backbone="resnet34", pretrained=False, num_layers=4))


def render(net, rays, streams, chunk):
    """rays (n, 8) in gen_video-style chunks; streams sliced per chunk (global indices)."""
    r = NeRFRenderer(n_coarse=KC, n_fine=KF, white_bkgd=True).cuda()
    par = r.bind_parallel(net, simple_output=True)
    out = []
    with torch.no_grad():
        for s in range(0, rays.shape[0], chunk):
            e = min(s + chunk, rays.shape[0])
            r.streams = tuple(t[s:e] for t in streams)
            rgb, _ = par(rays[s:e][None])
            out.append(rgb[0])
    return torch.cat(out)


def main():
    rank, world, _ = pdist.init_from_env("gloo")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    net = PixelNeRFNet(conf())
    net.load_state_dict(synth.pixelnerf_state(2), strict=False)
    net = net.to(dev).eval()
    sc = synth.scene_nmr(seed=5)
    net.encode_latent(sc["latent"].to(dev), sc["poses"].to(dev), sc["focal"].to(dev), (SIZE, SIZE))
    tgt = synth.srn_poses([20.0 * i for i in range(N_FRAMES)], phi=-20.0, radius=2.7)
    rays = util.gen_rays(tgt.to(dev), SIZE, SIZE, sc["focal"], 1.2, 4.0).reshape(-1, 8).contiguous()
    n = rays.shape[0]
    streams = synth.rng_streams(9, n, KC, KF, 0)
    start, end = pdist.shard_range(n, rank, world)
    mine = render(net, rays[start:end], tuple(t[start:end] for t in streams), chunk=5000)
    full = pdist.gather_to_rank0(mine.cpu(), n, rank, world)
    dist.barrier()
    if rank == 0:
        single = render(net, rays, streams, chunk=5000).cpu()
        res = dict(equal=bool(torch.equal(full, single)), n=n, world=world,
                   max_abs=float((full - single).abs().max()), finite=bool(torch.isfinite(full).all()))
        with open(sys.argv[1], "w") as fh:
            json.dump(res, fh)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
