#!/usr/bin/env python
"""eval/gen_video.py counterpart on the MI355X ray march (SRN-layout datasets).

Encodes the chosen source view(s) of one object, renders a 360-degree loop of
`--num_views` frames (util.pose_spherical at `--elevation`, radius (z_near + z_far) / 2
unless `--radius`), in `--ray_batch_size`-ray chunks through render_par, and writes the
frames as PNGs plus an animated GIF (mp4 needs imageio / ffmpeg, absent offline).

  python scripts/gen_video.py -c conf/exp/srn.conf -D <datadir>/cars -n srn_car \
      --checkpoints_path checkpoints --split test -S 0 -P "64" --num_views 40

Same flow and arithmetic as gen_video.py:63-236 (frames (rgb * 255).astype(uint8));
the DTU trajectory (IDR quaternion spline) is not implemented (no DTU loader here).
"""
import argparse
import os
import sys
import warnings

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pixel-nerf_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from pnr import util, video  # noqa: E402
from pnr.conf import parse_file  # noqa: E402
from pnr.data import get_split_dataset  # noqa: E402
from pnr.models import make_model  # noqa: E402
from pnr.renderer import NeRFRenderer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--conf", "-c", required=True)
    ap.add_argument("--datadir", "-D", required=True)
    ap.add_argument("--dataset_format", "-F", default="srn")
    ap.add_argument("--name", "-n", default="srn_car")
    ap.add_argument("--checkpoints_path", default="checkpoints")
    ap.add_argument("--visual_path", default="visuals")
    ap.add_argument("--subset", "-S", type=int, default=0)
    ap.add_argument("--split", default="train")
    ap.add_argument("--source", "-P", default="64")
    ap.add_argument("--num_views", type=int, default=40)
    ap.add_argument("--elevation", type=float, default=-10.0)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--radius", type=float, default=0.0)
    ap.add_argument("--fps", type=int, default=30)
    ap.add_argument("--ray_batch_size", "-R", type=int, default=50000)
    ap.add_argument("--gpu_id", type=int, default=0)
    args = ap.parse_args()
    args.resume = True

    conf = parse_file(args.conf)
    device = torch.device("cuda", args.gpu_id)
    dset = get_split_dataset(args.dataset_format, args.datadir, want_split=args.split, training=False)
    data = dset[args.subset]
    print("Data instance loaded:", data["path"])
    images, poses = data["images"], data["poses"]   # (NV, 3, H, W), (NV, 4, 4)
    focal = torch.as_tensor(data["focal"], dtype=torch.float32)[None]
    c = data.get("c")
    if c is not None:
        c = c.to(device=device).unsqueeze(0)
    NV, _, H, W = images.shape
    if args.scale != 1.0:
        Ht, Wt = int(H * args.scale), int(W * args.scale)
        if abs(Ht / args.scale - H) > 1e-10 or abs(Wt / args.scale - W) > 1e-10:
            warnings.warn("Inexact scaling, please check {} times ({}, {}) is integral".format(args.scale, H, W))
        H, W = Ht, Wt

    net = make_model(conf["model"]).to(device=device)
    net.load_weights(args)
    renderer = NeRFRenderer.from_conf(conf["renderer"], lindisp=dset.lindisp,
                                      eval_batch_size=args.ray_batch_size).to(device=device)
    render_par = renderer.bind_parallel(net, None, simple_output=True).eval()

    radius = (dset.z_near + dset.z_far) * 0.5 if args.radius == 0.0 else args.radius
    render_poses = torch.stack([util.pose_spherical(angle, args.elevation, radius)
                                for angle in np.linspace(-180, 180, args.num_views + 1)[:-1]], 0)
    render_rays = util.gen_rays(render_poses, W, H, focal * args.scale, dset.z_near, dset.z_far,
                                c=c * args.scale if c is not None else None).to(device=device)
    source = torch.tensor(list(map(int, args.source.split())), dtype=torch.long)
    random_source = len(source) == 1 and int(source[0]) == -1
    assert not (source >= NV).any()
    if renderer.n_coarse < 64:   # gen_video.py:193-196
        renderer.n_coarse = 64
        renderer.n_fine = 128
    with torch.no_grad():
        src_view = torch.randint(0, NV, (1,)) if random_source else source
        net.encode(images[src_view].unsqueeze(0), poses[src_view].unsqueeze(0).to(device=device),
                   focal.to(device=device), c=c)
        print("Rendering", args.num_views * H * W, "rays")
        frames = video.render_frames(render_par, render_rays, args.ray_batch_size)
    frames_u8 = video.to_uint8(frames)

    from PIL import Image

    vid_name = "{:04}".format(args.subset)
    vid_name = ("t" if args.split == "test" else "v" if args.split == "val" else "") + vid_name
    vid_name += "_v" + "_".join("{:03}".format(int(x)) for x in source)
    out_dir = os.path.join(args.visual_path, args.name, "video" + vid_name)
    os.makedirs(out_dir, exist_ok=True)
    for i, f in enumerate(frames_u8):
        Image.fromarray(f).save(os.path.join(out_dir, "%04d.png" % i))
    ims = [Image.fromarray(f) for f in frames_u8]
    ims[0].save(out_dir + ".gif", save_all=True, append_images=ims[1:], duration=int(1000 / args.fps), loop=0)
    view = ((images[src_view].permute(0, 2, 3, 1) * 0.5 + 0.5).numpy() * 255).astype(np.uint8)
    Image.fromarray(np.hstack(list(view))).save(out_dir + "_view.jpg")
    print("Wrote", out_dir + ".gif")


if __name__ == "__main__":
    main()
