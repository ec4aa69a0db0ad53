#!/usr/bin/env python
"""eval/eval.py counterpart on the MI355X ray march: per object of an SRN-layout split, encode
the source views, query the density on a mesh_res^3 grid over [-1, 1]^3 (PixelNeRFNet.forward as
a point query, coarse net, zero view directions, 65,536-point chunks: eval.py:93-103), and
write the grid; with --compare, render every non-source view and score it (PSNR / SSIM,
skimage's compare_* defaults as pnr.evaluate restates them) into <output>/finish.txt as
"<object> <psnr> <ssim> 1" (eval.py:110-144).

  python scripts/eval.py -c conf/exp/srn.conf -D <datadir>/cars -n srn_car \
      --checkpoints_path checkpoints [--split test] [-P "2"] [--mesh_res 256] [--compare]

The reference turns the grid into a mesh with skimage.measure.marching_cubes and trimesh
(eval.py:104-108); neither is installed offline, so the grid is written as
<output>/<object>/<object>_sigma.npy (float32, relu(sigma), [x][y][z] with torch.meshgrid's 'ij'
order) and the mesh is exported only where both libraries import.  In the fork the comparison
after the mesh is unreachable (a `continue` follows the export); --compare runs it."""
import argparse
import os
import sys
import time
import traceback

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pixel-nerf_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from pnr import evaluate, util  # noqa: E402
from pnr.conf import parse_file  # noqa: E402
from pnr.data import get_split_dataset  # noqa: E402
from pnr.models import make_model  # noqa: E402
from pnr.renderer import NeRFRenderer  # noqa: E402

CHUNK = 65536   # eval.py:99


def density_grid(net, res, device, chunk=CHUNK):
    """relu(sigma) of the coarse net on a res^3 grid over [-1, 1]^3 ('ij' order), (res, res, res)."""
    grid = torch.linspace(-1, 1, res, device=device)
    xs, ys, zs = torch.meshgrid(grid, grid, grid, indexing="ij")
    pts = torch.stack([xs, ys, zs], -1).reshape(-1, 3)
    out = torch.empty(pts.shape[0], device=device)
    with torch.no_grad():
        for i in range(0, pts.shape[0], chunk):
            p = pts[i:i + chunk][None]
            out[i:i + chunk] = net(p, coarse=True, viewdirs=torch.zeros_like(p))[0, :, 3]
    return torch.relu(out).view(res, res, res)


def export_mesh(sig, thresh, path):
    """The reference's mesh export (eval.py:104-108), where skimage and trimesh are installed."""
    try:
        import skimage.measure
        import trimesh
    except ImportError:
        return False
    verts, faces, _, _ = skimage.measure.marching_cubes(sig, level=thresh)
    trimesh.Trimesh(vertices=verts, faces=faces).export(path)
    return True


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--conf", "-c", required=True)
    ap.add_argument("--datadir", "-D", required=True)
    ap.add_argument("--dataset_format", "-F", default="srn")
    ap.add_argument("--name", "-n", default="srn_car")
    ap.add_argument("--checkpoints_path", default="checkpoints")
    ap.add_argument("--split", default="test")
    ap.add_argument("--source", "-P", default="2")
    ap.add_argument("--coarse", action="store_true")
    ap.add_argument("--output", "-O", default="eval")
    ap.add_argument("--mesh_res", type=int, default=256)
    ap.add_argument("--mesh_thresh", type=float, default=0.1)
    ap.add_argument("--compare", action="store_true", help="render and score the non-source views")
    ap.add_argument("--ray_batch_size", "-R", type=int, default=50000)
    ap.add_argument("--gpu_id", type=int, default=0)
    args = ap.parse_args(argv)
    args.resume = True

    device = torch.device("cuda", args.gpu_id)
    torch.cuda.set_device(device)
    conf = parse_file(args.conf)
    dset = get_split_dataset(args.dataset_format, args.datadir, want_split=args.split, training=False)
    net = make_model(conf["model"]).to(device=device).load_weights(args)
    net.eval()
    renderer = NeRFRenderer.from_conf(conf["renderer"], lindisp=dset.lindisp,
                                      eval_batch_size=args.ray_batch_size).to(device)
    if args.coarse:
        net.mlp_fine = None
    renderer.n_coarse = max(renderer.n_coarse, 64)
    render_par = renderer.bind_parallel(net, None, simple_output=True).eval()
    source = torch.tensor(sorted(map(int, args.source.split())), dtype=torch.long)
    os.makedirs(args.output, exist_ok=True)
    finish = open(os.path.join(args.output, "finish.txt"), "a", buffering=1)
    for obj_idx in range(len(dset)):
        name = str(obj_idx)
        try:
            data = dset[obj_idx]
            name = os.path.basename(data["path"])
            out_dir = os.path.join(args.output, name)
            os.makedirs(out_dir, exist_ok=True)
            images, poses = data["images"], data["poses"]
            if images.shape[0] < 2:
                print("Skipping %s - less than 2 views" % name, flush=True)
                continue
            focal = torch.as_tensor(data["focal"], dtype=torch.float32)[None].to(device)
            c = data.get("c")
            c = c.to(device).unsqueeze(0) if c is not None else None
            src = torch.zeros(images.shape[0], dtype=torch.bool)
            src[source] = True
            with torch.no_grad():
                net.encode(images[src].to(device).unsqueeze(0), poses[src].to(device).unsqueeze(0), focal, c=c)
            torch.cuda.synchronize(device)
            t0 = time.perf_counter()
            sig = density_grid(net, args.mesh_res, device)
            torch.cuda.synchronize(device)
            dt = time.perf_counter() - t0
            sig_np = sig.cpu().numpy()
            np.save(os.path.join(out_dir, name + "_sigma.npy"), sig_np)
            meshed = export_mesh(sig_np, args.mesh_thresh, os.path.join(out_dir, name + "_mesh.stl"))
            print("%s: density grid %d^3 in %.3f s (%.1f M points/s)%s" % (
                name, args.mesh_res, dt, args.mesh_res ** 3 / dt / 1e6,
                "" if meshed else "; mesh export skipped (skimage / trimesh not installed)"), flush=True)
            if not args.compare:
                continue
            tgt = ~src
            H, W = images.shape[-2:]
            rays = util.gen_rays(poses[tgt].to(device), W, H, focal, dset.z_near, dset.z_far, c=c).reshape(-1, 8)
            with torch.no_grad():
                rgb = torch.cat([render_par(r[None])[0][0] for r in torch.split(rays, args.ray_batch_size, dim=0)])
            rgb = rgb.clamp(0.0, 1.0).reshape(-1, H, W, 3).cpu().numpy()
            gt = (images[tgt] * 0.5 + 0.5).permute(0, 2, 3, 1).numpy()
            psnr = float(np.mean([evaluate.psnr_np(rgb[i], gt[i]) for i in range(len(gt))]))
            ssim = float(np.mean([evaluate.ssim(rgb[i], gt[i]) for i in range(len(gt))]))
            print("PSNR: %.2f, SSIM: %.4f" % (psnr, ssim), flush=True)
            finish.write("%s %.2f %.4f 1\n" % (name, psnr, ssim))
        except Exception as e:   # eval.py:146-149: report the object and go on
            print("ERROR processing %s: %s" % (name, e), flush=True)
            traceback.print_exc()
    finish.close()


if __name__ == "__main__":
    main()
