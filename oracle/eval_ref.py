"""ORACLE — test infrastructure only; never imported by the product path.

CPU restatement of the scoring loop of eval/eval_approx.py:100-153 for one evaluated batch:
render the target view's rays with the oracle renderer (ref_cpu.render over
ref_cpu.pixelnerf_forward, the given random draws) and score every object against its
ground-truth image with the reference's PSNR, util.psnr (util.py:474-481:
-10 log10(mse), data range 1).  The encoder CNN is outside the hot path: the batch carries
the latent the device encoder produced, so the comparison isolates the ray march.
"""
import math

import torch

from . import ref_cpu


def psnr(pred, target):
    """util.py:474-481 (fp64 mse here; the reference's fp32 mse agrees to ~1e-6 dB)."""
    mse = float(torch.mean((pred.double() - target.double()) ** 2))
    return math.inf if mse == 0.0 else -10.0 * math.log10(mse)


def score_batch(sd, latent, src_poses, focal, width, height, rays, streams, gt, n_coarse, n_fine,
                n_fine_depth=0, white_bkgd=True, c=None):
    """One eval_approx batch: latent (SB*NS, C, H_l, W_l), src_poses (SB, NS, 4, 4), rays
    (SB, H*W, 8), streams (u_coarse, u_fine, u_fine_jit, n_depth) for SB*H*W rays, gt
    (SB, H, W, 3) in [0, 1].  Returns (per-object PSNR list, fine rgb (SB, H, W, 3))."""
    scene = ref_cpu.Scene(latent.float(), src_poses.float(), focal, width, height, c)

    def model_fn(pts, coarse, dirs):
        return ref_cpu.pixelnerf_forward(sd, scene, pts, coarse, dirs)

    with torch.no_grad():
        out = ref_cpu.render(model_fn, rays.float(), n_coarse, n_fine, n_fine_depth, streams, white_bkgd)
    part = out["fine"] if n_fine > 0 else out["coarse"]
    rgb = part["rgb"].reshape(gt.shape)
    return [psnr(rgb[i], gt[i]) for i in range(gt.shape[0])], rgb
