"""Approximate PSNR / SSIM evaluation over an SRN-layout dataset.

Counterpart of eval/eval_approx.py:56-153: for every object one random target view is
rendered from the chosen source view(s) through ``render_par`` (bind_parallel,
simple_output) and scored against the ground-truth image with PSNR and SSIM at
data_range 1.  The view selection replays the reference's draws in order on torch's global
generator (seeded with ``seed``): per batch ``randint(0, NV, (SB, 1))`` for a random source,
then ``randint(0, NV - NS, (SB, 1))`` for the target, shifted past the sources.

``ssim`` restates skimage.measure.compare_ssim(X, Y, multichannel=True, data_range=1) with
its defaults (7 x 7 uniform window, sample covariance, K1 = 0.01, K2 = 0.03, per-channel
mean over the map cropped by 3 pixels); skimage is absent offline, so that restatement is
pinned by the brute-force window sum in tests/test_host.py, not by skimage itself.
"""
import numpy as np
import torch

from . import util

__all__ = ["ssim", "psnr_np", "select_views", "eval_approx"]


def psnr_np(pred, target, data_range=1.0):
    """skimage compare_psnr: 10 log10(data_range^2 / mse)."""
    mse = float(np.mean((np.asarray(pred, np.float64) - np.asarray(target, np.float64)) ** 2))
    return float("inf") if mse == 0.0 else 10.0 * np.log10(data_range ** 2 / mse)


def ssim(x, y, data_range=1.0, win_size=7, k1=0.01, k2=0.03):
    """Mean SSIM of two (H, W, C) images (skimage compare_ssim, multichannel, defaults)."""
    from scipy.ndimage import uniform_filter

    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64)
    assert x.shape == y.shape and x.ndim == 3
    vals = []
    for ch in range(x.shape[-1]):
        a, b = x[..., ch], y[..., ch]
        n = win_size ** 2
        cov_norm = n / (n - 1.0)
        ux = uniform_filter(a, size=win_size)
        uy = uniform_filter(b, size=win_size)
        uxx = uniform_filter(a * a, size=win_size)
        uyy = uniform_filter(b * b, size=win_size)
        uxy = uniform_filter(a * b, size=win_size)
        vx = cov_norm * (uxx - ux * ux)
        vy = cov_norm * (uyy - uy * uy)
        vxy = cov_norm * (uxy - ux * uy)
        c1 = (k1 * data_range) ** 2
        c2 = (k2 * data_range) ** 2
        s = ((2 * ux * uy + c1) * (2 * vxy + c2)) / ((ux ** 2 + uy ** 2 + c1) * (vx + vy + c2))
        pad = (win_size - 1) // 2
        vals.append(s[pad:-pad, pad:-pad].mean())
    return float(np.mean(vals))


def select_views(sb, nv, source):
    """(src_view (SB, NS), dest_view (SB, 1)) as eval_approx.py:111-118 draws them."""
    source = torch.as_tensor(source, dtype=torch.long).reshape(-1)
    ns = source.numel()
    if ns == 1 and int(source[0]) == -1:
        src_view = torch.randint(0, nv, (sb, 1))
    else:
        src_view = source.unsqueeze(0).expand(sb, -1)
    dest_view = torch.randint(0, nv - ns, (sb, 1))
    for i in range(ns):
        dest_view += dest_view >= src_view[:, i:i + 1]
    return src_view, dest_view


def eval_approx(net, renderer, dset, device, source=(64,), batch_size=4, seed=1234, coarse=False,
                ray_batch_size=50000, gpu_ids=None, log=None):
    """eval_approx.py:56-153 on an already built net / renderer / dataset.  Returns
    {"psnr": [...], "ssim": [...], "mean_psnr", "mean_ssim", "objects"}."""
    if coarse:
        net.mlp_fine = None
    renderer.eval_batch_size = ray_batch_size
    if renderer.n_coarse < 64:
        renderer.n_coarse = 64
    if coarse:
        renderer.n_coarse = 64
        renderer.n_fine = 128
        renderer.using_fine = True
    render_par = renderer.bind_parallel(net, gpu_ids, simple_output=True).eval()
    loader = torch.utils.data.DataLoader(dset, batch_size=batch_size, shuffle=False, num_workers=0)
    z_near, z_far = dset.z_near, dset.z_far
    torch.random.manual_seed(seed)
    ns = len(torch.as_tensor(source).reshape(-1))
    psnrs, ssims = [], []
    with torch.no_grad():
        for data in loader:
            images = data["images"]          # (SB, NV, 3, H, W) in [-1, 1]
            poses = data["poses"]            # (SB, NV, 4, 4)
            focal = data["focal"][0]
            images_0to1 = images * 0.5 + 0.5
            SB, NV, _, H, W = images.shape
            src_view, dest_view = select_views(SB, NV, source)
            dest_poses = util.batched_index_select_nd(poses, dest_view)
            all_rays = util.gen_rays(dest_poses.reshape(-1, 4, 4), W, H, focal, z_near, z_far).reshape(SB, -1, 8)
            pri_images = util.batched_index_select_nd(images, src_view)
            pri_poses = util.batched_index_select_nd(poses, src_view)
            net.encode(pri_images.to(device=device), pri_poses.to(device=device), focal.to(device=device))
            rgb_fine, _ = render_par(all_rays.to(device=device))
            rgb_fine = rgb_fine.reshape(SB, H, W, 3).cpu().numpy()
            gt = util.batched_index_select_nd(images_0to1, dest_view).reshape(SB, 3, H, W)
            gt = gt.permute(0, 2, 3, 1).contiguous().numpy()
            for sb in range(SB):
                ssims.append(ssim(rgb_fine[sb], gt[sb]))
                psnrs.append(psnr_np(rgb_fine[sb], gt[sb]))
            if log is not None:
                log("curr psnr %.4f ssim %.4f" % (np.mean(psnrs), np.mean(ssims)))
    assert ns >= 1
    return {"psnr": psnrs, "ssim": ssims, "mean_psnr": float(np.mean(psnrs)) if psnrs else None,
            "mean_ssim": float(np.mean(ssims)) if ssims else None, "objects": len(psnrs)}
