"""Host-side geometry helpers that the ray-march callers use.

These mirror the semantics (not the code) of the reference's ``src/util/util.py``:

* ``repeat_interleave``   — util.py:58-65 (expand + reshape along dim 0)
* ``combine_interleaved`` — util.py:461-471 (multi-view mean at the combine layer)
* ``unproj_map``          — util.py:113-143 (unit camera-ray directions per pixel)
* ``gen_rays``            — util.py:238-276 (rays ``[o(3), d(3), near, far]``)
* ``pose_spherical``      — util.py:309-323 (NeRF 360° camera path)
* ``psnr``                — util.py:474-481
* ``bbox_sample``         — util.py:220-235 (the training step's pixel picks inside object boxes)

They run on whatever device their inputs live on; none of them is on the
per-point hot path (ray generation on device is SURVEY §8(f) rank 1).
"""
import math

import numpy as np
import torch

__all__ = [
    "repeat_interleave",
    "combine_interleaved",
    "unproj_map",
    "gen_rays",
    "pose_spherical",
    "psnr",
    "batched_index_select_nd",
    "bbox_sample",
]


def repeat_interleave(t, repeats, dim=0):
    """Repeat every row ``repeats`` times along dim 0 (util.py:58-65)."""
    out = t.unsqueeze(1).expand(-1, repeats, *t.shape[1:])
    return out.reshape(-1, *t.shape[1:])


def combine_interleaved(t, inner_dims=(1,), agg_type="average"):
    """Reduce interleaved views (util.py:461-471): (N*NS*P, C) -> (N*P, C)."""
    if len(inner_dims) == 1 and inner_dims[0] == 1:
        return t
    t = t.reshape(-1, *inner_dims, *t.shape[1:])
    if agg_type == "average":
        return torch.mean(t, dim=1)
    if agg_type == "max":
        return torch.max(t, dim=1)[0]
    raise NotImplementedError("Unsupported combine type " + agg_type)


def batched_index_select_nd(t, inds):
    """Gather along dim 1 of a batched tensor (util.py:33-42)."""
    return t.gather(1, inds[(...,) + (None,) * (len(t.shape) - 2)].expand(-1, -1, *t.shape[2:]))


def bbox_sample(bboxes, num_pix):
    """(num_pix, 3) pixel picks [view, row, col] inside per-view boxes (util.py:220-235):
    ``bboxes`` (NV, 4) = [cmin, rmin, cmax, rmax] (inclusive).  Draws from torch's default host
    generator in the reference's order -- the view ids, then the columns, then the rows -- so a
    seeded call picks the reference's pixels."""
    view = torch.randint(0, bboxes.shape[0], (num_pix,))
    box = bboxes[view]
    col = (torch.rand(num_pix) * (box[:, 2] + 1 - box[:, 0]) + box[:, 0]).long()
    row = (torch.rand(num_pix) * (box[:, 3] + 1 - box[:, 1]) + box[:, 1]).long()
    return torch.stack((view, row, col), dim=-1)


def unproj_map(width, height, f, c=None, device="cpu"):
    """(H, W, 3) unit directions of the camera ray through each pixel centre-less
    integer grid, camera looking down -z, y up (util.py:113-143)."""
    if c is None:
        cx, cy = width * 0.5, height * 0.5
    else:
        c = torch.as_tensor(c).reshape(-1)
        cx, cy = float(c[0]), float(c[-1] if c.numel() > 1 else c[0])
    if isinstance(f, (float, int)):
        fx = fy = float(f)
    else:
        f = torch.as_tensor(f).reshape(-1)
        fx, fy = float(f[0]), float(f[-1])
    ys = torch.arange(height, dtype=torch.float32) - float(cy)
    xs = torch.arange(width, dtype=torch.float32) - float(cx)
    Y, X = torch.meshgrid(ys, xs, indexing="ij")
    X = X.to(device=device) / fx
    Y = Y.to(device=device) / fy
    Z = torch.ones_like(X)
    d = torch.stack((X, -Y, -Z), dim=-1)
    d /= torch.norm(d, dim=-1).unsqueeze(-1)
    return d


def _focal_c(width, height, focal, c):
    """(fx, fy, cx, cy) as the reference resolves them (util.py:124-134, 250-251)."""
    f = focal.squeeze() if torch.is_tensor(focal) else focal
    if isinstance(f, (float, int)):
        fx = fy = float(f)
    else:
        f = torch.as_tensor(f).reshape(-1)
        fx, fy = float(f[0]), float(f[-1])
    if c is None:
        cx, cy = width * 0.5, height * 0.5
    else:
        c = torch.as_tensor(c).reshape(-1)
        cx, cy = float(c[0]), float(c[-1] if c.numel() > 1 else c[0])
    return fx, fy, cx, cy


def gen_rays(poses, width, height, focal, z_near, z_far, c=None):
    """Camera rays for every pixel of every pose: (NV, H, W, 8) (util.py:238-276).

    Poses on the HIP device run the ``pnr_gen_rays`` kernel (the rays are born in HBM);
    host poses use the host restatement below, as the reference's host code does."""
    if poses.is_cuda:
        from . import _lib

        fx, fy, cx, cy = _focal_c(width, height, focal, c)
        p = poses.detach().to(torch.float32).contiguous()
        rows = p.shape[-2]
        out = torch.empty(p.shape[0], height, width, 8, dtype=torch.float32, device=p.device)
        _lib.check(_lib.load().pnr_gen_rays(_lib.ptr(p), p.shape[0], rows, width, height, fx, fy, cx,
                                            cy, float(z_near), float(z_far), _lib.ptr(out),
                                            _lib.stream_of(p.device)), "pnr_gen_rays")
        return out
    nv = poses.shape[0]
    device = poses.device
    f = focal.squeeze() if torch.is_tensor(focal) else focal
    dirs_cam = unproj_map(width, height, f, c=c, device=device).unsqueeze(0).repeat(nv, 1, 1, 1)
    centers = poses[:, None, None, :3, 3].expand(-1, height, width, -1)
    dirs = torch.matmul(poses[:, None, None, :3, :3], dirs_cam.unsqueeze(-1))[..., 0]
    nears = torch.full((nv, height, width, 1), float(z_near), device=device)
    fars = torch.full((nv, height, width, 1), float(z_far), device=device)
    return torch.cat((centers, dirs, nears, fars), dim=-1)


def _trans_t(t):
    return torch.tensor(
        [[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, t], [0, 0, 0, 1]], dtype=torch.float32
    )


def _rot_phi(phi):
    return torch.tensor(
        [[1, 0, 0, 0],
         [0, np.cos(phi), -np.sin(phi), 0],
         [0, np.sin(phi), np.cos(phi), 0],
         [0, 0, 0, 1]],
        dtype=torch.float32,
    )


def _rot_theta(th):
    return torch.tensor(
        [[np.cos(th), 0, -np.sin(th), 0],
         [0, 1, 0, 0],
         [np.sin(th), 0, np.cos(th), 0],
         [0, 0, 0, 1]],
        dtype=torch.float32,
    )


def pose_spherical(theta, phi, radius):
    """Camera-to-world matrix on a sphere, NeRF convention (util.py:309-323)."""
    c2w = _trans_t(radius)
    c2w = _rot_phi(phi / 180.0 * np.pi) @ c2w
    c2w = _rot_theta(theta / 180.0 * np.pi) @ c2w
    flip = torch.tensor(
        [[-1, 0, 0, 0], [0, 0, 1, 0], [0, 1, 0, 0], [0, 0, 0, 1]], dtype=torch.float32
    )
    return flip @ c2w


def psnr(pred, target):
    """PSNR in dB of two tensors (util.py:474-481)."""
    mse = ((pred - target) ** 2).mean()
    return -10 * math.log10(float(mse))
