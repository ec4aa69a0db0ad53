"""Host-side geometry helpers that the ray-march callers use.

These mirror the semantics (not the code) of the reference's ``src/util/util.py``:

* ``repeat_interleave``   — util.py:58-65 (expand + reshape along dim 0)
* ``combine_interleaved`` — util.py:461-471 (multi-view mean at the combine layer)
* ``unproj_map``          — util.py:113-143 (unit camera-ray directions per pixel)
* ``gen_rays``            — util.py:238-276 (rays ``[o(3), d(3), near, far]``)
* ``pose_spherical``      — util.py:309-323 (NeRF 360° camera path)
* ``psnr``                — util.py:474-481
* ``bbox_sample``         — util.py:220-235 (the training step's pixel picks inside object boxes)

and the rest of what the reference's callers reach through ``util.X`` (eval/gen_video.py,
eval/eval_approx.py, eval/eval.py, eval/eval_real.py, train/train.py; tests/test_dropin.py scans
them): ``get_cuda`` (util.py:193-202), ``cmap`` / ``image_float_to_uint8`` (util.py:13-30),
``quat_to_rot`` / ``rot_to_quat`` (util.py:484-528), ``coord_from_blender`` / ``coord_to_blender``
(util.py:146-171), ``look_at`` (util.py:174-190), ``get_image_to_tensor_balanced`` /
``get_mask_to_tensor`` (util.py:68-81), ``masked_sample`` (util.py:205-217), ``homogeneous``,
``gen_grid``, ``batched_index_select_nd_last``, ``count_parameters``, ``get_module``.

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
    "batched_index_select_nd_last",
    "bbox_sample",
    "masked_sample",
    "get_cuda",
    "image_float_to_uint8",
    "cmap",
    "quat_to_rot",
    "rot_to_quat",
    "coord_from_blender",
    "coord_to_blender",
    "look_at",
    "homogeneous",
    "gen_grid",
    "get_image_to_tensor_balanced",
    "get_mask_to_tensor",
    "count_parameters",
    "get_module",
    "trans_t",
    "rot_phi",
    "rot_theta",
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


def gen_rays(poses, width, height, focal, z_near, z_far, c=None, ndc=False):
    """Camera rays for every pixel of every pose: (NV, H, W, 8) (util.py:238-276).

    Poses on the HIP device run the ``pnr_gen_rays`` kernel (the rays are born in HBM);
    host poses use the host restatement below, as the reference's host code does.
    ``ndc=True`` is refused: the reference's NDC branch calls an ``ndc_rays`` its util module
    does not define (util.py:254-262), so no caller can use it."""
    if ndc:
        raise NotImplementedError("gen_rays(ndc=True): the reference defines no ndc_rays (util.py:262)")
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


def trans_t(t):
    return torch.tensor(
        [[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, t], [0, 0, 0, 1]], dtype=torch.float32
    )


def rot_phi(phi):
    return torch.tensor(
        [[1, 0, 0, 0],
         [0, np.cos(phi), -np.sin(phi), 0],
         [0, np.sin(phi), np.cos(phi), 0],
         [0, 0, 0, 1]],
        dtype=torch.float32,
    )


def rot_theta(th):
    return torch.tensor(
        [[np.cos(th), 0, -np.sin(th), 0],
         [0, 1, 0, 0],
         [np.sin(th), 0, np.cos(th), 0],
         [0, 0, 0, 1]],
        dtype=torch.float32,
    )


def pose_spherical(theta, phi, radius):
    """Camera-to-world matrix on a sphere, NeRF convention (util.py:309-323)."""
    c2w = trans_t(radius)
    c2w = rot_phi(phi / 180.0 * np.pi) @ c2w
    c2w = rot_theta(theta / 180.0 * np.pi) @ c2w
    flip = torch.tensor(
        [[-1, 0, 0, 0], [0, 0, 1, 0], [0, 1, 0, 0], [0, 0, 0, 1]], dtype=torch.float32
    )
    return flip @ c2w


def psnr(pred, target):
    """PSNR in dB of two tensors (util.py:474-481)."""
    mse = ((pred - target) ** 2).mean()
    return -10 * math.log10(float(mse))


# ------------------------------------------------- the callers' other util.X helpers ----
def batched_index_select_nd_last(t, inds):
    """Gather along the last dim (util.py:45-55): t (..., n, m), inds (..., k) -> (..., n, k)."""
    idx = inds.unsqueeze(-2).expand(*inds.shape[:-1], t.size(-2), inds.size(-1))
    return t.gather(-1, idx)


def masked_sample(masks, num_pix, prop_inside, thresh=0.5):
    """(num_pix, 3) [view, row, col] picks, a share ``prop_inside`` from mask >= thresh
    (util.py:205-217); draws inside picks, then outside picks, from torch's host generator."""
    n_in = int(num_pix * prop_inside + 0.5)
    inside = (masks >= thresh).nonzero(as_tuple=False)
    outside = (masks < thresh).nonzero(as_tuple=False)
    pick_in = inside[torch.randint(0, inside.shape[0], (n_in,))]
    pick_out = outside[torch.randint(0, outside.shape[0], (num_pix - n_in,))]
    return torch.cat((pick_in, pick_out))


def get_cuda(gpu_id):
    """``cuda:<gpu_id>`` when a HIP device is present, else the CPU device (util.py:193-202).
    The ray march itself has no CPU path: a CPU net fails loudly at its first render."""
    return torch.device("cuda:%d" % gpu_id) if torch.cuda.is_available() else torch.device("cpu")


def image_float_to_uint8(img):
    """Min-max stretch of a float image to uint8 (util.py:13-23; truncating cast)."""
    lo, hi = np.min(img), np.max(img)
    if hi - lo < 1e-10:
        hi += 1e-10
    out = (img - lo) / (hi - lo)
    out *= 255.0
    return out.astype(np.uint8)


def _hot_lut():
    """OpenCV's COLORMAP_HOT as a (256, 3) BGR uint8 table: the colormap is defined by 64 samples
    of r = 5x/2, g = 5x/2 - 1, b = 5x - 4 (each clipped to [0, 1]; x = i/63), linearly interpolated
    to 256 entries and scaled by 255 with rounding.  cv2 is absent offline, so the table is a
    restatement of that definition, not pinned to cv2's own output (parity unpinned)."""
    x = np.arange(64, dtype=np.float64) / 63.0
    r = np.clip(2.5 * x, 0.0, 1.0)
    g = np.clip(2.5 * x - 1.0, 0.0, 1.0)
    b = np.clip(5.0 * x - 4.0, 0.0, 1.0)
    xi = np.linspace(0.0, 1.0, 256)
    rgb = np.stack([np.interp(xi, x, ch) for ch in (b, g, r)], -1)
    return np.clip(np.rint(rgb * 255.0), 0, 255).astype(np.uint8)


_HOT = None


def cmap(img, color_map=None):
    """HOT colouring of a float image (util.py:26-30: cv2.applyColorMap(image_float_to_uint8(img),
    COLORMAP_HOT)): (H, W) or (H, W, 1) float -> (H, W, 3) uint8 in cv2's BGR channel order.
    Only the HOT map is provided (the one the callers use, train.py:363-384)."""
    global _HOT
    if color_map not in (None, 11):   # cv2.COLORMAP_HOT == 11
        raise NotImplementedError("util.cmap implements COLORMAP_HOT only")
    if _HOT is None:
        _HOT = _hot_lut()
    u8 = image_float_to_uint8(np.asarray(img))
    if u8.ndim == 3 and u8.shape[-1] == 1:
        u8 = u8[..., 0]
    return _HOT[u8]


def quat_to_rot(q):
    """(B, 4) quaternions [w, x, y, z] -> (B, 3, 3) rotations, normalising first (util.py:484-504)."""
    q = torch.nn.functional.normalize(q, dim=1)
    w, x, y, z = q.unbind(1)
    rows = [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
            2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
            2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]
    return torch.stack(rows, 1).reshape(-1, 3, 3)


def rot_to_quat(R):
    """(B, 3, 3) rotations -> (B, 4) [w, x, y, z], the trace branch only (util.py:507-528)."""
    w = torch.sqrt(1.0 + R[:, 0, 0] + R[:, 1, 1] + R[:, 2, 2]) / 2
    return torch.stack((w, (R[:, 2, 1] - R[:, 1, 2]) / (4 * w), (R[:, 0, 2] - R[:, 2, 0]) / (4 * w),
                        (R[:, 1, 0] - R[:, 0, 1]) / (4 * w)), 1)


def coord_from_blender(dtype=torch.float32, device="cpu"):
    """Blender axes (x right, y in, z up) -> x right, y up, z out (util.py:146-157)."""
    return torch.tensor([[1, 0, 0, 0], [0, 0, 1, 0], [0, -1, 0, 0], [0, 0, 0, 1]], dtype=dtype, device=device)


def coord_to_blender(dtype=torch.float32, device="cpu"):
    """The inverse of coord_from_blender (util.py:160-171)."""
    return torch.tensor([[1, 0, 0, 0], [0, 0, -1, 0], [0, 1, 0, 0], [0, 0, 0, 1]], dtype=dtype, device=device)


def look_at(origin, target, world_up=np.array([0, 1, 0], dtype=np.float32)):
    """4 x 4 camera-to-world matrix of a camera at ``origin`` looking at ``target`` (util.py:174-190)."""
    back = origin - target
    back = back / np.linalg.norm(back)
    right = np.cross(world_up, back)
    right = right / np.linalg.norm(right)
    up = np.cross(back, right)
    m = np.zeros((4, 4), dtype=np.float32)
    m[:3, 0], m[:3, 1], m[:3, 2], m[:3, 3] = right, up, back, origin
    m[3, 3] = 1.0
    return m


def homogeneous(points):
    """Append a 1 to every point: (..., 3) -> (..., 4) (util.py:84-90)."""
    return torch.nn.functional.pad(points, (0, 1), "constant", 1.0)


def gen_grid(*args, ij_indexing=False):
    """Points of a grid with one (lo, hi, n) per dimension, (prod n, len(args)) (util.py:93-110)."""
    axes = [np.linspace(lo, hi, n, dtype=np.float32) for lo, hi, n in args]
    mesh = np.meshgrid(*axes, indexing="ij" if ij_indexing else "xy")
    return torch.from_numpy(np.vstack(mesh).reshape(len(args), -1).T)


class _ToTensorNormalize:
    """torchvision ToTensor() + Normalize(mean, std) (+ an optional Resize of the shorter edge)
    for (H, W, C) uint8 arrays or PIL images -> (C, H, W) float32 (torchvision is absent)."""

    def __init__(self, mean, std, image_size=0):
        self.mean, self.std, self.size = float(mean), float(std), image_size

    def __call__(self, img):
        if self.size and self.size > 0:
            from PIL import Image

            im = img if isinstance(img, Image.Image) else Image.fromarray(np.asarray(img))
            w, h = im.size
            if w <= h:
                nw, nh = self.size, int(self.size * h / w)
            else:
                nw, nh = int(self.size * w / h), self.size
            img = im.resize((nw, nh), Image.BILINEAR)
        a = np.asarray(img)
        if a.ndim == 2:
            a = a[..., None]
        t = torch.from_numpy(np.ascontiguousarray(a)).permute(2, 0, 1).float()
        if a.dtype == np.uint8:
            t = t.div(255.0)
        return (t - self.mean) / self.std


def get_image_to_tensor_balanced(image_size=0):
    """ToTensor + Normalize(0.5, 0.5): uint8 image -> [-1, 1] (util.py:68-75)."""
    return _ToTensorNormalize(0.5, 0.5, image_size)


def get_mask_to_tensor():
    """ToTensor + Normalize(0, 1): uint8 mask -> [0, 1] (util.py:78-81)."""
    return _ToTensorNormalize(0.0, 1.0)


def count_parameters(model):
    """Trainable parameter count (util.py:326-327)."""
    return sum(p.numel() for p in model.parameters() if p.requires_grad)


def get_module(net):
    """``net.module`` of a DataParallel wrapper, else ``net`` (util.py:531-538)."""
    return net.module if isinstance(net, torch.nn.DataParallel) else net
