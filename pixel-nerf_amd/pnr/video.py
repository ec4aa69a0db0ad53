"""Frame rendering as eval/gen_video.py does it (gen_video.py:174-236): the build-side
counterpart of the reference's video caller.

``render_frames`` walks the frames' rays in ``ray_batch_size`` chunks through
``render_par`` (the ``bind_parallel(..., simple_output=True)`` wrapper), keeps the fine
rgb, and reshapes it to (NV, H, W, 3).  ``to_uint8`` is the reference's
``(frames * 255).astype(np.uint8)``: truncation, not rounding.
"""
import numpy as np
import torch

__all__ = ["render_frames", "to_uint8"]


def render_frames(render_par, render_rays, ray_batch_size=50000):
    """render_rays (NV, H, W, 8) on the HIP device -> frames (NV, H, W, 3)."""
    H, W = render_rays.shape[1], render_rays.shape[2]
    all_rgb = []
    with torch.no_grad():
        for rays in torch.split(render_rays.reshape(-1, 8), ray_batch_size, dim=0):
            rgb, _depth = render_par(rays[None])
            all_rgb.append(rgb[0])
    return torch.cat(all_rgb).view(-1, H, W, 3)


def to_uint8(frames):
    """gen_video.py:236: (frames * 255).astype(np.uint8) -- truncates toward zero."""
    return (frames.cpu().numpy() * 255).astype(np.uint8)
