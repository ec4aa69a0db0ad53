"""ORACLE — test infrastructure only; never imported by the product path.

Fine-pass parity by cause (VERDICT r1 "What's weak" 1).

The fine pass draws its importance samples with ``searchsorted(cdf, u, right=True)``
over the coarse weights (nerf.py:126-139), a discontinuous function of those weights.
When the HIP coarse weights differ from the reference's by fp32 reassociation
(≤ 5e-5), a ray whose ``u`` sits within that distance of a cdf boundary can pick the
neighbouring bin: a "bin flip".  Such a ray is excluded from the fine comparison only
when the flip is *proven*:

* the bin indices of every importance sample are recomputed here, on the CPU, from the
  HIP coarse weights and from the reference's coarse weights with the SAME ``u``
  (``fine_bins``, the reference's arithmetic, nerf.py:126-139);
* a ray counts as flipped only when those two index sets differ;
* every ray whose returned fine sample set ``z_fine`` differs from the reference's must
  be one of them (no unexplained sample difference), and every other ray is held to the
  full tolerance on rgb / depth / weights / z.

``classify_fine`` returns the masks; the callers (tests, ``smoke()``, bench.py's PSNR
leg) assert on them.
"""
import torch

ATOL, RTOL = 5e-5, 1e-5
# cdf rounding between the device scan (double, rounded per prefix) and torch's fp32 cumsum
MARGIN = 1e-6


def fine_cdf(coarse_weights):
    """nerf.py:126-133: (B, Kc) weights -> (B, Kc + 1) cdf."""
    w = coarse_weights.detach().float().cpu() + 1e-5
    pdf = w / torch.sum(w, -1, keepdim=True)
    cdf = torch.cumsum(pdf, -1)
    return torch.cat([torch.zeros_like(cdf[:, :1]), cdf], -1)


def fine_bins(coarse_weights, u_fine):
    """nerf.py:126-139 up to the bin index: (B, Kc) weights, (B, nf) u -> (B, nf) int64."""
    cdf = fine_cdf(coarse_weights)
    ind = torch.searchsorted(cdf, u_fine.float().cpu().contiguous(), right=True) - 1
    return torch.clamp_min(ind, 0)


def boundary_distance(coarse_weights, u_fine):
    """(B,) min over a ray's samples of |u - nearest cdf value|: how close each ray's draw
    sits to a bin boundary of the cdf built from these weights."""
    cdf = fine_cdf(coarse_weights)
    u = u_fine.float().cpu().reshape(cdf.shape[0], -1)
    return (u.unsqueeze(-1) - cdf.unsqueeze(1)).abs().amin(-1).amin(-1)


def close_mask(a, b, atol=ATOL, rtol=RTOL):
    return (a - b).abs() <= atol + rtol * b.abs()


def _marginal_alt_fine(rays, w_coarse, n_coarse, u, u_jit, lindisp):
    """sample_fine (nerf.py:126-148) with every draw that sits within MARGIN of a boundary
    of the cdf built from ``w_coarse`` moved to the bin on the OTHER side of that boundary.
    The device sums the pdf normaliser and scans the cdf in a different order than torch,
    so a draw placed on a boundary (the fixtures' force_u_high rays, u = 1 - 2^-24 against
    cdf[-1] = 1 +- ulp) may land in either neighbouring bin from the same weights."""
    cdf = fine_cdf(w_coarse)
    u = u.float().cpu().reshape(cdf.shape[0], -1)
    ind = torch.clamp_min(torch.searchsorted(cdf, u.contiguous(), right=True) - 1, 0)
    dist = (u.unsqueeze(-1) - cdf.unsqueeze(1)).abs()
    near_j = dist.argmin(-1)                             # nearest boundary cdf[j]
    marginal = dist.amin(-1) <= MARGIN
    # u >= cdf[j] gives bin j; u < cdf[j] gives bin j - 1: take the other one
    alt = torch.where(ind >= near_j, near_j - 1, near_j).clamp_min(0)
    ind = torch.where(marginal, alt, ind).float()
    z_steps = (ind + u_jit.float().cpu().reshape(u.shape)) / n_coarse
    near, far = rays[:, -2:-1], rays[:, -1:]
    if not lindisp:
        return near * (1 - z_steps) + far * z_steps
    return 1 / (1 / near * (1 - z_steps) + 1 / far * z_steps)


def expected_fine_z(rays, z_coarse, w_coarse, depth_coarse, streams, n_coarse, n_fine, n_fine_depth,
                    depth_std=0.01, lindisp=False, marginal_alt=False):
    """The reference's fine sample set (nerf.py:284-295: sort(cat(z_coarse, sample_fine,
    sample_fine_depth))) recomputed on the CPU from GIVEN coarse-pass outputs -- the HIP
    ones, to check that a flipped ray's HIP samples are exactly what the reference
    algorithm draws from the HIP coarse weights.  streams = (u_coarse, u_fine, u_fine_jit,
    n_depth); returns (B, Kc + Kf).  ``marginal_alt``: draws within MARGIN of a cdf
    boundary take the other neighbouring bin (``_marginal_alt_fine``)."""
    from . import ref_cpu

    rays = rays.reshape(-1, 8).float().cpu()
    B = rays.shape[0]
    parts = [z_coarse.reshape(B, -1).float().cpu()]
    nf = n_fine - n_fine_depth
    if nf > 0:
        w = w_coarse.reshape(B, -1).float().cpu()
        u, uj = streams[1].reshape(B, -1), streams[2].reshape(B, -1)
        parts.append(_marginal_alt_fine(rays, w, n_coarse, u, uj, lindisp) if marginal_alt
                     else ref_cpu.sample_fine(rays, w, n_coarse, u, uj, lindisp))
    if n_fine_depth > 0:
        parts.append(ref_cpu.sample_fine_depth(rays, depth_coarse.reshape(B).float().cpu(), n_fine_depth,
                                               depth_std, streams[3].reshape(B, -1)))
    return torch.sort(torch.cat(parts, -1), -1)[0]


def expected_fine_sets(*args, **kw):
    """(expected_fine_z(...), expected_fine_z(..., marginal_alt=True)): the two sample sets a
    flipped ray may take from its own coarse weights (pass to ``classify_fine``)."""
    return expected_fine_z(*args, **kw), expected_fine_z(*args, marginal_alt=True, **kw)


def classify_fine(w_coarse_hip, w_coarse_ref, u_fine, z_fine_hip, z_fine_ref, z_expected_hip=None):
    """Classify the fine pass of B rays.

    Returns a dict of (B,) bool masks:
      flip        — the importance-sample bins differ between the HIP and reference coarse
                    weights (a proven searchsorted flip), or the samples differ and a draw
                    sits within MARGIN of a boundary of the HIP cdf (the device's double
                    cdf scan and torch's fp32 cumsum round a boundary differently);
      z_differs   — the returned sorted fine samples differ beyond the fp32 tolerance;
      unexplained — z_differs but no bin differs (must be empty: a kernel bug);
      inconsistent — (with ``z_expected_hip``, from ``expected_fine_z`` on the HIP coarse
                    outputs, or a tuple of it and its ``marginal_alt=True`` variant) a
                    flipped ray whose HIP samples are NOT the reference algorithm's draw
                    from the HIP coarse weights (must be empty);
    plus ``flip_idx`` (list of ray indices) for messages."""
    B = z_fine_ref.shape[0]
    zh = z_fine_hip.detach().float().cpu().reshape(B, -1)
    zr = z_fine_ref.detach().float().cpu().reshape(B, -1)
    if u_fine is not None and u_fine.numel() > 0:
        u = u_fine.reshape(B, -1)
        bh = fine_bins(w_coarse_hip.reshape(B, -1), u)
        br = fine_bins(w_coarse_ref.reshape(B, -1), u)
        bins_differ = (bh != br).any(-1)
        marginal = boundary_distance(w_coarse_hip.reshape(B, -1), u) <= MARGIN
    else:
        bins_differ = marginal = torch.zeros(B, dtype=torch.bool)
    z_differs = ~close_mask(zh, zr).all(-1)
    flip = bins_differ | (marginal & z_differs)
    unexplained = z_differs & ~flip
    inconsistent = torch.zeros(B, dtype=torch.bool)
    if z_expected_hip is not None:
        # a tuple: the expected set and its marginal-draw alternative (either may match)
        sets = z_expected_hip if isinstance(z_expected_hip, (tuple, list)) else (z_expected_hip,)
        follows = torch.zeros(B, dtype=torch.bool)
        for ze in sets:
            follows |= close_mask(zh, ze.detach().float().cpu().reshape(B, -1)).all(-1)
        inconsistent = flip & ~follows
    return dict(flip=flip, z_differs=z_differs, unexplained=unexplained, inconsistent=inconsistent,
                flip_idx=[int(i) for i in torch.nonzero(flip).reshape(-1)])
