"""ORACLE — test infrastructure only; never imported by the product path.

CPU fp32 restatement of the reference pixelNeRF ray march (etiiiR/pixel-nerf),
written as plain functions over tensors with the reference's op order so its
results reproduce the reference's own outputs on the same CPU.  It is the
checker for the HIP path (tests/, ``__graft_entry__.smoke()``) and the timed
``cpu_baseline`` leg of ``bench.py`` (kind "port").  Only those may import it.

Pinned against golden vectors produced by the reference itself
(``tests/golden/make_golden.py`` imports ``/root/reference/src`` with stubs and
injects the random streams) — see ``tests/test_oracle_golden.py``.

Functions and the reference lines they restate:

* ``sample_coarse``      nerf.py:98-118
* ``sample_fine``        nerf.py:120-148
* ``sample_fine_depth``  nerf.py:150-161
* ``composite``          nerf.py:163-249 (model output passed in)
* ``render``             nerf.py:251-303 (+ _format_outputs 305-316)
* ``encode_buffers``     models.py:89-141 (post-CNN part: poses/focal/c)
* ``pixelnerf_forward``  models.py:146-266
* ``positional_encoding`` code.py:30-42
* ``index_latent``       encoder.py:80-109 (grid_sample, align_corners, border)
* ``resnetfc_forward``   resnetfc.py:132-184 with ResnetBlockFC 53-62
* ``combine_interleaved`` util.py:461-471
"""
import torch
import torch.nn.functional as F


# ------------------------------------------------------------------ model --
def repeat_interleave(t, repeats):
    # util.py:58-65
    return t.unsqueeze(1).expand(-1, repeats, *t.shape[1:]).reshape(-1, *t.shape[1:])


def combine_interleaved(t, inner_dims):
    # util.py:461-471 (average)
    if len(inner_dims) == 1 and inner_dims[0] == 1:
        return t
    t = t.reshape(-1, *inner_dims, *t.shape[1:])
    return torch.mean(t, dim=1)


def positional_encoding(x, freqs, phases):
    """code.py:30-42: [x, sin(x*f0+0), sin(x*f0+pi/2), ...] (N, 3) -> (N, 39)."""
    n_rep = freqs.shape[1]
    embed = x.unsqueeze(1).repeat(1, n_rep, 1)
    embed = torch.sin(torch.addcmul(phases, embed, freqs))
    embed = embed.view(x.shape[0], -1)
    return torch.cat((x, embed), dim=-1)


def resnetfc_forward(sd, prefix, zx, d_latent, n_blocks, combine_layer, inner_dims, relu=None):
    """resnetfc.py:132-184; blocks are x + fc_1(relu(fc_0(relu(x)))) (53-62).

    ``relu(t, site)`` (tests only) replaces torch.relu at each ReLU: site ("x", b) before
    block b's fc_0, ("h", b) before its fc_1, ("xf", n_blocks) before lin_out."""
    if relu is None:
        def relu(t, site):
            return torch.relu(t)

    def lin(name, t):
        return F.linear(t, sd[prefix + name + ".weight"], sd[prefix + name + ".bias"])

    z = zx[..., :d_latent]
    x = zx[..., d_latent:]
    x = lin("lin_in", x)
    for blk in range(n_blocks):
        if blk == combine_layer:
            x = combine_interleaved(x, inner_dims)
        if d_latent > 0 and blk < combine_layer:
            x = x + lin("lin_z.%d" % blk, z)
        net = lin("blocks.%d.fc_0" % blk, relu(x, ("x", blk)))
        dx = lin("blocks.%d.fc_1" % blk, relu(net, ("h", blk)))
        x = x + dx
    return lin("lin_out", relu(x, ("xf", n_blocks)))


def encode_buffers(poses, focal, width, height, c=None):
    """models.py:89-141 minus the CNN: world->camera poses, focal (fy negated), c.

    poses (NS, 4, 4) or (SB, NS, 4, 4).  Returns (poses_wc (SB*NS, 3, 4), focal,
    c, NS, image_shape [W, H])."""
    if poses.dim() == 4:
        ns = poses.shape[1]
        poses = poses.reshape(-1, 4, 4)
    else:
        ns = 1
    rot = poses[:, :3, :3].transpose(1, 2)
    trans = -torch.bmm(rot, poses[:, :3, 3:])
    poses_wc = torch.cat((rot, trans), dim=-1)
    image_shape = torch.tensor([float(width), float(height)])
    focal = torch.as_tensor(focal, dtype=torch.float32)
    if focal.dim() == 0:
        focal = focal[None, None].repeat((1, 2))
    elif focal.dim() == 1:
        focal = focal.unsqueeze(-1).repeat((1, 2))
    else:
        focal = focal.clone()
    focal = focal.float()
    focal[..., 1] *= -1.0
    if c is None:
        c = (image_shape * 0.5).unsqueeze(0)
    else:
        c = torch.as_tensor(c, dtype=torch.float32)
        if c.dim() == 0:
            c = c[None, None].repeat((1, 2))
        elif c.dim() == 1:
            c = c.unsqueeze(-1).repeat((1, 2))
    return poses_wc, focal, c, ns, image_shape


def latent_scaling(latent):
    # encoder.py:161-163
    s = torch.empty(2, dtype=torch.float32)
    s[0] = latent.shape[-1]
    s[1] = latent.shape[-2]
    return s / (s - 1) * 2.0


def index_latent(latent, uv, image_shape):
    """encoder.py:80-109: bilinear grid_sample, align_corners=True, border."""
    if uv.shape[0] == 1 and latent.shape[0] > 1:
        uv = uv.expand(latent.shape[0], -1, -1)
    scale = latent_scaling(latent) / image_shape
    uv = uv * scale - 1.0
    uv = uv.unsqueeze(2)
    samples = F.grid_sample(latent, uv, align_corners=True, mode="bilinear",
                            padding_mode="border")
    return samples[:, :, :, 0]


class Scene:
    """Everything ``encode()`` leaves in the model (models.py:111-141)."""

    def __init__(self, latent, poses, focal, width, height, c=None):
        self.latent = latent
        self.poses, self.focal, self.c, self.ns, self.image_shape = encode_buffers(
            poses, focal, width, height, c)


def pixelnerf_forward(sd, scene, xyz, coarse=True, viewdirs=None, d_latent=512,
                      n_blocks=5, combine_layer=3, has_fine=True, relu=None):
    """models.py:146-266 for the shipped conf (use_xyz, normalize_z, use_code,
    use_viewdirs, use_code_viewdirs=False, no global encoder).  MLP rows before
    combine_layer are (object, view, point), after it (object, point); ``relu`` as
    resnetfc_forward."""
    SB, B, _ = xyz.shape
    NS = scene.ns
    poses = scene.poses
    xyz = repeat_interleave(xyz, NS)
    xyz_rot = torch.matmul(poses[:, None, :3, :3], xyz.unsqueeze(-1))[..., 0]
    xyz = xyz_rot + poses[:, None, :3, 3]
    z_feature = xyz_rot.reshape(-1, 3)
    z_feature = positional_encoding(z_feature, sd["code._freqs"], sd["code._phases"])
    vd = viewdirs.reshape(SB, B, 3, 1)
    vd = repeat_interleave(vd, NS)
    vd = torch.matmul(poses[:, None, :3, :3], vd).reshape(-1, 3)
    z_feature = torch.cat((z_feature, vd), dim=1)
    uv = -xyz[:, :, :2] / xyz[:, :, 2:]
    uv *= repeat_interleave(scene.focal.unsqueeze(1), NS if scene.focal.shape[0] > 1 else 1)
    uv += repeat_interleave(scene.c.unsqueeze(1), NS if scene.c.shape[0] > 1 else 1)
    latent = index_latent(scene.latent, uv, scene.image_shape)
    latent = latent.transpose(1, 2).reshape(-1, d_latent)
    mlp_input = torch.cat((latent, z_feature), dim=-1)
    prefix = "mlp_coarse." if (coarse or not has_fine) else "mlp_fine."
    out = resnetfc_forward(sd, prefix, mlp_input, d_latent, n_blocks, combine_layer, (NS, B), relu=relu)
    out = out.reshape(-1, B, 4)
    out = torch.cat([torch.sigmoid(out[..., :3]), torch.relu(out[..., 3:4])], dim=-1)
    return out.reshape(SB, B, -1)


# --------------------------------------------------------------- renderer --
def sample_coarse(rays, n_coarse, u, lindisp=False):
    """nerf.py:98-118 with the U[0,1) draw injected as ``u`` (B, Kc)."""
    near, far = rays[:, -2:-1], rays[:, -1:]
    step = 1.0 / n_coarse
    B = rays.shape[0]
    z_steps = torch.linspace(0, 1 - step, n_coarse).unsqueeze(0).repeat(B, 1)
    z_steps += u * step
    if not lindisp:
        return near * (1 - z_steps) + far * z_steps
    return 1 / (1 / near * (1 - z_steps) + 1 / far * z_steps)


def sample_fine(rays, weights, n_coarse, u, u_jit, lindisp=False):
    """nerf.py:120-148: inverse CDF over Kc uniform bins in t (not the jittered z)."""
    weights = weights.detach() + 1e-5
    pdf = weights / torch.sum(weights, -1, keepdim=True)
    cdf = torch.cumsum(pdf, -1)
    cdf = torch.cat([torch.zeros_like(cdf[:, :1]), cdf], -1)
    inds = torch.searchsorted(cdf, u, right=True).float() - 1.0
    inds = torch.clamp_min(inds, 0.0)
    z_steps = (inds + u_jit) / n_coarse
    near, far = rays[:, -2:-1], rays[:, -1:]
    if not lindisp:
        return near * (1 - z_steps) + far * z_steps
    return 1 / (1 / near * (1 - z_steps) + 1 / far * z_steps)


def sample_fine_depth(rays, depth, n_fine_depth, depth_std, n):
    """nerf.py:150-161 with the N(0,1) draw injected as ``n`` (B, Kfd)."""
    z = depth.unsqueeze(1).repeat((1, n_fine_depth))
    z += n * depth_std
    return torch.max(torch.min(z, rays[:, -1:]), rays[:, -2:-1])


def composite(rays, z_samp, raw, white_bkgd):
    """nerf.py:176-249 given the model output ``raw`` (B, K, 4)."""
    deltas = z_samp[:, 1:] - z_samp[:, :-1]
    delta_inf = rays[:, -1:] - z_samp[:, -1:]
    deltas = torch.cat([deltas, delta_inf], -1)
    rgbs = raw[..., :3]
    sigmas = raw[..., 3]
    alphas = 1 - torch.exp(-deltas * torch.relu(sigmas))
    alphas_shifted = torch.cat([torch.ones_like(alphas[:, :1]), 1 - alphas + 1e-10], -1)
    T = torch.cumprod(alphas_shifted, -1)
    weights = alphas * T[:, :-1]
    rgb = torch.sum(weights.unsqueeze(-1) * rgbs, -2)
    depth = torch.sum(weights * z_samp, -1)
    if white_bkgd:
        pix_alpha = weights.sum(dim=1)
        rgb = rgb + 1 - pix_alpha.unsqueeze(-1)
    return weights, rgb, depth


def _points(rays, z):
    B, K = z.shape
    pts = rays[:, None, :3] + z.unsqueeze(2) * rays[:, None, 3:6]
    dirs = rays[:, None, 3:6].expand(-1, K, -1)
    return pts, dirs


def render(model_fn, rays, n_coarse, n_fine, n_fine_depth, streams, white_bkgd,
           lindisp=False, depth_std=0.01, using_fine=None, sigma_noise=None):
    """nerf.py:251-303.  ``model_fn(points (SB, P, 3), coarse, viewdirs) -> (SB, P, 4)``;
    ``streams`` = (u_coarse, u_fine, u_fine_jit, n_depth).  ``using_fine`` (default
    n_fine > 0) is the flag nerf.py:87 fixes at construction: with it set and no fine
    samples, the fine pass re-evaluates the coarse samples (nerf.py:284-298).
    ``sigma_noise`` = (coarse (B, Kc), fine (B, K)) N(0,1)·noise_std draws added to sigma
    before compositing (training mode, nerf.py:225-226).  Returns a dict
    {"coarse": {rgb, depth, weights, z}, "fine": {...}} shaped (SB, B', ...)."""
    u_c, u_f, u_j, n_d = streams
    SB = rays.shape[0]
    rays = rays.reshape(-1, 8)
    B = rays.shape[0]
    if using_fine is None:
        using_fine = n_fine > 0

    def one_pass(z, coarse):
        pts, dirs = _points(rays, z)
        K = z.shape[1]
        raw = model_fn(pts.reshape(SB, -1, 3), coarse, dirs.reshape(SB, -1, 3)).reshape(B, K, -1)
        if sigma_noise is not None:
            raw = torch.cat([raw[..., :3], raw[..., 3:] + sigma_noise[0 if coarse else 1].unsqueeze(-1)], -1)
        w, rgb, depth = composite(rays, z, raw, white_bkgd)
        return dict(rgb=rgb.reshape(SB, -1, 3), depth=depth.reshape(SB, -1),
                    weights=w.reshape(SB, -1, K), z=z, raw=raw.reshape(-1, 4),
                    _w=w, _depth=depth)

    z_c = sample_coarse(rays, n_coarse, u_c, lindisp)
    out = {"coarse": one_pass(z_c, True)}
    if using_fine:
        samps = [z_c]
        if n_fine - n_fine_depth > 0:
            samps.append(sample_fine(rays, out["coarse"]["_w"], n_coarse, u_f, u_j, lindisp))
        if n_fine_depth > 0:
            samps.append(sample_fine_depth(rays, out["coarse"]["_depth"], n_fine_depth,
                                           depth_std, n_d))
        z_f, _ = torch.sort(torch.cat(samps, -1), -1)
        out["fine"] = one_pass(z_f, False)
    return out
