"""Deterministic synthetic scenes for fixtures, parity tests and the benchmark.

There is no network in this pipeline, so no pretrained checkpoint or dataset can
be fetched.  Every input is generated from an integer hash so a
fixture only has to store seeds, and so the GPU box regenerates bit-identical
inputs without the reference present:

* ``hash_uniform(seed, n)``  — splitmix64(seed, i) -> 24-bit U[0, 1) float32.
* MLP weights  U(-1, 1) * sqrt(3 / fan_in) (kaiming-uniform scale); biases
  U(-0.1, 0.1).  The reference init zeroes ``fc_1`` (resnetfc.py:39), which
  would make every residual block the identity, so it is not used here.
* latent  ~ approx N(0, 1) (sum of 4 uniforms, rescaled), channels-first
  ``(NS, C, H_l, W_l)`` exactly as ``SpatialEncoder.latent`` (encoder.py:160).
* cameras  SRN-style ``pose_spherical(theta, -10, 1.3)`` (util.py:309-323).

State-dict key names follow the reference's checkpoint layout.
"""
import numpy as np
import torch

from . import util

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x):
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def hash_uniform(seed, n):
    """n float32 values in [0, 1), a pure function of (seed, index)."""
    with np.errstate(over="ignore"):
        base = _splitmix64(np.uint64(seed) * np.uint64(0x100000001B3) + np.uint64(0x5EED))
        idx = np.arange(n, dtype=np.uint64) + base
    h = _splitmix64(idx)
    return ((h >> np.uint64(40)).astype(np.float64) / float(1 << 24)).astype(np.float32)


def hash_sym(seed, shape, scale=1.0):
    """U(-scale, scale) float32 array of the given shape."""
    n = int(np.prod(shape))
    u = hash_uniform(seed, n).astype(np.float64)
    return ((2.0 * u - 1.0) * scale).astype(np.float32).reshape(shape)


def hash_normal(seed, shape):
    """Approximately N(0,1): Irwin-Hall(4) rescaled; deterministic and cheap."""
    n = int(np.prod(shape))
    u = hash_uniform(seed, 4 * n).astype(np.float64).reshape(4, n)
    x = (u.sum(0) - 2.0) * np.sqrt(3.0)
    return x.astype(np.float32).reshape(shape)


def _linear(seed, d_out, d_in):
    w = hash_sym(seed, (d_out, d_in), np.sqrt(3.0 / d_in))
    b = hash_sym(seed + 7919, (d_out,), 0.1)
    return w, b


def resnetfc_state(seed, d_in=42, d_latent=512, d_hidden=512, n_blocks=5,
                   combine_layer=3, d_out=4, prefix="", use_spade=False):
    """State dict of a ResnetFC (resnetfc.py:65-130) with hash-init weights (scale_z too with
    use_spade, after every other layer so the other layers' seeds do not move)."""
    sd = {}
    k = 0

    def put(name, d_o, d_i):
        nonlocal k
        w, b = _linear(seed * 1000 + k, d_o, d_i)
        k += 1
        sd[prefix + name + ".weight"] = torch.from_numpy(w)
        sd[prefix + name + ".bias"] = torch.from_numpy(b)

    put("lin_in", d_hidden, d_in)
    put("lin_out", d_out, d_hidden)
    for i in range(n_blocks):
        put("blocks.%d.fc_0" % i, d_hidden, d_hidden)
        put("blocks.%d.fc_1" % i, d_hidden, d_hidden)
    if d_latent > 0:
        for i in range(min(combine_layer, n_blocks)):
            put("lin_z.%d" % i, d_hidden, d_latent)
        if use_spade:
            for i in range(min(combine_layer, n_blocks)):
                put("scale_z.%d" % i, d_hidden, d_latent)
    return sd


def pe_buffers(num_freqs=6, freq_factor=1.5):
    """``code._freqs`` / ``code._phases`` buffers (code.py:6-28)."""
    freqs = freq_factor * 2.0 ** torch.arange(0, num_freqs)
    f = torch.repeat_interleave(freqs, 2).view(1, -1, 1).float()
    ph = torch.zeros(2 * num_freqs)
    ph[1::2] = np.pi * 0.5
    return f, ph.view(1, -1, 1).float()


def pixelnerf_state(seed, d_in=42, d_latent=512, d_hidden=512, n_blocks=5,
                    combine_layer=3, with_fine=True, num_freqs=6, freq_factor=1.5, use_spade=False):
    """Non-encoder part of a PixelNeRFNet state dict (62 keys)."""
    sd = {}
    f, ph = pe_buffers(num_freqs, freq_factor)
    sd["code._freqs"] = f
    sd["code._phases"] = ph
    sd.update(resnetfc_state(seed, d_in, d_latent, d_hidden, n_blocks, combine_layer,
                             prefix="mlp_coarse.", use_spade=use_spade))
    if with_fine:
        sd.update(resnetfc_state(seed + 1, d_in, d_latent, d_hidden, n_blocks,
                                 combine_layer, prefix="mlp_fine.", use_spade=use_spade))
    return sd


def encoder_state(seed, template):
    """Hash-initialised values for an encoder trunk state dict ``template`` (name -> tensor), in the
    template's order: convolutions U(-1, 1) sqrt(3 / fan_in) (unit-variance activations), BatchNorm
    gamma U(0.5, 1.5), beta U(-0.1, 0.1), running_mean U(-0.2, 0.2), running_var U(0.5, 2.0)
    (non-trivial statistics, so the BatchNorm arithmetic is exercised), num_batches_tracked 0."""
    out = {}
    for i, (k, v) in enumerate(template.items()):
        s = seed * 1000 + i
        if k.endswith("num_batches_tracked"):
            out[k] = torch.zeros_like(v)
        elif v.dim() == 4:
            out[k] = torch.from_numpy(hash_sym(s, tuple(v.shape), float(np.sqrt(3.0 / v[0].numel()))))
        else:
            lo, hi = {"weight": (0.5, 1.5), "bias": (-0.1, 0.1), "running_mean": (-0.2, 0.2),
                      "running_var": (0.5, 2.0)}[k.rsplit(".", 1)[1]]
            u = hash_uniform(s, v.numel()).astype(np.float32).reshape(tuple(v.shape))
            out[k] = torch.from_numpy(lo + (hi - lo) * u)
    return out


def latent(seed, n_views, channels, h_l, w_l):
    """(NS, C, H_l, W_l) float32 latent, channels-first as the encoder emits it."""
    return torch.from_numpy(hash_normal(seed, (n_views, channels, h_l, w_l)))


def srn_poses(thetas, phi=-10.0, radius=1.3):
    return torch.stack([util.pose_spherical(t, phi, radius) for t in thetas], 0)


def rng_streams(seed, n_rays, n_coarse, n_fine, n_fine_depth):
    """Injected random streams in the order the reference draws them
    (nerf.py:111, 135-141, 158): u_coarse, u_fine, u_fine_jit, n_depth."""
    g = torch.Generator().manual_seed(seed)
    nf = n_fine - n_fine_depth
    u_c = torch.rand(n_rays, n_coarse, generator=g)
    u_f = torch.rand(n_rays, nf, generator=g) if nf > 0 else torch.zeros(n_rays, 0)
    u_j = torch.rand(n_rays, nf, generator=g) if nf > 0 else torch.zeros(n_rays, 0)
    n_d = torch.randn(n_rays, n_fine_depth, generator=g) if n_fine_depth > 0 else torch.zeros(n_rays, 0)
    return u_c, u_f, u_j, n_d


def scene_srn(seed=0, n_rays=256, width=128, height=128, focal=131.25, theta_src=0.0,
              theta_tgt=30.0, near=0.01, far=4.0, channels=512, h_l=64, w_l=64,
              pick="centre"):
    """SRN-cars-like single-view scene.

    Returns dict with latent (1, C, H_l, W_l), src pose (1, 4, 4), focal, c,
    image size and target rays (n_rays, 8)."""
    src = srn_poses([theta_src])
    tgt = srn_poses([theta_tgt])
    rays = util.gen_rays(tgt, width, height, torch.tensor(focal), near, far).reshape(-1, 8)
    if pick == "centre":
        n_all = rays.shape[0]
        start = max(0, n_all // 2 - n_rays // 2 - width // 2)
        rays = rays[start:start + n_rays]
    elif pick == "hash":
        idx = (hash_uniform(seed + 17, n_rays) * rays.shape[0]).astype(np.int64)
        rays = rays[torch.from_numpy(idx)]
    else:  # "all" / frame prefix
        rays = rays[:n_rays]
    return dict(
        latent=latent(seed, 1, channels, h_l, w_l),
        poses=src,
        focal=torch.tensor(focal, dtype=torch.float32),
        c=None,
        width=width,
        height=height,
        rays=rays.contiguous(),
        near=near,
        far=far,
        latent_seed=seed,
    )


def scene_nmr(seed=0, n_rays=128, size=64, focal=70.0, theta_src=0.0, theta_tgt=45.0,
              near=1.2, far=4.0, radius=2.7, channels=512, pick="hash"):
    """ShapeNet-NMR-like single-view scene: 64x64 images, the latent
    at half resolution (32x32, use_first_pool=False, conf/exp/sn64.conf:4-8), near/far
    1.2/4.0 (DVRDataset.py:26-27), a synthetic focal of ~70 px, cameras on a sphere of
    radius 2.7.  ``pick`` as scene_srn ("hash" = n_rays hashed pixels, "all" = prefix)."""
    src = srn_poses([theta_src], phi=-20.0, radius=radius)
    tgt = srn_poses([theta_tgt], phi=-20.0, radius=radius)
    rays = util.gen_rays(tgt, size, size, torch.tensor(focal), near, far).reshape(-1, 8)
    if pick == "hash":
        idx = (hash_uniform(seed + 29, n_rays) * rays.shape[0]).astype(np.int64)
        rays = rays[torch.from_numpy(idx)]
    else:
        rays = rays[:n_rays]
    return dict(
        latent=latent(seed, 1, channels, size // 2, size // 2),
        poses=src,
        focal=torch.tensor(focal, dtype=torch.float32),
        c=None,
        width=size,
        height=size,
        rays=rays.contiguous(),
        near=near,
        far=far,
        latent_seed=seed,
    )


def scene_multiview(seed=0, n_views=3, n_rays=64, width=400, height=300,
                    focal=(300.0, 310.0), c=(195.0, 152.0), near=0.1, far=5.0,
                    channels=512, h_l=150, w_l=200, radius=2.0):
    """DTU-like multi-view scene: NS source views, (fx, fy), (cx, cy)."""
    src = srn_poses([-25.0 + 25.0 * i for i in range(n_views)], phi=-15.0, radius=radius)
    tgt = srn_poses([10.0], phi=-12.0, radius=radius)
    f = torch.tensor(focal, dtype=torch.float32)
    cc = torch.tensor(c, dtype=torch.float32)
    rays = util.gen_rays(tgt, width, height, f, near, far, c=cc).reshape(-1, 8)
    idx = (hash_uniform(seed + 23, n_rays) * rays.shape[0]).astype(np.int64)
    rays = rays[torch.from_numpy(idx)]
    return dict(
        latent=latent(seed, n_views, channels, h_l, w_l),
        poses=src,
        focal=f,
        c=cc,
        width=width,
        height=height,
        rays=rays.contiguous(),
        near=near,
        far=far,
        latent_seed=seed,
    )
