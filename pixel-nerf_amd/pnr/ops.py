"""Tensor-level wrappers over the C ABI (device tensors in, device tensors out).

Each wrapper validates device / dtype / contiguity, allocates outputs with torch
(the library never allocates), and launches on the current HIP stream.
"""
import torch

from . import _lib


def _dev(t, name):
    if not torch.is_tensor(t):
        raise TypeError("%s must be a tensor" % name)
    if t.device.type != "cuda":
        raise ValueError("pnr: %s must be on a HIP device (got %s); the HIP path has no CPU "
                         "fallback" % (name, t.device))
    if t.dtype != torch.float32:
        raise ValueError("pnr: %s must be float32 (got %s)" % (name, t.dtype))
    return t.contiguous()


def sample_coarse(rays, n_coarse, u_coarse, lindisp=False):
    """NeRFRenderer.sample_coarse (nerf.py:98-118): (B, 8), (B, Kc) -> z (B, Kc)."""
    rays = _dev(rays, "rays")
    u = _dev(u_coarse, "u_coarse")
    B = rays.shape[0]
    assert u.shape == (B, n_coarse), (u.shape, B, n_coarse)
    z = torch.empty(B, n_coarse, device=rays.device, dtype=torch.float32)
    lib = _lib.load()
    _lib.check(lib.pnr_sample_coarse(_lib.ptr(rays), B, n_coarse, _lib.ptr(u), int(bool(lindisp)),
                                     _lib.ptr(z), _lib.stream_of(rays.device)), "pnr_sample_coarse")
    return z


def sample_fine(rays, z_coarse, coarse_weights, coarse_depth, n_fine, n_fine_depth, depth_std,
                u_fine, u_fine_jit, n_depth, lindisp=False):
    """sample_fine + sample_fine_depth + cat + sort (nerf.py:120-161, 284-295).
    Returns the sorted fine-pass depths (B, Kc + Kf)."""
    rays = _dev(rays, "rays")
    zc = _dev(z_coarse, "z_coarse")
    w = _dev(coarse_weights, "coarse_weights")
    B, kc = zc.shape
    nf = n_fine - n_fine_depth
    d = _dev(coarse_depth, "coarse_depth") if n_fine_depth > 0 else None
    uf = _dev(u_fine, "u_fine") if nf > 0 else None
    uj = _dev(u_fine_jit, "u_fine_jit") if nf > 0 else None
    nd = _dev(n_depth, "n_depth") if n_fine_depth > 0 else None
    out = torch.empty(B, kc + n_fine, device=rays.device, dtype=torch.float32)
    lib = _lib.load()
    _lib.check(lib.pnr_sample_fine(_lib.ptr(rays), B, kc, _lib.ptr(zc), _lib.ptr(w), _lib.ptr(d),
                                   n_fine, n_fine_depth, float(depth_std), _lib.ptr(uf),
                                   _lib.ptr(uj), _lib.ptr(nd), int(bool(lindisp)), _lib.ptr(out),
                                   _lib.stream_of(rays.device)), "pnr_sample_fine")
    return out


def composite(z, raw, rays, white_bkgd, want_weights=True):
    """Alpha composite (nerf.py:176-249): z (B, K), raw (B, K, 4) -> (weights, rgb, depth)."""
    z = _dev(z, "z")
    raw = _dev(raw, "raw")
    rays = _dev(rays, "rays")
    from . import torchops

    B, K = z.shape
    assert raw.shape[:2] == (B, K) and raw.shape[-1] == 4, raw.shape
    w, rgb, depth = torchops.load().composite(z, raw, rays, bool(white_bkgd), bool(want_weights))
    return (w if want_weights else None), rgb, depth


def rng_fill(seed, offset, stream, n_rays, width, device="cuda"):
    """The counter-mode draws of one stream (pnr_rng_fill; include/pnr_abi.h pnr_rng):
    (n_rays, width) for rays offset .. offset + n_rays - 1, exactly as the render kernels
    draw them in counter mode.  stream: _lib.RNG_U_COARSE .. RNG_N_DEPTH."""
    out = torch.empty(n_rays, width, device=device, dtype=torch.float32)
    lib = _lib.load()
    _lib.check(lib.pnr_rng_fill(int(seed), int(offset), int(stream), int(n_rays), int(width), _lib.ptr(out),
                                _lib.stream_of(out.device)), "pnr_rng_fill")
    return out


def rng_render_streams(seed, offset, n_rays, n_coarse, n_fine, n_fine_depth, device="cuda"):
    """(u_coarse, u_fine, u_fine_jit, n_depth) of a counter-mode render call, materialised."""
    nf = max(n_fine - n_fine_depth, 0)
    return (rng_fill(seed, offset, _lib.RNG_U_COARSE, n_rays, n_coarse, device),
            rng_fill(seed, offset, _lib.RNG_U_FINE, n_rays, nf, device),
            rng_fill(seed, offset, _lib.RNG_U_FINE_JIT, n_rays, nf, device),
            rng_fill(seed, offset, _lib.RNG_N_DEPTH, n_rays, n_fine_depth, device))
