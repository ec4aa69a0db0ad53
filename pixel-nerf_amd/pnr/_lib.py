"""ctypes binding of libpnr.so (include/pnr_abi.h).

The product path has no fallback: if the HIP library is missing or fails to load,
every call raises.  ``torch`` is imported first so that the HIP runtime torch
ships (soname libamdhip64.so.7) is the one libpnr.so binds to.
"""
import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime before libpnr.so)

_HERE = os.path.dirname(os.path.abspath(__file__))
# PNR_LIB_PATH: alternate build (diagnostic ablation builds only)
LIB_PATH = os.environ.get("PNR_LIB_PATH") or os.path.join(_HERE, "libpnr.so")

c_f = ctypes.c_float
c_i32 = ctypes.c_int32
c_i64 = ctypes.c_int64
c_size = ctypes.c_size_t
c_vp = ctypes.c_void_p
PF = ctypes.POINTER(ctypes.c_float)


class Scene(ctypes.Structure):
    _fields_ = [("latent", c_vp), ("cams", c_vp), ("n_obj", c_i32), ("n_views", c_i32),
                ("latent_h", c_i32), ("latent_w", c_i32), ("latent_c", c_i32),
                ("image_w", c_f), ("image_h", c_f)]


class MlpDesc(ctypes.Structure):
    _fields_ = [("d_in", c_i32), ("d_latent", c_i32), ("d_hidden", c_i32), ("d_out", c_i32),
                ("n_blocks", c_i32), ("combine_layer", c_i32), ("pe_n", c_i32),
                ("precision", c_i32)]


class MlpWeights(ctypes.Structure):
    _fields_ = [("desc", MlpDesc), ("lin_in_w", c_vp), ("lin_in_b", c_vp),
                ("lin_z_w", c_vp * 8), ("lin_z_b", c_vp * 8),
                ("fc0_w", c_vp * 8), ("fc0_b", c_vp * 8),
                ("fc1_w", c_vp * 8), ("fc1_b", c_vp * 8),
                ("lin_out_w", c_vp), ("lin_out_b", c_vp),
                ("pe_freqs", c_vp), ("pe_phases", c_vp)]


class Rays(ctypes.Structure):
    _fields_ = [("rays", c_vp), ("n_rays", c_i64), ("rays_per_obj", c_i64)]


class Rng(ctypes.Structure):
    """Injected streams, or counter mode (Philox {seed, offset}) when all four are NULL."""
    _fields_ = [("u_coarse", c_vp), ("u_fine", c_vp), ("u_fine_jit", c_vp), ("n_depth", c_vp),
                ("seed", ctypes.c_uint64), ("offset", ctypes.c_uint64)]


# pnr_rng counter-mode stream ids (PNR_RNG_*)
RNG_U_COARSE, RNG_U_FINE, RNG_U_FINE_JIT, RNG_N_DEPTH = 0, 1, 2, 3
ABI_VERSION = 8


class RenderCfg(ctypes.Structure):
    _fields_ = [("n_coarse", c_i32), ("n_fine", c_i32), ("n_fine_depth", c_i32),
                ("depth_std", c_f), ("white_bkgd", c_i32), ("lindisp", c_i32),
                ("march_mode", c_i32),   # ABI 3: -1 = the pnr_render_set_fused default
                ("ray_order", c_vp)]     # ABI 8: the fused march's processing order (NULL: input order)


class RenderOut(ctypes.Structure):
    _fields_ = [("coarse_rgb", c_vp), ("coarse_depth", c_vp), ("coarse_weights", c_vp),
                ("fine_rgb", c_vp), ("fine_depth", c_vp), ("fine_weights", c_vp),
                ("z_coarse", c_vp), ("z_fine", c_vp)]


# name -> (restype, argtypes); must match include/pnr_abi.h exactly
SIGNATURES = {
    "pnr_abi_version": (c_i32, []),
    "pnr_last_error": (ctypes.c_char_p, []),
    "pnr_mlp_packed_bytes": (c_size, [ctypes.POINTER(MlpDesc)]),
    "pnr_mlp_pack": (c_i32, [ctypes.POINTER(MlpWeights), c_vp, c_size, c_vp]),
    "pnr_point_query_workspace_bytes": (c_size, [ctypes.POINTER(Scene), c_i64]),
    "pnr_point_query": (c_i32, [ctypes.POINTER(Scene), ctypes.POINTER(MlpDesc), c_vp, c_vp, c_vp,
                                c_i64, c_vp, c_vp, c_size, c_vp]),
    "pnr_render_workspace_bytes": (c_size, [ctypes.POINTER(Scene), ctypes.POINTER(RenderCfg), c_i64]),
    "pnr_render_forward": (c_i32, [ctypes.POINTER(Scene), ctypes.POINTER(MlpDesc), c_vp, c_vp,
                                   ctypes.POINTER(Rays), ctypes.POINTER(Rng),
                                   ctypes.POINTER(RenderCfg), ctypes.POINTER(RenderOut), c_vp,
                                   c_size, c_vp]),
    "pnr_render_forward_events": (c_i32, [ctypes.POINTER(Scene), ctypes.POINTER(MlpDesc), c_vp, c_vp,
                                          ctypes.POINTER(Rays), ctypes.POINTER(Rng),
                                          ctypes.POINTER(RenderCfg), ctypes.POINTER(RenderOut),
                                          c_vp, c_size, c_vp, ctypes.POINTER(c_vp)]),
    "pnr_latent_project_bytes": (c_size, [ctypes.POINTER(Scene), ctypes.POINTER(MlpDesc)]),
    "pnr_latent_project": (c_i32, [ctypes.POINTER(Scene), ctypes.POINTER(MlpWeights), c_vp, c_size, c_vp]),
    "pnr_point_query_proj": (c_i32, [ctypes.POINTER(Scene), ctypes.POINTER(MlpDesc), c_vp, c_vp, c_vp, c_vp,
                                     c_i64, c_vp, c_vp, c_size, c_vp]),
    "pnr_render_forward_proj": (c_i32, [ctypes.POINTER(Scene), ctypes.POINTER(MlpDesc), c_vp, c_vp, c_vp, c_vp,
                                        ctypes.POINTER(Rays), ctypes.POINTER(Rng),
                                        ctypes.POINTER(RenderCfg), ctypes.POINTER(RenderOut),
                                        c_vp, c_size, c_vp, ctypes.POINTER(c_vp)]),
    "pnr_render_set_fused": (c_i32, [c_i32]),
    "pnr_sample_coarse": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_i32, c_vp, c_vp]),
    "pnr_sample_fine": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_vp, c_vp, c_i32, c_i32, c_f, c_vp,
                                c_vp, c_vp, c_i32, c_vp, c_vp]),
    "pnr_composite": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp]),
    "pnr_rng_fill": (c_i32, [ctypes.c_uint64, ctypes.c_uint64, c_i32, c_i64, c_i32, c_vp, c_vp]),
    "pnr_gen_rays": (c_i32, [c_vp, c_i64, c_i32, c_i32, c_i32, c_f, c_f, c_f, c_f, c_f, c_f, c_vp, c_vp]),
    "pnr_latent_channels_last": (c_i32, [ctypes.POINTER(c_vp), ctypes.POINTER(c_i32), ctypes.POINTER(c_i32),
                                         ctypes.POINTER(c_i32), c_i32, c_i32, c_vp, c_i32, c_i32, c_vp]),
    "pnr_latent_channels_last_nhwc": (c_i32, [ctypes.POINTER(c_vp), ctypes.POINTER(c_i32), ctypes.POINTER(c_i32),
                                              ctypes.POINTER(c_i32), c_i32, c_i32, c_vp, c_i32, c_i32, c_vp]),
    "pnr_fold_batchnorm": (c_i32, [c_vp, c_i32, c_i64, c_vp]),
    "pnr_latent_channels_last_backward": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_vp]),
    "pnr_point_save_floats": (c_size, [ctypes.POINTER(MlpDesc), c_i64]),
    "pnr_render_points": (c_i32, [ctypes.POINTER(Scene), ctypes.POINTER(MlpDesc), c_vp,
                                  ctypes.POINTER(Rays), c_vp, c_i32, c_vp, c_vp, c_vp, c_size, c_vp]),
    "pnr_composite_backward": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp,
                                       c_vp, c_vp]),
    "pnr_points_input_backward": (c_i32, [ctypes.POINTER(Scene), ctypes.POINTER(MlpDesc), c_vp,
                                          ctypes.POINTER(Rays), c_vp, c_i32, c_vp, c_vp, c_vp, c_vp,
                                          c_vp]),
    "pnr_points_input_backward_masked": (c_i32, [ctypes.POINTER(Scene), ctypes.POINTER(MlpDesc), c_vp,
                                                 ctypes.POINTER(Rays), c_vp, c_i32, c_vp, c_vp, c_vp, c_vp,
                                                 c_vp, c_vp]),
    "pnr_mlp_packed_t_bytes": (c_size, [ctypes.POINTER(MlpDesc)]),
    "pnr_mlp_pack_t": (c_i32, [ctypes.POINTER(MlpWeights), c_vp, c_vp, c_size, c_vp]),
    "pnr_mlp_backward": (c_i32, [ctypes.POINTER(MlpDesc), c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp,
                                 c_vp]),
    "pnr_mlp_backward_workspace_bytes": (c_size, [ctypes.POINTER(MlpDesc), c_i64]),
    "pnr_mlp_backward_bias": (c_i32, [ctypes.POINTER(MlpDesc), c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp,
                                      c_vp, c_vp, c_size, c_vp]),
    "pnr_mlp_backward_views": (c_i32, [ctypes.POINTER(MlpDesc), c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_vp,
                                       c_vp, c_vp, c_vp, c_size, c_vp]),
    "pnr_weight_grad_workspace_bytes": (c_size, [c_i32, c_i64]),
    "pnr_weight_grad": (c_i32, [ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), c_i32, c_i64,
                                c_vp, c_size, c_vp]),
    "pnr_weight_grad_arith": (c_i32, [ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), c_i32,
                                      c_i64, c_i32, c_vp, c_size, c_vp]),
}

# pnr_weight_grad_arith arithmetics (PNR_WGRAD_*, ABI 4)
WGRAD_ARITH = {"f16x3": 0, "bf16x6": 1}

_lib = None


class PnrError(RuntimeError):
    pass


def load():
    """Load libpnr.so once; raise loudly if it is missing (no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise PnrError("libpnr.so not built (%s); run `make -C pixel-nerf_amd` or "
                       "__graft_entry__.build()" % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        if os.environ.get("PNR_LIB_PATH") and not hasattr(lib, name):
            continue   # an older diagnostic build (A/B against a previous revision)
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.pnr_abi_version() != ABI_VERSION:
        raise PnrError("libpnr.so ABI version %d, this binding expects %d; rebuild it"
                       % (lib.pnr_abi_version(), ABI_VERSION))
    _lib = lib
    return lib


def check(rc, what):
    if rc != 0:
        msg = load().pnr_last_error().decode(errors="replace")
        raise PnrError("%s failed (status %d): %s" % (what, rc, msg))


def ptr(t):
    """Device pointer of a tensor (or None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


class fused_march:
    """Context manager: pnr_render_set_fused(mode) inside, the previous DEFAULT restored after
    (2, the default: fused passes + fine-draw kernel; 1: fine draws in the coarse epilogue too;
    0: the separate sample / composite kernels).  It changes the process default, which only
    calls without their own mode use; ``NeRFRenderer.march_mode`` names the mode per renderer
    (pnr_render_cfg.march_mode, no process state)."""

    def __init__(self, mode):
        self.on = int(mode)

    def __enter__(self):
        self.prev = load().pnr_render_set_fused(self.on)
        return self

    def __exit__(self, *exc):
        load().pnr_render_set_fused(self.prev)
        return False


def stream_of(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
