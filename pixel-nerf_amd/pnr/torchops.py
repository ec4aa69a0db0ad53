"""torch.ops.pnr.* — the operators of libpnr_torch.so (csrc/torch_ops.cpp), registered with
TORCH_LIBRARY over the C ABI of libpnr.so (SURVEY §8(b) "where the new code plugs in").

``NeRFRenderer.forward`` dispatches the fused march to ``torch.ops.pnr.render_rays``,
``PixelNeRFNet.forward`` to ``torch.ops.pnr.point_query`` and ``pnr.ops.composite`` to
``torch.ops.pnr.composite``.  Meta kernels make them traceable (torch.compile / FakeTensor).
There is no fallback: a missing library raises.
"""
import os

import torch

from . import _lib

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PNR_TORCH_LIB_PATH") or os.path.join(_HERE, "libpnr_torch.so")
_loaded = False
# benchmark hook: a callable (n_rays, n_coarse, n_fine) -> list of 7 hipEvent_t handles (ints)
# recorded around the launches of the next render_rays call, or None
EVENTS_HOOK = None


def load():
    """Register torch.ops.pnr.* once (libpnr.so is loaded first: the operators call it)."""
    global _loaded
    if not _loaded:
        _lib.load()
        if not os.path.exists(LIB_PATH):
            raise _lib.PnrError("libpnr_torch.so not built (%s); run `make -C pixel-nerf_amd` or "
                                "__graft_entry__.build()" % LIB_PATH)
        torch.ops.load_library(LIB_PATH)
        _loaded = True
    return torch.ops.pnr


def desc_list(desc):
    """pnr_mlp_desc (ctypes) -> the operators' int[8] desc."""
    return [int(desc.d_in), int(desc.d_latent), int(desc.d_hidden), int(desc.d_out), int(desc.n_blocks),
            int(desc.combine_layer), int(desc.pe_n), int(desc.precision)]


def scene_args(net):
    """(latent_cl, cams, n_obj, n_views, image_w, image_h) of an encoded PixelNeRFNet."""
    sc = net.hip_scene()
    return (net.encoder.latent_cl, net.cams, int(sc.n_obj), int(sc.n_views), float(sc.image_w),
            float(sc.image_h))
