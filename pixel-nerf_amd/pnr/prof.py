"""Profiler ranges with the reference's names (SURVEY §5 "Tracing / profiling"): the reference
wraps its hot-path calls in torch.autograd.profiler.record_function ranges -- renderer_forward
(nerf.py:264), renderer_composite (nerf.py:175), model_inference (models.py:156),
encoder_index (encoder.py:90), resnetfc_infer (resnetfc.py:139), resblock (resnetfc.py:54),
positional_enc (code.py:36).  The same names mark the same calls here, so a torch.profiler (or
rocprofv3 --marker-trace through roctx) timeline of a user's script reads as before; the HIP
kernels inside appear under them."""
import functools

import torch

__all__ = ["ranged"]


def ranged(name):
    """Decorator: run the function inside record_function(name)."""
    def deco(fn):
        @functools.wraps(fn)
        def wrapper(*args, **kwargs):
            with torch.autograd.profiler.record_function(name):
                return fn(*args, **kwargs)
        return wrapper
    return deco
