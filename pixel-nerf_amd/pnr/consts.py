"""Small device constants without a host sync.

``torch.tensor([...], device="cuda")`` copies from pageable host memory, which waits
for the stream to drain; in the training loop (encode every step) that idles the GPU.
Constants such as the image size or the latent scale repeat from step to step, so one
device copy per (values, device, dtype) is kept and reused.  Callers must not modify
the returned tensor in place.
"""
import torch

_cache = {}


def device_const(values, device, dtype=torch.float32):
    device = torch.device(device)
    if device.type == "cuda" and device.index is None:
        device = torch.device("cuda", torch.cuda.current_device())
    key = (tuple(float(v) for v in values), device, dtype)
    t = _cache.get(key)
    if t is None:
        if len(_cache) > 256:
            _cache.clear()
        t = torch.tensor(list(key[0]), dtype=dtype, device=device)
        _cache[key] = t
    return t
