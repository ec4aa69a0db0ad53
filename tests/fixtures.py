"""Load golden vectors (tests/golden/*.npz) and rebuild their hash-generated inputs."""
import json
import os

import numpy as np
import torch

from pnr import synth

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    cfg = json.loads(str(z["config"]))
    arr = {k: torch.from_numpy(z[k].copy()) for k in z.files if k != "config"}
    return cfg, arr


def state_dict(cfg):
    o = cfg.get("opts", {})
    return synth.pixelnerf_state(cfg["seed"], d_in=78 if o.get("use_code_viewdirs") else 42,
                                 d_latent=cfg["d_latent"] + o.get("global_latent_size", 0),
                                 d_hidden=cfg["d_hidden"], n_blocks=cfg.get("n_blocks", 5),
                                 combine_layer=cfg.get("combine_layer", 3),
                                 with_fine=cfg.get("with_fine", True), use_spade=o.get("use_spade", False))


def model_conf(cfg):
    """The PixelNeRFNet conf of a render fixture (make_golden.model_conf): the shipped conf at the
    fixture's widths, with its ``opts`` (the alt_* fixtures: options the fused kernel does not
    implement)."""
    o = cfg.get("opts", {})
    mlp = dict(type="resnet", n_blocks=cfg.get("n_blocks", 5), d_hidden=cfg["d_hidden"],
               combine_layer=cfg.get("combine_layer", 3), combine_type=o.get("combine_type", "average"),
               beta=o.get("beta", 0.0), use_spade=o.get("use_spade", False))
    num_layers = {64: 1, 128: 2, 256: 3, 512: 4}[cfg["d_latent"]]
    conf = dict(use_encoder=True, use_xyz=True, use_code=True,
                code=dict(num_freqs=6, freq_factor=1.5, include_input=True), use_viewdirs=True,
                use_code_viewdirs=o.get("use_code_viewdirs", False), mlp_coarse=dict(mlp), mlp_fine=dict(mlp),
                encoder=dict(backbone="resnet34", pretrained=False, num_layers=num_layers,
                             index_padding=o.get("index_padding", "border"),
                             index_interp=o.get("index_interp", "bilinear")),
                use_global_encoder="global_latent_size" in o)
    if "global_latent_size" in o:
        conf["global_encoder"] = dict(backbone="resnet34", pretrained=False, latent_size=o["global_latent_size"])
    return conf


def c_or_none(arr):
    c = arr["c"]
    return None if c.numel() == 0 else c


def focal_of(arr):
    f = arr["focal"]
    return f.reshape(()) if f.numel() == 1 else f


def latent_of(cfg):
    n, c, h, w = cfg["latent_shape"]
    return synth.latent(cfg["latent_seed"], n, c, h, w)
