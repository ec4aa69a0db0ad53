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
    return synth.pixelnerf_state(cfg["seed"], d_latent=cfg["d_latent"], d_hidden=cfg["d_hidden"],
                                 n_blocks=cfg.get("n_blocks", 5),
                                 combine_layer=cfg.get("combine_layer", 3),
                                 with_fine=cfg.get("with_fine", True))


def c_or_none(arr):
    c = arr["c"]
    return None if c.numel() == 0 else c


def focal_of(arr):
    f = arr["focal"]
    return f.reshape(()) if f.numel() == 1 else f


def latent_of(cfg):
    n, c, h, w = cfg["latent_shape"]
    return synth.latent(cfg["latent_seed"], n, c, h, w)
