#!/usr/bin/env python
"""Golden vectors for the image encoder (SpatialEncoder.forward, encoder.py:111-164) from the
REFERENCE's src/model/encoder.py (read-only at /root/reference).

Test infrastructure.  torchvision is absent offline, so its ``models.resnet34(pretrained,
norm_layer)`` is stubbed by the in-repo ResNet-34 trunk (pnr.encoder.ResNetTrunk: torchvision's
module names and shapes, tests/test_host.py checks them against torchvision's architecture); the
REFERENCE's SpatialEncoder then runs its own forward -- feature_scale resize, conv1 / bn1 / relu,
the optional first max-pool, layer1..layer3, the align_corners upsample of every map to the
first one's size, the concat and latent_scaling -- on hash-initialised weights with
non-trivial BatchNorm statistics (pnr.synth.encoder_state).  Cases: use_first_pool x num_layers
{3, 4} x feature_scale {1, 0.5} in eval mode (running statistics), and one train-mode case (batch
statistics over 2 images, the training encode).  The fixture stores the images, the cases, the
latents, latent_scaling and the weight seed only (weights are regenerated from the seed).

Run:  python tests/golden/make_encoder_golden.py   (skips if /root/reference is absent)
"""
import json
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference/src"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "pixel-nerf_amd"))

from pnr import synth  # noqa: E402
from pnr.encoder import ResNetTrunk  # noqa: E402

CASES = [dict(use_first_pool=p, num_layers=n, feature_scale=f, train=False)
         for p in (True, False) for n in (4, 3) for f in (1.0, 0.5)] + \
        [dict(use_first_pool=True, num_layers=4, feature_scale=1.0, train=True)]
SEED = 5
SIZE = 24


def _stubs():
    tv = types.ModuleType("torchvision")
    tvt = types.ModuleType("torchvision.transforms")
    tvm = types.ModuleType("torchvision.models")
    tvt.functional = types.SimpleNamespace()
    tvm.resnet34 = lambda pretrained=False, norm_layer=torch.nn.BatchNorm2d: ResNetTrunk(norm_layer=norm_layer)
    tv.transforms, tv.models = tvt, tvm
    for name, mod in (("torchvision", tv), ("torchvision.transforms", tvt), ("torchvision.models", tvm)):
        sys.modules[name] = mod
    cv2 = types.ModuleType("cv2")
    cv2.COLORMAP_HOT = 11
    sys.modules["cv2"] = cv2
    ph = types.ModuleType("pyhocon")
    ph.ConfigFactory = types.SimpleNamespace(parse_file=lambda *a, **k: None)
    sys.modules["pyhocon"] = ph
    dm = types.ModuleType("dotmap")
    dm.DotMap = type("DotMap", (dict,), {})
    sys.modules["dotmap"] = dm


def main():
    if not os.path.isdir(REF):
        print("reference absent; skipping")
        return
    _stubs()
    sys.path.insert(0, REF)
    from model.encoder import SpatialEncoder   # the reference's encoder

    imgs = torch.from_numpy(synth.hash_sym(61, (2, 3, SIZE, SIZE), 1.0))
    out = {"images": imgs.numpy(), "cases": np.frombuffer(json.dumps(CASES).encode(), np.uint8),
           "weight_seed": np.array(SEED), "size": np.array(SIZE)}
    for i, c in enumerate(CASES):
        enc = SpatialEncoder(pretrained=False, num_layers=c["num_layers"], feature_scale=c["feature_scale"],
                             use_first_pool=c["use_first_pool"])
        enc.model.load_state_dict(synth.encoder_state(SEED, enc.model.state_dict()))
        enc.train(c["train"])
        with torch.no_grad():
            lat = enc(imgs if c["train"] else imgs[:1])
        out["latent_%d" % i] = lat.numpy()
        out["latent_scaling_%d" % i] = enc.latent_scaling.numpy()
        if c["train"]:
            out["running_mean_after_%d" % i] = enc.model.bn1.running_mean.numpy()
        print(i, c, tuple(lat.shape))
    np.savez_compressed(os.path.join(HERE, "encoder_fw.npz"), **out)
    print("wrote", os.path.join(HERE, "encoder_fw.npz"))


if __name__ == "__main__":
    main()
