#!/usr/bin/env python
"""Golden vectors for the SRN-layout loader (pnr.data.SRNDataset) from the REFERENCE's
src/data/SRNDataset.py (read-only at /root/reference).

Test infrastructure.  A small synthetic SRN directory (2 objects x 3 views, 24 x 24 RGBA
PNGs on a white background, random poses, SRN-style intrinsics.txt) is written to a temp
dir and read by the reference's SRNDataset at its native size, through its area-resize path
and with world_scale.  Stubs (absent offline, none of them loader logic):
  * imageio.imread -> PIL decode to the same uint8 array;
  * torchvision.transforms Compose / ToTensor / Normalize -> their documented tensor
    semantics (HWC uint8 -> CHW float / 255; (x - mean) / std per channel);
  * cv2, pyhocon, dotmap: imported by util, unused by the loader.
The fixture stores the inputs (pixels, poses, intrinsics) and the loader's outputs only.

Run:  python tests/golden/make_srn_golden.py   (skips if /root/reference is absent)
"""
import os
import sys
import tempfile
import types

import numpy as np
import torch

REF = "/root/reference/src"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "tests"))

from srn_synth import make_inputs, write_srn_dir  # noqa: E402


def _stubs():
    from PIL import Image

    io = types.ModuleType("imageio")
    io.imread = lambda p: np.asarray(Image.open(p))
    sys.modules["imageio"] = io

    tv = types.ModuleType("torchvision")
    tvt = types.ModuleType("torchvision.transforms")

    class Compose:
        def __init__(self, ops):
            self.ops = ops

        def __call__(self, x):
            for op in self.ops:
                x = op(x)
            return x

    class ToTensor:
        def __call__(self, a):
            t = torch.from_numpy(np.ascontiguousarray(a)).permute(2, 0, 1)
            return t.float().div(255.0) if t.dtype == torch.uint8 else t.float()

    class Normalize:
        def __init__(self, mean, std):
            self.mean, self.std = torch.tensor(mean), torch.tensor(std)

        def __call__(self, t):
            return (t - self.mean[:, None, None]) / self.std[:, None, None]

    class Resize:
        def __init__(self, *a, **k):
            raise NotImplementedError

    tvt.Compose, tvt.ToTensor, tvt.Normalize, tvt.Resize = Compose, ToTensor, Normalize, Resize
    tvt.ColorJitter = Resize
    tvt.functional = types.SimpleNamespace()
    tvm = types.ModuleType("torchvision.models")
    tvm.resnet34 = tvm.resnet18 = lambda **k: torch.nn.Module()
    tv.transforms, tv.models = tvt, tvm
    for name, mod in (("torchvision", tv), ("torchvision.transforms", tvt), ("torchvision.models", tvm)):
        sys.modules[name] = mod
    cv2 = types.ModuleType("cv2")
    cv2.COLORMAP_HOT = 11
    sys.modules.setdefault("cv2", cv2)
    ph = types.ModuleType("pyhocon")       # util.args only (arg parsing)
    ph.ConfigFactory = types.SimpleNamespace(parse_file=lambda *a, **k: None)
    sys.modules.setdefault("pyhocon", ph)
    dm = types.ModuleType("dotmap")        # renderer output container, imported by util

    class DotMap(dict):
        pass

    dm.DotMap = DotMap
    sys.modules.setdefault("dotmap", dm)


def main():
    if not os.path.isdir(REF):
        print("reference absent; skipping")
        return
    _stubs()
    sys.path.insert(0, REF)
    # the module file alone: data/__init__ pulls in the other loaders and their augmentations
    import importlib.util

    spec = importlib.util.spec_from_file_location("ref_srn", os.path.join(REF, "data", "SRNDataset.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    SRNDataset = mod.SRNDataset   # the reference's loader

    inp = make_inputs()
    out = dict(inp)
    with tempfile.TemporaryDirectory() as tmp:
        root = write_srn_dir(tmp, inp)
        for tag, kw in (("native", {}), ("resized", dict(image_size=(12, 12))),
                        ("scaled", dict(world_scale=1.5))):
            d = SRNDataset(root, stage="test", **{"image_size": (24, 24), **kw})
            assert len(d) == inp["images"].shape[0]
            for i in range(len(d)):
                item = d[i]
                for k in ("focal", "c", "images", "masks", "bbox", "poses"):
                    out["%s_%d_%s" % (tag, i, k)] = item[k].numpy()
            out["%s_near_far" % tag] = np.array([d.z_near, d.z_far], np.float32)
    np.savez_compressed(os.path.join(HERE, "srn_loader.npz"), **out)
    print("wrote", os.path.join(HERE, "srn_loader.npz"))


if __name__ == "__main__":
    main()
