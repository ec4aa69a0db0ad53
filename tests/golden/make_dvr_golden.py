#!/usr/bin/env python
"""Golden vectors for the DVR-layout loader (pnr.data.DVRDataset: ShapeNet-NMR and DTU) and the
multi-object loader (pnr.data.MultiObjectDataset) from the REFERENCE's src/data/DVRDataset.py and
src/data/MultiObjectDataset.py (read-only at /root/reference).

Test infrastructure.  Small synthetic datasets (tests/dvr_synth.py) are written to a temp dir and
read by the reference's loaders: NMR with and without masks, at native size and through the
area-resize path; DTU (decomposed projection matrices, scale matrices, averaged intrinsics); the
multi-object layout (an all-transparent frame included).  Stubs (absent offline):
  * imageio.imread -> PIL decode to the same uint8 array;
  * torchvision.transforms Compose / ToTensor / Normalize -> their documented tensor semantics
    (HWC or HW uint8 -> CHW float / 255; (x - mean) / std per channel);
  * cv2.decomposeProjectionMatrix -> scipy.linalg.rq with the diagonal signs moved into R and the
    camera centre as P's SVD null vector (an implementation independent of pnr.data's QR-based one;
    the synthetic P = s K [R | -R C] with s > 0 and a positive-diagonal K has one such
    decomposition);
  * pyhocon, dotmap: imported by util, unused by the loaders.
The fixture stores the inputs and the loaders' outputs only (multi-object items keyed by scene).

Run:  python tests/golden/make_dvr_golden.py   (skips if /root/reference is absent)
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

import dvr_synth  # noqa: E402

CASES = [  # (tag, sub_format, masks, loader kwargs)
    ("nmr", "shapenet", True, {}),
    ("nmr_nomask", "shapenet", False, {}),
    ("nmr_resized", "shapenet", True, dict(image_size=(10, 10))),
    ("dtu", "dtu", True, dict(list_prefix="new_", sub_format="dtu", scale_focal=False, z_near=0.1, z_far=5.0)),
    ("dtu_resized", "dtu", False, dict(list_prefix="new_", sub_format="dtu", scale_focal=False,
                                       image_size=(10, 10))),
]
KEYS = ("focal", "c", "images", "masks", "bbox", "poses")


def _stubs():
    import scipy.linalg
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
            a = np.asarray(a)
            if a.ndim == 2:
                a = a[..., None]
            t = torch.from_numpy(np.ascontiguousarray(a)).permute(2, 0, 1)
            return t.float().div(255.0) if t.dtype == torch.uint8 else t.float()

    class Normalize:
        def __init__(self, mean, std):
            self.mean, self.std = torch.tensor(mean), torch.tensor(std)

        def __call__(self, t):
            return (t - self.mean[:, None, None]) / self.std[:, None, None]

    tvt.Compose, tvt.ToTensor, tvt.Normalize = Compose, ToTensor, Normalize
    tvt.Resize = tvt.ColorJitter = None
    tvt.functional = types.SimpleNamespace()
    tvm = types.ModuleType("torchvision.models")
    tv.transforms, tv.models = tvt, tvm
    for name, mod in (("torchvision", tv), ("torchvision.transforms", tvt), ("torchvision.models", tvm)):
        sys.modules[name] = mod
    cv2 = types.ModuleType("cv2")
    cv2.COLORMAP_HOT = 11

    def decompose(P):
        K, R = scipy.linalg.rq(np.asarray(P, np.float64)[:, :3])
        D = np.diag(np.sign(np.diag(K)))
        _, _, vt = np.linalg.svd(P)
        return K @ D, D @ R, vt[-1][:, None]

    cv2.decomposeProjectionMatrix = decompose
    sys.modules["cv2"] = cv2
    ph = types.ModuleType("pyhocon")
    ph.ConfigFactory = types.SimpleNamespace(parse_file=lambda *a, **k: None)
    sys.modules.setdefault("pyhocon", ph)
    dm = types.ModuleType("dotmap")
    dm.DotMap = type("DotMap", (dict,), {})
    sys.modules.setdefault("dotmap", dm)


def _load(name):
    import importlib.util

    spec = importlib.util.spec_from_file_location("ref_" + name, os.path.join(REF, "data", name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _arr(v):
    if v is None:
        return None
    if torch.is_tensor(v):
        return v.numpy()
    if isinstance(v, list):
        return np.zeros((0,), np.float32) if not v else np.stack([_arr(x) for x in v])
    return np.asarray(v)


def main():
    if not os.path.isdir(REF):
        print("reference absent; skipping")
        return
    _stubs()
    sys.path.insert(0, REF)
    DVRDataset = _load("DVRDataset").DVRDataset
    MultiObjectDataset = _load("MultiObjectDataset").MultiObjectDataset
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        for tag, sub, with_masks, kw in CASES:
            inp = dvr_synth.make_dvr_inputs(sub, with_masks=with_masks, seed=len(tag))
            out["%s_images_in" % tag] = inp["images"]
            if with_masks:
                out["%s_masks_in" % tag] = inp["masks"]
            for o, cam in enumerate(inp["cams"]):
                for k, v in cam.items():
                    out["%s_cam%d_%s" % (tag, o, k)] = v
            root = dvr_synth.write_dvr_dir(os.path.join(tmp, tag), inp, list_prefix=kw.get("list_prefix", "softras_"))
            d = DVRDataset(root, stage="test", **kw)
            out["%s_meta" % tag] = np.array([len(d), d.z_near, d.z_far], np.float64)
            for i in range(len(d)):
                item = d[i]
                for k in KEYS:
                    if k in item and _arr(item[k]) is not None:
                        out["%s_%d_%s" % (tag, i, k)] = _arr(item[k])
        inp = dvr_synth.make_multiobj_inputs()
        out["multi_images_in"], out["multi_poses_in"], out["multi_angle_in"] = inp["images"], inp["poses"], inp["angle"]
        root = dvr_synth.write_multiobj_dir(tmp, inp)
        d = MultiObjectDataset(root, stage="test")
        for i in range(len(d)):
            item = d[i]
            scene = os.path.basename(item["path"])
            for k in KEYS:
                if k in item:
                    out["multi_%s_%s" % (scene, k)] = _arr(item[k])
    np.savez_compressed(os.path.join(HERE, "dvr_loader.npz"), **out)
    print("wrote", os.path.join(HERE, "dvr_loader.npz"), len(out), "arrays")


if __name__ == "__main__":
    main()
