"""Synthetic SRN-layout dataset on disk (tests and the SRN loader golden generator).

make_inputs() draws deterministic pixels / poses / intrinsics; write_srn_dir() lays them out
as <root>/cars/cars_<stage>/<object>/{intrinsics.txt, rgb/*.png, pose/*.txt} and returns
<root>/cars (the datadir the reference's loader takes)."""
import os

import numpy as np


def make_inputs(n_obj=2, n_views=3, size=24, seed=0):
    rng = np.random.default_rng(seed)
    imgs = np.full((n_obj, n_views, size, size, 4), 255, np.uint8)
    for o in range(n_obj):
        for v in range(n_views):
            y0, x0 = rng.integers(2, size // 2, 2)
            h, w = rng.integers(4, size // 2, 2)
            blob = rng.integers(0, 255, (h, w, 3)).astype(np.uint8)
            imgs[o, v, y0:y0 + h, x0:x0 + w, :3] = blob
            imgs[o, v, ..., 3] = rng.integers(0, 256, (size, size)).astype(np.uint8)   # alpha ignored
    poses = rng.normal(size=(n_obj, n_views, 4, 4)).astype(np.float32)
    poses[..., 3, :] = [0, 0, 0, 1]
    intr = np.array([[30.0 + 5 * o, 11.5 + o, 12.25 - o] for o in range(n_obj)], np.float32)
    return {"images": imgs, "poses": poses, "intrinsics": intr, "size": np.array(size)}


def write_srn_dir(tmp, inp, name="cars", stage="test"):
    from PIL import Image

    root = os.path.join(tmp, name)
    n_obj, n_views = inp["images"].shape[:2]
    size = int(inp["size"])
    for o in range(n_obj):
        d = os.path.join(root, "%s_%s" % (name, stage), "obj%03d" % o)
        os.makedirs(os.path.join(d, "rgb"))
        os.makedirs(os.path.join(d, "pose"))
        f, cx, cy = (float(x) for x in inp["intrinsics"][o])
        with open(os.path.join(d, "intrinsics.txt"), "w") as fh:
            fh.write("%r %r %r 0.\n0. 0. 0.\n1.\n%d %d\n" % (f, cx, cy, size, size))
        for v in range(n_views):
            Image.fromarray(inp["images"][o, v]).save(os.path.join(d, "rgb", "%06d.png" % v))
            np.savetxt(os.path.join(d, "pose", "%06d.txt" % v), inp["poses"][o, v].reshape(1, 16))
    return root
