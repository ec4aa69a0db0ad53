"""Synthetic DVR-layout (ShapeNet-NMR and DTU) and multi-object datasets on disk (tests and
tests/golden/make_dvr_golden.py).

make_dvr_inputs() draws deterministic pixels, masks and cameras; write_dvr_dir() lays them out as
<root>/<category>/<list_prefix><stage>.lst + <category>/<object>/{image/*.png, mask/*.png,
cameras.npz}, the layout DVRDataset.py:42-64 / 109-121 read.  ShapeNet cameras: world_mat_i
(3 x 4 for even i, 4 x 4 for odd i), a world_mat_inv_i for view 0, camera_mat_i with fx = fy on
the [-1, 1] image convention.  DTU cameras: world_mat_i = [P; 0 0 0 1] with P = s K [R | -R C]
(s > 0, K upper triangular with a positive diagonal) and a scale_mat_i.
make_multiobj_inputs() / write_multiobj_dir(): <root>/<stage>/<scene>/transforms.json with RGBA
<frame>_obj.png images (MultiObjectDataset.py:19-27, 71-77)."""
import json
import os

import numpy as np


def _rot(rng):
    a = rng.normal(size=3)
    from scipy.spatial.transform import Rotation

    return Rotation.from_rotvec(a).as_matrix()


def make_dvr_inputs(sub_format="shapenet", n_obj=2, n_views=3, size=20, seed=0, with_masks=True):
    rng = np.random.default_rng(seed + (100 if sub_format == "dtu" else 0))
    imgs = rng.integers(0, 256, (n_obj, n_views, size, size, 3)).astype(np.uint8)
    masks = np.zeros((n_obj, n_views, size, size), np.uint8)
    for o in range(n_obj):
        for v in range(n_views):
            y0, x0 = rng.integers(1, size // 2, 2)
            h, w = rng.integers(3, size // 2, 2)
            masks[o, v, y0:y0 + h, x0:x0 + w] = 255
    cams = []
    for o in range(n_obj):
        c = {}
        for v in range(n_views):
            R, C = _rot(rng), rng.normal(size=3) * 2.0
            if sub_format == "dtu":
                K = np.array([[rng.uniform(200, 300), rng.uniform(-1, 1), rng.uniform(8, 12)],
                              [0.0, rng.uniform(200, 300), rng.uniform(8, 12)], [0.0, 0.0, 1.0]])
                P = rng.uniform(0.5, 2.0) * K @ np.hstack([R, -(R @ C)[:, None]])
                c["world_mat_%d" % v] = np.vstack([P, [0, 0, 0, 1]])
                S = np.eye(4)
                S[:3, :3] *= rng.uniform(0.5, 2.0)
                S[:3, 3] = rng.normal(size=3)
                c["scale_mat_%d" % v] = S
            else:
                E = np.vstack([np.hstack([R, -(R @ C)[:, None]]), [0, 0, 0, 1]])
                c["world_mat_%d" % v] = E[:3] if v % 2 == 0 else E
                if v == 0:
                    c["world_mat_inv_%d" % v] = np.linalg.inv(E)
                f = 1.75 + 0.25 * o
                c["camera_mat_%d" % v] = np.array([[f, 0, 0, 0], [0, f, 0, 0], [0, 0, 1, 0], [0, 0, 0, 1.0]])
        cams.append(c)
    return {"images": imgs, "masks": masks if with_masks else None, "cams": cams, "size": size}


def write_dvr_dir(tmp, inp, list_prefix="softras_", stage="test", category="02958343"):
    """Returns the datadir (<tmp>/dvr) that DVRDataset takes."""
    from PIL import Image

    root = os.path.join(tmp, "dvr")
    cat = os.path.join(root, category)
    n_obj, n_views = inp["images"].shape[:2]
    names = ["obj%03d" % o for o in range(n_obj)]
    os.makedirs(cat, exist_ok=True)
    with open(os.path.join(cat, list_prefix + stage + ".lst"), "w") as f:
        f.write("\n".join(names) + "\n")
    for o, name in enumerate(names):
        d = os.path.join(cat, name)
        os.makedirs(os.path.join(d, "image"), exist_ok=True)
        if inp["masks"] is not None:
            os.makedirs(os.path.join(d, "mask"), exist_ok=True)
        for v in range(n_views):
            Image.fromarray(inp["images"][o, v]).save(os.path.join(d, "image", "%06d.png" % v))
            if inp["masks"] is not None:
                Image.fromarray(inp["masks"][o, v]).save(os.path.join(d, "mask", "%03d.png" % v))
        np.savez(os.path.join(d, "cameras.npz"), **inp["cams"][o])
    return root


def make_multiobj_inputs(n_scene=2, n_views=3, size=16, seed=0):
    rng = np.random.default_rng(seed + 7)
    imgs = rng.integers(0, 256, (n_scene, n_views, size, size, 4)).astype(np.uint8)
    imgs[0, 1] = 0                                   # an all-transparent, all-zero frame (empty box)
    imgs[..., 3] = np.where(rng.random((n_scene, n_views, size, size)) < 0.5, 0, imgs[..., 3])
    poses = rng.normal(size=(n_scene, n_views, 4, 4))
    poses[..., 3, :] = [0, 0, 0, 1]
    return {"images": imgs, "poses": poses, "angle": np.array(0.69)}


def write_multiobj_dir(tmp, inp, stage="test"):
    from PIL import Image

    root = os.path.join(tmp, "multi")
    for s in range(inp["images"].shape[0]):
        d = os.path.join(root, stage, "scene%02d" % s)
        os.makedirs(d, exist_ok=True)
        frames = []
        for v in range(inp["images"].shape[1]):
            Image.fromarray(inp["images"][s, v]).save(os.path.join(d, "r_%d_obj.png" % v))
            frames.append({"file_path": "./r_%d" % v, "transform_matrix": inp["poses"][s, v].tolist()})
        with open(os.path.join(d, "transforms.json"), "w") as f:
            json.dump({"camera_angle_x": float(inp["angle"]), "frames": frames}, f)
    return root
