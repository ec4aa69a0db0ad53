"""Dataset readers for the eval / training callers of the ray march (the ``data`` package).

Counterparts of the reference's loaders -- the producers of the images, poses and intrinsics
that feed ``PixelNeRFNet.encode`` and ``util.gen_rays`` in eval/gen_video.py, eval_approx.py,
eval.py and train/train.py -- and of ``data.get_split_dataset`` (src/data/__init__.py:10-72),
with the same directory layouts, item keys, value conventions and near / far planes:

* ``SRNDataset`` (SRNDataset.py:10-145; formats ``srn``, ``pollen``):
    <datadir>/<name>_<stage>/<object>/intrinsics.txt   "f cx cy _" on line 1, "H W" on the last
                                     /rgb/*.png          RGB(A) uint8
                                     /pose/*.txt          4 x 4 camera-to-world (OpenCV axes)
* ``DVRDataset`` (DVRDataset.py:11-274; formats ``dvr`` (ShapeNet-NMR, BASELINE cfg3),
  ``dvr_gen``, ``dvr_dtu`` (DTU, cfg4)):
    <datadir>/<category>/<list_prefix><stage>.lst, <category>/<object>/image/*.png|jpg,
    /mask/*.png (optional), /cameras.npz (world_mat_i, camera_mat_i / scale_mat_i)
* ``MultiObjectDataset`` (MultiObjectDataset.py:14-117; format ``multi_obj``):
    <datadir>/<stage>/**/transforms.json + <frame>_obj.png (RGBA)
* ``ColorJitterDataset`` (data_util.py:14-56): the DTU training augmentation.

Image decoding uses PIL (the reference uses imageio, absent offline); the array handed to the
conversions is the same uint8 image.  ``cameras.npz`` is read with numpy's default
``allow_pickle=False``.
"""
import glob
import os

import numpy as np
import torch
import torch.nn.functional as F

__all__ = ["SRNDataset", "DVRDataset", "MultiObjectDataset", "ColorJitterDataset", "get_split_dataset",
           "image_to_tensor_balanced", "mask_to_tensor", "decompose_projection"]


def _imread(path):
    """imageio.imread: the file's uint8 array as stored ((H, W) grey, (H, W, 3|4) colour)."""
    from PIL import Image

    with Image.open(path) as im:
        return np.array(im)   # a writable copy


def _imread_rgb(path):
    a = _imread(path)
    if a.ndim == 2:                      # greyscale: imageio returns (H, W)
        a = np.repeat(a[..., None], 3, axis=-1)
    return a[..., :3]


def image_to_tensor_balanced(img):
    """util.get_image_to_tensor_balanced() (util.py:68-75): ToTensor then Normalize(0.5, 0.5):
    (H, W, 3) uint8 -> (3, H, W) float32 in [-1, 1]."""
    t = torch.from_numpy(np.ascontiguousarray(img)).permute(2, 0, 1).float().div(255.0)
    return (t - 0.5) / 0.5


def mask_to_tensor(mask):
    """util.get_mask_to_tensor() (util.py:78-81): (H, W, 1) or (H, W) uint8 -> (1, H, W) float32 in
    [0, 1] (ToTensor gives a 2-D array one channel)."""
    mask = np.asarray(mask)
    if mask.ndim == 2:
        mask = mask[..., None]
    t = torch.from_numpy(np.ascontiguousarray(mask)).permute(2, 0, 1).float().div(255.0)
    return (t - 0.0) / 1.0


class SRNDataset(torch.utils.data.Dataset):
    """SRNDataset.py:10-145.  ``dataset[i]`` is one object with all its views."""

    def __init__(self, datadir, stage="train", image_size=(128, 128), world_scale=1.0):
        super().__init__()
        self.path = datadir
        self.stage = stage
        self.image_size = tuple(image_size)
        self.world_scale = world_scale
        # the category prefix is the basename of datadir (SRNDataset.py:29-33)
        self.list_prefix = os.path.basename(self.path) or os.path.basename(os.path.dirname(self.path))
        self.dataset_name = self.list_prefix
        self.base_path = os.path.join(self.path, self.list_prefix + "_" + self.stage)
        if not os.path.isdir(self.base_path):
            raise FileNotFoundError("SRN dataset base path not found: %s" % self.base_path)
        self.intrins = sorted(glob.glob(os.path.join(self.base_path, "*", "intrinsics.txt")))
        # OpenCV -> OpenGL camera axes (SRNDataset.py:54-56)
        self._coord_trans = torch.diag(torch.tensor([1, -1, -1, 1], dtype=torch.float32))
        # the fork evaluates with the test planes for every split (SRNDataset.py:57-63)
        self.z_near, self.z_far = 0.01, 4.0
        self.lindisp = False

    def __len__(self):
        return len(self.intrins)

    @staticmethod
    def _intrinsics(path):
        """(focal, cx, cy) from line 1 of intrinsics.txt ("f cx cy _"; the last line's "H W" is
        not used: the image itself fixes the size)."""
        with open(path, "r") as f:
            first = f.readline().split()
        return float(first[0]), float(first[1]), float(first[2])

    def _view(self, rgb_path, pose_path):
        """One view: the balanced image tensor, its foreground mask (every channel != 255), the
        OpenGL-axes camera-to-world pose and the mask's [cmin, rmin, cmax, rmax] box."""
        img = _imread_rgb(rgb_path)
        fg = np.all(img != 255, axis=-1)
        ys, xs = np.nonzero(fg.any(axis=1))[0], np.nonzero(fg.any(axis=0))[0]
        if ys.size == 0:
            raise RuntimeError("Bad image at %s (no foreground pixel)" % rgb_path)
        box = torch.tensor([xs[0], ys[0], xs[-1], ys[-1]], dtype=torch.float32)
        c2w = torch.from_numpy(np.loadtxt(pose_path, dtype=np.float32).reshape(4, 4)) @ self._coord_trans
        mask = fg[..., None].astype(np.uint8) * 255
        return image_to_tensor_balanced(img), mask_to_tensor(mask), c2w, box

    def __getitem__(self, index):
        intrin_path = self.intrins[index]
        obj_dir = os.path.dirname(intrin_path)
        rgb_paths = sorted(glob.glob(os.path.join(obj_dir, "rgb", "*")))
        pose_paths = sorted(glob.glob(os.path.join(obj_dir, "pose", "*")))
        assert len(rgb_paths) == len(pose_paths)
        focal, cx, cy = self._intrinsics(intrin_path)
        images, masks, poses, boxes = (torch.stack(t) for t in
                                       zip(*[self._view(r, q) for r, q in zip(rgb_paths, pose_paths)]))
        if tuple(images.shape[-2:]) != self.image_size:
            # area-resampled to image_size; intrinsics and boxes follow the row scale
            k = self.image_size[0] / images.shape[-2]
            focal, cx, cy, boxes = focal * k, cx * k, cy * k, boxes * k
            images = F.interpolate(images, size=self.image_size, mode="area")
            masks = F.interpolate(masks, size=self.image_size, mode="area")
        if self.world_scale != 1.0:
            focal = focal * self.world_scale
            poses[:, :3, 3] *= self.world_scale
        return dict(path=obj_dir, img_id=index, focal=torch.tensor(focal, dtype=torch.float32),
                    c=torch.tensor([cx, cy], dtype=torch.float32), images=images, masks=masks,
                    bbox=boxes, poses=poses)


def decompose_projection(P):
    """cv2.decomposeProjectionMatrix(P)[:3] for a 3 x 4 projection P = s K [R | -R C] (s > 0):
    (K, R, t) with K upper triangular with a positive diagonal (not normalised), R the rotation and
    t = (C, 1) the homogeneous camera centre (4 x 1).  The RQ factorisation of P[:, :3] by a QR of
    its row- and column-reversed transpose; the diagonal signs moved into R.  cv2 is absent offline,
    so this restates the decomposition, not cv2's code (DVRDataset.py:169)."""
    P = np.asarray(P, dtype=np.float64)
    M = P[:, :3]
    flip = np.eye(3)[::-1]
    q, r = np.linalg.qr((flip @ M).T)
    K = flip @ r.T @ flip
    R = flip @ q.T
    d = np.diag(np.sign(np.diag(K)))
    K, R = K @ d, d @ R
    C = -np.linalg.solve(M, P[:, 3])
    return K, R, np.concatenate([C, [1.0]])[:, None]


class DVRDataset(torch.utils.data.Dataset):
    """DVRDataset.py:11-274: ShapeNet-NMR / 3D-R2N2 renderings (``sub_format="shapenet"``) and DTU
    (``"dtu"``).  ``dataset[i]`` is one object with all its views (at most ``max_imgs``, drawn
    with numpy's global generator as the reference does)."""

    def __init__(self, path, stage="train", list_prefix="softras_", image_size=None, sub_format="shapenet",
                 scale_focal=True, max_imgs=100000, z_near=1.2, z_far=4.0, skip_step=None):
        super().__init__()
        self.base_path = path
        assert os.path.exists(self.base_path)
        cats = [x for x in glob.glob(os.path.join(path, "*")) if os.path.isdir(x)]
        lists = [os.path.join(x, list_prefix + stage + ".lst") for x in cats]
        self.all_objs = []
        for fl in lists:
            if not os.path.exists(fl):
                continue
            base = os.path.dirname(fl)
            with open(fl, "r") as f:
                self.all_objs.extend((os.path.basename(base), os.path.join(base, x.strip())) for x in f.readlines())
        self.stage = stage
        self.image_to_tensor = image_to_tensor_balanced
        self.mask_to_tensor = mask_to_tensor
        print("Loading DVR dataset", self.base_path, "stage", stage, len(self.all_objs), "objs", "type:", sub_format)
        self.image_size = image_size
        flip_yz = torch.tensor([[1, 0, 0, 0], [0, -1, 0, 0], [0, 0, -1, 0], [0, 0, 0, 1]], dtype=torch.float32)
        self._coord_trans_cam = flip_yz
        self._coord_trans_world = flip_yz if sub_format == "dtu" else torch.tensor(
            [[1, 0, 0, 0], [0, 0, -1, 0], [0, 1, 0, 0], [0, 0, 0, 1]], dtype=torch.float32)
        self.sub_format = sub_format
        self.scale_focal = scale_focal
        self.max_imgs = max_imgs
        self.z_near, self.z_far = z_near, z_far
        self.lindisp = False

    def __len__(self):
        return len(self.all_objs)

    def _dtu_pose(self, cams, i):
        """(pose, K) of view i: P = world_mat_i decomposed, then normalised by scale_mat_i."""
        K, R, t = decompose_projection(cams["world_mat_" + str(i)][:3])
        K = K / K[2, 2]
        pose = np.eye(4, dtype=np.float32)
        pose[:3, :3] = R.transpose()
        pose[:3, 3] = (t[:3] / t[3])[:, 0]
        key = "scale_mat_" + str(i)
        if key in cams:
            S = cams[key]
            pose[:3, 3:] -= S[:3, 3:]
            pose[:3, 3:] /= np.diagonal(S[:3, :3])[..., None]
        return pose, K

    def __getitem__(self, index):
        _, root = self.all_objs[index]
        rgb_paths = sorted(x for x in glob.glob(os.path.join(root, "image", "*"))
                           if x.endswith(".jpg") or x.endswith(".png"))
        mask_paths = sorted(glob.glob(os.path.join(root, "mask", "*.png"))) or [None] * len(rgb_paths)
        if len(rgb_paths) <= self.max_imgs:
            sel = np.arange(len(rgb_paths))
        else:
            sel = np.random.choice(len(rgb_paths), self.max_imgs, replace=False)
            rgb_paths = [rgb_paths[i] for i in sel]
            mask_paths = [mask_paths[i] for i in sel]
        cams = np.load(os.path.join(root, "cameras.npz"))
        shapenet = self.sub_format == "shapenet"
        imgs, poses, masks, boxes = [], [], [], []
        focal = None
        fx = fy = cx = cy = 0.0
        mask_path = None
        for k, (rgb_path, mask_path) in enumerate(zip(rgb_paths, mask_paths)):
            i = sel[k]
            img = _imread(rgb_path)[..., :3]
            if self.scale_focal:
                xs, ys, delta = img.shape[1] / 2.0, img.shape[0] / 2.0, 1.0
            else:
                xs = ys = 1.0
                delta = 0.0
            if mask_path is not None:
                mask = _imread(mask_path)
                mask = (mask[..., None] if mask.ndim == 2 else mask)[..., :1]
            if not shapenet:
                pose, K = self._dtu_pose(cams, i)
                fx += torch.tensor(K[0, 0]) * xs
                fy += torch.tensor(K[1, 1]) * ys
                cx += (torch.tensor(K[0, 2]) + delta) * xs
                cy += (torch.tensor(K[1, 2]) + delta) * ys
            else:
                if "world_mat_inv_" + str(i) in cams:
                    pose = cams["world_mat_inv_" + str(i)]
                else:
                    w = cams["world_mat_" + str(i)]
                    if w.shape[0] == 3:
                        w = np.vstack((w, np.array([0, 0, 0, 1])))
                    pose = np.linalg.inv(w)
                intr = cams["camera_mat_" + str(i)]
                f0 = intr[0, 0]
                assert abs(f0 - intr[1, 1]) < 1e-9
                f0 = f0 * xs
                if focal is None:
                    focal = f0
                else:
                    assert abs(f0 - focal) < 1e-5
            poses.append(self._coord_trans_world @ torch.tensor(pose, dtype=torch.float32) @ self._coord_trans_cam)
            imgs.append(self.image_to_tensor(img))
            if mask_path is not None:
                rnz = np.where(np.any(mask, axis=1))[0]
                cnz = np.where(np.any(mask, axis=0))[0]
                if len(rnz) == 0:
                    raise RuntimeError("ERROR: Bad image at", rgb_path, "please investigate!")
                masks.append(self.mask_to_tensor(mask))
                boxes.append(torch.tensor([cnz[0], rnz[0], cnz[-1], rnz[-1]], dtype=torch.float32))
        c = None
        if not shapenet:
            n = len(rgb_paths)
            focal = torch.tensor((fx / n, fy / n), dtype=torch.float32)
            c = torch.tensor((cx / n, cy / n), dtype=torch.float32)
            boxes = None
        elif mask_path is not None:
            boxes = torch.stack(boxes)
        imgs = torch.stack(imgs)
        poses = torch.stack(poses)
        masks = torch.stack(masks) if masks else None
        if self.image_size is not None and tuple(imgs.shape[-2:]) != tuple(self.image_size):
            scale = self.image_size[0] / imgs.shape[-2]
            focal *= scale
            if not shapenet:
                c *= scale
            elif mask_path is not None:
                boxes *= scale
            imgs = F.interpolate(imgs, size=self.image_size, mode="area")
            if masks is not None:
                masks = F.interpolate(masks, size=self.image_size, mode="area")
        out = {"path": root, "img_id": index, "focal": focal, "images": imgs, "poses": poses}
        if masks is not None:
            out["masks"] = masks
        if not shapenet:
            out["c"] = c
        else:
            out["bbox"] = boxes
        return out


class MultiObjectDataset(torch.utils.data.Dataset):
    """MultiObjectDataset.py:14-117: NeRF-synthetic style scenes of several ShapeNet objects,
    <path>/<stage>/**/transforms.json with RGBA ``<frame>_obj.png`` images composited on white."""

    def __init__(self, path, stage="train", z_near=4, z_far=9, n_views=None):
        super().__init__()
        self.base_path = os.path.join(path, stage)
        print("Loading NeRF synthetic dataset", self.base_path)
        self.trans_files = [os.path.join(root, "transforms.json") for root, _, files in os.walk(self.base_path)
                            if "transforms.json" in files]
        self.image_to_tensor = image_to_tensor_balanced
        self.mask_to_tensor = mask_to_tensor
        self.z_near, self.z_far = z_near, z_far
        self.lindisp = False
        self.n_views = n_views
        print("{} instances in split {}".format(len(self.trans_files), stage))

    def __len__(self):
        return len(self.trans_files)

    def _check_valid(self, index):
        if self.n_views is None:
            return True
        import json

        path = self.trans_files[index]
        try:
            with open(path, "r") as f:
                tr = json.load(f)
        except Exception as e:   # noqa: BLE001 -- the reference reports and skips the scene
            print("Problematic transforms.json file", path)
            print("JSON loading exception", e)
            return False
        return (len(tr["frames"]) == self.n_views
                and len(glob.glob(os.path.join(os.path.dirname(path), "*.png"))) == self.n_views)

    def __getitem__(self, index):
        import json

        if not self._check_valid(index):
            return {}
        path = self.trans_files[index]
        d = os.path.dirname(path)
        with open(path, "r") as f:
            tr = json.load(f)
        imgs, boxes, masks, poses = [], [], [], []
        for fr in tr["frames"]:
            base = os.path.splitext(os.path.basename(fr["file_path"]))[0]
            img = _imread(os.path.join(d, "{}_obj.png".format(base)))
            mask = self.mask_to_tensor(img[..., 3])
            rnz = np.where(np.any(img, axis=1))[0]
            cnz = np.where(np.any(img, axis=0))[0]
            if len(rnz) == 0:
                cmin = rmin = 0
                cmax, rmax = mask.shape[-1], mask.shape[-2]
            else:
                rmin, rmax = rnz[[0, -1]]
                cmin, cmax = cnz[[0, -1]]
            boxes.append(torch.tensor([cmin, rmin, cmax, rmax], dtype=torch.float32))
            imgs.append(self.image_to_tensor(img[..., :3]) * mask + (1.0 - mask))   # white where transparent
            masks.append(mask)
            poses.append(torch.tensor(fr["transform_matrix"]))
        imgs = torch.stack(imgs)
        W = imgs.shape[-1]
        focal = 0.5 * W / np.tan(0.5 * tr.get("camera_angle_x"))
        return {"path": d, "img_id": index, "focal": focal, "images": imgs, "masks": torch.stack(masks),
                "bbox": torch.stack(boxes), "poses": torch.stack(poses)}


def _gray(img):
    r, g, b = img.unbind(-3)
    return (0.2989 * r + 0.587 * g + 0.114 * b).unsqueeze(-3)


def _blend(a, b, ratio):
    return (ratio * a + (1.0 - ratio) * b).clamp(0.0, 1.0)


def _rgb_to_hsv(img):
    r, g, b = img.unbind(-3)
    mx, mn = img.max(-3).values, img.min(-3).values
    flat = mx == mn
    rng = mx - mn
    one = torch.ones_like(mx)
    s = rng / torch.where(flat, one, mx)
    div = torch.where(flat, one, rng)
    rc, gc, bc = (mx - r) / div, (mx - g) / div, (mx - b) / div
    h = ((mx == r) * (bc - gc) + ((mx == g) & (mx != r)) * (2.0 + rc - bc)
         + ((mx != g) & (mx != r)) * (4.0 + gc - rc))
    return torch.stack((torch.fmod(h / 6.0 + 1.0, 1.0), s, mx), -3)


def _hsv_to_rgb(img):
    h, s, v = img.unbind(-3)
    i = torch.floor(h * 6.0)
    f = h * 6.0 - i
    i = i.to(torch.int64) % 6
    p = (v * (1.0 - s)).clamp(0.0, 1.0)
    q = (v * (1.0 - s * f)).clamp(0.0, 1.0)
    t = (v * (1.0 - s * (1.0 - f))).clamp(0.0, 1.0)
    table = [(v, t, p), (q, v, p), (p, v, t), (p, q, v), (t, p, v), (v, p, q)]
    out = torch.zeros_like(img)
    for k, (a, b, c) in enumerate(table):
        sel = (i == k).unsqueeze(-3)
        out = torch.where(sel, torch.stack((a, b, c), -3), out)
    return out


class ColorJitterDataset(torch.utils.data.Dataset):
    """data_util.py:14-56: the same random saturation, hue, contrast and brightness change over all
    views of an object (factors drawn with numpy's global generator in the reference's order),
    applied to images in [-1, 1].  The reference calls ``torchvision.transforms.adjust_*``
    (data_util.py:41-44), names torchvision's transforms namespace does not define; this applies
    the adjustments of torchvision.transforms.functional on tensors that the call evidently meant
    (grey = 0.2989 r + 0.587 g + 0.114 b; blends clamped to [0, 1]; hue by an HSV round trip).
    torchvision is absent offline: parity unpinned."""

    def __init__(self, base_dset, hue_range=0.1, saturation_range=0.1, brightness_range=0.1,
                 contrast_range=0.1, extra_inherit_attrs=()):
        self.hue_range = [-hue_range, hue_range]
        self.saturation_range = [1 - saturation_range, 1 + saturation_range]
        self.brightness_range = [1 - brightness_range, 1 + brightness_range]
        self.contrast_range = [1 - contrast_range, 1 + contrast_range]
        self.base_dset = base_dset
        for name in ["z_near", "z_far", "lindisp", "base_path", "image_to_tensor", *extra_inherit_attrs]:
            setattr(self, name, getattr(base_dset, name))

    def apply_color_jitter(self, images):
        hue = np.random.uniform(*self.hue_range)
        sat = np.random.uniform(*self.saturation_range)
        bri = np.random.uniform(*self.brightness_range)
        con = np.random.uniform(*self.contrast_range)
        for i in range(len(images)):
            x = (images[i] + 1.0) * 0.5
            x = _blend(x, _gray(x), sat)
            hsv = _rgb_to_hsv(x)
            x = _hsv_to_rgb(torch.stack((torch.remainder(hsv[0] + hue, 1.0), hsv[1], hsv[2]), 0))
            x = _blend(x, _gray(x).mean(dim=(-3, -2, -1), keepdim=True), con)
            x = _blend(x, torch.zeros_like(x), bri)
            images[i] = x * 2.0 - 1.0
        return images

    def __len__(self):
        return len(self.base_dset)

    def __getitem__(self, idx):
        data = self.base_dset[idx]
        data["images"] = self.apply_color_jitter(data["images"])
        return data


def get_split_dataset(dataset_type, datadir, want_split="all", training=True, **kwargs):
    """data/__init__.py:10-72: ``srn`` / ``pollen`` (SRNDataset), ``multi_obj``
    (MultiObjectDataset), ``dvr`` / ``dvr_gen`` / ``dvr_dtu`` (DVRDataset; DTU with at most 49
    training views, unscaled focal, near / far 0.1 / 5.0 and the colour jitter on the training
    split).  Returns (train, val, test), or the one split asked for by want_split."""
    flags, aug, aug_flags = {}, None, {}
    if dataset_type in ("srn", "pollen"):
        cls = SRNDataset
    elif dataset_type == "multi_obj":
        cls = MultiObjectDataset
    elif dataset_type.startswith("dvr"):
        cls = DVRDataset
        if dataset_type == "dvr_gen":
            flags["list_prefix"] = "gen_"
        elif dataset_type == "dvr_dtu":
            flags.update(list_prefix="new_", sub_format="dtu", scale_focal=False, z_near=0.1, z_far=5.0)
            if training:
                flags["max_imgs"] = 49
            aug, aug_flags = ColorJitterDataset, {"extra_inherit_attrs": ["sub_format"]}
    else:
        raise NotImplementedError("Unsupported dataset type", dataset_type)
    want_train = want_split not in ("val", "test")
    want_val = want_split not in ("train", "test")
    want_test = want_split not in ("train", "val")
    train_set = cls(datadir, stage="train", **flags, **kwargs) if want_train else None
    if train_set is not None and aug is not None:
        train_set = aug(train_set, **aug_flags)
    val_set = cls(datadir, stage="val", **flags, **kwargs) if want_val else None
    test_set = cls(datadir, stage="test", **flags, **kwargs) if want_test else None
    if want_split == "train":
        return train_set
    if want_split == "val":
        return val_set
    if want_split == "test":
        return test_set
    return train_set, val_set, test_set
