"""SRN-format dataset reader for the eval / training callers of the ray march.

Counterpart of the reference's ``data.SRNDataset`` (src/data/SRNDataset.py:10-145) and of
``data.get_split_dataset`` (src/data/__init__.py:9-68) for the ``srn`` / ``pollen`` formats:
the loader whose images, poses and intrinsics feed ``PixelNeRFNet.encode`` and
``util.gen_rays`` in eval/eval_approx.py and train/train.py.  Same directory layout, item
keys, value conventions and near / far planes:

  <datadir>/<name>_<stage>/<object>/intrinsics.txt   "f cx cy _" on line 1, "H W" on the last
                                   /rgb/*.png          RGB(A) uint8
                                   /pose/*.txt          4 x 4 camera-to-world (OpenCV axes)

PNG decoding uses PIL (the reference uses imageio, absent offline); the array handed to the
conversions is the same (H, W, 3) uint8 image.
"""
import glob
import os

import numpy as np
import torch
import torch.nn.functional as F

__all__ = ["SRNDataset", "get_split_dataset", "image_to_tensor_balanced", "mask_to_tensor"]


def _imread_rgb(path):
    from PIL import Image

    with Image.open(path) as im:
        a = np.array(im)   # a writable copy
    if a.ndim == 2:                      # greyscale: imageio returns (H, W)
        a = np.repeat(a[..., None], 3, axis=-1)
    return a[..., :3]


def image_to_tensor_balanced(img):
    """util.get_image_to_tensor_balanced() (util.py:68-75): ToTensor then Normalize(0.5, 0.5):
    (H, W, 3) uint8 -> (3, H, W) float32 in [-1, 1]."""
    t = torch.from_numpy(np.ascontiguousarray(img)).permute(2, 0, 1).float().div(255.0)
    return (t - 0.5) / 0.5


def mask_to_tensor(mask):
    """util.get_mask_to_tensor() (util.py:78-81): (H, W, 1) uint8 -> (1, H, W) float32 in [0, 1]."""
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


def get_split_dataset(dataset_type, datadir, want_split="all", training=True, **kwargs):
    """data/__init__.py:9-68 for the SRN-layout formats (``srn``, ``pollen``).  Returns
    (train, val, test), or the one split asked for by want_split = train / val / test."""
    if dataset_type not in ("srn", "pollen"):
        raise NotImplementedError("pnr.data implements the SRN layout (srn, pollen); got %r" % dataset_type)
    want_train = want_split not in ("val", "test")
    want_val = want_split not in ("train", "test")
    want_test = want_split not in ("train", "val")
    train_set = SRNDataset(datadir, stage="train", **kwargs) if want_train else None
    val_set = SRNDataset(datadir, stage="val", **kwargs) if want_val else None
    test_set = SRNDataset(datadir, stage="test", **kwargs) if want_test else None
    if want_split == "train":
        return train_set
    if want_split == "val":
        return val_set
    if want_split == "test":
        return test_set
    return train_set, val_set, test_set
