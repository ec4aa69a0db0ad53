#!/usr/bin/env python
"""Train pixelNeRF on an SRN-layout dataset with the HIP ray march: the counterpart of the
reference's train/train.py (+ trainlib), SURVEY §8(b) "build-side counterparts".

  python scripts/train.py -c conf/exp/srn.conf -D <datadir>/cars -n srn_car -B 4 -V 1
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 scripts/train.py ...

The same flags and defaults as the reference (train.py's extra_args through util.args.parse_args,
util/args.py:9-112, -R 256 as train.py:72), the same
checkpoint files (<checkpoints_path>/<name>/pixel_nerf_latest, _optim, _lrsched, _iter,
_renderer) and the same loss (lambda_coarse MSE(coarse) + lambda_fine MSE(fine), conf loss.*).
One process per GPU under torch.distributed (pnr.trainer.Trainer), where the reference runs
nn.DataParallel over --gpu_id; a single process uses --gpu_id's first device."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pixel-nerf_amd"))

import torch  # noqa: E402

from pnr import dist as pdist  # noqa: E402
from util import args as uargs  # noqa: E402
from pnr.data import get_split_dataset  # noqa: E402
from pnr.models import make_model  # noqa: E402
from pnr.renderer import NeRFRenderer  # noqa: E402
from pnr.trainer import Trainer, seed_everything  # noqa: E402


def extra_args(ap):
    """train/train.py's extra_args (train.py:35-69), same names and defaults, plus this caller's
    own --max_steps / --image_size / --seed."""
    ap.add_argument("--batch_size", "-B", type=int, default=4, help="Object batch size ('SB'), per rank")
    ap.add_argument("--nviews", "-V", type=str, default="2",
                    help="Number of source views (multiview); several (space delimited) to pick one per batch")
    ap.add_argument("--gamma_delay", type=int, default=0,
                    help="Number of scheduler.step() calls to wait before applying gamma decay")
    ap.add_argument("--freeze_enc", action="store_true", default=None, help="Freeze encoder weights, train the MLP")
    ap.add_argument("--no_bbox_step", type=int, default=100000, help="Step to stop using bbox sampling")
    ap.add_argument("--fixed_test", action="store_true", default=None, help="accepted; unused (as in train.py)")
    ap.add_argument("--max_steps", type=int, default=None, help="stop after this many steps (then save)")
    ap.add_argument("--image_size", type=int, default=None,
                    help="resample every image to this square size (default: the loader's own -- SRN 128, "
                         "DVR NMR / DTU and multi-object their native size, as train.py passes none)")
    ap.add_argument("--seed", type=int, default=0)
    return ap


def load_datasets(fmt, datadir, image_size=None):
    """train.py:74's get_split_dataset(args.dataset_format, args.datadir): the loaders' own image
    size unless --image_size is given (train.py passes none, so ShapeNet-NMR stays 64 x 64 and DTU
    300 x 400 with their own intrinsics; MultiObjectDataset takes no size at all)."""
    kw = {} if image_size is None else {"image_size": (image_size, image_size)}
    return get_split_dataset(fmt, datadir, **kw)


def main(argv=None):
    # the reference's flags and defaults exactly: util/args.py's common flags (-c -n -D -F -G -r
    # --gpu_id --lr --gamma --epochs --logs_path --checkpoints_path --visual_path, -R default 256 as
    # train.py:72 passes it) plus train.py's extra_args
    args, conf = uargs.parse_args(extra_args, training=True, default_ray_batch_size=256, argv=argv)
    args.nviews = list(map(int, args.nviews.split()))

    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        rank, world, local = pdist.init_from_env("nccl")   # RCCL on ROCm
        device = torch.device("cuda", local)
    else:
        rank, world = 0, 1
        device = torch.device("cuda", args.gpu_id[0])
    torch.cuda.set_device(device)
    seed_everything(args.seed + rank)

    dset, val_dset, _ = load_datasets(args.dataset_format, args.datadir, args.image_size)
    net = make_model(conf["model"]).to(device=device)
    net.stop_encoder_grad = args.freeze_enc
    if args.freeze_enc:
        net.encoder.eval()
    renderer = NeRFRenderer.from_conf(conf["renderer"], lindisp=dset.lindisp).to(device=device)
    tconf = dict(conf.get("train", {}) or {})
    lconf = conf.get("loss", {}) or {}
    rgb = lconf.get("rgb", {}) or {}
    if rgb.get("use_uncertainty", False):
        raise NotImplementedError("pnr trainer: the rgb loss is MSE (loss.rgb.use_uncertainty = False)")
    tconf["lambda_coarse"] = float(lconf.get("lambda_coarse", 1.0))
    tconf["lambda_fine"] = float(lconf.get("lambda_fine", 1.0))
    trainer = Trainer(net, renderer, dset, val_dset, args, tconf, device)
    last = trainer.start(max_steps=args.max_steps)
    if rank == 0:
        print("final losses", " ".join("%s:%.6f" % kv for kv in last.items()), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
