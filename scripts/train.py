#!/usr/bin/env python
"""Train pixelNeRF on an SRN-layout dataset with the HIP ray march: the counterpart of the
reference's train/train.py (+ trainlib), SURVEY §8(b) "build-side counterparts".

  python scripts/train.py -c conf/exp/srn.conf -D <datadir>/cars -n srn_car -B 4 -V 1
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 scripts/train.py ...

The same flags as the reference (train.py extra_args + util/args.py's training flags), the same
checkpoint files (<checkpoints_path>/<name>/pixel_nerf_latest, _optim, _lrsched, _iter,
_renderer) and the same loss (lambda_coarse MSE(coarse) + lambda_fine MSE(fine), conf loss.*).
One process per GPU under torch.distributed (pnr.trainer.Trainer), where the reference runs
nn.DataParallel over --gpu_id; a single process uses --gpu_id's first device."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pixel-nerf_amd"))

import torch  # noqa: E402

from pnr import dist as pdist  # noqa: E402
from pnr.conf import parse_file  # noqa: E402
from pnr.data import get_split_dataset  # noqa: E402
from pnr.models import make_model  # noqa: E402
from pnr.renderer import NeRFRenderer  # noqa: E402
from pnr.trainer import Trainer, seed_everything  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--conf", "-c", required=True)
    ap.add_argument("--datadir", "-D", required=True)
    ap.add_argument("--dataset_format", "-F", default="srn")
    ap.add_argument("--name", "-n", default="srn_car")
    ap.add_argument("--checkpoints_path", default="checkpoints")
    ap.add_argument("--resume", action="store_true")
    ap.add_argument("--batch_size", "-B", type=int, default=4, help="objects per step (per rank)")
    ap.add_argument("--nviews", "-V", default="1", help="source views; several (space separated): one per batch")
    ap.add_argument("--ray_batch_size", "-R", type=int, default=128, help="rays per object")
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--gamma", type=float, default=1.0)
    ap.add_argument("--gamma_delay", type=int, default=0)
    ap.add_argument("--epochs", type=int, default=10000000)
    ap.add_argument("--max_steps", type=int, default=None, help="stop after this many steps (then save)")
    ap.add_argument("--no_bbox_step", type=int, default=100000)
    ap.add_argument("--freeze_enc", action="store_true")
    ap.add_argument("--image_size", type=int, default=128)
    ap.add_argument("--gpu_id", default="0")
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args(argv)
    args.nviews = list(map(int, args.nviews.split()))

    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        rank, world, local = pdist.init_from_env("nccl")   # RCCL on ROCm
        device = torch.device("cuda", local)
    else:
        rank, world = 0, 1
        device = torch.device("cuda", int(args.gpu_id.split()[0]))
    torch.cuda.set_device(device)
    seed_everything(args.seed + rank)

    conf = parse_file(args.conf)
    dset, val_dset, _ = get_split_dataset(args.dataset_format, args.datadir,
                                          image_size=(args.image_size, args.image_size))
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
