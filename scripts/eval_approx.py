#!/usr/bin/env python
"""eval/eval_approx.py counterpart on the MI355X ray march: approximate PSNR / SSIM over an
SRN-layout dataset, one random target view per object (pnr.evaluate.eval_approx).

  python scripts/eval_approx.py -c conf/exp/srn.conf -D <datadir>/cars -n srn_car \
      --checkpoints_path checkpoints [--split test] [-P "64"] [--coarse] [--seed 1234]

The conf is read with pnr.conf.parse_file (HOCON subset; pyhocon is absent offline) and the
checkpoint with PixelNeRFNet.load_weights (torch.load, weights_only=True).
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pixel-nerf_amd"))

import torch  # noqa: E402

from pnr import evaluate  # noqa: E402
from pnr.conf import parse_file  # noqa: E402
from pnr.data import get_split_dataset  # noqa: E402
from pnr.models import make_model  # noqa: E402
from pnr.renderer import NeRFRenderer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--conf", "-c", required=True)
    ap.add_argument("--datadir", "-D", required=True)
    ap.add_argument("--dataset_format", "-F", default="srn")
    ap.add_argument("--name", "-n", default="srn_car")
    ap.add_argument("--checkpoints_path", default="checkpoints")
    ap.add_argument("--split", default="val")
    ap.add_argument("--source", "-P", default="64")
    ap.add_argument("--batch_size", type=int, default=4)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--coarse", action="store_true")
    ap.add_argument("--ray_batch_size", "-R", type=int, default=50000)
    ap.add_argument("--gpu_id", type=int, default=0)
    args = ap.parse_args()
    args.resume = True

    conf = parse_file(args.conf)
    dev = torch.device("cuda", args.gpu_id)
    net = make_model(conf["model"]).to(device=dev)
    net.load_weights(args)
    dset = get_split_dataset(args.dataset_format, args.datadir, want_split=args.split, training=False)
    renderer = NeRFRenderer.from_conf(conf["renderer"], eval_batch_size=args.ray_batch_size).to(device=dev)
    res = evaluate.eval_approx(net, renderer, dset, dev, source=[int(s) for s in args.source.split()],
                               batch_size=args.batch_size, seed=args.seed, coarse=args.coarse,
                               ray_batch_size=args.ray_batch_size, log=print)
    print("final psnr", res["mean_psnr"], "ssim", res["mean_ssim"])


if __name__ == "__main__":
    main()
