"""The training caller (SURVEY §8(b) "build-side counterparts": train/train.py + trainlib).

The reference trains with ``train/train.py``'s ``PixelNeRFTrainer.calc_losses``
(train.py:193-283) inside ``trainlib.Trainer.start`` (trainlib/trainer.py): per step, every
object's rays for all of its views, a random pixel subset (inside the object boxes while
``bbox`` sampling is on), source views picked at random, ``encode``, ``render_par(rays,
want_weights=True)``, lambda_c MSE(coarse) + lambda_f MSE(fine), backward, Adam; checkpoints
``pixel_nerf_latest`` / ``_optim`` / ``_lrsched`` / ``_iter`` / ``_renderer`` under
``<checkpoints_path>/<name>/``.  This module restates that loop on this package's renderer,
model and SRN loader:

* ``calc_losses`` -- train.py:193-283's semantics: host RNG for the pixel / view picks (torch's
  default generator, the same calls in the same order), rays from ``util.gen_rays`` on the
  device, gathered per object;
* ``Trainer`` -- trainlib's schedule (save / print / eval intervals, gradient accumulation,
  gamma decay with delay, resume) with one process per GPU: ``torch.distributed`` ranks take
  disjoint object batches (DistributedSampler), the gradient mean is ``pnr.dist.GradReducer``
  (bucketed RCCL all-reduce from the backward's grad hooks) and the encoder's BatchNorm spans
  the ranks (``pnr.dist.set_batchnorm_mode(..., "sync")``), where the reference runs
  nn.DataParallel over ``--gpu_id``.

The model / renderer calls are the reference's public API, so the same loop drives the
reference's own modules (train.py imports them the same way)."""
import os
import random

import numpy as np
import torch
import torch.distributed as dist

from . import dist as pdist
from . import util

__all__ = ["calc_losses", "Trainer"]


def _mse(a, b):
    return torch.nn.functional.mse_loss(a, b)


def calc_losses(net, render_par, data, *, device, z_near, z_far, nviews=(1,), ray_batch_size=128,
                use_bbox=False, lambda_coarse=1.0, lambda_fine=1.0, is_train=True, nviews_gen=None):
    """One batch's losses (train.py:193-283).  ``data`` is a collated SRN batch: images
    (SB, NV, 3, H, W) in [-1, 1], poses (SB, NV, 4, 4), focal (SB) or (SB, 2), optional c
    (SB, 2) and bbox (SB, NV, 4).  Returns {"rc", "rf" (if fine), "t"} as floats; with
    ``is_train`` the loss is back-propagated first.  ``nviews_gen``: the torch.Generator the
    batch's view count is drawn from (None: torch's default generator, as train.py:214 does); the
    Trainer passes one seeded identically on every rank, so all ranks encode the same NS in a step,
    as the reference's single process does for the whole SB batch."""
    if "images" not in data:
        return {}
    images = data["images"].to(device=device)
    SB, NV, _, H, W = images.shape
    poses = data["poses"].to(device=device)
    focals = data["focal"]
    bboxes = data.get("bbox") if (is_train and use_bbox) else None
    cs = data.get("c")

    # views per object this batch: one of ``nviews`` (train.py:214-218)
    cur = nviews[torch.randint(0, len(nviews), (), generator=nviews_gen).item()]
    order = torch.randint(0, NV, (SB, 1)) if cur == 1 else torch.empty((SB, cur), dtype=torch.long)
    rgb_gt, rays = [], []
    for o in range(SB):
        if cur > 1:
            order[o] = torch.from_numpy(np.random.choice(NV, cur, replace=False))
        c = cs[o] if cs is not None else None
        cam_rays = util.gen_rays(poses[o], W, H, focals[o], z_near, z_far, c=c)   # (NV, H, W, 8)
        gt_all = (images[o] * 0.5 + 0.5).permute(0, 2, 3, 1).reshape(-1, 3)
        if bboxes is not None:
            pix = util.bbox_sample(bboxes[o], ray_batch_size)
            inds = pix[..., 0] * H * W + pix[..., 1] * W + pix[..., 2]
        else:
            inds = torch.randint(0, NV * H * W, (ray_batch_size,))
        inds = inds.to(device)
        rgb_gt.append(gt_all[inds])
        rays.append(cam_rays.reshape(-1, cam_rays.shape[-1])[inds])
    rgb_gt = torch.stack(rgb_gt)   # (SB, B', 3)
    rays = torch.stack(rays)       # (SB, B', 8)

    order = order.to(device)
    src_images = util.batched_index_select_nd(images, order)   # (SB, NS, 3, H, W)
    src_poses = util.batched_index_select_nd(poses, order)     # (SB, NS, 4, 4)
    net.encode(src_images, src_poses, focals.to(device=device),
               c=cs.to(device=device) if cs is not None else None)
    out = render_par(rays, want_weights=True)
    coarse, fine = out["coarse"], out.get("fine")
    using_fine = fine is not None and len(fine) > 0
    losses = {}
    loss = _mse(coarse["rgb"], rgb_gt)
    losses["rc"] = loss.item() * lambda_coarse
    if using_fine:
        lf = _mse(fine["rgb"], rgb_gt)
        loss = loss * lambda_coarse + lf * lambda_fine
        losses["rf"] = lf.item() * lambda_fine
    if is_train:
        loss.backward()
    losses["t"] = loss.item()
    return losses


class Trainer:
    """trainlib.Trainer's loop (trainlib/trainer.py) for ``calc_losses``, one process per GPU.

    ``net`` a PixelNeRFNet (load_weights / save_weights), ``renderer`` its NeRFRenderer,
    ``dset`` / ``val_dset`` SRN-layout datasets (pnr.data), ``args`` a namespace with
    checkpoints_path, name, resume, batch_size, lr, gamma, gamma_delay, epochs, ray_batch_size,
    nviews (list of ints), no_bbox_step; ``conf`` a dict with save_interval, print_interval,
    eval_interval, accu_grad (and loss lambdas lambda_coarse / lambda_fine).  Under
    torch.distributed each rank takes its own objects (batch_size per rank) and the gradient
    mean runs over the ranks."""

    def __init__(self, net, renderer, dset, val_dset, args, conf, device, log=print):
        self.net, self.renderer, self.args, self.conf, self.device = net, renderer, args, conf, device
        self.log = log
        self.world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        self.rank = dist.get_rank() if self.world > 1 else 0
        self.sampler = (torch.utils.data.distributed.DistributedSampler(dset, shuffle=True)
                        if self.world > 1 else None)
        self.loader = torch.utils.data.DataLoader(dset, batch_size=args.batch_size, shuffle=self.sampler is None,
                                                  sampler=self.sampler, num_workers=0)
        self.val_loader = (torch.utils.data.DataLoader(val_dset, batch_size=min(args.batch_size, 16), shuffle=True,
                                                       num_workers=0) if val_dset is not None else None)
        if self.world > 1:
            pdist.set_batchnorm_mode(net.encoder, "sync")
        self.render_par = renderer.bind_parallel(net)
        self.optim = torch.optim.Adam(net.parameters(), lr=args.lr)
        gamma, delay = getattr(args, "gamma", 1.0), getattr(args, "gamma_delay", 0)
        self.lr_scheduler = (torch.optim.lr_scheduler.LambdaLR(
            self.optim, lr_lambda=lambda e: 1.0 if e < delay else gamma ** (e - delay)) if gamma != 1.0 else None)
        self.reducer = pdist.GradReducer(list(net.parameters()), self.world)
        self.ckpt_dir = os.path.join(args.checkpoints_path, args.name)
        os.makedirs(self.ckpt_dir, exist_ok=True)
        self.paths = {k: os.path.join(self.ckpt_dir, k) for k in ("_iter", "_optim", "_lrsched", "_renderer")}
        net.load_weights(args, device=device)
        self.start_iter = 0
        if args.resume:
            if os.path.exists(self.paths["_optim"]):
                self.optim.load_state_dict(torch.load(self.paths["_optim"], map_location=device, weights_only=True))
            if self.lr_scheduler is not None and os.path.exists(self.paths["_lrsched"]):
                self.lr_scheduler.load_state_dict(torch.load(self.paths["_lrsched"], map_location=device,
                                                             weights_only=True))
            if os.path.exists(self.paths["_iter"]):
                self.start_iter = torch.load(self.paths["_iter"], map_location="cpu", weights_only=True)["iter"]
            if os.path.exists(self.paths["_renderer"]):
                renderer.load_state_dict(torch.load(self.paths["_renderer"], map_location=device, weights_only=True))
        self.use_bbox = args.no_bbox_step > 0

    def losses(self, data, is_train, step):
        if self.use_bbox and step >= self.args.no_bbox_step:
            self.use_bbox = False
            self.log(">>> Stopped using bbox sampling @ iter %d" % step)
        c = self.conf
        gen = None
        if self.world > 1:   # the same view count on every rank
            gen = torch.Generator().manual_seed(getattr(self.args, "seed", 0) * 1000003 + 2 * step + int(not is_train))
        return calc_losses(self.net, self.render_par, data, device=self.device, z_near=self.z_near, z_far=self.z_far,
                           nviews=self.args.nviews, ray_batch_size=self.args.ray_batch_size,
                           use_bbox=self.use_bbox, lambda_coarse=c.get("lambda_coarse", 1.0),
                           lambda_fine=c.get("lambda_fine", 1.0), is_train=is_train, nviews_gen=gen)

    def save(self, step):
        if self.rank != 0:
            return
        self.net.save_weights(self.args)
        torch.save(self.optim.state_dict(), self.paths["_optim"])
        if self.lr_scheduler is not None:
            torch.save(self.lr_scheduler.state_dict(), self.paths["_lrsched"])
        torch.save({"iter": step + 1}, self.paths["_iter"])
        torch.save(self.renderer.state_dict(), self.paths["_renderer"])

    def start(self, max_steps=None):
        """Run the epochs (or ``max_steps`` steps); returns the last step's losses."""
        a, c = self.args, self.conf
        self.z_near, self.z_far = self.loader.dataset.z_near, self.loader.dataset.z_far
        step = self.start_iter
        batches = len(self.loader)
        accu = c.get("accu_grad", 1)
        val_iter = iter(self.val_loader) if self.val_loader is not None else None
        last = {}
        # train.py builds render_par with .eval() (train.py:93): step 0 runs with the net and the
        # renderer in eval mode (BatchNorm on running statistics, no sigma noise); trainlib's
        # batch-0 eval step then switches them to train (trainer.py:185-189)
        self.net.eval()
        self.renderer.eval()
        self.optim.zero_grad(set_to_none=True)
        for epoch in range(a.epochs):
            if self.sampler is not None:
                self.sampler.set_epoch(epoch)
            for batch, data in enumerate(self.loader):
                self.reducer.arm()
                last = self.losses(data, True, step)
                self.reducer.finish()
                if batch % c.get("print_interval", 10) == 0 and self.rank == 0:
                    self.log("E %d B %d %s lr %g" % (epoch, batch, " ".join("%s:%.6f" % kv for kv in last.items()),
                                                     self.optim.param_groups[0]["lr"]))
                if val_iter is not None and batch % c.get("eval_interval", 50) == 0:
                    try:
                        vdata = next(val_iter)
                    except StopIteration:
                        val_iter = iter(self.val_loader)
                        vdata = next(val_iter)
                    self.net.eval()
                    self.renderer.eval()
                    with torch.no_grad():
                        vl = self.losses(vdata, False, step)
                    self.renderer.train()
                    self.net.train()
                    if self.rank == 0:
                        self.log("*** Eval: E %d B %d %s" % (epoch, batch, " ".join("%s:%.6f" % kv for kv in vl.items())))
                elif val_iter is None and not self.net.training:
                    self.renderer.train()   # no eval split: train mode from the second step
                    self.net.train()
                if batch % c.get("save_interval", 50) == 0 and (epoch > 0 or batch > 0):
                    self.save(step)
                if batch == batches - 1 or batch % accu == accu - 1:
                    self.optim.step()
                    self.optim.zero_grad(set_to_none=True)
                self.renderer.sched_step(a.batch_size)
                step += 1
                if max_steps is not None and step - self.start_iter >= max_steps:
                    self.save(step - 1)
                    return last
            if self.lr_scheduler is not None:
                self.lr_scheduler.step()
        self.save(step - 1)
        return last


def seed_everything(seed):
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
