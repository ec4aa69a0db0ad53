"""RGB losses of the training caller (reference src/model/loss.py; train.py:106-116, 271-276).

``get_rgb_loss(conf, coarse)`` is what train.py calls: an MSE (or L1 with ``use_l1``) with mean
reduction, or -- for the fine pass with ``use_uncertainty`` -- the Kendall '17 uncertainty loss
(loss.py:91-103).  The alpha loss and the background-weighted loss are the file's other two
objects (loss.py:4-88); the shipped confs turn neither on.  The render path's gradient into the
loss is torch autograd here as in the reference.
"""
import torch

from .conf import as_conf

__all__ = ["AlphaLossNV2", "RGBWithUncertainty", "RGBWithBackground", "get_alpha_loss", "get_rgb_loss"]


def _element_loss(conf):
    conf = as_conf(conf)
    return torch.nn.L1Loss(reduction="none") if conf.get_bool("use_l1") else torch.nn.MSELoss(reduction="none")


class AlphaLossNV2(torch.nn.Module):
    """Neural Volumes' alpha prior (loss.py:4-37): from ``init_epoch`` on, the mean of
    log(a) + log(1 - a) over alpha clamped to [0.01, 0.99], clamped below at -clamp_alpha and scaled
    by lambda_alpha -- or a BCE towards 1 with ``force_opaque``.  ``epoch`` is a persistent buffer
    advanced by ``sched_step``."""

    def __init__(self, lambda_alpha, clamp_alpha, init_epoch, force_opaque=False):
        super().__init__()
        self.lambda_alpha = lambda_alpha
        self.clamp_alpha = clamp_alpha
        self.init_epoch = init_epoch
        self.force_opaque = force_opaque
        if force_opaque:
            self.bceloss = torch.nn.BCELoss()
        self.register_buffer("epoch", torch.tensor(0, dtype=torch.long), persistent=True)

    def sched_step(self, num=1):
        self.epoch += num

    def forward(self, alpha_fine):
        if not (self.lambda_alpha > 0.0 and int(self.epoch) >= self.init_epoch):
            return torch.zeros(1, device=alpha_fine.device)
        a = torch.clamp(alpha_fine, 0.01, 0.99)
        if self.force_opaque:
            return self.lambda_alpha * self.bceloss(a, torch.ones_like(a))
        prior = torch.clamp_min(torch.log(a) + torch.log(1.0 - a), -self.clamp_alpha)
        return self.lambda_alpha * prior.mean()


def get_alpha_loss(conf):
    """loss.py:40-48."""
    conf = as_conf(conf)
    return AlphaLossNV2(conf.get_float("lambda_alpha"), conf.get_float("clamp_alpha"),
                        conf.get_int("init_epoch"), force_opaque=conf.get_bool("force_opaque", False))


class RGBWithUncertainty(torch.nn.Module):
    """mean(mean_c(err(out, target)) / beta) + mean(log beta) (loss.py:51-67)."""

    def __init__(self, conf):
        super().__init__()
        self.element_loss = _element_loss(conf)

    def forward(self, outputs, targets, betas):
        err = torch.mean(self.element_loss(outputs, targets), -1) / betas
        return torch.mean(err) + torch.mean(torch.log(betas))


class RGBWithBackground(torch.nn.Module):
    """mean(mean_c(err) / (1 + lambda_bg)) + mean(log lambda_bg) (loss.py:70-86)."""

    def __init__(self, conf):
        super().__init__()
        self.element_loss = _element_loss(conf)

    def forward(self, outputs, targets, lambda_bg):
        err = torch.mean(self.element_loss(outputs, targets), -1) / (1 + lambda_bg)
        return torch.mean(err) + torch.mean(torch.log(lambda_bg))


def get_rgb_loss(conf, coarse=True, using_bg=False, reduction="mean"):
    """loss.py:91-103: the uncertainty loss for the fine pass when ``use_uncertainty``, else
    L1 (``use_l1``) or MSE with ``reduction``.  ``using_bg`` is accepted and unused, as there."""
    conf = as_conf(conf)
    if conf.get_bool("use_uncertainty", False) and not coarse:
        print("using loss with uncertainty")
        return RGBWithUncertainty(conf)
    print("using vanilla rgb loss")
    return torch.nn.L1Loss(reduction=reduction) if conf.get_bool("use_l1") else torch.nn.MSELoss(reduction=reduction)
