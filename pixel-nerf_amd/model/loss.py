"""Compat shim: ``from model import loss`` (reference src/model/loss.py)."""
from pnr.loss import *  # noqa: F401,F403
from pnr.loss import AlphaLossNV2, RGBWithBackground, RGBWithUncertainty, get_alpha_loss, get_rgb_loss  # noqa: F401
