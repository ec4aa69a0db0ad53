"""Compat shim: ``from model import make_model`` / ``from model import loss`` (reference
src/model/__init__.py, src/model/loss.py)."""
from pnr.models import PixelNeRFNet, make_model  # noqa: F401

from . import loss  # noqa: F401,E402
