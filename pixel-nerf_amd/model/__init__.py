"""Compat shim: ``from model import make_model`` (reference src/model/__init__.py)."""
from pnr.models import PixelNeRFNet, make_model  # noqa: F401
