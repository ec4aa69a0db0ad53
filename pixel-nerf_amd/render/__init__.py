"""Compat shim: ``from render import NeRFRenderer`` (reference src/render/__init__.py)."""
from pnr.renderer import NeRFRenderer  # noqa: F401
