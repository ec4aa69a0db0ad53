"""Compat shim: ``from data import get_split_dataset`` (reference src/data/__init__.py)."""
from pnr.data import *  # noqa: F401,F403
from pnr.data import SRNDataset, get_split_dataset  # noqa: F401
