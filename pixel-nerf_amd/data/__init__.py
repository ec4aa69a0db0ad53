"""Compat shim: ``from data import get_split_dataset`` (reference src/data/__init__.py): the SRN,
DVR (ShapeNet-NMR / DTU) and multi-object loaders and the DTU colour jitter, from pnr.data."""
from pnr.data import *  # noqa: F401,F403
from pnr.data import (ColorJitterDataset, DVRDataset, MultiObjectDataset, SRNDataset,  # noqa: F401
                      get_split_dataset)
