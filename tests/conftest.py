"""pytest configuration: the ``gpu`` marker and import paths.

``-m "not gpu"`` runs here (no GPU): oracle vs golden vectors, host logic, the
C-ABI library's exports, and world_size-2 gloo tests.  ``-m gpu`` runs on an
MI355X and compares the HIP path against the oracle / golden vectors.
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "pixel-nerf_amd"), os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) to run")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.device_count() > 0:
        return
    skip = pytest.mark.skip(reason="no HIP device")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
