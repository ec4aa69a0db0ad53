"""pnr — MI355X-native pixelNeRF ray march (HIP kernels in libpnr.so).

Drop-in for the reference's hot path:
  render.NeRFRenderer          -> pnr.renderer.NeRFRenderer
  model.make_model / PixelNeRFNet -> pnr.models
  util.{gen_rays, pose_spherical, ...} -> pnr.util

Put ``pixel-nerf_amd/`` on sys.path (as the reference puts ``src/``) and the
``render`` / ``model`` / ``util`` shim packages resolve to these.
"""
from . import util  # noqa: F401
from .conf import Conf, parse_file  # noqa: F401
from .models import PixelNeRFNet, make_model  # noqa: F401
from .renderer import DotMap, NeRFRenderer  # noqa: F401

__version__ = "0.1.0"
