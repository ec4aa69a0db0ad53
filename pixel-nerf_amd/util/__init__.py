"""Compat shim: ``import util`` (reference src/util/__init__.py) — the geometry
helpers the ray-march callers use, and ``util.args``-free config loading."""
from pnr.util import *  # noqa: F401,F403
from pnr.util import combine_interleaved, repeat_interleave  # noqa: F401
from pnr.conf import parse_file  # noqa: F401
