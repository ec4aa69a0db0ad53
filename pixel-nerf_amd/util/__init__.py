"""Compat shim: ``import util`` (reference src/util/__init__.py: ``from .util import *`` and
``from . import args``).  Every helper the reference's callers reach as ``util.X`` resolves here
(tests/test_dropin.py scans eval/*.py and train/*.py for them), plus ``util.args.parse_args``."""
from pnr.util import *  # noqa: F401,F403
from pnr.util import combine_interleaved, repeat_interleave  # noqa: F401
from pnr.conf import parse_file  # noqa: F401

from . import args  # noqa: F401,E402
