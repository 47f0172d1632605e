"""Reference module name `utils` -> sgc_amd.utils (drop-in shim).

Put dropin/ first on sys.path (or PYTHONPATH) and the reference's callers
(citation.py, reddit.py, tuning.py: `from utils import ...`) run on the
MI355X engine unchanged.  See INTEGRATION.md.
"""
import os as _os
import sys as _sys

_ROOT = _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))
if _ROOT not in _sys.path:
    _sys.path.insert(0, _ROOT)

from sgc_amd.utils import *  # noqa: E402,F401,F403
from sgc_amd import utils as _impl  # noqa: E402

__all__ = [n for n in dir(_impl) if not n.startswith("_")]
globals().update({n: getattr(_impl, n) for n in __all__})
