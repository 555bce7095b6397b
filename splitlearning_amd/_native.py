"""Loader for the in-tree native extension (`_C`, built by `splitlearning_amd.build`)."""
from __future__ import annotations

import importlib
import os

_MOD = None


def available() -> bool:
    try:
        load()
        return True
    except Exception:
        return False


def load():
    """Import `splitlearning_amd._C`; build it first if the .so is absent and
    SL_AUTOBUILD=1.  Raises ImportError otherwise (no silent fallback)."""
    global _MOD
    if _MOD is not None:
        return _MOD
    try:
        _MOD = importlib.import_module("splitlearning_amd._C")
    except ImportError:
        if os.environ.get("SL_AUTOBUILD", "0") == "1":
            from . import build
            build.build(verbose=False)
            _MOD = importlib.import_module("splitlearning_amd._C")
        else:
            raise ImportError("splitlearning_amd._C is not built: run `python -m splitlearning_amd.build`")
    return _MOD
