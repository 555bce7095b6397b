"""Per-role file loggers with the reference's format and vocabulary.

Reference: `logging.getLogger("bob"|"alice{k}")`, INFO, FileHandler("logs/<role>.log",
mode='w'), format "%(asctime)s: %(message)s" (data_entities.py:116-128,169-180).
Unlike the reference (Q15) the log directory is created if missing.  A role's
logger exists only on the process that hosts the role; elsewhere a no-op
logger is returned so SPMD code can log unconditionally.
"""
from __future__ import annotations

import logging
import os


class _Null:
    def info(self, *a, **k):
        pass

    warning = error = debug = info


NULL = _Null()


def role_logger(name: str, log_dir: str, active: bool):
    if not active:
        return NULL
    os.makedirs(log_dir, exist_ok=True)
    lg = logging.getLogger(name)
    lg.setLevel(logging.INFO)
    lg.propagate = False
    for h in list(lg.handlers):
        lg.removeHandler(h)
        h.close()
    fh = logging.FileHandler(os.path.join(log_dir, f"{name}.log"), mode="w")
    fh.setFormatter(logging.Formatter("%(asctime)s: %(message)s"))
    fh.setLevel(logging.INFO)
    lg.addHandler(fh)
    return lg


def close_all(names):
    for n in names:
        lg = logging.getLogger(n)
        for h in list(lg.handlers):
            h.flush()
            h.close()
            lg.removeHandler(h)
