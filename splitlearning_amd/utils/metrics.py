"""Phase timers and throughput metrics (new: the reference has none).

Each schedule phase (local training, activation dump, server training, eval, ...)
is bracketed by a device synchronisation and timed on the host; the sample
count of the phase gives samples/s, the BASELINE metric.  Results go to the
Bob log ("[perf] ...") and to `<log_dir>/metrics.json` on rank 0.
"""
from __future__ import annotations

import json
import os
import time
from contextlib import contextmanager

import torch

from .trace import NULL_TRACER


def sync(device):
    if device is not None and torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)


class PhaseTimer:
    def __init__(self, device, logger=None, barrier=None, beacon=None):
        self.device = device
        self.logger = logger
        self.barrier = barrier
        self.beacon = beacon          # progress callback (runtime/watchdog.py): beacon(tag)
        self.tracer = NULL_TRACER     # utils/trace.py: one "phase" span per phase
        self.check = None             # phase-end health check after the sync (raises on failure)
        self.records: list[dict] = []

    @contextmanager
    def phase(self, name: str, samples: int = 0):
        if self.beacon is not None:
            self.beacon(name)
        sync(self.device)
        t0 = time.perf_counter()
        box = {"samples": samples}
        span = self.tracer.span(name, "phase")
        info = span.__enter__()
        try:
            yield box
        finally:
            info["samples"] = box["samples"]
            span.__exit__(None, None, None)
            sync(self.device)
            if self.check is not None:
                self.check()
            if self.barrier is not None:
                self.barrier()
            dt = time.perf_counter() - t0
            n = box["samples"]
            rec = {"phase": name, "seconds": dt, "samples": n,
                   "samples_per_s": (n / dt) if (n and dt > 0) else None}
            self.records.append(rec)
            if self.beacon is not None:
                self.beacon(f"{name}:done")
            if self.logger is not None:
                if n:
                    self.logger.info(f"[perf] {name}: {n} samples in {dt:.4f} s = {n / dt:.1f} samples/s")
                else:
                    self.logger.info(f"[perf] {name}: {dt:.4f} s")

    def dump(self, path: str, extra: dict | None = None):
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        with open(path, "w") as f:
            json.dump({"phases": self.records, **(extra or {})}, f, indent=1)
