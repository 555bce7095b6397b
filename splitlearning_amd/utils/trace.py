"""Chrome-trace timeline per rank (`--trace_dir`): host spans + device (HIP-event) spans.

The reference has no tracing (one commented-out timer and tqdm bars).
Here, with `--trace_dir DIR`, every rank writes `DIR/trace_rank<r>.json` in the Chrome
trace-event format (open in chrome://tracing or Perfetto):

* `phase` spans — every schedule phase (PhaseTimer), tid "host";
* `comm` spans — every data-plane operation of `parallel.dist.Comm` with its byte count
  (multicast, batched exchange, reduce-to, send/recv, barrier, all-reduce), tid "host";
* `gpu` spans — device time of marked regions (Bob's server epoch per client, each
  Alice's local epoch) measured with HIP events on the compute stream and placed on
  the host clock through one anchor event, tid "gpu".  Events are only resolved at
  `dump()`, so tracing adds no synchronisation to the timed loop.

Disabled tracing is a no-op object (`NULL_TRACER`), so call sites stay unconditional.
rocprofv3 (`scripts/gpu_prof*.sh`) remains the tool for per-kernel device time.
"""
from __future__ import annotations

import json
import os
import time
from contextlib import contextmanager

import torch


class Tracer:
    on = True

    def __init__(self, rank: int, path: str, device: torch.device | None = None):
        self.rank = rank
        self.path = path
        self.device = device
        self.events: list[dict] = []
        self._t0 = time.perf_counter()
        self._gpu: list[tuple] = []
        self._anchor = None
        if device is not None and device.type == "cuda":
            self._anchor = torch.cuda.Event(enable_timing=True)
            self._anchor.record()
            torch.cuda.synchronize(device)
            self._anchor_host = self._us()

    def _us(self) -> float:
        return (time.perf_counter() - self._t0) * 1e6

    @contextmanager
    def span(self, name: str, cat: str = "host", **args):
        """Host span; yields its args dict so the block can add results (e.g. bytes)."""
        t = self._us()
        try:
            yield args
        finally:
            self.events.append({"name": name, "cat": cat, "ph": "X", "ts": t, "dur": self._us() - t,
                                "pid": self.rank, "tid": "host", "args": args})

    def instant(self, name: str, **args):
        self.events.append({"name": name, "ph": "i", "s": "p", "ts": self._us(), "pid": self.rank,
                            "tid": "host", "args": args})

    def counter(self, name: str, **values):
        self.events.append({"name": name, "ph": "C", "ts": self._us(), "pid": self.rank, "args": values})

    @contextmanager
    def gpu_span(self, name: str, **args):
        """Device time of the work enqueued inside the block (current stream)."""
        if self._anchor is None:
            with self.span(name, "gpu", **args):
                yield args
            return
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        try:
            yield args
        finally:
            e.record()
            self._gpu.append((name, s, e, args))

    def dump(self):
        if self._gpu:
            torch.cuda.synchronize(self.device)
            for name, s, e, args in self._gpu:
                ts = self._anchor_host + self._anchor.elapsed_time(s) * 1e3
                self.events.append({"name": name, "cat": "gpu", "ph": "X", "ts": ts,
                                    "dur": s.elapsed_time(e) * 1e3, "pid": self.rank, "tid": "gpu",
                                    "args": args})
            self._gpu.clear()
        os.makedirs(os.path.dirname(self.path) or ".", exist_ok=True)
        meta = [{"name": "process_name", "ph": "M", "pid": self.rank, "args": {"name": f"rank {self.rank}"}}]
        with open(self.path, "w") as f:
            json.dump({"traceEvents": meta + self.events, "displayTimeUnit": "ms"}, f)


class _NullTracer:
    on = False

    @contextmanager
    def span(self, name, cat="host", **args):
        yield args

    gpu_span = span

    def instant(self, name, **args):
        pass

    def counter(self, name, **values):
        pass

    def dump(self):
        pass


NULL_TRACER = _NullTracer()


def make_tracer(args, rank: int, device) -> Tracer | _NullTracer:
    d = getattr(args, "trace_dir", "")
    if not d:
        return NULL_TRACER
    return Tracer(rank, os.path.join(d, f"trace_rank{rank}.json"), device)
