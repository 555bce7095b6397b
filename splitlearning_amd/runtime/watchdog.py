"""Failure detection: liveness heartbeats, progress beacons, stall reports, fault injection.

The reference has none: control calls pass `timeout=0` (no timeout), so a
hung Alice hangs Bob forever, and a crashed rank shows up only as TensorPipe `eof`
errors on the others.  Here every process runs a `Watchdog` thread over the job's
rendezvous store (a separate TCPStore client connection, keys namespaced per run):

* **heartbeat** — each rank bumps `hb/<rank>` every `interval` seconds from its own
  thread, so a rank that *died* (killed, segfault, lost node) is noticed by every peer
  after `dead_after` seconds even while they sit inside a blocking collective;
* **progress** — the schedule calls `beat(tag)` at every phase boundary (PhaseTimer) and
  `tick()` inside its loops (every data-plane message, server step chunk, local epoch);
  when no rank has made progress for `stall_after` seconds, rank 0 writes a stall report
  naming each rank's last phase — the "which rank is stuck where" question a hung
  collective otherwise leaves open — to `<log_dir>/watchdog_rank0.json` and to Bob's log;
* **policy** — on a dead peer or a stall the watchdog either only reports
  (`--watchdog report`) or aborts the process with exit code `EXIT_CODE`
  (`--watchdog abort`, the default), so `mp.spawn` / `torchrun` tear the job down
  instead of waiting out the collective timeout;
* **fault injection** — `--fault_inject RANK:TAG[:MODE]` makes rank RANK crash
  (`crash`, exit 17), hang with its heartbeat alive (`hang`: a stall) or hang with its
  heartbeat stopped (`silent`: looks dead) when it reaches the beacon TAG; the failure
  paths above are tested this way on CPU/gloo (tests/test_watchdog_cpu.py).

A rank that finishes cleanly publishes `done/<rank>`; peers stop watching it.
"""
from __future__ import annotations

import json
import os
import sys
import threading
import time
from datetime import timedelta

EXIT_CODE = 86
CRASH_CODE = 17


def parse_fault(spec: str):
    """'RANK:TAG[:MODE]' -> (rank, tag, mode) or None."""
    if not spec:
        return None
    parts = spec.split(":")
    if len(parts) not in (2, 3):
        raise ValueError(f"--fault_inject wants RANK:TAG[:MODE], got {spec!r}")
    mode = parts[2] if len(parts) == 3 else "crash"
    if mode not in ("crash", "hang", "silent"):
        raise ValueError(f"unknown fault mode {mode!r} (crash | hang | silent)")
    return int(parts[0]), parts[1], mode


class Watchdog:
    def __init__(self, store, rank: int, world: int, *, interval: float = 1.0, dead_after: float = 30.0,
                 stall_after: float = 0.0, policy: str = "abort", log_dir: str = "", logger=None,
                 fault: tuple | None = None):
        self.store = store
        self.rank, self.world = rank, world
        self.interval = interval
        self.dead_after = dead_after
        self.stall_after = stall_after
        self.policy = policy
        self.log_dir = log_dir
        self.logger = logger
        self.fault = fault
        self.failed: str | None = None
        self._count = 0
        self._published = -1
        self._tag = "start"
        self._hb = 0
        self._stop = threading.Event()
        self._silent = threading.Event()
        self._lock = threading.Lock()
        self._thread = threading.Thread(target=self._run, name=f"sl-watchdog-{rank}", daemon=True)
        # last value seen per peer and when it last changed (local monotonic clock: no skew)
        now = time.monotonic()
        self._hb_seen = {r: (None, now) for r in range(world) if r != rank}
        self._prog_seen = {r: (None, now) for r in range(world)}
        self._done: set[int] = set()

    # ------------------------------------------------------------------ public
    def start(self):
        self._publish_progress()
        self.store.set(f"hb/{self.rank}", "0")
        self._thread.start()
        return self

    def beat(self, tag: str):
        """Progress beacon with a phase name (main thread, at phase boundaries)."""
        with self._lock:
            self._count += 1
            self._tag = tag
        self._publish_progress()
        if self.fault and self.fault[0] == self.rank and self.fault[1] == tag:
            self._inject(self.fault[2])

    def tick(self):
        """Cheap progress mark for hot loops (no store traffic: the watchdog thread publishes
        the counter once per interval)."""
        self._count += 1

    def stop(self):
        """Clean shutdown: peers stop watching this rank."""
        try:
            self.store.set(f"done/{self.rank}", "1")
        except Exception:
            pass
        self._stop.set()
        if self._thread.is_alive():
            self._thread.join(timeout=5 * self.interval)

    # ------------------------------------------------------------------ internals
    def _publish_progress(self):
        with self._lock:
            self._published = self._count
            val = f"{self._count}|{self._tag}"
        try:
            self.store.set(f"prog/{self.rank}", val)
        except Exception:
            pass

    def _inject(self, mode: str):
        self._say(f"fault injection: rank {self.rank} {mode} at '{self._tag}'")
        if mode == "crash":
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(CRASH_CODE)
        if mode == "silent":
            self._silent.set()
        while True:                       # hang (the heartbeat thread keeps running unless silent)
            time.sleep(3600)

    def _say(self, msg: str):
        print(f"[watchdog rank {self.rank}] {msg}", file=sys.stderr, flush=True)
        if self.logger is not None:
            try:
                self.logger.info(f"[watchdog] {msg}")
            except Exception:
                pass

    def _get(self, key: str):
        if not self.store.check([key]):
            return None
        return self.store.get(key).decode()

    def _run(self):
        while not self._stop.wait(self.interval):
            try:
                if not self._silent.is_set():
                    self._hb += 1
                    self.store.set(f"hb/{self.rank}", str(self._hb))
                    if self._count != self._published:
                        self._publish_progress()
                self._check()
            except Exception as e:       # store gone = the job is tearing down
                if not self._stop.is_set():
                    self._say(f"store unreachable ({type(e).__name__}: {e}); watchdog stops")
                return

    def _check(self):
        now = time.monotonic()
        for r in list(self._hb_seen):
            if r in self._done:
                continue
            if self._get(f"done/{r}") is not None:
                self._done.add(r)
                continue
            v = self._get(f"hb/{r}")
            last, since = self._hb_seen[r]
            if v != last:
                self._hb_seen[r] = (v, now)
            elif now - since > self.dead_after:
                return self._fail("dead_peer", f"rank {r} sent no heartbeat for {now - since:.1f} s")
        if self.rank != 0 or self.stall_after <= 0:
            return
        moved = False
        for r in self._prog_seen:
            v = self._get(f"prog/{r}")
            last, _ = self._prog_seen[r]
            if v != last:
                self._prog_seen[r] = (v, now)
                moved = True
        newest = max(t for _, t in self._prog_seen.values())
        if not moved and now - newest > self.stall_after:
            return self._fail("stall", f"no rank made progress for {now - newest:.1f} s")

    def report(self) -> dict:
        ranks = {}
        for r in range(self.world):
            v = self._prog_seen.get(r, (None, 0))[0]
            cnt, tag = (v.split("|", 1) if v else ("?", "?"))
            ranks[r] = {"beats": cnt, "last_phase": tag, "done": r in self._done}
        return ranks

    def _fail(self, kind: str, msg: str):
        if self.failed:
            return
        self.failed = kind
        rep = {"kind": kind, "message": msg, "reporter": self.rank, "ranks": self.report()}
        self._say(f"{kind}: {msg}; last phase per rank: " +
                  ", ".join(f"{r}={d['last_phase']}" for r, d in rep["ranks"].items()))
        if self.log_dir:
            try:
                os.makedirs(self.log_dir, exist_ok=True)
                with open(os.path.join(self.log_dir, f"watchdog_rank{self.rank}.json"), "w") as f:
                    json.dump(rep, f, indent=1)
            except OSError:
                pass
        if self.policy == "abort":
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(EXIT_CODE)


def connect_store(addr: str, port: int, timeout_s: float = 60.0):
    """A fresh client connection to the job's rendezvous TCPStore (the watchdog thread must
    not share the process group's connection)."""
    import torch.distributed as dist
    return dist.TCPStore(addr, int(port), is_master=False, timeout=timedelta(seconds=timeout_s),
                         wait_for_workers=False)


def make_watchdog(args, comm, logger=None) -> Watchdog | None:
    """Build and start the job's watchdog (collective: every rank calls it), or None
    when `--watchdog off` or the job is a single process with no fault to inject."""
    policy = getattr(args, "watchdog", "abort")
    fault = parse_fault(getattr(args, "fault_inject", ""))
    if policy == "off" or not comm.distributed:
        return None
    import torch.distributed as dist
    run_id = comm.broadcast_obj(os.urandom(6).hex(), 0)
    addr = os.environ.get("MASTER_ADDR", getattr(args, "master_addr", "127.0.0.1"))
    port = int(os.environ.get("MASTER_PORT", getattr(args, "master_port", 29500)))
    store = dist.PrefixStore(f"sl_wd/{run_id}/", connect_store(addr, port))
    wd = Watchdog(store, comm.rank, comm.world, interval=float(getattr(args, "watchdog_interval", 1.0)),
                  dead_after=float(getattr(args, "dead_after_s", 30.0)),
                  stall_after=float(getattr(args, "stall_after_s", 0.0)), policy=policy,
                  log_dir=getattr(args, "log_dir", ""), logger=logger, fault=fault)
    return wd.start()
