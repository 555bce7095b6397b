"""Process topology, role placement and the data-plane primitives.

Replaces the reference's TensorPipe RPC agent + distributed autograd
(SURVEY §2.6 N1/N2, §2.8 M1-M20).  The MI355X design is SPMD over
`torch.distributed`:

* one OS process per GPU (backend "nccl" = RCCL over xGMI); on CPU one process
  per role (backend "gloo") like the reference's `mp.spawn`;
* every process runs the same Bob schedule; a "request" is a collective step in
  which only the ranks hosting the involved roles move data — there is no
  command plane to lose messages on, and ordering comes from program order;
* roles are *placed*: Alice_c lives on `alice_rank(c)`; Bob's server tail is
  tensor-parallel over `bob_ranks` (TP degree `bob_tp`).  Co-located roles share
  a process (and a GPU), so the same-GPU case needs no IPC channel
  and RCCL never sees two ranks on one device;
* data plane = point-to-point isend/irecv (cut activation + labels to Bob, cut
  gradient back, Alice->Alice weight relay, SISA activation dump) and one
  all-reduce inside Bob's TP group.  On an 8x MI355X node every pair has its own
  xGMI link, so a one-to-many "multicast" as concurrent p2p sends is per-link
  parallel — better than a ring broadcast for these latency-bound messages.

All waits are bounded by the process-group timeout (`--timeout_s`).
"""
from __future__ import annotations

import datetime
import functools
import os
from dataclasses import dataclass, field

import torch
import torch.distributed as dist

from ..utils.trace import NULL_TRACER


def _noop():
    pass


def _dataplane(fn):
    """Data-plane op: tick the watchdog's progress counter and, when tracing, record a
    "comm" span with the bytes this rank sent."""
    name = fn.__name__

    @functools.wraps(fn)
    def op(self, *a, **k):
        self.progress()
        if not self.tracer.on:
            return fn(self, *a, **k)
        b0, m0 = self.bytes_sent, self.msgs_sent
        with self.tracer.span(name, "comm") as info:
            out = fn(self, *a, **k)
            info["bytes_sent"] = self.bytes_sent - b0
            info["msgs_sent"] = self.msgs_sent - m0
        return out
    return op


@dataclass
class Placement:
    world_size: int          # roles: 1 Bob + k Alices (reference --world_size)
    nprocs: int              # OS processes
    bob_tp: int              # Bob's tensor-parallel degree
    alice_ranks: dict = field(default_factory=dict)
    bob_ranks: list = field(default_factory=list)

    @staticmethod
    def make(world_size: int, nprocs: int, bob_tp: int) -> "Placement":
        k = world_size - 1
        if nprocs < 1:
            raise ValueError("nprocs must be >= 1")
        bob_tp = max(1, min(bob_tp, nprocs))
        if nprocs >= world_size:
            # one process per role, like the reference: rank 0 = Bob, rank c = Alice_c
            alice = {c: c for c in range(1, k + 1)}
        else:
            alice = {c: (c - 1) % nprocs for c in range(1, k + 1)}
        return Placement(world_size, nprocs, bob_tp, alice, list(range(bob_tp)))

    def alice_rank(self, cid: int) -> int:
        return self.alice_ranks[cid]

    def local_alices(self, rank: int) -> list[int]:
        return [c for c, r in sorted(self.alice_ranks.items()) if r == rank]

    def is_bob(self, rank: int) -> bool:
        return rank in self.bob_ranks

    @property
    def bob_root(self) -> int:
        return self.bob_ranks[0]


class Comm:
    """Thin SPMD data-plane wrapper.  With one process every op is local."""

    def __init__(self, rank: int, world: int, device: torch.device, placement: Placement,
                 tp_group=None):
        self.rank = rank
        self.world = world
        self.device = device
        self.pl = placement
        self.tp_group = tp_group
        self.bytes_sent = 0
        self.msgs_sent = 0
        self.progress = _noop        # watchdog tick (runtime/watchdog.py), called per data-plane op
        self.tracer = NULL_TRACER    # utils/trace.py: one "comm" span per data-plane op
        # GPU data plane: a native RCCL communicator over ALL ranks (`_C.TpComm`, set by the
        # session).  Every p2p op below is then issued from C++ on the current HIP stream,
        # grouped, without a host-side wait (torch.distributed isend/irecv + req.wait() from
        # Python otherwise).  None on CPU (gloo).
        self.native = None
        self.msg_log = None          # list of (op, src, dst, nbytes) when a test enables it
        # GPU tensors over a gloo group (several ranks sharing ONE GPU, where RCCL refuses the
        # pair: the N > 1 rehearsal of bench.py --ranks_share_gpu): p2p and collectives are
        # staged through host memory.  Never set on a real multi-GPU run.
        self.host_staging = False

    def _wire(self, t: torch.Tensor) -> torch.Tensor:
        return t.cpu() if self.host_staging else t

    def _buf(self, shape, dtype) -> torch.Tensor:
        return torch.empty(shape, dtype=dtype, device="cpu" if self.host_staging else self.device)

    def _land(self, b: torch.Tensor) -> torch.Tensor:
        return b.to(self.device) if self.host_staging else b

    def _count(self, t: torch.Tensor, n: int, op: str, dst=None):
        nb = t.numel() * t.element_size()
        self.bytes_sent += nb * n
        self.msgs_sent += n
        if self.msg_log is not None:
            for d in (dst if isinstance(dst, (list, tuple)) else [dst]):
                self.msg_log.append((op, self.rank, d, nb))

    @property
    def distributed(self) -> bool:
        return self.world > 1

    # ---------------------------------------------------------------- p2p
    @_dataplane
    def multicast(self, t: torch.Tensor | None, src: int, dsts, shape=None, dtype=None) -> torch.Tensor | None:
        """`src` sends `t` to every rank in `dsts` (concurrent p2p).  Returns the tensor on
        src and on each dst (freshly received), None elsewhere."""
        dsts = [d for d in dict.fromkeys(dsts) if d != src]
        nat = self.native
        if self.rank == src:
            if dsts:
                t = t.contiguous()
                if nat is not None:
                    nat.group_start()
                    for d in dsts:
                        nat.send(t, d)
                    nat.group_end()
                else:
                    w = self._wire(t)
                    reqs = [dist.isend(w, d) for d in dsts]
                    for r in reqs:
                        r.wait()
                self._count(t, len(dsts), "multicast", dsts)
            return t
        if self.rank in dsts:
            if nat is not None:
                buf = torch.empty(shape, dtype=dtype, device=self.device)
                nat.recv(buf, src)
                return buf
            buf = self._buf(shape, dtype)
            dist.recv(buf, src)
            return self._land(buf)
        return None

    @_dataplane
    def exchange(self, sends, recvs):
        """One batched round of point-to-point transfers: `sends` = [(tensor, dst)],
        `recvs` = [(buffer, src)] (this rank's side of every pair).  All transfers are
        posted together (RCCL groups them), so distinct peers' xGMI links run
        concurrently instead of one message after another."""
        sends = [(t.contiguous(), d) for t, d in sends if d != self.rank]
        recvs = [(b, s) for b, s in recvs if s != self.rank]
        if not sends and not recvs:
            return
        if self.native is not None:
            nat = self.native
            nat.group_start()
            for t, d in sends:
                nat.send(t, d)
            for b, s in recvs:
                nat.recv(b, s)
            nat.group_end()
        else:
            stage = [self._buf(b.shape, b.dtype) if self.host_staging else b for b, _ in recvs]
            ops = [dist.P2POp(dist.isend, self._wire(t), d) for t, d in sends]
            ops += [dist.P2POp(dist.irecv, h, s) for h, (_, s) in zip(stage, recvs)]
            for r in dist.batch_isend_irecv(ops):
                r.wait()
            if self.host_staging:
                for h, (b, _) in zip(stage, recvs):
                    b.copy_(h)
        for t, d in sends:
            self._count(t, 1, "exchange", d)

    @_dataplane
    def reduce_to_async(self, t: torch.Tensor | None, dst: int, srcs, shape=None, dtype=None):
        """Post the sum-to-`dst` of `t` over `srcs` (each src sends its partial, dst adds)
        and return a `finish()` callable giving the sum on dst (None elsewhere).  Work the
        caller enqueues between post and finish (Bob's wgrad + optimizer) overlaps the
        transfer of the cut-layer gradient."""
        srcs = list(dict.fromkeys(srcs))
        others = [s for s in srcs if s != dst]
        nat = self.native
        if self.rank == dst:
            mine = t if self.rank in srcs else None
            if not others:
                return lambda: mine
            bufs = [(torch.empty(shape, dtype=dtype, device=self.device) if nat is not None
                     else self._buf(shape, dtype)) for _ in others]
            if nat is not None:
                # every partial arrives on the compute stream; the sum is stream-ordered after it
                nat.group_start()
                for b, s in zip(bufs, others):
                    nat.recv(b, s)
                nat.group_end()
                reqs = []
            else:
                reqs = [dist.irecv(b, s) for b, s in zip(bufs, others)]

            def finish():
                for r in reqs:
                    r.wait()
                if nat is None and self.host_staging:
                    bufs[:] = [self._land(b) for b in bufs]
                acc = mine
                for b in bufs:
                    acc = b if acc is None else acc.add_(b) if acc is not mine else acc + b
                return acc
            return finish
        if self.rank in others:
            t = t.contiguous()
            self._count(t, 1, "reduce_to", dst)
            if nat is not None:
                nat.send(t, dst)
                return lambda: None
            req = dist.isend(self._wire(t), dst)

            def finish_send():
                req.wait()
                return None
            return finish_send
        return lambda: None

    def reduce_to(self, t: torch.Tensor | None, dst: int, srcs, shape=None, dtype=None):
        return self.reduce_to_async(t, dst, srcs, shape, dtype)()

    @_dataplane
    def send_recv(self, t: torch.Tensor | None, src: int, dst: int, shape=None, dtype=None):
        if src == dst:
            return t
        if self.rank == src:
            t = t.contiguous()
            if self.native is not None:
                self.native.send(t, dst)
            else:
                dist.send(self._wire(t), dst)
            self._count(t, 1, "send_recv", dst)
            return t
        if self.rank == dst:
            if self.native is not None:
                buf = torch.empty(shape, dtype=dtype, device=self.device)
                self.native.recv(buf, src)
                return buf
            buf = self._buf(shape, dtype)
            dist.recv(buf, src)
            return self._land(buf)
        return None

    # ---------------------------------------------------------------- collectives
    def tp_allreduce(self, t: torch.Tensor):
        if self.tp_group is not None:
            w = self._wire(t)
            dist.all_reduce(w, group=self.tp_group)
            if w is not t:
                t.copy_(w)
        return t

    @_dataplane
    def tp_allgather(self, t: torch.Tensor) -> list[torch.Tensor]:
        if self.tp_group is None:
            return [t]
        n = dist.get_world_size(self.tp_group)
        dev = t.device
        t = self._wire(t)
        # shards may differ in size by a few rows: gather padded
        size = torch.tensor([t.shape[0] if t.dim() else 1], device=t.device)
        sizes = [torch.zeros_like(size) for _ in range(n)]
        dist.all_gather(sizes, size, group=self.tp_group)
        mx = int(max(s.item() for s in sizes))
        pad = torch.zeros((mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        pad[:t.shape[0]] = t
        outs = [torch.empty_like(pad) for _ in range(n)]
        dist.all_gather(outs, pad, group=self.tp_group)
        return [o[:int(s.item())].to(dev) for o, s in zip(outs, sizes)]

    @_dataplane
    def allreduce_sum_(self, t: torch.Tensor):
        if self.distributed:
            w = self._wire(t)
            dist.all_reduce(w)
            if w is not t:
                t.copy_(w)
        return t

    def broadcast_obj(self, obj, src: int = 0):
        if not self.distributed:
            return obj
        box = [obj]
        dist.broadcast_object_list(box, src=src)
        return box[0]

    def gather_obj(self, obj, dst: int = 0):
        if not self.distributed:
            return [obj]
        out = [None] * self.world if self.rank == dst else None
        dist.gather_object(obj, out, dst=dst)
        return out

    @_dataplane
    def barrier(self):
        if self.distributed:
            if self.device.type == "cuda" and not self.host_staging:
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()


# Bob's TP degree policy (`--bob_tp 0`).  SISA / concat / control: all GPUs — the server phase
# is Bob-local (no per-batch messages), so a shard's share of the optimizer stream is pure
# gain and the only added cost is one fc2 all-reduce per step.  The serial split modes move
# messages every batch, and each extra TP rank adds message rounds on the critical path:
# the fc2 all-reduce, the activation multicast to the shards and the reduction of their
# partial cut gradients (U-shape also multicasts the head's gradient and returns the
# middle's output).  Cost model per batch, us:
#     t(T) = STREAM_B * params / T / HBM  +  rounds(T) * MSG_US
# STREAM_B = bytes per parameter per step (SGD-m 16 + the fc1 forward read 4 without the
# look-ahead, Adam 24 + 4); HBM = 5.5 TB/s (the fused wgrad stream, docs/PERF.md);
# MSG_US = 20 us per p2p / small-collective round on xGMI (RCCL launch + latency, assumed:
# no multi-GPU box was available to measure it).  T = 1 keeps the Alice <-> Bob pair's own
# rounds (2 vanilla, 4 U-shape) for a remote Alice and none for the co-located one.
MSG_US = 20.0
HBM_BPS = 5.5e12
_SERIAL = {"vanilla": (32.146e6, 20, 2, 3), "ushape": (5.509e6, 28, 4, 5)}   # params, B/param, rounds T=1, T>1


def measured_msg_us() -> float | None:
    """A recorded per-message cost (us): `SL_MSG_US`, e.g. the `msg_us` a calibration run
    (`parallel/calibrate.py`, bench.py's `calib` field, `split_nn.py --calibrate`) measured."""
    v = os.environ.get("SL_MSG_US", "")
    try:
        return float(v) if v else None
    except ValueError:
        return None


def choose_bob_tp(mode: str, nprocs: int, msg_us: float | None = None) -> int:
    """Bob's tensor-parallel degree for `mode` on `nprocs` GPUs (see the cost model above).
    `msg_us`: the measured per-message cost; default a recorded one (`measured_msg_us`), else
    the MSG_US assumption."""
    if nprocs <= 1:
        return 1
    if mode not in _SERIAL:
        return nprocs
    if msg_us is None:
        msg_us = measured_msg_us()
    if msg_us is None:
        msg_us = MSG_US
    params, bpp, r1, rt = _SERIAL[mode]
    remote = (nprocs - 1) / nprocs                 # Alices round-robin over the GPUs; Bob on rank 0

    def cost(T):
        return bpp * params / T / HBM_BPS * 1e6 + (rt if T > 1 else r1 * remote) * msg_us
    cands = [T for T in (1, 2, 4, 8, 16) if T <= nprocs and nprocs % T == 0] or [1]
    return min(cands, key=lambda T: (cost(T), T))


class GlooP2PShim:
    """The native RCCL communicator's p2p interface (`_C.TpComm`: send / recv / group_start /
    group_end, ranks = world ranks) over torch.distributed, for CPU tests of the GPU data-plane
    code path in `Comm` (`--native_p2p_shim`).  It keeps RCCL's ordering semantics: an
    un-grouped send or recv blocks until its peer's matching op (on the GPU that blocks the
    stream: a protocol that would deadlock there deadlocks here), and the ops between
    group_start and group_end are posted together and complete together."""

    def __init__(self):
        self._group = None

    def group_start(self):
        assert self._group is None, "nested RCCL group"
        self._group = []

    def group_end(self):
        ops, self._group = self._group, None
        if ops:
            for r in dist.batch_isend_irecv(ops):
                r.wait()

    def send(self, t: torch.Tensor, peer: int):
        if self._group is not None:
            self._group.append(dist.P2POp(dist.isend, t, peer))
        else:
            dist.send(t, peer)

    def recv(self, t: torch.Tensor, peer: int):
        if self._group is not None:
            self._group.append(dist.P2POp(dist.irecv, t, peer))
        else:
            dist.recv(t, peer)


def init_process(rank: int, world: int, backend: str, addr: str, port: int, timeout_s: float,
                 device: torch.device):
    os.environ.setdefault("MASTER_ADDR", addr)
    os.environ.setdefault("MASTER_PORT", str(port))
    if backend == "nccl":
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    kw = {}
    if backend == "nccl" and device.type == "cuda":
        kw["device_id"] = device
    dist.init_process_group(backend, rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=timeout_s), **kw)


def make_tp_group(placement: Placement, backend: str):
    """Sub-group for Bob's TP ranks (every rank must call new_group)."""
    if placement.bob_tp <= 1:
        return None
    if placement.bob_tp == dist.get_world_size():
        return dist.group.WORLD
    return dist.new_group(placement.bob_ranks, backend=backend)
