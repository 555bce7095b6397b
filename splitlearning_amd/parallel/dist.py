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

    @property
    def distributed(self) -> bool:
        return self.world > 1

    # ---------------------------------------------------------------- p2p
    @_dataplane
    def multicast(self, t: torch.Tensor | None, src: int, dsts, shape=None, dtype=None) -> torch.Tensor | None:
        """`src` sends `t` to every rank in `dsts` (concurrent p2p).  Returns the tensor on
        src and on each dst (freshly received), None elsewhere."""
        dsts = [d for d in dict.fromkeys(dsts) if d != src]
        if self.rank == src:
            if dsts:
                t = t.contiguous()
                reqs = [dist.isend(t, d) for d in dsts]
                for r in reqs:
                    r.wait()
                self.bytes_sent += t.numel() * t.element_size() * len(dsts)
                self.msgs_sent += len(dsts)
            return t
        if self.rank in dsts:
            buf = torch.empty(shape, dtype=dtype, device=self.device)
            dist.recv(buf, src)
            return buf
        return None

    @_dataplane
    def exchange(self, sends, recvs):
        """One batched round of point-to-point transfers: `sends` = [(tensor, dst)],
        `recvs` = [(buffer, src)] (this rank's side of every pair).  All transfers are
        posted together (RCCL groups them), so distinct peers' xGMI links run
        concurrently instead of one message after another."""
        ops = [dist.P2POp(dist.isend, t.contiguous(), d) for t, d in sends if d != self.rank]
        ops += [dist.P2POp(dist.irecv, b, s) for b, s in recvs if s != self.rank]
        if not ops:
            return
        for r in dist.batch_isend_irecv(ops):
            r.wait()
        for t, d in sends:
            if d != self.rank:
                self.bytes_sent += t.numel() * t.element_size()
                self.msgs_sent += 1

    @_dataplane
    def reduce_to_async(self, t: torch.Tensor | None, dst: int, srcs, shape=None, dtype=None):
        """Post the sum-to-`dst` of `t` over `srcs` (each src sends its partial, dst adds)
        and return a `finish()` callable giving the sum on dst (None elsewhere).  Work the
        caller enqueues between post and finish (Bob's wgrad + optimizer) overlaps the
        transfer of the cut-layer gradient."""
        srcs = list(dict.fromkeys(srcs))
        others = [s for s in srcs if s != dst]
        if self.rank == dst:
            mine = t if self.rank in srcs else None
            if not others:
                return lambda: mine
            bufs = [torch.empty(shape, dtype=dtype, device=self.device) for _ in others]
            reqs = [dist.irecv(b, s) for b, s in zip(bufs, others)]

            def finish():
                for r in reqs:
                    r.wait()
                acc = mine
                for b in bufs:
                    acc = b if acc is None else acc.add_(b) if acc is not mine else acc + b
                return acc
            return finish
        if self.rank in others:
            t = t.contiguous()
            req = dist.isend(t, dst)
            self.bytes_sent += t.numel() * t.element_size()
            self.msgs_sent += 1

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
            dist.send(t.contiguous(), dst)
            self.bytes_sent += t.numel() * t.element_size()
            self.msgs_sent += 1
            return t
        if self.rank == dst:
            buf = torch.empty(shape, dtype=dtype, device=self.device)
            dist.recv(buf, src)
            return buf
        return None

    # ---------------------------------------------------------------- collectives
    def tp_allreduce(self, t: torch.Tensor):
        if self.tp_group is not None:
            dist.all_reduce(t, group=self.tp_group)
        return t

    @_dataplane
    def tp_allgather(self, t: torch.Tensor) -> list[torch.Tensor]:
        if self.tp_group is None:
            return [t]
        n = dist.get_world_size(self.tp_group)
        # shards may differ in size by a few rows: gather padded
        size = torch.tensor([t.shape[0] if t.dim() else 1], device=self.device)
        sizes = [torch.zeros_like(size) for _ in range(n)]
        dist.all_gather(sizes, size, group=self.tp_group)
        mx = int(max(s.item() for s in sizes))
        pad = torch.zeros((mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=self.device)
        pad[:t.shape[0]] = t
        outs = [torch.empty_like(pad) for _ in range(n)]
        dist.all_gather(outs, pad, group=self.tp_group)
        return [o[:int(s.item())] for o, s in zip(outs, sizes)]

    @_dataplane
    def allreduce_sum_(self, t: torch.Tensor):
        if self.distributed:
            dist.all_reduce(t)
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
            if self.device.type == "cuda":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()


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
