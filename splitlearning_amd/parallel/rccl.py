"""Native RCCL communicators (`_C.TpComm`) bootstrapped over torch.distributed.

The control plane (rendezvous, timeouts, object broadcast) stays with the
torch.distributed process group; the hot data plane — Bob's per-step tensor-parallel
all-reduce — goes through a communicator the C++ side owns, issued on the current
HIP stream, so it can be captured in the server-step HIP graph.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def make_native_comm(ranks: list[int], my_rank: int, group=None):
    """Collective over every process: returns a `_C.TpComm` on members of `ranks`,
    None elsewhere.  `group` is the torch.distributed group containing `ranks`."""
    from .. import _native
    C = _native.load()
    box = [C.nccl_unique_id() if my_rank == ranks[0] else None]
    dist.broadcast_object_list(box, src=ranks[0], group=group)
    if my_rank not in ranks:
        return None
    return C.TpComm(box[0], len(ranks), ranks.index(my_rank))


def self_comm():
    """A 1-rank communicator (tests / single-GPU graph capture of the collective path)."""
    from .. import _native
    C = _native.load()
    return C.TpComm(C.nccl_unique_id(), 1, 0)


def native_allreduce(tpc):
    def _ar(t: torch.Tensor):
        tpc.allreduce_sum(t)
        return t
    _ar.capturable = True
    _ar.comm = tpc            # the native executor (engine.ServerEpoch) issues it from C++
    return _ar
