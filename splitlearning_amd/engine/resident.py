"""Adoption of the register-resident server epoch (csrc/resident.hip) by every Bob rank.

Reference: bob.train_and_backward's loop (data_entities_vanilla_sisa.py:298-313) is the work
the resident executor runs; the reference's failure rule is that a child failure must not leave
the survivors inconsistent (split_nn.py:183-186, mp.spawn join=True).

Tensor-parallel, the resident executor exchanges fc2 product rows between the ranks inside its
persistent launch, through the same peer-mapped region as the launch-per-stage executor's fused
all-reduce (csrc/ipc_ar.h).  Before adopting it every Bob rank runs a short self-test epoch on a
scratch copy of its shard (`probe`); the ranks adopt it only if every one finished and the
replicated fc3 came out bitwise equal.  A probe whose exchange timed out has raised the region's
error word, which would make every later wait of the launch-per-stage executor give up at once;
so when the agreement is "no", every rank re-arms the region collectively (`rearm`): device
synchronised, error word and host mirror cleared, all ranks continue at one agreed generation
above anything already in the region.  The job then trains on the launch-per-stage executor
instead of dying (tests/test_resident_gpu.py::test_failed_probe_falls_back_on_every_rank).
"""
from __future__ import annotations

import copy
import os
import warnings

import torch

PROBE_TIMEOUT_S = 5.0
# fault injection (tests): the TP rank named here skips its probe launch, so every peer's
# in-launch exchange times out
FAULT_ENV = "SL_FAULT_RESIDENT_PROBE"


def probe(tail, slot, B: int, kind: str = "resident") -> int:
    """One short epoch of a scratch shard on the persistent executor `kind` ("resident":
    csrc/resident.hip, "hybrid": csrc/hybrid.hip) with this rank's layout and peer-mapped
    region (fixed random weights, synthetic inputs, every in-launch wait bounded by
    PROBE_TIMEOUT_S: the hand-offs and the peer exchange).  Returns an integer fingerprint of
    the replicated fc3 weight it produced; raises RuntimeError when a wait gave up."""
    from . import OptSlot, TailEngine
    dev = tail.device
    if os.environ.get(FAULT_ENV, "") == str(tail.tp_rank):
        raise RuntimeError(f"fault injected ({FAULT_ENV}={tail.tp_rank}): probe launch skipped")
    g = torch.Generator().manual_seed(1234)
    mod = copy.deepcopy(tail.module)
    for prm in mod.parameters():
        prm.data = (torch.rand(prm.shape, generator=g) - 0.5) * 0.05
    pt = TailEngine(mod, tail.spec, dev, tail.tp_rank, tail.tp_size, allreduce=tail.allreduce,
                    seed_base=77, ws_tag="#resident_probe")
    pt.resident_timeout_s = PROBE_TIMEOUT_S
    pt.resident_workgroups = int(getattr(tail, "resident_workgroups", 0))
    pslot = type(slot)(slot.cfg)
    n = 8 * B
    x = (torch.rand(n, pt.layers[0].W.shape[1], generator=g) * 4).to(dev)
    y = torch.randint(0, pt.layers[2].W.shape[0], (n,), generator=g).to(dev)
    ipc = getattr(tail.allreduce, "ipc", None)
    old = ipc.timeout_s if ipc is not None else None
    if ipc is not None:
        ipc.set_timeout_s(PROBE_TIMEOUT_S)
    try:
        run = pt.run_hybrid_epoch if kind == "hybrid" else pt.run_resident_epoch
        loss = run(x, y, pslot, B)
        torch.cuda.synchronize(dev)
    finally:
        if ipc is not None:
            ipc.set_timeout_s(old)
    if not bool(torch.isfinite(loss).all().item()):
        raise RuntimeError("non-finite losses")
    bits = pt.layers[2].W.detach().reshape(-1).view(torch.int32).to(torch.int64)
    mult = torch.arange(1, bits.numel() + 1, device=dev, dtype=torch.int64) % 1000003
    return int(((bits * mult) % ((1 << 61) - 1)).sum().item())


def _coll_device():
    import torch.distributed as dist
    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else "cpu"


KINDS = ("resident", "hybrid")


def decide(tail, slot, B: int, distributed: bool, want: bool = True, want_hybrid: bool = True) -> tuple[str, str]:
    """Collective over every process of the default group when `distributed` (ranks that are
    not Bob pass tail=None): which persistent executor Bob's server epochs run on, and why (the
    reason string the bench JSON reports next to `server_executor`).  Returns (kind, why) with
    kind "resident" (the whole shard on-chip: TP >= 7), "hybrid" (a wide shard: fc2 / fc3 on-
    chip, fc1 streamed) or "launch_per_stage".

    Single shard: the first that fits.  Tensor-parallel: every Bob rank probes that executor;
    adopted only if every rank chose the same one and passed with the same fc3 fingerprint.
    When not adopted after any probe ran, every rank re-arms the peer-mapped region at the
    largest generation any rank reserved."""
    kind, fp, why = None, None, "" if want else "off"
    ran_probe = False
    if tail is not None and want:
        if tail.resident_ok(slot, B):
            kind = "resident"
        elif want_hybrid and tail.hybrid_ok(slot, B):
            kind = "hybrid"
        else:
            why = "no persistent executor fits this shard"
        if kind is not None and tail.tp_size > 1:
            ran_probe = True
            try:
                fp = probe(tail, slot, B, kind)
            except RuntimeError as e:            # a wait gave up, or the launch was refused
                warnings.warn(f"{kind} server epoch self-test failed: {e}")
                why = f"{kind} self-test failed on this rank: {str(e).splitlines()[0][:160]}"
                kind = None
    code = KINDS.index(kind) + 1 if kind is not None else 0
    if not distributed:
        return (kind, "adopted") if kind is not None else ("launch_per_stage", why)
    import torch.distributed as dist
    dev = _coll_device()
    big = 1 << 62
    is_bob = tail is not None
    # MIN / MAX over the Bob ranks of (fingerprint, executor code); the other ranks are neutral
    lo = torch.tensor([fp if fp is not None else big, code if is_bob else 99, 0 if ran_probe else 1],
                      dtype=torch.int64, device=dev)
    hi = torch.tensor([fp if fp is not None else -big, code if is_bob else -1], dtype=torch.int64, device=dev)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    same_kind = int(lo[1].item()) == int(hi[1].item()) and int(lo[1].item()) > 0
    fp_ok = int(lo[0].item()) == int(hi[0].item()) or int(lo[0].item()) == big
    any_probe = int(lo[2].item()) == 0
    if same_kind and fp_ok:
        return KINDS[int(lo[1].item()) - 1], "adopted"
    if not why:
        why = ("self-test failed on another rank" if not same_kind else "replicated fc3 differs across ranks")
    if any_probe:
        rearm(tail)
    return "launch_per_stage", why


def rearm(tail):
    """Collective over the default group: clear the peer-mapped region's error word on every
    Bob rank and continue all of them at one generation (the MAX of the generations reserved)."""
    import torch.distributed as dist
    ipc = getattr(getattr(tail, "allreduce", None), "ipc", None) if tail is not None else None
    if ipc is not None:
        torch.cuda.synchronize()
    gen = int(ipc.generation) if ipc is not None else 0
    t = torch.tensor([gen], dtype=torch.int64, device=_coll_device())
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if ipc is not None:
        ipc.rearm(int(t.item()))
