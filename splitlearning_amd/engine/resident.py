"""Adoption of the register-resident server epoch (csrc/resident.hip) by every Bob rank.

Reference: bob.train_and_backward's loop (data_entities_vanilla_sisa.py:298-313) is the work
the resident executor runs; the reference's failure rule is that a child failure must not leave
the survivors inconsistent (split_nn.py:183-186, mp.spawn join=True).

Tensor-parallel, the resident executor exchanges fc2 product rows between the ranks inside its
persistent launch, through the same peer-mapped region as the launch-per-stage executor's fused
all-reduce (csrc/ipc_ar.h).  Before adopting it every Bob rank runs a short self-test epoch on a
scratch copy of its shard (`probe`); the ranks adopt it only if every one finished, its result
agreed with the launch-per-stage executor's on the same scratch epoch, and the replicated fc3
came out bitwise equal across ranks.  A probe whose exchange timed out has raised the region's
error word, which would make every later wait of the launch-per-stage executor give up at once;
so when the agreement is "no", every rank re-arms the region collectively (`rearm`): device
synchronised, error word and host mirror cleared, all ranks continue at one agreed generation
above anything already in the region.  The job then trains on the launch-per-stage executor
instead of dying (tests/test_resident_gpu.py::test_failed_probe_falls_back_on_every_rank).

After adoption, every client epoch goes through `Failsafe`: a launch that fails mid-epoch is
rolled back on every Bob rank and the job continues on launch-per-stage
(tests/test_hybrid_gpu.py::test_tensor_parallel_mid_epoch_failure_survived_across_processes).
"""
from __future__ import annotations

import copy
import os
import warnings

import torch

PROBE_TIMEOUT_S = 5.0
# the probe's fc3 may differ from the launch-per-stage executor's by this fraction of the
# epoch's whole fc3 update (fp32 sum order: ~1e-4 of it; a wrong exchange: O(1))
PROBE_REL_TOL = 0.02


def _launch_per_stage_epoch(t, slot, x, y, B):
    """The scratch epoch on the launch-per-stage executor (as SisaSession.server_epoch runs it
    when no persistent executor is adopted).  Returns the per-row losses."""
    n = x.shape[0]
    if t.lookahead_ok(B) and t.native_epoch_ok(B):
        t.lookahead_prologue(x[:B])
        return t.run_native_epoch(x.contiguous(), y.contiguous(), slot, B, True)
    losses = []
    for s in range(0, n, B):
        lo, _ = t.train_fwd_bwd3(x[s:s + B], y[s:s + B], need_dx=False)
        t.fused_step(slot)
        losses.append(lo)
    return torch.cat(losses)


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
    # the same scratch shard on the launch-per-stage executor: the reference result
    rt = TailEngine(copy.deepcopy(mod), tail.spec, dev, tail.tp_rank, tail.tp_size, allreduce=tail.allreduce,
                    seed_base=77, ws_tag="#resident_probe_ref")
    rslot = type(slot)(slot.cfg)
    w0 = rt.layers[2].W.detach().clone()
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
        ref_loss = _launch_per_stage_epoch(rt, rslot, x, y, B)
        torch.cuda.synchronize(dev)
    finally:
        if ipc is not None:
            ipc.set_timeout_s(old)
    if not bool(torch.isfinite(loss).all().item()):
        raise RuntimeError("non-finite losses")
    # every rank checks its own result against the reference executor: a rank-consistent but
    # wrong exchange (e.g. every rank reading the same stale granule) fails here, where the
    # cross-rank fingerprint agreement alone would adopt it
    if not torch.allclose(loss, ref_loss, rtol=1e-3, atol=1e-3):
        d = (loss - ref_loss).abs().max().item()
        raise RuntimeError(f"losses differ from the launch-per-stage executor's (max |d| {d:.3g})")
    upd = (rt.layers[2].W - w0).norm().item()
    dev_w = (pt.layers[2].W - rt.layers[2].W).norm().item()
    if not dev_w <= PROBE_REL_TOL * upd + 1e-12:
        raise RuntimeError(f"fc3 after the probe epoch differs from the launch-per-stage executor's "
                           f"({dev_w:.3g} vs an update of {upd:.3g})")
    return fingerprint(pt.layers[2].W)


def _coll_device():
    import torch.distributed as dist
    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else "cpu"


KINDS = ("resident", "hybrid")


def _wanted(w) -> bool:
    """An executor flag: True / False, or a string naming why it is unwanted (= False)."""
    return bool(w) and not isinstance(w, str)


def decide(tail, slot, B: int, distributed: bool, want: bool = True, want_hybrid: bool = True) -> tuple[str, str]:
    """Collective over every process of the default group when `distributed` (ranks that are
    not Bob pass tail=None): which persistent executor Bob's server epochs run on, and why (the
    reason string the bench JSON reports next to `server_executor`).  Returns (kind, why) with
    kind "resident" (the whole shard on-chip: TP >= 7), "hybrid" (a wide shard: fc2 / fc3 on-
    chip, fc1 streamed) or "launch_per_stage".

    `want` gates the resident executor (`--resident`), `want_hybrid` the hybrid one (`--hybrid`):
    the two flags are independent.  Passing a string instead of False gives the reason the
    executor is unwanted (e.g. "dtype bf16"); it is reported when nothing was adopted.

    Single shard: the first that fits.  Tensor-parallel: every Bob rank probes that executor;
    adopted only if every rank chose the same one and passed with the same fc3 fingerprint
    and, per rank, the probe's result agreed with the launch-per-stage executor's on the same
    scratch epoch (`probe`).  When not adopted after any probe ran, every rank re-arms the
    peer-mapped region at the largest generation any rank reserved."""
    kind, fp = None, None
    on_r, on_h = _wanted(want), _wanted(want_hybrid)
    off = [w for w in (want, want_hybrid) if isinstance(w, str) and w]
    why = off[0] if off else ("off" if not on_r and not on_h else "")
    ran_probe = False
    if tail is not None and (on_r or on_h):
        if on_r and tail.resident_ok(slot, B):
            kind = "resident"
        elif on_h and tail.hybrid_ok(slot, B):
            kind = "hybrid"
        elif not why:
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


FAULT_EPOCH_ENV = "SL_FAULT_PERSIST_EPOCH"


class Failsafe:
    """Client epochs on a persistent executor that survive an in-launch failure.

    Before each epoch the shard's weights, optimizer state and step / dropout counters are
    copied device-to-device (`TailEngine.snapshot_state`, one buffer reused).  A launch whose
    in-launch waits gave up (a hand-off timeout; across GPUs, the peer-mapped fc2 exchange
    failing; an injected fault) raises after updating part of the shard.  `run` then agrees
    with the other Bob ranks (a MAX all-reduce of one flag over `group`, every epoch, since a
    rank whose launch finished before its peer failed has nothing to report by itself), and if
    ANY rank failed, every rank restores its copy, re-arms the peer-mapped region collectively
    (`rearm`) and returns False: the caller runs that epoch, and every later one, on the
    launch-per-stage executor.  The restored shard is bitwise the pre-epoch one, so the job's
    result is exactly that of a job which switched executors at that epoch.

    Fault injection (tests): SL_FAULT_PERSIST_EPOCH="TP_RANK:EPOCH:STEP" stops every workgroup
    of TP rank TP_RANK's launch at step STEP of its EPOCH-th persistent epoch (0-based): that
    step's first hand-off wait is never met, times out (error word 2) and every other wait of
    the launch gives up, as a hand-off that never arrives would make them (the kernels'
    `fault_step`)."""

    def __init__(self, tail, slot, B: int, group=None, enabled: bool = True):
        self.tail, self.slot, self.B, self.group, self.enabled = tail, slot, B, group, enabled
        self.snap = None
        self.epochs = 0
        self.fallback = None

    def run(self, kind: str, acts: torch.Tensor, labels: torch.Tensor, step_rows=None) -> bool:
        tail, slot, B = self.tail, self.slot, self.B
        idx = self.epochs
        self.epochs += 1
        if self.enabled:
            self.snap = tail.snapshot_state(slot, self.snap)
        ex = tail._resident_executor(slot, B) if kind == "resident" else tail._hybrid_executor(slot, B)
        f = os.environ.get(FAULT_EPOCH_ENV, "").split(":")
        if len(f) == 3 and int(f[0]) == tail.tp_rank and int(f[1]) == idx:
            ex.set_fault_step(int(f[2]))
        err = None
        fatal = None
        self.loss = None
        try:
            if kind == "resident":
                self.loss = tail.run_resident_epoch(acts, labels, slot, B, step_rows)
            else:
                self.loss = tail.run_hybrid_epoch(acts, labels, slot, B, step_rows)
        except RuntimeError as e:
            if "in-launch wait gave up" not in str(e) or not self.enabled:
                fatal = e
            else:
                err = str(e).splitlines()[0][:200]
        if fatal is None and err is None and self.enabled:
            # a launch that finished but produced garbage (a non-finite loss, or a non-finite
            # value anywhere in the shard) is rolled back like one that timed out: the
            # snapshot is the pre-epoch state, and launch-per-stage re-runs the epoch
            bad = self.nonfinite(tail, slot, self.loss)
            if bad:
                err = f"non-finite result after the launch ({bad})"
        # 0 = ok, 1 = recoverable on this rank, 2 = fatal on this rank.  Every rank joins the
        # agreement before anything is raised, so a fatal error ends every Bob rank together
        # instead of leaving the others blocked in this all-reduce
        code = 2 if fatal is not None else (1 if err is not None else 0)
        if tail.tp_size > 1:
            import torch.distributed as dist
            flag = torch.tensor([code], dtype=torch.int32, device=_coll_device())
            dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self.group)
            code = int(flag.item())
        if fatal is not None:
            raise fatal
        if code == 2:
            raise RuntimeError(f"{kind} server epoch {idx}: another Bob rank's persistent launch failed fatally")
        failed = code > 0
        if not failed:
            return True
        tail.restore_state(slot, self.snap)
        if tail.tp_size > 1:
            rearm(tail, group=self.group)
        why = err if err is not None else "another Bob rank's persistent epoch failed"
        warnings.warn(f"{kind} server epoch {idx} failed ({why}); shard restored, continuing on launch-per-stage")
        self.fallback = {"from": kind, "epoch": idx, "reason": why}
        return False

    @staticmethod
    def nonfinite(tail, slot, loss) -> str:
        """'' when the epoch's losses and every weight / bias / optimizer-state tensor of the
        shard are finite, else a short description of the first offender.  One sum per tensor
        (a NaN or an infinity anywhere makes it non-finite; no tensor-sized temporaries) and ONE
        host sync per epoch (~0.1 ms at TP = 1 against a ~0.5 s server epoch)."""
        ts = [("loss", loss)] if loss is not None else []
        for L in tail.layers:
            for nm, p in ((f"{L.spec.name}.weight", L.W), (f"{L.spec.name}.bias", L.b)):
                ts.append((nm, p))
                st = slot.state(nm, p)
                ts += [(f"{nm}.{k}", st[k]) for k in sorted(st)]
        flags = torch.isfinite(torch.stack([t.detach().sum(dtype=torch.float64) for _, t in ts])).cpu()
        for (nm, _), ok in zip(ts, flags.tolist()):
            if not ok:
                return nm
        return ""


def rearm(tail, group=None):
    """Collective over `group` (default: the default group; a mid-epoch fallback passes the Bob
    ranks' group): clear the peer-mapped region's error word on every Bob rank and continue all
    of them at one generation (the MAX of the generations reserved)."""
    import torch.distributed as dist
    ipc = getattr(getattr(tail, "allreduce", None), "ipc", None) if tail is not None else None
    if ipc is not None:
        torch.cuda.synchronize()
    gen = int(ipc.generation) if ipc is not None else 0
    t = torch.tensor([gen], dtype=torch.int64, device=_coll_device())
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    if ipc is not None:
        ipc.rearm(int(t.item()))


def fingerprint(t: torch.Tensor) -> int:
    """Integer fingerprint of a tensor's exact bits (the probe's fc3 check): equal fingerprints
    on every rank = bitwise-equal replicas, with overwhelming probability."""
    bits = t.detach().reshape(-1).contiguous().view(torch.int32).to(torch.int64)
    mult = torch.arange(1, bits.numel() + 1, device=bits.device, dtype=torch.int64) % 1000003
    return int(((bits * mult) % ((1 << 61) - 1)).sum().item())


def validate(sess, steps: int = 32) -> dict:
    """Self-check of a finished run (bench.py, after its timed region; collective over every
    rank of the job): is what the adopted server executor computed right?

    * Every Bob rank replays `steps` steps of its first cached client epoch twice from one
      snapshot: on the adopted persistent executor (resident / hybrid) and on the launch-per-
      stage executor, and compares the losses (rtol / atol 1e-3, as the adoption probe) and
      the fc3 weight (within PROBE_REL_TOL of that slice's fc3 update); then restores the
      snapshot, so the job's state is untouched.
    * The replicated fc3 (identical on every TP rank by construction: rank-ordered sums) is
      fingerprinted and compared across the Bob ranks.
    Returns {validated, max_loss_diff, fc3_dev_over_update, fc3_replicas_equal, executor,
    steps}; `validated` is the AND over all ranks (None when the mode has no server epochs)."""
    import torch.distributed as dist
    mode = getattr(sess, "mode", "")
    if mode not in ("sisa", "control", "concat"):
        return {"validated": None, "reason": f"mode {mode}: no server executor to validate"}
    kind = getattr(sess, "server_executor", "launch_per_stage")
    out = {"executor": kind, "steps": 0, "max_loss_diff": None, "fc3_dev_over_update": None,
           "fc3_replicas_equal": None}
    ok = True
    tail = sess.tail if sess.is_bob else None
    if tail is not None:
        slot, B = sess.bob_slot, sess.B
        cache = sess.activation_and_labels_cache
        if kind in KINDS and cache:
            acts, labels = cache[min(cache)]
            n = min(int(labels.numel()) // B, steps) * B
            if n >= B:
                x = acts[:n].float().contiguous()
                y = labels[:n].contiguous()
                snap = tail.snapshot_state(slot)
                w0 = tail.layers[2].W.detach().clone()
                lp = (tail.run_resident_epoch if kind == "resident" else tail.run_hybrid_epoch)(x, y, slot, B)
                wp = tail.layers[2].W.detach().clone()
                tail.restore_state(slot, snap)
                ll = _launch_per_stage_epoch(tail, slot, x, y, B)
                wl = tail.layers[2].W.detach().clone()
                tail.restore_state(slot, snap)
                torch.cuda.synchronize(tail.device) if tail.device.type == "cuda" else None
                d = (lp - ll).abs().max().item()
                upd = (wl - w0).norm().item()
                dev_w = (wp - wl).norm().item() / max(upd, 1e-30)
                out.update(steps=n // B, max_loss_diff=d, fc3_dev_over_update=dev_w)
                ok = (bool(torch.isfinite(lp).all().item()) and torch.allclose(lp, ll, rtol=1e-3, atol=1e-3)
                      and dev_w <= PROBE_REL_TOL)
        if tail.tp_size > 1:
            fp = fingerprint(tail.layers[2].W)
            dev = _coll_device()
            lo = torch.tensor([fp], dtype=torch.int64, device=dev)
            hi = lo.clone()
            g = sess.comm.tp_group
            dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=g)
            dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=g)
            same = int(lo.item()) == int(hi.item())
            out["fc3_replicas_equal"] = same
            ok = ok and same
    if getattr(sess.comm, "distributed", False):
        f = torch.tensor([1 if ok else 0], dtype=torch.int32, device=_coll_device())
        dist.all_reduce(f, op=dist.ReduceOp.MIN)
        ok = bool(int(f.item()))
    out["validated"] = ok
    return out
