"""Native split-mode epochs: a vanilla / U-shape `split_epoch` issued from C++
(`_C.SplitEpoch`, csrc/split.cpp) when the Alice and the whole Bob (TP = 1) live in this
process — the one-GPU BASELINE point (ws = 2) and every co-located placement — and, for an
Alice remote from a one-shard Bob (BASELINE config 2, U-shape ws = 2 on 2 GPUs; vanilla
with `--bob_tp 1`), each side's half of the same loop with the per-batch messages on the
split channel (csrc/ipc_p2p.h peer-mapped messages, or RCCL).

The executor issues the same launches, with the same arguments, dropout seeds, workspaces
and optimizer step counts, as `VanillaSession.split_epoch` / `UShapeSession.split_epoch` in
their look-ahead order, so the parameters it produces are bit-identical to the Python
loop's (tests/test_split_native_gpu.py); the Python loop
stays the path for every other placement and for `--python_epoch`.

Reference hot loops: data_entities_vanilla.py:66-76 and data_entities.py:65-81.
"""
from __future__ import annotations

import os

import torch

_KIND = {"sgd": 1, "adam": 2}
# rows per batch `_C.SplitEpoch` accepts on every role (csrc/split.cpp, the constructor's check)
SPLIT_MIN_B, SPLIT_MAX_B = 1, 64


def _opt(cfg) -> dict:
    return {"kind": _KIND[cfg.kind], "lr": cfg.lr, "beta1": cfg.beta1, "beta2": cfg.beta2, "eps": cfg.eps,
            "wd": cfg.weight_decay, "momentum": cfg.momentum}


def _param(slot, name: str, p: torch.Tensor) -> dict:
    st = slot.state(name, p)
    return {"p": p, "s0": st["m"] if "m" in st else st["buf"], "s1": st.get("v")}


def native_split_ok(sess, cid: int, mode: str) -> bool:
    """Whether `run_native_split_epoch` can drive this epoch: Alice_cid hosted here, Bob a
    single shard in this process, the HIP kernels, the look-ahead order and its batch bound."""
    a = sess.alices.get(cid)
    if a is None or not getattr(sess.args, "native_epoch", True) or not sess.is_bob:
        return False
    if list(sess.bob_ranks) != [sess.rank] or sess.tail.tp_size != 1 or sess.device.type != "cuda":
        return False
    if not hasattr(sess.ops, "C") or a.front.frozen or a.train.x.dtype != torch.uint8:
        return False
    if not sess.split_lookahead(cid):
        return False
    B = sess.B
    if mode == "vanilla":
        return sess.tail.fused3_ok() and sess.tail.lookahead_ok(B)
    return (sess.tail.grouped_ok(B) and len(sess.tail.layers) == 2 and sess.head_fused(B)
            and a.head.head_step_ok(B))


def _alice_cfg(sess, cid: int, mode: str) -> dict:
    a = sess.alices[cid]
    a.front.flush()
    w, b = a.front.params
    pre = "front." if mode == "ushape" else ""
    cfg = {"x": a.train.x, "y": a.train.y,
           "front": {"w": _param(a.slot, pre + "conv.weight", w), "b": _param(a.slot, pre + "conv.bias", b)},
           "front_opt": _opt(a.slot.cfg)}
    if mode == "ushape":
        H = a.head.layers[0]
        cfg["head"] = {"w": _param(a.slot, f"head.{H.spec.name}.weight", H.W),
                       "b": _param(a.slot, f"head.{H.spec.name}.bias", H.b)}
    return cfg


def _bob_cfg(sess, cid: int, mode: str) -> dict:
    tail, ops, dev, B = sess.tail, sess.ops, sess.device, sess.B
    bslot = sess.bob_slot(cid)
    layers = []
    for L in tail.layers:
        layers.append({"w": _param(bslot, f"{L.spec.name}.weight", L.W),
                       "b": _param(bslot, f"{L.spec.name}.bias", L.b)})
    N2 = tail.layers[1].W.shape[0]
    nmax = max(L.W.shape[0] for L in tail.layers)
    kmax = max(L.W.shape[1] for L in tail.layers)
    cfg = {"bob_opt": _opt(bslot.cfg), "tail": layers,
           "p1": tail.layers[0].spec.dropout, "p2": tail.layers[1].spec.dropout,
           # the Python path's own workspaces (ops/hip_ops.py), so every split factor matches
           "fwdws": ops._workspace(dev, 16 * B * nmax, "fwd"),
           "dgws": ops._workspace(dev, 16 * B * kmax, "dgrad")}
    if mode == "vanilla":
        C3 = tail.layers[2].W.shape[0]
        cfg["p2ws"] = ops._workspace(dev, 16 * B * N2, "fc2p")
        cfg["headws"] = ops._workspace(dev, ops.C().head3_slices(N2) * B * C3, "head")
    return cfg


def _bob_done(sess, cid: int, t_b: int, fc: int):
    tail = sess.tail
    sess.bob_slot(cid).t, tail.fwd_count = int(t_b), int(fc)
    tail._pre = None
    tail.acts, tail.dz, tail._wg = [], [], []


def _count(sess, kind: str):
    """Per-session tally of native split epochs by kind (bench.py reports it)."""
    c = sess.__dict__.setdefault("native_split_epochs", {})
    c[kind] = c.get(kind, 0) + 1


def run_native_split_epoch(sess, cid: int, order: torch.Tensor, mode: str):
    """One split epoch of Alice_cid over `order` through `_C.SplitEpoch`."""
    _count(sess, "colocated")
    a = sess.alices[cid]
    B = sess.B
    cfg = {"mode": 1 if mode == "vanilla" else 2, "B": B}
    cfg.update(_alice_cfg(sess, cid, mode))
    cfg.update(_bob_cfg(sess, cid, mode))
    ex = sess.ops.C().SplitEpoch(cfg)
    order = order.to(sess.device, torch.int64).contiguous()
    sess.tail._pre = None
    t_a, t_b, fc = ex.run(order, a.slot.t, sess.bob_slot(cid).t, sess.tail.fwd_count, sess.tail.seed_base)
    nb = -(-int(order.numel()) // B)
    a.slot.t = int(t_a)
    _bob_done(sess, cid, t_b, fc)
    if a.head is not None:
        a.head.fwd_count += nb
    return ex


# ---------------------------------------------------------------------- persistent vanilla epoch
def persistent_vanilla_ok(sess, cid: int) -> bool:
    """Whether `run_persistent_vanilla_epoch` may drive this epoch: the co-located native
    conditions, fp32 SGD-momentum on both sides, batches of at most 16 rows, the flag, and no
    earlier failure of the persistent executor in this session."""
    if getattr(sess.args, "split_persist", "auto") == "off" or sess.__dict__.get("_va_off"):
        return False
    if getattr(sess.comm, "host_staging", False):
        return False   # ranks share this GPU (--ranks_share_gpu): 256 co-resident workgroups are not assured
    if not native_split_ok(sess, cid, "vanilla") or not hasattr(sess.ops.C(), "VanillaEpoch"):
        return False
    # vanilla.hip computes in exact fp32 only: a bf16 run (fp32 master weights, bf16 operands
    # through the global compute-dtype switch) stays on the per-batch executor, whose kernels
    # honour it, instead of silently running fp32
    dt = getattr(sess.args, "dtype", "fp32")
    C = sess.ops.C()
    if dt != "fp32" or (hasattr(C, "get_compute_dtype") and C.get_compute_dtype() != "fp32"):
        sess.__dict__["split_persist_reason"] = f"dtype {dt if dt != 'fp32' else C.get_compute_dtype()}: fp32 only"
        return False
    a = sess.alices[cid]
    if not 1 <= sess.B <= 16:
        # every product's MFMA row block is the batch (csrc/vanilla.hip): larger batches run per batch
        sess.__dict__["split_persist_reason"] = f"batch {sess.B} > 16: per-batch executor"
        return False
    return (a.slot.cfg.kind == "sgd" and sess.bob_slot(cid).cfg.kind == "sgd"
            and len(sess.tail.layers) == 3 and all(L.W.dtype == torch.float32 for L in sess.tail.layers))


def _va_cfg(sess, cid: int) -> dict:
    a = sess.alices[cid]
    a.front.flush()
    w, b = a.front.params
    aw, ab = _param(a.slot, "conv.weight", w), _param(a.slot, "conv.bias", b)
    bslot = sess.bob_slot(cid)
    layers = []
    for L in sess.tail.layers:
        pw, pb = _param(bslot, f"{L.spec.name}.weight", L.W), _param(bslot, f"{L.spec.name}.bias", L.b)
        layers.append({"W": pw["p"], "b": pb["p"], "s0": pw["s0"], "sb0": pb["s0"]})
    bo, ao = bslot.cfg, a.slot.cfg
    return {"layers": layers, "lr": bo.lr, "momentum": bo.momentum, "wd": bo.weight_decay,
            "alice": {"w": aw["p"], "b": ab["p"], "s0w": aw["s0"], "s0b": ab["s0"]},
            "alice_lr": ao.lr, "alice_momentum": ao.momentum, "alice_wd": ao.weight_decay,
            "x": a.train.x, "y": a.train.y, "B": sess.B,
            "p1": sess.tail.layers[0].spec.dropout, "p2": sess.tail.layers[1].spec.dropout,
            "timeout_s": float(getattr(sess.args, "persist_timeout_s", 30.0)),
            # a plain (non-cooperative) launch of the same grid for rocprofv3, whose process dies at
            # exit after any cooperative launch (docs/PERF.md, tools/coop_repro.hip)
            "workgroups": int(os.environ.get("SL_PERSIST_WORKGROUPS", "0"))}


def run_persistent_vanilla_epoch(sess, cid: int, order: torch.Tensor) -> bool:
    """One vanilla epoch of a co-located Alice_cid as ONE launch (`_C.VanillaEpoch`,
    csrc/vanilla.hip).  Fail-safe: the Alice's and Bob's parameters and momentum buffers are
    copied first; if the launch fails they are restored, the persistent executor is switched
    off for the session (`split_persist_fallback`) and False is returned, so the caller runs
    the epoch on the per-batch executor instead."""
    cfg = _va_cfg(sess, cid)
    ex = sess.ops.C().VanillaEpoch(cfg)
    if not ex.ok():
        sess.__dict__["_va_off"] = True
        sess.__dict__["split_persist_reason"] = ex.why()
        return False
    a = sess.alices[cid]
    order = order.to(sess.device, torch.int64).contiguous()
    state = [L["W"] for L in cfg["layers"]] + [L["b"] for L in cfg["layers"]]
    state += [L["s0"] for L in cfg["layers"]] + [L["sb0"] for L in cfg["layers"]] + list(cfg["alice"].values())
    snap = [t.clone() for t in state] if getattr(sess.args, "persistent_failsafe", "on") != "off" else None
    B = sess.B
    nb = -(-int(order.numel()) // B)
    loss = torch.empty(max(nb, 1) * B, dtype=torch.float32, device=sess.device)
    sess.tail._pre = None
    if sess.__dict__.get("_va_max_steps"):
        ex.set_max_steps(int(sess._va_max_steps))      # tests: the epoch as several launches
    fault = sess.__dict__.pop("_va_fault_step", None)
    if fault is not None:
        ex.set_fault_step(int(fault))
    try:
        t_a, t_b, fc = ex.run(order, loss, a.slot.t, sess.bob_slot(cid).t, sess.tail.fwd_count, sess.tail.seed_base)
    except RuntimeError as e:
        if snap is None:
            raise
        for t, s in zip(state, snap):
            t.copy_(s)
        sess.__dict__["_va_off"] = True
        sess.__dict__["split_persist_fallback"] = str(e).splitlines()[0][:200]
        return False
    _count(sess, "persistent")
    a.slot.t = int(t_a)
    _bob_done(sess, cid, t_b, fc)
    sess.__dict__["last_split_losses"] = loss[:order.numel()]
    return True


# ---------------------------------------------------------------------- persistent U-shape epoch
def persistent_ushape_ok(sess, cid: int) -> bool:
    """Whether `run_persistent_ushape_epoch` may drive this epoch: the co-located native
    conditions, Adam on both sides, fp32 or bf16 compute (as --dtype), batches of at most 16 rows, the flag, and no
    earlier failure of the persistent executor in this session."""
    if getattr(sess.args, "split_persist", "auto") == "off" or sess.__dict__.get("_us_off"):
        return False
    if getattr(sess.comm, "host_staging", False):
        return False   # ranks share this GPU (--ranks_share_gpu): 256 co-resident workgroups are not assured
    if not native_split_ok(sess, cid, "ushape") or not hasattr(sess.ops.C(), "UShapeEpoch"):
        return False
    dt = getattr(sess.args, "dtype", "fp32")
    C = sess.ops.C()
    cdt = C.get_compute_dtype() if hasattr(C, "get_compute_dtype") else "fp32"
    if dt not in ("fp32", "bf16") or cdt != dt:
        # bf16 runs the kernel's bf16 instantiation (bf16 operands, fp32 state), but only when the
        # compute dtype the per-batch kernels use agrees with --dtype
        sess.__dict__["split_persist_reason"] = f"dtype {dt} with compute dtype {cdt}"
        return False
    a = sess.alices[cid]
    if not 1 <= sess.B <= 16:
        sess.__dict__["split_persist_reason"] = f"batch {sess.B} > 16: per-batch executor"
        return False
    return (a.slot.cfg.kind == "adam" and sess.bob_slot(cid).cfg.kind == "adam"
            and len(sess.tail.layers) == 2 and all(L.W.dtype == torch.float32 for L in sess.tail.layers))


def _six(slot, name: str, W: torch.Tensor, b: torch.Tensor) -> dict:
    sw, sb = slot.state(name + ".weight", W), slot.state(name + ".bias", b)
    return {"W": W, "m": sw["m"], "v": sw["v"], "b": b, "mb": sb["m"], "vb": sb["v"]}


def _adam(cfg) -> dict:
    return {"lr": cfg.lr, "beta1": cfg.beta1, "beta2": cfg.beta2, "eps": cfg.eps, "wd": cfg.weight_decay}


def _us_cfg(sess, cid: int) -> dict:
    a = sess.alices[cid]
    a.front.flush()
    w, b = a.front.params
    H = a.head.layers[0]
    bslot = sess.bob_slot(cid)
    L1, L2 = sess.tail.layers
    return {"fc1": _six(bslot, L1.spec.name, L1.W, L1.b), "fc2": _six(bslot, L2.spec.name, L2.W, L2.b),
            "conv": _six(a.slot, "front.conv", w, b), "head": _six(a.slot, f"head.{H.spec.name}", H.W, H.b),
            "bob_opt": _adam(bslot.cfg), "alice_opt": _adam(a.slot.cfg),
            "x": a.train.x, "y": a.train.y, "B": sess.B,
            "timeout_s": float(getattr(sess.args, "persist_timeout_s", 30.0)),
            "workgroups": int(os.environ.get("SL_PERSIST_WORKGROUPS", "0")),
            "bf16": getattr(sess.args, "dtype", "fp32") == "bf16"}


def run_persistent_ushape_epoch(sess, cid: int, order: torch.Tensor) -> bool:
    """One U-shape epoch of a co-located Alice_cid as ONE launch (`_C.UShapeEpoch`,
    csrc/ushape.hip: every parameter and Adam moment of model1 / model2 / model3 on-chip).
    Fail-safe as `run_persistent_vanilla_epoch`: parameters and moments are copied first; a
    failed launch restores them, switches the persistent executor off for the session
    (`split_persist_fallback`) and returns False, so the caller runs the epoch per batch."""
    cfg = _us_cfg(sess, cid)
    ex = sess.ops.C().UShapeEpoch(cfg)
    if not ex.ok():
        sess.__dict__["_us_off"] = True
        sess.__dict__["split_persist_reason"] = ex.why()
        return False
    a = sess.alices[cid]
    order = order.to(sess.device, torch.int64).contiguous()
    state = [t for k in ("fc1", "fc2", "conv", "head") for t in cfg[k].values()]
    snap = [t.clone() for t in state] if getattr(sess.args, "persistent_failsafe", "on") != "off" else None
    B = sess.B
    nb = -(-int(order.numel()) // B)
    loss = torch.empty(max(nb, 1) * B, dtype=torch.float32, device=sess.device)
    sess.tail._pre = None
    if sess.__dict__.get("_us_max_steps"):
        ex.set_max_steps(int(sess._us_max_steps))      # tests: the epoch as several launches
    fault = sess.__dict__.pop("_us_fault_step", None)
    if fault is not None:
        ex.set_fault_step(int(fault))
    try:
        t_a, t_b = ex.run(order, loss, a.slot.t, sess.bob_slot(cid).t)
    except RuntimeError as e:
        if snap is None:
            raise
        for t, s in zip(state, snap):
            t.copy_(s)
        sess.__dict__["_us_off"] = True
        sess.__dict__["split_persist_fallback"] = str(e).splitlines()[0][:200]
        return False
    _count(sess, "persistent")
    a.slot.t = int(t_a)
    _bob_done(sess, cid, t_b, sess.tail.fwd_count + nb)
    a.head.fwd_count += nb
    sess.__dict__["last_split_losses"] = loss[:order.numel()]
    return True


# ---------------------------------------------------------------------- remote placements
def _remote_placement_ok(sess, cid: int) -> bool:
    """Conditions every rank evaluates identically (placement, flags, the link): the Alice
    remote from a one-shard Bob, an fp32 wire, the native kernels, a split channel."""
    return (getattr(sess.args, "native_epoch", True) and sess.device.type == "cuda"
            and getattr(sess, "split_channel", None) is not None and sess.pl.bob_tp == 1
            and sess.host(cid) != sess.pl.bob_root and sess.act_dtype == torch.float32
            and hasattr(sess.ops, "C"))


def _remote_side_ok(sess, cid: int, mode: str) -> bool:
    """This rank's side of the pair can run natively (the same per-side rules as
    `native_split_ok`), including `_C.SplitEpoch`'s batch bound (csrc/split.cpp: 1..64 rows on
    every role), so a larger `--batch_size` keeps the Python loop instead of raising."""
    B = sess.B
    if not SPLIT_MIN_B <= B <= SPLIT_MAX_B:
        return False
    if sess.hosts(cid):
        a = sess.alices[cid]
        if a.front.frozen or a.train.x.dtype != torch.uint8:
            return False
        return mode == "vanilla" or (sess.head_fused(B) and a.head.head_step_ok(B))
    t = sess.tail
    if mode == "vanilla":
        return t.fused3_ok()
    return t.grouped_ok(B) and len(t.layers) == 2 and sess.head_fused(B)


def native_remote_role(sess, cid: int, mode: str):
    """Collective over the pair (the Alice's rank, Bob's): whether this epoch of a remote
    Alice runs on the native split executor.  Returns "alice" / "bob" on the pair's ranks
    when both sides agree, "skip" on every other rank (it moves nothing in this epoch either
    way), None when the Python loop runs it."""
    if not _remote_placement_ok(sess, cid):
        return None
    host, bob = sess.host(cid), sess.pl.bob_root
    if sess.rank not in (host, bob):
        return "skip"
    peer = bob if sess.rank == host else host
    mine = torch.tensor([1 if _remote_side_ok(sess, cid, mode) else 0], dtype=torch.int32, device=sess.device)
    theirs = torch.empty_like(mine)
    sess.comm.exchange([(mine, peer)], [(theirs, peer)])
    if int(mine.item()) and int(theirs.item()):
        return "alice" if sess.rank == host else "bob"
    return None


def persistent_remote_ok(sess, cid: int, mode: str) -> bool:
    """Bob's side only (the Alice's side is the same run_alice either way): whether Bob serves
    this remote Alice's epoch with ONE persistent launch that speaks the peer-mapped channel
    itself (`_C.VanillaEpoch.run_remote` / `_C.UShapeEpoch.run_remote`, csrc/vanilla.hip and
    csrc/ushape.hip REM).  Needs the peer-mapped channel (not RCCL), B <= 16, the flag, no
    earlier decline, vanilla: fp32 SGD-momentum; U-shape: Adam, fp32 or bf16 as the compute
    dtype; and a GPU of its own: with ranks sharing one GPU the Alice's kernels need CUs the
    launch would hold, so only an explicit reduced grid (SL_VA_REMOTE_G / SL_US_REMOTE_G, the
    one-GPU tests) runs there."""
    if mode not in ("vanilla", "ushape") or getattr(sess.args, "split_persist", "auto") == "off":
        return False
    if sess.__dict__.get("_va_rem_off" if mode == "vanilla" else "_us_rem_off"):
        return False
    ch = getattr(sess, "split_channel", None)
    C = sess.ops.C()
    if ch is None or not hasattr(ch, "host_error") or not hasattr(C, "VanillaEpoch" if mode == "vanilla" else "UShapeEpoch"):
        return False
    if getattr(sess.comm, "host_staging", False) and not os.environ.get("SL_VA_REMOTE_G" if mode == "vanilla" else "SL_US_REMOTE_G"):
        return False
    dt = getattr(sess.args, "dtype", "fp32")
    cdt = C.get_compute_dtype() if hasattr(C, "get_compute_dtype") else "fp32"
    t = sess.tail
    if not (1 <= sess.B <= 16 and t.tp_size == 1 and all(L.W.dtype == torch.float32 for L in t.layers)):
        return False
    if mode == "vanilla":
        return dt == "fp32" and cdt == "fp32" and sess.bob_slot(cid).cfg.kind == "sgd" and len(t.layers) == 3
    return dt in ("fp32", "bf16") and cdt == dt and sess.bob_slot(cid).cfg.kind == "adam" and len(t.layers) == 2


def _run_remote_persistent_ushape(sess, cid: int, n: int, peer: int):
    """Bob's half of a remote U-shape epoch as one persistent launch (`_C.UShapeEpoch.run_remote`),
    as `_run_remote_persistent` for vanilla."""
    bslot = sess.bob_slot(cid)
    L1, L2 = sess.tail.layers
    cfg = {"fc1": _six(bslot, L1.spec.name, L1.W, L1.b), "fc2": _six(bslot, L2.spec.name, L2.W, L2.b),
           "bob_opt": _adam(bslot.cfg), "B": sess.B,
           "timeout_s": float(getattr(sess.args, "persist_timeout_s", 30.0)),
           "channel": sess.split_channel, "peer": int(peer),
           "G": int(os.environ.get("SL_US_REMOTE_G", "256")),
           "workgroups": int(os.environ.get("SL_PERSIST_WORKGROUPS", "0")),
           "bf16": getattr(sess.args, "dtype", "fp32") == "bf16"}
    ex = sess.ops.C().UShapeEpoch(cfg)
    if not ex.ok():
        sess.__dict__["_us_rem_off"] = True
        sess.__dict__["split_persist_reason"] = "remote: " + ex.why()
        return None
    sess.tail._pre = None
    t_b = ex.run_remote(int(n), bslot.t)
    _bob_done(sess, cid, t_b, sess.tail.fwd_count + -(-int(n) // sess.B))
    _count(sess, "remote_persistent")
    return ex


def _run_remote_persistent(sess, cid: int, n: int, peer: int, mode: str = "vanilla"):
    """Bob's half of a remote vanilla epoch as one persistent launch; None when the executor
    declines this configuration (the caller then runs run_bob, which Alice cannot tell apart).
    A launch that fails mid-epoch raises: the Alice is then stopped at a message of this epoch
    and times out on her side, so there is no state both sides could roll back to (fail-stop,
    docs/DEVIATIONS.md)."""
    if mode == "ushape":
        return _run_remote_persistent_ushape(sess, cid, n, peer)
    bslot = sess.bob_slot(cid)
    layers = []
    for L in sess.tail.layers:
        pw, pb = _param(bslot, f"{L.spec.name}.weight", L.W), _param(bslot, f"{L.spec.name}.bias", L.b)
        layers.append({"W": pw["p"], "b": pb["p"], "s0": pw["s0"], "sb0": pb["s0"]})
    bo = bslot.cfg
    cfg = {"layers": layers, "lr": bo.lr, "momentum": bo.momentum, "wd": bo.weight_decay, "B": sess.B,
           "p1": sess.tail.layers[0].spec.dropout, "p2": sess.tail.layers[1].spec.dropout,
           "timeout_s": float(getattr(sess.args, "persist_timeout_s", 30.0)),
           "channel": sess.split_channel, "peer": int(peer),
           "G": int(os.environ.get("SL_VA_REMOTE_G", "256")),
           "workgroups": int(os.environ.get("SL_PERSIST_WORKGROUPS", "0"))}
    ex = sess.ops.C().VanillaEpoch(cfg)
    if not ex.ok():
        sess.__dict__["_va_rem_off"] = True
        sess.__dict__["split_persist_reason"] = "remote: " + ex.why()
        return None
    nb = -(-int(n) // sess.B)
    loss = torch.empty(max(nb, 1) * sess.B, dtype=torch.float32, device=sess.device)
    sess.tail._pre = None
    t_b, fc = ex.run_remote(int(n), loss, bslot.t, sess.tail.fwd_count, sess.tail.seed_base)
    _bob_done(sess, cid, t_b, fc)
    sess.__dict__["last_split_losses"] = loss[:int(n)]
    _count(sess, "remote_persistent")
    return ex


def run_native_remote_epoch(sess, cid: int, order, n: int, mode: str, role: str):
    """This rank's half of one split epoch of a remote Alice_cid (`_C.SplitEpoch` roles 1 / 2,
    csrc/split.cpp run_alice / run_bob): the per-batch messages go over `sess.split_channel`
    on the compute stream.  Same launches and step counts as the Python loop of this
    placement (the §3.2 overlap order: no look-ahead).  Bob's side of a vanilla epoch runs as
    ONE persistent launch when `persistent_remote_ok` (the same messages, from inside it)."""
    if role == "skip":
        return None
    _count(sess, "remote_" + role)
    C = sess.ops.C()
    host, bob = sess.host(cid), sess.pl.bob_root
    cfg = {"mode": 1 if mode == "vanilla" else 2, "B": sess.B, "channel": sess.split_channel}
    comm = sess.comm
    comm.progress()
    ex = _run_remote_persistent(sess, cid, n, host, mode) if role == "bob" and persistent_remote_ok(sess, cid, mode) else None
    if ex is not None:
        pass                      # Bob's side ran as one persistent launch
    elif role == "alice":
        a = sess.alices[cid]
        cfg.update(_alice_cfg(sess, cid, mode))
        cfg.update({"role": 1, "peer": bob})
        ex = C.SplitEpoch(cfg)
        order = order.to(sess.device, torch.int64).contiguous()
        a.slot.t = int(ex.run_alice(order, a.slot.t))
        if a.head is not None:
            a.head.fwd_count += -(-int(order.numel()) // sess.B)
    else:
        cfg.update(_bob_cfg(sess, cid, mode))
        cfg.update({"role": 2, "peer": host})
        ex = C.SplitEpoch(cfg)
        sess.tail._pre = None
        t_b, fc = ex.run_bob(int(n), sess.bob_slot(cid).t, sess.tail.fwd_count, sess.tail.seed_base)
        _bob_done(sess, cid, t_b, fc)
    for op, peer, nb in ex.messages():
        if op == "send":
            comm.bytes_sent += nb
            comm.msgs_sent += 1
            if comm.msg_log is not None:
                comm.msg_log.append(("native_send", comm.rank, peer, nb))
    comm.progress()
    return ex
