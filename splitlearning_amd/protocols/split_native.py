"""Native split-mode epochs: a vanilla / U-shape `split_epoch` issued from C++
(`_C.SplitEpoch`, csrc/split.cpp) when the Alice and the whole Bob (TP = 1) live in this
process — the one-GPU BASELINE point (ws = 2) and every co-located placement.

The executor issues the same launches, with the same arguments, dropout seeds, workspaces
and optimizer step counts, as `VanillaSession.split_epoch` / `UShapeSession.split_epoch` in
their look-ahead order, so the parameters it produces are bit-identical to the Python
loop's (tests/test_split_native_gpu.py); the Python loop
stays the path for every other placement and for `--python_epoch`.

Reference hot loops: data_entities_vanilla.py:66-76 and data_entities.py:65-81.
"""
from __future__ import annotations

import torch

_KIND = {"sgd": 1, "adam": 2}


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


def run_native_split_epoch(sess, cid: int, order: torch.Tensor, mode: str):
    """One split epoch of Alice_cid over `order` through `_C.SplitEpoch`."""
    a = sess.alices[cid]
    tail = sess.tail
    ops, dev = sess.ops, sess.device
    B = sess.B
    a.front.flush()
    w, b = a.front.params
    pre = "front." if mode == "ushape" else ""
    bslot = sess.bob_slot(cid)
    layers = []
    for L in tail.layers:
        layers.append({"w": _param(bslot, f"{L.spec.name}.weight", L.W),
                       "b": _param(bslot, f"{L.spec.name}.bias", L.b)})
    N2 = tail.layers[1].W.shape[0]
    nmax = max(L.W.shape[0] for L in tail.layers)
    kmax = max(L.W.shape[1] for L in tail.layers)
    cfg = {"mode": 1 if mode == "vanilla" else 2, "B": B, "x": a.train.x, "y": a.train.y,
           "front": {"w": _param(a.slot, pre + "conv.weight", w), "b": _param(a.slot, pre + "conv.bias", b)},
           "front_opt": _opt(a.slot.cfg), "bob_opt": _opt(bslot.cfg), "tail": layers,
           "p1": tail.layers[0].spec.dropout, "p2": tail.layers[1].spec.dropout,
           # the Python path's own workspaces (ops/hip_ops.py), so every split factor matches
           "fwdws": ops._workspace(dev, 16 * B * nmax, "fwd"),
           "dgws": ops._workspace(dev, 16 * B * kmax, "dgrad")}
    if mode == "vanilla":
        C3 = tail.layers[2].W.shape[0]
        cfg["p2ws"] = ops._workspace(dev, 16 * B * N2, "fc2p")
        cfg["headws"] = ops._workspace(dev, ops.C().head3_slices(N2) * B * C3, "head")
    else:
        H = a.head.layers[0]
        cfg["head"] = {"w": _param(a.slot, f"head.{H.spec.name}.weight", H.W),
                       "b": _param(a.slot, f"head.{H.spec.name}.bias", H.b)}
    ex = ops.C().SplitEpoch(cfg)
    order = order.to(dev, torch.int64).contiguous()
    tail._pre = None
    t_a, t_b, fc = ex.run(order, a.slot.t, bslot.t, tail.fwd_count, tail.seed_base)
    nb = -(-int(order.numel()) // B)
    a.slot.t, bslot.t, tail.fwd_count = int(t_a), int(t_b), int(fc)
    if a.head is not None:
        a.head.fwd_count += nb
    tail.acts, tail.dz, tail._wg = [], [], []
    return ex
