"""Schedule-step snapshots and exact resume (`--ckpt_dir`, `--resume`).

The reference has no checkpointing at all: a crashed rank ends the job
(`mp.spawn(join=True)`, §5.3) and everything trained so far is lost.  Here every rank
writes, after each top-level step of the Bob schedule (`protocols/schedule.py`), the
complete mutable state it owns, so a job killed at any point (the watchdog's abort, a
lost node, `--fault_inject`) is restarted with `--resume` and continues from the last
completed step with results bitwise equal to an uninterrupted run
(`tests/test_distributed_cpu.py::test_crash_and_resume_matches_uninterrupted`).

Per rank (`<ckpt_dir>/step<k>/rank<r>.pt`, loadable with `torch.load(weights_only=True)`):
* Bob's local tail shard (every TP rank its own), his optimizer slots (per-Alice Adam /
  SGD-m state and step counters), the forward counter that keys the dropout
  hash, train/eval mode, and the SISA activation cache with its keys (the
  retrain phase reuses untouched clients' cached activations, so they are state);
* each hosted Alice's front (and U-shape head) weights, optimizer slot, shuffle
  generator state, unlearn order and frozen flag;
* the session's round-robin position (`last_alice_id`).
A snapshot is complete when rank 0 has written `step<k>/DONE` after a barrier; `latest`
names the newest complete one.  Placement must match on resume (same mode, world size,
process count, TP degree and seed) — it is checked.
"""
from __future__ import annotations

import os
import shutil

import torch

VERSION = 1


def _cpu(t):
    return None if t is None else t.detach().to("cpu").clone()


def _slot_state(slot) -> dict:
    return {"kind": slot.cfg.kind, "t": int(slot.t),
            "states": {n: {k: _cpu(v) for k, v in st.items()} for n, st in slot.states.items()}}


def _load_slot(slot, d: dict, device):
    if d["kind"] != slot.cfg.kind:
        raise ValueError(f"snapshot optimizer kind {d['kind']} != {slot.cfg.kind}")
    slot.t = int(d["t"])
    for n, st in d["states"].items():
        have = slot.states.get(n)
        if have is None:
            slot.states[n] = {k: v.to(device).contiguous() for k, v in st.items()}
        else:                         # keep tensors that executors may already point at
            for k, v in st.items():
                have[k].copy_(v)


def _meta(sess) -> dict:
    a = sess.args
    return {"version": VERSION, "mode": sess.mode, "world_size": int(a.world_size), "nprocs": int(sess.comm.world),
            "bob_tp": int(sess.pl.bob_tp), "seed": int(sess.seed), "rank": int(sess.rank)}


def rank_state(sess) -> dict:
    """Everything this rank owns that a later schedule step reads."""
    st = {"meta": _meta(sess), "last_alice_id": sess.last_alice_id, "bob": None, "alices": {}}
    if sess.tail is not None:
        t = sess.tail
        st["bob"] = {
            "layers": [(_cpu(L.W), _cpu(L.b)) for L in t.layers],
            "fwd_count": int(t.fwd_count), "training": bool(t.training),
            "slots": [(k, _slot_state(s)) for k, s in sess.bob_slots.items()],
            # the SISA activation cache is identical on every Bob TP rank: only the root
            # writes it (one copy per snapshot instead of bob_tp copies); resume multicasts it
            "cache": ([(list(k), _cpu(v[0]), _cpu(v[1])) for k, v in sess.activation_and_labels_cache.items()]
                      if sess.rank == sess.pl.bob_root else None),
        }
    st["cache_keys"] = [list(k) for k in sorted(getattr(sess, "_ck", set()), key=repr)]
    for cid, a in sess.alices.items():
        st["alices"][cid] = {
            "front": {k: _cpu(v) for k, v in a.front.module.state_dict().items()},
            "head": None if a.head is None else [(_cpu(L.W), _cpu(L.b)) for L in a.head.layers],
            "head_fwd_count": None if a.head is None else int(a.head.fwd_count),
            "slot": _slot_state(a.slot),
            "gen": a.gen.get_state(),
            "unlearn_order": _cpu(a.unlearn_order),
            "frozen": bool(a.front.frozen),
        }
    return st


def load_rank_state(sess, st: dict):
    want, got = _meta(sess), st["meta"]
    for k in ("version", "mode", "world_size", "nprocs", "bob_tp", "seed", "rank"):
        if want[k] != got[k]:
            raise ValueError(f"snapshot {k}={got[k]!r} does not match this job's {want[k]!r}")
    dev = sess.device
    sess.last_alice_id = st["last_alice_id"]
    b = st["bob"]
    if (b is None) != (sess.tail is None):
        raise ValueError("snapshot Bob placement does not match")
    if b is not None:
        t = sess.tail
        with torch.no_grad():
            for L, (W, bias) in zip(t.layers, b["layers"]):
                L.W.copy_(W)
                L.b.copy_(bias)
        t.fwd_count = b["fwd_count"]
        t.training = b["training"]
        t._pre = None
        for key, d in b["slots"]:
            if key not in sess.bob_slots:
                from ..engine.slots import OptSlot
                sess.bob_slots[key] = OptSlot(sess.bob_optim())
            _load_slot(sess.bob_slots[key], d, dev)
        sess.activation_and_labels_cache.clear()
        if b["cache"] is not None:
            for key, acts, labels in b["cache"]:
                sess.activation_and_labels_cache[tuple(key)] = (acts.to(dev), labels.to(dev))
    _share_cache(sess, b)
    if st["cache_keys"] or hasattr(sess, "_ck"):
        sess._ck = {tuple(k) for k in st["cache_keys"]}
    for cid, d in st["alices"].items():
        a = sess.alices[int(cid)]
        a.front.module.load_state_dict({k: v.to(dev) for k, v in d["front"].items()})
        if d["head"] is not None:
            with torch.no_grad():
                for L, (W, bias) in zip(a.head.layers, d["head"]):
                    L.W.copy_(W)
                    L.b.copy_(bias)
            a.head.fwd_count = d["head_fwd_count"]
        from ..engine.slots import OptSlot
        a.slot = OptSlot(sess.alice_optim())
        _load_slot(a.slot, d["slot"], dev)
        a.gen.set_state(d["gen"])
        a.unlearn_order = None if d["unlearn_order"] is None else d["unlearn_order"].to(dev)
        a.front.frozen = d["frozen"]


def _share_cache(sess, b):
    """Collective over all ranks: the Bob root sends its restored activation cache to the
    other Bob TP ranks (every rank learns the key order and shapes from the root)."""
    if not sess.comm.distributed or sess.pl.bob_tp <= 1:
        return
    root = sess.pl.bob_root
    meta = None
    if sess.rank == root:
        meta = [(tuple(k), tuple(v[0].shape), str(v[0].dtype).split(".")[-1], int(v[1].numel()))
                for k, v in sess.activation_and_labels_cache.items()]
    meta = sess.comm.broadcast_obj(meta, root)
    others = [r for r in sess.pl.bob_ranks if r != root]
    for key, shape, dt, n in meta:
        acts = labels = None
        if sess.rank == root:
            acts, labels = sess.activation_and_labels_cache[key]
        acts = sess.comm.multicast(acts, root, others, shape, getattr(torch, dt))
        labels = sess.comm.multicast(labels, root, others, (n,), torch.int64)
        if sess.rank in others:
            sess.activation_and_labels_cache[key] = (acts, labels)


def _step_dir(root: str, k: int) -> str:
    return os.path.join(root, f"step{k:04d}")


def save(sess, root: str, k: int, name: str, keep: int = 2):
    """Collective: every rank writes its state for 'after step k'; rank 0 marks it complete."""
    d = _step_dir(root, k)
    os.makedirs(d, exist_ok=True)
    if sess.device.type == "cuda":
        torch.cuda.synchronize(sess.device)
    path = os.path.join(d, f"rank{sess.rank}.pt")
    torch.save(rank_state(sess), path + ".tmp")
    os.replace(path + ".tmp", path)
    sess.comm.barrier()
    if sess.rank == 0:
        with open(os.path.join(d, "DONE"), "w") as f:
            f.write(f"{k} {name}\n")
        with open(os.path.join(root, "latest.tmp"), "w") as f:
            f.write(str(k))
        os.replace(os.path.join(root, "latest.tmp"), os.path.join(root, "latest"))
        for old in sorted(x for x in os.listdir(root) if x.startswith("step")):
            j = int(old[4:])
            if j <= k - max(1, keep):
                shutil.rmtree(os.path.join(root, old), ignore_errors=True)
    sess.comm.barrier()


def latest(root: str) -> int:
    """Newest complete snapshot index in `root` (0 = none)."""
    try:
        with open(os.path.join(root, "latest")) as f:
            k = int(f.read().strip())
    except (OSError, ValueError):
        return 0
    return k if os.path.exists(os.path.join(_step_dir(root, k), "DONE")) else 0


def load(sess, root: str) -> int:
    """Collective: load this rank's part of the newest complete snapshot; returns the
    number of completed schedule steps (0 = start from the beginning)."""
    k = int(sess.comm.broadcast_obj(latest(root) if sess.rank == 0 else None, 0))
    if k == 0:
        return 0
    st = torch.load(os.path.join(_step_dir(root, k), f"rank{sess.rank}.pt"), weights_only=True)
    load_rank_state(sess, st)
    sess.comm.barrier()
    return k
