"""Golden tests of the U-shape and SISA-concat PRODUCTION paths against fp32 eager PyTorch.

* U-shape (`UShapeSession.split_epoch`: Alice's conv front with the deferred in-kernel
  update, Bob's `model2` middle with its per-Alice Adam slot, Alice's fused head step
  `_C.head_step` that also applies Bob's final ReLU mask, the grouped wgrad + Adam) against
  the composed reference `model1` -> `model2` -> `model3` trained by ONE Adam over all three
  (data_entities.py:43-47,65-81);
* SISA-concat (`ConcatSession.concat_epoch`: the epoch-wide [rows, 5408 k] layout, the k-head
  cross-entropy pinned in protocols/concat.py, the grouped wgrad + Adam with the fc1
  look-ahead) against `model2_sisa_concat(k)` (models.py:66-82) trained by
  `torch.optim.Adam(lr, weight_decay=1e-5)`, k = 2 and 4, uneven client shards.

Per-step tests re-synchronise torch with the engine (weights, Adam moments, step counts)
before every step and then require one step of both to agree (`_step_close`: rounding-level
except the rare element whose gradient is ~0, where Adam's m / sqrt(v) sign is rounding
noise, <= 2 lr).  Free-running multi-step tests (the look-ahead pipelines, which reorder work
across steps) use the `_close_adam` bound over the run: <= 2 lr per step, and all but a
small fraction of elements at rounding level.
"""
import copy

import pytest
import torch
import torch.nn.functional as F

from splitlearning_amd.ops import rng

pytestmark = pytest.mark.gpu


def _close_adam(a, b, lr, steps, frac=1e-3, tol=1e-4, msg=""):
    d = (a.float() - b.float()).abs()
    assert d.max().item() <= 2 * lr * steps + 1e-6, (msg, d.max().item())
    assert (d > tol).float().mean().item() < frac, (msg, (d > tol).float().mean().item(), d.max().item())


def _step_close(e, p, lr, msg, frac=1e-3, tol=1e-5):
    d = (e.float() - p.detach().float()).abs()
    assert d.max().item() <= 2 * lr + 1e-6, (msg, d.max().item())
    assert (d > tol).float().mean().item() < frac, (msg, (d > tol).float().mean().item(), d.max().item())


def _set_adam(opt, p, st, t):
    opt.state[p] = {"step": torch.tensor(float(t)), "exp_avg": st["m"].clone().view_as(p),
                    "exp_avg_sq": st["v"].clone().view_as(p)}


def _moments_close(opt, p, st, msg):
    for k, tk in (("m", "exp_avg"), ("v", "exp_avg_sq")):
        ref = opt.state[p][tk]
        torch.testing.assert_close(st[k].view_as(ref), ref, rtol=1e-3, atol=1e-5 * ref.abs().max().item() + 1e-30,
                                   msg=f"{msg} {k}")


# ------------------------------------------------------------------------------------ U-shape
def _ushape_session(tmp_path, cuda, num_samples=2000):
    from splitlearning_amd.config import parse_args
    from splitlearning_amd.data.mnist import write_shards
    from splitlearning_amd.parallel.dist import Comm, Placement
    from splitlearning_amd.protocols import UShapeSession
    args = parse_args(["--world_size", "2", "--seed", "7", "--num_samples", str(num_samples), "--no_tqdm",
                       "--datapath", str(tmp_path / "d"), "--log_dir", str(tmp_path / "logs")])
    write_shards(args, verbose=False)
    return UShapeSession(args, Comm(0, 1, cuda, Placement.make(2, 1, 1)), cuda)


class _UShapeRef:
    """model1 -> model2 -> model3 in eager torch with one Adam over all of them."""

    def __init__(self, sess, cuda):
        a = sess.alices[1]
        self.sess, self.a = sess, a
        self.front = copy.deepcopy(a.front.module).to(cuda)
        self.mid = copy.deepcopy(sess.tail.module).to(cuda)
        self.head = copy.deepcopy(a.head.module).to(cuda)
        self.lr = sess.args.lr
        self.opt = torch.optim.Adam(list(self.front.parameters()) + list(self.mid.parameters())
                                    + list(self.head.parameters()), lr=self.lr)

    def _pairs(self):
        """(torch param, engine tensor, optimizer-state dict, engine step count) for every
        parameter of the three parts."""
        sess, a = self.sess, self.a
        bslot = sess.bob_slot(1)
        out = []
        for (name, p), (_, e) in zip(self.front.named_parameters(), a.front.module.named_parameters()):
            out.append((p, e, a.slot.states.get("front.conv." + name.split(".")[-1]), a.slot.t, f"front.{name}"))
        for name, p in self.mid.named_parameters():
            L = sess.tail.layers[int(name[2]) - 1]
            out.append((p, L.W if name.endswith("weight") else L.b, bslot.states.get(name), bslot.t, f"bob.{name}"))
        for name, p in self.head.named_parameters():
            L = a.head.layers[0]
            out.append((p, L.W if name.endswith("weight") else L.b, a.slot.states.get("head." + name), a.slot.t,
                        f"head.{name}"))
        return out

    def sync(self):
        with torch.no_grad():
            for p, e, st, t, _ in self._pairs():
                p.copy_(e.view_as(p))
                if st is not None:
                    _set_adam(self.opt, p, st, t)
                else:
                    self.opt.state.pop(p, None)

    def step(self, idx):
        a = self.a
        self.opt.zero_grad()
        logits = self.head(self.mid(self.front(a.train.x_float(idx))))
        loss = F.cross_entropy(logits, a.train.y[idx])
        loss.backward()
        self.opt.step()
        return loss.detach()


def test_ushape_split_epoch_matches_composed_torch_adam_every_step(cuda, tmp_path):
    """The U-shape split epoch, one batch per call, 30 batches + a partial one, against one
    torch Adam over model1 + model2 + model3, re-synchronised before every batch: every
    parameter and Adam moment of all three parts must agree after each step."""
    sess = _ushape_session(tmp_path, cuda)
    a = sess.alices[1]
    ref = _UShapeRef(sess, cuda)
    order = a.train.shuffled_order(torch.Generator().manual_seed(3))[:16 * 30 + 7]
    n = order.numel()
    for i, s in enumerate(range(0, n, 16)):
        idx = order[s:s + 16]
        ref.sync()
        ref.step(idx)
        sess.split_epoch(1, idx, idx.numel())          # one batch of the production U-shape epoch
        for p, e, st, _, name in ref._pairs():
            _step_close(e.view_as(p), p, ref.lr, f"batch {i} {name}")
            _moments_close(ref.opt, p, st, f"batch {i} {name}")
    torch.cuda.synchronize()
    assert sess.bob_slot(1).t == a.slot.t == -(-n // 16)
    # every batch above ran as a one-step launch of the persistent U-shape epoch (csrc/ushape.hip,
    # the co-located default), so this pins that kernel to torch at every step
    assert sess.native_split_epochs.get("persistent") == -(-n // 16), (
        sess.native_split_epochs, sess.__dict__.get("split_persist_reason"), sess.__dict__.get("split_persist_fallback"))


def test_ushape_lookahead_epoch_free_running_matches_torch(cuda, tmp_path):
    """The pipelined U-shape epoch over 12 batches in ONE call (Bob's update of batch i issued
    after Alice's forward of batch i+1, with the fc1 look-ahead; Alice's deferred update)
    against 12 free-running torch Adam steps from the same start: within the Adam bound."""
    sess = _ushape_session(tmp_path, cuda)
    a = sess.alices[1]
    ref = _UShapeRef(sess, cuda)
    steps = 12
    order = a.train.shuffled_order(torch.Generator().manual_seed(4))[:16 * steps]
    ref.sync()
    for i in range(steps):
        ref.step(order[16 * i:16 * (i + 1)])
    sess.split_epoch(1, order, order.numel())
    torch.cuda.synchronize()
    for p, e, _, _, name in ref._pairs():
        _close_adam(e.view_as(p), p.detach(), ref.lr, steps, msg=name)


# ------------------------------------------------------------------------------------ concat
def _concat_session(tmp_path, cuda, k):
    from splitlearning_amd.config import parse_args
    from splitlearning_amd.data.mnist import write_shards
    from splitlearning_amd.parallel.dist import Comm, Placement
    from splitlearning_amd.protocols import ConcatSession
    args = parse_args(["--sisa", "--concat", "--world_size", str(k + 1), "--seed", "11", "--num_samples", "1500",
                       "--no_tqdm", "--datapath", str(tmp_path / "d"), "--log_dir", str(tmp_path / "logs")])
    write_shards(args, verbose=False)
    return ConcatSession(args, Comm(0, 1, cuda, Placement.make(k + 1, 1, 1)), cuda)


def _concat_caches(cuda, k, B, ns, seed):
    g = torch.Generator().manual_seed(seed)
    return [((torch.rand(n, 5408, generator=g) * 10).to(cuda), torch.randint(0, 10, (n,), generator=g).to(cuda))
            for n in ns]


def _concat_ref_step(ref, opt, caches, t, B, k, seed_base, step):
    """One reference server step: row b = [act_1[b] | ... | act_k[b]] (zeros past a client's
    rows), loss = sum_j mean-over-client-j's-rows CE(logits[:, 100 j : 100 j + 100], y_j)."""
    rows = [max(0, min(B, c[1].numel() - t * B)) for c in caches]
    M = max(rows)
    dev = caches[0][0].device
    X = torch.zeros(M, 5408 * k, device=dev)
    for j, ((acts, _), r) in enumerate(zip(caches, rows)):
        X[:r, 5408 * j:5408 * (j + 1)] = acts[t * B:t * B + r]
    h = X
    for i, lin in enumerate(ref.linears()):
        ls = ref.spec.layers[i]
        h = F.linear(h, lin.weight, lin.bias)
        if ls.relu:
            h = F.relu(h)
        if ls.dropout:
            keep = rng.keep_mask(rng.step_seed(seed_base, i, step), h.shape[0], h.shape[1], ls.dropout, device=dev)
            h = h * keep / (1 - ls.dropout)
    loss = 0.0
    for j, ((_, labels), r) in enumerate(zip(caches, rows)):
        if r:
            loss = loss + F.cross_entropy(h[:r, 100 * j:100 * (j + 1)], labels[t * B:t * B + r])
    opt.zero_grad()
    loss.backward()
    opt.step()
    return M


@pytest.mark.parametrize("k", [2, 4])
def test_concat_epoch_matches_torch_adam_every_step(cuda, tmp_path, k):
    """`concat_epoch`, one step per call (a one-batch slice of every client's cache), against
    `model2_sisa_concat(k)` with `torch.optim.Adam(lr, weight_decay=1e-5)` re-synchronised
    before every step.  Uneven shards: clients run out at different steps, and the last batch
    of each is partial, so the k-head CE's per-client row counts and the zero-padded slots are
    exercised."""
    sess = _concat_session(tmp_path, cuda, k)
    B = sess.B
    ns = [B * 5 + 3, B * 3 + 11, B * 6, B * 2 + 1][:k]
    caches = _concat_caches(cuda, k, B, ns, seed=k)
    T = max(-(-n // B) for n in ns)
    tail, slot = sess.tail, sess.bob_slot
    lr = sess.args.lr
    ref = copy.deepcopy(tail.module).to(cuda)
    opt = torch.optim.Adam(ref.parameters(), lr=lr, weight_decay=1e-5)
    for t in range(T):
        with torch.no_grad():
            for name, p in ref.named_parameters():
                L = tail.layers[int(name[2]) - 1]
                p.copy_(L.W if name.endswith("weight") else L.b)
                st = slot.states.get(name)
                if st is not None:
                    _set_adam(opt, p, st, slot.t)
                else:
                    opt.state.pop(p, None)
        step = tail.fwd_count + 1
        _concat_ref_step(ref, opt, caches, t, B, k, tail.seed_base, step)
        one = [(acts[t * B:(t + 1) * B], labels[t * B:(t + 1) * B]) for acts, labels in caches]
        sess.concat_epoch(one)
        for name, p in ref.named_parameters():
            L = tail.layers[int(name[2]) - 1]
            _step_close(L.W if name.endswith("weight") else L.b, p, lr, f"k={k} step {t} {name}")
            _moments_close(opt, p, slot.states[name], f"k={k} step {t} {name}")
    assert slot.t == T and tail.fwd_count == T


def test_concat_lookahead_epoch_free_running_matches_torch(cuda, tmp_path):
    """`concat_epoch` over a whole uneven epoch in one call (the fc1 look-ahead pipeline,
    k = 2) against free-running torch Adam steps from the same start: within the Adam bound."""
    k = 2
    sess = _concat_session(tmp_path, cuda, k)
    B = sess.B
    ns = [B * 6 + 5, B * 4 + 2]
    caches = _concat_caches(cuda, k, B, ns, seed=9)
    T = max(-(-n // B) for n in ns)
    tail = sess.tail
    lr = sess.args.lr
    ref = copy.deepcopy(tail.module).to(cuda)
    opt = torch.optim.Adam(ref.parameters(), lr=lr, weight_decay=1e-5)
    f0 = tail.fwd_count
    for t in range(T):
        _concat_ref_step(ref, opt, caches, t, B, k, tail.seed_base, f0 + t + 1)
    sess.concat_epoch(caches)
    torch.cuda.synchronize()
    for name, p in ref.named_parameters():
        L = tail.layers[int(name[2]) - 1]
        _close_adam(L.W if name.endswith("weight") else L.b, p.detach(), lr, T, msg=name)
