"""Golden tests on the GPU: the PRODUCTION fused paths against fp32 eager PyTorch.

* the native SISA server epoch (`_C.ServerEpoch`: fc1 look-ahead inside the fused
  wgrad+Adam kernel, 128 optimizer steps) against `model2_sisa` trained by
  `torch.optim.Adam(lr, weight_decay=1e-5)` (data_entities_vanilla_sisa.py:266,305-313);
* the vanilla `split_epoch` (the persistent vanilla epoch, csrc/vanilla.hip, one launch per
  batch here) against the
  composed `model1_sisa` + `model2_sisa` with two `torch.optim.SGD(momentum=0.9)`
  (data_entities_vanilla.py:37-42,66-76).
Dropout masks are the framework's counter hash (`ops/rng.keep_mask`), regenerated for the
reference from the same (seed, layer, step).  Bounds follow the CPU golden tests'
`assert_adam_close` form: Adam normalises each update, so an element whose gradient is ~0
moves by up to lr per step on rounding noise; everything else must agree closely.
"""
import copy

import pytest
import torch
import torch.nn.functional as F

from splitlearning_amd.engine import OptSlot, TailEngine, adam
from splitlearning_amd.models import ClientFrontSisa, ServerTailSisa, sisa_server_spec
from splitlearning_amd.ops import rng

pytestmark = pytest.mark.gpu


def _ref_tail_forward(mod, x, seed_base, step):
    h = x
    lins = mod.linears()
    for i, lin in enumerate(lins):
        ls = mod.spec.layers[i]
        h = F.linear(h, lin.weight, lin.bias)
        if ls.relu:
            h = F.relu(h)
        if ls.dropout:
            keep = rng.keep_mask(rng.step_seed(seed_base, i, step), h.shape[0], h.shape[1], ls.dropout,
                                 device=h.device)
            h = h * keep / (1 - ls.dropout)
    return h


def _close_adam(a, b, lr, steps, frac=1e-3, tol=1e-4, msg=""):
    d = (a.float() - b.float()).abs()
    assert d.max().item() <= 2 * lr * steps + 1e-6, (msg, d.max().item())
    assert (d > tol).float().mean().item() < frac, (msg, (d > tol).float().mean().item(), d.max().item())


def _load_adam(ref, opt, te, slot, t):
    """torch model + Adam state := the engine's weights, moments and step count."""
    with torch.no_grad():
        for name, p in ref.named_parameters():
            L = te.layers[int(name[2]) - 1]
            p.copy_(L.W if name.endswith("weight") else L.b)
            st = slot.states[name]
            opt.state[p] = {"step": torch.tensor(float(t)), "exp_avg": st["m"].clone(),
                            "exp_avg_sq": st["v"].clone()}


@pytest.mark.parametrize("scale,B", [(1.0, 16), (30.0, 16), (1.0, 64)])
def test_sisa_server_epoch_matches_torch_adam_every_step(cuda, scale, B):
    """The production SISA server epoch (fused fwd/dgrad kernels, fc1 look-ahead inside the
    wgrad+Adam kernel), 128 steps, checked against `torch.optim.Adam(lr, weight_decay=1e-5)`
    on `model2_sisa` at EVERY step: before step i torch is given the engine's weights, Adam
    moments and step count, takes step i on the same batch with the same dropout masks, and
    both post-step states and the step's losses must agree.  (Free-running fp32 trajectories of
    this random-label training are chaotic — any summation-order change grows to O(1) loss
    gaps within ~30 steps, measured — so per-step re-synchronisation is what makes a tight
    128-step comparison possible.)  The run is also the native executor's: its free-running
    128-step result must be bitwise the per-step Python path's."""
    steps, lr, seed_base = 128 if B == 16 else 48, 1e-3, 99
    g = torch.Generator().manual_seed(21)
    n = B * steps
    acts = (torch.rand(n, 5408, generator=g) * scale).to(cuda)
    labels = torch.randint(0, 10, (n,), generator=g).to(cuda)
    torch.manual_seed(4)
    base = ServerTailSisa()
    # the native executor, free-running
    nat = TailEngine(copy.deepcopy(base), sisa_server_spec(), cuda, seed_base=seed_base, ws_tag="#nat")
    nslot = OptSlot(adam(lr, 1e-5))
    nat.lookahead_prologue(acts[:B])
    loss_nat = nat.run_native_epoch(acts, labels, nslot, B, True)
    # the same kernels step by step, with torch re-synchronised before every step
    te = TailEngine(copy.deepcopy(base), sisa_server_spec(), cuda, seed_base=seed_base)
    slot = OptSlot(adam(lr, 1e-5))
    for L in te.layers:
        slot.state(f"{L.spec.name}.weight", L.W)
        slot.state(f"{L.spec.name}.bias", L.b)
    ref = copy.deepcopy(base).to(cuda)
    opt = torch.optim.Adam(ref.parameters(), lr=lr, weight_decay=1e-5)
    te.lookahead_prologue(acts[:B])
    pre = True
    worst = {}
    losses = []
    for i in range(steps):
        x, y = acts[i * B:(i + 1) * B], labels[i * B:(i + 1) * B]
        _load_adam(ref, opt, te, slot, i)
        opt.zero_grad()
        loss_r = F.cross_entropy(_ref_tail_forward(ref, x, seed_base, i + 1), y, reduction="none")
        loss_r.mean().backward()
        opt.step()
        nxt = acts[(i + 1) * B:(i + 2) * B] if i + 1 < steps else None
        loss_e, _ = te.train_fwd_bwd3(x, y, need_dx=False, pre=pre)
        te.fused_step(slot, x_next=nxt)
        pre = nxt is not None
        losses.append(loss_e)
        torch.testing.assert_close(loss_e, loss_r.detach(), rtol=2e-4, atol=1e-4)
        for name, p in ref.named_parameters():
            L = te.layers[int(name[2]) - 1]
            e = L.W if name.endswith("weight") else L.b
            d = (e - p.detach()).abs()
            # one Adam step from the same state: rounding-level differences, except elements
            # whose gradient is ~0, where the sign of m / sqrt(v) is rounding noise (<= 2 lr)
            assert d.max().item() <= 2 * lr + 1e-6, (i, name, d.max().item())
            frac = (d > 1e-6).float().mean().item()
            worst[name] = max(worst.get(name, 0.0), frac)
            assert frac < 1e-4, (i, name, frac)
            st, mine = opt.state[p], slot.states[name]
            # the moments carry the gradient's own rounding (fp32 sums over 16 rows in another
            # order than hipBLASLt's): absolute tolerance relative to the tensor's scale
            for k, tk in (("m", "exp_avg"), ("v", "exp_avg_sq")):
                ref_k = st[tk]
                torch.testing.assert_close(mine[k], ref_k, rtol=1e-3, atol=1e-5 * ref_k.abs().max().item() + 1e-30,
                                           msg=f"step {i} {name} {k}")
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(losses), loss_nat)
    for L1, L2 in zip(te.layers, nat.layers):
        assert torch.equal(L1.W, L2.W) and torch.equal(L1.b, L2.b)
    assert (te.fwd_count, slot.t) == (nat.fwd_count, nslot.t) == (steps, steps)


def test_vanilla_split_epoch_matches_composed_torch_sgd(cuda, tmp_path):
    """The vanilla split epoch (`split_epoch`: packed act+labels, Bob's fused step, Alice's
    deferred in-kernel update + flush) against composed `model1_sisa` + `model2_sisa` with two
    `torch.optim.SGD(lr, momentum=0.9)`, re-synchronised before every batch (weights and
    momentum buffers of both sides copied from the engine), 40 batches + a partial one."""
    from splitlearning_amd.config import parse_args
    from splitlearning_amd.data.mnist import write_shards
    from splitlearning_amd.parallel.dist import Comm, Placement
    from splitlearning_amd.protocols import VanillaSession
    args = parse_args(["--vanilla", "--world_size", "2", "--seed", "5", "--num_samples", "2000", "--no_tqdm",
                       "--datapath", str(tmp_path / "d"), "--log_dir", str(tmp_path / "logs")])
    write_shards(args, verbose=False)
    sess = VanillaSession(args, Comm(0, 1, cuda, Placement.make(2, 1, 1)), cuda)
    a = sess.alices[1]
    front_r = copy.deepcopy(a.front.module).to(cuda)
    tail_r = copy.deepcopy(sess.tail.module).to(cuda)
    lr = args.lr
    opt_a = torch.optim.SGD(front_r.parameters(), lr=lr, momentum=0.9)
    opt_b = torch.optim.SGD(tail_r.parameters(), lr=lr, momentum=0.9)
    order = a.train.shuffled_order(torch.Generator().manual_seed(9))[:16 * 40 + 6]   # partial last batch
    n = order.numel()
    bslot = sess.bob_slot(1)

    def sync_torch():
        with torch.no_grad():
            for (name, p), (_, e) in zip(front_r.named_parameters(), a.front.module.named_parameters()):
                p.copy_(e)
                st = a.slot.states.get("conv." + name.split(".")[-1])
                opt_a.state[p] = {"momentum_buffer": st["buf"].clone().view_as(p)} if st else {}
            for name, p in tail_r.named_parameters():
                L = sess.tail.layers[int(name[2]) - 1]
                p.copy_(L.W if name.endswith("weight") else L.b)
                st = bslot.states.get(name)
                opt_b.state[p] = {"momentum_buffer": st["buf"].clone()} if st else {}
    for i, s in enumerate(range(0, n, 16)):
        idx = order[s:s + 16]
        sync_torch()
        opt_a.zero_grad()
        opt_b.zero_grad()
        step = sess.tail.fwd_count + 1
        out = _ref_tail_forward(tail_r, front_r(a.train.x_float(idx)), sess.tail.seed_base, step)
        F.cross_entropy(out, a.train.y[idx]).backward()
        opt_a.step()
        opt_b.step()
        sess.split_epoch(1, idx, idx.numel())         # one batch of the production split epoch
        for name, p in tail_r.named_parameters():
            L = sess.tail.layers[int(name[2]) - 1]
            e = L.W if name.endswith("weight") else L.b
            torch.testing.assert_close(e, p.detach(), rtol=1e-4, atol=1e-6, msg=f"batch {i} {name}")
        for (name, p), (_, e) in zip(front_r.named_parameters(), a.front.module.named_parameters()):
            # raw 0..255 pixels: conv gradients are O(1e3), summed over 16 x 676 positions
            torch.testing.assert_close(e, p.detach(), rtol=1e-4, atol=1e-4, msg=f"batch {i} {name}")
    torch.cuda.synchronize()
    assert bslot.t == -(-n // 16)
    # every batch above ran as a one-step launch of the persistent vanilla epoch
    # (csrc/vanilla.hip; the co-located default), so this pins that kernel to torch per step
    assert sess.native_split_epochs.get("persistent") == -(-n // 16), sess.native_split_epochs


class _BF16Linear(torch.autograd.Function):
    """Linear with the `--dtype bf16` rule: every product's operands rounded to bf16 (values
    only), fp32 accumulation, in forward, data gradient and weight gradient."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        r = lambda t: t.bfloat16().float()  # noqa: E731
        return r(x) @ r(w).t() + b

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        r = lambda t: t.bfloat16().float()  # noqa: E731
        return r(dy) @ r(w), r(dy).t() @ r(x), r(dy).sum(0)


def _ref_tail_forward_bf16(mod, x, seed_base, step):
    h = x
    for i, lin in enumerate(mod.linears()):
        ls = mod.spec.layers[i]
        h = _BF16Linear.apply(h, lin.weight, lin.bias)
        if ls.relu:
            h = F.relu(h)
        if ls.dropout:
            keep = rng.keep_mask(rng.step_seed(seed_base, i, step), h.shape[0], h.shape[1], ls.dropout,
                                 device=h.device)
            h = h * keep / (1 - ls.dropout)
    return h


def test_bf16_compute_server_steps_match_torch(cuda):
    """`--dtype bf16` (BASELINE config 2's precision): the fused SISA server step with bf16
    operands (bf16 MFMA in the forward, bf16-rounded operands elsewhere, fp32 accumulation,
    fp32 master weights and Adam state), 32 steps re-synchronised before each, against torch
    with the same rounding rule (`_BF16Linear`) -- and its losses within bf16 tolerance of
    the exact-fp32 model's."""
    from splitlearning_amd.ops import hip_ops
    B, steps, lr, seed_base = 16, 32, 1e-3, 5
    g = torch.Generator().manual_seed(2)
    acts = torch.rand(B * steps, 5408, generator=g).to(cuda)
    labels = torch.randint(0, 10, (B * steps,), generator=g).to(cuda)
    torch.manual_seed(6)
    base = ServerTailSisa()
    te = TailEngine(copy.deepcopy(base), sisa_server_spec(), cuda, seed_base=seed_base, ws_tag="#bf")
    slot = OptSlot(adam(lr, 1e-5))
    for L in te.layers:
        slot.state(f"{L.spec.name}.weight", L.W)
        slot.state(f"{L.spec.name}.bias", L.b)
    ref = copy.deepcopy(base).to(cuda)
    opt = torch.optim.Adam(ref.parameters(), lr=lr, weight_decay=1e-5)
    C = hip_ops.C()
    C.set_compute_dtype("bf16")
    try:
        te.lookahead_prologue(acts[:B])
        pre = True
        for i in range(steps):
            x, y = acts[i * B:(i + 1) * B], labels[i * B:(i + 1) * B]
            _load_adam(ref, opt, te, slot, i)
            with torch.no_grad():
                loss32 = F.cross_entropy(_ref_tail_forward(ref, x, seed_base, i + 1), y, reduction="none")
            opt.zero_grad()
            loss_r = F.cross_entropy(_ref_tail_forward_bf16(ref, x, seed_base, i + 1), y, reduction="none")
            loss_r.mean().backward()
            opt.step()
            nxt = acts[(i + 1) * B:(i + 2) * B] if i + 1 < steps else None
            loss_e, _ = te.train_fwd_bwd3(x, y, need_dx=False, pre=pre)
            te.fused_step(slot, x_next=nxt)
            pre = nxt is not None
            torch.testing.assert_close(loss_e, loss_r.detach(), rtol=1e-3, atol=1e-3)
            torch.testing.assert_close(loss_e, loss32, rtol=3e-2, atol=3e-2)     # bf16 vs exact fp32
            for name, p in ref.named_parameters():
                L = te.layers[int(name[2]) - 1]
                e = L.W if name.endswith("weight") else L.b
                d = (e - p.detach()).abs()
                assert d.max().item() <= 2 * lr + 1e-6, (i, name, d.max().item())
                assert (d > 1e-6).float().mean().item() < 2e-3, (i, name, (d > 1e-6).float().mean().item())
    finally:
        C.set_compute_dtype("fp32")
