"""Golden tests: the fused engines reproduce the composed eager PyTorch model.

Vanilla split learning is mathematically one model (front + tail) trained with
one optimizer per Alice-Bob pair.  We train the engines and
an autograd reference side by side for several steps — same init, same batches,
same dropout masks (regenerated from the counter hash) — and compare parameters.
"""
import torch
import torch.nn.functional as F

from splitlearning_amd.config import OptimCfg
from splitlearning_amd.data.device_dataset import DeviceShard
from splitlearning_amd.data.mnist import synthetic_mnist
from splitlearning_amd.engine import FrontEngine, OptSlot, TailEngine
from splitlearning_amd.models import (ClientFrontSisa, ClientFront, Head, ServerTailSisa, ServerTailUShape,
                                      head_spec, sisa_server_spec, ushape_server_spec)
from splitlearning_amd.ops import rng

DEV = torch.device("cpu")


def assert_adam_close(a, b, lr, steps, msg=""):
    """Adam normalises the update, so an element whose gradient is ~0 (|g| << eps or
    cancelling sums) moves by up to lr in a direction set by rounding noise.  Require
    near-equality everywhere except a tiny fraction of such elements, and bound those."""
    d = (a - b).abs()
    assert d.max().item() <= 2 * lr * steps + 1e-6, msg
    assert (d > 1e-5).float().mean().item() < 1e-4, msg


def _shard(n=64, seed=0):
    x, y = synthetic_mnist(n, seed=seed)
    return DeviceShard(torch.from_numpy(x), torch.from_numpy(y), DEV)


def _ref_tail_forward(tail_mod, x, seed_base, step, train):
    h = x
    for i, lin in enumerate(tail_mod.linears()):
        ls = tail_mod.spec.layers[i]
        h = F.linear(h, lin.weight, lin.bias)
        if ls.relu:
            h = F.relu(h)
        if ls.dropout and train:
            keep = rng.keep_mask(rng.step_seed(seed_base, i, step), h.shape[0], h.shape[1], ls.dropout)
            h = h * keep / (1 - ls.dropout)
    return h


def test_vanilla_split_step_equals_composed_model():
    torch.manual_seed(0)
    front_e = ClientFrontSisa()
    tail_e = ServerTailSisa()
    front_r = ClientFrontSisa()
    tail_r = ServerTailSisa()
    front_r.load_state_dict(front_e.state_dict())
    tail_r.load_state_dict(tail_e.state_dict())
    shard = _shard(64)
    fe = FrontEngine(front_e, DEV)
    te = TailEngine(tail_e, sisa_server_spec(), DEV, seed_base=11)
    cfg = OptimCfg("sgd", 0.01, momentum=0.9)
    a_slot, b_slot = OptSlot(cfg), OptSlot(cfg)
    opt_a = torch.optim.SGD(front_r.parameters(), lr=0.01, momentum=0.9)
    opt_b = torch.optim.SGD(tail_r.parameters(), lr=0.01, momentum=0.9)
    from splitlearning_amd.ops import torch_ops as K
    for step in range(1, 5):
        idx = torch.arange((step - 1) * 16, step * 16)
        # engine path (what VanillaSession.split_step runs, single process)
        act, am = fe.forward(shard, idx)
        out = te.forward(act, train=True)
        _, dout = K.softmax_ce(out, shard.y[idx], 1.0 / 16)
        dx = te.backward_dgrad(dout, need_dx=True)
        te.backward_step(b_slot)
        fe.backward_step(dx, act, am, shard, idx, a_slot)
        # reference: composed autograd
        opt_a.zero_grad()
        opt_b.zero_grad()
        xr = shard.x_float(idx)
        outr = _ref_tail_forward(tail_r, front_r(xr), 11, step, True)
        F.cross_entropy(outr, shard.y[idx]).backward()
        opt_a.step()
        opt_b.step()
        torch.testing.assert_close(out, outr.detach(), rtol=1e-4, atol=1e-4)
    for (k, v), (k2, v2) in zip(tail_e.state_dict().items(), tail_r.state_dict().items()):
        torch.testing.assert_close(v, v2, rtol=1e-4, atol=1e-5, msg=k)
    for (k, v), (k2, v2) in zip(front_e.state_dict().items(), front_r.state_dict().items()):
        torch.testing.assert_close(v, v2, rtol=1e-3, atol=1e-4, msg=k)


def test_sisa_server_step_adam_equals_torch():
    torch.manual_seed(1)
    tail_e, tail_r = ServerTailSisa(), ServerTailSisa()
    tail_r.load_state_dict(tail_e.state_dict())
    te = TailEngine(tail_e, sisa_server_spec(), DEV, seed_base=5)
    slot = OptSlot(OptimCfg("adam", 1e-3, weight_decay=1e-5))
    opt = torch.optim.Adam(tail_r.parameters(), lr=1e-3, weight_decay=1e-5)
    from splitlearning_amd.ops import torch_ops as K
    g = torch.Generator().manual_seed(0)
    for step in range(1, 4):
        x = torch.rand(16, 5408, generator=g) * 50
        y = torch.randint(0, 10, (16,), generator=g)
        out = te.forward(x, train=True)
        _, d = K.softmax_ce(out, y, 1 / 16)
        te.backward_dgrad(d, need_dx=False)
        te.backward_step(slot)
        opt.zero_grad()
        F.cross_entropy(_ref_tail_forward(tail_r, x, 5, step, True), y).backward()
        opt.step()
    for (k, v), (_, v2) in zip(tail_e.state_dict().items(), tail_r.state_dict().items()):
        assert_adam_close(v, v2, 1e-3, 3, msg=k)


def test_ushape_step_equals_composed_model():
    torch.manual_seed(2)
    mods_e = (ClientFront(), ServerTailUShape(), Head())
    mods_r = (ClientFront(), ServerTailUShape(), Head())
    for a, b in zip(mods_e, mods_r):
        b.load_state_dict(a.state_dict())
    shard = _shard(48, seed=3)
    fe = FrontEngine(mods_e[0], DEV)
    te = TailEngine(mods_e[1], ushape_server_spec(), DEV)
    he = TailEngine(mods_e[2], head_spec(), DEV)
    cfg = OptimCfg("adam", 1e-3)
    a_slot, b_slot = OptSlot(cfg), OptSlot(cfg)
    opt_a = torch.optim.Adam(list(mods_r[2].parameters()) + list(mods_r[0].parameters()), lr=1e-3)
    opt_b = torch.optim.Adam(mods_r[1].parameters(), lr=1e-3)
    from splitlearning_amd.ops import torch_ops as K
    for step in range(3):
        idx = torch.arange(step * 16, step * 16 + 16)
        act, am = fe.forward(shard, idx)
        mid = te.forward(act, train=True)
        logits = he.forward(mid, train=True)
        _, dlog = K.softmax_ce(logits, shard.y[idx], 1 / 16)
        dmid = he.backward_dgrad(dlog, need_dx=True)
        t = a_slot.tick()
        he.backward_step(a_slot, t, prefix="head.")
        dx = te.backward_dgrad(dmid, need_dx=True)
        te.backward_step(b_slot)
        fe.backward_step(dx, act, am, shard, idx, a_slot, t=t, prefix="front.")
        opt_a.zero_grad()
        opt_b.zero_grad()
        out = mods_r[2](mods_r[1](mods_r[0](shard.x_float(idx))))
        F.cross_entropy(out, shard.y[idx]).backward()
        opt_a.step()
        opt_b.step()
    for me, mr in zip(mods_e, mods_r):
        for (k, v), (_, v2) in zip(me.state_dict().items(), mr.state_dict().items()):
            assert_adam_close(v, v2, 1e-3, 3, msg=k)
