"""Native split-mode epochs (`_C.SplitEpoch`, csrc/split.cpp; protocols/split_native.py): a
vanilla / U-shape `split_epoch` issued from C++ must leave exactly — bitwise — the parameters,
optimizer states, step counts and dropout counters of the Python loop it replaces (same
launches, seeds and workspaces), over several epochs with a partial last batch, and also
across an unlearn (fresh slots, filtered order).  Reference hot loops:
data_entities_vanilla.py:66-76, data_entities.py:65-81."""
import pytest
import torch

from splitlearning_amd.config import parse_args
from splitlearning_amd.data.mnist import write_shards
from splitlearning_amd.parallel.dist import Comm, Placement

pytestmark = pytest.mark.gpu


def _session(kind, tmp_path, native, dev, B=16, persist=False):
    from splitlearning_amd.protocols import UShapeSession, VanillaSession
    flags = ["--vanilla"] if kind == "vanilla" else []
    if not native:
        flags.append("--python_epoch")
    if not persist:
        flags += ["--split_persist", "off"]   # the per-batch executor (csrc/vanilla.hip has its own tests)
    args = parse_args(flags + ["--world_size", "2", "--seed", "11", "--num_samples", "900", "--no_tqdm",
                               "--batch_size", str(B), "--datapath", str(tmp_path / "d"),
                               "--log_dir", str(tmp_path / ("logs_n" if native else "logs_p"))])
    if not (tmp_path / "d").exists():
        write_shards(args, verbose=False)
    cls = VanillaSession if kind == "vanilla" else UShapeSession
    return cls(args, Comm(0, 1, dev, Placement.make(2, 1, 1)), dev)


def _states(sess, kind):
    a = sess.alices[1]
    out = {}
    for L in sess.tail.layers:
        out[f"bob.{L.spec.name}.W"] = L.W
        out[f"bob.{L.spec.name}.b"] = L.b
    for name, st in sess.bob_slot(1).states.items():
        for k, v in st.items():
            out[f"bobslot.{name}.{k}"] = v
    w, b = a.front.params
    out["front.w"], out["front.b"] = w, b
    if kind == "ushape":
        out["head.W"], out["head.b"] = a.head.layers[0].W, a.head.layers[0].b
    for name, st in a.slot.states.items():
        for k, v in st.items():
            out[f"aslot.{name}.{k}"] = v
    return out


@pytest.mark.parametrize("kind", ["vanilla", "ushape"])
@pytest.mark.parametrize("B", [16, 5])
def test_native_split_epoch_matches_python(cuda, tmp_path, kind, B):
    from splitlearning_amd.protocols.split_native import native_split_ok
    sp = _session(kind, tmp_path, False, cuda, B)
    sn = _session(kind, tmp_path, True, cuda, B)
    assert native_split_ok(sn, 1, kind) and not native_split_ok(sp, 1, kind)
    order = sp.alices[1].train.shuffled_order(torch.Generator().manual_seed(4))[:B * 6 + 3].to(cuda)
    for _ in range(2):
        for s in (sp, sn):
            s.split_epoch(1, order, order.numel())
    # an unlearn in between: fresh client + Bob slots, then more epochs
    for s in (sp, sn):
        s.alices[1].slot = type(s.alices[1].slot)(s.alice_optim())
        s.bob_slots[1] = type(s.bob_slots[1])(s.bob_optim())
        s.split_epoch(1, order[: B * 3], B * 3)
    torch.cuda.synchronize()
    a, b = _states(sp, kind), _states(sn, kind)
    assert a.keys() == b.keys()
    for k in a:
        assert torch.equal(a[k], b[k]), k
    assert sp.alices[1].slot.t == sn.alices[1].slot.t and sp.bob_slot(1).t == sn.bob_slot(1).t
    assert sp.tail.fwd_count == sn.tail.fwd_count


def test_native_split_ushape_large_batch_uses_python(cuda, tmp_path):
    """B > 40: the U-shape head is not one head_step launch; the Python loop runs."""
    from splitlearning_amd.protocols.split_native import native_split_ok
    assert not native_split_ok(_session("ushape", tmp_path, True, cuda, 64), 1, "ushape")
    assert native_split_ok(_session("vanilla", tmp_path, True, cuda, 64), 1, "vanilla")


@pytest.mark.parametrize("k", [2, 4])
def test_native_concat_epoch_matches_python(cuda, tmp_path, k):
    """SISA-concat server epochs (k-head grouped CE, uneven shards): `_C.ServerEpoch` with the
    grouped head against the same launches issued step by step from Python (`--python_epoch`):
    bitwise equal parameters, Adam moments and counters."""
    from splitlearning_amd.parallel.dist import Comm, Placement
    from splitlearning_amd.protocols import ConcatSession

    def session(native):
        flags = [] if native else ["--python_epoch"]
        args = parse_args(["--sisa", "--concat", "--world_size", str(k + 1), "--seed", "11", "--num_samples",
                           "1500", "--no_tqdm", "--datapath", str(tmp_path / "d"),
                           "--log_dir", str(tmp_path / ("ln" if native else "lp"))] + flags)
        if not (tmp_path / "d").exists():
            write_shards(args, verbose=False)
        return ConcatSession(args, Comm(0, 1, cuda, Placement.make(k + 1, 1, 1)), cuda)

    sp, sn = session(False), session(True)
    B = sn.B
    g = torch.Generator().manual_seed(k)
    ns = [B * 5 + 3, B * 3 + 11, B * 6, B * 2 + 1][:k]
    caches = [((torch.rand(n, 5408, generator=g) * 10).to(cuda), torch.randint(0, 10, (n,), generator=g).to(cuda))
              for n in ns]
    for _ in range(2):
        for s in (sp, sn):
            s.concat_epoch(caches)
    torch.cuda.synchronize()
    for La, Lb in zip(sp.tail.layers, sn.tail.layers):
        assert torch.equal(La.W, Lb.W) and torch.equal(La.b, Lb.b), La.spec.name
    for name, st in sp.bob_slot.states.items():
        for key, v in st.items():
            assert torch.equal(v, sn.bob_slot.states[name][key]), (name, key)
    assert sp.bob_slot.t == sn.bob_slot.t and sp.tail.fwd_count == sn.tail.fwd_count
