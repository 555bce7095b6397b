"""Split-mode schedule policy (protocols/base.py::split_lookahead): the look-ahead order
(Bob's update after the Alice's next forward) when a Bob shard shares her GPU, the §3.2
overlap order (Bob's update right after the cut gradient leaves) when none does.  Both
orders are the per-batch step's math (reference data_entities_vanilla.py:66-76: each side
steps on batch i before either runs batch i+1), so `split_epoch` in either order must equal
one `split_step` per batch."""
import pytest
import torch

from splitlearning_amd.config import parse_args
from splitlearning_amd.data.mnist import write_shards
from splitlearning_amd.parallel.dist import Comm, Placement

DEV = torch.device("cpu")


def _session(kind, tmp_path, seed):
    from splitlearning_amd.protocols import UShapeSession, VanillaSession
    flags = ["--vanilla"] if kind == "vanilla" else []
    args = parse_args(flags + ["--world_size", "2", "--seed", str(seed), "--num_samples", "900", "--no_tqdm",
                               "--datapath", str(tmp_path / "d"), "--log_dir", str(tmp_path / "logs")])
    if not (tmp_path / "d").exists():
        write_shards(args, verbose=False)
    cls = VanillaSession if kind == "vanilla" else UShapeSession
    return cls(args, Comm(0, 1, DEV, Placement.make(2, 1, 1)), DEV)


def test_policy_follows_placement():
    """Look-ahead exactly when the Alice's rank hosts a Bob shard."""
    from splitlearning_amd.protocols.base import Session
    cases = [(Placement.make(3, 1, 1), {1: True, 2: True}),      # one GPU: everything co-located
             (Placement.make(3, 2, 1), {1: True, 2: False}),     # U-shape TP = 1 on 2 GPUs
             (Placement.make(3, 2, 2), {1: True, 2: True}),      # Bob over every GPU
             (Placement.make(5, 4, 2), {1: True, 2: True, 3: False, 4: False}),
             (Placement.make(3, 3, 1), {1: False, 2: False})]    # one process per role
    for pl, want in cases:
        s = Session.__new__(Session)
        s.pl = pl
        assert {c: s.split_lookahead(c) for c in want} == want, pl


@pytest.mark.parametrize("kind", ["vanilla", "ushape"])
@pytest.mark.parametrize("ahead", [True, False])
def test_split_epoch_order_matches_per_batch_steps(kind, ahead, tmp_path):
    sa = _session(kind, tmp_path, 7)
    sb = _session(kind, tmp_path, 7)
    sb.split_lookahead = lambda cid: ahead
    order = sa.alices[1].train.shuffled_order(torch.Generator().manual_seed(4))[:16 * 4 + 5]
    n = order.numel()
    for s in range(0, n, 16):
        sa.split_step(1, order[s:s + 16], min(16, n - s))
    sb.split_epoch(1, order, n)
    for L1, L2 in zip(sa.tail.layers, sb.tail.layers):
        torch.testing.assert_close(L1.W, L2.W, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(L1.b, L2.b, rtol=1e-5, atol=1e-6)
    mods = [(sa.alices[1].front.module, sb.alices[1].front.module)]
    if kind == "ushape":
        mods.append((sa.alices[1].head.module, sb.alices[1].head.module))
    for ma, mb in mods:
        for (k, va), vb in zip(ma.state_dict().items(), mb.state_dict().values()):
            torch.testing.assert_close(va, vb, rtol=1e-5, atol=1e-6, msg=k)


def test_bob_tp_policy():
    """--bob_tp 0 (parallel/dist.py::choose_bob_tp): the server-phase modes use every GPU;
    the serial split modes weigh the optimizer stream a shard saves against the message
    rounds it adds — vanilla's 32 M-parameter Bob shards across every GPU, the U-shape
    middle (5.5 M) stays on one."""
    from splitlearning_amd.parallel.dist import choose_bob_tp
    for n in (1, 2, 4, 8):
        for mode in ("sisa", "concat", "control"):
            assert choose_bob_tp(mode, n) == n
        assert choose_bob_tp("vanilla", n) == n
        assert choose_bob_tp("ushape", n) == 1
    assert choose_bob_tp("vanilla", 6) in (1, 2, 6) and 6 % choose_bob_tp("vanilla", 6) == 0


@pytest.mark.parametrize("B,ok", [(16, True), (64, True), (65, False), (128, False)])
def test_remote_native_split_respects_executor_batch_bound(B, ok):
    """A remote Alice's epoch runs on `_C.SplitEpoch` only within its batch bound (1..64 rows on
    every role, csrc/split.cpp); beyond it both sides of the pair report "not native", so the
    Python loop runs it instead of both ranks raising in the executor's constructor."""
    from types import SimpleNamespace

    from splitlearning_amd.protocols import split_native as sn

    class _Tail:
        layers = [0, 0, 0]

        def fused3_ok(self):
            return True

    alice = SimpleNamespace(front=SimpleNamespace(frozen=False), train=SimpleNamespace(x=torch.zeros(1, dtype=torch.uint8)))
    for hosts in (True, False):   # the Alice's side and Bob's side of the pair
        s = SimpleNamespace(B=B, alices={1: alice}, tail=_Tail(), hosts=lambda cid, h=hosts: h)
        assert sn._remote_side_ok(s, 1, "vanilla") is ok
