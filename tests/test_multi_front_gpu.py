"""Concurrent frozen-front forwards of co-located Alices (`_C.conv_fwd_multi`,
FrontEngine.forward_multi): one launch per chunk of rows for every hosted Alice, used by the
evaluation (base.py `_eval_counts`) and the SISA activation dumps (sisa.py `_give_many`).
Each Alice's activations must be bitwise her own `forward_chunked` (the training forward
kernel), for shuffled / filtered / sequential orders of different lengths, several chunks,
and more Alices than one launch takes.  Reference: data_entities_vanilla_sisa.py:196-211,370-371."""
import pytest
import torch

from splitlearning_amd.data.device_dataset import DeviceShard
from splitlearning_amd.engine.front import FrontEngine
from splitlearning_amd.models import ClientFrontSisa

pytestmark = pytest.mark.gpu


def _alices(dev, k, seed=0):
    g = torch.Generator().manual_seed(seed)
    fronts, shards = [], []
    for a in range(k):
        torch.manual_seed(seed + 100 + a)
        fronts.append(FrontEngine(ClientFrontSisa(), dev))
        n = 40 + 23 * a
        x = torch.randint(0, 256, (n, 28, 28), generator=g, dtype=torch.uint8)
        y = torch.randint(0, 10, (n,), generator=g)
        shards.append(DeviceShard(x, y, dev))
    return fronts, shards


@pytest.mark.parametrize("k,chunk", [(3, 8192), (3, 7), (18, 16)])
def test_forward_multi_is_each_alices_forward(cuda, k, chunk):
    fronts, shards = _alices(cuda, k)
    orders = []
    for a, sh in enumerate(shards):
        if a % 3 == 0:
            orders.append(None)                                          # sequential (eval)
        elif a % 3 == 1:
            orders.append(torch.randperm(sh.n, device=cuda))             # shuffled dump
        else:
            orders.append(torch.randperm(sh.n, device=cuda)[: sh.n // 2])  # filtered (unlearn)
    got = FrontEngine.forward_multi(fronts, shards, orders, chunk=chunk)
    for f, sh, o, y in zip(fronts, shards, orders, got):
        ref = f.forward_chunked(sh, o if o is not None else sh.sequential_order())
        assert y.shape == ref.shape and torch.equal(y, ref)


def test_sisa_eval_and_dump_match_per_alice(cuda, tmp_path, monkeypatch):
    """A ws = 5 SISA session on one GPU: evaluation counters and the activation cache from
    the concurrent forwards equal the one-Alice-at-a-time path's, bitwise."""
    from splitlearning_amd.config import parse_args
    from splitlearning_amd.data.mnist import write_shards
    from splitlearning_amd.parallel.dist import Comm, Placement
    from splitlearning_amd.protocols import SisaSession

    def session():
        args = parse_args(["--sisa", "--world_size", "5", "--seed", "3", "--num_samples", "1200", "--no_tqdm",
                           "--datapath", str(tmp_path / "d"), "--log_dir", str(tmp_path / "logs")])
        if not (tmp_path / "d").exists():
            write_shards(args, verbose=False)
        return SisaSession(args, Comm(0, 1, cuda, Placement.make(5, 1, 1)), cuda)

    sa = session()
    sa.prefetch_activations()
    ca = sa._eval_counts(3)
    per_alice = staticmethod(lambda fronts, shards, orders, chunk=8192: [
        f.forward_chunked(sh, o if o is not None else sh.sequential_order(), chunk)
        for f, sh, o in zip(fronts, shards, orders)])
    monkeypatch.setattr(FrontEngine, "forward_multi", per_alice)
    sb = session()
    sb.prefetch_activations()
    cb = sb._eval_counts(3)
    assert torch.equal(ca, cb)
    assert sa.activation_and_labels_cache.keys() == sb.activation_and_labels_cache.keys()
    for key in sa.activation_and_labels_cache:
        (xa, ya), (xb, yb) = sa.activation_and_labels_cache[key], sb.activation_and_labels_cache[key]
        assert torch.equal(xa, xb) and torch.equal(ya, yb), key
