"""CLI parity, data pipeline invariants and checkpoint (state_dict) layout."""
import os

import numpy as np
import pytest
import torch

from splitlearning_amd.config import build_parser, parse_args
from splitlearning_amd.data import (dirichlet_partition, make_client_shards, synthetic_mnist, write_shards,
                                    load_shard, shard_paths)
from splitlearning_amd.models import (model1, model1_sisa, model2, model2_sisa, model2_sisa_concat, model3)


def test_reference_flags_and_defaults():
    a = parse_args([])
    assert (a.world_size, a.epochs, a.iterations, a.batch_size) == (3, 1, 5, 16)
    assert a.partition_alpha == 0.5 and a.datapath == "data/mnist_flat" and a.lr == 0.001
    assert a.server_epochs == 3 and not (a.vanilla or a.sisa or a.concat or a.control)
    assert a.mode == "ushape" and a.client_num_in_total == 2
    assert parse_args(["--vanilla"]).mode == "vanilla"
    assert parse_args(["--sisa"]).mode == "sisa"
    assert parse_args(["--sisa", "--concat"]).mode == "concat"
    assert parse_args(["--control"]).mode == "control"
    flags = {a.dest for a in build_parser()._actions}
    for f in ["world_size", "epochs", "iterations", "batch_size", "partition_alpha", "datapath", "lr",
              "server_epochs", "vanilla", "sisa", "concat", "control"]:
        assert f in flags


def test_server_executor_flags():
    """Bob's server-epoch executors beyond the reference's flags: the register-resident epoch
    (default where it fits) or the launch-per-stage executor."""
    a = parse_args(["--sisa"])
    assert a.resident == "auto"
    a = parse_args(["--sisa", "--resident", "off"])
    assert a.resident == "off"
    with pytest.raises(SystemExit):
        parse_args(["--resident", "on"])


class _FakeTail:
    """decide()'s view of a single-shard tail: which persistent executors fit."""
    tp_size = 1

    def __init__(self, res_ok, hy_ok):
        self.res_ok, self.hy_ok = res_ok, hy_ok

    def resident_ok(self, slot, B):
        return self.res_ok

    def hybrid_ok(self, slot, B):
        return self.hy_ok


@pytest.mark.parametrize("argv,res_ok,hy_ok,kind,why", [
    (["--sisa"], True, True, "resident", "adopted"),
    (["--sisa"], False, True, "hybrid", "adopted"),
    (["--sisa"], False, False, "launch_per_stage", "no persistent executor fits this shard"),
    # --resident off leaves the hybrid on (round-4 bug: it turned both off)
    (["--sisa", "--resident", "off"], True, True, "hybrid", "adopted"),
    (["--sisa", "--resident", "off"], True, False, "launch_per_stage", "no persistent executor fits this shard"),
    (["--sisa", "--hybrid", "off"], False, True, "launch_per_stage", "no persistent executor fits this shard"),
    (["--sisa", "--hybrid", "off"], True, True, "resident", "adopted"),
    (["--sisa", "--resident", "off", "--hybrid", "off"], True, True, "launch_per_stage", "off"),
    # bf16 compute: both persistent executors are fp32-only, and the reason says so
    (["--sisa", "--dtype", "bf16"], True, True, "launch_per_stage", "dtype bf16"),
])
def test_server_executor_decision_table(argv, res_ok, hy_ok, kind, why):
    from splitlearning_amd.engine.resident import decide
    from splitlearning_amd.protocols.sisa import executor_wants
    want, want_h = executor_wants(parse_args(argv))
    k, w = decide(_FakeTail(res_ok, hy_ok), None, 16, distributed=False, want=want, want_hybrid=want_h)
    assert k == kind
    assert w.startswith(why)


@pytest.mark.parametrize("argv,msg", [
    (["--concat"], "--concat option can only be used with the --sisa"),
    (["--vanilla", "--sisa"], "--vanilla option cannot be used"),
    (["--vanilla", "--sisa", "--concat"], "--vanilla option cannot be used"),
    (["--control", "--sisa"], "--control option cannot be used"),
])
def test_reference_validation_errors(argv, msg):
    with pytest.raises(ValueError, match=msg):
        parse_args(argv)


def test_dirichlet_partition_invariants():
    y = np.random.default_rng(0).integers(0, 10, 5000)
    for k in (1, 2, 4, 8):
        parts = dirichlet_partition(y, k, 10, 0.5, rng=np.random.default_rng(k))
        allidx = np.concatenate(list(parts.values()))
        assert len(allidx) == len(y) and len(np.unique(allidx)) == len(y)
        assert min(len(p) for p in parts.values()) >= 10
    p1 = dirichlet_partition(y, 4, 10, 0.5, rng=np.random.default_rng(3))
    p2 = dirichlet_partition(y, 4, 10, 0.5, rng=np.random.default_rng(3))
    assert all(np.array_equal(p1[i], p2[i]) for i in range(4))


def test_dirichlet_is_non_iid_at_small_alpha():
    y = np.random.default_rng(0).integers(0, 10, 20000)
    parts = dirichlet_partition(y, 4, 10, 0.1, rng=np.random.default_rng(0))
    hist = np.stack([np.bincount(y[p], minlength=10) / len(p) for p in parts.values()])
    assert hist.max(axis=1).mean() > 0.3          # skewed label mixtures


def test_synthetic_mnist_shape_and_range():
    x, y = synthetic_mnist(100, seed=0)
    assert x.shape == (100, 1, 28, 28) and x.dtype == np.uint8 and y.dtype == np.int64
    assert set(np.unique(y)) <= set(range(10))


def test_shards_tensor_only_roundtrip(tmp_path):
    class A:
        pass
    a = A()
    a.datapath = str(tmp_path)
    a.client_num_in_total = 3
    a.partition_alpha = 0.5
    a.num_samples = 900
    a.seed = 1
    a.mnist_npz = ""
    sizes = write_shards(a, verbose=False)
    total = 0
    for cid in (1, 2, 3):
        ptr, pte = shard_paths(str(tmp_path), cid)
        assert os.path.basename(ptr) == f"data_worker{cid}_train.pt"
        tr, te = load_shard(str(tmp_path), cid)          # weights_only=True inside
        assert tr["x"].dtype == torch.uint8 and tr["x"].shape[1:] == (1, 28, 28)
        assert sizes[cid] == (len(tr["y"]), len(te["y"]))
        # 80/20 split per client (relational_table_preprocessor.py:80)
        n = len(tr["y"]) + len(te["y"])
        assert len(tr["y"]) == int(n * 0.8)
        total += n
    assert total == 900


def test_make_client_shards_disjoint():
    x, y = synthetic_mnist(500, seed=0)
    sh = make_client_shards(x, y, 2, 0.5, seed=0)
    assert sum(len(v[1]) + len(v[3]) for v in sh.values()) == 500


REF_KEYS = {
    model1: {"conv1.weight": (32, 1, 3, 3), "conv1.bias": (32,)},
    model1_sisa: {"conv_layers.0.weight": (32, 1, 3, 3), "conv_layers.0.bias": (32,)},
    model2: {"fc1.weight": (1000, 5408), "fc1.bias": (1000,), "fc2.weight": (100, 1000), "fc2.bias": (100,)},
    model2_sisa: {"fc1.weight": (5000, 5408), "fc1.bias": (5000,), "fc2.weight": (1000, 5000),
                  "fc2.bias": (1000,), "fc3.weight": (100, 1000), "fc3.bias": (100,)},
    model3: {"fc3.weight": (10, 100), "fc3.bias": (10,)},
}


@pytest.mark.parametrize("cls", list(REF_KEYS))
def test_state_dict_layout_matches_reference(cls):
    sd = cls().state_dict()
    assert {k: tuple(v.shape) for k, v in sd.items()} == REF_KEYS[cls]


def test_param_counts_match_survey():
    count = lambda m: sum(p.numel() for p in m.parameters())
    assert count(model1()) == 320 and count(model1_sisa()) == 320
    assert count(model2()) == 5_509_100 and count(model2_sisa()) == 32_146_100
    assert count(model2_sisa_concat(4)) == 113_566_400 and count(model3()) == 1_010


def test_model_forward_shapes():
    x = torch.zeros(2, 1, 28, 28)
    assert model1_sisa()(x).shape == (2, 5408)
    assert model2_sisa()(torch.zeros(2, 5408)).shape == (2, 100)
    assert model2_sisa_concat(3)(torch.zeros(2, 5408 * 3)).shape == (2, 300)
    assert model2()(torch.zeros(2, 32, 13, 13)).shape == (2, 100)
    assert model3()(torch.zeros(2, 100)).shape == (2, 10)


# ---------------------------------------------------------------- reference-named data API
def test_reference_data_api(tmp_path):
    from types import SimpleNamespace

    import numpy as np

    from splitlearning_amd.data import (DeviceLoader, image_preprocess_dl, load_mnist_flat, load_mnist_image,
                                        load_shard, non_iid_partition_with_dirichlet_distribution,
                                        partition_class_samples_with_dirichlet_distribution,
                                        record_data_stats, relational_table_preprocess_dl)
    from splitlearning_amd.data.device_dataset import DeviceShard
    from splitlearning_amd.data.mnist import synthetic_mnist

    x, y = synthetic_mnist(600, seed=1)
    rng = np.random.default_rng(0)
    idx_map = non_iid_partition_with_dirichlet_distribution(y, 3, 10, 0.5, rng=rng)
    allidx = sorted(i for v in idx_map.values() for i in v)
    assert allidx == list(range(600)) and min(len(v) for v in idx_map.values()) >= 10
    stats = record_data_stats(y, idx_map)
    assert sum(sum(c.values()) for c in stats.values()) == 600
    buckets = [[], []]
    _, mn = partition_class_samples_with_dirichlet_distribution(600, 0.5, 2, buckets, np.arange(50),
                                                                 rng=np.random.default_rng(1))
    assert sum(len(b) for b in buckets) == 50 and mn == min(len(b) for b in buckets)

    args = SimpleNamespace(client_num_in_total=3, partition_alpha=0.5, batch_size=16, class_num=10, seed=0)
    out = image_preprocess_dl(args, x.astype(np.float32), y)
    train_num, test_num, tg, teg, tln, tl, tel, cn = out
    assert train_num + test_num == 600 and cn == 10 and set(tl) == {0, 1, 2}
    assert sum(tln.values()) == train_num and len(tg.dataset[1]) == train_num
    xb, yb = next(iter(tl[0]))
    assert xb.shape[1:] == (1, 28, 28) and xb.shape[0] == yb.shape[0] <= 16
    assert sum(b[1].numel() for b in tl[1]) == tln[1]          # one epoch covers the shard
    tab = relational_table_preprocess_dl(args, x.reshape(600, -1).astype(np.float32), y)
    assert next(iter(tab[5][0]))[0].shape[1] == 784
    ld = DeviceLoader(torch.arange(10.0).view(10, 1), torch.arange(10), 4)
    assert len(ld) == 3 and [b[1].tolist() for b in ld] == [[0, 1, 2, 3], [4, 5, 6, 7], [8, 9]]

    for fn, shape in ((load_mnist_image, (1, 28, 28)), (load_mnist_flat, (784,))):
        d = tmp_path / fn.__name__
        a = SimpleNamespace(datapath=str(d), client_num_in_total=2, partition_alpha=0.5, seed=0, num_samples=500,
                            mnist_npz="")
        sizes = fn(a, verbose=False)
        tr, te = load_shard(str(d), 1)
        assert tuple(tr["x"].shape[1:]) == shape and len(tr["y"]) == sizes[1][0]
        assert DeviceShard(tr["x"], tr["y"], torch.device("cpu")).x.shape[1] == 784


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B", [1, 5, 16])
def test_act_label_message_pack_roundtrip(dtype, B):
    """The per-batch [activation | labels] message (protocols/base.py Session.pack, the layout the
    native split executor sends: labels as int64 words behind the rows, 16-byte padded) carries
    the labels bit-exactly in any wire dtype and the activation unchanged."""
    from splitlearning_amd.config import CUT_FEATURES
    from splitlearning_amd.protocols.base import Session
    g = torch.Generator().manual_seed(B)
    act = torch.randn(B, CUT_FEATURES, generator=g).to(dtype)
    labels = torch.randint(0, 10, (B,), generator=g)
    labels[0] = 9
    buf = Session.pack(act, labels)
    assert buf.dtype == dtype and buf.numel() == Session.packed_len(B, dtype)
    assert (buf.numel() * buf.element_size()) % 16 == 0
    a2, l2 = Session.unpack(buf, B)
    assert torch.equal(a2, act) and torch.equal(l2, labels) and l2.dtype == torch.int64
    if dtype == torch.float32:
        # csrc/split.cpp act_msg_words: M * 5408 + 2 M floats rounded up to 4
        assert Session.packed_len(B, dtype) == (B * CUT_FEATURES + 2 * B + 3) // 4 * 4


def test_split_persist_flag_and_cpu_decision(tmp_path):
    """--split_persist defaults to auto; the persistent vanilla epoch is never chosen off the GPU
    (csrc/vanilla.hip needs 256 co-resident workgroups), so CPU sessions keep the Python loop."""
    import torch
    from splitlearning_amd.config import parse_args
    from splitlearning_amd.data.mnist import write_shards
    from splitlearning_amd.parallel.dist import Comm, Placement
    from splitlearning_amd.protocols import VanillaSession
    from splitlearning_amd.protocols.split_native import persistent_vanilla_ok
    assert parse_args(["--vanilla"]).split_persist == "auto"
    assert parse_args(["--vanilla", "--split_persist", "off"]).split_persist == "off"
    args = parse_args(["--vanilla", "--world_size", "2", "--num_samples", "300", "--no_tqdm",
                       "--datapath", str(tmp_path / "d"), "--log_dir", str(tmp_path / "l")])
    write_shards(args, verbose=False)
    dev = torch.device("cpu")
    s = VanillaSession(args, Comm(0, 1, dev, Placement.make(2, 1, 1)), dev)
    assert not persistent_vanilla_ok(s, 1)


def test_split_persist_batch_bound_is_reported(tmp_path, monkeypatch):
    """--batch_size > 16 keeps the per-batch executor (the persistent epochs' MFMA row block is the
    batch) and says so in split_persist_reason (bench.py reports it), instead of dropping silently."""
    import torch
    from splitlearning_amd.config import parse_args
    from splitlearning_amd.data.mnist import write_shards
    from splitlearning_amd.parallel.dist import Comm, Placement
    from splitlearning_amd.protocols import VanillaSession
    from splitlearning_amd.protocols import split_native

    class _C:
        VanillaEpoch = object

        def get_compute_dtype(self):
            return "fp32"

    class _Ops:
        def C(self):
            return _C()

    monkeypatch.setattr(split_native, "native_split_ok", lambda sess, cid, mode: True)
    args = parse_args(["--vanilla", "--world_size", "2", "--num_samples", "300", "--no_tqdm", "--batch_size", "32",
                       "--datapath", str(tmp_path / "d"), "--log_dir", str(tmp_path / "l")])
    write_shards(args, verbose=False)
    dev = torch.device("cpu")
    s = VanillaSession(args, Comm(0, 1, dev, Placement.make(2, 1, 1)), dev)
    s.ops = _Ops()
    assert not split_native.persistent_vanilla_ok(s, 1)
    assert "batch 32 > 16" in s.split_persist_reason


def test_persistent_vanilla_refuses_bf16(tmp_path, monkeypatch):
    """csrc/vanilla.hip is exact fp32 only: with --dtype bf16 (fp32 master weights, bf16 operands
    through the global compute-dtype switch) the persistent vanilla epoch must not be chosen, and
    the reason is reported.  The GPU-only conditions are stubbed so the dtype gate
    itself is what decides."""
    import torch
    from splitlearning_amd.config import parse_args
    from splitlearning_amd.data.mnist import write_shards
    from splitlearning_amd.parallel.dist import Comm, Placement
    from splitlearning_amd.protocols import VanillaSession
    from splitlearning_amd.protocols import split_native

    class _C:
        VanillaEpoch = object

        def __init__(self, dt):
            self.dt = dt

        def get_compute_dtype(self):
            return self.dt

    class _Ops:
        def __init__(self, dt):
            self.c = _C(dt)

        def C(self):
            return self.c

    monkeypatch.setattr(split_native, "native_split_ok", lambda sess, cid, mode: True)
    for flag, dt, want in (("fp32", "fp32", True), ("bf16", "bf16", False), ("fp32", "bf16", False)):
        args = parse_args(["--vanilla", "--world_size", "2", "--num_samples", "300", "--no_tqdm", "--dtype", flag,
                           "--datapath", str(tmp_path / "d"), "--log_dir", str(tmp_path / "l")])
        write_shards(args, verbose=False)
        dev = torch.device("cpu")
        s = VanillaSession(args, Comm(0, 1, dev, Placement.make(2, 1, 1)), dev)
        s.ops = _Ops(dt)
        assert split_native.persistent_vanilla_ok(s, 1) is want, (flag, dt)
        if not want:
            assert "bf16" in s.__dict__.get("split_persist_reason", "")


def test_persistent_remote_vanilla_decision(tmp_path, monkeypatch):
    """Bob's side of a remote Alice's vanilla epoch adopts the persistent launch
    (`_C.VanillaEpoch.run_remote`, csrc/vanilla.hip REM) only with the peer-mapped channel, fp32,
    SGD-momentum, B <= 16 and a GPU of its own (ranks sharing one GPU need an explicit reduced grid,
    SL_VA_REMOTE_G); never for U-shape or with --split_persist off.  The GPU objects are stubbed."""
    import torch
    from splitlearning_amd.config import parse_args
    from splitlearning_amd.data.mnist import write_shards
    from splitlearning_amd.parallel.dist import Comm, Placement
    from splitlearning_amd.protocols import VanillaSession
    from splitlearning_amd.protocols import split_native

    class _C:
        VanillaEpoch = object

        def get_compute_dtype(self):
            return "fp32"

    class _Ops:
        c = _C()

        def C(self):
            return self.c

    class _Chan:
        def host_error(self):
            return 0

    monkeypatch.delenv("SL_VA_REMOTE_G", raising=False)

    def sess(*flags):
        args = parse_args(["--vanilla", "--world_size", "2", "--num_samples", "300", "--no_tqdm",
                           "--datapath", str(tmp_path / "d"), "--log_dir", str(tmp_path / "l")] + list(flags))
        write_shards(args, verbose=False)
        dev = torch.device("cpu")
        s = VanillaSession(args, Comm(0, 1, dev, Placement.make(2, 1, 1)), dev)
        s.ops = _Ops()
        s.split_channel = _Chan()
        return s

    s = sess()
    assert split_native.persistent_remote_ok(s, 1, "vanilla")
    assert not split_native.persistent_remote_ok(s, 1, "ushape")
    assert not split_native.persistent_remote_ok(sess("--split_persist", "off"), 1, "vanilla")
    assert not split_native.persistent_remote_ok(sess("--batch_size", "32"), 1, "vanilla")
    s = sess()
    s.split_channel = object()            # RCCL link: the kernel speaks the peer-mapped protocol only
    assert not split_native.persistent_remote_ok(s, 1, "vanilla")
    s = sess()
    s.comm.host_staging = True            # ranks share one GPU
    assert not split_native.persistent_remote_ok(s, 1, "vanilla")
    monkeypatch.setenv("SL_VA_REMOTE_G", "64")
    assert split_native.persistent_remote_ok(s, 1, "vanilla")
    s._va_rem_off = True                  # an earlier decline in this session
    assert not split_native.persistent_remote_ok(s, 1, "vanilla")


def test_persistent_remote_ushape_decision(tmp_path, monkeypatch):
    """The U-shape counterpart (`_C.UShapeEpoch.run_remote`, csrc/ushape.hip REM): Adam on Bob's
    side, fp32 or bf16 as the compute dtype, the peer-mapped channel, a GPU of its own unless
    SL_US_REMOTE_G sets a reduced grid.  The GPU objects are stubbed."""
    import torch
    from splitlearning_amd.config import parse_args
    from splitlearning_amd.data.mnist import write_shards
    from splitlearning_amd.parallel.dist import Comm, Placement
    from splitlearning_amd.protocols import UShapeSession
    from splitlearning_amd.protocols import split_native

    class _C:
        UShapeEpoch = object

        def __init__(self, dt):
            self.dt = dt

        def get_compute_dtype(self):
            return self.dt

    class _Ops:
        def __init__(self, dt):
            self.c = _C(dt)

        def C(self):
            return self.c

    class _Chan:
        def host_error(self):
            return 0

    monkeypatch.delenv("SL_US_REMOTE_G", raising=False)

    def sess(dt="fp32", *flags):
        args = parse_args(["--world_size", "2", "--num_samples", "300", "--no_tqdm", "--dtype", dt,
                           "--datapath", str(tmp_path / "d"), "--log_dir", str(tmp_path / "l")] + list(flags))
        write_shards(args, verbose=False)
        dev = torch.device("cpu")
        s = UShapeSession(args, Comm(0, 1, dev, Placement.make(2, 1, 1)), dev)
        s.ops = _Ops(dt)
        s.split_channel = _Chan()
        return s

    assert split_native.persistent_remote_ok(sess(), 1, "ushape")
    assert split_native.persistent_remote_ok(sess("bf16"), 1, "ushape")
    assert not split_native.persistent_remote_ok(sess(), 1, "vanilla")       # U-shape's Adam Bob
    s = sess()
    s.ops = _Ops("bf16")                                                    # --dtype fp32, bf16 kernels
    assert not split_native.persistent_remote_ok(s, 1, "ushape")
    assert not split_native.persistent_remote_ok(sess("fp32", "--split_persist", "off"), 1, "ushape")
    s = sess()
    s.comm.host_staging = True
    assert not split_native.persistent_remote_ok(s, 1, "ushape")
    monkeypatch.setenv("SL_US_REMOTE_G", "64")
    assert split_native.persistent_remote_ok(s, 1, "ushape")
