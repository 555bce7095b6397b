"""The reference-named role API (splitlearning_amd/api.py) drives a SISA run in one
process on the CPU, with the schedule of split_nn.py:74-117 written against
`bob.*` / `alice.*` names."""
import os

import torch

from splitlearning_amd import api
from splitlearning_amd.config import parse_args
from splitlearning_amd.parallel.dist import Comm, Placement
from splitlearning_amd.protocols import make_session
from splitlearning_amd.runtime.launcher import prepare_data, resolve


def test_reference_named_api_sisa(tmp_path):
    args = resolve(parse_args(["--sisa", "--world_size", "3", "--num_samples", "1200", "--seed", "0",
                               "--no_tqdm", "--device", "cpu", "--datapath", str(tmp_path / "d"),
                               "--log_dir", str(tmp_path / "logs")]))
    os.makedirs(args.log_dir, exist_ok=True)
    prepare_data(args, verbose=False)
    pl = Placement.make(args.world_size, 1, args.bob_tp)
    sess = make_session(args, Comm(0, 1, torch.device("cpu"), pl, None), torch.device("cpu"))
    bob, alices = api.roles(sess)
    assert sorted(alices) == [1, 2]
    bob.train_request_parallel()
    bob.freeze_alice_weights([1, 2])
    bob.train_and_backward([], None)
    before = alices[1].eval_breakdown(9)
    assert len(before) == 6 and before[1] > 0
    corr, tot = alices[2].eval()
    assert 0 <= corr <= tot and tot > 0
    alices[1].unfreeze_weights()
    alices[1].unlearn(9)
    alices[1].freeze_weights()
    bob.train_and_backward([1], 9)
    s = bob.eval_request_breakdown(9)
    assert len(s) == 6
    w = alices[1].give_weights()
    assert w is not None and any(k.endswith("weight") for k in w)
    acts, labels = alices[2].give_activation_and_labels()
    assert acts.shape[1] == 5408 and acts.shape[0] == labels.numel()
    assert bob.inference(acts[:4]).shape == (4, 100)
    assert bob.start_logger() is sess.bob_log
    sess.close()
