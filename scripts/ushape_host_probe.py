"""Is the co-located U-shape epoch bound by the host's launch issue or by the GPU?  Times one
native split epoch (`_C.SplitEpoch.run`, csrc/split.cpp) twice: the host returns once every
launch is issued (t_issue), the GPU finishes at the synchronize (t_done).  t_issue ~ t_done:
the GPU waits on the host.  Usage: python scripts/ushape_host_probe.py [variant20] [ushape|vanilla]
(variant 20 selected the fused U-shape middle + head launch of an A/B that was removed:
profiles/r5w_misc/ushape_fused_mid_head_ab.txt)."""
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from splitlearning_amd.config import parse_args  # noqa: E402
from splitlearning_amd.data.mnist import write_shards  # noqa: E402
from splitlearning_amd.ops import hip_ops  # noqa: E402
from splitlearning_amd.parallel.dist import Comm, Placement  # noqa: E402
from splitlearning_amd.protocols import UShapeSession, VanillaSession  # noqa: E402


def main():
    var = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    kind = sys.argv[2] if len(sys.argv) > 2 else "ushape"
    hip_ops.C().set_variant(20, var)
    dev = torch.device("cuda", 0)
    tmp = tempfile.mkdtemp()
    flags = ["--vanilla"] if kind == "vanilla" else []
    args = parse_args(flags + ["--world_size", "2", "--seed", "11", "--num_samples", "30000", "--no_tqdm",
                               "--batch_size", "16", "--datapath", os.path.join(tmp, "d"), "--log_dir",
                               os.path.join(tmp, "logs")])
    write_shards(args, verbose=False)
    cls = VanillaSession if kind == "vanilla" else UShapeSession
    s = cls(args, Comm(0, 1, dev, Placement.make(2, 1, 1)), dev)
    order = s.alices[1].train.shuffled_order(torch.Generator().manual_seed(4)).to(dev)
    n = order.numel() // 16 * 16
    for r in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.split_epoch(1, order[:n], n)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        b = n // 16
        print(f"{kind} variant20={var} batches {b}: issue {1e6 * (t1 - t0) / b:.2f} us/batch, done "
              f"{1e6 * (t2 - t0) / b:.2f} us/batch", flush=True)


if __name__ == "__main__":
    main()
