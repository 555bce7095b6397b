"""Interleaved A/B of the wgrad kernel's cache behaviour on Bob's look-ahead server step.

Variants (csrc/fused.hip `set_traversal`):
  fwd     variant 7 = 1, 4 = 1: layer 0's tiles always walked first-to-last, plain stores
  zigzag  variant 7 = 0, 4 = 1: direction alternates every step, so the tiles a step touched
          last are the next step's first (still resident in the 256 MiB Infinity Cache)
  zz+wt   variant 7 = 0, 4 = 0 (the default): zig-zag plus write-through (sc1) W/m/v stores
  zz+wt2d / zz+wt1d   the same, forcing the 2-D grid (empty workgroups where a layer is
          narrower than the widest) / the 1-D grid over the real tiles; by default the
          launcher picks 2-D only when < 10 % of its workgroups would be empty

All variants run in ONE process, in interleaved rounds (rule: cross-process variance is
larger than the effect), each round `--steps` timed steps after `--settle` untimed ones
so the cache reaches the variant's steady state.  Prints per-variant median / min us/step.

    python scripts/cache_ab.py --tp 1 [--rounds 5 --steps 200]
"""
import argparse
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from splitlearning_amd import ops  # noqa: E402
from splitlearning_amd.engine import OptSlot, TailEngine, adam  # noqa: E402
from splitlearning_amd.models import ServerTailSisa, sisa_server_spec  # noqa: E402
from splitlearning_amd.ops import hip_ops as H  # noqa: E402

VARIANTS = {"fwd": {7: 1, 4: 1, 2: 0}, "zigzag": {7: 0, 4: 1, 2: 0}, "zz+wt": {7: 0, 4: 0, 2: 0},
            "zz+wt2d": {7: 0, 4: 0, 2: 1}, "zz+wt1d": {7: 0, 4: 0, 2: 2},
            # fc2 dgrad split-N cap (csrc/linear.hip linear_dgrad, variant 5): max S, 16-row slices
            "dgS1": {5: 1}, "dgS2": {5: 2}, "dgS16": {5: 16}, "dgS32": {5: 32}, "dgS64": {5: 64}}
SLOTS = (2, 4, 5, 7)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, nargs="+", default=[1])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--settle", type=int, default=20)
    ap.add_argument("--variants", nargs="+", default=list(VARIANTS))
    a = ap.parse_args()
    C = H.C()
    dev = torch.device("cuda", 0)
    ops.set_backend("hip")
    for tp in a.tp:
        torch.manual_seed(0)
        n = 16 * 64
        acts = torch.rand(n, 5408, device=dev) * 20
        labels = torch.randint(0, 10, (n,), device=dev)
        ar = None
        if tp > 1:
            from splitlearning_amd.parallel.rccl import native_allreduce, self_comm
            ar = native_allreduce(self_comm())
        tail = TailEngine(ServerTailSisa(), sisa_server_spec(), dev, tp_rank=0, tp_size=tp, allreduce=ar)
        slot = OptSlot(adam(1e-3, 1e-5))
        tail.lookahead_prologue(acts[:16])
        i = 0

        def steps(k):
            nonlocal i
            for _ in range(k):
                s = (i * 16) % n
                tail.train_fwd_bwd3(acts[s:s + 16], labels[s:s + 16], need_dx=False, pre=True)
                s2 = ((i + 1) * 16) % n
                tail.fused_step(slot, x_next=acts[s2:s2 + 16])
                i += 1

        res = {v: [] for v in a.variants}
        for _ in range(a.rounds):
            for v in a.variants:
                for slot_id in SLOTS:
                    C.set_variant(slot_id, 0)
                for slot_id, val in VARIANTS[v].items():
                    C.set_variant(slot_id, val)
                steps(a.settle)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                steps(a.steps)
                torch.cuda.synchronize()
                res[v].append((time.perf_counter() - t0) / a.steps * 1e6)
        for slot_id in SLOTS:
            C.set_variant(slot_id, 0)       # back to the defaults
        for v, xs in res.items():
            print(f"tp={tp} {v:7s} median {statistics.median(xs):7.2f} us/step  min {min(xs):7.2f}  "
                  f"({' '.join(f'{x:.1f}' for x in xs)})", flush=True)
        del tail, slot, acts
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
