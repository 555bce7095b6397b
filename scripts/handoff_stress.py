"""Hand-off stress test of the persistent kernels' publication primitive (csrc/handoff.hip):
every mode x a few geometries, mismatching words out of words checked, and us per round.

    python scripts/handoff_stress.py [rounds]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from splitlearning_amd import _native  # noqa: E402

MODES = {0: "shipped: sc1 stores + drained add / poll + sc1 loads",
         1: "control: plain stores, plain loads, no fences",
         2: "sc1 stores, plain loads",
         3: "LLVM form: plain stores + agent release / agent acquire + plain loads",
         4: "shipped + agent acquire after the poll"}


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    C = _native.load()
    torch.cuda.init()
    G = 256
    for P, nsrc, stride, busy in ((1024, 4, 37, 4.0), (256, 8, 9, 2.0), (4096, 2, 65, 8.0)):
        print(f"== G {G}, payload {4 * P} B per producer rewritten in place every round, {nsrc} sources per "
              f"consumer (stride {stride}), random delay <= {busy} us, R {R}", flush=True)
        for mode in (0, 4, 3, 2, 1):
            nbad, rmin, err, ms, first = C.handoff_stress(G, P, R, nsrc, stride, mode, busy, 10.0)
            words = G * nsrc * P * rmin
            print(f"mode {mode} ({MODES[mode]}): {nbad} stale of {words} words; rounds {rmin}/{R}; err {err}; "
                  f"{1000.0 * ms / R:.2f} us/round" + (f"; first {first}" if nbad else ""), flush=True)


if __name__ == "__main__":
    main()
