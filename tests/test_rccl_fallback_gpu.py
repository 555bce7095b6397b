"""Native communicator set-up across real processes on the GPU box (parallel/rccl.py).

Two ranks share the box's one GPU with a gloo control plane.  RCCL rejects two ranks on
one device ('invalid usage'), which is exactly the failure the set-up must survive: every
rank has to see it and fall back together (a rank that kept a communicator its peer lacks
would deadlock the first collective).  If a runtime does accept the pair, the all-reduce
and the grouped send/recv on the compute stream must give the right values instead.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_native_comm_setup_agrees_across_ranks():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "rccl_two_ranks_one_gpu.py")],
                         capture_output=True, text=True, timeout=150, cwd=ROOT)
    text = out.stdout + out.stderr
    assert out.returncode == 0, text[-3000:]
    # the two ranks' status lines may interleave on one stdout line
    assert all(f"rank {r}: native comm" in out.stdout for r in (0, 1)), text[-3000:]
    up = [f"rank {r}: native comm up" in out.stdout for r in (0, 1)]
    assert up[0] == up[1], out.stdout                   # both ranks decided the same
    if up[0]:
        assert out.stdout.count("allreduce -> 3.0") == 2, out.stdout
        assert "sendrecv got 11.0" in out.stdout and "sendrecv got 10.0" in out.stdout, out.stdout
