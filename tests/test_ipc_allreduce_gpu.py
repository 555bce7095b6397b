"""Peer-mapped all-reduce (csrc/ipc_ar.h, parallel/rccl.make_ipc_allreduce) across real
processes on the box's one GPU: set-up + self-test agree on every rank, and random fp32
messages come back bitwise equal to the rank-ordered sum (scripts/ipc_allreduce_one_gpu.py).
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("T", [2, 4])
def test_ipc_allreduce_across_processes(T):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "ipc_allreduce_one_gpu.py"), str(T)],
                         capture_output=True, text=True, timeout=110, cwd=ROOT)
    text = out.stdout + out.stderr
    assert out.returncode == 0, text[-3000:]
    assert out.stdout.count("ipc allreduce up") == T, text[-3000:]
    assert out.stdout.count("PASS") == T, text[-3000:]


def test_ipc_allreduce_single_rank_identity(cuda):
    import torch
    from splitlearning_amd import _native
    C = _native.load()
    ipc = C.IpcAllReduce(1, 0, 4096)
    ipc.open([ipc.handle()])
    x = torch.randn(4000, device=cuda)
    y = x.clone()
    for _ in range(3):
        ipc.allreduce_sum(y)
    torch.cuda.synchronize()
    assert torch.equal(x, y) and ipc.error() == 0


def test_ipc_allreduce_wait_is_bounded():
    """A rank whose peer never issues the matching all-reduce gives up after its timeout and
    raises the error word (checked at every phase end: protocols/base.py _check_transport)
    instead of spinning forever."""
    env = dict(os.environ, SL_IPC_TIMEOUT_CHECK="1")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "ipc_allreduce_one_gpu.py"), "2"],
                         capture_output=True, text=True, timeout=110, cwd=ROOT, env=env)
    text = out.stdout + out.stderr
    assert out.returncode == 0, text[-3000:]
    assert "error word 1" in out.stdout and out.stdout.count("PASS") == 2, text[-3000:]
