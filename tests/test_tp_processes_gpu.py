"""Tensor-parallel Bob across REAL processes on the box's one GPU: T ranks each run their
shard of the production native executor with the peer-mapped all-reduce between them, and
every rank's shard is bitwise the single-process emulation's (scripts/tp_processes_one_gpu.py).
This is the N > 1 server step end to end (shard math + cross-process all-reduce protocol),
short of the xGMI links themselves.

Reference semantics: bob.train_and_backward's loop (data_entities_vanilla_sisa.py:298-313).
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("T", [2, 4])
def test_tp_server_epoch_across_processes_is_bitwise_emulation(T):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "tp_processes_one_gpu.py"), str(T), "2"],
                         capture_output=True, text=True, timeout=115, cwd=ROOT)
    text = out.stdout + out.stderr
    assert out.returncode == 0, text[-3000:]
    assert out.stdout.count("ipc allreduce up") == T, text[-3000:]
    assert out.stdout.count("bitwise-emulation True") == 2 * T, text[-3000:]
    assert out.stdout.count("PASS") == T, text[-3000:]
