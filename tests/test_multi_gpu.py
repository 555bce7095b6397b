"""Multi-GPU tier: the cross-process protocols with every rank on its OWN device (over xGMI),
where the rest of the suite rehearses them with all ranks sharing cuda:0.  Skipped with fewer
than 2 visible GPUs (the driver's test box has one; the 8-GPU scaling node runs bench.py,
whose N > 1 result validates itself: engine/resident.validate).

Covered, T = 2 ranks on cuda:0 / cuda:1 (scripts/*_one_gpu.py with SL_RANK_DEVICES=2):
* the peer-mapped TP all-reduce (csrc/ipc_ar.hip) against the rank-ordered sum;
* the peer-mapped split channel (csrc/ipc_p2p.hip) of a remote Alice's native vanilla / U-shape
  epoch, bitwise the Python loop of the same placement with the same message sequence;
* the hybrid and register-resident persistent epochs tensor-parallel over the two devices
  (in-launch fc2 exchange): replicated state bitwise equal across ranks and close to fp32 torch;
* the mid-epoch failure of those epochs survived across devices (rolled back, launch-per-stage);
* Bob's persistent vanilla / U-shape epochs of a remote Alice on the full grid of his own device,
  her per-batch side on the other (the in-launch channel protocol over xGMI).
Reference: split_nn.py:183-186 (one process per role, mp.spawn)."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs 2 GPUs (one rank per device)")]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, passes=2, timeout=240):
    env = dict(os.environ, SL_RANK_DEVICES="2")
    out = subprocess.run([sys.executable, *args], capture_output=True, text=True, timeout=timeout, cwd=ROOT, env=env)
    text = out.stdout + out.stderr
    assert out.returncode == 0, text[-3000:]
    assert out.stdout.count("PASS") >= passes, text[-3000:]


def test_ipc_allreduce_across_devices():
    _run(os.path.join(ROOT, "scripts", "ipc_allreduce_one_gpu.py"), "2")


@pytest.mark.parametrize("kind", ["vanilla", "ushape"])
def test_remote_split_epoch_across_devices(kind):
    _run(os.path.join(ROOT, "scripts", "split_remote_one_gpu.py"), kind, "16")


@pytest.mark.parametrize("kind", ["hybrid", "resident"])
def test_persistent_tp2_across_devices(kind):
    _run(os.path.join(ROOT, "scripts", "resident_tp_one_gpu.py"), "2", kind)


@pytest.mark.parametrize("kind", ["hybrid", "resident"])
def test_persistent_tp2_failure_survived_across_devices(kind):
    _run(os.path.join(ROOT, "scripts", "persist_fallback_one_gpu.py"), "2", kind)


def test_remote_vanilla_persistent_across_devices():
    """Bob's vanilla epoch of a remote Alice as one persistent launch speaking the channel from
    inside (csrc/vanilla.hip REM), the full 256-workgroup grid on his own device, her per-batch
    run_alice on the other (scripts/vanilla_remote_one_gpu.py)."""
    _run(os.path.join(ROOT, "scripts", "vanilla_remote_one_gpu.py"), "16", "256")


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_remote_ushape_persistent_across_devices(dtype):
    """The U-shape counterpart (csrc/ushape.hip REM), 8 row groups = the full 256-workgroup grid."""
    _run(os.path.join(ROOT, "scripts", "ushape_remote_one_gpu.py"), "16", "8", dtype)
