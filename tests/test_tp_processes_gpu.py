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


def test_bench_full_schedule_with_ranks_sharing_the_gpu(tmp_path):
    """bench.py's N = 2 path end to end on the one GPU (two torchrun ranks on cuda:0, Bob
    TP = 2 over the peer-mapped all-reduce, host-staged p2p): every SISA phase completes and
    the JSON line reports the TP layout it ran."""
    import json
    out_json = tmp_path / "b.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29791", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--ranks_share_gpu", "--steps", "1", "--warmup", "0", "--num_samples", "7000",
           "--server_epochs", "1", "--json_out", str(out_json)]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=115, cwd=ROOT)
    assert out.returncode == 0, (out.stdout + out.stderr)[-3000:]
    d = json.loads(out_json.read_text())
    c = d["config"]
    assert d["n_gpus"] == 2 and c["parallelism"] == "alices2_on_2gpus+bob_tp2" and c["tp_allreduce"] == "ipc"
    assert c["ranks_share_gpu"] is True and d["value"] > 0
    assert set(c["phase_seconds"]) >= {"local_training", "server_training", "eval_breakdown", "unlearn_local",
                                       "server_retraining"}


def test_stalled_tp_peer_aborts_every_survivor_within_one_timeout():
    """A Bob TP rank that stops issuing mid-epoch: every surviving rank's fused head times out
    once on its flags, every later wait gives up at once, and the native executor raises from
    the host-pinned error mirror, so each survivor exits non-zero within 2x the wait timeout
    (scripts/tp_peer_failure_one_gpu.py; reference: a child failure ends the job,
    split_nn.py:183-186)."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "tp_peer_failure_one_gpu.py"), "3", "2.0"],
                         capture_output=True, text=True, timeout=115, cwd=ROOT)
    text = out.stdout + out.stderr
    assert out.returncode == 0, text[-3000:]
    assert out.stdout.count("aborted ") == 2 and "PASS" in out.stdout, text[-3000:]
