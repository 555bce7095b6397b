"""Native split epochs of a REMOTE Alice (`_C.SplitEpoch` roles 1 / 2, csrc/split.cpp; the
per-batch messages over the peer-mapped channel, csrc/ipc_p2p.h) across real processes on
the box's one GPU.

* bitwise the Python loop of the same placement on both sides (parameters, optimizer states,
  step counts, Bob's dropout counter) and the same per-batch message sequence (source,
  destination, bytes), vanilla and U-shape, full and partial batches
  (scripts/split_remote_one_gpu.py);
* bench.py's vanilla ws = 5 on 4 ranks with a one-shard Bob (BASELINE config 3's topology
  with `--bob_tp 1`) and U-shape ws = 2 on 2 ranks (config 2) run their whole schedules with
  the remote Alices' epochs on the native executor.

Reference hot loops: data_entities_vanilla.py:66-76, data_entities.py:65-81.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("kind,B", [("vanilla", 16), ("vanilla", 5), ("ushape", 16), ("ushape", 5)])
def test_remote_split_epoch_is_bitwise_python_loop(kind, B):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "split_remote_one_gpu.py"), kind, str(B)],
                         capture_output=True, text=True, timeout=115, cwd=ROOT)
    text = out.stdout + out.stderr
    assert out.returncode == 0, text[-3000:]
    assert out.stdout.count("message sequence equal True") == 2, text[-3000:]
    assert out.stdout.count("PASS") == 2, text[-3000:]


@pytest.mark.parametrize("B", [16, 5])
def test_remote_vanilla_persistent_bob_matches_per_batch(B):
    """Bob's side of a remote Alice's vanilla epoch as ONE persistent launch that sends and
    receives the per-batch messages on the peer-mapped channel itself (csrc/vanilla.hip REM),
    her side the unchanged run_alice: within fp32 rounding of the per-batch run_bob, one launch
    bitwise its chunked launches, run_bob's message sequence, executors mixed on one channel
    (scripts/vanilla_remote_one_gpu.py; Bob on 64 of the one GPU's CUs, a scaled tail)."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "vanilla_remote_one_gpu.py"), str(B), "64"],
                         capture_output=True, text=True, timeout=115, cwd=ROOT)
    text = out.stdout + out.stderr
    assert out.returncode == 0, text[-3000:]
    assert out.stdout.count("one launch bitwise chunked: True") == 2, text[-3000:]
    assert "message sequence equal True" in out.stdout, text[-3000:]
    assert out.stdout.count("PASS") == 2, text[-3000:]


@pytest.mark.parametrize("B,dtype", [(16, "fp32"), (5, "fp32"), (16, "bf16")])
def test_remote_ushape_persistent_bob_matches_per_batch(B, dtype):
    """Bob's side of a remote Alice's U-shape epoch (BASELINE config 2's placement) as ONE
    persistent launch exchanging run_bob's four messages per step on the peer-mapped channel
    (csrc/ushape.hip REM), her side the unchanged run_alice: within fp32 rounding of the
    per-batch run_bob (bf16: of the per-batch bf16 executor), one launch bitwise its chunked
    launches, run_bob's message sequence (scripts/ushape_remote_one_gpu.py; 2 row groups = 64 CUs)."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "ushape_remote_one_gpu.py"), str(B), "2", dtype],
                         capture_output=True, text=True, timeout=115, cwd=ROOT)
    text = out.stdout + out.stderr
    assert out.returncode == 0, text[-3000:]
    assert out.stdout.count("one launch bitwise chunked: True") == 2, text[-3000:]
    assert "message sequence equal True" in out.stdout, text[-3000:]
    assert out.stdout.count("PASS") == 2, text[-3000:]


@pytest.mark.parametrize("mode,n,ws,port", [("ushape", 2, 2, 29793), ("vanilla", 4, 5, 29795)])
def test_bench_split_schedule_with_remote_alices(tmp_path, mode, n, ws, port):
    out_json = tmp_path / "b.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--mode", mode, "--gpus", str(n), "--world_size", str(ws), "--bob_tp", "1", "--ranks_share_gpu",
           "--steps", "1", "--warmup", "0", "--num_samples", "3000", "--json_out", str(out_json)]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=115, cwd=ROOT)
    assert out.returncode == 0, (out.stdout + out.stderr)[-3000:]
    d = json.loads(out_json.read_text())
    c = d["config"]
    assert c["split_channel"] == "ipc" and d["value"] > 0, c
    k = ws - 1
    remote = k if mode == "ushape" else k - 1          # vanilla: Alice_1 shares rank 0 with Bob
    # every remote Alice's train epoch (and Alice_1's unlearn epoch when remote) ran natively
    # on both sides of its pair
    assert c["split_epochs"].get("remote_alice", 0) >= remote, c["split_epochs"]
    assert c["split_epochs"].get("remote_alice") == c["split_epochs"].get("remote_bob"), c["split_epochs"]
