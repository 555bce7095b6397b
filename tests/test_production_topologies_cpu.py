"""The BASELINE configs' production topologies end to end on CPU (gloo): the process counts and
Bob tensor-parallel degrees the 8-GPU node runs, with small data.

* `--sisa` / `--sisa --concat --concat_unlearn` / `--control` at world_size 9 on 8 ranks with
  Bob tensor-parallel over all 8 (BASELINE configs 4 and 5: one Alice per GPU, co-located
  with a Bob shard; the reference spawns world_size processes and trains every Alice
  concurrently, split_nn.py:183-186, data_entities_vanilla_sisa.py:326-334);
* `--vanilla` at world_size 5 on 4 ranks (config 3) and U-shape at world_size 2 on 2 ranks
  (config 2), both through the GPU data-plane code path (`--native_p2p_shim`: grouped p2p
  with RCCL's ordering semantics over gloo);
* bench.py (the driver's entry point) at 8 ranks: its JSON shows `bob_tp8`, `dist_world` 8
  and every phase of the schedule.
"""
import json
import os
import subprocess
import sys

import pytest

from test_distributed_cpu import _free_port, _run

pytestmark = pytest.mark.slow
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("flags,ws,np_,tp", [
    (["--sisa"], 9, 8, 8),                                   # config 4
    (["--sisa", "--concat", "--concat_unlearn"], 9, 8, 8),  # config 5
    (["--control"], 9, 8, 8),
    (["--vanilla", "--native_p2p_shim"], 5, 4, 1),          # config 3 (one-shard Bob, remote Alices)
    (["--native_p2p_shim"], 2, 2, 1),                       # config 2 (U-shape, one process per role)
])
def test_production_topology_end_to_end(tmp_path, flags, ws, np_, tp, monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    m, bob, logs = _run(tmp_path, flags, ws, np_, tp, extra=["--num_samples", str(120 * ws)])
    assert m["nprocs"] == np_ and m["bob_tp"] == tp
    assert "Bob Started Getting Tipsy" in bob and "Accuracy over all data" in bob
    for cid in range(1, ws):
        alog = (logs / f"alice{cid}.log").read_text()
        assert "Alice is going insane!" in alog and "Local Data Statistics:" in alog
    if "--vanilla" in flags:
        assert "Unlearn Request for Alice-1" in bob
        for cid in range(2, ws):
            assert f"receiving weights from Alice-{cid - 1}" in (logs / f"alice{cid}.log").read_text()
    if "--sisa" in flags or "--control" in flags:
        assert "Global training completed." in bob
    if "--control" in flags:
        assert "Filtered dataset:" in (logs / "alice1.log").read_text()
    if "--concat" in flags or ("--sisa" in flags):
        assert "Unfreezing weights for Alices-1." in bob


@pytest.mark.parametrize("mode", ["sisa", "concat", "control"])
def test_bench_eight_ranks_gloo(tmp_path, mode):
    """bench.py under torch.distributed.run with 8 CPU ranks at world_size 9 (the driver's N = 8
    launch): one JSON line with Bob tensor-parallel over all 8 ranks and the whole schedule."""
    out = tmp_path / "b.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--mode", mode, "--gpus", "8", "--steps", "1", "--warmup", "0", "--num_samples", "1200",
           "--server_epochs", "1", "--json_out", str(out)]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads(out.read_text())
    c = rec["config"]
    assert rec["n_gpus"] == 8 and rec["value"] > 0 and c["world_size"] == 9 and c["dist_world"] == 8
    assert c["parallelism"] == "alices8_on_8gpus+bob_tp8", c["parallelism"]
    assert len(c["bytes_sent_per_rank_per_step"]) == 8 and sum(c["bytes_sent_per_rank_per_step"]) > 0
    phases = (("control_local", "server_training", "eval") if mode == "control" else
              ("local_training", "server_training", "eval_breakdown", "unlearn_local", "server_retraining"))
    for p in phases:
        assert p in c["phase_seconds"], p
    # the post-run self-check: the replicated fc3 agrees bitwise across the 8 Bob ranks
    assert c["validated"] is True, c["validation"]
    assert c["validation"]["fc3_replicas_equal"] is True
