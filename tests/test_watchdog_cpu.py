"""Failure detection (runtime/watchdog.py): heartbeats, stall reports, fault injection.

The reference has no failure handling at all (`timeout=0` RPCs hang forever);
these tests pin the new subsystem's behaviour on CPU/gloo."""
import json
import os
import socket
import time

import pytest
import torch.distributed as dist

from splitlearning_amd.runtime.watchdog import CRASH_CODE, EXIT_CODE, Watchdog, parse_fault


def _wait(pred, timeout=5.0):
    t = time.monotonic()
    while time.monotonic() - t < timeout:
        if pred():
            return True
        time.sleep(0.02)
    return False


def _pair(**kw):
    store = dist.HashStore()
    a = Watchdog(store, 0, 2, interval=0.05, policy="report", **kw)
    b = Watchdog(store, 1, 2, interval=0.05, policy="report", **kw)
    return a.start(), b.start()


def test_parse_fault():
    assert parse_fault("") is None
    assert parse_fault("2:eval_breakdown") == (2, "eval_breakdown", "crash")
    assert parse_fault("1:server_training:hang") == (1, "server_training", "hang")
    with pytest.raises(ValueError):
        parse_fault("1:x:explode")


def test_dead_peer_detected():
    a, b = _pair(dead_after=0.4)
    try:
        time.sleep(0.3)
        assert a.failed is None and b.failed is None
        b._silent.set()                          # rank 1 stops heartbeating (looks dead)
        assert _wait(lambda: a.failed == "dead_peer")
    finally:
        a.stop()
        b.stop()


def test_clean_exit_is_not_death(tmp_path):
    a, b = _pair(dead_after=0.3)
    try:
        b.stop()                                 # publishes done/1
        time.sleep(0.8)
        assert a.failed is None
    finally:
        a.stop()


def test_stall_report(tmp_path):
    store = dist.HashStore()
    a = Watchdog(store, 0, 2, interval=0.05, policy="report", stall_after=0.4, log_dir=str(tmp_path)).start()
    b = Watchdog(store, 1, 2, interval=0.05, policy="report", stall_after=0.4).start()
    try:
        a.beat("server_training")
        b.beat("eval_breakdown")
        for _ in range(5):                       # progress keeps the detector quiet
            time.sleep(0.1)
            a.beat("server_training")
        assert a.failed is None
        assert _wait(lambda: a.failed == "stall")
        rep = json.loads((tmp_path / "watchdog_rank0.json").read_text())
        assert rep["kind"] == "stall"
        assert rep["ranks"]["1"]["last_phase"] == "eval_breakdown"
        assert rep["ranks"]["0"]["last_phase"] == "server_training"
    finally:
        a.stop()
        b.stop()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cli(tmp_path, extra):
    from splitlearning_amd.runtime.launcher import main as launch_main
    argv = ["--sisa", "--world_size", "3", "--nprocs", "3", "--server_epochs", "1", "--num_samples", "600",
            "--seed", "1", "--no_tqdm", "--device", "cpu", "--datapath", str(tmp_path / "data"),
            "--log_dir", str(tmp_path / "logs"), "--master_port", str(_free_port()),
            "--watchdog_interval", "0.2"] + extra
    return launch_main(argv)


@pytest.mark.slow
def test_injected_hang_is_reported_and_aborts(tmp_path):
    import torch.multiprocessing as mp
    t0 = time.monotonic()
    with pytest.raises(mp.ProcessExitedException) as ei:
        _cli(tmp_path, ["--fault_inject", "2:eval_breakdown:hang", "--stall_after_s", "3"])
    assert ei.value.exit_code == EXIT_CODE
    assert time.monotonic() - t0 < 120
    rep = json.loads((tmp_path / "logs" / "watchdog_rank0.json").read_text())
    assert rep["kind"] == "stall" and rep["ranks"]["2"]["last_phase"] == "eval_breakdown"
    assert "[watchdog] stall" in (tmp_path / "logs" / "bob.log").read_text()


@pytest.mark.slow
def test_injected_crash_ends_the_job(tmp_path):
    import torch.multiprocessing as mp
    with pytest.raises(mp.ProcessExitedException) as ei:
        _cli(tmp_path, ["--fault_inject", "1:server_training:crash"])
    assert ei.value.exit_code == CRASH_CODE and ei.value.error_index == 1


@pytest.mark.slow
def test_watchdog_quiet_on_healthy_run(tmp_path):
    m = _cli(tmp_path, ["--stall_after_s", "60"])
    assert m is not None and m["mode"] == "sisa"
    assert not os.path.exists(tmp_path / "logs" / "watchdog_rank0.json")


@pytest.mark.slow
def test_trace_timeline(tmp_path):
    """--trace_dir: one Chrome-trace file per rank with phase spans, data-plane spans
    carrying byte counts, and the marked epoch regions."""
    _cli(tmp_path, ["--trace_dir", str(tmp_path / "tr")])
    for r in range(3):
        ev = json.loads((tmp_path / "tr" / f"trace_rank{r}.json").read_text())["traceEvents"]
        names = {e["name"] for e in ev}
        assert "server_training" in names and "eval_breakdown" in names
        comm = [e for e in ev if e.get("cat") == "comm"]
        assert comm and all("bytes_sent" in e["args"] for e in comm)
        assert all(e["dur"] >= 0 for e in ev if e.get("ph") == "X")
    ev0 = json.loads((tmp_path / "tr" / "trace_rank0.json").read_text())["traceEvents"]
    assert any(e["name"].startswith("server_epoch[alice") for e in ev0)
    assert any(e.get("cat") == "comm" and e["args"]["bytes_sent"] > 0
               for r in range(3) for e in json.loads((tmp_path / "tr" / f"trace_rank{r}.json").read_text())["traceEvents"])
