"""Failure detection and elastic restart: a rank killed by fault
injection (or stuck and caught by the watchdog) makes the launcher restart the
process group, which resumes from the newest complete checkpoint and ends with the
same parameters as an uninterrupted run."""
import os
import subprocess
import sys

import pytest
import torch

from paddle_amd.distributed.elastic import CheckpointManager

HERE = os.path.dirname(os.path.abspath(__file__))
SCRIPT = os.path.join(HERE, "elastic_train_script.py")


def _launch(tmp, port, extra_env=None, restarts=1, steps=8):
    env = dict(os.environ, **(extra_env or {}))
    env.pop("PADDLE_FAULT_INJECT", None) if not extra_env or "PADDLE_FAULT_INJECT" not in extra_env else None
    out = os.path.join(tmp, "w.pt")
    cmd = [sys.executable, "-m", "paddle_amd.distributed.launch", "--nproc_per_node", "2",
           "--master_port", str(port), "--max_restarts", str(restarts), "--log_dir", os.path.join(tmp, "logs"),
           SCRIPT, os.path.join(tmp, "ckpt"), out, str(steps)]
    r = subprocess.run(cmd, env=env, cwd=os.path.dirname(HERE), timeout=240, capture_output=True, text=True)
    return r, out


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_restart_after_injected_failure_matches_clean_run(tmp_path):
    clean, out0 = _launch(str(tmp_path / "clean"), _free_port(), restarts=0)
    assert clean.returncode == 0, clean.stderr[-2000:]
    faulty, out1 = _launch(str(tmp_path / "faulty"), _free_port(), {"PADDLE_FAULT_INJECT": "1:5"}, restarts=1)
    assert faulty.returncode == 0, faulty.stderr[-2000:]
    assert "restarting" in faulty.stderr
    assert torch.allclose(torch.load(out0, weights_only=True), torch.load(out1, weights_only=True), atol=1e-6)
    logs = os.listdir(tmp_path / "faulty" / "logs")
    assert any("restart1" in f for f in logs)


def test_watchdog_catches_hang_and_group_restarts(tmp_path):
    r, out = _launch(str(tmp_path), _free_port(), {"PADDLE_FAULT_INJECT": "0:3:hang", "TEST_WATCHDOG_S": "2"},
                     restarts=1)
    assert r.returncode == 0, r.stderr[-2000:]
    assert os.path.exists(out)
    log0 = open(tmp_path / "logs" / "workerlog.0").read()
    assert "[watchdog:rank0]" in log0


def test_checkpoint_manager_rotation_and_success_marker(tmp_path):
    m = CheckpointManager(str(tmp_path), max_num_checkpoints=2)
    for s in (1, 3, 5):
        m.save(s, {"model": {"w": torch.full((2,), float(s))}})
    os.makedirs(m.dir(7))          # incomplete (no _SUCCESS): ignored by latest()
    serial, state = m.load()
    assert serial == 5 and torch.equal(state["model"]["w"], torch.full((2,), 5.0))
    assert sorted(os.listdir(tmp_path)) == ["checkpoint_3", "checkpoint_5", "checkpoint_7"]
