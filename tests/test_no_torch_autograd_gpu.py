"""1-GPU training through benchmarks/train_lm.py on the framework tape with recompute,
with torch autograd and torch.utils.checkpoint patched to raise."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_RUNNER = r"""
import runpy, sys, torch
def boom(*a, **k):
    raise AssertionError("torch autograd was used")
torch.autograd.backward = boom
torch.autograd.grad = boom
torch.Tensor.backward = boom
import torch.utils.checkpoint as ckpt
ckpt.checkpoint = boom
sys.argv = ["train_lm.py"] + sys.argv[1:]
runpy.run_path(%r, run_name="__main__")
""" % os.path.join(ROOT, "benchmarks", "train_lm.py")


@pytest.mark.parametrize("model", ["gpt-tiny", "llama-tiny"])
def test_train_lm_recompute_without_torch_autograd(model):
    r = subprocess.run([sys.executable, "-c", _RUNNER, "--model", model, "--recompute", "--seq-len", "256",
                        "--micro-batch", "2", "--accum", "2", "--steps", "3", "--warmup", "1"],
                       cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["config"]["autograd"] == "tape" and rec["config"]["recompute"] is True
    ls = rec["losses"]
    assert all(l == l for l in ls) and ls[-1] < ls[0] + 0.5, ls
