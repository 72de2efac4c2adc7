"""The LLaMA training step runs on the framework's own kernels: a rocprofv3 kernel
trace of LLaMA-tiny on the tape (torch autograd off) at 1 and at 3 steps; every
kernel whose call count grows with the step count is a paddle_amd kernel or a
plain fill / copy -- no ATen compute kernel is on the step path."""
import os
import shutil
import sqlite3
import subprocess
import sys
from collections import Counter

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _kernel_counts(tmp, steps, script=("llama_tiny_step.py",)):
    out = os.path.join(tmp, f"{'_'.join(script)}_s{steps}".replace(".py", ""))
    env = dict(os.environ, TMPDIR="/tmp")
    cmd = [shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3", "--kernel-trace", "-d", out, "-o", "run", "--",
           sys.executable, os.path.join(ROOT, "tools", script[0]), *script[1:], str(steps)]
    subprocess.run(cmd, check=True, cwd="/tmp", env=env, timeout=240, stdout=subprocess.DEVNULL)
    dbs = [os.path.join(d, f) for d, _, fs in os.walk(out) for f in fs if f.endswith("_results.db")]
    assert dbs, f"no rocpd database under {out}"
    c = sqlite3.connect(dbs[0])
    return Counter(name for (name,) in c.execute("select name from kernels"))


def _allowed(name):
    if "pa::" in name or not name.startswith(("void at::", "at::")) and "at::native" not in name:
        return True  # paddle_amd kernels (namespaced or extern "C" launchers) and runtime blits
    return any(k in name for k in ("FillFunctor", "copy_kernel", "direct_copy", "CatArrayBatchedCopy"))


@pytest.mark.skipif(shutil.which("rocprofv3") is None and not os.path.exists("/opt/rocm/bin/rocprofv3"),
                    reason="rocprofv3 not installed")
def test_llama_tiny_step_runs_no_aten_compute_kernels(tmp_path):
    one = _kernel_counts(str(tmp_path), 1)
    three = _kernel_counts(str(tmp_path), 3)
    per_step = {k: three[k] - one.get(k, 0) for k in three if three[k] > one.get(k, 0)}
    assert per_step, "no kernels recorded per step"
    bad = sorted(k[:120] for k in per_step if not _allowed(k))
    assert not bad, f"ATen compute kernels on the step path: {bad}"
    assert any("gemm_kernel" in k for k in per_step) and any("fa_" in k for k in per_step)


def _aten_compute(name):
    """An ATen device kernel that computes (fills / copies are data movement)."""
    return ("at::native" in name or name.startswith(("void at::", "at::"))) and not any(
        k in name for k in ("FillFunctor", "copy_kernel", "direct_copy", "CatArrayBatchedCopy"))


@pytest.mark.skipif(shutil.which("rocprofv3") is None and not os.path.exists("/opt/rocm/bin/rocprofv3"),
                    reason="rocprofv3 not installed")
@pytest.mark.parametrize("model", ["eager18", "fluid50"])
def test_resnet_step_runs_no_aten_compute_kernels(tmp_path, model):
    """DyGraph ResNet-18 bf16 (eager engine + native tensor-op dispatch) and Fluid
    ResNet-50 (static program, native op kernels): the kernels that grow with the
    step count include no ATen compute kernel."""
    one = _kernel_counts(str(tmp_path), 1, ("resnet_steps.py", model))
    three = _kernel_counts(str(tmp_path), 3, ("resnet_steps.py", model))
    per_step = {k: three[k] - one.get(k, 0) for k in three if three[k] > one.get(k, 0)}
    assert per_step, "no kernels recorded per step"
    bad = sorted(k[:120] for k in per_step if _aten_compute(k))
    assert not bad, f"ATen compute kernels on the {model} step path: {bad}"
