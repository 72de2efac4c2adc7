"""C++ training demo (reference paddle/fluid/train/demo): the driver links the
native executor (libpaddle_amd_native.so, no Python), trains the demo network from
its own startup initialisation and the loss falls.  The trajectory match against
the Python executor is tests/test_native_cpu.py::test_cpp_demo_trainer_matches_python."""
import os
import re
import shutil
import subprocess

import pytest

from paddle_amd import _build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_cpp_demo_trainer(tmp_path):
    from paddle_amd.train_demo import save_demo_programs

    model = tmp_path / "model"
    save_demo_programs(str(model))
    exe = _build.build_native_program(os.path.join(ROOT, "paddle_amd", "csrc", "train_demo", "demo_trainer.cc"),
                                      str(tmp_path / "demo_trainer"))
    out = subprocess.run([exe, str(model), "20"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    losses = [float(m) for m in re.findall(r"loss: ([0-9.eE+-]+)", out.stdout)]
    assert len(losses) == 20 and losses[-1] < losses[0], out.stdout
    assert "run_time_ms" in out.stdout
    # the binary is a native program: no libpython in its dependencies
    ldd = subprocess.run(["ldd", exe], capture_output=True, text=True).stdout
    assert "libpython" not in ldd and "libpaddle_amd_native" in ldd
