"""C++ training demo (reference paddle/fluid/train/demo): build the C++ driver with
the embedded interpreter, save the demo programs, train from C++ and see the
loss fall."""
import os
import re
import shutil
import subprocess
import sys
import sysconfig

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_cpp_demo_trainer(tmp_path):
    from paddle_amd.train_demo import save_demo_programs

    model = tmp_path / "model"
    save_demo_programs(str(model))
    exe = tmp_path / "demo_trainer"
    inc = sysconfig.get_paths()["include"]
    libdir = sysconfig.get_config_var("LIBDIR")
    ver = sysconfig.get_config_var("LDVERSION")
    src = os.path.join(ROOT, "paddle_amd", "csrc", "train_demo", "demo_trainer.cc")
    subprocess.run(["g++", "-O2", "-std=c++17", src, f"-I{inc}", f"-L{libdir}", f"-lpython{ver}",
                    f"-Wl,-rpath,{libdir}", "-o", str(exe)], check=True, timeout=120)
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""),
               PYTHONHOME=sys.base_prefix)
    out = subprocess.run([str(exe), str(model), "20"], capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    losses = [float(m) for m in re.findall(r"loss: ([0-9.eE+-]+)", out.stdout)]
    assert len(losses) == 20 and losses[-1] < losses[0], out.stdout
    assert "run_time_ms" in out.stdout
