"""The rocprofiler-sdk tool library builds and binds on a machine without a GPU:
registration succeeds before any HIP call, the record buffer is empty, and the
timestamp source works (tests/test_device_tracer_gpu.py covers real kernels)."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_tracer_library_registers_and_binds():
    code = ("from paddle_amd.utils import device_tracer as d\n"
            "assert d.install(), d.error()\n"
            "assert d.records() == []\n"
            "t0 = d.now_ns(); t1 = d.now_ns(); assert 0 <= t1 - t0 < 10**9\n"
            "assert d.summary([]) == {}\n"
            "print('ok')\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=REPO, env=dict(os.environ, PYTHONPATH=REPO),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]
