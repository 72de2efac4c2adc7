"""FLAGS_strict_native=1 acceptance: the GPU op library tests (Fluid op kernels,
the fluidk kernels) and the eager-engine tests pass with every ATen device kernel
inside a framework region refused (utils/strict.py) -- i.e. they stay on the
framework's HIP kernels.  Run as one child pytest (the flag is read per call)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_op_and_eager_suites_pass_under_strict_native():
    env = dict(os.environ, FLAGS_strict_native="1")
    files = [os.path.join(ROOT, "tests", f) for f in ("test_ops_gpu.py", "test_fluidk_gpu.py",
                                                      "test_eager_engine_gpu.py")]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", *files],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
