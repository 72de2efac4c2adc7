"""Host-side sanitizer builds of the native runtime (the reference has
none).  The runtime sources and tests/native/runtime_selftest.cc are compiled with
AddressSanitizer + UndefinedBehaviorSanitizer, and separately ThreadSanitizer, and
the self-test must run clean.  (GPU ASan / xnack are unavailable on this pool, so
device kernels are covered by the numerics tests instead.)"""
import glob
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRCS = sorted(glob.glob(os.path.join(ROOT, "paddle_amd", "csrc", "runtime", "*.cc")))
TEST = os.path.join(ROOT, "tests", "native", "runtime_selftest.cc")


def _torch_lib():
    import torch

    return os.path.join(os.path.dirname(torch.__file__), "lib")


@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_runtime_under_sanitizer(tmp_path, san):
    # ROCm's clang: its TSan runtime intercepts pthread_cond_clockwait (GCC 11's does
    # not, which makes every std::condition_variable wait a false "double lock")
    cxx = "/opt/rocm/lib/llvm/bin/clang++"
    if not os.path.exists(cxx):
        cxx = shutil.which("clang++") or shutil.which("g++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path / "selftest")
    tl = _torch_lib()
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", f"-fsanitize={san}", "-pthread",
           "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__", TEST] + SRCS + \
          ["-o", exe, "-lz", f"-L{tl}", f"-Wl,-rpath,{tl}", "-lamdhip64"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0", UBSAN_OPTIONS="halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=300, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "runtime selftest OK" in out, out[-6000:]
    assert "Sanitizer" not in out and "runtime error" not in out, out[-6000:]
