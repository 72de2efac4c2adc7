"""Platform layer on the GPU: peer access set-up (InitP2P), peer copies, HBM
memory queries, HIP error names in EnforceError."""
import ctypes

import pytest
import torch

from paddle_amd import platform
from paddle_amd.ops import _native as N

pytestmark = pytest.mark.gpu


def test_device_memory_info_and_stats():
    free, total = platform.device_memory_info(0)
    assert total > 200 * 2**30 and 0 < free <= total  # MI355X: 288 GB HBM3E
    st = platform.memory_stats(0)
    assert st["device_total"] == total and "allocated" in st


def test_init_p2p_and_memcpy_peer():
    pairs = platform.init_p2p()
    n = platform.device_count()
    assert all(a != b and a < n and b < n for a, b in pairs)
    src = torch.arange(1 << 20, dtype=torch.float32, device="cuda:0")
    dst = torch.empty_like(src, device=f"cuda:{n - 1}")
    platform.memcpy_peer(dst, src)
    torch.cuda.synchronize()
    assert torch.equal(dst.cpu(), src.cpu())


def test_enforce_error_from_a_failing_hip_call():
    bogus = ctypes.create_string_buffer(b"\x01" * 64, 64)
    p = ctypes.c_void_p()
    rc = N.lib().pa_p2p_ipc_open(bogus, ctypes.byref(p))
    assert rc != 0
    with pytest.raises(N.EnforceError) as ei:
        N.check(rc, "pa_p2p_ipc_open")
    assert "hipError" in str(ei.value)
    # the failure does not leak into the next launch (check() cleared the last error)
    torch.ones(4, device="cuda").add_(1)
    torch.cuda.synchronize()
