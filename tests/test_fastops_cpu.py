"""The C++ launch entry for flat elementwise ops (csrc/fastops) builds in-tree, loads
next to the kernel library and declines what it does not cover (host tensors,
mismatched shapes) so the callers take their general path."""
import torch

from paddle_amd.ops import _native as N


def test_fastops_loads_and_declines_host_tensors():
    F = N.fastops()
    assert F is not None, "paddle_amd/lib/pa_fastops.so missing: run __graft_entry__.build()"
    x = torch.ones(16)
    assert F.ew2(50, -1, x, x, x, 1.0, 0.0, 0) is False
    assert F.ew0(1, -1, x, 0.0, 0.0, 0) is False
