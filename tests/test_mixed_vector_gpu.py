"""LoD offsets mirrored to the device once (framework/mixed_vector.py, the
reference's MixedVector): sequence kernels fed the same LoD reuse one upload, and
results match the host reference."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_sequence_kernels_reuse_one_offset_upload():
    from paddle_amd.framework import mixed_vector as mv
    from paddle_amd.ops import fluidk

    mv.clear()
    off = [0, 3, 3, 10, 17]
    x = torch.randn(17, device="cuda")
    s0 = mv.stats()
    y1 = fluidk.seq_softmax(x, off)
    y2 = fluidk.seq_softmax(x * 2, off)
    g = fluidk.seq_softmax_grad(y1, torch.ones_like(y1), off)
    s1 = mv.stats()
    assert s1["uploads"] - s0["uploads"] == 1 and s1["hits"] - s0["hits"] >= 2
    ref = torch.cat([torch.softmax(x[a:b].cpu(), 0) for a, b in zip(off[:-1], off[1:])])
    assert torch.allclose(y1.cpu(), ref, atol=1e-5)
    ref2 = torch.cat([torch.softmax(2 * x[a:b].cpu(), 0) for a, b in zip(off[:-1], off[1:])])
    assert torch.allclose(y2.cpu(), ref2, atol=1e-5)
    assert g.abs().max().item() < 1e-5  # d/dx of sum(softmax) is 0
    t = mv.device_offsets(off, "cuda", torch.int32)
    assert t.is_cuda and t.dtype == torch.int32 and t.cpu().tolist() == off
