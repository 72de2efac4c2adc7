"""Depthwise NHWC bf16 convolution (csrc/kernels/dwconv.hip) vs an fp32 torch
reference: MobileNet-style 3x3 stride 1/2, channel multiplier 2, dilation,
forward and all gradients, and the nn.functional.conv2d dispatch."""
import pytest
import torch
import torch.nn.functional as F

from paddle_amd.ops import conv as C

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N,H,W,Cin,mult,k,s,p,d", [
    (4, 28, 28, 32, 1, 3, 1, 1, 1), (2, 56, 56, 64, 1, 3, 2, 1, 1), (2, 14, 14, 16, 2, 5, 1, 2, 1),
    (1, 17, 13, 24, 1, 3, 1, 2, 2)])
def test_dwconv_fwd_bwd_vs_fp32(N, H, W, Cin, mult, k, s, p, d):
    g = torch.Generator().manual_seed(H * 131 + Cin)
    x = torch.randn(N, H, W, Cin, generator=g).to(torch.bfloat16)
    w = (torch.randn(Cin * mult, 1, k, k, generator=g) * 0.2).to(torch.bfloat16)
    b = torch.randn(Cin * mult, generator=g).to(torch.bfloat16)
    xr, wr, br = (t.float().requires_grad_(True) for t in (x, w, b))
    ref = F.conv2d(xr.permute(0, 3, 1, 2), wr, br, s, p, d, groups=Cin).permute(0, 2, 3, 1)
    xd, wd, bd = (t.cuda().requires_grad_(True) for t in (x, w, b))
    y = C.dwconv2d_nhwc(xd, wd, bd, s, p, d)
    torch.testing.assert_close(y.float().cpu(), ref.detach(), rtol=2e-2, atol=2e-2)
    gy = torch.randn(ref.shape, generator=g).to(torch.bfloat16)
    ref.backward(gy.float())
    y.backward(gy.cuda())
    torch.testing.assert_close(xd.grad.float().cpu(), xr.grad, rtol=2e-2, atol=3e-2)
    scale = wr.grad.abs().max().item()
    assert (wd.grad.float().cpu() - wr.grad).abs().max().item() < 2e-2 * scale + 1e-2
    assert (bd.grad.float().cpu() - br.grad).abs().max().item() < 2e-2 * br.grad.abs().max().item() + 1e-2


def test_functional_conv2d_dispatches_depthwise():
    import paddle_amd.nn.functional as PF

    x = torch.randn(2, 8, 8, 16, device="cuda").to(torch.bfloat16)
    w = torch.randn(16, 1, 3, 3, device="cuda").to(torch.bfloat16)
    y = PF.conv2d(x, w, None, 1, 1, 1, groups=16, data_format="NHWC")
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float(), None, 1, 1, 1, 16).permute(0, 2, 3, 1)
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=5e-2)
