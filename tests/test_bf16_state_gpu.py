"""Momentum on bf16 parameters without a master copy (optimizer.hip pa_momentum_p):
the DyGraph Momentum optimizer updates a bf16 model in place in one kernel per
parameter instead of the cast / scale / add / cast chain of elementwise ops.
Reference semantics: momentum_op.h (v = mu*v + g; p -= lr*v, or Nesterov)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nesterov", [False, True])
@pytest.mark.parametrize("gdt", [torch.float32, torch.bfloat16])
def test_momentum_flat_bf16_param_matches_fp32_reference(nesterov, gdt):
    from paddle_amd.ops import optim

    torch.manual_seed(0)
    n = 4099  # odd: no vector-width assumption
    p0 = torch.randn(n, device="cuda").to(torch.bfloat16)
    v0 = torch.randn(n, device="cuda")
    g = torch.randn(n, device="cuda").to(gdt)
    p, v = p0.clone(), v0.clone()
    optim.momentum_flat(p, g, v, lr=0.05, mu=0.9, nesterov=nesterov, weight_decay=1e-3, grad_scale=0.5)
    # fp32 reference of the same op on the same (bf16-valued) inputs
    pf = p0.float()
    gg = g.float() * 0.5 + 1e-3 * pf
    vr = 0.9 * v0 + gg
    pr = pf - (0.05 * (gg + 0.9 * vr) if nesterov else 0.05 * vr)
    torch.testing.assert_close(v, vr, rtol=1e-6, atol=1e-6)
    assert p.dtype == torch.bfloat16
    # one bf16 rounding of the fp32 result (FMA contraction may move a tie: <= 1 ulp)
    torch.testing.assert_close(p.float(), pr.to(torch.bfloat16).float(), rtol=2 ** -7, atol=1e-6)


def test_dygraph_momentum_bf16_model_uses_native_update():
    import paddle_amd.ops._native as N
    from paddle_amd.optimizer.optimizer import Momentum

    N.lib()
    w = torch.randn(64, 32, device="cuda").to(torch.bfloat16).requires_grad_(True)
    w.grad = torch.randn(64, 32, device="cuda").to(torch.bfloat16)
    ref = w.detach().float().clone()
    opt = Momentum(learning_rate=0.1, momentum=0.9, parameters=[w])
    opt.step()
    # first step: v = g, p -= lr * g
    want = (ref - 0.1 * w.grad.float()).to(torch.bfloat16)
    torch.testing.assert_close(w.detach().float(), want.float(), rtol=2 ** -7, atol=1e-6)


def test_bn_bf16_running_stats_native_update():
    """BatchNorm of a bf16-cast model keeps bf16 running statistics: they are updated
    by one native launch (conv_aux.hip pa_bn_running_update) from the batch mean /
    rstd; checked against the fp32 formula (unbiased variance, momentum blend)."""
    from paddle_amd.ops import conv as CV

    torch.manual_seed(0)
    N_, H, W, C = 4, 5, 6, 32
    x = (torch.randn(N_, H, W, C, device="cuda") * 2 + 0.5).to(torch.bfloat16)
    w = torch.rand(C, device="cuda") + 0.5
    b = torch.randn(C, device="cuda")
    rm = torch.randn(C, device="cuda").to(torch.bfloat16)
    rv = (torch.rand(C, device="cuda") + 0.5).to(torch.bfloat16)
    rm0, rv0 = rm.float().clone(), rv.float().clone()
    CV._BatchNormNHWC.apply(x, w, b, rm, rv, 0.9, 1e-5, False, None)
    torch.cuda.synchronize()
    xf = x.float().reshape(-1, C)
    mean, var_unb = xf.mean(0), xf.var(0, unbiased=True)
    torch.testing.assert_close(rm.float(), (0.9 * rm0 + 0.1 * mean).to(torch.bfloat16).float(), rtol=2 ** -7, atol=1e-3)
    torch.testing.assert_close(rv.float(), (0.9 * rv0 + 0.1 * var_unb).to(torch.bfloat16).float(), rtol=2 ** -6, atol=1e-3)
