"""csrc/fastops on the device: the flat elementwise launches through the C++ entry
match torch for add / scale / cast / copy / fill across dtypes, broadcast or strided
operands are declined (the Python path handles them), and the framework's direct
callers (oplib.add_ / fill_) run through it."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_fastops_elementwise_matches_torch():
    from paddle_amd.ops import _native as N, aten_native as A

    F = N.fastops()
    assert F is not None
    st = N.stream()
    for dt in (torch.float32, torch.bfloat16):
        x = torch.randn(1000, 7, device="cuda").to(dt)
        y = torch.randn(1000, 7, device="cuda").to(dt)
        out = torch.empty_like(x)
        assert F.ew2(A.B["add"], -1, out, x, y, 1.0, 0.0, st)
        torch.testing.assert_close(out.float(), (x.float() + y.float()).to(dt).float(), rtol=1e-2, atol=1e-2)
        assert F.ew1(A.U["affine"], -1, out, x, 2.5, 1.0, st)
        torch.testing.assert_close(out.float(), (x.float() * 2.5 + 1.0).to(dt).float(), rtol=1e-2, atol=1e-2)
        o32 = torch.empty(x.shape, device="cuda")
        assert F.ew1(A.U["copy"], -1, o32, x, 0.0, 0.0, st)
        assert torch.equal(o32, x.float())
        assert F.ew0(A.U["fill"], -1, out, 3.0, 0.0, st)
        assert torch.all(out == 3)
    for src, dc, dt in ((torch.float32, 1, torch.bfloat16), (torch.bfloat16, 0, torch.float32),
                        (torch.int64, 0, torch.float32), (torch.float32, 4, torch.int64)):
        x = (torch.randn(33, 8, device="cuda") * 10).to(src)
        r = F.cast(x, dc)
        assert r.dtype == dt and torch.equal(r, x.to(dt))
    # broadcast / non-contiguous operands: declined
    x = torch.randn(8, 4, device="cuda")
    assert not F.ew2(A.B["add"], -1, torch.empty_like(x), x, torch.randn(4, device="cuda"), 1.0, 0.0, st)
    assert not F.ew1(A.U["copy"], -1, torch.empty(4, 8, device="cuda"), x.t(), 0.0, 0.0, st)


def test_direct_callers_use_fastops():
    from paddle_amd.ops import _native as N, oplib

    g = torch.ones(64, device="cuda", dtype=torch.bfloat16)
    oplib.add_(g, torch.full_like(g, 2.0))
    assert torch.all(g == 3)
    oplib.fill_(g, 0.0)
    assert not torch.any(g)
    assert N.fastops() is not None
