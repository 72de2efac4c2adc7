"""Native dispatch of tensor ops (ops/aten_native.py -> csrc/kernels/tensor_ops.hip).

Inside a framework region every covered ATen op on a GPU tensor must run on the
HIP kernels (counted in strict.NATIVE_OPS, no entry in strict.ATEN_KERNELS) and
match the same op run by ATen outside any region (the oracle): exactly for casts,
copies, fills, comparisons and integer math; to fp32 / bf16 rounding otherwise."""
import pytest
import torch

from paddle_amd.utils import strict as S

pytestmark = pytest.mark.gpu

dev = "cuda"


def _run(fn, *args):
    S.reset()
    with S.region("test"):
        got = fn(*args)
    return got


def _check(fn, *args, atol=1e-6, rtol=1e-5, exact=False, expect_native=True):
    ref = fn(*args)
    got = _run(fn, *args)
    rep = S.report()
    if expect_native:
        assert not rep["aten_kernels"], rep
        assert rep["native_ops"], rep
    refs = ref if isinstance(ref, (tuple, list)) else (ref,)
    gots = got if isinstance(got, (tuple, list)) else (got,)
    for r, g in zip(refs, gots):
        assert g.shape == r.shape and g.dtype == r.dtype, (g.shape, r.shape, g.dtype, r.dtype)
        if exact or not r.is_floating_point():
            assert torch.equal(g, r), (g, r)
        else:
            torch.testing.assert_close(g.float(), r.float(), atol=atol, rtol=rtol, equal_nan=True)


@pytest.fixture(autouse=True)
def _count(monkeypatch):
    monkeypatch.setenv("FLAGS_count_aten", "1")
    yield


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_binary_broadcast_and_scalars(dt):
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(4, 5, 6, device=dev, generator=g).to(dt)
    y = torch.randn(5, 1, device=dev, generator=g).to(dt)
    tol = dict(atol=1e-2, rtol=1e-2) if dt == torch.bfloat16 else {}
    _check(lambda a, b: a + b, x, y, **tol)
    _check(lambda a, b: a - 2 * b, x, y, **tol)
    _check(lambda a, b: torch.add(a, b, alpha=0.5), x, y, **tol)
    _check(lambda a, b: a * b, x, y, **tol)
    _check(lambda a, b: a / (b.abs() + 1), x, y, **tol)
    _check(lambda a: a * 3.0 + 1.5, x, **tol)
    _check(lambda a: 1.0 - a, x, **tol)
    _check(lambda a: a / 4.0, x, **tol)
    _check(lambda a: a ** 2, x, **tol)
    _check(lambda a, b: torch.maximum(a, b), x, y, exact=True)
    _check(lambda a, b: torch.minimum(a, b), x, y, exact=True)
    _check(lambda a, b: a > b, x, y, exact=True)
    _check(lambda a, b: a == b, x, x, exact=True)
    _check(lambda a: torch.where(a > 0, a, torch.zeros_like(a)), x, exact=True)
    _check(lambda a: a.masked_fill(a < 0, -1.0), x, exact=True)


def test_transposed_and_noncontiguous_operands():
    x = torch.randn(64, 48, device=dev)
    y = torch.randn(48, 64, device=dev)
    _check(lambda a, b: a + b.t(), x, y, exact=True)
    _check(lambda a: a[:, ::2] * 2, x, exact=True)
    _check(lambda a: a.t().contiguous(), x, exact=True)
    z = torch.randn(2, 3, 8, 8, device=dev).to(memory_format=torch.channels_last)
    with S.region("test"):
        zz = z + 1
    assert zz.stride() == (z + 1).stride()  # channels-last activations stay channels-last
    _check(lambda a: a + 1, z, exact=True)


def test_unary_and_activations():
    x = torch.randn(1000, device=dev)
    for f in (torch.neg, torch.abs, torch.exp, torch.sigmoid, torch.tanh, torch.relu, torch.sin, torch.floor,
              torch.erf, torch.nn.functional.silu, torch.nn.functional.gelu, torch.sign):
        _check(f, x, atol=1e-5, rtol=1e-5)
    p = x.abs() + 0.1
    for f in (torch.log, torch.sqrt, torch.rsqrt, torch.reciprocal, torch.log1p):
        _check(f, p, atol=1e-5, rtol=1e-5)
    _check(lambda a: torch.nn.functional.gelu(a, approximate="tanh"), x, atol=1e-5, rtol=1e-5)
    _check(lambda a: torch.nn.functional.leaky_relu(a, 0.2), x, exact=True)
    _check(lambda a: a.clamp(-0.5, 0.5), x, exact=True)
    _check(lambda a: a.clamp(min=0.1), x, exact=True)


def test_backward_pointwise_ops():
    x = torch.randn(256, 33, device=dev)
    gr = torch.randn(256, 33, device=dev)
    _check(lambda g, a: torch.ops.aten.threshold_backward(g, a, 0.0), gr, x, exact=True)
    _check(lambda g, a: torch.ops.aten.sigmoid_backward(g, torch.sigmoid(a)), gr, x, atol=1e-6)
    _check(lambda g, a: torch.ops.aten.tanh_backward(g, torch.tanh(a)), gr, x, atol=1e-6)
    _check(lambda g, a: torch.ops.aten.gelu_backward(g, a), gr, x, atol=1e-5)
    _check(lambda g, a: torch.ops.aten.gelu_backward(g, a, approximate="tanh"), gr, x, atol=1e-5)
    _check(lambda g, a: torch.ops.aten.silu_backward(g, a), gr, x, atol=1e-5)


@pytest.mark.parametrize("src,dst", [(torch.float32, torch.bfloat16), (torch.bfloat16, torch.float32),
                                     (torch.float32, torch.float16), (torch.float32, torch.int64),
                                     (torch.int64, torch.float32), (torch.int32, torch.int64),
                                     (torch.float32, torch.bool), (torch.bool, torch.float32)])
def test_casts_exact(src, dst):
    x = (torch.randn(3, 1000, device=dev) * 50)
    x = x.to(src) if src != torch.bool else x > 0
    _check(lambda a: a.to(dst), x, exact=True)
    _check(lambda a: a.t().to(dst), x, exact=True)


def test_fill_copy_flip_cat_factories():
    x = torch.randn(7, 9, 11, device=dev)
    _check(lambda a: a.clone().zero_(), x, exact=True)
    _check(lambda a: a.clone().fill_(2.5), x, exact=True)
    _check(lambda a: torch.zeros_like(a), x, exact=True)
    _check(lambda a: torch.full_like(a, -3.0), x, exact=True)
    _check(lambda a: torch.ones(5, 4, device=dev, dtype=torch.bfloat16), x, exact=True)
    _check(lambda a: torch.zeros(3, device=dev, dtype=torch.int64), x, exact=True)
    for dims in ([0], [2], [0, 2], [1]):
        _check(lambda a, d=dims: a.flip(d), x, exact=True)
    _check(lambda a: torch.cat([a, a * 2, a[:, :3]], dim=1), x, exact=True)
    _check(lambda a: torch.stack([a, a + 1], dim=0), x, exact=True)

    def cp(a):
        out = torch.empty(9, 7, 11, device=dev, dtype=torch.bfloat16)
        out.copy_(a.transpose(0, 1))
        return out
    _check(cp, x, exact=True)


def test_integer_math():
    a = torch.randint(-50, 50, (1000,), device=dev)
    b = torch.randint(1, 9, (1000,), device=dev)
    _check(lambda x, y: x + y, a, b, exact=True)
    _check(lambda x, y: x * y - 3, a, b, exact=True)
    _check(lambda x, y: torch.div(x, y, rounding_mode="floor"), a, b, exact=True)
    _check(lambda x, y: torch.remainder(x, y), a, b, exact=True)
    _check(lambda x, y: x // y, a, b, exact=True)
    _check(lambda x: x.abs(), a, exact=True)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_reductions(dt):
    x = torch.randn(8, 300, 17, device=dev).to(dt)
    tol = dict(atol=5e-2, rtol=2e-2) if dt == torch.bfloat16 else dict(atol=1e-4, rtol=1e-5)
    _check(lambda a: a.sum(), x, **tol)
    _check(lambda a: a.sum(1), x, **tol)
    _check(lambda a: a.sum((0, 2), keepdim=True), x, **tol)
    _check(lambda a: a.sum(-1), x, **tol)
    _check(lambda a: a.mean(1), x, **tol)
    _check(lambda a: a.sum(1, dtype=torch.float32), x, **tol)
    _check(lambda a: a.amax(1), x, exact=True)
    _check(lambda a: a.max(), x, exact=True)
    _check(lambda a: a.max(1), x, exact=True)
    _check(lambda a: a.min(2), x, exact=True)
    _check(lambda a: a.argmax(1), x, exact=True)
    _check(lambda a: a.argmin(), x, exact=True)
    _check(lambda a: (a > 0).any(1), x, exact=True)
    _check(lambda a: (a > -10).all(), x, exact=True)
    _check(lambda a: torch.linalg.vector_norm(a.float(), 2, dim=1), x, **tol)


def test_tall_reduction_split_path():
    x = torch.randn(1 << 20, 4, device=dev)
    _check(lambda a: a.sum(0), x, atol=2e-3, rtol=1e-4)
    y = torch.randn(1 << 22, device=dev)
    _check(lambda a: a.sum(), y, atol=5e-2, rtol=1e-4)
    _check(lambda a: a.amax(), y, exact=True)


def test_softmax_native():
    x = torch.randn(64, 1000, device=dev)
    _check(lambda a: torch.softmax(a, -1), x, atol=1e-6)
    _check(lambda a: torch.log_softmax(a, -1), x, atol=1e-5)


def test_strict_mode_raises_on_uncovered_op(monkeypatch):
    monkeypatch.setenv("FLAGS_strict_native", "1")
    x = torch.randn(16, 16, device=dev)
    with pytest.raises(S.StrictNativeError):
        with S.region("test"):
            torch.linalg.qr(x)
    with S.region("test"):
        (x + 1).sum()  # covered: no error


def test_indexing_scans_padding_var():
    x = torch.randn(6, 5, 7, device=dev)
    idx = torch.tensor([4, 0, 0, 2], device=dev)
    _check(lambda a, i: a.index_select(1, i), x, idx, exact=True)
    _check(lambda a, i: a[i], x, idx, exact=True)
    w = torch.randn(20, 8, device=dev).to(torch.bfloat16)
    ids = torch.randint(0, 20, (3, 5), device=dev)
    _check(lambda a, i: torch.nn.functional.embedding(i, a), w, ids, exact=True)
    _check(lambda a: torch.arange(3, 17, 2, device=dev) + 0 * a.sum().long(), x, expect_native=False)
    _check(lambda a: torch.nn.functional.pad(a, (1, 2, 0, 3), value=-1.0), x, exact=True)
    _check(lambda a: a.cumsum(1), x, atol=1e-5)
    _check(lambda a: torch.var(a, 2), x, atol=1e-5)
    _check(lambda a: torch.var_mean(a, (0, 2), keepdim=True), x, atol=1e-5)


def test_matmul_handlers():
    a = torch.randn(64, 48, device=dev)
    b = torch.randn(48, 40, device=dev)
    _check(lambda x, y: x @ y, a, b, atol=1e-4, rtol=1e-4)
    _check(lambda x, y: torch.addmm(torch.ones(40, device=dev), x, y), a, b, atol=1e-4, rtol=1e-4)
    ab, bb = a.to(torch.bfloat16), b.to(torch.bfloat16)
    _check(lambda x, y: x @ y, ab, bb, atol=3e-2, rtol=2e-2)
    _check(lambda x, y: x.t() @ y.t().contiguous().t(), ab[:48, :40].contiguous(), bb, atol=3e-2, rtol=2e-2)


def test_full_int64_beyond_double_precision_and_like_memory_format():
    """the fill kernel takes a double; int64 values beyond 2**53 must stay
    exact, and *_like creation keeps the input's memory format."""
    import paddle_amd.tensor_api as T

    big = 2 ** 62 + 1
    t = T.full([2], big, "int64")
    assert t.tolist() == [big, big]
    m = torch.iinfo(torch.int64).max
    assert T.full([3], m, "int64").tolist() == [m] * 3
    from paddle_amd.ops import oplib

    z = torch.empty(4, dtype=torch.int64, device=dev)
    assert oplib.fill_(z, big).tolist() == [big] * 4
    assert oplib.fill_(z, -m).tolist() == [-m] * 4
    x = torch.randn(2, 3, 4, 5, device=dev).to(memory_format=torch.channels_last)
    y = T.ones_like(x)
    assert y.is_contiguous(memory_format=torch.channels_last) and bool((y == 1).all())
