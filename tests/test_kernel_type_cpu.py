"""Typed kernel selection + input data transform (framework/op_kernel_type.py;
reference framework/operator.cc:657-795, data_transform.cc, op_kernel_type.h)."""
import pytest
import torch

from paddle_amd.framework import core
from paddle_amd.framework import op_kernel_type as K
from paddle_amd.framework import registry as R

SEEN = []


@R.register_op("_kt_test_op", ["X", "Y?"], ["Out"], {"data_format": "AnyLayout"}, grad=None)
def _plain(ctx):
    SEEN.append(("plain", ctx.input("X").dtype, tuple(ctx.input("X").shape)))
    ctx.set_output("Out", ctx.input("X") * 2)


@K.register_op_kernel("_kt_test_op", "CPU", [torch.float64])
def _f64(ctx):
    x = ctx.input("X")
    SEEN.append(("f64", x.dtype, tuple(x.shape), ctx.input("Y").dtype if ctx.has_input("Y") else None))
    ctx.set_output("Out", x * 3)


@K.register_op_kernel("_kt_test_op", "CPU", [torch.float32], layout=K.DataLayout.NHWC)
def _nhwc(ctx):
    x = ctx.input("X")
    SEEN.append(("nhwc", x.dtype, tuple(x.shape)))
    ctx.set_output("Out", x)


def _run(ins, attrs=None):
    SEEN.clear()
    info = R.get_op_info("_kt_test_op")
    ctx = R.KernelContext("_kt_test_op", ins, {"Out": ["o"]}, dict(info.attrs, **(attrs or {})))
    R.run_kernel(info, ctx)
    return SEEN[-1], ctx.results["Out"][0]


def test_exact_kernel_by_dtype():
    seen, out = _run({"X": [core.LoDTensor(torch.ones(2, 3, dtype=torch.float64))]})
    assert seen[0] == "f64" and torch.equal(out.tensor, torch.full((2, 3), 3.0, dtype=torch.float64))


def test_dtype_fallback_casts_inputs():
    # no (CPU, fp16) kernel: the inputs are cast to the fp64 kernel's type; Y too
    seen, out = _run({"X": [core.LoDTensor(torch.ones(2, 3, dtype=torch.float16))],
                      "Y": [core.LoDTensor(torch.ones(1, dtype=torch.float32))]})
    assert seen[0] == "f64" and seen[1] == torch.float64 and seen[3] == torch.float64


def test_layout_transform_to_kernel_layout():
    x = torch.arange(2 * 3 * 4 * 5, dtype=torch.float32).reshape(2, 3, 4, 5)
    lt = core.LoDTensor(x, layout=K.DataLayout.NCHW)
    seen, out = _run({"X": [lt]}, {"data_format": "NHWC"})
    assert seen[0] == "nhwc" and seen[2] == (2, 4, 5, 3)
    assert torch.equal(out.tensor, x.permute(0, 2, 3, 1))
    assert out.tensor is not lt.tensor and lt.tensor.shape == (2, 3, 4, 5)  # scope variable untouched


def test_expected_kernel_type_and_select():
    info = R.get_op_info("_kt_test_op")
    ctx = R.KernelContext("_kt_test_op", {"X": [core.LoDTensor(torch.ones(1, dtype=torch.float64))]}, {"Out": ["o"]},
                          dict(info.attrs))
    key = K.expected_kernel_type(info, ctx)
    assert key == K.OpKernelType("CPU", torch.float64)
    fn, kt = K.select(info, key)
    assert fn is _f64 and kt == key
    assert "data_type[torch.float64]" in str(key)


def test_need_transform_rules():
    a = K.OpKernelType("CPU", torch.float32)
    assert not K.need_transform(a, K.OpKernelType("CPU", torch.float32))
    assert K.need_transform(a, K.OpKernelType("GPU", torch.float32))
    assert K.need_transform(a, K.OpKernelType("CPU", torch.bfloat16))
    assert not K.need_transform(K.OpKernelType("CPU", None), K.OpKernelType("CPU", torch.float32))  # int inputs
    assert K.need_transform(K.OpKernelType("CPU", torch.float32, "NCHW"), K.OpKernelType("CPU", torch.float32, "NHWC"))
    assert not K.need_transform(K.OpKernelType("CPU", torch.float32, "NCHW"), K.OpKernelType("CPU", torch.float32))


def test_typed_gpu_kernels_registered_for_native_ops():
    from paddle_amd import operators  # noqa: F401

    for op in ("roi_pool", "warpctc", "multiclass_nms", "box_coder", "iou_similarity", "adamax", "ftrl", "rmsprop",
               "fake_quantize_abs_max"):
        info = R.get_op_info(op)
        assert any(k.place == "GPU" and k.library == K.LibraryType.NATIVE for k in info.kernels), op
        # CPU places still run the place-agnostic kernel
        fn, kt = K.select(info, K.OpKernelType("CPU", torch.float32))
        assert kt is None and fn is info.kernel


def test_gpu_place_moves_host_inputs(monkeypatch):
    """The device transform: a GPU-place kernel receives its CPU inputs on the
    device (checked here with a fake device move, no GPU needed)."""
    moved = []
    orig = K.transform_data

    def fake(exp_t, var_t, t):
        moved.append((var_t.place, exp_t.place))
        return t

    monkeypatch.setattr(K, "transform_data", fake)
    info = R.get_op_info("_kt_test_op")
    ctx = R.KernelContext("_kt_test_op", {"X": [core.LoDTensor(torch.ones(1))]}, {"Out": ["o"]}, dict(info.attrs))
    K.prepare_inputs(info, ctx, K.OpKernelType("GPU", torch.float32))
    assert moved == [("CPU", "GPU")]
    monkeypatch.setattr(K, "transform_data", orig)
