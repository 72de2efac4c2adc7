"""More table-driven operator tests (forward vs numpy, gradients vs finite
differences) for op types not covered by test_ops_cpu.py.  Mirrors the
reference's unittests (test_activation_op.py brelu / hard_shrink / softshrink /
stanh / thresholded_relu / soft_relu / hard_sigmoid, test_arg_min_max_op.py,
test_compare_op.py, test_logical_op.py, test_maxout_op.py, test_norm_op.py,
test_clip_by_norm_op.py, test_*_loss_op.py, test_crop_op.py, test_multiplex_op.py,
test_minus_op.py, test_reverse_op.py, test_pad2d_op.py, test_lrn_op.py,
test_row_conv_op.py, test_conv_shift_op.py, test_shuffle_channel_op.py,
test_sequence_*.py, test_spp_op.py, test_unstack_op.py, ...).  The same cases run
on the HIP device in tests/test_ops_gpu.py."""
import numpy as np
import pytest

from op_test import OpTest

rng = np.random.RandomState(321)


def R(*shape, lo=-1.0, hi=1.0):
    return rng.uniform(lo, hi, shape).astype("float32")


def _away(x, pts=(0.0,), eps=0.05):
    """Move values off the kinks of piecewise ops so finite differences are valid."""
    x = x.copy()
    for p in pts:
        m = np.abs(x - p) < eps
        x[m] = p + np.sign(x[m] - p + 1e-9) * eps * 2
    return x


MORE = []


def case(op, inputs, outputs, attrs=None, grad=None, grad_out="Out", tol=0.005, atol=1e-5, no_check=()):
    MORE.append((op, inputs, outputs, attrs or {}, grad, grad_out, tol, atol, no_check))


# ------------------------------------------------------------------ activations with parameters
xa = _away(R(4, 6, lo=-2, hi=2), (0.0, -0.5, 0.5, 1.0, -1.0))
case("brelu", {"X": xa * 10}, {"Out": np.clip(xa * 10, 1.0, 6.0)}, {"t_min": 1.0, "t_max": 6.0})
case("hard_shrink", {"X": xa}, {"Out": np.where(np.abs(xa) > 0.5, xa, 0)}, {"threshold": 0.5}, grad=["X"])
case("softshrink", {"X": xa}, {"Out": np.where(xa > 0.5, xa - 0.5, np.where(xa < -0.5, xa + 0.5, 0))},
     {"lambda": 0.5}, grad=["X"])
case("thresholded_relu", {"X": xa}, {"Out": np.where(xa > 1.0, xa, 0)}, {"threshold": 1.0})
case("stanh", {"X": xa}, {"Out": 1.7159 * np.tanh(0.67 * xa)}, {"scale_a": 0.67, "scale_b": 1.7159}, grad=["X"])
case("soft_relu", {"X": xa}, {"Out": np.log1p(np.exp(np.clip(xa, -40, 40)))}, {"threshold": 40.0}, grad=["X"],
     tol=0.01)
case("hard_sigmoid", {"X": xa}, {"Out": np.clip(0.2 * xa + 0.5, 0, 1)}, {"slope": 0.2, "offset": 0.5})
case("ceil", {"X": xa}, {"Out": np.ceil(xa)})
case("floor", {"X": xa}, {"Out": np.floor(xa)})
case("round", {"X": xa}, {"Out": np.round(xa)})
xp = R(3, 5, lo=0.2, hi=2.0)
case("rsqrt", {"X": xp}, {"Out": 1 / np.sqrt(xp)}, grad=["X"], tol=0.01)
case("log_softmax", {"X": xa}, {"Out": xa - xa.max(-1, keepdims=True)
                                - np.log(np.exp(xa - xa.max(-1, keepdims=True)).sum(-1, keepdims=True))},
     grad=["X"], tol=0.01)

# ------------------------------------------------------------------ arg / compare / logical
xm = R(3, 5, 4)
case("arg_max", {"X": xm}, {"Out": xm.argmax(1)}, {"axis": 1})
case("arg_min", {"X": xm}, {"Out": xm.argmin(2)}, {"axis": 2})
xs_ = R(4, 7)
case("argsort", {"X": xs_}, {"Out": np.sort(xs_, -1), "Indices": np.argsort(xs_, -1, kind="stable")}, {"axis": -1})
a, b = rng.randint(0, 3, (4, 5)).astype("float32"), rng.randint(0, 3, (4, 5)).astype("float32")
case("equal", {"X": a, "Y": b}, {"Out": a == b})
case("not_equal", {"X": a, "Y": b}, {"Out": a != b})
case("greater_than", {"X": a, "Y": b}, {"Out": a > b})
case("greater_equal", {"X": a, "Y": b}, {"Out": a >= b})
case("less_equal", {"X": a, "Y": b}, {"Out": a <= b})
ba, bb = rng.rand(3, 4) > 0.5, rng.rand(3, 4) > 0.5
case("logical_and", {"X": ba, "Y": bb}, {"Out": ba & bb})
case("logical_or", {"X": ba, "Y": bb}, {"Out": ba | bb})
case("logical_xor", {"X": ba, "Y": bb}, {"Out": ba ^ bb})
case("logical_not", {"X": ba}, {"Out": ~ba})

# ------------------------------------------------------------------ elementwise / reduce extras
xe, ye = R(3, 4), R(3, 4)
case("elementwise_min", {"X": xe, "Y": ye}, {"Out": np.minimum(xe, ye)})
ie, je = rng.randint(1, 20, (3, 4)).astype("int64"), rng.randint(1, 6, (3, 4)).astype("int64")
case("elementwise_mod", {"X": ie, "Y": je}, {"Out": ie % je})
case("elementwise_floordiv", {"X": ie, "Y": je}, {"Out": ie // je})
xr = R(3, 4, 5, lo=0.5, hi=1.5)
case("reduce_min", {"X": xr}, {"Out": xr.min(1)}, {"dim": [1]})
case("reduce_prod", {"X": xr}, {"Out": xr.prod(2)}, {"dim": [2]}, grad=["X"], tol=0.01)
case("minus", {"X": xe, "Y": ye}, {"Out": xe - ye}, grad=["X", "Y"])
case("squared_l2_norm", {"X": xe}, {"Out": np.array([(xe ** 2).sum()], "float32")}, grad=["X"], atol=1e-4)

# ------------------------------------------------------------------ shape / layout
xt = R(2, 3, 4)
case("flatten", {"X": xt}, {"Out": xt.reshape(2, 12)}, {"axis": 1})
case("reshape2", {"X": xt}, {"Out": xt.reshape(6, 4)}, {"shape": [-1, 4]}, no_check=("XShape",))
case("transpose2", {"X": xt}, {"Out": xt.transpose(2, 0, 1)}, {"axis": [2, 0, 1]}, no_check=("XShape",))
case("reverse", {"X": xt}, {"Out": xt[:, ::-1, ::-1].copy()}, {"axis": [1, 2]}, grad=["X"])
case("unstack", {"X": xt}, {"Y": [("u0", xt[:, 0]), ("u1", xt[:, 1]), ("u2", xt[:, 2])]}, {"axis": 1, "num": 3})
xc = R(3, 5)
case("crop", {"X": xc}, {"Out": xc[1:3, 2:5]}, {"offsets": [1, 2], "shape": [2, 3]}, grad=["X"])
x4 = R(2, 8, 3, 3)
g = 2
case("shuffle_channel", {"X": x4}, {"Out": x4.reshape(2, g, 4, 3, 3).transpose(0, 2, 1, 3, 4).reshape(2, 8, 3, 3)},
     {"group": g})
case("maxout", {"X": x4}, {"Out": x4.reshape(2, 4, 2, 3, 3).max(2)}, {"groups": 2})
ids = np.array([[1], [0], [2]], dtype="int32")
m0, m1, m2 = R(3, 4), R(3, 4), R(3, 4)
case("multiplex", {"Ids": ids, "X": [("m0", m0), ("m1", m1), ("m2", m2)]},
     {"Out": np.stack([m1[0], m0[1], m2[2]])})
case("size", {"Input": xt}, {"Out": np.array([xt.size], "int64")})
case("shape", {"Input": xt}, {"Out": np.array(xt.shape, "int32")})
case("fill_constant_batch_size_like", {"Input": R(5, 2)}, {"Out": np.full((5, 3), 2.5, "float32")},
     {"shape": [-1, 3], "value": 2.5, "dtype": 5})
case("assign", {"X": xt}, {"Out": xt})

# ------------------------------------------------------------------ normalisation / clipping
xn = R(3, 4, 2)
case("norm", {"X": xn}, {"Out": xn / np.sqrt((xn ** 2).sum(1, keepdims=True) + 1e-10)}, {"axis": 1, "epsilon": 1e-10},
     grad=["X"], tol=0.01, no_check=("Norm",))
big = R(4, 5) * 3
case("clip_by_norm", {"X": big}, {"Out": big * (1.0 / max(1.0, np.sqrt((big ** 2).sum())))}, {"max_norm": 1.0})

# ------------------------------------------------------------------ losses
lg = R(6, 1)
lb = rng.randint(0, 2, (6, 1)).astype("float32")
case("hinge_loss", {"Logits": lg, "Labels": lb}, {"Loss": np.maximum(0, 1 - (2 * lb - 1) * lg)}, grad_out="Loss")
x1, x2 = R(5, 1), R(5, 1)
lr_ = np.where(rng.rand(5, 1) > 0.5, 1, -1).astype("float32")
case("margin_rank_loss", {"X1": x1, "X2": x2, "Label": lr_}, {"Out": np.maximum(0, -lr_ * (x1 - x2) + 0.1)},
     {"margin": 0.1}, no_check=("Activated",))
lab01 = rng.randint(0, 2, (5, 1)).astype("float32")
case("rank_loss", {"Label": lab01, "Left": x1, "Right": x2},
     {"Out": np.log1p(np.exp(x1 - x2)) - lab01 * (x1 - x2)}, grad=["Left", "Right"], tol=0.01)
mx, my = R(6, 1) * 2, np.where(rng.rand(6, 1) > 0.5, 1, 0).astype("float32")
z = mx * (2 * my - 1)
case("modified_huber_loss", {"X": mx, "Y": my},
     {"Out": np.where(z < -1, -4 * z, np.where(z < 1, (1 - z) ** 2, 0))}, no_check=("IntermediateVal",))
kx = np.log(np.clip(R(4, 5, lo=0.05, hi=1), 1e-3, 1))
kt = R(4, 5, lo=0.05, hi=1)
case("kldiv_loss", {"X": kx, "Target": kt}, {"Loss": np.array([(kt * (np.log(kt) - kx)).mean()], "float32")},
     {"reduction": "mean"}, grad=["X"], grad_out="Loss", tol=0.02)

# ------------------------------------------------------------------ image-ish ops
xi = R(2, 3, 5, 6)
case("pad2d", {"X": xi}, {"Out": np.pad(xi, ((0, 0), (0, 0), (1, 2), (3, 1)), constant_values=0.5)},
     {"paddings": [1, 2, 3, 1], "mode": "constant", "pad_value": 0.5}, grad=["X"])
case("pad2d", {"X": xi}, {"Out": np.pad(xi, ((0, 0), (0, 0), (1, 2), (3, 1)), mode="reflect")},
     {"paddings": [1, 2, 3, 1], "mode": "reflect"}, grad=["X"])
case("pad2d", {"X": xi}, {"Out": np.pad(xi, ((0, 0), (0, 0), (1, 2), (3, 1)), mode="edge")},
     {"paddings": [1, 2, 3, 1], "mode": "edge"}, grad=["X"])


def _lrn(x, n, k, alpha, beta):
    C = x.shape[1]
    pre = (n - 1) // 2
    mid = np.empty_like(x)
    for c in range(C):
        lo, hi = max(0, c - pre), min(C, c - pre + n)
        mid[:, c] = k + alpha * (x[:, lo:hi] ** 2).sum(1)
    return x * mid ** (-beta), mid


xl = R(2, 6, 3, 3)
lo_, mid_ = _lrn(xl, 5, 2.0, 1e-2, 0.75)
case("lrn", {"X": xl}, {"Out": lo_, "MidOut": mid_}, {"n": 5, "k": 2.0, "alpha": 1e-2, "beta": 0.75}, grad=["X"],
     tol=0.01)
# spp_op.h windows for H=5, W=6 at 2 bins: kernel (3, 3), padding (1, 0): rows {0,1} / {2,3,4}
case("spp", {"X": xi}, {"Out": np.concatenate(
    [xi.max((2, 3)),
     np.stack([xi[:, :, :2, :3].max((2, 3)), xi[:, :, :2, 3:].max((2, 3)),
               xi[:, :, 2:, :3].max((2, 3)), xi[:, :, 2:, 3:].max((2, 3))], 2).reshape(2, -1)], 1)},
     {"pyramid_height": 2, "pooling_type": "max"})
case("spp", {"X": xi}, {"Out": np.concatenate(
    [xi.mean((2, 3)),
     np.stack([xi[:, :, :2, :3].mean((2, 3)), xi[:, :, :2, 3:].mean((2, 3)),
               xi[:, :, 2:, :3].mean((2, 3)), xi[:, :, 2:, 3:].mean((2, 3))], 2).reshape(2, -1)], 1)},
     {"pyramid_height": 2, "pooling_type": "avg"})

# ------------------------------------------------------------------ sequences (LoD)
xq = R(7, 3)
case("row_conv", {"X": (xq, [[3, 4]]), "Filter": R(2, 3)}, {"Out": None}, grad=["X", "Filter"], tol=0.01)


def _seq_softmax(x, lens):
    out, s = np.empty_like(x), 0
    for n in lens:
        e = np.exp(x[s:s + n] - x[s:s + n].max())
        out[s:s + n] = e / e.sum()
        s += n
    return out


xsq = R(6, 1)
case("sequence_softmax", {"X": (xsq, [[2, 4]])}, {"Out": _seq_softmax(xsq, [2, 4])}, grad=["X"], tol=0.01)
case("sequence_mask", {"X": np.array([1, 3, 2], "int64")},
     {"Y": (np.arange(4)[None, :] < np.array([1, 3, 2])[:, None]).astype("int64")}, {"maxlen": 4, "out_dtype": 3})
xse = R(3, 2)
case("sequence_expand", {"X": (xse, [[1, 1, 1]]), "Y": (R(6, 1), [[2, 3, 1]])},
     {"Out": np.repeat(xse, [2, 3, 1], 0)}, grad=["X"])
xsc1, xsc2 = R(3, 2), R(4, 2)
case("sequence_concat", {"X": [("q0", (xsc1, [[1, 2]])), ("q1", (xsc2, [[3, 1]]))]},
     {"Out": np.concatenate([xsc1[:1], xsc2[:3], xsc1[1:], xsc2[3:]])})
# two LoD levels (reference sequence_concat_op.h ConcatLoD): level 0 joins the finest
# sequences, level 1 the outer ones; axis 1 joins the columns of equal-length slices
xsc3, xsc4 = R(4, 2), R(4, 2)
case("sequence_concat", {"X": [("q2", (xsc3, [[2, 1], [1, 2, 1]])), ("q3", (xsc4, [[1, 2], [2, 1, 1]]))]},
     {"Out": np.concatenate([xsc3[0:1], xsc4[0:2], xsc3[1:3], xsc4[2:3], xsc3[3:4], xsc4[3:4]])}, {"level": 0})
case("sequence_concat", {"X": [("q4", (xsc3, [[2, 1], [1, 2, 1]])), ("q5", (xsc4, [[1, 2], [2, 1, 1]]))]},
     {"Out": np.concatenate([xsc3[0:3], xsc4[0:2], xsc3[3:4], xsc4[2:4]])}, {"level": 1})
case("sequence_concat", {"X": [("q6", (xsc3, [[1, 3]])), ("q7", (xsc4, [[1, 3]]))]},
     {"Out": np.concatenate([xsc3, xsc4], 1)}, {"axis": 1})
xer = np.array([[2], [1], [2], [3], [1], [5]], "int64")
case("sequence_erase", {"X": (xer, [[4, 2]])}, {"Out": np.array([[3], [5]], "int64")}, {"tokens": [2, 1]})
xen = np.array([[1], [2], [3], [4], [5]], "int64")
case("sequence_enumerate", {"X": (xen, [[3, 2]])},
     {"Out": np.array([[1, 2], [2, 3], [3, 0], [4, 5], [5, 0]], "int64")}, {"win_size": 2, "pad_value": 0})
xsr = R(4, 6)
case("sequence_reshape", {"X": (xsr, [[1, 3]])}, {"Out": xsr.reshape(12, 2)}, {"new_dim": 2})
xcs, ycs = R(3, 5), R(3, 3)


def _conv_shift(x, y):
    M, N = x.shape[1], y.shape[1]
    out = np.zeros_like(x)
    for i in range(M):
        for j in range(N):
            out[:, i] += x[:, (i + j - (N - 1) // 2) % M] * y[:, j]
    return out


case("conv_shift", {"X": xcs, "Y": ycs}, {"Out": _conv_shift(xcs, ycs)}, grad=["X", "Y"], tol=0.01)
bx, by, bw = R(3, 4), R(3, 5), R(2, 4, 5)
case("bilinear_tensor_product", {"X": bx, "Y": by, "Weight": bw},
     {"Out": np.einsum("bi,kij,bj->bk", bx, bw, by)}, grad=["X", "Y", "Weight"], tol=0.01)


@pytest.mark.parametrize("op,inputs,outputs,attrs,grad,grad_out,tol,atol,no_check", MORE,
                         ids=[f"{c[0]}_{i}" for i, c in enumerate(MORE)])
def test_op_more(op, inputs, outputs, attrs, grad, grad_out, tol, atol, no_check):
    t = OpTest()
    t.op_type, t.inputs, t.attrs = op, inputs, attrs
    t.outputs = {k: v for k, v in outputs.items() if v is not None}
    if t.outputs:
        t.check_output(atol=atol, rtol=1e-4, no_check_set=no_check)
    else:
        t.outputs = {k: np.zeros(1, "float32") for k in outputs}
        t.check_output(exec_only=True)
    t.outputs = {k: (v if v is not None else np.zeros(1, "float32")) for k, v in outputs.items()}
    if grad:
        t.check_grad(grad, [grad_out], max_relative_error=tol, places=[__import__("paddle_amd").fluid.CPUPlace()])
