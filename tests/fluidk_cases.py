"""Shared cases for the Fluid operator-library kernels (csrc/kernels/fluid_ops.hip):
every activation with its explicit ``<name>_grad`` op and the ops whose gradients
are hand-written grad kernels (no automatic VJP) -- checked on CPUPlace by
test_fluidk_cpu.py and on the HIP device by test_fluidk_gpu.py."""
import numpy as np

rng = np.random.RandomState(2024)


def U(*s, lo=-1.0, hi=1.0):
    return rng.uniform(lo, hi, s).astype("float32")


# activation -> (attrs, input low, input high); inputs avoid the kinks where the
# numeric difference is ill-defined (|x| near thresholds)
ACT_CASES = {
    "relu": ({}, 0.1, 1.0), "sigmoid": ({}, -2, 2), "logsigmoid": ({}, -2, 2), "exp": ({}, -1, 1),
    "tanh": ({}, -2, 2), "tanh_shrink": ({}, -2, 2), "softshrink": ({"lambda": 0.3}, 0.4, 1.5),
    "sqrt": ({}, 0.5, 2), "rsqrt": ({}, 0.5, 2), "abs": ({}, 0.2, 1.0), "cos": ({}, -2, 2),
    "sin": ({}, -2, 2), "reciprocal": ({}, 0.5, 2), "log": ({}, 0.5, 2), "square": ({}, -1, 1),
    "softplus": ({}, -2, 2), "softsign": ({}, 0.1, 2), "brelu": ({"t_min": -0.5, "t_max": 0.5}, -0.4, 0.4),
    "leaky_relu": ({"alpha": 0.1}, 0.1, 1.0), "soft_relu": ({"threshold": 4.0}, -2, 2),
    "elu": ({"alpha": 0.7}, 0.1, 1.5), "relu6": ({"threshold": 6.0}, 0.5, 5.5), "pow": ({"factor": 2.5}, 0.5, 2),
    "stanh": ({"scale_a": 0.67, "scale_b": 1.7159}, -2, 2), "hard_shrink": ({"threshold": 0.3}, 0.4, 1.5),
    "thresholded_relu": ({"threshold": 0.2}, 0.3, 1.5), "hard_sigmoid": ({"slope": 0.2, "offset": 0.5}, -2, 2),
    "swish": ({"beta": 1.5}, -2, 2), "gelu": ({}, -2, 2), "silu": ({}, -2, 2),
}

_lab01 = rng.randint(0, 2, (5, 3)).astype("float32")
_logits = U(6, 9, lo=-2, hi=2)
_hard = rng.randint(0, 9, (6, 1)).astype("int64")
_soft = rng.uniform(0.1, 1, (6, 9)).astype("float32")
_soft /= _soft.sum(-1, keepdims=True)

# (op, inputs, attrs, grad inputs, output slot)
GRAD_CASES = [
    ("transpose2", {"X": U(2, 3, 4)}, {"axis": [2, 0, 1]}, ["X"], "Out"),
    ("transpose", {"X": U(3, 5)}, {"axis": [1, 0]}, ["X"], "Out"),
    ("expand", {"X": U(2, 1, 3)}, {"expand_times": [2, 3, 1]}, ["X"], "Out"),
    ("slice", {"Input": U(4, 5, 3)}, {"axes": [0, 1], "starts": [1, -4], "ends": [3, 10]}, ["Input"], "Out"),
    ("reverse", {"X": U(3, 4, 2)}, {"axis": [0, 2]}, ["X"], "Out"),
    ("cast", {"X": U(3, 4)}, {"in_dtype": 5, "out_dtype": 5}, ["X"], "Out"),
    ("hinge_loss", {"Logits": U(5, 3, lo=-3, hi=3), "Labels": _lab01}, {}, ["Logits"], "Loss"),
    ("huber_loss", {"X": U(5, 1, lo=-3, hi=3), "Y": U(5, 1, lo=-3, hi=3)}, {"delta": 1.0}, ["X"], "Out"),
    ("log_loss", {"Predicted": U(5, 1, lo=0.1, hi=0.9), "Labels": _lab01[:, :1].copy()}, {"epsilon": 1e-4},
     ["Predicted"], "Loss"),
    ("modified_huber_loss", {"X": U(6, 1, lo=-3, hi=3), "Y": rng.randint(0, 2, (6, 1)).astype("float32")}, {},
     ["X"], "Out"),
    ("sigmoid_cross_entropy_with_logits", {"X": U(5, 3, lo=-3, hi=3), "Label": _lab01}, {}, ["X"], "Out"),
    ("softmax_with_cross_entropy", {"Logits": _logits, "Label": _hard}, {}, ["Logits"], "Loss"),
    ("softmax_with_cross_entropy", {"Logits": _logits, "Label": _soft}, {"soft_label": True}, ["Logits"], "Loss"),
    ("sequence_softmax", {"X": (U(7, 1, lo=-2, hi=2), [[3, 4]])}, {}, ["X"], "Out"),
    ("layer_norm", {"X": U(2, 3, 16, lo=-2, hi=2), "Scale": U(16, lo=0.5, hi=1.5), "Bias": U(16)},
     {"begin_norm_axis": 2, "epsilon": 1e-5}, ["X", "Scale", "Bias"], "Y"),
    ("layer_norm", {"X": U(4, 16, lo=-2, hi=2), "Scale": U(16, lo=0.5, hi=1.5)},
     {"begin_norm_axis": 1, "epsilon": 1e-5}, ["X", "Scale"], "Y"),
]


def seq_conv_ref(x, off, w, cl, cs, pad=None):
    """Naive context projection (math/context_project.h semantics) + GEMM."""
    T, D = x.shape
    up = max(0, -cs)
    cols = np.zeros((T, cl * D), dtype=np.float64)
    for s, e in zip(off[:-1], off[1:]):
        for r in range(s, e):
            for k in range(cl):
                src = r + cs + k
                if s <= src < e:
                    cols[r, k * D:(k + 1) * D] = x[src]
                elif pad is not None:
                    cols[r, k * D:(k + 1) * D] = pad[up + (src - s if src < s else src - e)]
    return (cols @ w).astype("float32")


_sx = U(9, 4)
_soff = [0, 2, 7, 9]
_sw = U(3 * 4, 5)
_spad = U(3, 4)  # up_pad 1 + down_pad 2 (cs=-1, cl=3 -> down_pad = cs + cl - 1 = 1; extra row unused)
SEQ_CASES = [
    # (op, inputs, attrs, grad inputs, expected Out or None)
    ("sequence_conv", {"X": (_sx, [[2, 5, 2]]), "Filter": _sw}, {"contextLength": 3, "contextStart": -1},
     ["X", "Filter"], seq_conv_ref(_sx, _soff, _sw, 3, -1)),
    ("sequence_conv", {"X": (_sx, [[2, 5, 2]]), "Filter": _sw, "PaddingData": _spad},
     {"contextLength": 3, "contextStart": -1, "paddingTrainable": True}, ["X", "Filter", "PaddingData"],
     seq_conv_ref(_sx, _soff, _sw, 3, -1, _spad)),
    ("sequence_conv", {"X": (_sx, [[2, 5, 2]]), "Filter": _sw, "PaddingData": U(2, 4)},
     {"contextLength": 3, "contextStart": 0, "paddingTrainable": True}, ["X", "PaddingData"], None),
    ("sequence_expand_as", {"X": U(3, 2), "Y": (U(6, 1), [[1, 3, 2]])}, {}, ["X"], None),
    ("sequence_expand", {"X": (U(4, 2), [[1, 3]]), "Y": (U(5, 1), [[2, 3]])}, {"ref_level": 0}, ["X"], None),
]
