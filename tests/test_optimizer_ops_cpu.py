"""Fluid optimizer update operators vs NumPy transcriptions of the reference update
rules (operators/{sgd,momentum,lars_momentum,adam,adamax,adagrad,decayed_adagrad,
adadelta,rmsprop,ftrl,proximal_gd,proximal_adagrad}_op.h; reference tests
test_*_op.py).  ``OPT_CASES`` also runs on CUDAPlace (tests/test_optimizer_ops_gpu.py),
where every dense fp32 update is a single fused kernel (optimizer.hip, optim_ext.hip)."""
import numpy as np
import pytest

import paddle_amd.fluid as fluid
from op_test import OpTest

rng = np.random.RandomState(11)
S = (13, 7)


def _r(lo=-1.0, hi=1.0, shape=S):
    return rng.uniform(lo, hi, shape).astype("float32")


def _cases():
    c = []
    p, g, lr = _r(), _r(), np.array([0.05], "float32")
    c.append(("sgd", {"Param": p, "Grad": g, "LearningRate": lr}, {"ParamOut": p - lr * g}, {}))

    v = _r()
    for nest in (False, True):
        v2 = 0.9 * v + g
        po = p - (g + 0.9 * v2) * lr if nest else p - lr * v2
        c.append(("momentum", {"Param": p, "Grad": g, "Velocity": v, "LearningRate": lr},
                  {"ParamOut": po, "VelocityOut": v2}, {"mu": 0.9, "use_nesterov": nest}))

    pn, gn = np.linalg.norm(p), np.linalg.norm(g)
    local = lr * 0.001 * pn / (gn + 0.0005 * pn)
    v2 = 0.9 * v + local * (g + 0.0005 * p)
    c.append(("lars_momentum", {"Param": p, "Grad": g, "Velocity": v, "LearningRate": lr},
              {"ParamOut": p - v2, "VelocityOut": v2}, {"mu": 0.9, "lars_coeff": 0.001, "lars_weight_decay": 0.0005}))

    m1, m2 = _r(), _r(0, 1)
    bp1, bp2 = np.array([0.9 ** 3], "float32"), np.array([0.999 ** 3], "float32")
    m1o = 0.9 * m1 + 0.1 * g
    m2o = 0.999 * m2 + 0.001 * g * g
    lr_t = lr * np.sqrt(1 - bp2) / (1 - bp1)
    c.append(("adam", {"Param": p, "Grad": g, "LearningRate": lr, "Moment1": m1, "Moment2": m2, "Beta1Pow": bp1,
                       "Beta2Pow": bp2},
              {"ParamOut": p - lr_t * m1o / (np.sqrt(m2o) + 1e-8), "Moment1Out": m1o, "Moment2Out": m2o}, {}))

    m, u = _r(), _r(0.1, 1)
    mo = 0.9 * m + 0.1 * g
    uo = np.maximum(0.999 * u + 1e-8, np.abs(g))
    c.append(("adamax", {"Param": p, "Grad": g, "LearningRate": lr, "Moment": m, "InfNorm": u, "Beta1Pow": bp1},
              {"ParamOut": p - lr / (1 - bp1) * mo / uo, "MomentOut": mo, "InfNormOut": uo}, {}))

    ma = _r(0, 1)
    mao = ma + g * g
    c.append(("adagrad", {"Param": p, "Grad": g, "Moment": ma, "LearningRate": lr},
              {"ParamOut": p - lr * g / (np.sqrt(mao) + 1e-6), "MomentOut": mao}, {}))
    mdo = 0.95 * ma + 0.05 * g * g
    c.append(("decayed_adagrad", {"Param": p, "Grad": g, "Moment": ma, "LearningRate": lr},
              {"ParamOut": p - lr * g / (np.sqrt(mdo) + 1e-6), "MomentOut": mdo}, {}))

    ag, au = _r(0, 1), _r(0, 1)
    ago = 0.95 * ag + 0.05 * g * g
    upd = -np.sqrt((au + 1e-6) / (ago + 1e-6)) * g
    auo = 0.95 * au + 0.05 * upd * upd
    c.append(("adadelta", {"Param": p, "Grad": g, "AvgSquaredGrad": ag, "AvgSquaredUpdate": au},
              {"ParamOut": p + upd, "AvgSquaredGradOut": ago, "AvgSquaredUpdateOut": auo}, {}))

    ms, mom, mg = _r(0.5, 1), _r(), _r(-0.1, 0.1)
    mso = 0.9 * ms + 0.1 * g * g
    momo = 0.5 * mom + lr * g / np.sqrt(mso + 1e-10)
    c.append(("rmsprop", {"Param": p, "MeanSquare": ms, "Grad": g, "Moment": mom, "LearningRate": lr},
              {"ParamOut": p - momo, "MomentOut": momo, "MeanSquareOut": mso}, {"momentum": 0.5}))
    mgo = 0.9 * mg + 0.1 * g
    momc = 0.5 * mom + lr * g / np.sqrt(mso - mgo * mgo + 1e-10)
    c.append(("rmsprop", {"Param": p, "MeanSquare": ms, "Grad": g, "Moment": mom, "LearningRate": lr,
                          "MeanGrad": mg},
              {"ParamOut": p - momc, "MomentOut": momc, "MeanSquareOut": mso, "MeanGradOut": mgo},
              {"momentum": 0.5, "centered": True}))

    sq, lin = _r(0.1, 1), _r()
    for lp in (-0.5, -0.3):
        nsq = sq + g * g
        if lp == -0.5:
            sigma = (np.sqrt(nsq) - np.sqrt(sq)) / lr
            y = np.sqrt(nsq) / lr + 2 * 0.1
        else:
            sigma = (nsq ** -lp - sq ** -lp) / lr
            y = nsq ** -lp / lr + 2 * 0.1
        nlin = lin + g - sigma * p
        po = np.where(np.abs(nlin) > 0.2, (0.2 * np.sign(nlin) - nlin) / y, 0.0)
        c.append(("ftrl", {"Param": p, "SquaredAccumulator": sq, "LinearAccumulator": lin, "Grad": g,
                           "LearningRate": lr},
                  {"ParamOut": po, "SquaredAccumOut": nsq, "LinearAccumOut": nlin},
                  {"l1": 0.2, "l2": 0.1, "lr_power": lp}))

    prox = p - lr * g
    c.append(("proximal_gd", {"Param": p, "Grad": g, "LearningRate": lr},
              {"ParamOut": np.sign(prox) * np.maximum(np.abs(prox) - lr * 0.3, 0) / (1 + lr * 0.2)},
              {"l1": 0.3, "l2": 0.2}))
    mpo = ma + g * g
    lt = lr / np.sqrt(mpo)
    prox = p - lt * g
    c.append(("proximal_adagrad", {"Param": p, "Moment": ma, "Grad": g, "LearningRate": lr},
              {"ParamOut": np.sign(prox) * np.maximum(np.abs(prox) - lt * 0.3, 0) / (1 + lt * 0.2),
               "MomentOut": mpo}, {"l1": 0.3, "l2": 0.2}))
    return [(op, ins, {k: v.astype("float32") for k, v in outs.items()}, attrs) for op, ins, outs, attrs in c]


OPT_CASES = _cases()


def run_case(op, inputs, outputs, attrs, place):
    t = OpTest()
    t.op_type, t.inputs, t.outputs, t.attrs = op, inputs, outputs, attrs
    t.check_output(atol=2e-5, rtol=2e-4, places=[place])


@pytest.mark.parametrize("op,inputs,outputs,attrs", OPT_CASES, ids=[f"{c[0]}_{i}" for i, c in enumerate(OPT_CASES)])
def test_optimizer_op(op, inputs, outputs, attrs):
    run_case(op, inputs, outputs, attrs, fluid.CPUPlace())
