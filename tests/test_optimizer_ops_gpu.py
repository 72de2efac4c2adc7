"""The optimizer OpTest table (test_optimizer_ops_cpu.py) on CUDAPlace: dense fp32
updates run the fused kernels of optimizer.hip / optim_ext.hip."""
import pytest
import torch

import paddle_amd.fluid as fluid
from test_optimizer_ops_cpu import OPT_CASES, run_case

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("op,inputs,outputs,attrs", OPT_CASES, ids=[f"{c[0]}_{i}" for i, c in enumerate(OPT_CASES)])
def test_optimizer_op_on_device(op, inputs, outputs, attrs):
    run_case(op, inputs, outputs, attrs, fluid.CUDAPlace(0))


def test_native_kernels_are_used(monkeypatch):
    from paddle_amd.ops import oplib

    calls = []
    orig = oplib.opt_update_

    def spy(kind, *a, **k):
        r = orig(kind, *a, **k)
        calls.append((kind, r is not None))
        return r

    monkeypatch.setattr(oplib, "opt_update_", spy)
    ops = ("adamax", "ftrl", "rmsprop", "lars_momentum", "adadelta", "decayed_adagrad", "proximal_gd")
    for op, inputs, outputs, attrs in OPT_CASES:
        if op in ops:
            run_case(op, inputs, outputs, attrs, fluid.CUDAPlace(0))
    # the Python kernels that ran took the fused HIP update; the rest ran as device
    # kernels of the C++ executor (every one of these has one now)
    assert all(ok for _, ok in calls), calls
    from paddle_amd import native
    dev_ops = set(native.registered_ops(device=True))
    assert all(op in dev_ops for op in ops if op not in {k for k, _ in calls}), sorted(dev_ops & set(ops))


@pytest.mark.parametrize("opt", ["sgd", "momentum", "adam", "adagrad", "rmsprop", "adamax"])
def test_optimizer_updates_in_place_on_device(opt):
    """Fluid program whose optimizer ops write ParamOut == Param: the device update
    keeps the parameter's storage (no per-step clones) and matches the CPU run."""
    import numpy as np

    from paddle_amd.framework import core

    def run(place):
        prog, start = fluid.Program(), fluid.Program()
        with fluid.program_guard(prog, start):
            x = fluid.layers.data("x", [8], dtype="float32")
            y = fluid.layers.fc(x, 4, param_attr=fluid.ParamAttr(name="w",
                                initializer=fluid.initializer.Constant(0.1)), bias_attr=False)
            loss = fluid.layers.mean(fluid.layers.square(y))
            o = {"sgd": fluid.optimizer.SGD(0.1), "momentum": fluid.optimizer.Momentum(0.1, 0.9),
                 "adam": fluid.optimizer.Adam(0.01), "adagrad": fluid.optimizer.Adagrad(0.1),
                 "rmsprop": fluid.optimizer.RMSProp(0.01), "adamax": fluid.optimizer.Adamax(0.01)}[opt]
            o.minimize(loss)
        scope = core.Scope()
        exe = fluid.Executor(place)
        exe.run(start, scope=scope)
        ptrs = []
        xs = np.linspace(-1, 1, 3 * 8, dtype="float32").reshape(3, 8)
        for _ in range(3):
            exe.run(prog, feed={"x": xs}, fetch_list=[loss], scope=scope)
            ptrs.append(scope.find_var("w").get().tensor.data_ptr())
        return np.array(scope.find_var("w").get().tensor.cpu()), ptrs

    wg, ptrs = run(fluid.CUDAPlace(0))
    wc, _ = run(fluid.CPUPlace())
    np.testing.assert_allclose(wg, wc, rtol=1e-4, atol=1e-6)
    assert len(set(ptrs)) == 1, "device optimizer update reallocated the parameter"


@pytest.mark.parametrize("nesterov", [False, True])
def test_momentum_multi_tensor_matches_per_parameter(monkeypatch, nesterov):
    """One pa_momentum_multi launch over every parameter == the per-parameter path
    (bf16 params with fp32 masters, fp32 params, L2 decay, a no-decay parameter, a
    param group with an lr multiplier); the device table is re-used across steps."""
    import paddle_amd as paddle

    def run(multi):
        monkeypatch.setenv("FLAGS_multi_tensor_momentum", "1" if multi else "0")
        g = torch.Generator(device="cuda").manual_seed(0)
        ps = [torch.nn.Parameter(torch.randn(*s, generator=g, device="cuda").to(dt))
              for s, dt in [((300, 7), torch.bfloat16), ((5000,), torch.bfloat16), ((64, 3, 3, 3), torch.float32),
                            ((13,), torch.float32), ((4097,), torch.bfloat16)]]
        ps[3].no_weight_decay = True
        opt = paddle.optimizer.Momentum(learning_rate=0.05, momentum=0.9, use_nesterov=nesterov,
                                        parameters=[{"params": ps[:4]}, {"params": ps[4:], "learning_rate": 0.5}],
                                        weight_decay=paddle.optimizer.L2Decay(1e-2), multi_precision=True)
        for it in range(3):
            for i, p in enumerate(ps):
                p.grad = (torch.randn(p.shape, generator=g, device="cuda") * (i + 1)).to(p.dtype)
            opt.step()
        return [p.detach().float().clone() for p in ps], opt

    ref, _ = run(False)
    got, opt = run(True)
    assert opt._multi is not None and opt._multi._nt == 5
    for a, b in zip(got, ref):
        torch.testing.assert_close(a, b, rtol=2e-2, atol=1.6e-2)  # 1 bf16 ulp at |p| ~ 2-4
