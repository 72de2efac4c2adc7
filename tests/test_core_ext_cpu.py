"""paddle_amd_core, the CPython extension over the native C++ framework
(csrc/pybind/core_module.cc; reference pybind/pybind.cc:89-708): ProgramDesc from a
Fluid program's bytes, Scope / LoDTensor numpy round trips and zero-copy lending
of torch storage, Executor.run of a startup + training program, and the native
engine of fluid.Executor driving the C++ objects through it."""
import numpy as np
import pytest
import torch

import paddle_amd.fluid as fluid
from paddle_amd import core_ext

C = core_ext.module()
pytestmark = pytest.mark.skipif(C is None, reason="paddle_amd_core not built")


def test_scope_tensor_roundtrip_and_lending():
    s = C.Scope()
    t = s.var("a").get_tensor()
    a = np.arange(12, dtype="float32").reshape(3, 4)
    t.set(a)
    assert s.find_var("a").get_tensor().shape() == [3, 4]
    np.testing.assert_array_equal(s.find_var("a").get_tensor().numpy(), a)
    np.testing.assert_array_equal(np.array(t), a)
    t.set_lod([[0, 1, 3]])
    assert t.lod() == [[0, 1, 3]]
    kid = s.new_scope()
    assert kid.find_var("a") is not None and kid.find_local_var("a") is None
    # zero-copy: the native tensor views the torch storage
    x = torch.arange(6, dtype=torch.int64)
    s.var("x").get_tensor().share_external(x.data_ptr(), C.VarType.INT64, [2, 3], -1)
    x.add_(10)
    np.testing.assert_array_equal(s.find_var("x").get_tensor().numpy(), x.view(2, 3).numpy())
    assert "a" in s.local_var_names()
    with pytest.raises(TypeError):
        s.var("c").get_tensor().set(np.zeros(2, dtype=np.complex64))


def test_executor_runs_fluid_programs():
    main, startup = fluid.Program(), fluid.Program()
    main.random_seed = startup.random_seed = 3
    with fluid.program_guard(main, startup):
        x = fluid.layers.data("x", [8])
        y = fluid.layers.data("y", [1], dtype="int64")
        pred = fluid.layers.fc(x, 4, act="softmax")
        loss = fluid.layers.mean(fluid.layers.cross_entropy(pred, y))
        fluid.optimizer.SGD(0.5).minimize(loss)
    sp = C.ProgramDesc(startup.desc.serialize_to_string())
    mp = C.ProgramDesc(main.desc.serialize_to_string())
    assert "mul" in mp.op_types() and "sgd" in mp.op_types()
    scope = C.Scope()
    exe = C.Executor(-1)
    exe.run(sp, scope)
    rs = np.random.RandomState(0)
    xs = rs.randn(16, 8).astype("float32")
    ys = rs.randint(0, 4, (16, 1)).astype("int64")
    losses = []
    for _ in range(8):
        scope.var("x").get_tensor().set(xs)
        scope.var("y").get_tensor().set(ys)
        exe.run(mp, scope)
        losses.append(float(scope.find_var(loss.name).get_tensor().numpy().ravel()[0]))
    assert losses[-1] < losses[0]


def test_fluid_native_engine_uses_the_extension():
    place = fluid.CPUPlace()
    exe = fluid.Executor(place, engine="native")
    main, startup = fluid.Program(), fluid.Program()
    with fluid.program_guard(main, startup):
        x = fluid.layers.data("x", [4])
        out = fluid.layers.relu(fluid.layers.scale(x, scale=2.0))
    fluid.Executor(place).run(startup)
    (o,) = exe.run(main, feed={"x": np.array([[-1, 2, -3, 4]], "float32")}, fetch_list=[out])
    np.testing.assert_array_equal(o, [[0, 4, 0, 8]])
    assert exe._native.binding == "pybind"
