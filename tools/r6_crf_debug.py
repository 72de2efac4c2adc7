"""linear_chain_crf (+grad) on a HIP place, native vs interpreter: the loss and every
@GRAD variable of one step (emission / transition / fc gradients)."""
import os
import sys

import numpy as np
import torch

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _ROOT)
import paddle_amd.fluid as fluid  # noqa: E402
from paddle_amd.framework import core  # noqa: E402

T = 5


def go(engine, init=None, use_gpu=True):
    main, startup = fluid.Program(), fluid.Program()
    main.random_seed = startup.random_seed = 7
    with fluid.unique_name.guard(), fluid.program_guard(main, startup):
        x = fluid.layers.data(name="x", shape=[4], dtype="float32", lod_level=1)
        lab = fluid.layers.data(name="lab", shape=[1], dtype="int64", lod_level=1)
        feat = fluid.layers.fc(x, T)
        cost = fluid.layers.linear_chain_crf(input=feat, label=lab, param_attr=fluid.ParamAttr(name="crfw"))
        avg = fluid.layers.mean(cost)
        fluid.optimizer.SGD(learning_rate=0.1).minimize(avg)
    grads = [v.name for v in main.list_vars() if v.name.endswith("@GRAD") and not v.name.startswith(("lab", "x@"))]
    place = fluid.CUDAPlace(0) if use_gpu else fluid.CPUPlace()
    scope = core.Scope()
    rs = np.random.RandomState(3)
    off = [0, 3, 7, 8]
    fd = {"x": core.LoDTensor(torch.from_numpy(rs.randn(8, 4).astype("float32")), [off]),
          "lab": core.LoDTensor(torch.from_numpy(rs.randint(0, T, (8, 1)).astype("int64")), [off])}
    with fluid.executor.scope_guard(scope):
        fluid.Executor(place, engine="python").run(startup)
        pers = [v.name for v in main.list_vars() if v.persistable and scope.find_var(v.name) is not None
                and scope.find_var(v.name).get() is not None]
        if init is None:
            init = {n: np.array(scope.find_var(n).get_tensor().numpy()) for n in pers}
        else:
            for n in pers:
                scope.find_var(n).get_tensor().set(init[n], place)
        exe = fluid.Executor(place, engine=engine)
        res = exe.run(main, feed=fd, fetch_list=[avg, cost] + grads)
    return [np.array(r) for r in res], ["avg", "cost"] + grads, init


for gpu in (False, True):
    ref, names, init = go("python", use_gpu=gpu)
    got, _, _ = go("native", init, use_gpu=gpu)
    print("== gpu" if gpu else "== cpu")
    for n, a, b in zip(names, ref, got):
        print(f"{n:28s} maxabs={float(np.abs(a.astype('float64') - b.astype('float64')).max()):.3e} "
              f"ref_norm={float(np.abs(a).max()):.3e}")
