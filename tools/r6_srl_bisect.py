"""SRL on a HIP place: fetch every forward intermediate at each step from the native
engine and the interpreter (same init) and print the first var (program order) whose
values diverge, per step."""
import os
import sys

import numpy as np

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _ROOT)
sys.path.insert(0, os.path.join(_ROOT, "tests"))
import paddle_amd.fluid as fluid  # noqa: E402
from paddle_amd.framework import core  # noqa: E402
from native_rnn_cases import srl, srl_feeds  # noqa: E402


def go(engine, init=None, steps=3):
    main, startup = fluid.Program(), fluid.Program()
    main.random_seed = startup.random_seed = 7
    with fluid.unique_name.guard(), fluid.program_guard(main, startup):
        srl()()
    blk = main.global_block()
    names = []
    for op in blk.ops:
        if op.type.endswith("_grad") or op.type in ("sgd",):
            break
        for n in op.output_arg_names:
            v = blk.vars.get(n)
            if v is not None and not v.persistable and n not in names:
                names.append(n)
    scope = core.Scope()
    place = fluid.CPUPlace() if os.environ.get("SRL_CPU") else fluid.CUDAPlace(0)
    out = []
    with fluid.executor.scope_guard(scope):
        fluid.Executor(place, engine="python").run(startup)
        pers = [v.name for v in main.list_vars() if v.persistable and v.name not in ("feed", "fetch")
                and scope.find_var(v.name) is not None and scope.find_var(v.name).get() is not None]
        if init is None:
            init = {n: np.array(scope.find_var(n).get_tensor().numpy()) for n in pers}
        else:
            for n in pers:
                scope.find_var(n).get_tensor().set(init[n], place)
        exe = fluid.Executor(place, engine=engine)
        for fd in srl_feeds(steps):
            res = exe.run(main, feed=fd, fetch_list=names, return_numpy=False)
            out.append({n: np.array(r) for n, r in zip(names, res)})
    ops = [(op.type, op.output_arg_names) for op in blk.ops]
    return out, init, names, ops


ref, init, names, ops = go("python")
got, _, _, _ = go("native", init)
prod = {}
for t, o in ops:
    for n in o:
        prod.setdefault(n, t)
for step, (r, g) in enumerate(zip(ref, got)):
    bad = []
    for n in names:
        a, b = r[n], g[n]
        if a.shape != b.shape:
            bad.append((n, prod.get(n), "shape", a.shape, b.shape))
        elif a.dtype.kind == "f" and a.size and np.abs(a.astype("float64") - b).max() > 1e-4 * (1 + np.abs(a).max()):
            bad.append((n, prod.get(n), float(np.abs(a.astype("float64") - b).max())))
        elif a.dtype.kind != "f" and not np.array_equal(a, b):
            bad.append((n, prod.get(n), "int-mismatch"))
    print(f"step {step}: {len(bad)} diverging of {len(names)}; first: {bad[:6]}", flush=True)
