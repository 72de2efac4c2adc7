"""SRL on a HIP place, native vs interpreter, 3 steps: per step the loss, the decayed
learning rate and the max abs diff of every parameter after the step."""
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
        fetch = srl()()
    sgd = [op for op in main.global_block().ops if op.type == "sgd"]
    lrn = sgd[0].input("LearningRate")[0]
    lr = [main.global_block().var(lrn)]
    print("lr op chain:", [(op.type, op.input_arg_names, op.output_arg_names) for op in main.global_block().ops
                           if op.type in ("increment", "cast", "elementwise_div", "floor", "elementwise_pow",
                                          "scale", "fill_constant", "elementwise_mul")][:12])
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
            res = exe.run(main, feed=fd, fetch_list=[fetch[0]] + lr[:3])
            params = {n: np.array(scope.find_var(n).get_tensor().numpy()) for n in pers
                      if scope.find_var(n).get() is not None}
            out.append(([np.array(r) for r in res], params))
    return out, init, [v.name for v in lr[:3]]


ref, init, lrn = go("python")
got, _, _ = go("native", init)
print("lr vars", lrn)
for t, ((ra, rp), (ga, gp)) in enumerate(zip(ref, got)):
    print(f"step {t}: loss py={ra[0]} native={ga[0]} lr py={[x.tolist() for x in ra[1:]]} native={[x.tolist() for x in ga[1:]]}")
    worst = sorted(((float(np.abs(rp[n].astype('float64') - gp[n].astype('float64')).max()), n) for n in rp
                    if n in gp and rp[n].shape == gp[n].shape), reverse=True)[:5]
    print("   worst params:", worst)
