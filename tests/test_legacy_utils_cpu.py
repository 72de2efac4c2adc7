"""Legacy utils counterparts (reference paddle/legacy/utils): Stat timers
(Stat.h StatSet / REGISTER_TIMER, printed by the v1 trainer with --log_stat) and the
operator stack of CustomStackTrace (utils/stack_trace.py)."""
import threading
import time

import numpy as np
import pytest

import paddle_amd.fluid as fluid
from paddle_amd.utils import stack_trace
from paddle_amd.utils.stat import StatSet


def test_stat_set_aggregates_across_threads():
    st = StatSet("t")

    def work():
        for _ in range(5):
            with st.timer("a"):
                time.sleep(0.001)

    ts = [threading.Thread(target=work) for _ in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    with st.timer("b"):
        pass
    d = st.as_dict()
    assert d["a"]["count"] == 20 and d["b"]["count"] == 1
    assert d["a"]["min"] >= 0.001 - 1e-4 and d["a"]["max"] >= d["a"]["min"]
    assert abs(d["a"]["total"] - sum([d["a"]["total"]])) < 1e-12
    text = st.status()
    assert "Stat=a" in text and "count=20" in text
    st.reset()
    assert st.as_dict() == {}


def test_failing_op_carries_the_operator_stack():
    main, startup = fluid.Program(), fluid.Program()
    with fluid.program_guard(main, startup):
        x = fluid.layers.data(name="x", shape=[4], dtype="float32")
        h = fluid.layers.fc(x, size=3)
        out = fluid.layers.mean(h)
    exe = fluid.Executor(fluid.CPUPlace(), engine="python")
    stack_trace.install()
    try:
        with fluid.scope_guard(fluid.core.Scope()):
            exe.run(startup)
            with pytest.raises(Exception) as ei:
                exe.run(main, feed={"x": np.ones((2, 5), "float32")}, fetch_list=[out])  # wrong width
        st = getattr(ei.value, "_pa_op_stack", None)
        assert st and st[-1] == "mul", st
        assert stack_trace.current() == []
    finally:
        stack_trace.uninstall()
