"""Platform layer (reference platform/enforce.h, init.cc, glog VLOG): HIP error
names in kernel-library errors, GLOG_v-controlled op logging in the executor."""
import numpy as np
import pytest

import paddle_amd.fluid as fluid
from paddle_amd import platform
from paddle_amd.ops import _native as N


def test_enforce_error_carries_hip_error_name():
    e = N.EnforceError("pa_fake", 1)
    assert "hipErrorInvalidValue" in str(e) and e.rc == 1
    with pytest.raises(N.EnforceError):
        N.check(1, "pa_fake")
    with pytest.raises(RuntimeError):
        platform.enforce(False, "bad %d", 3)


def test_vlog_levels_and_executor_op_log(capsys):
    old = platform.vlog_level()
    try:
        platform.set_vlog_level(3)
        main, st = fluid.Program(), fluid.Program()
        with fluid.program_guard(main, st):
            x = fluid.layers.data("x", [4])
            y = fluid.layers.fc(x, 2)
        exe = fluid.Executor(fluid.CPUPlace())
        exe.run(st, scope=fluid.core.Scope())
        scope = fluid.core.Scope()
        exe.run(st, scope=scope)
        exe.run(main, feed={"x": np.ones((1, 4), "float32")}, fetch_list=[y], scope=scope)
        err = capsys.readouterr().err
        assert "run op mul" in err and "paddle_amd]" in err
        platform.set_vlog_level(0)
        platform.vlog(1, "hidden")
        assert "hidden" not in capsys.readouterr().err
    finally:
        platform.set_vlog_level(old)
