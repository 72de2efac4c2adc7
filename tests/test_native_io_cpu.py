"""save / load / save_combine / load_combine on the C++ executor (csrc/native/ops_io.cc):
fluid.io.save_persistables / load_persistables run natively (no Python fallback), the
files are byte-identical to the Python engine's, and the loaded values round-trip.
Reference: operators/save_op.cc, load_op.cc, save_combine_op.cc, load_combine_op.cc."""
import os

import numpy as np
import pytest

import paddle_amd.fluid as fluid
from paddle_amd.framework import core


def _prog():
    main, startup = fluid.Program(), fluid.Program()
    main.random_seed = startup.random_seed = 3
    with fluid.unique_name.guard(), fluid.program_guard(main, startup):
        x = fluid.layers.data("x", [5])
        y = fluid.layers.fc(fluid.layers.fc(x, 7, act="relu"), 3)
    return main, startup, y


@pytest.mark.parametrize("combined", [False, True])
def test_native_save_load_matches_python_engine(tmp_path, combined):
    main, startup, _ = _prog()
    place = fluid.CPUPlace()
    scope = core.Scope()
    fname = "params" if combined else None
    with fluid.executor.scope_guard(scope):
        fluid.Executor(place).run(startup)
        names = [v.name for v in main.list_vars() if v.persistable and v.name not in ("feed", "fetch")]
        vals = {n: np.array(scope.find_var(n).get_tensor().numpy()) for n in names}
        fluid.io.save_persistables(fluid.Executor(place), str(tmp_path / "py"), main, filename=fname)
        nexe = fluid.Executor(place, engine="native")
        fluid.io.save_persistables(nexe, str(tmp_path / "nat"), main, filename=fname)
        assert not nexe._native.py_fallbacks, nexe._native.py_fallbacks
    py_files = sorted(os.listdir(tmp_path / "py"))
    assert py_files == sorted(os.listdir(tmp_path / "nat")) and py_files
    for f in py_files:
        assert (tmp_path / "py" / f).read_bytes() == (tmp_path / "nat" / f).read_bytes(), f
    scope2 = core.Scope()
    with fluid.executor.scope_guard(scope2):
        fluid.Executor(place).run(startup)
        for n in names:  # clobber, then load natively
            scope2.find_var(n).get_tensor().set(np.zeros_like(vals[n]), place)
        nexe = fluid.Executor(place, engine="native")
        fluid.io.load_persistables(nexe, str(tmp_path / "nat"), main, filename=fname)
        assert not nexe._native.py_fallbacks, nexe._native.py_fallbacks
        for n in names:
            np.testing.assert_array_equal(np.array(scope2.find_var(n).get_tensor().numpy()), vals[n])
