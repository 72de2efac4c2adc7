"""Loader of the ``paddle_amd_core`` CPython extension (csrc/pybind/core_module.cc):
pybind11 bindings of the native C++ framework -- ProgramDesc, Scope, LoDTensor,
Executor, registered_ops, load_persistables -- the counterpart of the reference's
``paddle.fluid.core`` built from paddle/fluid/pybind/pybind.cc.  ``module()``
returns it (None when it is not built)."""
from __future__ import annotations

import importlib.util
import os

_MOD = None


def module():
    global _MOD
    if _MOD is None:
        from . import _build

        path = _build.core_ext_path()
        if not os.path.exists(path):
            return None
        spec = importlib.util.spec_from_file_location("paddle_amd_core", path)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        _MOD = mod
    return _MOD
