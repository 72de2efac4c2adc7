"""High-level Inferencer (python/paddle/fluid/inferencer.py)."""
from __future__ import annotations

from ..framework import core
from . import io, unique_name
from .executor import Executor, scope_guard
from .framework import Program, program_guard


class Inferencer:
    def __init__(self, infer_func, param_path, place=None, parallel=False):
        self.param_path = param_path
        self.scope = core.Scope()
        self.parallel = parallel
        self.place = place or core.CPUPlace()
        self.inference_program = Program()
        with program_guard(self.inference_program):
            with unique_name.guard():
                self.predict_var = infer_func()
        with self._prog_and_scope_guard():
            io.load_params(Executor(self.place), param_path)
        self.inference_program = self.inference_program.clone(for_test=True)
        self.exe = Executor(self.place)

    def _prog_and_scope_guard(self):
        return scope_guard(self.scope)

    def infer(self, inputs, return_numpy=True):
        if not isinstance(inputs, dict):
            raise ValueError("inputs should be a map of {'input_name': input_var}")
        with scope_guard(self.scope):
            return self.exe.run(self.inference_program, feed=inputs, fetch_list=[self.predict_var],
                                return_numpy=return_numpy)
