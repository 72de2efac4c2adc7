"""Graph-side evaluators (python/paddle/fluid/evaluator.py): state kept in persistable vars."""
from __future__ import annotations

import numpy as np

from . import layers
from .framework import Program, program_guard
from .initializer import ConstantInitializer
from .layer_helper import LayerHelper

__all__ = ["Evaluator", "ChunkEvaluator", "EditDistance", "DetectionMAP"]


class Evaluator:
    def __init__(self, name, **kwargs):
        self.states = []
        self.metrics = []
        self.helper = LayerHelper(name, **kwargs)

    def reset(self, executor, reset_program=None):
        from ..framework import core

        for var in self.states:
            v = core.global_scope().find_var(var.name)
            if v is not None and v.get() is not None:
                t = v.get_tensor()
                t.set_tensor(t.tensor.zero_())

    def eval(self, executor, eval_program=None):
        raise NotImplementedError()

    def _create_state(self, suffix, dtype, shape):
        state = self.helper.create_variable(name="_".join([self.helper.name, suffix]), persistable=True,
                                            dtype=dtype, shape=shape)
        self.helper.set_variable_initializer(state, ConstantInitializer(0.0))
        self.states.append(state)
        return state


class ChunkEvaluator(Evaluator):
    def __init__(self, input, label, chunk_scheme, num_chunk_types, excluded_chunk_types=None):
        super().__init__("chunk_eval")
        self.num_infer_chunks = self._create_state("num_infer_chunks", "int64", [1])
        self.num_label_chunks = self._create_state("num_label_chunks", "int64", [1])
        self.num_correct_chunks = self._create_state("num_correct_chunks", "int64", [1])

    def eval(self, executor, eval_program=None):
        from ..framework import core

        vals = [int(core.global_scope().find_var(s.name).get_tensor().numpy().reshape(-1)[0]) for s in self.states]
        ni, nl, nc = vals
        p = nc / ni if ni else 0.0
        r = nc / nl if nl else 0.0
        f1 = 2 * p * r / (p + r) if nc else 0.0
        return np.array([p]), np.array([r]), np.array([f1])


class EditDistance(Evaluator):
    def __init__(self, input, label, ignored_tokens=None, **kwargs):
        super().__init__("edit_distance", **kwargs)
        self.total_distance = self._create_state("total_distance", "float32", [1])
        self.seq_num = self._create_state("seq_num", "int64", [1])
        self.instance_error = self._create_state("instance_error", "int64", [1])

    def eval(self, executor, eval_program=None):
        from ..framework import core

        td, sn, ie = [core.global_scope().find_var(s.name).get_tensor().numpy().reshape(-1)[0] for s in self.states]
        return np.array([td / max(sn, 1)]), np.array([ie / max(sn, 1)])


class DetectionMAP(Evaluator):
    def __init__(self, *args, **kwargs):
        super().__init__("map_eval")
