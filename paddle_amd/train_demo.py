"""Host side of the C++ training demo (csrc/train_demo/demo_trainer.cc; reference
paddle/fluid/train/demo/{demo_network.py, demo_trainer.cc}).

``save_demo_programs(dir)`` writes the demo network's startup / main ProgramDescs
(fc regression on 13 features, square error, SGD -- as the reference's
demo_network.py).  ``DemoTrainer`` is what the C++ program drives through the
embedded interpreter: load the two serialized programs, run startup, bind input
buffers the C++ side owns, run training steps, read the loss.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import fluid
from .framework import core


def save_demo_programs(d, with_optimize=True):
    os.makedirs(d, exist_ok=True)
    main, startup = fluid.Program(), fluid.Program()
    with fluid.program_guard(main, startup):
        x = fluid.layers.data(name="x", shape=[13], dtype="float32")
        y_predict = fluid.layers.fc(input=x, size=1, act=None)
        y = fluid.layers.data(name="y", shape=[1], dtype="float32")
        avg_cost = fluid.layers.mean(fluid.layers.square_error_cost(input=y_predict, label=y))
        if with_optimize:
            fluid.optimizer.SGD(learning_rate=1e-5).minimize(avg_cost)
        else:
            fluid.backward.append_backward(avg_cost)
    with open(os.path.join(d, "startup_program"), "wb") as f:
        f.write(startup.desc.serialize_to_string())
    with open(os.path.join(d, "main_program"), "wb") as f:
        f.write(main.desc.serialize_to_string())


class DemoTrainer:
    def __init__(self, model_dir, use_gpu=False):
        from .fluid.framework import Program

        def load(name):
            with open(os.path.join(model_dir, name), "rb") as f:
                return Program.parse_from_string(f.read())

        self.startup, self.main = load("startup_program"), load("main_program")
        self.loss_name = next(op.output("Out")[0] for op in self.main.global_block().ops if op.type == "mean")
        self.place = fluid.CUDAPlace(0) if use_gpu and torch.cuda.is_available() else fluid.CPUPlace()
        self.exe = fluid.Executor(self.place)
        self.scope = core.Scope()
        self.feed = {}

    def run_startup(self):
        with fluid.executor.scope_guard(self.scope):
            self.exe.run(self.startup)

    def set_input(self, name, buf, shape):
        """``buf``: a buffer owned by the caller (float32, C order)."""
        self.feed[name] = np.frombuffer(buf, dtype=np.float32).reshape(shape).copy()

    def step(self):
        with fluid.executor.scope_guard(self.scope):
            (loss,) = self.exe.run(self.main, feed=self.feed, fetch_list=[self.loss_name])
        return float(np.asarray(loss).reshape(-1)[0])
