"""Inference library (reference: paddle/fluid/inference/api/paddle_inference_api.h:36-162,
api_impl.cc:61-129 ``NativePaddlePredictor``, analysis/analyzer.h:53 ``Analyzer``).

* :class:`NativeConfig` / :class:`AnalysisConfig` -- model location, device, IR
  optimisation switches.
* :class:`PaddleTensor` / :class:`PaddleBuf` / :class:`PaddleDType` -- the I/O
  record of ``PaddlePredictor::Run``.
* :func:`create_paddle_predictor` -- ``CreatePaddlePredictor<ConfigT>``.
* ``NativePaddlePredictor``: load ``__model__`` + params once, prepare the block
  once, then ``run`` = feed -> prepared block -> fetch.  ``clone`` shares the
  parameter scope (api_impl.cc Clone) so several threads can serve one model.
* ``AnalysisPredictor``: additionally runs the IR pass pipeline
  (``framework.ir``: is_test, identity-op cleanup, conv+BN fold, fc fuse,
  fc+activation fuse, fc+lstm fuse) before preparing.

MI355X-specific (instead of TensorRT / Anakin subgraph engines, which have no
gfx950 backend):
  * ``AnalysisConfig.enable_bf16()`` converts float weights to bfloat16 once at
    load time so every GEMM/conv runs on the bf16 MFMA path (the reference's
    float16 transpiler, paddle/contrib/float16/float16_transpiler.py, did the same
    for V100 tensor cores);
  * ``AnalysisConfig.enable_hip_graph()`` captures the whole prepared block into a
    HIP graph after the first run for a given input signature and replays it --
    one launch per request instead of one per op, which is what small-batch
    serving is bound by.
"""
from __future__ import annotations

import copy
import enum
import os
import threading

import numpy as np
import torch

from ..framework import core
from ..framework.executor import BlockExecutor


class PaddleDType(enum.IntEnum):
    FLOAT32 = 0
    INT64 = 1
    INT32 = 2
    BFLOAT16 = 3
    FLOAT16 = 4


_NP = {PaddleDType.FLOAT32: np.float32, PaddleDType.INT64: np.int64, PaddleDType.INT32: np.int32,
       PaddleDType.FLOAT16: np.float16}


class PaddleBuf:
    """Owned or borrowed byte buffer (paddle_inference_api.h:36)."""

    def __init__(self, data=None):
        self._arr = None if data is None else np.ascontiguousarray(data)

    def resize(self, nbytes):
        self._arr = np.zeros(nbytes, dtype=np.uint8)

    def reset(self, data):
        self._arr = np.ascontiguousarray(data)

    def length(self):
        return 0 if self._arr is None else self._arr.nbytes

    def empty(self):
        return self._arr is None

    def data(self):
        return self._arr

    def float_data(self):
        return self._arr.view(np.float32).ravel().tolist()

    def int64_data(self):
        return self._arr.view(np.int64).ravel().tolist()


class PaddleTensor:
    """Named tensor with LoD (paddle_inference_api.h:62)."""

    def __init__(self, data=None, name="", lod=None, dtype=None):
        self.name = name
        self.lod = lod or []
        arr = None if data is None else np.asarray(data)
        if arr is not None and dtype is None:
            dtype = PaddleDType.INT64 if arr.dtype.kind in "iu" and arr.dtype.itemsize == 8 else \
                PaddleDType.INT32 if arr.dtype.kind in "iu" else PaddleDType.FLOAT32
            if arr.dtype.kind == "f":
                arr = arr.astype(np.float32, copy=False)
        self.dtype = dtype if dtype is not None else PaddleDType.FLOAT32
        self.shape = list(arr.shape) if arr is not None else []
        self.data = PaddleBuf(arr)

    def as_ndarray(self):
        a = self.data.data()
        return a.reshape(self.shape) if a is not None else None

    def __repr__(self):
        return f"PaddleTensor(name={self.name!r}, shape={self.shape}, dtype={self.dtype.name}, lod={self.lod})"


class NativeConfig:
    """api NativeConfig: model_dir | (prog_file, param_file), device selection."""

    def __init__(self, model_dir="", prog_file="", param_file="", use_gpu=None, device=0,
                 fraction_of_gpu_memory=-1.0, specify_input_name=False):
        self.model_dir = model_dir
        self.prog_file = prog_file
        self.param_file = param_file
        self.use_gpu = torch.cuda.is_available() if use_gpu is None else use_gpu
        self.device = device
        self.fraction_of_gpu_memory = fraction_of_gpu_memory
        self.specify_input_name = specify_input_name


class AnalysisConfig(NativeConfig):
    """NativeConfig + IR optimisation (analysis/analyzer.h, contrib AnalysisConfig)."""

    DEFAULT_PASSES = ["is_test_pass", "identity_op_clean_pass", "conv_bn_fuse_pass", "fc_fuse_pass",
                      "fc_act_fuse_pass", "fc_lstm_fuse_pass"]

    def __init__(self, model_dir="", prog_file="", param_file="", **kw):
        super().__init__(model_dir, prog_file, param_file, **kw)
        self.enable_ir_optim = True
        self.ir_passes = list(self.DEFAULT_PASSES)
        self.ir_passes_disabled: set = set()
        self.precision = "fp32"
        self.use_hip_graph = False

    def switch_ir_optim(self, x=True):
        self.enable_ir_optim = bool(x)

    def delete_pass(self, name):
        self.ir_passes_disabled.add(name)

    def pass_builder(self):
        return [p for p in self.ir_passes if p not in self.ir_passes_disabled]

    def enable_bf16(self):
        self.precision = "bf16"

    def enable_hip_graph(self, x=True):
        self.use_hip_graph = bool(x)


class PaddlePredictor:
    def run(self, inputs, batch_size=-1):
        raise NotImplementedError

    def clone(self):
        raise NotImplementedError

    # reference spellings
    def Run(self, inputs, output_data=None, batch_size=-1):
        outs = self.run(inputs, batch_size)
        if output_data is not None:
            output_data[:] = outs
        return True

    def Clone(self):
        return self.clone()


def _load_program(config):
    from ..fluid.framework import Program

    if config.prog_file:
        prog_path, params_dir = config.prog_file, os.path.dirname(config.prog_file)
    else:
        prog_path, params_dir = os.path.join(config.model_dir, "__model__"), config.model_dir
    with open(prog_path, "rb") as f:
        program = Program.parse_from_string(f.read())
    return program, params_dir


class NativePaddlePredictor(PaddlePredictor):
    def __init__(self, config, _shared=None):
        self.config = config
        self.place = core.CUDAPlace(config.device) if config.use_gpu and torch.cuda.is_available() \
            else core.CPUPlace()
        if _shared is not None:
            self.program, self.root_scope, self.feed_names, self.fetch_names = _shared
        else:
            self._load()
        self.scope = self.root_scope.new_scope()
        self.exe = BlockExecutor(self.place)
        self._prepared = self.exe.prepare(self.program, 0)
        BlockExecutor.create_variables(self.program, self.scope, 0)
        self._graphs = {}
        self._lock = threading.Lock()

    # -------------------------------------------------------------- loading
    def _load(self):
        from ..fluid import io as fio
        from ..fluid.executor import Executor, scope_guard

        program, params_dir = _load_program(self.config)
        self.root_scope = core.Scope()
        exe = Executor(self.place)
        with scope_guard(self.root_scope):
            fio.load_persistables(exe, params_dir, program,
                                  os.path.basename(self.config.param_file) if self.config.param_file else None)
        gb = program.global_block()
        feeds = sorted((op.attrs["col"], op.output("Out")[0]) for op in gb.ops if op.type == "feed")
        fetches = sorted((op.attrs["col"], op.input("X")[0]) for op in gb.ops if op.type == "fetch")
        self.feed_names = [n for _, n in feeds]
        self.fetch_names = [n for _, n in fetches]
        gb.ops = [op for op in gb.ops if op.type not in ("feed", "fetch")]
        program._version += 1
        self.program = program
        self._optimize()

    def _optimize(self):
        pass

    # -------------------------------------------------------------- running
    def _to_lod_tensor(self, t: PaddleTensor):
        arr = t.as_ndarray()
        ten = torch.from_numpy(np.ascontiguousarray(arr))
        if getattr(self.config, "precision", "fp32") == "bf16" and ten.is_floating_point():
            ten = ten.to(torch.bfloat16)
        dev = self.place.torch_device()
        if dev.type != "cpu":
            ten = ten.pin_memory().to(dev, non_blocking=True) if ten.numel() > 4096 else ten.to(dev)
        lt = core.LoDTensor(ten)
        if t.lod:
            lt.set_lod([list(l) for l in t.lod])
        return lt

    def _feed(self, inputs):
        if len(inputs) != len(self.feed_names):
            raise ValueError(f"expected {len(self.feed_names)} inputs ({self.feed_names}), got {len(inputs)}")
        if self.config.specify_input_name:
            by_name = {t.name: t for t in inputs}
            inputs = [by_name[n] for n in self.feed_names]
        for name, t in zip(self.feed_names, inputs):
            self.scope.var(name).set(self._to_lod_tensor(t))

    def _fetch(self):
        outs = []
        for name in self.fetch_names:
            v = self.scope.find_var(name).get()
            ten = v.tensor if isinstance(v, core.LoDTensor) else v
            arr = ten.detach().float().cpu().numpy() if ten.dtype in (torch.bfloat16, torch.float16) \
                else ten.detach().cpu().numpy()
            lod = v.lod() if isinstance(v, core.LoDTensor) else []
            outs.append(PaddleTensor(arr, name=name, lod=[list(l) for l in lod]))
        return outs

    def run(self, inputs, batch_size=-1):
        with torch.inference_mode():
            if getattr(self.config, "use_hip_graph", False) and self.place.torch_device().type == "cuda":
                return self._run_graph(inputs)
            self._feed(inputs)
            self.exe.run_prepared(self._prepared, self.scope)
            return self._fetch()

    # -------------------------------------------------------------- HIP graph replay
    def _run_graph(self, inputs):
        sig = tuple((tuple(t.shape), int(t.dtype), tuple(map(tuple, t.lod))) for t in inputs)
        g = self._graphs.get(sig)
        if g is None:
            # eager warm-up run (allocator, lazy library init), then capture
            self._feed(inputs)
            self.exe.run_prepared(self._prepared, self.scope)
            torch.cuda.synchronize()
            static_in = [self.scope.find_var(n).get().tensor for n in self.feed_names]
            graph = torch.cuda.CUDAGraph()
            try:
                with torch.cuda.graph(graph):
                    self.exe.run_prepared(self._prepared, self.scope)
            except Exception:  # an op synchronises with the host: not capturable
                self._graphs[sig] = "eager"
                self.config.use_hip_graph = False
                return self.run(inputs)
            g = self._graphs[sig] = (graph, static_in)
        if g == "eager":
            self._feed(inputs)
            self.exe.run_prepared(self._prepared, self.scope)
            return self._fetch()
        graph, static_in = g
        for dst, t in zip(static_in, inputs):
            dst.copy_(torch.from_numpy(np.ascontiguousarray(t.as_ndarray())).to(dst.dtype), non_blocking=True)
        graph.replay()
        return self._fetch()

    def clone(self):
        c = copy.copy(self.config)
        return type(self)(c, _shared=(self.program, self.root_scope, self.feed_names, self.fetch_names))

    def get_input_names(self):
        return list(self.feed_names)

    def get_output_names(self):
        return list(self.fetch_names)


class AnalysisPredictor(NativePaddlePredictor):
    def _optimize(self):
        from ..framework import ir
        from . import passes  # noqa: F401  (registers conv_bn_fuse_pass)

        cfg = self.config
        self.applied_passes = []
        if getattr(cfg, "enable_ir_optim", False):
            names = cfg.pass_builder()
            g = ir.apply_passes(self.program, names, __param_scope__=self.root_scope)
            self.applied_passes = g.get("__applied_passes__", [])
            self.pass_stats = {k: v for k, v in g._attrs.items() if k.endswith("_count") or k.endswith("_removed")}
        if getattr(cfg, "precision", "fp32") == "bf16":
            from .passes import convert_params_to_bf16

            convert_params_to_bf16(self.program, self.root_scope)


def create_paddle_predictor(config):
    """CreatePaddlePredictor<NativeConfig|AnalysisConfig>."""
    if isinstance(config, AnalysisConfig):
        return AnalysisPredictor(config)
    return NativePaddlePredictor(config)


__all__ = ["PaddleDType", "PaddleBuf", "PaddleTensor", "NativeConfig", "AnalysisConfig", "PaddlePredictor",
           "NativePaddlePredictor", "AnalysisPredictor", "create_paddle_predictor"]
