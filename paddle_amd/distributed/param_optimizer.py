"""Native parameter optimizer (csrc/runtime/param_optimizer.cc, the reference's
paddle/legacy/optimizer C library behind the Go pserver): an OptimizerConfig message
(proto/OptimizerConfig.proto) configures SGD / Adadelta / Adagrad / Adam with a
Const or Linear learning-rate policy; ``update`` applies one gradient; ``state()``
serialises the <Kind>OptimizerState message that ``ParameterOptimizer(...,
state=...)`` resumes from."""
from __future__ import annotations

import ctypes

import numpy as np

from .. import runtime
from ..trainer_config_helpers import config_proto as cp

SGD, ADADELTA, ADAGRAD, ADAM = 1, 2, 3, 4
_KIND = {"sgd": SGD, "momentum": SGD, "adadelta": ADADELTA, "adagrad": ADAGRAD, "adam": ADAM}

_schemas = {
    "SGDConfig": [("momentum", 21, "double", 0), ("decay", 23, "double", 0), ("nesterov", 24, "bool", 0)],
    "AdadeltaConfig": [("rho", 33, "double", 0), ("epsilon", 31, "double", 0), ("decay", 32, "double", 0)],
    "AdagradConfig": [("epsilon", 41, "double", 0), ("decay", 42, "double", 0)],
    "AdamConfig": [("beta_1", 41, "double", 0), ("beta_2", 42, "double", 0), ("epsilon", 43, "double", 0),
                   ("decay", 44, "double", 0)],
    "ConstLrConfig": [("learning_rate", 1, "double", 0)],
    "LinearLrConfig": [("learning_rate", 1, "double", 0), ("lr_decay_a", 2, "double", 0),
                       ("lr_decay_b", 3, "double", 0)],
    "OptimizerConfig": [
        ("optimizer", 1, "int32", 0), ("sgd", 3, "SGDConfig", 0), ("adadelta", 4, "AdadeltaConfig", 0),
        ("adagrad", 5, "AdagradConfig", 0), ("adam", 6, "AdamConfig", 0), ("lr_policy", 11, "int32", 0),
        ("const_lr", 12, "ConstLrConfig", 0), ("linear_lr", 13, "LinearLrConfig", 0),
        ("clip_norm", 101, "double", 0), ("clip_value", 102, "double", 0)],
}
for _m, _fs in _schemas.items():
    cp._S[_m] = _fs
    cp._FIELDS[_m] = {f[0]: f for f in _fs}
    cp._BYNUM[_m] = {f[1]: f for f in _fs}


def optimizer_config(kind="sgd", lr=0.01, lr_policy="const", lr_decay_a=0.0, lr_decay_b=0.0, **kw) -> bytes:
    """Serialised OptimizerConfig from keyword settings (momentum / decay / nesterov,
    rho / epsilon, beta_1 / beta_2)."""
    k = _KIND[kind]
    msg = {"optimizer": k}
    if k == SGD:
        msg["sgd"] = {f: kw[f] for f in ("momentum", "decay", "nesterov") if f in kw}
    elif k == ADADELTA:
        msg["adadelta"] = {f: kw[f] for f in ("rho", "epsilon", "decay") if f in kw}
    elif k == ADAGRAD:
        msg["adagrad"] = {f: kw[f] for f in ("epsilon", "decay") if f in kw}
    else:
        msg["adam"] = {f: kw[f] for f in ("beta_1", "beta_2", "epsilon", "decay") if f in kw}
    if lr_policy == "linear":
        msg.update(lr_policy=1, linear_lr={"learning_rate": lr, "lr_decay_a": lr_decay_a, "lr_decay_b": lr_decay_b})
    else:
        msg.update(lr_policy=0, const_lr={"learning_rate": lr})
    return cp.encode("OptimizerConfig", msg)


class ParameterOptimizer:
    def __init__(self, config: bytes, param, state: bytes | None = None):
        p = np.ascontiguousarray(param, np.float32)
        self.shape = p.shape
        L = runtime.lib()
        self._h = L.pa_opt_create(config, len(config), 4, p.ctypes.data, p.nbytes, state, len(state) if state else 0)
        if not self._h:
            raise ValueError("pa_opt_create: bad OptimizerConfig / state")

    def update(self, grad):
        g = np.ascontiguousarray(grad, np.float32)
        if runtime.lib().pa_opt_update(self._h, 4, g.ctypes.data, g.nbytes) != 0:
            raise ValueError("pa_opt_update: gradient size mismatch")

    def weights(self) -> np.ndarray:
        buf = ctypes.c_void_p()
        n = runtime.lib().pa_opt_get_weights(self._h, ctypes.byref(buf))
        return np.ctypeslib.as_array((ctypes.c_float * n).from_address(buf.value)).copy().reshape(self.shape)

    def state(self) -> bytes:
        buf = ctypes.c_char_p()
        n = runtime.lib().pa_opt_get_state(self._h, ctypes.byref(buf))
        return ctypes.string_at(buf, n)

    def close(self):
        if self._h:
            runtime.lib().pa_opt_release(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
