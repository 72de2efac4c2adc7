"""v1 model-config DSL (reference python/paddle/trainer_config_helpers/: layers.py,
activations.py, poolings.py, optimizers.py, evaluators.py, networks.py, attrs.py)
and its config parser (python/paddle/trainer/config_parser.py ``parse_config``).

A v1 config is a Python script that calls ``settings(...)``, builds a topology
with ``data_layer`` / ``fc_layer`` / ... and declares ``outputs(...)``; the
reference turns it into a ModelConfig proto for the legacy GradientMachine.  Here
the same DSL builds the v2 facade's Fluid program (paddle_amd/v2: each layer is
one or a few Fluid ops on the MI355X kernels), and ``parse_config`` returns a
``TrainerConfig`` whose ``make_trainer()`` gives a v2 ``trainer.SGD`` with the
optimizer that ``settings`` described.

Data-layer types: v1 takes them from the data provider (``@provider(input_types=
...)``); here ``data_layer(name, size, type=...)`` takes an explicit v2 data type,
and without one a layer whose name contains ``label`` is ``integer_value(size)``,
any other ``dense_vector(size)``.
"""
from __future__ import annotations

import os

from .. import v2
from ..v2 import activation as _act
from ..v2 import data_type as _dt
from ..v2 import evaluator as _ev
from ..v2 import layer as _l
from ..v2 import networks as _nets
from ..v2 import optimizer as _opt
from ..v2 import pooling as _pool
from ..v2._core import STATE
from . import config_proto as _cp
from . import layers_v1 as _v1
from .layers_v1 import *  # noqa: F401,F403  (the rest of layers.py __all__)

# ------------------------------------------------------------------ activations
TanhActivation, ReluActivation, SigmoidActivation = _act.Tanh, _act.Relu, _act.Sigmoid
SoftmaxActivation, LinearActivation, IdentityActivation = _act.Softmax, _act.Linear, _act.Identity
ExpActivation, AbsActivation, SquareActivation = _act.Exp, _act.Abs, _act.Square
BReluActivation, SoftReluActivation, STanhActivation = _act.BRelu, _act.SoftRelu, _act.STanh
SequenceSoftmaxActivation, LogActivation, SqrtActivation = _act.SequenceSoftmax, _act.Log, _act.Sqrt
ReciprocalActivation = _act.Reciprocal

# ------------------------------------------------------------------ poolings
MaxPooling, AvgPooling, SumPooling, SquareRootNPooling = _pool.Max, _pool.Avg, _pool.Sum, _pool.SquareRootN
CudnnMaxPooling, CudnnAvgPooling = _pool.Max, _pool.Avg


# ------------------------------------------------------------------ attributes
class ParameterAttribute:
    def __init__(self, name=None, initial_std=None, initial_mean=None, learning_rate=None, l2_rate=None,
                 initial_max=None, initial_min=None, is_static=False, **kw):
        self.name, self.initial_std, self.initial_mean = name, initial_std, initial_mean
        self.learning_rate, self.l2_rate = learning_rate, l2_rate
        self.initial_max, self.initial_min, self.is_static = initial_max, initial_min, is_static


class ExtraLayerAttribute:
    def __init__(self, drop_rate=None, error_clipping_threshold=None, device=None, **kw):
        self.drop_rate, self.error_clipping_threshold = drop_rate, error_clipping_threshold


ParamAttr, ExtraAttr = ParameterAttribute, ExtraLayerAttribute


# ------------------------------------------------------------------ optimizers / settings
class L2Regularization(_opt.L2Regularization):
    pass


class BaseSGDOptimizer:
    kind = None

    def __init__(self, **kw):
        self.kw = kw


class MomentumOptimizer(BaseSGDOptimizer):
    def __init__(self, momentum=None, sparse=False):
        super().__init__(momentum=momentum or 0.0)
        self.kind = _opt.Momentum


class AdamOptimizer(BaseSGDOptimizer):
    def __init__(self, beta1=0.9, beta2=0.999, epsilon=1e-8):
        super().__init__(beta1=beta1, beta2=beta2, epsilon=epsilon)
        self.kind = _opt.Adam


class AdamaxOptimizer(BaseSGDOptimizer):
    def __init__(self, beta1=0.9, beta2=0.999):
        super().__init__(beta1=beta1, beta2=beta2)
        self.kind = _opt.Adamax


class AdaGradOptimizer(BaseSGDOptimizer):
    def __init__(self):
        super().__init__()
        self.kind = _opt.AdaGrad


class DecayedAdaGradOptimizer(BaseSGDOptimizer):
    def __init__(self, rho=0.95, epsilon=1e-6):
        super().__init__(rho=rho, epsilon=epsilon)
        self.kind = _opt.DecayedAdaGrad


class AdaDeltaOptimizer(BaseSGDOptimizer):
    def __init__(self, rho=0.95, epsilon=1e-6):
        super().__init__(rho=rho, epsilon=epsilon)
        self.kind = _opt.AdaDelta


class RMSPropOptimizer(BaseSGDOptimizer):
    def __init__(self, rho=0.95, epsilon=1e-6):
        super().__init__(rho=rho, epsilon=epsilon)
        self.kind = _opt.RMSProp


_CFG: dict = {}


def settings(batch_size, learning_rate=1e-3, learning_method=None, regularization=None,
             gradient_clipping_threshold=None, model_average=None, **kw):
    """optimizers.py settings(): the optimization section of the config."""
    _CFG.update(batch_size=int(batch_size), learning_rate=float(learning_rate),
                learning_method=learning_method or MomentumOptimizer(), regularization=regularization,
                gradient_clipping_threshold=gradient_clipping_threshold, extra=kw)


def define_py_data_sources2(train_list, test_list, module, obj, args=None):
    """data_sources.py:158: the train / test file lists and the PyDataProvider2
    provider ``module.obj`` (``paddle_amd.trainer`` reads them)."""
    _CFG["data_sources"] = {"train_list": train_list, "test_list": test_list, "module": module, "obj": obj,
                            "args": args}


def outputs(*layers):
    if "outputs" not in _CFG:  # the model's input layers are traced from the first call's outputs
        _CFG["first_outputs"] = [v for x in layers for v in (x if isinstance(x, (list, tuple)) else [x])]
    out = list(_CFG.get("outputs") or [])  # repeated outputs(...) calls add up (reference Outputs)
    for x in layers:
        for v in (x if isinstance(x, (list, tuple)) else [x]):
            if all(v is not o for o in out):
                out.append(v)
    _CFG["outputs"] = out


def get_config_arg(name, type, default=None):
    """config_parser.get_config_arg: a value of ``config_arg_str`` ("a=1,b=x")."""
    v = _CFG.get("args", {}).get(name)
    if v is None:
        return default
    if type is bool:
        return v.lower() in ("1", "true", "t", "yes")
    return type(v)


# ------------------------------------------------------------------ layers
def data_layer(name, size, height=None, width=None, type=None, **kw):
    if type is None:
        type = _dt.integer_value(size) if "label" in name else _dt.dense_vector(size)
    out = _l.data(name=name, type=type)
    if height and width:
        out.v2_hw = (int(height), int(width))  # image layers read [C, H, W] from it
        if kw.get("depth"):
            out.v2_dhw = (int(kw["depth"]), int(height), int(width))  # 3-D layers: [C, D, H, W]
    return out


def _one(x):
    return x[0] if isinstance(x, (list, tuple)) and len(x) == 1 else x


def fc_layer(input, size, act=None, name=None, param_attr=None, bias_attr=None, layer_attr=None, **kw):
    """A list of inputs is one projection each, summed with one bias: the same as
    one fc over their concatenation."""
    x = _one(input)
    if isinstance(x, (list, tuple)):
        x = list(x)  # one weight per input (w0, w1, ...), summed before the bias
    out = _l.fc(input=x, size=size, act=act if act is not None else TanhActivation(), name=name,
                param_attr=param_attr, bias_attr=bias_attr)
    if layer_attr is not None and getattr(layer_attr, "drop_rate", None):
        out = _l.dropout(input=out, dropout_rate=layer_attr.drop_rate)
    return _v1._named(out, name)  # a recurrent_group memory(name=...) may read it


def embedding_layer(input, size, name=None, param_attr=None, **kw):
    out = _l.embedding(input=input, size=size)
    out.v2_size = size  # the v1 layer width (a table projection), whatever the id layout
    return out


def img_conv_layer(input, filter_size, num_filters, num_channels=None, stride=1, padding=0, act=None, groups=1,
                   name=None, bias_attr=None, param_attr=None, **kw):
    return _l.img_conv(input=input, filter_size=filter_size, num_filters=num_filters, num_channels=num_channels,
                       stride=stride, padding=padding, act=act if act is not None else ReluActivation(),
                       groups=groups, bias_attr=bias_attr, param_attr=param_attr, trans=kw.get("trans", False),
                       dilation=kw.get("dilation", 1))


def img_pool_layer(input, pool_size, stride=1, padding=0, pool_type=None, num_channels=None, name=None, **kw):
    return _l.img_pool(input=input, pool_size=pool_size, stride=stride, padding=padding,
                       pool_type=pool_type or MaxPooling(), num_channels=num_channels)


def batch_norm_layer(input, act=None, name=None, **kw):
    return _l.batch_norm(input=input, act=act if act is not None else ReluActivation())


def dropout_layer(input, dropout_rate, name=None):
    return _l.dropout(input=input, dropout_rate=dropout_rate)


def concat_layer(input, act=None, name=None, **kw):
    ins = list(input) if isinstance(input, (list, tuple)) else [input]
    ins = [x.build(x.size) if isinstance(x, _v1._Projection) else x for x in ins]  # concat of projections
    return _v1._named(_l.concat(input=ins), name)


def addto_layer(input, act=None, name=None, bias_attr=None, **kw):
    from .. import fluid

    with v2._core.guard():
        ins = list(input) if isinstance(input, (list, tuple)) else [input]
        s = fluid.layers.sums(ins) if len(ins) > 1 else ins[0]
        a = _act.act_name(act)
        out = getattr(fluid.layers, a)(s) if a and a not in ("linear", "identity") else s
        out.v2_size = getattr(ins[0], "v2_size", None)
        return _v1._named(out, name)


def pooling_layer(input, pooling_type=None, name=None, **kw):
    return _l.pooling(input=input, pooling_type=pooling_type or MaxPooling())


def last_seq(input, name=None, **kw):
    return _l.last_seq(input=input)


def first_seq(input, name=None, **kw):
    return _l.first_seq(input=input)


def maxid_layer(input, name=None, **kw):
    return _l.max_id(input=input)


def classification_cost(input, label, weight=None, name=None, evaluator=None, **kw):
    return _l.classification_cost(input=input, label=label, name=name, weight=weight)


def cross_entropy(input, label, weight=None, name=None, **kw):
    return _l.cross_entropy_cost(input=input, label=label, weight=weight)


def regression_cost(input, label, weight=None, name=None, **kw):
    return _l.square_error_cost(input=input, label=label, weight=weight)


mse_cost = square_error_cost = regression_cost

# ------------------------------------------------------------------ networks
simple_img_conv_pool = _nets.simple_img_conv_pool
sequence_conv_pool = _nets.sequence_conv_pool
from .networks_v1 import *  # noqa: E402,F401,F403  (recurrent units / groups, bidirectional RNNs, attention)
from . import layer_math  # noqa: E402  (layer_math.exp(x), 1 + x, y * z ... on v1 layers)

layer_math.install()

# ------------------------------------------------------------------ evaluators
classification_error_evaluator = _ev.classification_error
auc_evaluator = _ev.auc
precision_recall_evaluator = _ev.precision_recall
pnpair_evaluator = _ev.pnpair
chunk_evaluator = _ev.chunk
ctc_error_evaluator = _ev.ctc_error
sum_evaluator = _ev.sum
column_sum_evaluator = _ev.column_sum
value_printer_evaluator = _ev.value_printer
maxid_printer_evaluator = _ev.maxid_printer
classification_error_printer_evaluator = _ev.classification_error_printer


# ------------------------------------------------------------------ config parser
class TrainerConfig:
    """What config_parser.parse_config returns: the model (outputs, data layers,
    parameters -- a Fluid program) and the optimization settings; ``proto()`` /
    ``to_text()`` give the reference's TrainerConfig message (config_proto.py)."""

    def __init__(self, cfg, rec=None):
        self._cfg = dict(cfg)
        self._rec = rec
        self.outputs = cfg.get("outputs", [])
        self.batch_size = cfg.get("batch_size")
        self.learning_rate = cfg.get("learning_rate")
        self.learning_method = cfg.get("learning_method")
        self.regularization = cfg.get("regularization")
        self.gradient_clipping_threshold = cfg.get("gradient_clipping_threshold")
        self.program = STATE["main"]
        self.input_layer_names = list(STATE["data"])

    @property
    def cost(self):
        return self.outputs[0]

    def update_equation(self):
        m = self.learning_method or MomentumOptimizer()
        return m.kind(learning_rate=self.learning_rate, regularization=self.regularization,
                      gradient_clipping_threshold=self.gradient_clipping_threshold, **m.kw)

    def model_config(self) -> dict:
        """ModelConfig (layers, parameters, input / output layer names, root sub-model)."""
        return _cp.model_config(self._rec, self.outputs, self._cfg.get("first_outputs"))

    @property
    def parameter_name_map(self) -> dict:
        """v1 parameter name (``___fc_layer_0__.w0``) -> the Fluid parameter holding it."""
        return dict(self._rec.param_map)

    def trainer_config(self) -> dict:
        tc = {"model_config": self.model_config(), "opt_config": _cp.opt_config(self._cfg)}
        train, test = _cp.data_configs(self._cfg)
        if train:
            tc["data_config"] = train
        if test:
            tc["test_data_config"] = test
        # (config_files lists only Import()-ed sub-configs in the reference, never the
        # main config file itself)
        tc["save_dir"] = "./output/model"
        tc["start_pass"] = 0
        return tc

    def proto(self) -> bytes:
        """The serialised TrainerConfig (proto/TrainerConfig.proto wire format)."""
        return _cp.encode("TrainerConfig", self.trainer_config())

    def to_text(self, whole=False) -> str:
        """Text format of the ModelConfig (``whole``: of the TrainerConfig)."""
        if whole:
            return _cp.to_text("TrainerConfig", self.trainer_config()) + "\n"
        return _cp.to_text("ModelConfig", self.model_config()) + "\n"

    def make_trainer(self, parameters=None, **remote):
        """``remote``: is_local=False, pserver_spec=..., trainer_id=... (parameter servers)."""
        params = parameters or v2.parameters.create(self.cost)
        return v2.trainer.SGD(cost=self.cost, parameters=params, update_equation=self.update_equation(),
                              **remote), params


def parse_config(config, config_arg_str=""):
    """Runs a v1 config (a file path, or a callable taking no arguments) with this
    DSL in scope and returns its TrainerConfig.  ``config_arg_str``: "k=v,k2=v2",
    read inside the config with get_config_arg."""
    args = dict(kv.split("=", 1) for kv in config_arg_str.split(",") if "=" in kv)
    _CFG.clear()
    _CFG["args"] = args
    v2.init(use_gpu=STATE.get("use_gpu", False))
    rec = _cp.start()
    try:
        if callable(config):
            config()
        else:
            path = os.fspath(config)
            _CFG["config_file"] = path
            with open(path) as f:
                code = compile(f.read(), path, "exec")
            g = {k: v for k, v in globals().items() if not k.startswith("_")}
            g["__file__"] = path
            exec(code, g)  # noqa: S102  (a v1 config is a Python script, as in the reference)
    finally:
        _cp._REC.clear()
    if not _CFG.get("outputs"):
        raise ValueError("the config declared no outputs(...)")
    return TrainerConfig(_CFG, rec)


# every layer function records its LayerConfig while a config is parsed
for _n, _f in list(globals().items()):
    if _n in _cp._TYPE and callable(_f) and not isinstance(_f, type):
        globals()[_n] = _cp.recorded(_n, _f)
del _n, _f
