"""The v1 config parser's ModelConfig / TrainerConfig output
(trainer_config_helpers/config_proto.py) against the reference's own expected
outputs: python/paddle/trainer_config_helpers/tests/configs/protostr/*.protostr
(text-format ModelConfig files, read as data).  Each config below builds the
topology of the reference test config of the same name; the layer names, types,
sizes, activations, inputs, parameter names / sizes / dims and input / output
layer names must match.  Also: proto2 wire round trip of a whole TrainerConfig."""
import os

import pytest

import paddle_amd.trainer_config_helpers as tch
from paddle_amd.trainer_config_helpers import config_proto as cp

PROTOSTR = "/root/reference/python/paddle/trainer_config_helpers/tests/configs/protostr"


def _fc():
    tch.settings(batch_size=1000, learning_rate=1e-5)
    din = tch.data_layer(name="data", size=100)
    trans = tch.trans_layer(input=din)
    hidden = tch.fc_layer(input=trans, size=100, bias_attr=False)
    mask = tch.data_layer(name="mask", size=100)
    sel = tch.selective_fc_layer(input=din, select=mask, size=100, act=tch.SigmoidActivation())
    tch.outputs(hidden, sel)


def _activations():
    tch.settings(learning_rate=1e-4, batch_size=1000)
    din = tch.data_layer(name="input", size=100)
    acts = [tch.TanhActivation, tch.SigmoidActivation, tch.SoftmaxActivation, tch.IdentityActivation,
            tch.LinearActivation, tch.ExpActivation, tch.ReluActivation, tch.BReluActivation,
            tch.SoftReluActivation, tch.STanhActivation, tch.AbsActivation, tch.SquareActivation]
    tch.outputs([tch.fc_layer(input=din, size=100, act=a(), name="layer_%d" % i) for i, a in enumerate(acts)])


def _util():
    tch.settings(learning_rate=1e-4, batch_size=1000)
    a = tch.data_layer(name="a", size=10)
    b = tch.data_layer(name="b", size=10)
    r = tch.addto_layer(input=[a, b])
    c1 = tch.concat_layer(input=[a, b])
    c2 = tch.concat_layer(input=[tch.identity_projection(input=a), tch.identity_projection(input=b)])
    tch.outputs(r, c1, c2)


def _last_first_seq():
    tch.settings(batch_size=1000, learning_rate=1e-5)
    din = tch.data_layer(name="data", size=30)
    outs = []
    for op in (tch.first_seq, tch.last_seq):
        for al in (tch.AggregateLevel.TO_SEQUENCE, tch.AggregateLevel.TO_NO_SEQUENCE):
            outs.append(op(input=din, agg_level=al))
    for op in (tch.first_seq, tch.last_seq):
        outs.append(op(input=din, agg_level=tch.AggregateLevel.TO_NO_SEQUENCE, stride=5))
    tch.outputs(outs)


def _l2_distance():
    tch.outputs(tch.l2_distance_layer(x=tch.data_layer(name="x", size=128), y=tch.data_layer(name="y", size=128)))


def _repeat():
    tch.settings(batch_size=1000, learning_rate=1e-5)
    din = tch.data_layer(name="data", size=30)
    tch.outputs(tch.repeat_layer(input=din, num_repeats=10, as_row_vector=True),
                tch.repeat_layer(input=din, num_repeats=10, act=tch.TanhActivation(), as_row_vector=False))


def _clip():
    tch.outputs(tch.clip_layer(input=tch.data_layer(name="input", size=300), min=-10, max=10))


def _dot_prod():
    v1 = tch.data_layer(name="vector1", size=10)
    v2 = tch.data_layer(name="vector2", size=10)
    tch.outputs(tch.dot_prod_layer(input1=v1, input2=v2))


def _row_l2_norm():
    tch.outputs(tch.row_l2_norm_layer(input=tch.data_layer(name="input", size=300)))


def _fm():
    tch.outputs(tch.factorization_machine(input=tch.data_layer(name="data", size=1024), factor_size=10))


CONFIGS = {"test_fc": _fc, "layer_activations": _activations, "util_layers": _util,
           "last_first_seq": _last_first_seq, "test_l2_distance_layer": _l2_distance,
           "test_repeat_layer": _repeat, "test_clip_layer": _clip, "test_dot_prod_layer": _dot_prod,
           "test_row_l2_norm_layer": _row_l2_norm, "test_factorization_machine": _fm}


def _core(mc):
    layers = [(lc["name"], lc["type"], lc.get("size"), lc.get("active_type", ""),
               tuple((i["input_layer_name"], i.get("input_parameter_name")) for i in lc.get("inputs", [])),
               lc.get("bias_parameter_name")) for lc in mc.get("layers", [])]
    params = sorted((p["name"], p.get("size"), tuple(p.get("dims", []))) for p in mc.get("parameters", []))
    return layers, params, mc.get("input_layer_names", []), mc.get("output_layer_names", [])


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_model_config_matches_reference_protostr(name):
    path = os.path.join(PROTOSTR, name + ".protostr")
    if not os.path.exists(path):
        pytest.skip("reference protostr not present")
    c = tch.parse_config(CONFIGS[name])
    got = _core(c.model_config())
    exp = _core(cp.from_text("ModelConfig", open(path).read()))
    assert got[0] == exp[0]
    assert got[1] == exp[1]
    assert got[2:] == exp[2:]
    # the same message through the wire format and back
    mc = c.model_config()
    assert cp.decode("ModelConfig", cp.encode("ModelConfig", mc)) == cp.from_text("ModelConfig", cp.to_text(
        "ModelConfig", mc))


def test_trainer_config_wire_round_trip_and_text():
    def conf():
        tch.settings(batch_size=64, learning_rate=2e-3, learning_method=tch.AdamOptimizer(beta1=0.8),
                     regularization=tch.L2Regularization(1e-4))
        x = tch.data_layer(name="x", size=8)
        h = tch.fc_layer(input=x, size=16, act=tch.ReluActivation())
        p = tch.fc_layer(input=h, size=3, act=tch.SoftmaxActivation())
        tch.outputs(tch.classification_cost(input=p, label=tch.data_layer(name="label", size=3)))

    c = tch.parse_config(conf)
    tc = cp.decode("TrainerConfig", c.proto())
    oc = tc["opt_config"]
    assert oc["batch_size"] == 64 and oc["learning_method"] == "adam" and abs(oc["adam_beta1"] - 0.8) < 1e-12
    assert abs(oc["learning_rate"] - 2e-3) < 1e-15
    mc = tc["model_config"]
    assert [lc["type"] for lc in mc["layers"]] == ["data", "fc", "fc", "data", "multi-class-cross-entropy"]
    assert mc["layers"][1]["bias_parameter_name"] == "___fc_layer_0__.wbias"
    assert mc["input_layer_names"] == ["x", "label"]
    # every v1 parameter name maps onto the Fluid parameter that holds it, with its shape
    from paddle_amd.v2._core import STATE

    fluid_params = {p.name: tuple(p.shape) for p in STATE["main"].global_block().all_parameters()}
    for p in mc["parameters"]:
        fp = c.parameter_name_map[p["name"]]
        assert fp in fluid_params and int(p["size"]) == int(__import__("numpy").prod(fluid_params[fp]))
    txt = c.to_text(whole=True)
    assert cp.from_text("TrainerConfig", txt) == tc


def test_negative_and_packed_fields_decode():
    msg = {"name": "p", "size": 6, "dims": [2, 3], "device": -1, "initial_std": 0.5}
    b = cp.encode("ParameterConfig", msg)
    assert cp.decode("ParameterConfig", b) == msg
    # packed repeated dims (field 9, wire type 2) as another encoder may write them
    packed = cp._key(1, 2) + bytes([1]) + b"p" + cp._key(9, 2) + bytes([2, 2, 3])
    assert cp.decode("ParameterConfig", packed) == {"name": "p", "dims": [2, 3]}


def test_dump_config_cli(tmp_path, capsys):
    from paddle_amd.utils import dump_config

    cfg = tmp_path / "conf.py"
    cfg.write_text("from paddle_amd.trainer_config_helpers import *\n"
                   "settings(batch_size=10, learning_rate=0.1)\n"
                   "n = get_config_arg('n', int, 4)\n"
                   "x = data_layer(name='x', size=6)\n"
                   "outputs(fc_layer(input=x, size=n, act=SoftmaxActivation()))\n")
    assert dump_config.main([str(cfg), "n=5"]) == 0
    mc = cp.from_text("ModelConfig", capsys.readouterr().out)
    assert mc["layers"][1]["size"] == 5 and mc["layers"][1]["active_type"] == "softmax"
    assert dump_config.main([str(cfg), "n=5", "--whole"]) == 0
    tc = cp.from_text("TrainerConfig", capsys.readouterr().out)
    assert tc["opt_config"]["batch_size"] == 10 and tc["config_files"] == [str(cfg)]
