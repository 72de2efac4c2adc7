"""v1 config DSL + parse_config (reference trainer_config_helpers/, trainer/
config_parser.py): a v1-style config file with settings / data_layer / fc_layer /
classification_cost / evaluators / outputs and a config_arg_str, parsed into a
TrainerConfig and trained through the v2 trainer."""
import numpy as np

CONFIG = '''
from paddle.trainer_config_helpers import *

hidden = get_config_arg("hidden", int, 8)
settings(batch_size=32, learning_rate=0.05, learning_method=MomentumOptimizer(0.9),
         regularization=L2Regularization(1e-4))
img = data_layer(name="pixel", size=16)
lbl = data_layer(name="label", size=4)
h = fc_layer(input=img, size=hidden, act=ReluActivation())
h2 = fc_layer(input=[h, img], size=hidden, act=TanhActivation())
pred = fc_layer(input=h2, size=4, act=SoftmaxActivation())
cost = classification_cost(input=pred, label=lbl)
auc_evaluator(input=pred, label=lbl)
outputs(cost)
'''


def test_v1_config_parses_and_trains(tmp_path):
    import paddle.trainer_config_helpers as tch

    path = tmp_path / "mlp_conf.py"
    path.write_text(CONFIG)
    conf = tch.parse_config(str(path), "hidden=24")
    assert conf.batch_size == 32 and abs(conf.learning_rate - 0.05) < 1e-12
    assert conf.input_layer_names == ["pixel", "label"]
    # the config arg reached the topology: first fc weight is [16, 24]
    shapes = {op.type for op in conf.program.global_block().ops}
    assert "mul" in shapes and "softmax" in shapes
    trainer, params = conf.make_trainer()
    assert any(tuple(params.get_shape(k)) == (16, 24) for k in params.keys())
    rs = np.random.RandomState(0)
    w = rs.randn(16, 4)

    def reader():
        x = rs.randn(256, 16).astype("float32")
        y = (x @ w).argmax(1)
        for i in range(0, 256, conf.batch_size):
            yield [(x[j], int(y[j])) for j in range(i, i + conf.batch_size)]

    costs = []
    trainer.train(reader=reader, num_passes=4, feeding={"pixel": 0, "label": 1},
                  event_handler=lambda e: costs.append(e.cost) if hasattr(e, "cost") else None)
    assert np.mean(costs[-8:]) < np.mean(costs[:8])
    res = trainer.test(reader=reader, feeding={"pixel": 0, "label": 1})
    assert "auc_evaluator" in res.metrics and "classification_error_evaluator" in res.metrics


def test_parse_config_callable_and_missing_outputs():
    import pytest

    import paddle.trainer_config_helpers as tch

    def conf():
        tch.settings(batch_size=8, learning_rate=0.1, learning_method=tch.AdamOptimizer())
        x = tch.data_layer(name="x", size=4)
        y = tch.data_layer(name="y", size=1, type=__import__("paddle").v2.data_type.dense_vector(1))
        tch.outputs(tch.regression_cost(input=tch.fc_layer(input=x, size=1, act=tch.LinearActivation()), label=y))

    c = tch.parse_config(conf)
    assert c.update_equation().__class__.__name__ == "Adam"
    with pytest.raises(ValueError):
        tch.parse_config(lambda: tch.settings(batch_size=1))
