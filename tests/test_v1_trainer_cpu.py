"""v1 trainer front end + PyDataProvider2 (reference legacy/trainer TrainerMain.cpp,
python/paddle/trainer/PyDataProvider2.py, data_sources.py define_py_data_sources2):
a v1 config naming a @provider module and train/test file lists, trained and
tested through ``paddle_amd.trainer.main`` with parameter tars per pass."""
import os
import sys

import numpy as np

PROVIDER = '''
from paddle.trainer.PyDataProvider2 import *

def hook(settings, dim, **kw):
    settings.input_types = {"pixel": dense_vector(dim), "label": integer_value(3)}

@provider(init_hook=hook, cache=CacheType.CACHE_PASS_IN_MEM, check=True)
def process(settings, filename):
    with open(filename) as f:
        for line in f:
            v = [float(x) for x in line.split()]
            yield {"label": int(v[-1]), "pixel": v[:-1]}
'''

CONFIG = '''
from paddle.trainer_config_helpers import *

define_py_data_sources2(train_list="train.list", test_list="test.list", module="v1_provider", obj="process",
                        args={"dim": 8})
settings(batch_size=16, learning_rate=0.1, learning_method=MomentumOptimizer(0.9))
x = data_layer(name="pixel", size=8)
y = data_layer(name="label", size=3)
pred = fc_layer(input=fc_layer(input=x, size=16, act=ReluActivation()), size=3, act=SoftmaxActivation())
outputs(classification_cost(input=pred, label=y))
'''


def _write_data(d, name, n, seed, w):
    rs = np.random.RandomState(seed)
    x = rs.randn(n, 8)
    y = (x @ w).argmax(1)
    with open(os.path.join(d, name), "w") as f:
        for xi, yi in zip(x, y):
            f.write(" ".join(f"{v:.5f}" for v in xi) + f" {yi}\n")


def test_v1_trainer_trains_tests_and_saves(tmp_path, capsys):
    import paddle.trainer as T  # noqa: F401  (the paddle.trainer alias)
    from paddle_amd import trainer

    d = str(tmp_path)
    w = np.random.RandomState(0).randn(8, 3)
    for i in range(2):
        _write_data(d, f"part{i}.txt", 96, i, w)
    _write_data(d, "test0.txt", 64, 7, w)
    open(os.path.join(d, "train.list"), "w").write("part0.txt\npart1.txt\n")
    open(os.path.join(d, "test.list"), "w").write("test0.txt\n")
    open(os.path.join(d, "v1_provider.py"), "w").write(PROVIDER)
    conf = os.path.join(d, "conf.py")
    open(conf, "w").write(CONFIG)
    sys.path.insert(0, d)
    cwd = os.getcwd()
    os.chdir(d)
    try:
        costs = trainer.main(["--config", conf, "--num_passes", "4", "--log_period", "4",
                              "--save_dir", os.path.join(d, "out"), "--log_stat", "1"])
        out = capsys.readouterr().out
        assert "Pass 3 done" in out and "Test cost" in out
        assert "Stat=forwardBackward" in out and "Stat=trainBatch" in out  # legacy Stat timers
        assert np.mean(costs[-4:]) < np.mean(costs[:4])
        tar = os.path.join(d, "out", "pass-00003", "params.tar")
        assert os.path.exists(tar)
        trainer.main(["--config", conf, "--job", "test", "--init_model_path", tar])
        out = capsys.readouterr().out
        assert "Test cost" in out and "classification_error_evaluator" in out
        # --job=checkgrad: analytic vs central-difference directional derivatives
        rel = trainer.main(["--config", conf, "--job", "checkgrad", "--checkgrad_eps", "1e-3"])
        out = capsys.readouterr().out
        assert len(rel) == 4 and "checkgrad" in out
        assert max(rel.values()) < 2e-2, rel
        # --local=0: the updates run on block-sharded parameter servers (pserver2)
        from paddle_amd.distributed import pserver2

        ss = [pserver2.ParameterServer2(num_trainers=1).start() for _ in range(2)]
        try:
            spec = ",".join(f"127.0.0.1:{s.port}" for s in ss)
            costs_r = trainer.main(["--config", conf, "--num_passes", "4", "--log_period", "4", "--local", "0",
                                    "--pservers", spec])
            assert np.mean(costs_r[-4:]) < np.mean(costs_r[:4])
            assert all(len(s.blocks) > 0 for s in ss)
        finally:
            for s in ss:
                s.stop()
    finally:
        os.chdir(cwd)
        sys.path.remove(d)
