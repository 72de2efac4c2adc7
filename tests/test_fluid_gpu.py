"""Static-graph programs on the HIP device (CUDAPlace) -- same book nets as the CPU tests."""
import numpy as np
import pytest

import paddle_amd.fluid as fluid
from test_book_cpu import _train_digits, conv_net, mlp

pytestmark = pytest.mark.gpu


def test_recognize_digits_conv_gpu(tmp_path):
    first, last, acc = _train_digits(conv_net, fluid.CUDAPlace(0), epochs=3, tmpdir=str(tmp_path / "c"))
    assert last < first and acc > 0.2


def test_recognize_digits_mlp_gpu():
    # (initial weights come from the device RNG, so CPU and GPU runs start from
    # different points; both must converge)
    first, last, acc = _train_digits(mlp, fluid.CUDAPlace(0), epochs=5)
    assert last < first and acc > 0.2


def test_dynamic_rnn_trains_gpu():
    """DynamicRNN + while_grad on the device: LoD feeds from the host, loop counters
    and rank tables on the host, step math on the GPU."""
    import torch

    from paddle_amd.framework import core

    D, H, LOD = 5, 6, [0, 3, 5, 9]
    main, startup = fluid.Program(), fluid.Program()
    main.random_seed = startup.random_seed = 3
    with fluid.program_guard(main, startup):
        x = fluid.layers.data(name="x", shape=[D], dtype="float32", lod_level=1)
        y = fluid.layers.data(name="y", shape=[1], dtype="float32", lod_level=1)
        drnn = fluid.layers.DynamicRNN()
        with drnn.block():
            word = drnn.step_input(x)
            prev = drnn.memory(shape=[H], value=0.0)
            hidden = fluid.layers.fc(input=[word, prev], size=H, act="tanh")
            drnn.update_memory(prev, hidden)
            drnn.output(hidden)
        pred = fluid.layers.fc(drnn(), size=1)
        loss = fluid.layers.mean(fluid.layers.square_error_cost(pred, y))
        fluid.optimizer.Adam(learning_rate=0.05).minimize(loss)
    exe = fluid.Executor(fluid.CUDAPlace(0))
    rng = np.random.RandomState(1)
    xv = rng.randn(LOD[-1], D).astype("float32")
    yv = np.cumsum(xv[:, :1], 0).astype("float32") * 0.3
    with fluid.executor.scope_guard(core.Scope()):
        exe.run(startup)
        ls = [float(np.asarray(exe.run(main, feed={"x": core.LoDTensor(torch.from_numpy(xv), [LOD]),
                                                   "y": core.LoDTensor(torch.from_numpy(yv), [LOD])},
                                       fetch_list=[loss])[0]).reshape(-1)[0]) for _ in range(30)]
    assert ls[-1] < 0.5 * ls[0], ls


def test_stacked_lstm_benchmark_program_gpu(capsys):
    """The reference's stacked_dynamic_lstm benchmark program (embedding, DynamicRNN
    LSTM, sequence_pool last, Adam) runs on the device (benchmarks/reference_suite.py)."""
    import argparse
    import json
    import os
    import sys

    import torch

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "benchmarks"))
    import reference_suite as rs

    a = argparse.Namespace(batch=4, steps=2, warmup=1, max_len=12)
    rs.bench_stacked_lstm_fluid(a, torch.device("cuda"))
    line = [ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("{")][-1]
    assert json.loads(line)["value"] > 0
