"""Device path of the native double-buffer reader (csrc/runtime/reader.cc): batches
arrive on the GPU through the prefetch thread's own HIP stream, handed to the
consumer stream by event wait + device copy; a py_reader program trains on
CUDAPlace without a feed."""
import threading

import numpy as np
import pytest
import torch

import paddle_amd.fluid as fluid
from paddle_amd import runtime

pytestmark = pytest.mark.gpu


def test_double_buffer_reader_device_mode_order_and_values():
    r = runtime.DoubleBufferReader(capacity=3, nslots=2, device="cuda")
    rs = np.random.RandomState(1)
    # varying batch sizes: slots grow; a consumer kernel runs on each batch while the
    # next ones are copied
    batches = [[rs.randn(64 * (1 + i % 3), 257).astype("float32"), rs.randint(0, 9, (7,)).astype("int64")]
               for i in range(12)]

    def produce():
        for b in batches:
            assert r.push(b)
        r.close()

    t = threading.Thread(target=produce)
    t.start()
    n = 0
    while True:
        b = r.next(timeout_ms=60000)
        if b is None:
            break
        assert b[0].is_cuda and b[1].dtype == torch.int64
        y = (b[0] * 2).sum().item()
        np.testing.assert_allclose(y, 2 * batches[n][0].astype(np.float64).sum(), rtol=1e-3)
        np.testing.assert_array_equal(b[1].cpu().numpy(), batches[n][1])
        n += 1
    t.join()
    assert n == len(batches)


def test_py_reader_trains_on_gpu():
    main, startup = fluid.Program(), fluid.Program()
    with fluid.program_guard(main, startup):
        reader = fluid.layers.py_reader(capacity=4, shapes=[[-1, 16], [-1, 1]], dtypes=["float32", "int64"],
                                        name="gpr")
        x, y = fluid.layers.read_file(reader)
        pred = fluid.layers.fc(x, 4, act="softmax")
        loss = fluid.layers.mean(fluid.layers.cross_entropy(pred, y))
        fluid.optimizer.Adam(0.01).minimize(loss)
    rs = np.random.RandomState(0)
    w = rs.randn(16, 4)
    xs = rs.randn(32, 16).astype("float32")
    ys = (xs @ w).argmax(1).reshape(-1, 1).astype("int64")
    reader.decorate_tensor_provider(lambda: iter([(xs, ys)] * 30))
    exe = fluid.Executor(fluid.CUDAPlace(0))
    exe.run(startup)
    reader.start()
    losses = []
    try:
        while True:
            (l,) = exe.run(main, fetch_list=[loss])
            losses.append(float(np.asarray(l).ravel()[0]))
    except fluid.core.EOFException:
        reader.reset()
    assert len(losses) == 30 and losses[-1] < losses[0]
