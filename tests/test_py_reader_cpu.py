"""py_reader on the native double-buffer pipeline (csrc/runtime/reader.cc; reference
operators/reader/buffered_reader.cc, create_py_reader_op.cc): the program runs
without a feed, one batch per Executor.run, in order, EOFException at the end,
reset() + start() for the next pass; plus the pipeline's queue semantics in host
mode (bounded capacity, close / EOF, reset)."""
import threading

import numpy as np
import pytest

import paddle_amd.fluid as fluid
from paddle_amd import runtime


def test_double_buffer_reader_host_mode_queue_semantics():
    if not runtime.available():
        pytest.skip("runtime library not built")
    r = runtime.DoubleBufferReader(capacity=2, nslots=2, device=None)
    batches = [[np.full((3, 4), i, "float32"), np.arange(i, i + 5, dtype="int64")] for i in range(7)]

    def produce():
        for b in batches:
            assert r.push(b)
        r.close()

    t = threading.Thread(target=produce)
    t.start()
    got = []
    while True:
        b = r.next(timeout_ms=10000)
        if b is None:
            break
        got.append([x.numpy() for x in b])
    t.join()
    assert len(got) == 7
    for (a, i), (ra, ri) in zip(got, batches):
        np.testing.assert_array_equal(a, ra)
        np.testing.assert_array_equal(i, ri)
    assert r.next(timeout_ms=100) is None  # EOF is sticky until reset
    r.reset()
    assert r.push([np.ones(2, "float32")])
    assert r.next(timeout_ms=10000)[0].tolist() == [1.0, 1.0]
    with pytest.raises(TimeoutError):
        r.next(timeout_ms=50)


def test_py_reader_feeds_executor_until_eof_cpu():
    main, startup = fluid.Program(), fluid.Program()
    with fluid.program_guard(main, startup):
        reader = fluid.layers.py_reader(capacity=4, shapes=[[-1, 6], [-1, 1]], dtypes=["float32", "int64"],
                                        name="pr")
        x, y = fluid.layers.read_file(reader)
        pred = fluid.layers.fc(x, 3, act="softmax")
        loss = fluid.layers.mean(fluid.layers.cross_entropy(pred, y))
        xs = fluid.layers.reduce_sum(x)
        fluid.optimizer.SGD(0.1).minimize(loss)
    rs = np.random.RandomState(0)
    data = [(rs.randn(5, 6).astype("float32"), rs.randint(0, 3, (5, 1)).astype("int64")) for _ in range(6)]
    reader.decorate_tensor_provider(lambda: iter(data))
    exe = fluid.Executor(fluid.CPUPlace())
    exe.run(startup)
    for _ in range(2):  # two passes: reset + start re-arms the pipeline
        reader.start()
        sums = []
        try:
            while True:
                l, s = exe.run(main, fetch_list=[loss, xs])
                assert np.isfinite(l).all()
                sums.append(float(np.asarray(s).ravel()[0]))
        except fluid.core.EOFException:
            reader.reset()
        np.testing.assert_allclose(sums, [d[0].sum() for d in data], rtol=1e-5)
