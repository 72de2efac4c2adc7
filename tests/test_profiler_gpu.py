"""In-process device activity trace on the HIP device: every profiled op range gets
GPU start/end times on the device clock (HIP events against a start event), and
the timeline puts them on a gpu:<id> track (reference: platform/device_tracer.cc,
tools/timeline.py)."""
import json

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_device_trace_of_fluid_ops(tmp_path):
    import paddle_amd.fluid as fluid
    from paddle_amd.utils.profiler import chrome_trace

    main, st = fluid.Program(), fluid.Program()
    with fluid.program_guard(main, st):
        x = fluid.layers.data("x", [512])
        h = fluid.layers.fc(x, 1024, act="relu")
        loss = fluid.layers.mean(fluid.layers.fc(h, 256))
        fluid.optimizer.SGD(0.01).minimize(loss)
    place = fluid.CUDAPlace(0)
    exe = fluid.Executor(place)
    path = str(tmp_path / "prof")
    with fluid.scope_guard(fluid.Scope()):
        exe.run(st)
        with fluid.profiler.profiler("All", sorted_key="total", profile_path=path):
            for _ in range(2):
                exe.run(main, feed={"x": np.random.rand(256, 512).astype("float32")}, fetch_list=[loss])
    prof = json.load(open(path))
    gpu = [e for e in prof["events"] if e["type"] == "GPUKernel"]
    cpu = [e for e in prof["events"] if e["type"] == "CPU"]
    assert gpu and len(gpu) == len(cpu)
    assert all(e["end_ns"] >= e["start_ns"] >= 0 for e in gpu)
    starts = [e["start_ns"] for e in gpu]
    assert starts == sorted(starts)  # one stream: device ranges in issue order
    assert any(e["name"] == "mul" and e["end_ns"] > e["start_ns"] for e in gpu)
    tr = json.loads(chrome_trace({"trainer": prof}))["traceEvents"]
    assert any(e["ph"] == "M" and e["args"]["name"].startswith("trainer:gpu:") for e in tr)
