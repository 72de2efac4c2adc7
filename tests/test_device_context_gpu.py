"""Native device contexts (csrc/runtime/device_context.cc, platform.DeviceContextPool;
reference platform/device_context.h:39-179): per-device compute / comm / aux HIP
streams usable as torch streams, cross-stream ordering on the device, an event
pool that recycles events, and the pool handing out one context per device."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_device_context_streams_and_ordering():
    from paddle_amd import platform
    from paddle_amd.framework.core import CUDAPlace

    pool = platform.DeviceContextPool.instance()
    dc = pool.get(CUDAPlace(0))
    assert dc is pool.get(torch.device("cuda", 0)) and pool.get(torch.device("cpu")) is None
    streams = {dc.stream.cuda_stream, dc.comm_stream.cuda_stream, dc.aux_stream.cuda_stream}
    assert len(streams) == 3 and torch.cuda.current_stream().cuda_stream not in streams
    x = torch.zeros(1 << 22, device="cuda")
    with torch.cuda.stream(dc.stream):
        for _ in range(20):
            x.add_(1.0)
    dc.stream_wait(dc.COMM, dc.COMPUTE)  # comm waits for compute, on the device
    with torch.cuda.stream(dc.comm_stream):
        y = x * 2
    dc.wait()
    assert float(y[0]) == 40.0 and float(y[-1]) == 40.0
    before = dc.event_pool_stats()["created"]
    for _ in range(50):
        dc.stream_wait(dc.AUX, dc.COMM)
    st = dc.event_pool_stats()
    assert st["created"] - before <= 1 and st["pooled"] >= 1  # recycled, not re-created


def test_sharded_optimizer_runs_on_context_streams():
    from paddle_amd import platform
    from paddle_amd.parallel.sharding import FlatShardedOptimizer

    w = torch.nn.Parameter(torch.randn(64, 64, device="cuda"))
    opt = FlatShardedOptimizer([("w", w)], lr=1e-2, overlap_update=True)
    dc = platform.DeviceContextPool.instance().get(torch.device("cuda", 0))
    assert opt.opt_stream.cuda_stream == dc.aux_stream.cuda_stream
