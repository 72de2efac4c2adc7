"""parallel/rccl.py without a GPU: the library loads, operand checks fail cleanly,
and comm.py keeps torch.distributed unless FLAGS_comm_backend=pa_rccl."""
import torch

from paddle_amd.parallel import comm, rccl


def test_rccl_symbols_and_flag(monkeypatch):
    rccl._lib()  # the runtime library exports the communicator ABI
    assert not rccl.enabled()
    monkeypatch.setenv("FLAGS_comm_backend", "pa_rccl")
    assert rccl.enabled()
    # host tensors never reach RCCL
    assert comm._pa_comm(None, torch.zeros(4)) is None
