"""Layer-placement model parallelism and ring multi-device DP with device
placements on the GPU box (one MI355X: replicas share cuda:0, placements mix
cuda:0 and the host)."""
import copy

import pytest
import torch

from paddle_amd.distributed.legacy_parallel import MultiGradientMachine, ParallelNeuralNetwork

pytestmark = pytest.mark.gpu


def test_layer_placement_across_gpu_and_host():
    torch.manual_seed(0)
    layers = [torch.nn.Linear(16, 32), torch.nn.GELU(), torch.nn.Linear(32, 8)]
    ref = torch.nn.Sequential(*copy.deepcopy(layers)).double()
    pnn = ParallelNeuralNetwork(layers, ["cuda:0", "cpu", "cuda:0"])
    x = torch.randn(4, 16)
    y = pnn(x)
    assert y.device.type == "cuda"
    torch.testing.assert_close(y.double().cpu(), ref(x.double()), rtol=1e-4, atol=1e-5)
    y.sum().backward()
    ref(x.double()).sum().backward()
    for a, b in zip(pnn.parameters(), ref.parameters()):
        torch.testing.assert_close(a.grad.double().cpu(), b.grad, rtol=1e-4, atol=1e-5)
    pnn.close()


def test_multi_gradient_machine_on_device():
    def model_fn():
        torch.manual_seed(1)
        return torch.nn.Sequential(torch.nn.Linear(6, 12), torch.nn.ReLU(), torch.nn.Linear(12, 1))

    def loss_fn(m, x, y):
        return ((m(x) - y) ** 2).mean()

    mgm = MultiGradientMachine(model_fn, loss_fn, lambda ps: torch.optim.SGD(ps, lr=0.1), ["cuda:0", "cuda:0"])
    ref = model_fn().double()
    opt = torch.optim.SGD(ref.parameters(), lr=0.1)
    g = torch.Generator().manual_seed(2)
    for _ in range(3):
        x, y = torch.randn(8, 6, generator=g), torch.randn(8, 1, generator=g)
        mgm.step(x, y)
        opt.zero_grad()
        loss_fn(ref, x.double(), y.double()).backward()
        opt.step()
    for a, b in zip(mgm.replicas[1].parameters(), ref.parameters()):
        torch.testing.assert_close(a.double().cpu(), b, rtol=1e-4, atol=1e-5)
    mgm.close()
