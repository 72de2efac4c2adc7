"""Legacy single-process multi-device strategies (distributed/legacy_parallel.py):
layer-placement model parallelism and ring data parallelism, on CPU "devices"
(one thread per device) against single-device references."""
import copy

import torch

from paddle_amd.distributed.legacy_parallel import MultiGradientMachine, ParallelNeuralNetwork, ring_allreduce_


def test_ring_allreduce_sums_every_replica():
    g = torch.Generator().manual_seed(0)
    for n in (2, 3, 5):
        ts = [torch.randn(17, 3, generator=g) for _ in range(n)]
        ref = sum(t.clone() for t in ts)
        ring_allreduce_(ts)
        for t in ts:
            torch.testing.assert_close(t, ref, rtol=1e-6, atol=1e-6)


def test_parallel_neural_network_matches_sequential():
    torch.manual_seed(1)
    layers = [torch.nn.Linear(8, 16), torch.nn.Tanh(), torch.nn.Linear(16, 4)]
    ref = torch.nn.Sequential(*copy.deepcopy(layers))
    pnn = ParallelNeuralNetwork(layers, ["cpu", "cpu", "cpu"])
    x = torch.randn(5, 8)
    y = pnn(x)
    torch.testing.assert_close(y, ref(x))
    assert [t[0] for t in pnn.trace] == [0, 1, 2]
    assert all(t[2].startswith("pnn-") for t in pnn.trace)  # ran on the device threads
    y.sum().backward()
    ref(x).sum().backward()
    for a, b in zip(pnn.parameters(), ref.parameters()):
        torch.testing.assert_close(a.grad, b.grad)
    pnn.close()


def test_multi_gradient_machine_equals_full_batch_sgd():
    torch.manual_seed(2)

    def model_fn():
        torch.manual_seed(3)
        return torch.nn.Sequential(torch.nn.Linear(6, 12), torch.nn.ReLU(), torch.nn.Linear(12, 1))

    def loss_fn(m, x, y):
        return ((m(x) - y) ** 2).mean()

    mgm = MultiGradientMachine(model_fn, loss_fn, lambda ps: torch.optim.SGD(ps, lr=0.1), ["cpu"] * 3)
    ref = model_fn()
    opt = torch.optim.SGD(ref.parameters(), lr=0.1)
    for step in range(4):
        x, y = torch.randn(12, 6), torch.randn(12, 1)
        mgm.step(x, y)
        opt.zero_grad()
        loss_fn(ref, x, y).backward()
        opt.step()
    for r in mgm.replicas:  # replicas identical and equal to full-batch training
        for a, b in zip(r.parameters(), ref.parameters()):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    mgm.close()
