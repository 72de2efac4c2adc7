"""Persistent LSTM kernel (csrc/kernels/rnn.hip) vs a plain fp32 PyTorch recurrence
with the same length-freezing semantics (ops/rnn.py::_lstm_ref)."""
import pytest
import torch

from paddle_amd.ops import rnn

pytestmark = pytest.mark.gpu
dev = torch.device("cuda")


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("T,B,I,H,with_state", [(7, 3, 24, 128, False), (40, 32, 64, 512, True),
                                                (33, 50, 32, 256, False), (5, 64, 16, 1024, True), (9, 100, 32, 512, True)])
def test_lstm_persistent_matches_reference(T, B, I, H, with_state):
    torch.manual_seed(0)
    x = torch.randn(T, B, I, device=dev)
    w_ih = (torch.randn(I, 4 * H, device=dev) / I ** 0.5).requires_grad_()
    w_hh = (torch.randn(H, 4 * H, device=dev) / H ** 0.5).requires_grad_()
    b = (0.1 * torch.randn(4 * H, device=dev)).requires_grad_()
    lens = torch.randint(1, T + 1, (B,))
    lens[0] = T
    h0 = (0.5 * torch.randn(B, H, device=dev)).requires_grad_() if with_state else None
    c0 = (0.5 * torch.randn(B, H, device=dev)).requires_grad_() if with_state else None
    xr = x.clone().requires_grad_()
    x.requires_grad_()
    hs, h, c, cs = rnn.lstm(x, w_ih, w_hh, b, h0, c0, lens=lens, return_cells=True)
    torch.cuda.synchronize()
    ref_leaves = [t.detach().clone().requires_grad_() if t is not None else None for t in (w_ih, w_hh, b, h0, c0)]
    hr, hlr, clr, csr = rnn._lstm_ref(xr, *ref_leaves, lens=lens, cells=True)
    assert _rel(hs, hr) < 2e-2, _rel(hs, hr)
    assert _rel(h, hlr) < 2e-2 and _rel(c, clr) < 2e-2 and _rel(cs, csr) < 2e-2
    gh = torch.randn_like(hs)
    gl = torch.randn_like(h)
    gc = torch.randn_like(cs)
    ((hs * gh).sum() + (cs * gc).sum()).backward(retain_graph=True)
    (h * gl).sum().backward()
    ((hr * gh).sum() + (csr * gc).sum() + (hlr * gl).sum()).backward()
    assert _rel(x.grad, xr.grad) < 3e-2, _rel(x.grad, xr.grad)
    for got, ref, name in zip((w_ih, w_hh, b, h0, c0), ref_leaves, ("w_ih", "w_hh", "b", "h0", "c0")):
        if got is not None:
            assert _rel(got.grad, ref.grad) < 3e-2, (name, _rel(got.grad, ref.grad))


def test_reverse_padded_roundtrip():
    x = torch.arange(5 * 3, device=dev, dtype=torch.float32).view(5, 3, 1)
    lens = torch.tensor([5, 2, 3])
    r = rnn.reverse_padded(x, lens)
    assert r[:2, 1, 0].tolist() == [4.0, 1.0] and r[2:, 1, 0].tolist() == x[2:, 1, 0].tolist()
    assert torch.equal(rnn.reverse_padded(r, lens), x)


@pytest.mark.parametrize("direction,layers", [("forward", 1), ("bidirect", 2)])
def test_nn_lstm_persistent_matches_miopen(monkeypatch, direction, layers):
    """paddle.nn.LSTM on the persistent kernel vs the same module on MIOpen."""
    import paddle_amd as paddle

    torch.manual_seed(0)
    B, T, I, H = 12, 30, 48, 256
    m = paddle.nn.LSTM(I, H, num_layers=layers, direction=direction).to(dev)
    x = torch.randn(B, T, I, device=dev)
    lens = torch.randint(3, T + 1, (B,))
    lens[0] = T
    outs = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("PADDLE_AMD_PERSISTENT_LSTM", flag)
        m.zero_grad()
        xi = x.clone().requires_grad_()
        out, (h, c) = m(xi, sequence_length=lens)
        (out.square().sum() + h.sum() + c.sum()).backward()
        outs[flag] = (out.detach(), h.detach(), c.detach(), xi.grad, [p.grad.clone() for p in m.parameters()])
    a, r = outs["1"], outs["0"]
    for got, ref in zip(a[:4], r[:4]):
        assert _rel(got, ref) < 3e-2, _rel(got, ref)
    for got, ref in zip(a[4], r[4]):
        assert _rel(got, ref) < 5e-2, _rel(got, ref)


@pytest.mark.parametrize("B,Ts,Tt", [(4, 9, 5), (32, 40, 12)])
def test_attention_lstm_decoder_matches_reference(B, Ts, Tt):
    """Fused attention-decoder kernels vs the plain fp32 recurrence (values + all grads)."""
    torch.manual_seed(0)
    E, A, H = 1024, 512, 512
    enc = (0.5 * torch.randn(B, Ts, E, device=dev)).requires_grad_()
    ep = (0.5 * torch.randn(B, Ts, A, device=dev)).requires_grad_()
    lens = torch.randint(1, Ts + 1, (B,), device=dev)
    Y = (0.5 * torch.randn(Tt, B, 4 * H, device=dev)).requires_grad_()
    h0 = (0.5 * torch.randn(B, H, device=dev)).requires_grad_()
    c0 = (0.5 * torch.randn(B, H, device=dev)).requires_grad_()
    Wsp = (torch.randn(H, A, device=dev) / H ** 0.5).requires_grad_()
    w = (torch.randn(A, device=dev) / A ** 0.5).requires_grad_()
    Wg = (torch.randn(E + H, 4 * H, device=dev) / (E + H) ** 0.5).requires_grad_()
    leaves = [enc, ep, Y, h0, c0, Wsp, w, Wg]
    out = rnn.attention_lstm_decoder(enc, ep, lens, Y, h0, c0, Wsp, w, Wg)
    ref_leaves = [t.detach().clone().requires_grad_() for t in leaves]
    r = ref_leaves
    ref = rnn._attn_decoder_ref(r[0], r[1], lens, r[2], r[3], r[4], r[5], r[6], r[7])
    assert _rel(out, ref) < 2e-2, _rel(out, ref)
    g = torch.randn_like(ref)
    (out.float() * g).sum().backward()
    (ref * g).sum().backward()
    names = ["enc", "ep", "Y", "h0", "c0", "Wsp", "w", "Wg"]
    for got, want, nm in zip(leaves, ref_leaves, names):
        assert _rel(got.grad, want.grad) < 4e-2, (nm, _rel(got.grad, want.grad))


def test_fluid_dynamic_lstm_persistent_matches_generic(monkeypatch):
    """fluid.layers.dynamic_lstm (no peepholes) on the persistent kernel vs the generic
    per-step path of the same op: hidden, cell and parameter gradients."""
    import numpy as np

    import paddle_amd.fluid as fluid
    from paddle_amd.framework import core

    D, LOD = 128, [0, 5, 7, 15]
    res = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("PADDLE_AMD_PERSISTENT_LSTM", flag)
        main, startup = fluid.Program(), fluid.Program()
        main.random_seed = startup.random_seed = 4
        with fluid.program_guard(main, startup):
            x = fluid.layers.data(name="x", shape=[4 * D], dtype="float32", lod_level=1)
            h, c = fluid.layers.dynamic_lstm(input=x, size=4 * D, use_peepholes=False,
                                             param_attr=fluid.ParamAttr(name="lw"),
                                             bias_attr=fluid.ParamAttr(name="lb"))
            loss = fluid.layers.mean(h * h) + fluid.layers.mean(c)
            fluid.backward.append_backward(loss)
        exe = fluid.Executor(fluid.CUDAPlace(0))
        xv = np.random.RandomState(0).randn(LOD[-1], 4 * D).astype("float32")
        scope = core.Scope()
        with fluid.executor.scope_guard(scope):
            exe.run(startup)
            # the device RNG is not reseeded per program: pin the parameters
            g = torch.Generator().manual_seed(1)
            for name, scale in (("lw", D ** -0.5), ("lb", 0.1)):
                t = scope.find_var(name).get()
                t.set_tensor((scale * torch.randn(t.tensor.shape, generator=g)).to(t.tensor.device))
            res[flag] = exe.run(main, feed={"x": core.LoDTensor(torch.from_numpy(xv), [LOD])},
                                fetch_list=[h, c, "lw@GRAD", "lb@GRAD"])
    errs = [_rel(torch.as_tensor(np.asarray(got)), torch.as_tensor(np.asarray(ref)))
            for got, ref in zip(res["1"], res["0"])]
    assert max(errs) < 3e-2, dict(zip(["hidden", "cell", "dW", "db"], errs))


def test_fusion_lstm_persistent_matches_generic(monkeypatch):
    """fusion_lstm (X @ WeightX for all steps, then the recurrence) on the persistent
    kernel vs the generic per-step path of the same op."""
    from paddle_amd.framework import core
    from paddle_amd.framework import registry as Rg

    D, M, LOD = 128, 64, [0, 6, 9, 17]
    g = torch.Generator().manual_seed(5)
    x = torch.randn(LOD[-1], M, generator=g).cuda()
    wx = (torch.randn(M, 4 * D, generator=g) * M ** -0.5).cuda()
    wh = (torch.randn(D, 4 * D, generator=g) * D ** -0.5).cuda()
    b = (torch.randn(1, 4 * D, generator=g) * 0.1).cuda()
    info = Rg.get_op_info("fusion_lstm")
    res = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("PADDLE_AMD_PERSISTENT_LSTM", flag)
        ctx = Rg.KernelContext("fusion_lstm", {"X": [core.LoDTensor(x, [LOD])], "WeightX": [core.LoDTensor(wx)],
                                               "WeightH": [core.LoDTensor(wh)], "Bias": [core.LoDTensor(b)]},
                               {"Hidden": ["h"], "Cell": ["c"], "XX": ["xx"]},
                               dict(info.attrs, use_peepholes=False), core.CUDAPlace(0))
        Rg.run_kernel(info, ctx)
        res[flag] = [ctx.results[s][0].tensor.float().cpu() for s in ("Hidden", "Cell")]
    for got, ref in zip(res["1"], res["0"]):
        assert _rel(got, ref) < 3e-2
