"""seqdet.hip kernels against fp64 / exact references: CTC loss + gradient (vs
torch's ctc_loss autograd; warp-ctc contract for norm_by_times), roi_pool fwd/bwd
(vs the CPU operator that follows roi_pool_op.cu), edit_distance, ctc_align,
mean_iou histograms, fake quantisation, isfinite, sequence pad / unpad / scale, and
the Fluid operators routed to them."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import paddle_amd.fluid as fluid
from paddle_amd.ops import oplib

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _offs(lens):
    return np.concatenate([[0], np.cumsum(lens)]).astype(int).tolist()


def _ctc_ref(x, lab, xl, ll, blank):
    xo, lo = _offs(xl), _offs(ll)
    losses = []
    xr = torch.from_numpy(x).double().requires_grad_(True)
    for s in range(len(xl)):
        lp = torch.log_softmax(xr[xo[s]:xo[s + 1]], -1).unsqueeze(1)
        tg = torch.as_tensor(lab[lo[s]:lo[s + 1]]).long().unsqueeze(0)
        losses.append(F.ctc_loss(lp, tg, [xl[s]], [ll[s]], blank=blank, reduction="sum", zero_infinity=True))
    return torch.stack(losses), xr


@pytest.mark.parametrize("blank", [0, 5])
@pytest.mark.parametrize("norm", [False, True])
def test_ctc_loss_and_grad(blank, norm):
    rng = np.random.RandomState(blank + 3 * norm)
    C = 7
    xl = [12, 30, 5, 9, 1, 3]
    ll = [4, 10, 2, 0, 0, 4]  # the last one cannot align (T=3 < L=4): loss 0, grad 0
    labs = []
    for l in ll:
        cls = [c for c in range(C) if c != blank]
        seq = list(rng.choice(cls, l))
        if l >= 3:
            seq[2] = seq[1]  # a repeat forces a blank between
        labs += seq
    lab = np.array(labs, dtype=np.int64)
    x = rng.randn(sum(xl), C).astype("float32")
    ref, xr = _ctc_ref(x, lab, xl, ll, blank)
    w = torch.from_numpy(rng.rand(len(xl))).double()
    # warp-ctc gradient contract: d(loss_n)/dx scaled by w_n (/ T_n when norm_by_times)
    (ref * w).sum().backward()
    gref = xr.grad
    if norm:
        gref = gref / torch.repeat_interleave(torch.tensor(xl).double(), torch.tensor(xl))[:, None]
    xd = torch.from_numpy(x).to(DEV).requires_grad_(True)
    loss = oplib.ctc_loss_op(xd, torch.from_numpy(lab).to(DEV), _offs(xl), _offs(ll), blank, norm)
    torch.testing.assert_close(loss.reshape(-1).double().cpu(), ref.detach(), rtol=1e-4, atol=1e-4)
    (loss.reshape(-1) * w.float().to(DEV)).sum().backward()
    torch.testing.assert_close(xd.grad.double().cpu(), gref, rtol=1e-3, atol=1e-5)
    assert float(loss.detach()[-1]) == 0.0 and float(xd.grad[-3:].abs().max()) == 0.0


def test_warpctc_op_on_device():
    from op_test import OpTest

    rng = np.random.RandomState(0)
    xl, ll, C = [6, 4], [2, 2], 5
    x = rng.uniform(-1, 1, (10, C)).astype("float32")
    lab = np.array([1, 2, 3, 3], "int64").reshape(-1, 1)
    ref, _ = _ctc_ref(x, lab[:, 0], xl, ll, 0)
    t = OpTest()
    t.op_type, t.inputs, t.attrs = "warpctc", {"Logits": (x, [xl]), "Label": (lab, [ll])}, {"blank": 0}
    t.outputs = {"Loss": ref.detach().numpy().astype("float32").reshape(-1, 1)}
    t.check_output(atol=1e-4, rtol=1e-4, places=[fluid.CUDAPlace(0)])


def test_roi_pool_matches_cpu_op():
    from paddle_amd.framework import core
    from paddle_amd.operators import nn_ops  # noqa: F401

    rng = np.random.RandomState(1)
    x = rng.randn(2, 3, 12, 10).astype("float32")
    rois = np.array([[0, 0, 7, 7], [2.4, 1.5, 9.6, 11.2], [5, 5, 4, 4], [-3, -2, 3, 20], [1, 1, 1, 1]],
                    dtype="float32")
    lod = [[3, 2]]  # sequence lengths
    from op_test import OpTest

    res = []
    for place in (fluid.CPUPlace(), fluid.CUDAPlace(0)):
        t = OpTest()
        t.op_type = "roi_pool"
        t.inputs = {"X": x, "ROIs": (rois, lod)}
        t.outputs = {"Out": np.zeros((5, 3, 3, 4), "float32")}
        t.attrs = {"spatial_scale": 0.8, "pooled_height": 3, "pooled_width": 4}
        prog, _, feed, _, out_vars, _ = t._build()
        got = fluid.Executor(place).run(prog, feed=feed, fetch_list=[out_vars["Out"][0], out_vars["Argmax"][0]],
                                        scope=core.Scope())
        res.append([np.asarray(g) for g in got])
    (cpu_o, cpu_a), (gpu_o, gpu_a) = res
    np.testing.assert_allclose(gpu_o, cpu_o, rtol=0, atol=0)
    np.testing.assert_array_equal(gpu_a, cpu_a)
    # backward: scatter of dy into the argmax positions
    xd = torch.from_numpy(x).to(DEV).requires_grad_(True)
    out, am = oplib.roi_pool_op(xd, torch.from_numpy(rois).to(DEV), [0, 0, 0, 1, 1], 3, 4, 0.8)
    gy = torch.randn(out.shape)
    out.backward(gy.to(DEV))
    want = torch.zeros(2, 3, 12 * 10, dtype=torch.float64)
    amc = am.cpu()
    for r, b in enumerate([0, 0, 0, 1, 1]):
        for c in range(3):
            for i, a in enumerate(amc[r, c].reshape(-1).tolist()):
                if a >= 0:
                    want[b, c, a] += float(gy[r, c].reshape(-1)[i])
    torch.testing.assert_close(xd.grad.double().cpu().reshape(2, 3, -1), want, rtol=1e-5, atol=1e-5)
    assert (amc[2] >= 0).all()  # x2 < x1 still gives a 1-pixel ROI (max(w, 1))


def _lev(a, b):
    prev = list(range(len(b) + 1))
    for i, x in enumerate(a, 1):
        cur = [i] + [0] * len(b)
        for j, y in enumerate(b, 1):
            cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (x != y))
        prev = cur
    return prev[-1]


@pytest.mark.parametrize("normalized", [False, True])
def test_edit_distance(normalized):
    rng = np.random.RandomState(2)
    hl, rl = [5, 0, 17, 3, 9], [4, 6, 20, 0, 9]
    h = rng.randint(0, 4, sum(hl))
    r = rng.randint(0, 4, sum(rl))
    ho, ro = _offs(hl), _offs(rl)
    out = oplib.edit_distance_op(torch.from_numpy(h).to(DEV), torch.from_numpy(r).to(DEV), ho, ro, normalized)
    want = [_lev(list(h[ho[i]:ho[i + 1]]), list(r[ro[i]:ro[i + 1]])) / (max(rl[i], 1) if normalized else 1)
            for i in range(len(hl))]
    np.testing.assert_allclose(out.reshape(-1).cpu().numpy(), want, rtol=1e-6)


@pytest.mark.parametrize("merge", [True, False])
def test_ctc_align(merge):
    x = np.array([0, 1, 1, 0, 2, 2, 0, 3, 3, 3, 0, 0, 4, 0, 4], "int64")
    off = [0, 6, 10, 12, 15]
    out, new_off = oplib.ctc_align_op(torch.from_numpy(x).to(DEV), off, 0, merge)
    want, wo = [], [0]
    for i in range(4):
        prev = None
        for v in x[off[i]:off[i + 1]]:
            if v != 0 and not (merge and v == prev):
                want.append(int(v))
            prev = v
        wo.append(len(want))
    assert out.reshape(-1).cpu().tolist() == want and new_off == wo
    o2, no2 = oplib.ctc_align_op(torch.zeros(5, dtype=torch.int64, device=DEV), [0, 2, 5], 0, merge)
    assert o2.reshape(-1).tolist() == [-1] and no2 == [0, 1]


@pytest.mark.parametrize("dt", [torch.int32, torch.int64])
def test_mean_iou_hist(dt):
    g = torch.Generator().manual_seed(3)
    p = torch.randint(0, 6, (10000,), generator=g).to(dt)
    l = torch.randint(0, 6, (10000,), generator=g).to(dt)
    correct, wrong = oplib.mean_iou_hist(p.to(DEV), l.to(DEV), 6)
    pl, ll_ = p.long(), l.long()
    wc = torch.bincount(ll_[pl == ll_], minlength=6)
    ww = torch.bincount(pl[pl != ll_], minlength=6) + torch.bincount(ll_[pl != ll_], minlength=6)
    assert torch.equal(correct.long().cpu(), wc) and torch.equal(wrong.long().cpu(), ww)


def test_fake_quant():
    g = torch.Generator().manual_seed(4)
    x = torch.randn(1000, 37, generator=g) * 3
    out, s = oplib.fake_quant_op(x.to(DEV), 8)
    sm = x.abs().max()
    assert float(s) == float(sm)
    torch.testing.assert_close(out.cpu(), torch.round(x / sm * 127), rtol=0, atol=0)
    ins = torch.tensor([20.0])
    out, s = oplib.fake_quant_op(x.to(DEV), 4, ins.to(DEV), False, True)
    assert float(s) == 20.0
    torch.testing.assert_close(out.cpu(), torch.round(x.clamp(-20, 20) / 20 * 7), rtol=0, atol=0)
    ins = torch.tensor([2.0])
    out, s = oplib.fake_quant_op(x.to(DEV), 8, ins.to(DEV), True, True)  # is_test: in_scale, clipped
    torch.testing.assert_close(out.cpu(), torch.round(x.clamp(-2, 2) / 2 * 127), rtol=0, atol=0)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_isfinite(dt):
    x = torch.randn(100003, device=DEV).to(dt)
    assert bool(oplib.isfinite_op(x))
    for bad in (float("inf"), float("-inf"), float("nan")):
        y = x.clone()
        y[77777] = bad
        assert not bool(oplib.isfinite_op(y))
    flag = torch.zeros(1, dtype=torch.int32, device=DEV)
    assert oplib.isfinite_op(x, flag) and int(flag) == 0
    y = x.clone()
    y[5] = float("nan")
    oplib.isfinite_op(y, flag)
    assert int(flag) == 1


def test_amp_scaler_detects_overflow_on_device():
    from paddle_amd import amp

    p = torch.nn.Parameter(torch.ones(4, device=DEV))
    p.grad = torch.tensor([1.0, float("inf"), 0, 0], device=DEV)

    class _Opt:
        _parameter_list = [p]

        def step(self):
            raise AssertionError("step must be skipped on overflow")

    sc = amp.GradScaler(init_loss_scaling=8.0)
    sc.unscale_(_Opt())
    assert sc._found_inf


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_seq_pad_unpad_scale(dt):
    lens = [3, 1, 5, 0, 2]
    off = _offs(lens)
    x = torch.randn(sum(lens), 4, 3).to(dt)
    pv = torch.randn(12).to(dt)
    out = oplib.seq_pad_op(x.to(DEV), off, 6, pv)
    want = pv.reshape(1, 1, 4, 3).expand(5, 6, 4, 3).clone()
    for i in range(5):
        want[i, :lens[i]] = x[off[i]:off[i + 1]]
    assert torch.equal(out.cpu(), want)
    back = oplib.seq_unpad_op(out, off)
    assert torch.equal(back.cpu(), x)
    sc = torch.rand(5)
    got = oplib.seq_scale_op(x.to(DEV), off, sc)
    wt = torch.cat([x[off[i]:off[i + 1]].float() * sc[i] for i in range(5)]).to(dt)
    torch.testing.assert_close(got.cpu(), wt, rtol=1e-2, atol=1e-2)
