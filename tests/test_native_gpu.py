"""Native C++ executor on the GPU: the gfx950 device kernels (csrc/native/ops_gpu.hip,
f32 MFMA GEMM) against fp32 references, the C++ predictor with ``use_gpu`` against
the host predictor on the same saved models, and the C++ trainer on device 0."""
import os
import subprocess

import numpy as np
import pytest
import torch

from paddle_amd import _build, native

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True), (True, True)])
@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (37, 129, 65), (128, 128, 32), (300, 257, 513), (1024, 512, 2048)])
def test_native_device_sgemm_vs_fp64(M, N, K, ta, tb):
    g = torch.Generator().manual_seed(M * 7 + N * 3 + K)
    a = torch.randn((K, M) if ta else (M, K), generator=g)
    b = torch.randn((N, K) if tb else (K, N), generator=g)
    c0 = torch.randn(M, N, generator=g)
    ref = 0.5 * ((a.T if ta else a).double() @ (b.T if tb else b).double()) + 0.25 * c0.double()
    da, db, dc = a.cuda(), b.cuda(), c0.clone().cuda()
    s = torch.cuda.current_stream().cuda_stream
    rc = native.lib().pa_nat_device_sgemm(s, int(ta), int(tb), M, N, K, 0.5, da.data_ptr(), a.shape[1],
                                           db.data_ptr(), b.shape[1], 0.25, dc.data_ptr(), N)
    assert rc == 0
    torch.cuda.synchronize()
    err = (dc.double().cpu() - ref).abs().max().item()
    bound = 4e-7 * K ** 0.5 * (ref.abs().max().item() + 1) + 1e-6
    assert err < max(bound, 5e-5 * (K ** 0.5)), (err, bound)


def _save_models(tmp):
    sys_path = os.path.join(HERE)
    import importlib.util

    spec = importlib.util.spec_from_file_location("tnc", os.path.join(sys_path, "test_native_cpu.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize("name", ["cnn", "ngram", "misc"])
def test_native_gpu_predictor_matches_host(tmp_path, name):
    m = _save_models(tmp_path)
    d, gen = m._save(tmp_path, name)
    inputs = gen(np.random.RandomState(5), 7)
    host = native.NativePredictor(d, ir_optim=True).run(inputs)
    dev_pred = native.NativePredictor(d, use_gpu=True, device=0, ir_optim=True)
    dev = dev_pred.run(inputs)
    for a, b in zip(dev, host):
        np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-5)
    # steady state: a second run reuses the HBM buffers and gives the same answer
    for a, b in zip(dev_pred.run(inputs), dev):
        np.testing.assert_array_equal(a, b)


def test_native_gpu_demo_trainer_matches_host(tmp_path):
    from paddle_amd.train_demo import save_demo_programs

    import paddle_amd.fluid as fluid
    from paddle_amd.train_demo import DemoTrainer

    model = tmp_path / "model"
    save_demo_programs(str(model))
    tr = DemoTrainer(str(model))
    tr.run_startup()
    params = tmp_path / "params"
    with fluid.executor.scope_guard(tr.scope):
        fluid.io.save_persistables(tr.exe, str(params), tr.main)
    exe = _build.build_native_program(os.path.join(_build.ROOT, "csrc", "train_demo", "demo_trainer.cc"),
                                      str(tmp_path / "demo_trainer"))

    def losses(dev):
        r = subprocess.run([exe, str(model), "8", str(params), str(dev)], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        return [float(line.split("loss:")[1]) for line in r.stdout.splitlines() if "loss:" in line]

    np.testing.assert_allclose(losses(0), losses(-1), rtol=1e-4)
