"""Inference library on the device: AnalysisPredictor (IR passes) in fp32 and bf16,
and HIP-graph replay, against the Fluid executor on the same saved model."""
import numpy as np
import pytest
import torch

from paddle_amd import inference

from test_inference_ir_cpu import _save_conv_model

pytestmark = pytest.mark.gpu


def test_predictor_gpu_fp32_bf16_and_hip_graph(tmp_path):
    d = str(tmp_path / "model")
    x, ref = _save_conv_model(d)          # reference output from the CPU executor
    cfg = inference.AnalysisConfig(model_dir=d, use_gpu=True)
    p = inference.create_paddle_predictor(cfg)
    (o,) = p.run([inference.PaddleTensor(x)])
    np.testing.assert_allclose(o.as_ndarray(), ref, rtol=1e-3, atol=1e-4)

    cfg = inference.AnalysisConfig(model_dir=d, use_gpu=True)
    cfg.enable_bf16()
    cfg.enable_hip_graph()
    p = inference.create_paddle_predictor(cfg)
    outs = [p.run([inference.PaddleTensor(x)])[0].as_ndarray() for _ in range(3)]
    for o in outs:
        np.testing.assert_allclose(o, ref, rtol=5e-2, atol=2e-2)
    assert any(isinstance(g, tuple) for g in p._graphs.values()), "HIP graph was not captured"
    # new input data through the captured graph
    x2 = (x * 0.5).astype(np.float32)
    (o2,) = p.run([inference.PaddleTensor(x2)])
    (e2,) = inference.create_paddle_predictor(inference.AnalysisConfig(model_dir=d, use_gpu=True)).run(
        [inference.PaddleTensor(x2)])
    np.testing.assert_allclose(o2.as_ndarray(), e2.as_ndarray(), rtol=5e-2, atol=2e-2)
    torch.cuda.synchronize()
