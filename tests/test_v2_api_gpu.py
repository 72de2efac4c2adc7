"""paddle.v2 facade on CUDAPlace: an MNIST-shaped conv net (img_conv / img_pool /
fc / classification_cost) trains through the Fluid executor on the device
kernels (convnd.hip conv + pool, fp32 MFMA GEMM)."""
import numpy as np
import pytest

import paddle.v2 as paddle

pytestmark = pytest.mark.gpu


def test_v2_conv_net_trains_on_gpu():
    paddle.init(use_gpu=True)
    img = paddle.layer.data(name="pixel", type=paddle.data_type.dense_vector(196))
    lbl = paddle.layer.data(name="label", type=paddle.data_type.integer_value(3))
    conv = paddle.networks.simple_img_conv_pool(input=img, filter_size=3, num_filters=8, num_channel=1,
                                                pool_size=2, pool_stride=2)
    pred = paddle.layer.fc(input=conv, size=3, act=paddle.activation.Softmax())
    cost = paddle.layer.classification_cost(input=pred, label=lbl)
    params = paddle.parameters.create(cost)
    trainer = paddle.trainer.SGD(cost=cost, parameters=params,
                                 update_equation=paddle.optimizer.Adam(learning_rate=0.01))
    rs = np.random.RandomState(0)
    protos = rs.randn(3, 196).astype("float32")

    def reader():
        for _ in range(10):
            ys = rs.randint(3, size=32)
            yield [((protos[y] + 0.5 * rs.randn(196)).astype("float32"), int(y)) for y in ys]

    costs = []
    trainer.train(reader=reader, num_passes=3,
                  event_handler=lambda e: costs.append(e.cost) if isinstance(e, paddle.event.EndIteration) else None)
    assert np.mean(costs[-5:]) < 0.5 * np.mean(costs[:5])
    res = trainer.test(reader=reader)
    assert res.metrics["classification_error_evaluator"] < 0.2
