"""Static-graph programs on the HIP device (CUDAPlace) -- same book nets as the CPU tests."""
import numpy as np
import pytest

import paddle_amd.fluid as fluid
from test_book_cpu import _train_digits, conv_net, mlp

pytestmark = pytest.mark.gpu


def test_recognize_digits_conv_gpu(tmp_path):
    first, last, acc = _train_digits(conv_net, fluid.CUDAPlace(0), epochs=3, tmpdir=str(tmp_path / "c"))
    assert last < first and acc > 0.2


def test_recognize_digits_mlp_gpu():
    # (initial weights come from the device RNG, so CPU and GPU runs start from
    # different points; both must converge)
    first, last, acc = _train_digits(mlp, fluid.CUDAPlace(0), epochs=3)
    assert last < first and acc > 0.2
