"""prior_box / anchor_generator / polygon_box_transform / target_assign on the
device kernels (detect.hip) against the host operators: the same Fluid program run
on CPUPlace and CUDAPlace."""
import numpy as np
import pytest

import paddle_amd.fluid as fluid
from paddle_amd.framework import core

pytestmark = pytest.mark.gpu


def _both(build, feed):
    outs = []
    for place in (fluid.CPUPlace(), fluid.CUDAPlace(0)):
        main, startup = fluid.Program(), fluid.Program()
        with fluid.program_guard(main, startup):
            fetch = build()
        exe = fluid.Executor(place)
        with fluid.scope_guard(fluid.core.Scope()):
            exe.run(startup)
            outs.append([np.array(o) for o in exe.run(main, feed=feed(place), fetch_list=fetch)])
    return outs


def test_prior_box_and_anchor_generator():
    def build():
        feat = fluid.layers.data("feat", [8, 5, 6])
        img = fluid.layers.data("img", [3, 40, 48])
        b, v = fluid.layers.prior_box(feat, img, min_sizes=[8.0, 16.0], max_sizes=[16.0, 24.0],
                                      aspect_ratios=[2.0, 3.0], flip=True, clip=True)
        a, av = fluid.layers.anchor_generator(feat, anchor_sizes=[32.0, 64.0], aspect_ratios=[0.5, 1.0, 2.0],
                                              stride=[8.0, 8.0])
        return [b, v, a, av]

    rs = np.random.RandomState(0)
    f = rs.randn(2, 8, 5, 6).astype("float32")
    im = rs.randn(2, 3, 40, 48).astype("float32")
    cpu, gpu = _both(build, lambda p: {"feat": f, "img": im})
    for c, g in zip(cpu, gpu):
        np.testing.assert_allclose(g, c, rtol=1e-5, atol=1e-5)


def test_polygon_box_transform():
    def build():
        x = fluid.layers.data("x", [8, 4, 5])
        return [fluid.layers.polygon_box_transform(x)]

    x = np.random.RandomState(1).randn(2, 8, 4, 5).astype("float32")
    cpu, gpu = _both(build, lambda p: {"x": x})
    np.testing.assert_allclose(gpu[0], cpu[0], rtol=1e-6, atol=1e-6)


def test_target_assign_with_negatives():
    rs = np.random.RandomState(2)
    x = rs.randn(7, 4, 3).astype("float32")            # rows of 2 images (LoD [3, 4]), Pw = P = 4
    match = np.array([[0, -1, 2, 1], [-1, 3, 0, -1]], dtype="int64")
    neg = np.array([[1], [0], [3]], dtype="int64")      # image 0: prior 1; image 1: priors 0, 3

    def build():
        xv = fluid.layers.data("x", [4, 3], lod_level=1)
        mv = fluid.layers.data("m", [4], dtype="int64", append_batch_size=True)
        nv = fluid.layers.data("n", [1], dtype="int64", lod_level=1)
        out, w = fluid.layers.target_assign(xv, mv, negative_indices=nv, mismatch_value=-1.0)
        return [out, w]

    def feed(place):
        xt = core.LoDTensor()
        xt.set(x, place)
        xt.set_recursive_sequence_lengths([[3, 4]])
        nt = core.LoDTensor()
        nt.set(neg, place)
        nt.set_recursive_sequence_lengths([[1, 2]])
        return {"x": xt, "m": match, "n": nt}

    cpu, gpu = _both(build, feed)
    for c, g in zip(cpu, gpu):
        np.testing.assert_allclose(g, c, rtol=1e-6, atol=1e-6)
