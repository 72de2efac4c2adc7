"""Native C++ executor + inference API (csrc/native, libpaddle_amd_native.so).

Reference: paddle/fluid/inference/api/api_impl_tester.cc (native predictor vs the
executor on saved book models, cloned predictors on threads),
paddle/fluid/train/demo (C++ trainer), framework/program_desc_test.cc.  Every
native result is compared with this package's Python executor on the same saved
program and weights.
"""
import os
import subprocess

import numpy as np
import pytest

import paddle_amd.fluid as fluid
from paddle_amd import _build, native

pytestmark = pytest.mark.skipif(os.system("which g++ >/dev/null 2>&1") != 0, reason="no host compiler")


def _cnn():
    img = fluid.layers.data(name="img", shape=[3, 12, 12], dtype="float32")
    c = fluid.layers.conv2d(img, num_filters=6, filter_size=3, padding=1, stride=2, act=None)
    b = fluid.layers.batch_norm(c, act="relu")
    g = fluid.layers.conv2d(b, num_filters=6, filter_size=3, groups=3, padding=1, act="relu")
    p = fluid.layers.pool2d(g, pool_size=2, pool_stride=2, pool_type="avg")
    d = fluid.layers.dropout(p, 0.3)
    f = fluid.layers.fc(d, size=10, act="softmax")
    return ["img"], [f], lambda rs, n: [rs.randn(n, 3, 12, 12).astype("float32")]


def _ngram():  # word2vec N-gram model (book/test_word2vec.py shape)
    words = [fluid.layers.data(name=f"w{i}", shape=[1], dtype="int64") for i in range(4)]
    embs = [fluid.layers.embedding(w, size=[50, 16], param_attr="shared_w") for w in words]
    h = fluid.layers.fc(fluid.layers.concat(embs, axis=1), size=32, act="sigmoid")
    out = fluid.layers.fc(h, size=50, act="softmax")
    return [f"w{i}" for i in range(4)], [out], lambda rs, n: [rs.randint(0, 50, (n, 1)).astype("int64")
                                                               for _ in range(4)]


def _misc():
    x = fluid.layers.data(name="x", shape=[4, 6], dtype="float32")
    y = fluid.layers.data(name="y", shape=[4, 6], dtype="float32", append_batch_size=False)
    a = fluid.layers.elementwise_mul(x, y, axis=1)
    m = fluid.layers.matmul(a, a, transpose_y=True, alpha=0.5)  # [N, 4, 4]
    t = fluid.layers.transpose(m, [0, 2, 1])
    r = fluid.layers.reshape(t, [-1, 16])
    s = fluid.layers.scale(fluid.layers.tanh(r), scale=2.0, bias=0.5)
    red = fluid.layers.reduce_sum(s, dim=1, keep_dim=True)
    parts = fluid.layers.split(s, num_or_sections=2, dim=1)
    cat = fluid.layers.concat([parts[1], parts[0], red], axis=1)
    mx = fluid.layers.reduce_max(cat, dim=[1])
    return ["x", "y"], [cat, mx], lambda rs, n: [rs.randn(n, 4, 6).astype("float32"),
                                                 rs.randn(4, 6).astype("float32")]


MODELS = {"cnn": _cnn, "ngram": _ngram, "misc": _misc}


def _save(tmp, name, combined=False):
    main, startup = fluid.Program(), fluid.Program()
    with fluid.program_guard(main, startup):
        feeds, fetches, gen = MODELS[name]()
    exe = fluid.Executor(fluid.CPUPlace())
    scope = fluid.core.Scope()
    d = os.path.join(str(tmp), name + ("_c" if combined else ""))
    with fluid.executor.scope_guard(scope):
        exe.run(startup)
        fluid.io.save_inference_model(d, feeds, fetches, exe, main, params_filename="params" if combined else None)
    return d, gen


def _python_ref(d, inputs, combined=False):
    exe = fluid.Executor(fluid.CPUPlace())
    scope = fluid.core.Scope()
    with fluid.executor.scope_guard(scope):
        prog, feeds, fetches = fluid.io.load_inference_model(d, exe, params_filename="params" if combined else None)
        return exe.run(prog, feed=dict(zip(feeds, inputs)), fetch_list=fetches)


@pytest.mark.parametrize("name", sorted(MODELS))
@pytest.mark.parametrize("ir_optim", [False, True])
def test_native_predictor_matches_python_executor(tmp_path, name, ir_optim):
    d, gen = _save(tmp_path, name)
    inputs = gen(np.random.RandomState(1), 5)
    ref = _python_ref(d, inputs)
    pred = native.NativePredictor(d, ir_optim=ir_optim)
    outs = pred.run(inputs)
    assert len(outs) == len(ref)
    for o, r in zip(outs, ref):
        np.testing.assert_allclose(o, np.asarray(r), rtol=2e-5, atol=2e-6)
    # a clone shares the parameters and gives the same answer on another batch size
    inputs2 = gen(np.random.RandomState(2), 3)
    for o, r in zip(pred.clone().run(inputs2), _python_ref(d, inputs2)):
        np.testing.assert_allclose(o, np.asarray(r), rtol=2e-5, atol=2e-6)


def test_native_predictor_combined_params_file(tmp_path):
    d, gen = _save(tmp_path, "cnn", combined=True)
    inputs = gen(np.random.RandomState(3), 2)
    ref = _python_ref(d, inputs, combined=True)
    out = native.NativePredictor(d, param_file=os.path.join(d, "params")).run(inputs)
    np.testing.assert_allclose(out[0], np.asarray(ref[0]), rtol=2e-5, atol=2e-6)


def test_cpp_infer_demo_with_threaded_clones(tmp_path):
    d, gen = _save(tmp_path, "ngram")
    inputs = gen(np.random.RandomState(4), 6)
    ref = _python_ref(d, inputs)
    exe = _build.build_native_program(os.path.join(_build.NATIVE_INC, "demo", "infer_demo.cc"),
                                      str(tmp_path / "infer_demo"))
    args = [exe, d, str(tmp_path / "out.bin"), "4", "0", "1"]
    for i, a in enumerate(inputs):
        p = tmp_path / f"in{i}.bin"
        a.tofile(p)
        args += [str(p), "l", ",".join(map(str, a.shape))]
    r = subprocess.run(args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "clones_agree 4/4" in r.stdout
    out = np.fromfile(tmp_path / "out.bin", dtype=np.float32).reshape(np.asarray(ref[0]).shape)
    np.testing.assert_allclose(out, np.asarray(ref[0]), rtol=2e-5, atol=2e-6)


def test_native_executor_trains_like_python_executor(tmp_path):
    """An MLP classifier's training program (fc/relu/softmax/cross_entropy/mean +
    backward + SGD) run by the native executor from the same initial weights
    follows the Python executor's loss trajectory."""
    main, startup = fluid.Program(), fluid.Program()
    with fluid.program_guard(main, startup):
        x = fluid.layers.data(name="x", shape=[20], dtype="float32")
        lab = fluid.layers.data(name="lab", shape=[1], dtype="int64")
        h = fluid.layers.fc(x, size=32, act="relu")
        h2 = fluid.layers.fc(h, size=16, act="tanh")
        pr = fluid.layers.fc(h2, size=5, act="softmax")
        loss = fluid.layers.mean(fluid.layers.cross_entropy(pr, lab))
        fluid.optimizer.SGD(learning_rate=0.2).minimize(loss)
    rs = np.random.RandomState(0)
    xs = rs.randn(16, 20).astype("float32")
    ls = rs.randint(0, 5, (16, 1)).astype("int64")
    exe = fluid.Executor(fluid.CPUPlace())
    scope = fluid.core.Scope()
    with fluid.executor.scope_guard(scope):
        exe.run(startup)
        init = {v.name: np.array(scope.find_var(v.name).get_tensor().numpy(), copy=True)
                for v in main.list_vars() if v.persistable and scope.find_var(v.name) is not None
                and v.name not in ("feed", "fetch")}
        ref = [float(np.asarray(exe.run(main, feed={"x": xs, "lab": ls}, fetch_list=[loss])[0]).reshape(-1)[0])
               for _ in range(6)]
    prog = native.NativeProgram(data=main.desc.serialize_to_string())
    ns = native.NativeScope()
    for k, v in init.items():
        ns.set(k, v)
    ns.set("x", xs)
    ns.set("lab", ls)
    ne = native.NativeExecutor()
    got = []
    for _ in range(6):
        ne.run(prog, ns)
        got.append(float(ns.get(loss.name).reshape(-1)[0]))
    np.testing.assert_allclose(got, ref, rtol=1e-4)
    assert got[-1] < got[0]


def test_python_bias_grad_on_square_activation():
    """Regression found by the native trajectory test: the Python executor's
    elementwise_add_grad summed a [16] bias gradient over the wrong dim of a
    [16, 16] activation (raw-shape matching instead of the op's axis)."""
    import torch

    main, startup = fluid.Program(), fluid.Program()
    with fluid.program_guard(main, startup):
        x = fluid.layers.data(name="x", shape=[16], dtype="float32")
        h = fluid.layers.fc(x, size=16, act="tanh")
        loss = fluid.layers.mean(fluid.layers.square(h))
        fluid.backward.append_backward(loss)
    xs = np.random.RandomState(0).randn(16, 16).astype("float32")
    exe = fluid.Executor(fluid.CPUPlace())
    scope = fluid.core.Scope()
    wn, bn = sorted(p.name for p in main.global_block().all_parameters())[::-1]  # fc_k.w_0, fc_k.b_0
    with fluid.executor.scope_guard(scope):
        exe.run(startup)
        w = np.asarray(scope.find_var(wn).get_tensor().numpy())
        b = np.asarray(scope.find_var(bn).get_tensor().numpy())
        (gb,) = exe.run(main, feed={"x": xs}, fetch_list=[bn + "@GRAD"])
    bt = torch.tensor(b, requires_grad=True)
    torch.tanh(torch.tensor(xs) @ torch.tensor(w) + bt).square().mean().backward()
    np.testing.assert_allclose(np.asarray(gb), bt.grad.numpy(), rtol=1e-5, atol=1e-7)


def test_cpp_demo_trainer_matches_python(tmp_path):
    from paddle_amd.train_demo import DemoTrainer, save_demo_programs

    model = tmp_path / "model"
    save_demo_programs(str(model))
    # Python executor: startup, then dump the initial parameters for the C++ run
    tr = DemoTrainer(str(model))
    tr.run_startup()
    params = tmp_path / "params"
    with fluid.executor.scope_guard(tr.scope):
        fluid.io.save_persistables(tr.exe, str(params), tr.main)
    x = np.arange(26, dtype=np.float32).reshape(2, 13)
    y = np.arange(2, dtype=np.float32).reshape(2, 1)
    tr.set_input("x", x.tobytes(), (2, 13))
    tr.set_input("y", y.tobytes(), (2, 1))
    ref = [tr.step() for _ in range(10)]
    exe = _build.build_native_program(os.path.join(_build.ROOT, "csrc", "train_demo", "demo_trainer.cc"),
                                      str(tmp_path / "demo_trainer"))
    r = subprocess.run([exe, str(model), "10", str(params)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = [float(line.split("loss:")[1]) for line in r.stdout.splitlines() if "loss:" in line]
    np.testing.assert_allclose(got, ref, rtol=1e-5)
    assert "run_time_ms" in r.stdout and "mul_grad" in r.stdout  # per-op profile table


def test_program_decoder_rejects_malformed_input(tmp_path):
    d, _ = _save(tmp_path, "misc")
    data = open(os.path.join(d, "__model__"), "rb").read()
    p = native.NativeProgram(data=data)
    assert p.num_ops(0) > 5
    with pytest.raises(RuntimeError):
        native.NativeProgram(data=b"\x0a\xff\xff\xff\x0f" + b"\x00" * 8)
    rs = np.random.RandomState(0)
    for cut in rs.randint(1, len(data) - 1, 40):  # truncations: clean error or a parse, never a crash
        try:
            native.NativeProgram(data=data[:cut])
        except RuntimeError:
            pass


def test_registered_native_ops_cover_inference_set():
    host = set(native.registered_ops())
    need = {"feed", "fetch", "mul", "fc", "matmul", "conv2d", "pool2d", "batch_norm", "softmax", "elementwise_add",
            "relu", "sigmoid", "tanh", "lookup_table", "concat", "split", "reshape2", "transpose2", "dropout",
            "scale", "mul_grad", "sgd", "adam", "momentum", "softmax_with_cross_entropy"}
    assert need <= host, need - host
    dev = set(native.registered_ops(device=True))
    assert {"mul", "fc", "matmul", "conv2d", "pool2d", "batch_norm", "softmax", "elementwise_add"} <= dev


def _tensor_stream(dims, payload=b"", dtype=5):
    import struct

    d = bytes([0x08, dtype])
    for x in dims:
        v, b = x, bytearray()
        while v >= 0x80:
            b.append((v & 0x7F) | 0x80)
            v >>= 7
        b.append(v)
        d += bytes([0x10]) + bytes(b)
    return struct.pack("<IQ", 0, 0) + struct.pack("<Ii", 0, len(d)) + d + payload


@pytest.mark.parametrize("dims,payload", [
    ([2 ** 33, 2 ** 31], b""),          # numel wraps to 0 in int64 without the overflow check
    ([2 ** 39, 2 ** 39], b"\0" * 64),   # element count overflows u64
    ([1024, 1024], b"\0" * 64),         # declared 4 MiB, file holds 64 B
])
def test_native_loader_rejects_overflowing_dims(tmp_path, dims, payload):
    """NativePaddlePredictor's params reader (csrc/native/core.cc
    read_lod_tensor) must reject element counts that overflow and sizes beyond the
    file, before allocating."""
    main, startup = fluid.Program(), fluid.Program()
    with fluid.program_guard(main, startup):
        x = fluid.layers.data(name="x", shape=[4], dtype="float32")
        fluid.layers.fc(x, size=3)
    prog = native.NativeProgram(data=main.desc.serialize_to_string())
    persist = sorted(v.name for v in main.list_vars() if v.persistable and v.name not in ("feed", "fetch"))
    assert persist
    with open(tmp_path / "params", "wb") as f:
        for _ in persist:
            f.write(_tensor_stream(dims, payload))
    ns = native.NativeScope()
    with pytest.raises(RuntimeError):
        ns.load_persistables(prog, str(tmp_path), combined=str(tmp_path / "params"))


def test_c_api_gradient_machine_matches_python(tmp_path):
    """The legacy C-API function set (csrc/native/paddle_capi.h, capi.cc) from a plain
    C program: a merged model (utils/merge_model.py), a program + parameter directory
    and a shared-parameter clone give the Python executor's output."""
    import shutil

    from paddle_amd.utils.merge_model import merge_model

    main, startup = fluid.Program(), fluid.Program()
    with fluid.program_guard(main, startup):
        x = fluid.layers.data(name="x", shape=[12], dtype="float32")
        h = fluid.layers.fc(x, size=16, act="relu")
        out = fluid.layers.fc(h, size=5, act="softmax")
    exe = fluid.Executor(fluid.CPUPlace())
    d = str(tmp_path / "mlp")
    with fluid.executor.scope_guard(fluid.core.Scope()):
        exe.run(startup)
        fluid.io.save_inference_model(d, ["x"], [out], exe, main)
    merged = merge_model(d, str(tmp_path / "mlp.merged"))
    xs = np.random.RandomState(6).randn(7, 12).astype("float32")
    xs.tofile(tmp_path / "in.bin")
    ref = _python_ref(d, [xs])[0]
    cc = shutil.which("gcc") or "cc"
    exe_path = str(tmp_path / "capi_demo")
    lib = _build.build_native()
    r = subprocess.run([cc, "-O2", os.path.join(_build.NATIVE_INC, "demo", "capi_demo.c"), f"-L{_build.LIBDIR}",
                        "-lpaddle_amd_native", f"-Wl,-rpath,{_build.LIBDIR}", "-o", exe_path],
                       capture_output=True, text=True)
    assert r.returncode == 0 and os.path.exists(lib), r.stderr[-3000:]
    r = subprocess.run([exe_path, merged, os.path.join(d, "__model__"), d, str(tmp_path / "in.bin"), "7", "12",
                        str(tmp_path / "out.bin")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "machines_agree 7 x 5" in r.stdout
    got = np.fromfile(tmp_path / "out.bin", dtype=np.float32).reshape(7, 5)
    np.testing.assert_allclose(got, np.asarray(ref), rtol=2e-5, atol=2e-6)
