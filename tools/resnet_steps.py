"""A few training steps of a ResNet for kernel traces (rocprofv3 --kernel-trace):
``python tools/resnet_steps.py eager18|fluid50 STEPS`` -- DyGraph ResNet-18 bf16 NHWC
(eager engine, Momentum) or Fluid ResNet-50 NCHW fp32 (static program, Momentum),
small batches.  Prints one JSON line with the per-step losses."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

which, steps = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 3
losses = []
if which == "eager18":
    import paddle  # noqa: E402
    import paddle.nn.functional as F  # noqa: E402

    paddle.seed(0)
    paddle.set_device("gpu")
    model = paddle.vision.models.resnet18(num_classes=10, data_format="NHWC")
    model.to(device="cuda", dtype=torch.bfloat16)
    opt = paddle.optimizer.Momentum(learning_rate=0.01, momentum=0.9, parameters=model.parameters())
    x = paddle.randn([8, 32, 32, 3]).astype("bfloat16")
    y = paddle.to_tensor(np.arange(8) % 10)
    for _ in range(steps):
        loss = F.cross_entropy(model(x).astype("float32"), y)
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(float(loss))
else:
    import paddle_amd.fluid as fluid  # noqa: E402
    from benchmarks.fluid_resnet50 import resnet50  # noqa: E402

    main, startup = fluid.Program(), fluid.Program()
    with fluid.program_guard(main, startup):
        img = fluid.layers.data("img", [3, 64, 64])
        label = fluid.layers.data("label", [1], dtype="int64")
        loss = fluid.layers.mean(fluid.layers.cross_entropy(resnet50(img, 10), label))
        fluid.optimizer.Momentum(learning_rate=0.01, momentum=0.9).minimize(loss)
    place = fluid.CUDAPlace(0)
    exe = fluid.Executor(place)
    scope = fluid.core.Scope()
    rs = np.random.RandomState(0)
    feed = {"img": rs.rand(4, 3, 64, 64).astype("float32"), "label": (np.arange(4) % 10).reshape(4, 1)}
    with fluid.executor.scope_guard(scope):
        exe.run(startup)
        for _ in range(steps):
            (lv,) = exe.run(main, feed=feed, fetch_list=[loss])
            losses.append(float(np.asarray(lv).reshape(-1)[0]))
torch.cuda.synchronize()
print(json.dumps({"model": which, "losses": losses}))
