"""Shared programs for the native-engine trajectory tests (CPU and GPU): the same
Fluid training program run by ``fluid.Executor(place)`` (Python op interpreter)
and by ``fluid.Executor(place, engine="native")`` (C++ executor) from identical
initial parameters must follow the same loss trajectory."""
import numpy as np

import paddle_amd.fluid as fluid


def lenet(img, label):
    c = fluid.nets.simple_img_conv_pool(img, 8, 5, 2, 2, act="relu")
    c = fluid.nets.simple_img_conv_pool(c, 16, 3, 2, 2, act="relu")
    pred = fluid.layers.fc(c, 10, act="softmax")
    return fluid.layers.mean(fluid.layers.cross_entropy(pred, label))


def _conv_bn(x, ch, k, stride=1, act="relu"):
    c = fluid.layers.conv2d(x, ch, k, stride=stride, padding=(k - 1) // 2, bias_attr=False)
    return fluid.layers.batch_norm(c, act=act)


def resnet_tiny(img, label):
    x = _conv_bn(img, 8, 3)
    for ch, stride in ((8, 1), (16, 2)):
        short = _conv_bn(x, ch, 1, stride, act=None) if stride != 1 or x.shape[1] != ch else x
        y = _conv_bn(x, ch, 3, stride)
        y = _conv_bn(y, ch, 3, act=None)
        x = fluid.layers.relu(fluid.layers.elementwise_add(short, y))
    x = fluid.layers.pool2d(x, 2, "avg", global_pooling=True)
    pred = fluid.layers.fc(x, 10, act="softmax")
    return fluid.layers.mean(fluid.layers.cross_entropy(pred, label))


MODELS = {"lenet": (lenet, lambda: fluid.optimizer.Adam(learning_rate=0.002)),
          "resnet_tiny": (resnet_tiny, lambda: fluid.optimizer.Momentum(learning_rate=0.05, momentum=0.9))}


def build(model):
    net, opt = MODELS[model]
    main, startup = fluid.Program(), fluid.Program()
    main.random_seed = startup.random_seed = 7  # a fixed problem: same initial weights every run
    with fluid.unique_name.guard(), fluid.program_guard(main, startup):
        img = fluid.layers.data("img", [1, 16, 16])
        lbl = fluid.layers.data("label", [1], dtype="int64")
        loss = net(img, lbl)
        opt().minimize(loss)
    return main, startup, loss


def batches(steps, n=16, seed=0):
    """One fixed batch repeated: the loss of a memorised batch falls monotonically
    enough to assert on (fresh random batches with random labels need not)."""
    rs = np.random.RandomState(seed)
    b = (rs.randn(n, 1, 16, 16).astype("float32"), rs.randint(0, 10, (n, 1)).astype("int64"))
    return [b] * steps


def train(model, place, engine, steps=5, init=None):
    """Returns (losses, {param: final value}, init values, executor)."""
    main, startup, loss = build(model)
    scope = fluid.core.Scope()
    with fluid.executor.scope_guard(scope):
        fluid.Executor(place).run(startup)
        pers = [v.name for v in main.list_vars() if v.persistable and v.name not in ("feed", "fetch")
                and scope.find_var(v.name) is not None]
        if init is None:
            init = {n: np.array(scope.find_var(n).get_tensor().numpy()) for n in pers}
        else:
            for n in pers:
                scope.find_var(n).get_tensor().set(init[n], place)
        exe = fluid.Executor(place, engine=engine)
        losses = []
        for x, y in batches(steps):
            (lv,) = exe.run(main, feed={"img": x, "label": y}, fetch_list=[loss])
            losses.append(float(np.asarray(lv).reshape(-1)[0]))
        final = {p.name: np.array(scope.find_var(p.name).get_tensor().numpy())
                 for p in main.global_block().all_parameters()}
    return losses, final, init, exe
