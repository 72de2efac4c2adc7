"""Which part of the ResNet-50 bench step breaks HIP-graph capture?
usage: python tools/graph_debug.py STAGE  (stage: plain | stem | fwd | bwd | step)
env: CAPTURE_MODE (global | thread_local | relaxed), SET_DEVICE=1, NO_AMP=1"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import paddle_amd as paddle  # noqa: E402
from paddle_amd import nn  # noqa: E402

stage = sys.argv[1]
dev = torch.device("cuda")
if os.environ.get("SET_DEVICE") == "1":
    paddle.set_device("gpu")
paddle.seed(0)
model = paddle.vision.models.resnet50(num_classes=102, data_format="NHWC").to(dev)
opt = paddle.optimizer.Momentum(learning_rate=0.1, momentum=0.9, parameters=model.parameters(),
                                weight_decay=paddle.optimizer.L2Decay(1e-4))
if os.environ.get("NO_AMP") != "1":
    model, opt = paddle.amp.decorate(model, opt, level="O2", dtype="bfloat16")
loss_fn = nn.CrossEntropyLoss()
x = torch.randn(16, 224, 224, 3, device=dev, dtype=torch.bfloat16 if os.environ.get("NO_AMP") != "1" else torch.float32)
y = torch.randint(0, 102, (16, 1), device=dev)


def step(part):
    if part == "plain":  # a torch op alone: does capture work in this process at all?
        return x * 2
    if part == "stem":
        return model.conv1(x)
    out = model(x)
    if part == "fwd":
        return out
    loss = loss_fn(out.float(), y)
    loss.backward()
    if part == "bwd":
        return loss
    opt.step()
    opt.clear_grad(set_to_zero=False)
    return loss


for _ in range(2):
    step("step")
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
try:
    with torch.cuda.graph(g, capture_error_mode=os.environ.get("CAPTURE_MODE", "thread_local")):
        step(stage)
    print(stage, "CAPTURE OK", flush=True)
except Exception as e:  # noqa: BLE001
    print(stage, "CAPTURE FAILED:", repr(e)[:300], flush=True)
