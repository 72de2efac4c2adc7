"""Kernels of one DyGraph ResNet-18 NHWC bf16 training step on the eager engine,
recorded in-process by the rocprofiler-sdk tracer (FLAGS_device_tracer=1)."""
import json
import os
import sys

os.environ["FLAGS_device_tracer"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import paddle  # noqa: E402
import paddle.nn.functional as F  # noqa: E402
from paddle_amd.utils import device_tracer as dt  # noqa: E402
from paddle_amd.utils import profiler as P  # noqa: E402
from paddle_amd.utils import strict  # noqa: E402

assert dt.available(), dt.error()
paddle.seed(0)
paddle.set_device("gpu")
model = paddle.vision.models.resnet18(num_classes=10, data_format="NHWC")
model.to(device="cuda", dtype=torch.bfloat16)
opt = paddle.optimizer.Momentum(learning_rate=0.05, momentum=0.9, parameters=model.parameters())
x = paddle.randn([8, 32, 32, 3]).astype("bfloat16")
y = paddle.to_tensor(np.arange(8) % 10)


def step():
    # an outer region labels whatever ATen work the framework's own regions miss
    with strict.region("probe:step"):
        return _step()


def _step():
    loss = F.cross_entropy(model(x).astype("float32"), y)
    loss.backward()
    opt.step()
    opt.clear_grad()
    return loss


step()
torch.cuda.synchronize()
P.start("All")
with P.RecordEvent("train_step"):
    step()
P.stop(profile_path=None)
recs = P.kernel_records()
aten, ours = {}, {}
t_aten = t_all = 0
for r in recs:
    t_all += r["dur_ns"]
    k = r["name"][:140]
    if "at::native" in r["name"]:
        aten[k] = aten.get(k, 0) + 1
        t_aten += r["dur_ns"]
    else:
        ours[k] = ours.get(k, 0) + 1
print(json.dumps({"kernels": len(recs), "aten_kernels": sum(aten.values()), "aten_time_frac": t_aten / max(t_all, 1),
                  "aten": aten, "other": ours, "strict_report": strict.report()}, indent=1))
