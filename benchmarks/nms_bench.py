"""multiclass_nms at the SSD300 VOC shape (8 images, 21 classes, 8732 priors,
nms_top_k 400, keep_top_k 200): batched bitmask NMS kernel (detect.hip) vs the
per-class host loop of the same operator."""
import json
import time

import numpy as np
import torch

from paddle_amd.framework import core
from paddle_amd.framework import registry as R
from paddle_amd.operators import detection_ops  # noqa: F401
from paddle_amd.ops import oplib


def run_op(boxes, scores, attrs):
    ctx = R.KernelContext("multiclass_nms", {"BBoxes": [core.LoDTensor(boxes)], "Scores": [core.LoDTensor(scores)]},
                          {"Out": ["o"]}, dict(R.get_op_info("multiclass_nms").attrs, **attrs))
    R.run_kernel(R.get_op_info("multiclass_nms"), ctx)
    return ctx.results["Out"][0]


rng = np.random.RandomState(0)
N, C, M = 8, 21, 8732
xy = rng.uniform(0, 0.8, (N, M, 2))
wh = rng.uniform(0.02, 0.3, (N, M, 2))
boxes = torch.from_numpy(np.concatenate([xy, xy + wh], -1).astype("float32")).cuda()
scores = torch.softmax(torch.from_numpy(rng.randn(N, C, M).astype("float32") * 3), 1).cuda()
attrs = {"score_threshold": 0.01, "nms_top_k": 400, "nms_threshold": 0.45, "keep_top_k": 200}
res = {}
for name, enabled in (("native", True), ("host_loop", False)):
    oplib._ENABLED = enabled
    run_op(boxes, scores, attrs)
    torch.cuda.synchronize()
    it = 10 if enabled else 2
    t0 = time.perf_counter()
    for _ in range(it):
        out = run_op(boxes, scores, attrs)
    torch.cuda.synchronize()
    res[name + "_ms"] = round((time.perf_counter() - t0) / it * 1e3, 3)
    res[name + "_rows"] = int(out.tensor.shape[0] if hasattr(out, "tensor") else out.shape[0])
oplib._ENABLED = True
print(json.dumps({"shape": [N, C, M], **res}))
