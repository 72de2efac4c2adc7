"""Depthwise NHWC bf16 conv: native dwconv.hip vs torch (MIOpen) grouped conv,
MobileNet-v1/v2 shapes, fwd and fwd+bwd ms."""
import json

import torch
import torch.nn.functional as F

from paddle_amd.ops import conv as C


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it


for (N, H, Cc, s) in [(64, 112, 32, 1), (64, 112, 64, 2), (64, 56, 128, 1), (64, 28, 256, 1), (64, 14, 512, 1),
                      (64, 7, 1024, 1), (64, 56, 144, 1)]:
    x = torch.randn(N, H, H, Cc, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = torch.randn(Cc, 1, 3, 3, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    xc = x.detach().permute(0, 3, 1, 2).requires_grad_(True)  # channels_last view for MIOpen
    res = {"shape": [N, H, H, Cc], "stride": s}
    res["native_fwd_ms"] = timeit(lambda: C.dwconv2d_nhwc(x, w, None, s, 1, 1))
    res["torch_fwd_ms"] = timeit(lambda: F.conv2d(xc, w, None, s, 1, 1, Cc))
    g = torch.randn_like(C.dwconv2d_nhwc(x, w, None, s, 1, 1))
    gc = g.permute(0, 3, 1, 2)
    res["native_fb_ms"] = timeit(lambda: torch.autograd.grad(C.dwconv2d_nhwc(x, w, None, s, 1, 1), (x, w), g))
    res["torch_fb_ms"] = timeit(lambda: torch.autograd.grad(F.conv2d(xc, w, None, s, 1, 1, Cc), (xc, w), gc))
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)
