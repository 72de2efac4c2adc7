#!/usr/bin/env python3
"""ResNet-50 (bs 256, NHWC bf16) convolution shapes: the 256x256-tile implicit GEMM
(gemm.hip pa_conv_gemm) vs the 64-channel-tile kernel (convsn.hip pa_conv_sn), for
the forward (with and without the BN-statistics epilogue) and the data gradient.
One JSON line per shape; times in microseconds (median of 20 after 5 warm-up)."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from paddle_amd.ops import _native as _nat  # noqa: E402
from paddle_amd.ops import conv as _conv  # noqa: E402

B = int(os.environ.get("BATCH", "256"))
# (H_in, C_in, C_out, k, stride) of the distinct ResNet-50 convolutions with C_in % 64 == 0
SHAPES = [
    (56, 64, 64, 1, 1), (56, 64, 64, 3, 1), (56, 64, 256, 1, 1), (56, 256, 64, 1, 1),
    (56, 256, 128, 1, 1), (56, 128, 128, 3, 2), (28, 128, 128, 3, 1), (28, 128, 512, 1, 1), (28, 512, 128, 1, 1),
    (28, 512, 256, 1, 1), (28, 256, 256, 3, 2), (14, 256, 256, 3, 1), (14, 256, 1024, 1, 1),
    (14, 1024, 256, 1, 1),
]


def timeit(fn, it=20, warm=5):
    for _ in range(warm):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(it)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
    return ts[len(ts) // 2]


def main():
    L = _nat.lib()
    st = _nat.stream()
    for H, C, Co, k, s in SHAPES:
        p = k // 2
        OH = (H + 2 * p - k) // s + 1
        x = torch.randn(B, H, H, C, device="cuda").to(torch.bfloat16)
        wk = (torch.randn(Co, k * k * C, device="cuda") * 0.05).to(torch.bfloat16)
        y = torch.empty(B, OH, OH, Co, device="cuda", dtype=torch.bfloat16)
        geo = (B, H, H, C, OH, OH, Co, k, k, s, s, p, p, 1, 1, 0, 0)
        G = int(L.pa_conv_sn_tiles(B * OH * OH))
        part = torch.empty(G * 2 * Co, device="cuda")
        shift = torch.zeros(Co, device="cuda")
        rec = {"H": H, "C": C, "Cout": Co, "k": k, "s": s,
               "gflop": round(2.0 * B * OH * OH * Co * k * k * C / 1e9, 1)}
        rec["fwd_wide_us"] = timeit(lambda: L.pa_conv_gemm(_nat.ptr(x), _nat.ptr(wk), _nat.ptr(y), None, *geo, st))
        rec["fwd_sn_us"] = timeit(lambda: L.pa_conv_sn(_nat.ptr(x), _nat.ptr(wk), _nat.ptr(y), None, *geo, None,
                                                       None, st))
        rec["fwd_sn_stats_us"] = timeit(lambda: L.pa_conv_sn(_nat.ptr(x), _nat.ptr(wk), _nat.ptr(y), None, *geo,
                                                             _nat.ptr(part), _nat.ptr(shift), st))
        # data gradient: dY [B, OH, OH, Co] -> dX [B, H, H, C] (zero insertion = stride)
        if Co % 64 == 0:
            dy = torch.randn(B, OH, OH, Co, device="cuda").to(torch.bfloat16)
            wd = (torch.randn(C, k * k * Co, device="cuda") * 0.05).to(torch.bfloat16)
            dx = torch.empty(B, H, H, C, device="cuda", dtype=torch.bfloat16)
            pp = k - 1 - p
            dgeo = (B, OH, OH, Co, H, H, C, k, k, 1, 1, pp, pp, 1, 1, int(math.log2(s)), int(math.log2(s)))
            rec["dgrad_wide_us"] = timeit(lambda: L.pa_conv_gemm(_nat.ptr(dy), _nat.ptr(wd), _nat.ptr(dx), None,
                                                                 *dgeo, st))
            rec["dgrad_sn_us"] = timeit(lambda: L.pa_conv_sn(_nat.ptr(dy), _nat.ptr(wd), _nat.ptr(dx), None, *dgeo,
                                                             None, None, st))
        # weight gradient: wide (im2col when needed + split-K 256x256) vs gathered 64x256 kernel
        dyw = torch.randn(B, OH, OH, Co, device="cuda").to(torch.bfloat16)
        wshape = (Co, C, k, k)
        for mode, key in (("0", "wgrad_wide_us"), ("1", "wgrad_sn_us")):
            _conv._WGRAD_SN[0] = mode
            rec[key] = timeit(lambda: _conv._conv_wgrad(dyw, x, wshape, (s, s), (p, p), (1, 1), torch.bfloat16))
        _conv._WGRAD_SN[0] = "1"
        a = _conv._conv_wgrad(dyw, x, wshape, (s, s), (p, p), (1, 1)).float()
        _conv._WGRAD_SN[0] = "0"
        b_ = _conv._conv_wgrad(dyw, x, wshape, (s, s), (p, p), (1, 1)).float()
        _conv._WGRAD_SN[0] = "auto"
        rec["wgrad_rel_diff"] = float((a - b_).abs().max() / b_.abs().max())
        for kk in list(rec):
            if kk.endswith("_us"):
                rec[kk] = round(rec[kk], 1)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
