#!/usr/bin/env python3
"""Host cost of the native tensor-op dispatch (utils/strict.py + ops/aten_native.py)
per call, on GPU tensors: ATen add vs the same add inside a framework region (HIP
kernel), a view op passing through the dispatch mode, and region enter/exit.
Prints one JSON line (microseconds per call, host wall, median of 5 x 2000)."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from paddle_amd.utils import strict  # noqa: E402


def t(fn, n=2000):
    res = []
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        res.append((time.perf_counter() - t0) / n * 1e6)
    torch.cuda.synchronize()
    return round(statistics.median(res), 2)


x = torch.randn(1024, device="cuda")
y = torch.randn(1024, device="cuda")
r = strict.region("bench")
out = {
    "aten_add_us": t(lambda: x + y),
    "aten_view_us": t(lambda: x.view(32, 32)),
    "empty_region_us": t(lambda: (r.__enter__(), r.__exit__(None, None, None))),
}
with strict.region("bench"):
    out["native_add_in_region_us"] = t(lambda: x + y)
    out["view_in_region_us"] = t(lambda: x.view(32, 32))
    out["empty_in_region_us"] = t(lambda: torch.empty(1024, device="cuda"))
    out["cast_in_region_us"] = t(lambda: x.to(torch.bfloat16))
out["aten_cast_us"] = t(lambda: x.to(torch.bfloat16))
# framework hot paths that bypass the dispatch mode: direct kernel launches
from paddle_amd.ops import aten_native as A, oplib  # noqa: E402

out["direct_add_inplace_us"] = t(lambda: oplib.add_(x, y))
out["aten_add_inplace_us"] = t(lambda: x.add_(y))
out["direct_fill_us"] = t(lambda: oplib.fill_(x, 0.0))
from paddle_amd.ops import _native as _N  # noqa: E402

F = _N.fastops()
if F is not None:
    out["fastops_add_inplace_us"] = t(lambda: F.add_(x, y, 1.0))
    out["fastops_bin_add_us"] = t(lambda: F.bin(50, x, y, 1.0, False))
    out["fastops_cast_us"] = t(lambda: F.cast(x, 1))
z = torch.empty_like(x)
out["direct_add_out_us"] = t(lambda: A._launch(A.B["add"], z, [x, y], a=1.0))


class _Pass(torch.utils._python_dispatch.TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        return func(*args, **(kwargs or {}))


with _Pass():  # the bare cost of a Python dispatch-mode hop around the ATen kernel
    out["aten_add_under_passthrough_mode_us"] = t(lambda: x + y)
print(json.dumps(out))
